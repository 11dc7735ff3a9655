// Loads-only probe of K1's small-launch access pattern (tooling, not product;
// VERDICT r5 item 2).  A launch of B bytes gives every lane of a grid of one
// 1024-thread workgroup per CU one contiguous range of B / (CUs x 1024)
// bytes, as K1's per-launch chunk does below 1 GB, and reads it once:
//   lane64   K1 v3's pattern: each lane walks its own range in 64-byte lines
//            (four 16-byte loads), the next line in flight (double buffer)
//   lane128  the same with 128-byte lines (a whole L2 line per step)
//   group4   grouped: a step's four load instructions cover the wave's 64
//            next 64-byte lines, 4 adjacent lanes per line (16 B each), so an
//            instruction touches 16 lines instead of 64 (K1 would then need
//            an in-wave transpose to bring each line to its lane: not done)
//   group8   8 lanes per 128-byte line, 8 lines per instruction
// Prints GB/s per pattern and size (HIP events, median of reps).
//   hipcc --offload-arch=gfx950 -O3 tools/load_probe.hip -o tools/load_probe
//   tools/load_probe [MB ...]          (default 250 1000 4000)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned fold(v4u v) { return v.x ^ v.y ^ v.z ^ v.w; }
__device__ __forceinline__ v4u ld(const unsigned char* p) { return *reinterpret_cast<const v4u*>(p); }

template <int kW>   // 16-byte words per line: 4 (64 B) or 8 (128 B)
__global__ __launch_bounds__(1024) void lane_lines(const unsigned char* __restrict__ p, unsigned range, unsigned* out) {
  const size_t g = blockIdx.x * 1024ull + threadIdx.x;
  const unsigned char* q = p + g * range;
  constexpr unsigned kL = 16 * kW;
  v4u cur[kW], nxt[kW];
  unsigned acc = 0;
#pragma unroll
  for (int i = 0; i < kW; ++i) cur[i] = ld(q + 16 * i);
  for (unsigned off = 0; off < range; off += kL) {
    const bool more = off + kL < range;
    if (more) {
#pragma unroll
      for (int i = 0; i < kW; ++i) nxt[i] = ld(q + off + kL + 16 * i);
    }
#pragma unroll
    for (int i = 0; i < kW; ++i) acc ^= fold(cur[i]);
    if (more) {
#pragma unroll
      for (int i = 0; i < kW; ++i) cur[i] = nxt[i];
    }
  }
  if (acc == 0x12345678u) out[0] = acc;     // keeps the loads
}

// kG lanes per line of 16 * kG bytes; a step covers the wave's 64 lines in
// 64 / (64 / kG) = kG instructions
template <int kG>
__global__ __launch_bounds__(1024) void grouped(const unsigned char* __restrict__ p, unsigned range, unsigned* out) {
  const unsigned lane = threadIdx.x & 63u;
  const size_t wave_first = (blockIdx.x * 1024ull + (threadIdx.x & ~63u));   // the wave's lane 0 range index
  constexpr unsigned kL = 16 * kG, kPer = 64 / kG;                             // line bytes, lines per instruction
  const unsigned sub = (lane % kG) * 16, who = lane / kG;
  v4u cur[kG], nxt[kG];
  unsigned acc = 0;
#pragma unroll
  for (int j = 0; j < kG; ++j) cur[j] = ld(p + (wave_first + j * kPer + who) * range + sub);
  for (unsigned off = 0; off < range; off += kL) {
    const bool more = off + kL < range;
    if (more) {
#pragma unroll
      for (int j = 0; j < kG; ++j) nxt[j] = ld(p + (wave_first + j * kPer + who) * range + off + kL + sub);
    }
#pragma unroll
    for (int j = 0; j < kG; ++j) acc ^= fold(cur[j]);
    if (more) {
#pragma unroll
      for (int j = 0; j < kG; ++j) cur[j] = nxt[j];
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  std::vector<double> mbs;
  for (int i = 1; i < argc; ++i) mbs.push_back(atof(argv[i]));
  if (mbs.empty()) mbs = {250, 1000, 4000};
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  const unsigned cus = prop.multiProcessorCount, lanes = cus * 1024;
  const size_t maxb = static_cast<size_t>(*std::max_element(mbs.begin(), mbs.end()) * 1e6) + (1 << 20);
  unsigned char* d = nullptr;
  unsigned* o = nullptr;
  if (hipMalloc(&d, maxb) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
  if (hipMemset(d, 1, maxb) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (double mb : mbs) {
    const unsigned range = static_cast<unsigned>((mb * 1e6 / lanes)) & ~127u;
    const double bytes = static_cast<double>(range) * lanes;
    auto time = [&](const char* name, auto launch) {
      std::vector<float> ts;
      for (int r = 0; r < 12; ++r) {
        (void)hipEventRecord(a, 0);
        launch();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r >= 2) ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const float med = ts[ts.size() / 2];
      std::printf("%-8s %7.0f MB (range %5u B per lane, %u CUs): %.4f ms  %7.1f GB/s\n", name, bytes / 1e6, range, cus, med,
                  bytes / (med / 1e3) / 1e9);
    };
    time("lane64", [&] { hipLaunchKernelGGL(lane_lines<4>, dim3(cus), dim3(1024), 0, 0, d, range, o); });
    time("lane128", [&] { hipLaunchKernelGGL(lane_lines<8>, dim3(cus), dim3(1024), 0, 0, d, range, o); });
    time("group4", [&] { hipLaunchKernelGGL(grouped<4>, dim3(cus), dim3(1024), 0, 0, d, range, o); });
    time("group8", [&] { hipLaunchKernelGGL(grouped<8>, dim3(cus), dim3(1024), 0, 0, d, range, o); });
    if (hipGetLastError() != hipSuccess) return 1;
  }
  (void)hipFree(d);
  (void)hipFree(o);
  return 0;
}
