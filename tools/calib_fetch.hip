// FETCH_SIZE calibration for K1's access pattern (tools only, not product).
//
// MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports half the bytes of a wide
// coalesced streaming read, and other access widths are uncalibrated.  K1
// reads each lane's own chunk in whole 128-byte lines (8 x 16-byte
// nontemporal loads per lane, lanes 4 KiB apart), so this program reads a
// known byte count once with
//   calib_coalesced  16 B per lane, consecutive lanes adjacent
//   calib_k1pattern  K1's layout: lane l of the grid owns chunk l (4 KiB),
//                    walks it in 128-byte lines
// and prints the byte count; rocprofv3 --pmc FETCH_SIZE on the same run gives
// the counter per kernel, hence the scale for K1's FETCH_SIZE.
//   hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o tools/calib_fetch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void calib_coalesced(const v4u* __restrict__ p, size_t n16, unsigned* out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) {
    const v4u v = __builtin_nontemporal_load(p + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;   // keep the loads
}

__global__ __launch_bounds__(1024) void calib_k1pattern(const unsigned char* __restrict__ p, size_t nchunks,
                                                        unsigned chunk, unsigned* out) {
  unsigned acc = 0;
  for (size_t c = blockIdx.x * 1024ull + threadIdx.x; c < nchunks; c += gridDim.x * 1024ull) {
    const unsigned char* q = p + c * chunk;
    for (unsigned off = 0; off < chunk; off += 128) {
      v4u line[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) line[i] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(q + off + 16 * i));
#pragma unroll
      for (int i = 0; i < 8; ++i) acc ^= line[i].x ^ line[i].y ^ line[i].z ^ line[i].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// K1 v3's layout: lane-owned 4 KiB chunks walked in 64-byte lines of
// temporal 16-byte loads, one 1024-thread workgroup per CU.
__global__ __launch_bounds__(1024) void calib_k1v3(const unsigned char* __restrict__ p, size_t nchunks,
                                                   unsigned chunk, unsigned* out) {
  unsigned acc = 0;
  for (size_t c = blockIdx.x * 1024ull + threadIdx.x; c < nchunks; c += gridDim.x * 1024ull) {
    const unsigned char* q = p + c * chunk;
    for (unsigned off = 0; off < chunk; off += 64) {
      v4u line[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) line[i] = *reinterpret_cast<const v4u*>(q + off + 16 * i);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc ^= line[i].x ^ line[i].y ^ line[i].z ^ line[i].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// Same bytes per lane, but each load instruction covers 8 lines: the 8 lanes
// of a group read one 128-byte line (group g of load k -> lane 8k+g's line),
// optionally transposed through LDS so every lane ends up with its own line.
template <bool kLdsTranspose>
__global__ __launch_bounds__(1024) void calib_grouped(const unsigned char* __restrict__ p, size_t nchunks,
                                                      unsigned chunk, unsigned* out) {
  __shared__ v4u stage[kLdsTranspose ? 16 * 64 * 8 : 1];   // 8 KiB per wave
  const unsigned lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  unsigned acc = 0;
  for (size_t c0 = blockIdx.x * 1024ull + wid * 64ull; c0 < nchunks; c0 += gridDim.x * 1024ull) {
    for (unsigned off = 0; off < chunk; off += 128) {
      v4u v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const size_t owner = c0 + 8 * k + (lane >> 3);
        v[k] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p + owner * chunk + off + 16 * (lane & 7)));
      }
      if (kLdsTranspose) {
        v4u* w = stage + wid * 512;
#pragma unroll
        for (int k = 0; k < 8; ++k) w[(8 * k + (lane >> 3)) * 8 + (lane & 7)] = v[k];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = w[lane * 8 + ((i + lane) & 7)];
        __builtin_amdgcn_wave_barrier();
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// Generalised: kL lanes share one (16*kL)-byte piece of a lane's stream per
// load instruction (64/kL pieces per instruction); kL loads then an LDS
// transpose (64*16*kL bytes per wave) give each lane 16*kL bytes of its own
// stream per step.  kWaves waves per workgroup.
template <int kL, int kWaves>
__global__ __launch_bounds__(kWaves * 64) void calib_piece(const unsigned char* __restrict__ p, size_t nchunks,
                                                           unsigned chunk, unsigned* out) {
  __shared__ v4u stage[kWaves * 64 * kL];
  const unsigned lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  constexpr unsigned kG = 64 / kL;
  unsigned acc = 0;
  for (size_t c0 = blockIdx.x * (kWaves * 64ull) + wid * 64ull; c0 < nchunks; c0 += gridDim.x * (kWaves * 64ull)) {
    for (unsigned off = 0; off < chunk; off += 16 * kL) {
      v4u v[kL];
#pragma unroll
      for (int k = 0; k < kL; ++k) {
        const size_t owner = c0 + kG * k + lane / kL;
        v[k] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p + owner * chunk + off + 16 * (lane % kL)));
      }
      v4u* w = stage + wid * 64 * kL;
#pragma unroll
      for (int k = 0; k < kL; ++k) w[(kG * k + lane / kL) * kL + lane % kL] = v[k];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < kL; ++i) v[i] = w[lane * kL + ((i + lane) % kL)];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < kL; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// K1 candidate scheme: grouped loads (8 lanes per 128-byte line, 8 loads per
// round = one line for each of the wave's 64 streams), transposed through a
// 2 KiB-per-wave LDS stage in 4 sub-rounds (16 owners per sub-round read
// their whole line), optionally with the next round's loads issued before
// the current round is transposed.
template <bool kPrefetch>
__global__ __launch_bounds__(1024) void calib_sub(const unsigned char* __restrict__ p, size_t nchunks,
                                                  unsigned chunk, unsigned* out) {
  __shared__ v4u stage[16 * 128];
  const unsigned lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  unsigned acc = 0;
  v4u* w = stage + wid * 128;
  for (size_t c0 = blockIdx.x * 1024ull + wid * 64ull; c0 < nchunks; c0 += gridDim.x * 1024ull) {
    v4u nx[8];
    auto load = [&](unsigned off, v4u* v) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const size_t owner = c0 + 8 * k + (lane >> 3);
        v[k] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p + owner * chunk + off + 16 * (lane & 7)));
      }
    };
    if (kPrefetch) load(0, nx);
    for (unsigned off = 0; off < chunk; off += 128) {
      v4u v[8];
      if (kPrefetch) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = nx[k];
        if (off + 128 < chunk) load(off + 128, nx);
      } else {
        load(off, v);
      }
      v4u line[8];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        // loads 2s, 2s+1 hold the whole lines of owners 16s .. 16s+15
        w[(lane >> 3) * 8 + (lane & 7)] = v[2 * s];
        w[64 + (lane >> 3) * 8 + (lane & 7)] = v[2 * s + 1];
        __builtin_amdgcn_wave_barrier();
        if ((lane >> 4) == static_cast<unsigned>(s)) {
          const unsigned o = lane & 15u;   // owner 16s + o = 8k + g with k = 2s + (o >> 3), g = o & 7
#pragma unroll
          for (int i = 0; i < 8; ++i) line[i] = w[((o >> 3) * 64) + (o & 7) * 8 + ((i + o) & 7)];
        }
        __builtin_amdgcn_wave_barrier();
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) acc ^= line[i].x ^ line[i].y ^ line[i].z ^ line[i].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int kL, int kWaves>
void run_piece(const char* name, const unsigned char* d, size_t bytes, unsigned chunk, unsigned* o, int cus) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float ms = 0;
  hipEventRecord(a);
  hipLaunchKernelGGL((calib_piece<kL, kWaves>), dim3(cus), dim3(kWaves * 64), 0, 0, d, bytes / chunk, chunk, o);
  hipEventRecord(b);
  hipEventSynchronize(b);
  hipEventElapsedTime(&ms, a, b);
  printf("%s bytes %zu time %.3f ms %.1f GB/s\n", name, bytes, ms, bytes / ms / 1e6);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 4ull) << 30;
  const unsigned chunk = 4096;
  unsigned char* d = nullptr;
  unsigned* o = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) { fprintf(stderr, "hipMalloc failed\n"); return 1; }
  hipMemset(d, 1, bytes);
  hipDeviceSynchronize();
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 2; ++rep) {
    float ms = 0;
    hipEventRecord(a);
    hipLaunchKernelGGL(calib_coalesced, dim3(cus * 8), dim3(256), 0, 0, reinterpret_cast<const v4u*>(d), bytes / 16, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("calib_coalesced bytes %zu time %.3f ms %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    hipEventRecord(a);
    hipLaunchKernelGGL(calib_k1pattern, dim3(cus), dim3(1024), 0, 0, d, bytes / chunk, chunk, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("calib_k1pattern bytes %zu time %.3f ms %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    hipEventRecord(a);
    hipLaunchKernelGGL(calib_k1v3, dim3(cus), dim3(1024), 0, 0, d, bytes / chunk, chunk, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("calib_k1v3 bytes %zu time %.3f ms %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    hipEventRecord(a);
    hipLaunchKernelGGL(calib_grouped<false>, dim3(cus), dim3(1024), 0, 0, d, bytes / chunk, chunk, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("calib_grouped bytes %zu time %.3f ms %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    hipEventRecord(a);
    hipLaunchKernelGGL(calib_grouped<true>, dim3(cus), dim3(1024), 0, 0, d, bytes / chunk, chunk, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("calib_grouped_lds bytes %zu time %.3f ms %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    hipEventRecord(a);
    hipLaunchKernelGGL(calib_sub<false>, dim3(cus), dim3(1024), 0, 0, d, bytes / chunk, chunk, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("calib_sub bytes %zu time %.3f ms %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    hipEventRecord(a);
    hipLaunchKernelGGL(calib_sub<true>, dim3(cus), dim3(1024), 0, 0, d, bytes / chunk, chunk, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("calib_sub_prefetch bytes %zu time %.3f ms %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    run_piece<4, 16>("piece64_w16", d, bytes, chunk, o, cus);
    run_piece<2, 16>("piece32_w16", d, bytes, chunk, o, cus);
    run_piece<1, 16>("piece16_w16", d, bytes, chunk, o, cus);
    run_piece<4, 12>("piece64_w12", d, bytes, chunk, o, cus);
    run_piece<4, 8>("piece64_w8", d, bytes, chunk, o, cus);
    run_piece<2, 8>("piece32_w8", d, bytes, chunk, o, cus);
  }
  hipFree(d);
  hipFree(o);
  return 0;
}
