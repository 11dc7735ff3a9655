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
  }
  hipFree(d);
  hipFree(o);
  return 0;
}
