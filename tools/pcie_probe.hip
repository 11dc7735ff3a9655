// Host -> HBM feed ceiling on one MI355X: pinned-host copy variants and a
// zero-copy kernel read over PCIe.  Reported beside the scan (never the metric).
//   hipcc --offload-arch=gfx950 -O2 -o tools/pcie_probe tools/pcie_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } \
  } while (0)

__global__ void sum_kernel(const uint4* __restrict__ p, size_t n16, unsigned long long* out) {
  unsigned long long acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x123456789ull) out[0] = acc;   // keeps the loads live
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t total = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 8ull) << 30;
  unsigned flags_list[] = {hipHostMallocDefault, hipHostMallocNonCoherent, hipHostMallocWriteCombined};
  const char* flag_names[] = {"default", "noncoherent", "writecombined"};
  uint8_t* d = nullptr;
  CK(hipMalloc(&d, total));
  unsigned long long* dout = nullptr;
  CK(hipMalloc(&dout, 8));
  hipStream_t st[4];
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int fi = 0; fi < 3; ++fi) {
    uint8_t* h = nullptr;
    CK(hipHostMalloc(&h, total, flags_list[fi]));
    std::memset(h, 7, total);
    // one copy
    for (int rep = 0; rep < 2; ++rep) {
      double t0 = now_s();
      CK(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, st[0]));
      CK(hipStreamSynchronize(st[0]));
      double t = now_s() - t0;
      if (rep) std::printf("%-13s single copy          %.1f GB/s\n", flag_names[fi], total / t / 1e9);
    }
    // chunked over 1, 2, 4 streams
    for (size_t chunk : {64ull << 20, 256ull << 20, 1ull << 30}) {
      for (int ns : {1, 2, 4}) {
        double t0 = now_s();
        int k = 0;
        for (size_t o = 0; o < total; o += chunk, ++k) {
          size_t n = std::min(chunk, total - o);
          CK(hipMemcpyAsync(d + o, h + o, n, hipMemcpyHostToDevice, st[k % ns]));
        }
        for (int s = 0; s < ns; ++s) CK(hipStreamSynchronize(st[s]));
        double t = now_s() - t0;
        std::printf("%-13s chunk %5zu MB x %d streams %.1f GB/s\n", flag_names[fi], chunk >> 20, ns, total / t / 1e9);
      }
    }
    // zero-copy kernel read over PCIe
    void* hd = nullptr;
    CK(hipHostGetDevicePointer(&hd, h, 0));
    for (int rep = 0; rep < 2; ++rep) {
      double t0 = now_s();
      sum_kernel<<<2048, 256, 0, st[0]>>>(static_cast<const uint4*>(hd), total / 16, dout);
      CK(hipStreamSynchronize(st[0]));
      double t = now_s() - t0;
      if (rep) std::printf("%-13s zero-copy kernel read %.1f GB/s\n", flag_names[fi], total / t / 1e9);
    }
    CK(hipHostFree(h));
  }
  // pageable source
  {
    std::vector<uint8_t> pg(1ull << 30, 5);
    double t0 = now_s();
    CK(hipMemcpy(d, pg.data(), pg.size(), hipMemcpyHostToDevice));
    double t = now_s() - t0;
    std::printf("pageable      1 GB hipMemcpy      %.1f GB/s\n", pg.size() / t / 1e9);
  }
  // HBM -> HBM reference
  {
    double t0 = now_s();
    CK(hipMemcpyAsync(d + total / 2, d, total / 2, hipMemcpyDeviceToDevice, st[0]));
    CK(hipStreamSynchronize(st[0]));
    double t = now_s() - t0;
    std::printf("HBM->HBM copy                     %.0f GB/s (read+write %.0f)\n", total / 2 / t / 1e9, total / t / 1e9);
  }
  return 0;
}
