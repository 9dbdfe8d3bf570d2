// Kernel stores into page-locked host memory over PCIe vs the DMA copy of the same bytes
// (round 6: can the large-result emit write its 24 MB straight to the host block?)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_write_host(unsigned long long* dst, const unsigned long long* src, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(src[i], dst + i);
}
__global__ void k_write_host4(uint4* dst, const uint4* src, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

int main() {
  const size_t bytes = 24u << 20, n = bytes / 8;
  void *h = nullptr, *d = nullptr;
  hipHostMalloc(&h, bytes, hipHostMallocDefault);
  hipMalloc(&d, bytes);
  hipMemset(d, 1, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float ms;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(a);
    hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("DMA copy 24 MiB:               %.3f ms  %.1f GB/s\n", ms, bytes / (ms * 1e-3) / 1e9);
    for (int grid : {256, 1024, 4096}) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k_write_host, dim3(grid), dim3(256), 0, 0, (unsigned long long*)h, (const unsigned long long*)d, n);
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      printf("kernel 8 B/lane nt grid %5d:   %.3f ms  %.1f GB/s\n", grid, ms, bytes / (ms * 1e-3) / 1e9);
      hipEventRecord(a);
      hipLaunchKernelGGL(k_write_host4, dim3(grid), dim3(256), 0, 0, (uint4*)h, (const uint4*)d, bytes / 16);
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      printf("kernel 16 B/lane grid %5d:     %.3f ms  %.1f GB/s\n", grid, ms, bytes / (ms * 1e-3) / 1e9);
    }
  }
  printf("check %d\n", (int)((unsigned char*)h)[12345]);
  return 0;
}
