// D2H copy of a 24 MB, four-column result in one copy vs per-column copies vs per-(row chunk,
// column) copies, all into page-locked memory (round 6: can the large-result copy be split into
// row chunks that follow the emit's passes without paying per-copy overhead?)
#include <hip/hip_runtime.h>
#include <cstdio>

int main() {
  const size_t G = 1000000, sz[4] = {4, 4, 8, 8};
  size_t off[5] = {0};
  for (int j = 0; j < 4; ++j) off[j + 1] = off[j] + ((G * sz[j] + 255) & ~size_t(255));
  const size_t bytes = off[4];
  void *h = nullptr, *d = nullptr;
  if (hipHostMalloc(&h, bytes, hipHostMallocDefault) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
  (void)hipMemset(d, 1, bytes);
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int rep = 0; rep < 4; ++rep) {
    for (int chunks : {0, 1, 2, 4, 8}) {
      (void)hipEventRecord(a, st);
      if (chunks == 0) {
        (void)hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, st);
      } else {
        for (int c = 0; c < chunks; ++c)
          for (int j = 0; j < 4; ++j) {
            const size_t r0 = G * c / chunks, r1 = G * (c + 1) / chunks;
            (void)hipMemcpyAsync((char*)h + off[j] + r0 * sz[j], (char*)d + off[j] + r0 * sz[j], (r1 - r0) * sz[j],
                                 hipMemcpyDeviceToHost, st);
          }
      }
      (void)hipEventRecord(b, st);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      printf("rep %d  %s %d: %.3f ms  %.1f GB/s\n", rep, chunks ? "row chunks x 4 columns, chunks =" : "one copy", chunks, ms,
             bytes / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
