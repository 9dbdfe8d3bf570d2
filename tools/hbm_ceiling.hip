// hbm_ceiling.hip -- read-only HBM ceiling for the C2 access shape (measurement tool, not
// product code): three columns of 100 M rows (int32, int32, float64 = 16 B/row), consumed in
// 1024-row tiles by 256-thread workgroups with one tile prefetched, as k_scan_private does.
//   A: the scan's lane mapping (4 rows per lane; the 8-byte column as two 16-byte loads at a
//      32-byte lane stride)
//   B: same, but the 8-byte column's two loads cover the tile's two halves contiguously
//   C: plain grid-stride 16-byte streaming of the same bytes (no tile structure)
// build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_ceiling tools/hbm_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld(const unsigned char* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

template <int MODE>
__global__ __launch_bounds__(256, 4) void k_read(const unsigned char* a, const unsigned char* b,
                                                 const unsigned char* c, long ntiles, unsigned* out) {
  const int t = threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 r0, r1, r2, r3;
  auto load = [&](long tile) {
    r0 = ld(a + tile * 4096 + t * 16);
    r1 = ld(b + tile * 4096 + t * 16);
    if (MODE == 0) {
      r2 = ld(c + tile * 8192 + t * 32);
      r3 = ld(c + tile * 8192 + t * 32 + 16);
    } else {
      r2 = ld(c + tile * 8192 + t * 16);
      r3 = ld(c + tile * 8192 + 4096 + t * 16);
    }
  };
  long tile = blockIdx.x;
  if (tile < ntiles) load(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    const u32x4 c0 = r0, c1 = r1, c2 = r2, c3 = r3;
    const long next = tile + gridDim.x;
    load(next < ntiles ? next : tile);
    acc ^= c0 ^ c1 ^ c2 ^ c3;
  }
  const unsigned v = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (v == 0x12345678u) out[blockIdx.x] = v;  // keeps the loads live
}

__global__ __launch_bounds__(256) void k_stream(const unsigned char* a, long abytes, const unsigned char* b,
                                                long bbytes, const unsigned char* c, long cbytes, unsigned* out) {
  u32x4 acc = {0, 0, 0, 0};
  const long stride = (long)gridDim.x * blockDim.x * 16;
  const long start = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  for (long o = start; o < abytes; o += stride) acc ^= ld(a + o);
  for (long o = start; o < bbytes; o += stride) acc ^= ld(b + o);
  for (long o = start; o < cbytes; o += stride) acc ^= ld(c + o);
  const unsigned v = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (v == 0x12345678u) out[blockIdx.x] = v;
}

int main(int argc, char** argv) {
  const long rows = argc > 1 ? atol(argv[1]) : 100000000L;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const long ntiles = rows / 1024;
  const long abytes = ntiles * 4096, cbytes = ntiles * 8192;
  unsigned char *a, *b, *c;
  unsigned* out;
  CHECK(hipMalloc(&a, abytes + 4096));
  CHECK(hipMalloc(&b, abytes + 4096));
  CHECK(hipMalloc(&c, cbytes + 8192));
  CHECK(hipMalloc(&out, 1 << 20));
  CHECK(hipMemset(a, 1, abytes));
  CHECK(hipMemset(b, 2, abytes));
  CHECK(hipMemset(c, 3, cbytes));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double bytes = 2.0 * abytes + cbytes;
  for (int mode = 0; mode < 3; ++mode) {
    for (int per_cu = 2; per_cu <= 8; per_cu *= 2) {
      const int grid = cus * per_cu;
      auto run = [&] {
        if (mode == 0) hipLaunchKernelGGL(k_read<0>, dim3(grid), dim3(256), 0, 0, a, b, c, ntiles, out);
        else if (mode == 1) hipLaunchKernelGGL(k_read<1>, dim3(grid), dim3(256), 0, 0, a, b, c, ntiles, out);
        else hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, a, abytes, b, abytes, c, cbytes, out);
      };
      for (int i = 0; i < 3; ++i) run();
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) run();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double per = ms / reps;
      printf("mode %c  workgroups/CU %d  %.3f ms  %.2f TB/s\n", "ABC"[mode], per_cu, per, bytes / (per * 1e-3) / 1e12);
      fflush(stdout);
    }
  }
  return 0;
}
