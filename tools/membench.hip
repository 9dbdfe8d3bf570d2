// membench.hip -- read-bandwidth ceilings for the C2 scan's access pattern on gfx950.
// Three column streams (f64 + 2 x i32 = 16 B/row, 100 M rows) read the way k_scan_private
// reads them (1024-row tiles, 4 rows per lane, 16-byte loads, next tile prefetched), with
// variants for cache policy, prefetch depth and grid size, plus a float4 copy for calibration.
// Build: hipcc -O3 --offload-arch=gfx950 tools/membench.hip -o build/membench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4* p) {
  if (NT) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *p;
}

// DEPTH tiles in flight per workgroup (1 = current only + next prefetched, as the product)
template <bool NT, int DEPTH>
__global__ __launch_bounds__(256, 4) void read3(const double* f, const int* a, const int* b, int64_t n,
                                                unsigned long long* out) {
  const int tid = threadIdx.x;
  const int64_t ntiles = n / 1024;
  unsigned long long acc = 0;
  uint4 rf0[DEPTH], rf1[DEPTH], ra[DEPTH], rb[DEPTH];
  int64_t tile = blockIdx.x;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    const int64_t t = tile + (int64_t)d * gridDim.x;
    if (t < ntiles) {
      const int64_t r0 = t * 1024 + tid * 4;
      rf0[d] = ld<NT>(reinterpret_cast<const uint4*>(f + r0));
      rf1[d] = ld<NT>(reinterpret_cast<const uint4*>(f + r0 + 2));
      ra[d] = ld<NT>(reinterpret_cast<const uint4*>(a + r0));
      rb[d] = ld<NT>(reinterpret_cast<const uint4*>(b + r0));
    }
  }
  for (; tile < ntiles; tile += (int64_t)gridDim.x * DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int64_t t = tile + (int64_t)d * gridDim.x;
      if (t < ntiles) {
        acc += rf0[d].x ^ rf0[d].y ^ rf0[d].z ^ rf0[d].w ^ rf1[d].x ^ rf1[d].y ^ rf1[d].z ^ rf1[d].w;
        acc += (ra[d].x + ra[d].y + ra[d].z + ra[d].w) * (rb[d].x | rb[d].y | rb[d].z | rb[d].w);
        const int64_t tn = t + (int64_t)gridDim.x * DEPTH;
        if (tn < ntiles) {
          const int64_t r0 = tn * 1024 + tid * 4;
          rf0[d] = ld<NT>(reinterpret_cast<const uint4*>(f + r0));
          rf1[d] = ld<NT>(reinterpret_cast<const uint4*>(f + r0 + 2));
          ra[d] = ld<NT>(reinterpret_cast<const uint4*>(a + r0));
          rb[d] = ld<NT>(reinterpret_cast<const uint4*>(b + r0));
        }
      }
    }
  }
  if (acc == 0x123456789ull) out[blockIdx.x] = acc;
}

// one stream of the same total size
template <bool NT>
__global__ __launch_bounds__(256, 4) void read1(const uint4* p, int64_t n16, unsigned long long* out) {
  unsigned long long acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256 * 4) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = i + (int64_t)u * gridDim.x * 256;
      v[u] = j < n16 ? ld<NT>(p + j) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x123456789ull) out[blockIdx.x] = acc;
}


// The C2 query hand-specialised (i32 key, i32 "x >= 2" term, f64 sum + count + first row,
// private [slot][lane] LDS accumulators): what the generic k_scan_private could reach.
__global__ __launch_bounds__(256, 4) void c2spec(const int* key, const int* term, const double* val, int64_t n,
                                                 int kmin, int S, unsigned long long* out) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x;
  double* acc = reinterpret_cast<double*>(smem);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(acc + S * 256);
  uint32_t* fst = cnt + S * 256;
  for (int s = 0; s < S; ++s) {
    acc[s * 256 + tid] = 0.0;
    cnt[s * 256 + tid] = 0;
    fst[s * 256 + tid] = 0xFFFFFFFFu;
  }
  const int64_t ntiles = n / 1024;
  int64_t tile = blockIdx.x;
  uint4 rk, rt, rv0, rv1;
  auto load = [&](int64_t t) {
    const int64_t r0 = t * 1024 + tid * 4;
    rk = ld<true>(reinterpret_cast<const uint4*>(key + r0));
    rt = ld<true>(reinterpret_cast<const uint4*>(term + r0));
    rv0 = ld<true>(reinterpret_cast<const uint4*>(val + r0));
    rv1 = ld<true>(reinterpret_cast<const uint4*>(val + r0 + 2));
  };
  if (tile < ntiles) load(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    const int64_t row0 = tile * 1024 + tid * 4;
    const int k[4] = {(int)rk.x, (int)rk.y, (int)rk.z, (int)rk.w};
    const int tm[4] = {(int)rt.x, (int)rt.y, (int)rt.z, (int)rt.w};
    const double v[4] = {__hiloint2double(rv0.y, rv0.x), __hiloint2double(rv0.w, rv0.z),
                         __hiloint2double(rv1.y, rv1.x), __hiloint2double(rv1.w, rv1.z)};
    if (tile + gridDim.x < ntiles) load(tile + gridDim.x);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (tm[r] >= 2) {
        const int idx = (k[r] - kmin) * 256 + tid;
        const uint32_t c0 = cnt[idx];
        if (c0 == 0) fst[idx] = (uint32_t)(row0 + r);
        cnt[idx] = c0 + 1;
        acc[idx] += v[r];
      }
    }
  }
  __syncthreads();
  if (tid < S) {
    double a = 0;
    unsigned long long c = 0;
    for (int j = 0; j < 256; ++j) {
      a += acc[tid * 256 + j];
      c += cnt[tid * 256 + j];
    }
    out[blockIdx.x * 64 + tid] = c + (unsigned long long)a;
  }
}

__global__ void copy4(const float4* s, float4* d, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) d[i] = s[i];
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const int64_t n = 100000000 / 1024 * 1024;
  double* f;
  int *a, *b;
  unsigned long long* out;
  CK(hipMalloc(&f, n * 8 + 4096));
  CK(hipMalloc(&a, n * 4 + 4096));
  CK(hipMalloc(&b, n * 4 + 4096));
  CK(hipMalloc(&out, 1 << 24));
  CK(hipMemset(f, 1, n * 8));
  CK(hipMemset(a, 2, n * 4));
  CK(hipMemset(b, 3, n * 4));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cu = prop.multiProcessorCount;
  const double bytes = (double)n * 16;
  const int reps = 20;
  for (int per_cu : {2, 4, 8}) {
    const int g = cu * per_cu;
    float t;
    t = timeit([&] { hipLaunchKernelGGL((read3<false, 1>), dim3(g), dim3(256), 0, 0, f, a, b, n, out); }, reps);
    printf("read3 plain depth1 grid=%d: %.3f ms %.0f GB/s\n", g, t, bytes / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((read3<true, 1>), dim3(g), dim3(256), 0, 0, f, a, b, n, out); }, reps);
    printf("read3 nt    depth1 grid=%d: %.3f ms %.0f GB/s\n", g, t, bytes / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((read3<false, 2>), dim3(g), dim3(256), 0, 0, f, a, b, n, out); }, reps);
    printf("read3 plain depth2 grid=%d: %.3f ms %.0f GB/s\n", g, t, bytes / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((read3<true, 2>), dim3(g), dim3(256), 0, 0, f, a, b, n, out); }, reps);
    printf("read3 nt    depth2 grid=%d: %.3f ms %.0f GB/s\n", g, t, bytes / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((read1<false>), dim3(g), dim3(256), 0, 0, (const uint4*)f, n * 8 / 16, out); }, reps);
    printf("read1 plain        grid=%d: %.3f ms %.0f GB/s\n", g, t, n * 8.0 / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((read1<true>), dim3(g), dim3(256), 0, 0, (const uint4*)f, n * 8 / 16, out); }, reps);
    printf("read1 nt           grid=%d: %.3f ms %.0f GB/s\n", g, t, n * 8.0 / t / 1e6);
  }
  {
    // C2-shaped data: keys 0..5, term values 0..6
    std::vector<int> hk(n), ht(n);
    for (int64_t i = 0; i < n; ++i) {
      hk[i] = (int)((i * 2654435761ull >> 7) % 6);
      ht[i] = (int)((i * 40503ull >> 3) % 7);
    }
    CK(hipMemcpy(a, hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(b, ht.data(), n * 4, hipMemcpyHostToDevice));
    const int S = 6;
    const size_t lds = (size_t)S * 256 * 16;
    for (int per_cu : {2, 3, 4, 6}) {
      const int g = cu * per_cu;
      float t = timeit([&] { hipLaunchKernelGGL(c2spec, dim3(g), dim3(256), lds, 0, a, b, f, n, 0, S, out); }, reps);
      printf("c2spec grid=%d: %.3f ms %.0f GB/s\n", g, t, bytes / t / 1e6);
    }
  }
  {
    const int64_t n4 = n * 8 / 16;  // 800 MB copied
    float t = timeit([&] { hipLaunchKernelGGL(copy4, dim3(cu * 8), dim3(256), 0, 0, (const float4*)f, (float4*)a, n4 / 2); }, reps);
    printf("copy float4 %.0f MB: %.3f ms %.0f GB/s (r+w)\n", n4 / 2 * 16 / 1e6, t, 2.0 * n4 / 2 * 16 / t / 1e6);
  }
  return 0;
}
