// reduce_micro.hip -- where the C2 finish kernel's ~10 us go: one 1024-thread workgroup
// launched after a grid that writes 1024 x 30 per-workgroup partials, in variants that add one
// ingredient of k_private_reduce (k_scan_private.hip) at a time.  Durations come from
// rocprofv3 --kernel-trace --stats (kernel names carry the variant) and from HIP events.
//   v0  empty kernel (launch + dispatch floor)
//   v1  + the lane-strided loads of 30 x 1024 partials and the shuffle reduce, totals to LDS
//   v2  + a 2 KiB kernel-argument struct read by wave 0 (the EmitParams-sized argument)
//   v3  + 10 slots x 4 columns written to device memory
//   v4  + the same written to pinned host memory, then a system-scope fence
//   v5  v4 without the fence (the host reads after hipStreamSynchronize)
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/micro/reduce_micro.hip -o tools/micro/bin/reduce_micro
// run:   reduce_micro [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int kBlocks = 1024, kPairs = 30, kSlots = 10, kCols = 4;

struct BigArg {
  unsigned long long* out[kCols];
  unsigned long long* hdr;
  int pad[500];  // ~2 KiB, like EmitParams
};

__global__ void k_partials(unsigned long long* part) {
  const int b = blockIdx.x;
  if (threadIdx.x < kPairs) part[(size_t)threadIdx.x * kBlocks + b] = (unsigned long long)(b + threadIdx.x);
}

template <int V>
__global__ __launch_bounds__(1024) void k_finish(const unsigned long long* part, BigArg a) {
  __shared__ unsigned long long tot[kPairs];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (V >= 1) {
    for (int pair = wave; pair < kPairs; pair += 16) {
      unsigned long long x[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) x[i] = part[(size_t)pair * kBlocks + i * 64 + lane];
      unsigned long long acc = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc += x[i];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) acc += (unsigned long long)__shfl_xor((long long)acc, o, 64);
      if (lane == 0) tot[pair] = acc;
    }
    __syncthreads();
  }
  if (tid < kSlots) {
    unsigned long long v = V >= 1 ? tot[tid] + tot[kSlots + tid] : (unsigned long long)tid;
    if (V >= 2) v += (unsigned long long)a.pad[tid * 37 % 500];
    if (V >= 3) {
#pragma unroll
      for (int c = 0; c < kCols; ++c) a.out[c][tid] = v + c;
    }
  }
  if (V >= 3 && tid == 0) a.hdr[0] = kSlots;
  if (V == 4) __threadfence_system();
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  unsigned long long *part, *dout, *hout;
  CK(hipMalloc(&part, (size_t)kPairs * kBlocks * 8));
  CK(hipMalloc(&dout, 4096));
  CK(hipHostMalloc(&hout, 4096, hipHostMallocMapped));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int v = 0; v < 6; ++v) {
    BigArg a{};
    unsigned long long* base = v >= 4 ? hout : dout;
    for (int c = 0; c < kCols; ++c) a.out[c] = base + 16 + c * kSlots;
    a.hdr = base;
    auto launch = [&]() {
      switch (v) {
        case 0: hipLaunchKernelGGL(k_finish<0>, dim3(1), dim3(1024), 0, st, part, a); break;
        case 1: hipLaunchKernelGGL(k_finish<1>, dim3(1), dim3(1024), 0, st, part, a); break;
        case 2: hipLaunchKernelGGL(k_finish<2>, dim3(1), dim3(1024), 0, st, part, a); break;
        case 3: hipLaunchKernelGGL(k_finish<3>, dim3(1), dim3(1024), 0, st, part, a); break;
        case 4: hipLaunchKernelGGL(k_finish<4>, dim3(1), dim3(1024), 0, st, part, a); break;
        default: hipLaunchKernelGGL(k_finish<5>, dim3(1), dim3(1024), 0, st, part, a); break;
      }
    };
    float total = 0;
    int stale = 0;  // host-memory variants: the header read after the sync must be the kernel's
    for (int r = 0; r < reps; ++r) {
      if (v >= 4) ((volatile unsigned long long*)hout)[0] = 0;
      hipLaunchKernelGGL(k_partials, dim3(kBlocks), dim3(64), 0, st, part);
      CK(hipEventRecord(e0, st));
      launch();
      CK(hipEventRecord(e1, st));
      CK(hipStreamSynchronize(st));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      total += ms;
      if (v >= 4 && ((volatile unsigned long long*)hout)[0] != (unsigned long long)kSlots) ++stale;
    }
    printf("{\"variant\": %d, \"event_us\": %.2f, \"stale_reads\": %d}\n", v, 1e3 * total / reps, stale);
  }
  CK(hipStreamSynchronize(st));
  return 0;
}
