// k_scan_private.hip -- private-LDS fused scan: the hot path of the filtered
// low-cardinality groupby (config C2: bqueryd/worker.py:303 + :313 in one pass).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "scan_private.h"

namespace bqg {

template <int NC>
__global__ __launch_bounds__(kBlock, 4) void k_scan_private(ScanParams p, PrivateLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  scan_private_body<NC>(p, L, smem);
}

__device__ void private_finish_body(const FinishParams& f, const SlotArrays& sa, const EmitParams& e, int tid);

// One workgroup per (component, slot): sums / mins that slot's per-workgroup partials in a
// fixed order (coalesced reads, fixed LDS tree: bitwise deterministic).  The last workgroup
// to finish (device-scope counter) runs the finish step, so a query is one launch after the
// scan.
__global__ __launch_bounds__(kBlock) void k_private_reduce(FinishParams f, SlotArrays sa, EmitParams e) {
  __shared__ unsigned long long red[kBlock];
  const int pair = blockIdx.x, tid = threadIdx.x;
  const int S = f.nslots, nb = f.blocks;
  const int comp = pair / S;
  const bool isf = comp >= 2 && f.sum_is_float[comp - 2];
  const unsigned long long* src = f.partials + (size_t)pair * nb;
  unsigned long long v;
  if (comp == 1) {
    uint32_t m = kNoRow;
    for (int b = tid; b < nb; b += kBlock) m = min(m, (uint32_t)src[b]);
    v = m;
  } else if (isf) {
    double x = 0.0;
    for (int b = tid; b < nb; b += kBlock) x += as_f64(src[b]);
    v = as_u64(x);
  } else {
    unsigned long long x = 0;
    for (int b = tid; b < nb; b += kBlock) x += src[b];
    v = x;
  }
  red[tid] = v;
  __syncthreads();
  for (int w = kBlock / 2; w >= 1; w >>= 1) {
    if (tid < w) {
      const unsigned long long o = red[tid + w];
      if (comp == 1) red[tid] = min(red[tid], o);
      else if (isf) red[tid] = as_u64(as_f64(red[tid]) + as_f64(o));
      else red[tid] = red[tid] + o;
    }
    __syncthreads();
  }
  __shared__ bool last;
  if (tid == 0) {
    f.totals[pair] = red[0];
    __threadfence();  // release the total before counting this workgroup done
    last = atomicAdd(f.done, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();  // acquire every workgroup's total
  if (tid < 64) private_finish_body(f, sa, e, tid);
  if (tid == 0) *f.done = 0u;  // ready for the next launch (stream order)
}

// Emits the groups in first-appearance order (S is small: rank by counting), or stores the
// per-slot totals for the generic emit path.
__device__ void private_finish_body(const FinishParams& f, const SlotArrays& sa, const EmitParams& e, int tid) {
  const int S = f.nslots, nsum = f.nsum;
  const int P = (2 + nsum) * S;
  const unsigned long long* tot = f.totals;
  if (!f.emit_inline) {
    for (int i = tid; i < P; i += 64) {
      const int comp = i / S, s = i % S;
      if (comp == 0) sa.cnt[s] = tot[i];
      else if (comp == 1) sa.fst[s] = (uint32_t)tot[i];
      else sa.acc[(size_t)(comp - 2) * S + s] = tot[i];
    }
    return;
  }
  if (tid < S) {
    const int s = tid;
    if (tot[s] > 0) {
      const uint32_t first = (uint32_t)tot[S + s];
      unsigned int rank = 0;
      for (int q = 0; q < S; ++q)
        if (tot[q] > 0 && (uint32_t)tot[S + q] < first) ++rank;
      SlotTotals t;
      t.cnt = tot[s];
      t.fst = first;
#pragma unroll
      for (int q = 0; q < kMaxSums; ++q) {
        t.acc[q] = (q < nsum) ? tot[(2 + q) * S + s] : 0ull;
        t.acc2[q] = 0ull;
      }
      emit_slot(e, (uint64_t)s, (uint64_t)s, rank, t);
    }
  }
  if (tid == 0) {
    unsigned long long g = 0, total = 0;
    for (int q = 0; q < S; ++q) {
      g += tot[q] > 0 ? 1 : 0;
      total += tot[q];
    }
    f.out_hdr[0] = g;
    f.out_hdr[1] = total;
  }
  // the outputs may live in device-mapped host memory: make them visible at system scope
  __threadfence_system();
}

void launch_scan_private(const ScanParams& p, const PrivateLaunch& l, hipStream_t st) {
  BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scan_private<NC>), dim3(l.blocks), dim3(kBlock), l.lds_bytes, st, p, l));
}

void launch_private_finish(const FinishParams& f, const SlotArrays& s, const EmitParams& e, hipStream_t st) {
  hipLaunchKernelGGL(k_private_reduce, dim3((2 + f.nsum) * f.nslots), dim3(kBlock), 0, st, f, s, e);
}

}  // namespace bqg
