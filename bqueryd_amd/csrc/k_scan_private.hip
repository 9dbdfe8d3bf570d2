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

// emit_slot (device.h) restricted to what an inline private emit can hold: dense integer keys
// (no hash mode, no float keys) and sum / count / mean (distinct counts and std take the
// generic path) -- a fraction of the general function's code on the finish kernel's one
// pass through it
__device__ __forceinline__ void emit_slot_private(const EmitParams& e, uint64_t code, unsigned int rank,
                                                  const SlotTotals& t) {
  for (int j = 0; j < e.ncols; ++j) {
    const EmitCol& c = e.cols[j];
    uint64_t bits;
    if (c.kind == 0) {
      const DevKey& k = e.keys[c.key];
      bits = (uint64_t)k.min + key_offset(code, k);
    } else if (c.op == BQG_COUNT) {
      bits = t.cnt;
    } else {
      const unsigned long long a = t.acc[c.state];
      const double dec = e.sum_dec[c.state];
      if (c.op == BQG_MEAN) {
        const double sv = c.in_float ? (dec != 0.0 ? (double)(long long)a / dec : as_f64(a))
                                     : (c.in_dtype == BQG_U64 ? (double)(uint64_t)a : (double)(long long)a);
        bits = as_u64(sv / (double)t.cnt);
      } else {  // SUM
        bits = a;
        if (c.in_float && dec != 0.0) bits = as_u64((double)(long long)a / dec);
        if (c.in_float && c.out_dtype == BQG_F32) bits = (uint64_t)__float_as_uint((float)as_f64(bits));
      }
    }
    store_elem(c.out, c.out_dtype, rank, bits);
  }
}

// ONE workgroup: every (component, slot) pair's per-workgroup partials are reduced by one wave
// (lane-strided reads in a fixed order, then a fixed shuffle tree: bitwise deterministic) into
// LDS, and wave 0 runs the finish step -- no grid of reduce workgroups, no device-scope
// "last workgroup" counter and fences between them (the two-level version took ~11 us of C2's
// ~0.29 ms step).
constexpr int kPrivReduceThreads = 1024;
__global__ __launch_bounds__(kPrivReduceThreads) void k_private_reduce(FinishParams f, SlotArrays sa, EmitParams e) {
  __shared__ unsigned long long tot[(2 + kMaxSums) * kMaxPrivateSlots];
  // the emit description staged in LDS by all threads at once (one parallel load of the ~1.5
  // KiB kernel argument), so the finish wave's dependent field reads are LDS reads rather than
  // a chain of first-touch kernel-argument fetches
  __shared__ EmitParams es;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwaves = kPrivReduceThreads / 64;
  static_assert(sizeof(EmitParams) % 4 == 0 && sizeof(EmitParams) / 4 <= kPrivReduceThreads, "EmitParams copy: one word per thread");
  if (tid < (int)(sizeof(EmitParams) / 4))
    reinterpret_cast<uint32_t*>(&es)[tid] = reinterpret_cast<const uint32_t*>(&e)[tid];
  const int S = f.nslots, nb = f.blocks;
  const int P = (2 + f.nsum) * S;
  // every wave takes its pairs two at a time (pair, pair + 16): the loads of both issued together
  // -- one memory round trip per two pairs (C2: 30 pairs, one round)
  for (int pair0 = wave; pair0 < P; pair0 += 2 * nwaves) {
    unsigned long long acc[2];
    int comps[2];
    bool isfs[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pair = pair0 + h * nwaves;
      comps[h] = pair < P ? pair / S : 0;
      isfs[h] = pair < P && comps[h] >= 2 && f.sum_is_float[comps[h] - 2];
      acc[h] = comps[h] == 1 ? (unsigned long long)kNoRow : 0ull;
    }
    for (int b0 = 0; b0 < nb; b0 += 64 * 16) {
      unsigned long long x[2][16];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pair = pair0 + h * nwaves;
        const unsigned long long* src = f.partials + (size_t)(pair < P ? pair : 0) * nb;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int b = b0 + i * 64 + lane;
          x[h][i] = (pair < P && b < nb) ? src[b] : (comps[h] == 1 ? (unsigned long long)kNoRow : 0ull);
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if (comps[h] == 1) acc[h] = min(acc[h], x[h][i]);
          else if (isfs[h]) acc[h] = as_u64(as_f64(acc[h]) + as_f64(x[h][i]));
          else acc[h] += x[h][i];
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pair = pair0 + h * nwaves;
      unsigned long long v;
      if (comps[h] == 1) {
        uint32_t m = (uint32_t)acc[h];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o, 64));
        v = m;
      } else if (isfs[h]) {
        double xx = as_f64(acc[h]);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) xx += __shfl_xor(xx, o, 64);
        v = as_u64(xx);
      } else {
        unsigned long long xx = acc[h];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) xx += (unsigned long long)__shfl_xor((long long)xx, o, 64);
        v = xx;
      }
      if (lane == 0 && pair < P) tot[pair] = v;
    }
  }
  __syncthreads();
  if (tid < 64) {
    FinishParams g = f;
    g.totals = tot;  // the finish step reads the totals from LDS
    private_finish_body(g, sa, es, tid);
  }
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
      // in LDS, not registers: emit_slot indexes the sums by state (a dynamic index into a
      // register array is a scratch-memory round trip per access)
      __shared__ SlotTotals st_all[kMaxPrivateSlots];
      SlotTotals& t = st_all[s];
      t.cnt = tot[s];
      t.fst = first;
#pragma unroll
      for (int q = 0; q < kMaxSums; ++q) {
        t.acc[q] = (q < nsum) ? tot[(2 + q) * S + s] : 0ull;
        t.acc2[q] = 0ull;
      }
      emit_slot_private(e, (uint64_t)s, rank, t);
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
  // no system-scope fence: the host reads a pinned result only after hipStreamSynchronize,
  // whose completion covers the kernel's writes (the fence cost ~3.4 us of a ~8 us finish,
  // tools/micro/reduce_micro.hip)
}

void launch_scan_private(const ScanParams& p, const PrivateLaunch& l, hipStream_t st) {
  BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scan_private<NC>), dim3(l.blocks), dim3(kBlock), l.lds_bytes, st, p, l));
}

void launch_private_finish(const FinishParams& f, const SlotArrays& s, const EmitParams& e, hipStream_t st) {
  hipLaunchKernelGGL(k_private_reduce, dim3(1), dim3(kPrivReduceThreads), 0, st, f, s, e);
}

}  // namespace bqg
