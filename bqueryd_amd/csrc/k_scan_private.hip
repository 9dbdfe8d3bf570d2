// k_scan_private.hip -- private-LDS fused scan (hot path of the low-cardinality groupby)
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device.h"

namespace bqg {

// ------------------------------------------------------------------------------------
// PRIVATE mode: every lane owns a private accumulator row per slot in LDS ([slot][lane]
// layout: conflict-free ds_read/ds_write, no atomics).  Used for small dense slot spaces
// (the filtered low-cardinality groupby of config C2).
// ------------------------------------------------------------------------------------
template <int NC>
__global__ __launch_bounds__(kBlock) void k_scan_private(ScanParams p, SlotArrays sa, PrivateLaunch L, EmitParams e) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int S = (int)p.nslots;
  const int tid = threadIdx.x;
  const int nsum = p.nsum;
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem);          // [nsum][S][256]
  uint32_t* cnt = reinterpret_cast<uint32_t*>(acc + (size_t)nsum * S * kBlock);   // [S][256]
  uint32_t* fst = cnt + S * kBlock;                                                // [S][256]
  for (int s = 0; s < S; ++s) {
    cnt[s * kBlock + tid] = 0;
    fst[s * kBlock + tid] = kNoRow;
  }
  for (int i = 0; i < nsum * S; ++i) acc[i * kBlock + tid] = 0;

  const int64_t ntiles = (p.nrows + kTileRows - 1) / kTileRows;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t row0 = tile * kTileRows + (int64_t)tid * kRowsPerThread;
    Chunk raw[NC];
    load_rows4<NC>(p, row0, raw);
    const uint32_t pass = rows_pass<NC, 4>(p, row0, raw);
    uint64_t code[4];
    rows_code<NC, 4>(p, raw, code);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (pass & (1u << r)) {
        const int idx = (int)code[r] * kBlock + tid;
        const uint32_t c0 = cnt[idx];
        if (c0 == 0) fst[idx] = (uint32_t)(row0 + r);
        cnt[idx] = c0 + 1;
#pragma unroll
        for (int v = 0; v < (NC < kMaxSums ? NC : kMaxSums); ++v) {
          if (v < nsum) {
            unsigned long long* a = &acc[(size_t)v * S * kBlock + idx];
            if (p.sum_is_float[v]) {
              double x = chunk_f64(raw[v], p.cols[v].dtype, r);
              if (p.sum_centered[v]) {
                const double d = x - p.centers[v][code[r]];
                x = d * d;
              }
              *a = as_u64(as_f64(*a) + x);
            } else {
              *a += (unsigned long long)chunk_i64(raw[v], p.cols[v].dtype, r);
            }
          }
        }
      }
    }
  }
  __syncthreads();

  // ---- workgroup reduction of the lane-private tables -> partials[comp][block][slot]
  const int wave = tid >> 6, lane = tid & 63;
  const int nb = gridDim.x, b = blockIdx.x;
  for (int s = wave; s < S; s += kBlock / 64) {
    unsigned long long c = 0;
    uint32_t f = kNoRow;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c += cnt[s * kBlock + lane + 64 * j];
      f = min(f, fst[s * kBlock + lane + 64 * j]);
    }
    c = wave_sum_u64(c);
    f = wave_min_u32(f);
    if (lane == 0) {
      L.partials[((size_t)0 * nb + b) * S + s] = c;
      L.partials[((size_t)1 * nb + b) * S + s] = f;
    }
    for (int v = 0; v < nsum; ++v) {
      const unsigned long long* a = &acc[(size_t)v * S * kBlock + s * kBlock];
      unsigned long long out;
      if (p.sum_is_float[v]) {
        double x = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) x += as_f64(a[lane + 64 * j]);
        out = as_u64(wave_sum_f64(x));
      } else {
        unsigned long long x = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) x += a[lane + 64 * j];
        out = wave_sum_u64(x);
      }
      if (lane == 0) L.partials[((size_t)(2 + v) * nb + b) * S + s] = out;
    }
  }

  // ---- last-arriving workgroup combines the partials (Guideline 16 release/acquire)
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned int ticket = atomicAdd(L.done_counter, 1u);
    s_last = (ticket == (unsigned int)nb - 1u);
  }
  __syncthreads();
  if (!s_last) return;
  if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int P = (2 + nsum) * S;
  int tpp = 1;
  while (tpp * 2 * P <= kBlock) tpp *= 2;
  const int ppr = kBlock / tpp;  // pairs per round
  unsigned long long* red = reinterpret_cast<unsigned long long*>(smem);  // [256]
  unsigned long long* tot = red + kBlock;                                  // [P]
  for (int base = 0; base < P; base += ppr) {
    const int pair = base + tid / tpp, j = tid % tpp;
    const int comp = pair / S, s = pair % S;
    const bool isf = comp >= 2 && pair < P && p.sum_is_float[comp - 2];
    unsigned long long v = (comp == 1) ? (unsigned long long)kNoRow : 0ull;
    if (pair < P) {
      if (comp == 1) {
        uint32_t f = kNoRow;
        for (int bb = j; bb < nb; bb += tpp) f = min(f, (uint32_t)L.partials[((size_t)comp * nb + bb) * S + s]);
        v = f;
      } else if (isf) {
        double x = 0.0;
        for (int bb = j; bb < nb; bb += tpp) x += as_f64(L.partials[((size_t)comp * nb + bb) * S + s]);
        v = as_u64(x);
      } else {
        unsigned long long x = 0;
        for (int bb = j; bb < nb; bb += tpp) x += L.partials[((size_t)comp * nb + bb) * S + s];
        v = x;
      }
    }
    red[tid] = v;
    __syncthreads();
    for (int w = tpp / 2; w >= 1; w >>= 1) {
      if (j < w && pair < P) {
        const unsigned long long o = red[tid + w];
        if (comp == 1) red[tid] = min(red[tid], o);
        else if (isf) red[tid] = as_u64(as_f64(red[tid]) + as_f64(o));
        else red[tid] = red[tid] + o;
      }
      __syncthreads();
    }
    if (j == 0 && pair < P) tot[pair] = red[tid];
    __syncthreads();
  }

  if (!L.emit_inline) {
    for (int i = tid; i < P; i += kBlock) {
      const int comp = i / S, s = i % S;
      if (comp == 0) sa.cnt[s] = tot[i];
      else if (comp == 1) sa.fst[s] = (uint32_t)tot[i];
      else sa.acc[(size_t)(comp - 2) * p.nslots + s] = tot[i];
    }
    if (tid == 0) *L.done_counter = 0u;
    return;
  }
  // inline emit: rank occupied slots by first row (S is small)
  if (tid < S) {
    const int s = tid;
    if (tot[s] > 0) {
      const uint32_t f = (uint32_t)tot[S + s];
      unsigned int rank = 0;
      for (int q = 0; q < S; ++q)
        if (tot[q] > 0 && (uint32_t)tot[S + q] < f) ++rank;
      SlotTotals t;
      t.cnt = tot[s];
      t.fst = f;
#pragma unroll
      for (int v = 0; v < kMaxSums; ++v) {
        t.acc[v] = (v < nsum) ? tot[(2 + v) * S + s] : 0ull;
        t.acc2[v] = 0ull;
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
    L.out_hdr[0] = g;
    L.out_hdr[1] = total;
    *L.done_counter = 0u;
  }
}

void launch_scan_private(const ScanParams& p, const SlotArrays& s, const PrivateLaunch& l, const EmitParams& e,
                         hipStream_t st) {
  BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scan_private<NC>), dim3(l.blocks), dim3(kBlock), l.lds_bytes, st, p, s, l, e));
}
}  // namespace bqg
