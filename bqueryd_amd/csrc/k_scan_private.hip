// k_scan_private.hip -- private-LDS fused scan: the hot path of the filtered
// low-cardinality groupby (config C2: bqueryd/worker.py:303 + :313 in one pass).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device.h"

namespace bqg {

// Every lane owns a private accumulator row per slot in LDS, laid out [slot][lane] so that
// the per-row read-modify-writes are conflict-free ds_read/ds_write with no atomics.  Rows
// of a lane are processed in increasing order, so its first write to a slot is that slot's
// first row for the lane.  A workgroup streams tiles of 1024 rows (4 per lane, one 16-byte
// load per 4-byte column) and prefetches the next tile while it aggregates the current one.
template <int NC>
__global__ __launch_bounds__(kBlock, 4) void k_scan_private(ScanParams p, PrivateLaunch L) {
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
  int64_t tile = blockIdx.x;
  Chunk raw[NC];
  if (tile < ntiles) load_rows4<NC>(p, tile * kTileRows + (int64_t)tid * kRowsPerThread, raw);
  for (; tile < ntiles; tile += gridDim.x) {
    const int64_t row0 = tile * kTileRows + (int64_t)tid * kRowsPerThread;
    uint64_t v[NC][4];
    decode_all<NC, 4>(p, raw, v);
    const int64_t next = tile + gridDim.x;
    if (next < ntiles) load_rows4<NC>(p, next * kTileRows + (int64_t)tid * kRowsPerThread, raw);
    const uint32_t pass = vals_pass<NC, 4>(p, row0, v);
    uint64_t code[4];
    vals_code<NC, 4>(p, v, code);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (pass & (1u << r)) {
        const int idx = (int)code[r] * kBlock + tid;
        const uint32_t c0 = cnt[idx];
        if (c0 == 0) fst[idx] = (uint32_t)(row0 + r);
        cnt[idx] = c0 + 1;
#pragma unroll
        for (int s = 0; s < (NC < kMaxSums ? NC : kMaxSums); ++s) {
          if (s < nsum) {
            unsigned long long* a = &acc[(size_t)s * S * kBlock + idx];
            if (p.sum_is_float[s]) {
              double x = value_f64(v[s][r], p.sum_conv[s]);
              if (p.sum_centered[s]) {
                const double d = x - p.centers[s][code[r]];
                x = d * d;
              }
              *a = as_u64(as_f64(*a) + x);
            } else {
              *a += v[s][r];
            }
          }
        }
      }
    }
  }
  __syncthreads();

  // workgroup reduction of the lane-private tables -> partials[comp][slot][block]
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
      L.partials[((size_t)0 * S + s) * nb + b] = c;
      L.partials[((size_t)1 * S + s) * nb + b] = f;
    }
    for (int q = 0; q < nsum; ++q) {
      const unsigned long long* a = &acc[(size_t)q * S * kBlock + s * kBlock];
      unsigned long long out;
      if (p.sum_is_float[q]) {
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
      if (lane == 0) L.partials[((size_t)(2 + q) * S + s) * nb + b] = out;
    }
  }
}

// One workgroup per (component, slot): sums / mins that slot's per-workgroup partials in a
// fixed order (coalesced reads, fixed LDS tree: bitwise deterministic).
__global__ __launch_bounds__(kBlock) void k_private_reduce(FinishParams f) {
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
  if (tid == 0) f.totals[pair] = red[0];
}

// Emits the groups in first-appearance order (S is small: rank by counting), or stores the
// per-slot totals for the generic emit path.
__global__ __launch_bounds__(64) void k_private_finish(FinishParams f, SlotArrays sa, EmitParams e) {
  const int tid = threadIdx.x;
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
}

void launch_scan_private(const ScanParams& p, const PrivateLaunch& l, hipStream_t st) {
  BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scan_private<NC>), dim3(l.blocks), dim3(kBlock), l.lds_bytes, st, p, l));
}

void launch_private_finish(const FinishParams& f, const SlotArrays& s, const EmitParams& e, hipStream_t st) {
  hipLaunchKernelGGL(k_private_reduce, dim3((2 + f.nsum) * f.nslots), dim3(kBlock), 0, st, f);
  hipLaunchKernelGGL(k_private_finish, dim3(1), dim3(64), 0, st, f, s, e);
}

}  // namespace bqg
