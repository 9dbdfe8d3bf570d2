// k_distinct.hip -- count_distinct and sorted_count_distinct
#include <hip/hip_runtime.h>

#include <algorithm>

#include "scd.h"

namespace bqg {

// ------------------------------------------------------------------------------------
// count_distinct: set of (slot, value code) pairs; a bit per pair when the pair space is
// small (LDS pre-filter + HBM bitmap), else an open-addressing set of packed pairs.
// ------------------------------------------------------------------------------------
template <int NC, bool HASH>
__global__ __launch_bounds__(kBlock, 4) void k_count_distinct(ScanParams p, SlotArrays sa, DistinctLaunch d) {
  extern __shared__ __align__(16) unsigned char smem[];
  unsigned int* lbits = reinterpret_cast<unsigned int*>(smem);
  const int tid = threadIdx.x;
  for (int i = tid; i < d.lds_bitmap_words; i += kBlock) lbits[i] = 0;
  __syncthreads();
  const uint64_t hmask = p.nslots - 1;
  const int64_t ntiles = (p.nrows + kTileRows - 1) / kTileRows;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t row0 = tile * kTileRows + (int64_t)tid * kRowsPerThread;
    Chunk raw[NC];
    load_rows4<NC>(p, row0, raw);
    uint64_t v[NC][4];
    decode_all<NC, 4>(p, raw, v);
    const uint32_t pass = vals_pass<NC, 4>(p, row0, v);
    uint64_t code[4];
    vals_code<NC, 4>(p, v, code);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (!(pass & (1u << r))) continue;
      uint64_t s = code[r];
      if (HASH) {
        s = slot_lookup<NC, 4>(p, sa, hmask, v, code, r, (uint32_t)(row0 + r), false);
        if (s == kEmpty) continue;
      }
      uint64_t vcode = 0;
      bool vfloat = false;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (d.vcol == c) {
          const int dt = p.cols[c].dtype;
          vfloat = dtype_is_float(dt);
          vcode = vfloat ? canon_f64_bits(v[c][r]) : v[c][r] - (uint64_t)d.vmin;
        }
      if (d.pair_rows) {
        // vmin == 0 here: vcode is the value's full canonical identity
        const uint32_t row = (uint32_t)(row0 + r);
        const unsigned long long mine = (s << 32) | row;
        uint64_t pos = mix64(vcode ^ mix64(s + 0x9E3779B97F4A7C15ull)) & d.set_mask;
        for (uint64_t i = 0; i <= d.set_mask; ++i) {
          unsigned long long k = d.set[pos];
          if (k == kEmpty) {
            const unsigned long long prev = atomicCAS(&d.set[pos], kEmpty, mine);
            if (prev == kEmpty) {
              atomicAdd(&d.out[s], 1ull);
              const unsigned int f = atomicAdd(d.set_fill, 1u);
              if ((uint64_t)(f + 1) * 2 > d.set_mask + 1) atomicOr(d.overflow, 1u);
              break;
            }
            k = prev;
          }
          if ((k >> 32) == s) {
            const uint32_t rep = (uint32_t)k;
            uint64_t rv = 0;
#pragma unroll
            for (int c = 0; c < NC; ++c)
              if (d.vcol == c) rv = key_at_row(p.cols[c], vfloat, rep);
            if (rv == vcode) break;
          }
          pos = (pos + 1) & d.set_mask;
          if (i == d.set_mask) atomicOr(d.overflow, 1u);
        }
        continue;
      }
      if (d.bitmap) {
        const uint64_t bit = s * d.vrange + vcode;
        const unsigned int m = 1u << (bit & 31);
        if (d.lds_bitmap_words > 0) {
          if (!(lbits[bit >> 5] & m)) atomicOr(&lbits[bit >> 5], m);  // merged into the device bitmap at the end
          continue;
        }
        if (d.bitmap[bit >> 5] & m) continue;
        if (!(atomicOr(&d.bitmap[bit >> 5], m) & m)) atomicAdd(&d.out[s], 1ull);
      } else {
        const uint64_t key = s * d.vrange + vcode;
        uint64_t pos = mix64(key) & d.set_mask;
        for (uint64_t i = 0; i <= d.set_mask; ++i) {
          const unsigned long long k = d.set[pos];
          if (k == key) break;
          if (k == kEmpty) {
            const unsigned long long prev = atomicCAS(&d.set[pos], kEmpty, (unsigned long long)key);
            if (prev == kEmpty) {
              atomicAdd(&d.out[s], 1ull);
              const unsigned int f = atomicAdd(d.set_fill, 1u);
              if ((uint64_t)(f + 1) * 2 > d.set_mask + 1) atomicOr(d.overflow, 1u);
              break;
            }
            if (prev == key) break;
          }
          pos = (pos + 1) & d.set_mask;
          if (i == d.set_mask) atomicOr(d.overflow, 1u);
        }
      }
    }
  }
  // merge the workgroup's pair bitmap; every pair bit it sets first counts once for its slot
  if (d.bitmap && d.lds_bitmap_words > 0) {
    __syncthreads();
    for (int i = tid; i < d.lds_bitmap_words; i += kBlock) {
      const unsigned int word = lbits[i];
      if (!word) continue;
      unsigned int fresh = word & ~atomicOr(&d.bitmap[i], word);
      while (fresh) {
        const int b = __ffs(fresh) - 1;
        fresh &= fresh - 1u;
        atomicAdd(&d.out[((uint64_t)i * 32 + (uint64_t)b) / d.vrange], 1ull);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// sorted_count_distinct: each wave walks a contiguous chunk of rows 64 at a time and keeps
// per-slot (first row, first value, last value, changes) for its chunk; runs of one slot
// inside a 64-row step are resolved with ballots, so the whole chunk is processed in row
// order.  Chunk states are then combined in chunk order (k_scd_combine).
// ------------------------------------------------------------------------------------

constexpr int kScdU = 4;

template <int NC, bool HASH>
__global__ __launch_bounds__(kBlock, 4) void k_scd(ScanParams p, SlotArrays sa, ScdLaunch d) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int S = (int)p.nslots;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int w = blockIdx.x * (kBlock / 64) + wave;
  uint32_t* fr;
  unsigned long long *fv, *lv;
  uint32_t* ch;
  if (d.lds_state) {
    unsigned char* base = smem + (size_t)wave * S * 24;
    fv = reinterpret_cast<unsigned long long*>(base);
    lv = fv + S;
    fr = reinterpret_cast<uint32_t*>(lv + S);
    ch = fr + S;
    for (int i = lane; i < S; i += 64) {
      fr[i] = kNoRow;
      ch[i] = 0;
    }
  } else {
    fr = d.st_first_row + (size_t)w * S;
    fv = d.st_first + (size_t)w * S;
    lv = d.st_last + (size_t)w * S;
    ch = d.st_changes + (size_t)w * S;
  }
  if (w >= d.waves) return;
  const int64_t start = (int64_t)w * d.chunk_rows;
  int64_t end = start + d.chunk_rows;
  if (end > p.nrows) end = p.nrows;
  int vc = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (d.vcol == c) vc = c;
  const bool isf = dtype_is_float(p.cols[vc].dtype);
  const uint64_t hmask = p.nslots - 1;
  // Rows are consumed 64 at a time in row order, but loaded kScdU steps (kScdU x 64 rows) at
  // once and one group ahead, so every wave keeps 2 x kScdU x NC loads in flight instead of
  // waiting out one HBM round trip per 64-row step.
  uint2 cur[kScdU][NC], nxt[kScdU][NC];
  auto issue = [&](int64_t b, uint2 (&dst)[kScdU][NC]) {
#pragma unroll
    for (int u = 0; u < kScdU; ++u) {
      int64_t r = b + 64 * u + lane;
      r = r < end ? r : (end > start ? end - 1 : start);
#pragma unroll
      for (int c = 0; c < NC; ++c) dst[u][c] = load_row_word(p.cols[c], r);
    }
  };
  if (start < end) issue(start, cur);
  for (int64_t gbase = start; gbase < end; gbase += 64 * kScdU) {
    if (gbase + 64 * kScdU < end) issue(gbase + 64 * kScdU, nxt);
#pragma unroll
    for (int u = 0; u < kScdU; ++u) {
      const int64_t row = gbase + 64 * u + lane;
      bool act = false;
      uint64_t slot = 0, vb = 0;
      if (row < end) {
        Chunk raw[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) row_word_to_chunk(raw[c], p.cols[c], row, cur[u][c]);
        uint64_t v[NC][1];
        decode_all<NC, 1>(p, raw, v);
        act = vals_pass<NC, 1>(p, row, v) & 1u;
        uint64_t code[1];
        vals_code<NC, 1>(p, v, code);
        slot = code[0];
        if (HASH && act) {
          slot = slot_lookup<NC, 1>(p, sa, hmask, v, code, 0, (uint32_t)row, false);
          if (slot == kEmpty) act = false;
        }
#pragma unroll
        for (int c = 0; c < NC; ++c)
          if (vc == c) vb = v[c][0];
      }
      // Lanes sharing this lane's slot, from one ballot per slot bit (cost independent of how
      // many distinct slots the 64-row step holds).
      const uint64_t actm = __ballot(act);
      if (actm == 0) continue;
      uint64_t match = actm;
      for (int b = 0; b < d.slot_bits; ++b) {
        const bool bit = (slot >> b) & 1ull;
        const uint64_t bb = __ballot(act && bit);
        match &= bit ? bb : ~bb;
      }
      const uint64_t self = 1ull << lane;
      const uint64_t below = match & (self - 1ull);
      const uint64_t above = match & ~((self - 1ull) | self);
      const int pl = below ? 63 - __clzll((long long)below) : lane;
      const uint64_t pv = __shfl(vb, pl, 64);  // previous row of the same slot in this step
      const bool is_first = act && below == 0;
      const bool is_last = act && above == 0;
      bool diff = act && below != 0 && !scd_equal(vb, pv, isf);
      if (is_first) {
        // the slot's previous row lies in an earlier step of this chunk (or none)
        if (fr[slot] == kNoRow) {
          fr[slot] = (uint32_t)row;
          fv[slot] = vb;
        } else {
          diff = !scd_equal(lv[slot], vb, isf);
        }
      }
      const uint64_t dm = __ballot(diff);
      if (is_first) {
        const unsigned int n = (unsigned int)__popcll(dm & match);
        if (n) ch[slot] += n;
      }
      if (is_last) lv[slot] = vb;  // after every first-lane read of lv (program order)
    }
#pragma unroll
    for (int u = 0; u < kScdU; ++u)
#pragma unroll
      for (int c = 0; c < NC; ++c) cur[u][c] = nxt[u][c];
  }
  if (d.lds_state) {
    for (int i = lane; i < S; i += 64) {
      d.st_first_row[(size_t)w * S + i] = fr[i];
      d.st_first[(size_t)w * S + i] = fv[i];
      d.st_last[(size_t)w * S + i] = lv[i];
      d.st_changes[(size_t)w * S + i] = ch[i];
    }
  }
}


// k_scd_fused: sorted_count_distinct + per-slot rows / first rows (+ one count_distinct) in
// one pass -- body in scd.h
template <int NC, bool COMPACT, bool RUNS = false>
__global__ __launch_bounds__(kBlock) void k_scd_fused(ScanParams p, ScdLaunch d) {
  extern __shared__ __align__(16) unsigned char smem[];
  scd_fused_body<NC, COMPACT, RUNS>(p, d, smem);
}

// (ScdState / scd_combine: scd.h, shared with the fused pass's in-workgroup fold)
__device__ __forceinline__ ScdState scd_load(const ScdLaunch& d, size_t idx, bool valid) {
  ScdState x;
  x.first_row = d.st_first_row[idx];
  x.present = valid && x.first_row != kNoRow;
  x.first = d.st_first[idx];
  x.last = d.st_last[idx];
  x.changes = d.st_changes[idx];
  x.rows = d.st_count ? d.st_count[idx] : 0u;
  return x;
}

__device__ __forceinline__ void scd_store_final(const ScdLaunch& d, uint64_t s, const ScdState& t) {
  d.out_changes[s] = t.changes;
  d.out_first[s] = t.first;
  if (d.slot_cnt) {
    d.slot_cnt[s] = t.present ? t.rows : 0ull;
    d.slot_fst[s] = t.present ? t.first_row : kNoRow;
  }
}

// Stage 1 of the chunk combine: one thread per (slot, run of `per` consecutive chunks);
// consecutive threads take consecutive slots, so every load of a wave is one coalesced row
// segment of the [chunk][slot] state arrays.  The run's combined state is written back in
// place over the run's first chunk (no other thread reads that run).
__global__ __launch_bounds__(kBlock) void k_scd_combine_runs(ScdLaunch d, uint64_t nslots, int per, int runs,
                                                          int isf) {
  const uint64_t item = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (item >= nslots * (uint64_t)runs) return;
  const uint64_t s = item % nslots;
  const int g = (int)(item / nslots);
  const int beg = g * per, end = min(d.waves, beg + per);
  ScdState st = {0, kNoRow, 0, 0, 0, 0};
  constexpr int kU = 8;
  for (int w0 = beg; w0 < end; w0 += kU) {
    ScdState x[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) x[k] = scd_load(d, (size_t)min(w0 + k, end - 1) * nslots + s, w0 + k < end);
#pragma unroll
    for (int k = 0; k < kU; ++k) st = scd_combine(st, x[k], isf);
  }
  if (runs == 1) {  // the run is the whole slot: final values
    scd_store_final(d, s, st);
    return;
  }
  const size_t o = (size_t)beg * nslots + s;
  d.st_first_row[o] = st.present ? st.first_row : kNoRow;
  d.st_first[o] = st.first;
  d.st_last[o] = st.last;
  d.st_changes[o] = (uint32_t)st.changes;
  if (d.st_count) d.st_count[o] = (uint32_t)st.rows;
}

// Stage 2: one workgroup per slot over the `runs` run states (chunk rows 0, per, 2 per, ...):
// each of its 4 waves takes a contiguous quarter, each lane a contiguous part of that quarter
// (loads clamped, not branched, so they pipeline), an ordered shuffle tree folds the lanes,
// and the 4 wave results are folded in order.
__global__ __launch_bounds__(kBlock) void k_scd_combine(ScdLaunch d, uint64_t nslots, int per, int runs, int isf) {
  __shared__ ScdState part[kBlock / 64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nw = kBlock / 64;
  for (uint64_t s = blockIdx.x; s < nslots; s += gridDim.x) {
  const int wbeg = (int)((int64_t)runs * wave / nw), wend = (int)((int64_t)runs * (wave + 1) / nw);
  const int span = wend - wbeg;
  const int lper = (span + 63) / 64;
  const int lbeg = wbeg + min(span, lane * lper), lend = wbeg + min(span, (lane + 1) * lper);
  ScdState st = {0, kNoRow, 0, 0, 0, 0};
  constexpr int kU = 4;  // run states loaded per round (clamped, all in flight at once)
  for (int w0 = lbeg; w0 < lend; w0 += kU) {
    ScdState x[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) x[k] = scd_load(d, (size_t)min(w0 + k, lend - 1) * per * nslots + s, w0 + k < lend);
#pragma unroll
    for (int k = 0; k < kU; ++k) st = scd_combine(st, x[k], isf);
  }
  for (int o = 1; o < 64; o <<= 1) {
    ScdState other;
    other.present = __shfl_down(st.present, o, 64);
    other.first_row = __shfl_down(st.first_row, o, 64);
    other.first = __shfl_down(st.first, o, 64);
    other.last = __shfl_down(st.last, o, 64);
    other.changes = __shfl_down(st.changes, o, 64);
    other.rows = __shfl_down(st.rows, o, 64);
    if ((lane % (2 * o)) == 0 && lane + o < 64) st = scd_combine(st, other, isf);
  }
  if (lane == 0) part[wave] = st;
  __syncthreads();
  if (threadIdx.x == 0) {
    ScdState t = part[0];
    for (int q = 1; q < nw; ++q) t = scd_combine(t, part[q], isf);
    scd_store_final(d, s, t);
  }
  __syncthreads();  // part[] is rewritten for the next slot
  }
}

void launch_count_distinct(const ScanParams& p, const SlotArrays& s, const DistinctLaunch& d, int blocks,
                           hipStream_t st) {
  const size_t lds = (size_t)d.lds_bitmap_words * 4;
  if (p.hash) {
    BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_count_distinct<NC, true>), dim3(blocks), dim3(kBlock), lds, st, p, s, d));
  } else {
    BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_count_distinct<NC, false>), dim3(blocks), dim3(kBlock), lds, st, p, s, d));
  }
}
void launch_scd(const ScanParams& p, const SlotArrays& s, const ScdLaunch& d, hipStream_t st, hipFunction_t fused_fn,
                hipEvent_t pass_done) {
  const int blocks = (d.waves + (kBlock / 64) - 1) / (kBlock / 64);
  if (d.fused) {
    const size_t lds = (kBlock / 64) * d.wave_lds + (size_t)d.cd.lds_bitmap_words * 4;
    if (fused_fn) {
      void* args[] = {(void*)&p, (void*)&d};
      (void)hipModuleLaunchKernel(fused_fn, (unsigned)blocks, 1, 1, kBlock, 1, 1, (unsigned)lds, st, args, nullptr);
    } else {
      if (d.compact && d.runs) {
        BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scd_fused<NC, true, true>), dim3(blocks), dim3(kBlock), lds, st, p, d));
      } else if (d.compact) {
        BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scd_fused<NC, true>), dim3(blocks), dim3(kBlock), lds, st, p, d));
      } else {
        BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scd_fused<NC, false>), dim3(blocks), dim3(kBlock), lds, st, p, d));
      }
    }
  } else {
    const size_t lds = d.lds_state ? (size_t)(kBlock / 64) * p.nslots * 24 : 0;
    if (p.hash) {
      BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scd<NC, true>), dim3(blocks), dim3(kBlock), lds, st, p, s, d));
    } else {
      BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scd<NC, false>), dim3(blocks), dim3(kBlock), lds, st, p, s, d));
    }
  }
  if (pass_done) (void)hipEventRecord(pass_done, st);
  int isf = 0;
  for (int c = 0; c < p.ncols; ++c)
    if (c == d.vcol) isf = dtype_is_float(p.cols[c].dtype);
  // the fused pass folds its workgroup's waves and flushes one state per workgroup: `blocks`
  // chunks; the per-wave pass flushes one per wave
  ScdLaunch dc = d;
  if (d.fused) dc.waves = blocks;
  // stage 1: ~2 threads per CU lane over (slot, run of chunks); stage 2 folds the runs per slot
  const uint64_t S = p.nslots;
  const uint64_t target = (uint64_t)device_cu_count() * kBlock * 2;
  uint64_t want = (target + S - 1) / S;
  if (want > (uint64_t)dc.waves) want = (uint64_t)dc.waves;
  if (want < 1) want = 1;
  int per = (int)(((uint64_t)dc.waves + want - 1) / want);
  // few slots: runs of up to 16 chunks, >= 64 runs per slot -- stage 2 then folds one or two
  // runs per lane (C4's 1792 chunks x 265 slots: 19.2 + 15.8 us at 16 chunks a run, 30.3 + 13.3
  // at 28, 15.4 + 21.8 at 8, profiles/r6bc_c4_combine_sweep.txt; 20.5 + 34.0 at 4, r5s_)
  if (per < 16 && dc.waves > 64 * per) per = std::min(16, (int)((dc.waves + 63) / 64));
  const int runs = (int)(((uint64_t)dc.waves + per - 1) / per);
  const uint64_t items = S * (uint64_t)runs;
  hipLaunchKernelGGL(k_scd_combine_runs, dim3((unsigned)((items + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, dc, S,
                     per, runs, isf);
  if (runs > 1) {
    const uint64_t cblocks = S < 65536 ? S : 65536;  // grid-stride over slots beyond
    hipLaunchKernelGGL(k_scd_combine, dim3((unsigned)cblocks), dim3(kBlock), 0, st, dc, S, per, runs, isf);
  }
}
}  // namespace bqg
