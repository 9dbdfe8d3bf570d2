// scd.h -- body of the fused sorted_count_distinct pass (config C4), shared by the
// precompiled kernel (k_distinct.hip) and the query-specialised JIT kernel (jit_kernels.h).
//
// sorted_count_distinct counts, per group and in row order, the rows whose value differs
// from the previous row OF THE SAME GROUP (bquery's `last[g]` loop, with its zero-initialised
// `last` and first-row rule applied at emit).  Each wave owns a contiguous chunk of rows and
// consumes it 64 rows per step in row order, one row per lane (coalesced 4- or 8-byte loads,
// kScdAhead steps in flight).  Inside a step the lanes of one slot find each other through a
// per-slot 64-bit lane mask in wave-private LDS (every lane ORs its bit, then reads the word
// back); the previous row of a slot inside the step is the
// highest lower lane of its match mask (one bpermute); the slot's first lane in the step
// folds the whole step into the per-slot state {last, first, rows, changes, first row} in LDS
// with one read and one write.  Per-slot row counts and first rows come out of the same pass
// (so count / distinct-only queries need no other scan), and one count_distinct over a small
// (slot, value) space is folded in through a per-workgroup LDS pair bitmap that is merged
// into the device-wide bitmap once, at the end of the workgroup.  Chunk states are combined in chunk order by k_scd_combine.
#pragma once

#include "device.h"

namespace bqg {

// Per-slot chunk state.  Wide: 64-bit value bits (floats, or integer value spaces of 2^32 and
// more).  Compact: 32-bit value codes (v - vmin), so that a slot's state is 16 bytes plus its
// first row and twice as many waves fit in LDS.
struct __align__(16) ScdSlot {
  unsigned long long last;   // value bits of the slot's last row so far
  unsigned long long first;  // value bits of the slot's first row in the chunk
  uint32_t rows;             // rows of the slot in the chunk (0: absent)
  uint32_t changes;          // value changes between consecutive rows of the slot
  uint32_t first_row;
  uint32_t pad;
};
// Compact: 8 bytes of hot state per slot -- the first lane of a slot in a step reads and
// writes it with one ds_read_b64 / ds_write_b64 -- rows and changes as 16-bit halves of `rc`
// (chunks of at most kScdCompactMaxRows rows); the first value and first row live apart
// (written once per slot and chunk).
struct __align__(8) ScdSlot32 {
  uint32_t last;  // value code of the slot's last row so far
  uint32_t rc;    // rows (bits 0-15) | changes (bits 16-31)
};

constexpr int kScdAhead = 4;  // 64-row steps loaded ahead of the one being folded

__device__ __forceinline__ bool scd_equal(uint64_t a, uint64_t b, bool isf) {
  return isf ? (as_f64(a) == as_f64(b)) : (a == b);
}

// One chunk's state of one slot as the chunk combine folds it (k_distinct.hip): two
// consecutive chunks fold as rows and changes added, plus one change where the first chunk's
// last value differs from the second's first.
struct ScdState {
  uint32_t present;
  uint32_t first_row;
  unsigned long long first, last, changes, rows;
};

__device__ __forceinline__ ScdState scd_combine(const ScdState& a, const ScdState& b, bool isf) {
  if (!a.present) return b;
  if (!b.present) return a;
  ScdState r;
  r.present = 1;
  r.first_row = a.first_row;
  r.rows = a.rows + b.rows;
  r.first = a.first;
  r.last = b.last;
  r.changes = a.changes + b.changes + (scd_equal(a.last, b.first, isf) ? 0ull : 1ull);
  return r;
}

// Row loads of one 64-row step: rows are addressed relative to the wave's chunk (32-bit lane
// offsets from a uniform base, so the address math is one VALU op per column), 4- and 8-byte
// columns load their element directly, narrower ones the aligned 8-byte word holding it.
template <int NC>
__device__ __forceinline__ void scd_issue(const ScanParams& p, int64_t start, uint32_t rb, uint32_t nrel, int lane,
                                          uint2 (&dst)[NC]) {
  uint32_t r = rb + (uint32_t)lane;
  r = r < nrel ? r : nrel - 1;  // lanes past the chunk re-read its last row (nrel > 0)
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const DevCol& col = p.cols[c];
    // a chunk spans < 2^29 rows (nrows < 2^32, >= 64 waves), so its byte offsets fit 32 bits:
    // the loads use a scalar base plus a 32-bit lane offset
    const unsigned char* base = col.ptr + (start << col.lg);
    if (col.lg == 2) {
      dst[c] = make_uint2(*reinterpret_cast<const uint32_t*>(base + (r << 2)), 0u);
    } else if (col.lg == 3) {
      dst[c] = *reinterpret_cast<const uint2*>(base + (r << 3));
    } else {
      dst[c] = load_row_word(col, start + (int64_t)r);
    }
  }
}

__device__ __forceinline__ void scd_word_to_chunk(Chunk& c, const DevCol& col, int64_t row, uint2 w) {
  if (col.lg >= 2) {
    c.a = make_uint4(w.x, w.y, 0u, 0u);
    c.b = make_uint4(0u, 0u, 0u, 0u);
    c.sh = 0;
  } else {
    row_word_to_chunk(c, col, row, w);
  }
}

// count_distinct pair bit of (slot, value): LDS pre-filter (merged per workgroup) or the
// device bitmap (first setter counts the pair)
__device__ __forceinline__ void scd_cd_pair(const ScdLaunch& d, int cd_mode, unsigned int* cdb, uint32_t s, uint32_t vcd) {
  // 32-bit arithmetic: the planner fuses pair spaces < 2^30 only
  const uint32_t bit = s * (uint32_t)d.cd.vrange + (vcd - (uint32_t)d.cd.vmin);
  const unsigned int m = 1u << (bit & 31);
  if (cd_mode == 1) {
    // read first: lanes of one word broadcast; only a new pair pays the (serialising)
    // same-address atomic
    if (!(cdb[bit >> 5] & m)) atomicOr(&cdb[bit >> 5], m);
  } else if (!(d.cd.bitmap[bit >> 5] & m) && !(atomicOr(&d.cd.bitmap[bit >> 5], m) & m)) {
    atomicAdd(&d.cd.out[s], 1ull);
  }
}

// The RUNS loop of the compact fused pass (see scd_fused_body): 256-row steps of 16-byte loads,
// uniform full steps folded in registers, every other step handed to `fold` as four 64-row
// steps re-read one row per lane (`derive` decodes them like the 64-row loop).
constexpr int kScdRunsAhead = 2;  // 256-row steps loaded ahead of the one being folded
template <int NC, typename Fold, typename Derive>
__device__ __forceinline__ void scd_runs_loop(const ScanParams& p, const ScdLaunch& d, int64_t start, int64_t end,
                                              uint32_t nrel, int lane, int vc, int cc, bool do_cd, bool cd_runs,
                                              int cd_mode, ScdSlot32* st32, uint32_t* fv32, uint32_t* fr32, bool p16,
                                              unsigned int* cdb, Fold& fold, Derive& derive) {
  if (!nrel) return;
  const uint32_t all = (1u << NC) - 1u;
  Chunk ring[kScdRunsAhead][NC];
#pragma unroll
  for (int a = 0; a < kScdRunsAhead; ++a)
    load_rows4_clamped<NC>(p, start + 256 * a + 4 * lane, end, ring[a], all, start);
  for (uint32_t gbase = 0; gbase < nrel; gbase += 256u * kScdRunsAhead) {
#pragma unroll
    for (int a = 0; a < kScdRunsAhead; ++a) {
      const uint32_t rb = gbase + 256u * a;
      const int64_t row0 = start + (int64_t)rb + 4 * lane;
      uint64_t v[NC][4], code[4];
      decode_all<NC, 4>(p, ring[a], v);
      const uint32_t pass = vals_pass<NC, 4, false>(p, row0, v);
      vals_code<NC, 4>(p, v, code);
      uint32_t s[4], vb[4], vcd[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        uint64_t x = 0, y = 0;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if (vc == c) x = v[c][r];
          if (cc == c) y = v[c][r];
        }
        s[r] = (uint32_t)code[r];
        vb[r] = (uint32_t)(x - (uint64_t)d.vmin);
        vcd[r] = (uint32_t)y;
      }
      // derived before the refill (ring[a] dead at the refill, as in the 64-row loop)
      asm volatile("" : "+v"(s[0]), "+v"(s[1]), "+v"(s[2]), "+v"(s[3]), "+v"(vb[0]), "+v"(vb[1]), "+v"(vb[2]),
                   "+v"(vb[3]));
      __builtin_amdgcn_sched_barrier(0);
      load_rows4_clamped<NC>(p, row0 + 256 * kScdRunsAhead, end, ring[a], all, start);
      if (rb >= nrel) continue;
      const int64_t rem = end - row0;
      const uint32_t act4 = pass & (rem >= 4 ? 0xFu : (rem > 0 ? (1u << rem) - 1u : 0u));
      const uint32_t s0 = __builtin_amdgcn_readfirstlane(s[0]);
      const bool uni = __ballot(act4 != 0xFu || s[0] != s0 || s[1] != s0 || s[2] != s0 || s[3] != s0) == 0;
      if (!uni) {
        // a key boundary, a filtered row or the chunk's tail: four 64-row steps in row order
#pragma unroll 1
        for (int t = 0; t < 4; ++t) {
          const uint32_t rbt = rb + 64u * t;
          if (rbt >= nrel) break;
          uint2 w[NC];
          scd_issue<NC>(p, start, rbt, nrel, lane, w);
          const uint32_t rel = rbt + (uint32_t)lane;
          const int64_t row = start + (int64_t)rel;
          bool act;
          uint32_t sl;
          uint64_t x, y;
          derive(w, rel, row, act, sl, x, y);
          fold(rel, row, act, sl, (uint64_t)(uint32_t)(x - (uint64_t)d.vmin), (uint64_t)(uint32_t)y);
        }
        continue;
      }
      // one slot, 256 active rows: value changes inside each lane's 4 rows and across the lane
      // boundary (the lane below's last row: a DPP wave shift)
      const uint32_t pv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)vb[3], 0x138, 0xF, 0xF, false);  // wave_shr:1
      const bool d0 = lane > 0 && vb[0] != pv, d1 = vb[1] != vb[0], d2 = vb[2] != vb[1], d3 = vb[3] != vb[2];
      const uint32_t add_ch = (uint32_t)(__popcll(__ballot(d0)) + __popcll(__ballot(d1)) + __popcll(__ballot(d2)) +
                                         __popcll(__ballot(d3)));
      const uint32_t lastv = (uint32_t)__builtin_amdgcn_readlane(vb[3], 63);
      bool rs0 = d0;  // row 0 of the lane starts a value run of the slot
      if (lane == 0) {
        const ScdSlot32 cur = st32[s0];
        const uint32_t rows = cur.rc & 0xFFFFu;
        uint32_t ch = (cur.rc >> 16) + add_ch;
        if (rows == 0) {
          if (p16) {
            fv32[s0] = (vb[0] & 0xFFFFu) | (rb << 16);
          } else {
            fv32[s0] = vb[0];
            fr32[s0] = (uint32_t)(start + rb);
          }
          rs0 = true;
        } else if (cur.last != vb[0]) {
          ch += 1u;
          rs0 = true;
        }
        st32[s0] = ScdSlot32{lastv, (rows + 256u) | (ch << 16)};
      }
      if (do_cd) {
        const bool rs[4] = {rs0, d1, d2, d3};
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (cd_runs ? rs[r] : true) scd_cd_pair(d, cd_mode, cdb, s0, vcd[r]);
      }
    }
  }
}

// RUNS (compact only): clustered keys (the planner's run count of the key column) -- 256-row
// steps, 4 rows per lane from 16-byte loads.  A step whose 256 rows are all active and carry
// one slot (all but ~one step per key run) is folded without LDS: in-lane value changes, the
// lane boundary's through a DPP shift, four ballots, one state update; any other step is
// folded as four 64-row steps over the same rows re-read one per lane (L1 / L2 hits).
template <int NC, bool COMPACT, bool RUNS = false>
__device__ __forceinline__ void scd_fused_body(const ScanParams& p, const ScdLaunch& d, unsigned char* smem) {
  const int S = (int)p.nslots;
  // wave-uniform in a register the compiler knows to be uniform: the chunk bounds and step
  // counters below become scalar (SALU) instead of per-lane 64-bit VALU arithmetic
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  unsigned char* wbase = smem + (size_t)wave * d.wave_lds;
  ScdSlot* st = reinterpret_cast<ScdSlot*>(wbase);          // wide state [S]
  ScdSlot32* st32 = reinterpret_cast<ScdSlot32*>(wbase);    // compact state [S] ...
#ifdef BQ_SCD_P16
  constexpr bool p16 = BQ_SCD_P16 != 0;
#else
  const bool p16 = d.pack16 != 0;
#endif
  // first value code and first row of each slot in the chunk: two words, or with p16 (value
  // codes and chunk-relative rows below 2^16) one word {code | rel << 16} -- a smaller wave
  // footprint, so more waves fit in LDS
  uint32_t* fv32 = reinterpret_cast<uint32_t*>(st32 + S);   // ... + first value codes [S]
  uint32_t* fr32 = fv32 + S;                                // ... + first rows [S] (not with p16)
  // per-slot lane masks of the current step (after the wide or compact state, 8-aligned)
  unsigned long long* tbl = reinterpret_cast<unsigned long long*>(
      wbase + (COMPACT ? (((size_t)S * (p16 ? 12 : 16) + 7) & ~size_t(7)) : (size_t)S * 32));
  unsigned int* cdb = reinterpret_cast<unsigned int*>(smem + (size_t)(blockDim.x >> 6) * d.wave_lds);
  for (int i = lane; i < S; i += 64) {
    tbl[i] = 0ull;
    if (COMPACT) {
      st32[i] = ScdSlot32{0u, 0u};
      fv32[i] = 0u;
      if (!p16) fr32[i] = kNoRow;
    } else {
      st[i] = ScdSlot{0ull, 0ull, 0u, 0u, kNoRow, 0u};
    }
  }
  // count_distinct mode: 0 none, 1 LDS pair bitmap (merged at the end), 2 device bitmap.  The
  // JIT build fixes it at compile time: a device-bitmap branch in the loop (a load and a
  // returning atomic) would make the compiler drain every prefetched load at each step.
#ifdef BQ_SCD_CD
  constexpr int cd_mode = BQ_SCD_CD;
#else
  const int cd_mode = d.cd.bitmap == nullptr ? 0 : (d.cd.lds_bitmap_words > 0 ? 1 : 2);
#endif
  const bool do_cd = cd_mode != 0;
  for (int i = threadIdx.x; i < d.cd.lds_bitmap_words; i += blockDim.x) cdb[i] = 0u;
  __syncthreads();
  const int w = blockIdx.x * (blockDim.x >> 6) + wave;
  const bool live = w < d.waves;  // every wave stays for the block's final count_distinct flush
  const int64_t start = live ? (int64_t)w * d.chunk_rows : 0;
  const int64_t end = live ? min(start + d.chunk_rows, p.nrows) : 0;
#ifdef BQ_SCD_VC
  // the JIT build fixes the value columns: no per-step select between column registers
  constexpr int vc = BQ_SCD_VC, cc = BQ_SCD_CC;
#else
  int vc = 0, cc = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (d.vcol == c) vc = c;
    if (d.cd.vcol == c) cc = c;
  }
#endif
  const bool isf = !COMPACT && dtype_is_float(p.cols[vc].dtype);
  const bool cd_runs = cc == vc;  // count_distinct of the sorted_count_distinct column
  const uint64_t lanes_below = (1ull << lane) - 1ull;
  // one 64-row step in row order (lane = row - rb): the per-slot lane masks, the previous row of
  // each row's slot, the slot's state update and the count_distinct pairs
  auto fold = [&](uint32_t rel, int64_t row, bool act, uint32_t s, uint64_t vb, uint64_t vcd) {
      const uint64_t actm = __ballot(act);
      if (actm == 0) return;
      // one slot for the whole step (sorted or clustered keys): the active lanes are its lanes,
      // and the LDS mask -- 64 same-address atomics, serialised -- is skipped
      const uint32_t s0 = __builtin_amdgcn_readlane(s, (uint32_t)__builtin_ctzll(actm));
      const bool uni = __ballot(act && s != s0) == 0;
      uint64_t match;
      if (uni) {
        match = act ? actm : 0ull;
      } else {
        // lanes of this lane's slot: every lane ORs its bit into the slot's LDS mask word, then
        // reads the word back (a wave's LDS instructions execute in program order; OR does not
        // depend on the order of the lanes); the slot's first lane clears it below
        // (32-bit ORs into the word's half of this lane's half-wave: the lanes of a hot slot
        // -- same-address atomics, serialised -- split over two addresses)
        if (act) atomicOr(reinterpret_cast<unsigned int*>(&tbl[s]) + (lane >> 5), 1u << (lane & 31));
        match = act ? tbl[s] : 0ull;
      }
      const uint64_t below = match & lanes_below;
      uint64_t pv, lastv = 0;
      if (COMPACT) {
        // compact state: with several slots in the step, each slot's last lane stores `last`
        // itself (below), so no lane needs the slot's last value -- only its previous row's;
        // with one slot, the last value is a scalar read and the first lane stores it
        if (uni && (actm & (actm + 1)) == 0) {
          // one slot on lanes 0..k: the previous row is the lane below (a DPP wave shift, no LDS)
          pv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)vb, 0x138, 0xF, 0xF, false);  // wave_shr:1
        } else {
          // previous row of the slot in this step: lane 63 - clz(below), as the byte address
          // (~clz) << 2 (ds_bpermute takes the lane from address bits 7..2); with below == 0 it
          // reads an arbitrary lane, which `diff` below ignores
          const uint32_t lz = (uint32_t)__clzll((long long)below);
          pv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(~lz << 2), (int)(uint32_t)vb);
        }
        if (uni) lastv = (uint32_t)__builtin_amdgcn_readlane((uint32_t)vb, 63 - __clzll((long long)actm));
      } else {
        const int pl = below ? 63 - __clzll((long long)below) : lane;
        const int hl = (act && match) ? 63 - __clzll((long long)match) : lane;
        pv = __shfl(vb, pl, 64);
        lastv = __shfl(vb, hl, 64);  // last row of the slot in this step
      }
      const bool diff = act && below != 0 && !scd_equal(vb, pv, isf);
      const uint64_t dm = __ballot(diff);
      bool run_start = diff;  // first row of a value run of its slot (set below for first lanes)
      if (act && below == 0) {
        if (!uni) tbl[s] = 0ull;  // after every lane's read of the mask (program order)
        const uint32_t add_rows = (uint32_t)__popcll(match), add_ch = (uint32_t)__popcll(dm & match);
        if (COMPACT) {
          const ScdSlot32 cur = st32[s];
          const uint32_t rows = cur.rc & 0xFFFFu;
          uint32_t ch = (cur.rc >> 16) + add_ch;
          if (rows == 0) {
            if (p16) {
              fv32[s] = ((uint32_t)vb & 0xFFFFu) | (rel << 16);
            } else {
              fv32[s] = (uint32_t)vb;
              fr32[s] = (uint32_t)row;
            }
            run_start = true;
          } else if (cur.last != (uint32_t)vb) {
            ch += 1u;
            run_start = true;
          }
          const uint32_t rc = (rows + add_rows) | (ch << 16);
          if (uni) st32[s] = ScdSlot32{(uint32_t)lastv, rc};
          else st32[s].rc = rc;  // `last`: the slot's last lane, below
        } else {
          ScdSlot cur = st[s];
          uint32_t ch = cur.changes + add_ch;
          if (cur.rows == 0) {
            cur.first = vb;
            cur.first_row = (uint32_t)row;
            run_start = true;
          } else if (!scd_equal(cur.last, vb, isf)) {
            ch += 1u;
            run_start = true;
          }
          cur.last = lastv;
          cur.rows += add_rows;
          cur.changes = ch;
          st[s] = cur;
        }
      }
      // compact: the slot's last lane in the step (the highest lane of its match mask) stores
      // its value as the slot's `last` -- after the first lane's read of the state above
      // (program order; the same address in both lanes' expressions)
      if (COMPACT && !uni && act && (match >> lane) == 1ull) st32[s].last = (uint32_t)vb;
      // count_distinct of the same column: only the first row of a value run of its slot can
      // add a (slot, value) pair (every later row of the run repeats one already added), so
      // the pair check runs at run starts only (most rows of a sorted column skip it)
      if (do_cd && (cd_runs ? run_start : act)) {
        // (slot, value) pair bit (the planner fuses pair spaces < 2^30 only): an LDS
        // fire-and-forget OR (merged into the device bitmap once per workgroup at the end);
        // without an LDS bitmap, the device bitmap directly
        // 32-bit arithmetic: the pair space is < 2^30
        const uint32_t bit = s * (uint32_t)d.cd.vrange + ((uint32_t)vcd - (uint32_t)d.cd.vmin);
        const unsigned int m = 1u << (bit & 31);
        if (cd_mode == 1) {
          // read first: lanes of one word broadcast; only a new pair pays the (serialising)
          // same-address atomic
          if (!(cdb[bit >> 5] & m)) atomicOr(&cdb[bit >> 5], m);
        } else if (!(d.cd.bitmap[bit >> 5] & m) && !(atomicOr(&d.cd.bitmap[bit >> 5], m) & m)) {
          atomicAdd(&d.cd.out[s], 1ull);
        }
      }
  };
  // rows of the chunk (< 2^32: N < kNoRow); the last waves' chunks may start past the end
  const uint32_t nrel = end > start ? (uint32_t)(end - start) : 0u;
  // one 64-row step's values, one row per lane: decoded and coded
  auto derive = [&](const uint2 (&w)[NC], uint32_t rel, int64_t row, bool& act, uint32_t& s, uint64_t& vb,
                    uint64_t& vcd) {
    Chunk raw[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) scd_word_to_chunk(raw[c], p.cols[c], row, w[c]);
    uint64_t v[NC][1];
    decode_all<NC, 1>(p, raw, v);
    act = rel < nrel && (vals_pass<NC, 1, false>(p, row, v) & 1u);
    uint64_t code[1];
    vals_code<NC, 1>(p, v, code);
    vb = 0;
    vcd = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (vc == c) vb = v[c][0];
      if (cc == c) vcd = v[c][0];
    }
    s = (uint32_t)code[0];
  };
  if (RUNS) {
    scd_runs_loop<NC>(p, d, start, end, nrel, lane, vc, cc, do_cd, cd_runs, cd_mode, st32, fv32, fr32, p16, cdb, fold,
                      derive);
  } else {
  uint2 ring[kScdAhead][NC];
  if (nrel) {
#pragma unroll
    for (int a = 0; a < kScdAhead; ++a) scd_issue<NC>(p, start, 64u * a, nrel, lane, ring[a]);
  }
  for (uint32_t gbase = 0; gbase < nrel; gbase += 64 * kScdAhead) {
#pragma unroll
    for (int a = 0; a < kScdAhead; ++a) {
      const uint32_t rb = gbase + 64u * a;
      const uint32_t rel = rb + (uint32_t)lane;
      const int64_t row = start + (int64_t)rel;
      Chunk raw[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) scd_word_to_chunk(raw[c], p.cols[c], row, ring[a][c]);
      uint64_t v[NC][1];
      decode_all<NC, 1>(p, raw, v);
      // everything the step needs from its rows is derived before ring[a]'s refill is issued,
      // so ring[a] is dead at the refill and the loads land in the loop-carried registers
      // (otherwise they land in fresh ones, copied back at the loop head behind a vmcnt(0)
      // that drains the whole prefetch); rel < nrel is the row bound (32-bit), vals_pass
      // applies the terms only
      const bool act = rel < nrel && (vals_pass<NC, 1, false>(p, row, v) & 1u);
      uint64_t code[1];
      vals_code<NC, 1>(p, v, code);
      uint64_t vb = 0, vcd = 0;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (vc == c) vb = v[c][0];
        if (cc == c) vcd = v[c][0];
      }
      uint32_t s = (uint32_t)code[0];
      if (COMPACT) {
        // the derived 32-bit values are pinned here (an empty asm that redefines them): the
        // compiler would otherwise sink their arithmetic below the refill, keeping ring[a] live
        uint32_t vb32 = (uint32_t)(vb - (uint64_t)d.vmin), vcd32 = (uint32_t)vcd;
        asm volatile("" : "+v"(s), "+v"(vb32), "+v"(vcd32));
        vb = vb32;
        vcd = vcd32;
      }
      __builtin_amdgcn_sched_barrier(0);
      // unconditional (clamped) prefetch: the same number of loads is in flight on every
      // path, so the compiler waits for exactly the step it consumes (vmcnt(N), not vmcnt(0));
      // steps past the chunk end skip their work but not their loads (no `break`, whose exit
      // edge would merge a shorter load history into the loop header)
      scd_issue<NC>(p, start, rb + 64u * kScdAhead, nrel, lane, ring[a]);
      if (rb >= nrel) continue;
      fold(rel, row, act, s, vb, vcd);
    }
  }
  }
  // count_distinct: merge the workgroup's pair bitmap into the device bitmap; every pair bit
  // this workgroup sets first counts once for its slot
  if (cd_mode == 1) {
    __syncthreads();
    for (int i = threadIdx.x; i < d.cd.lds_bitmap_words; i += blockDim.x) {
      const unsigned int word = cdb[i];
      if (!word) continue;
      unsigned int fresh = word & ~atomicOr(&d.cd.bitmap[i], word);
      while (fresh) {
        const int b = __ffs(fresh) - 1;
        fresh &= fresh - 1u;
        atomicAdd(&d.cd.out[((uint64_t)i * 32 + (uint64_t)b) / d.cd.vrange], 1ull);
      }
    }
  }
  // the workgroup's waves own consecutive chunks: their states are folded here, in chunk order,
  // and flushed as ONE chunk state per (workgroup, slot) -- a quarter of the per-wave states for
  // the chunk combine to read (C4: 53 -> 13 MB; launch_scd combines `blocks` chunks)
  __syncthreads();  // every wave's LDS state is final
  const int nwv = (int)(blockDim.x >> 6);
  for (int i = threadIdx.x; i < S; i += blockDim.x) {
    ScdState acc = {0u, kNoRow, 0ull, 0ull, 0ull, 0ull};
    for (int v = 0; v < nwv; ++v) {
      const int wv = blockIdx.x * nwv + v;
      if (wv >= d.waves) break;
      const unsigned char* vb = smem + (size_t)v * d.wave_lds;
      ScdState x;
      if (COMPACT) {
        const ScdSlot32* s32 = reinterpret_cast<const ScdSlot32*>(vb);
        const uint32_t* f32 = reinterpret_cast<const uint32_t*>(s32 + S);
        const ScdSlot32 c = s32[i];
        const uint32_t rows = c.rc & 0xFFFFu;
        x.present = rows != 0;
        x.rows = rows;
        x.changes = c.rc >> 16;
        x.last = (uint64_t)d.vmin + c.last;
        if (p16) {
          x.first_row = (uint32_t)((int64_t)wv * d.chunk_rows) + (f32[i] >> 16);
          x.first = (uint64_t)d.vmin + (f32[i] & 0xFFFFu);
        } else {
          x.first_row = f32[S + i];
          x.first = (uint64_t)d.vmin + f32[i];
        }
      } else {
        const ScdSlot c = reinterpret_cast<const ScdSlot*>(vb)[i];
        x.present = c.rows != 0;
        x.first_row = c.first_row;
        x.first = c.first;
        x.last = c.last;
        x.changes = c.changes;
        x.rows = c.rows;
      }
      acc = scd_combine(acc, x, isf);
    }
    const size_t o = (size_t)blockIdx.x * S + i;
    d.st_first_row[o] = acc.present ? acc.first_row : kNoRow;
    d.st_first[o] = acc.first;
    d.st_last[o] = acc.last;
    d.st_changes[o] = (uint32_t)acc.changes;
    d.st_count[o] = (uint32_t)acc.rows;
  }
}

}  // namespace bqg
