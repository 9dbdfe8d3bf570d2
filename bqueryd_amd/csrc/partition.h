// partition.h -- body of the partitioned-aggregation scatter pass (config C3), shared by the
// precompiled kernel (k_partition.hip) and the query-specialised JIT kernel (jit_kernels.h):
// with the query shape folded into constants the per-row dtype / operator dispatch of the
// generic body disappears.
//
// Workgroups exchange data through LDS only, so every barrier here is lds_barrier(): a
// __syncthreads() would also drain the tile's prefetched column loads and its streaming
// entry stores at each of the scatter's barriers.
#pragma once

#include "device.h"

namespace bqg {

// ------------------------------------------------------------------------------------
// block-wide scans
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// exclusive scan over the workgroup (blockDim.x a multiple of 64, <= 1024); *total receives
// the sum (visible to every thread after the call)
__device__ __forceinline__ uint32_t block_excl_scan_1024(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[17];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan_u32(v, lane);
  if (lane == 63) wsum[wave] = incl;
  lds_barrier();
  if (wave == 0) {
    const uint32_t w = lane < (int)(blockDim.x >> 6) ? wsum[lane] : 0u;
    const uint32_t wi = wave_incl_scan_u32(w, lane);
    if (lane < 16) wsum[lane] = wi - w;
    if (lane == 63) wsum[16] = wi;
  }
  lds_barrier();
  const uint32_t r = wsum[wave] + incl - v;
  if (total) *total = wsum[16];
  lds_barrier();
  return r;
}

// One-barrier variant for a loop body: every wave scans the (<= 16) wave totals itself, and
// the caller alternates `wsum` buffers between iterations so that no trailing barrier is
// needed before the next call overwrites them.
__device__ __forceinline__ uint32_t block_excl_scan_1b(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan_u32(v, lane);
  if (lane == 63) wsum[wave] = incl;
  lds_barrier();
  const int nw = (int)(blockDim.x >> 6);
  const uint32_t w = lane < nw ? wsum[lane] : 0u;
  const uint32_t wi = wave_incl_scan_u32(w, lane);
  const uint32_t before = (uint32_t)__shfl((int)(wi - w), wave, 64);
  *total = (uint32_t)__shfl((int)wi, nw - 1, 64);
  return before + incl - v;
}

// scatter: workgroups of up to 1024 threads, each over a contiguous range of whole tiles
constexpr int kPartBlock = 1024;

// one 16-byte streaming store (the entries are read back by the aggregate only: no cache
// residency to keep)
__device__ __forceinline__ void st_nt16(void* dst, const void* src) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(*reinterpret_cast<const v4u*>(src), reinterpret_cast<v4u*>(dst));
}

// Tile-layout scatter.  A tile is T * 4 * K rows (TR).  The workgroup counting-sorts each of its
// tiles by partition (slot >> wbits) in LDS and writes the sorted tile back LINEARLY to the
// tile's own entry range [tile * TR, tile * TR + TR) with 16-byte stores of whole lines --
// the same stores on every path (positions past the tile's passing rows carry left-over
// staging words that no reader looks at), so the loop waits for the next tile's loads with
// vmcnt(N) instead of draining.  The tile's header hdr[tile][0 .. P] holds the 16-bit offset of
// each partition's run (hdr[tile][P] = passing rows).  An entry is a 32-bit meta word
// (row-in-tile << wbits | slot_low) and one 64-bit value per summed column -- or, NARROW, one
// exact 32-bit integer code per summed column (PartLaunch::enc_kind: 8-byte entries for C3).
//
// Measured on MI355X (tools/micro/part_micro.hip, C3 shape): the region layout this replaces
// (count pass, scan, per-(partition, block) regions) wrote each tile as ~P runs of ~32
// entries into P far-apart regions and ran at 3.4 TB/s of moved bytes; the linear tile
// writes run at copy speed (2.8 GB in 0.57 ms), with no count pass and no scan.
// The exact 32-bit code of a summed float value (narrow entries, PartLaunch::enc_kind)
// (the query-specialised build fixes the code kinds -- BQ_PART_ENC, one per summed column --
// so a dyadic code is one multiply and conversion, with no per-row branch to the cents rounding)
__device__ __forceinline__ int part_kind(const PartLaunch& L, int q) {
#ifdef BQ_PART_ENC
  constexpr int kinds[kMaxSums] = {BQ_PART_ENC};
  return kinds[q];
#else
  return L.enc_kind[q];
#endif
}

__device__ __forceinline__ uint32_t part_enc(const ScanParams& p, const PartLaunch& L, int q, uint64_t v) {
  const int kind = part_kind(L, q);
  if (kind == 3) return (uint32_t)(v - (uint64_t)L.enc_off[q]);  // canonical int64 value
  const double d = value_f64(v, p.sum_conv[q]) * L.enc_mul[q];
  return (uint32_t)(int32_t)(kind == 1 ? d : rint(d));
}

// PACK (PartLaunch::pack): one 32-bit word per entry, the summed column's 16-bit code (if
// any) above the 16-bit slot_low -- no row: first appearance comes from each slot's first
// tile (k_part_aggregate) and a re-read of only those tiles (k_part_first_rows).
__device__ __forceinline__ uint32_t part_code16(const ScanParams& p, const PartLaunch& L, uint64_t v) {
  return (part_enc(p, L, 0, v) - (uint32_t)L.enc_base16) << 16;
}

// RING (packed entries): the tiles' row loads are issued RING tiles ahead (RING register sets
// used in turn), so a workgroup keeps RING tiles of reads in flight across the barriers of the
// tile it sorts; a block's last group of RING tiles may run past its rows -- such a tile
// passes no row and writes its header and entry words to the spare tile past the last
// (PartLaunch::ntiles; allocated, never read).
template <int NC, int K = 1, bool NARROW = false, bool PACK = false, int RING = 1>
__device__ __forceinline__ void part_scatter_body(const ScanParams& p, const PartLaunch& L, unsigned char* smem) {
  static_assert(RING == 1 || PACK, "only packed entries have a spare tile for the ring's tail");
  // K 4-row chunks per thread and tile (TR = T * 4 * K rows): chunk k of thread t covers rows
  // base + k * T * 4 + t * 4 .. + 3, so every chunk load of the workgroup is one coalesced block
  const int T = blockDim.x, tid = threadIdx.x;
  const int P = L.nparts;
  const int TR = T * kRowsPerThread * K;
  const int nsum = p.nsum;
  constexpr int NS = NC < kMaxSums ? NC : kMaxSums;
  unsigned long long* sval = reinterpret_cast<unsigned long long*>(smem);  // [nsum][TR] (wide)
  uint32_t* sval32 = reinterpret_cast<uint32_t*>(smem);                    // [nsum][TR] (narrow)
  uint32_t* smeta = reinterpret_cast<uint32_t*>(smem) + (PACK ? 0 : (size_t)nsum * TR * (NARROW ? 1 : 2));  // [TR]
  uint16_t* srit = reinterpret_cast<uint16_t*>(smeta + TR);                // PACK: [TR] rows in tile
  uint32_t* hist2 = smeta + TR + (PACK ? TR / 2 : 0);                      // [2][P] tile counts
  uint32_t* toff = hist2 + 2 * P;                                          // [P] tile offsets
  uint32_t* wsum2 = toff + P;                                              // [2][16] scan totals
  for (int i = tid; i < 2 * P; i += T) hist2[i] = 0;
  lds_barrier();
  const int64_t begin = (int64_t)blockIdx.x * L.rows_per_block;
  const int64_t end = (p.nrows < begin + L.rows_per_block ? p.nrows : begin + L.rows_per_block);
  if (PACK) {
    // the aggregate's first-tile marks of this block's tiles and (block 0) the marked list's
    // length, zeroed here rather than by a fill between the two kernels (round 6)
    for (int64_t t = begin / TR + tid; t < (end + TR - 1) / TR; t += T) L.tile_mark[t] = 0u;
    if (blockIdx.x == 0 && tid == 0) *L.nmarked = 0u;
  }
  if (begin >= end) return;
  const uint64_t lowmask = (1ull << L.wbits) - 1ull;
  const int per = (P + T - 1) / T;  // partitions per thread in the tile scan
  const int q0 = tid * per;
  const int q1 = min(P, q0 + per);
  const uint32_t all = (1u << NC) - 1u;
  const int64_t CH = (int64_t)T * kRowsPerThread;  // rows of one chunk block
  Chunk ring[RING][K][NC];
#pragma unroll
  for (int g = 0; g < RING; ++g)
#pragma unroll
    for (int k = 0; k < K; ++k)
      load_rows4_clamped<NC>(p, begin + g * TR + k * CH + (int64_t)tid * kRowsPerThread, end, ring[g][k], all, begin);
  int parity = 0;
  for (int64_t gbase = begin; gbase < end; gbase += RING * TR) {
#pragma unroll
  for (int g = 0; g < RING; ++g, parity ^= 1) {
    const int64_t base = gbase + g * TR;
    Chunk (&raw)[K][NC] = ring[g];
    // the tile whose header and entries this one writes (RING: the spare tile past the last
    // when the block's rows ended before it)
    const int64_t tile = RING == 1 || base < end ? base / TR : L.ntiles;
    const int64_t obase = tile * TR;
    // the tile histogram alternates between two buffers: the one this tile zeroes at its end
    // is next counted into two tiles later, past the next tile's barriers
    uint32_t* hist = hist2 + parity * P;
    // PACK keeps one 32-bit staged word and one part|rank word per row across the tile's
    // barriers (the summed value is packed right after the decode); the wide layouts keep
    // the values themselves
    uint32_t pass[K], part[K][4], rank[K][4], low[K][4];
    uint64_t sv[PACK ? 1 : NS][K][4];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t row0 = base + k * CH + (int64_t)tid * kRowsPerThread;
      uint64_t v[NC][4], code[4];
      decode_all<NC, 4>(p, raw[k], v);
      load_rows4_clamped<NC>(p, row0 + RING * TR, end, raw[k], all, begin);
      pass[k] = vals_pass<NC, 4>(p, row0, v);
      const int64_t rem = end - row0;
      pass[k] &= rem >= 4 ? 0xFu : (rem > 0 ? ((1u << rem) - 1u) : 0u);
      vals_code<NC, 4>(p, v, code);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        part[k][r] = (uint32_t)(code[r] >> L.wbits);
        low[k][r] = (uint32_t)(code[r] & lowmask);
        if (PACK) {
          low[k][r] |= nsum ? part_code16(p, L, v[0][r]) : 0u;
          continue;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) sv[s][k][r] = v[s][r];
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        rank[k][r] = (pass[k] & (1u << r)) ? atomicAdd(&hist[part[k][r]], 1u) : 0u;
        // partitions < 2^16 and tile ranks < 2^16 (TR <= 16384): one word
        if (PACK) part[k][r] = (part[k][r] << 16) | rank[k][r];
      }
    lds_barrier();
    // tile offsets: exclusive scan of the tile histogram, also the tile's header
    uint32_t local = 0;
    for (int i = q0; i < q1; ++i) local += hist[i];
    uint32_t n_tile;
    uint32_t run = block_excl_scan_1b(local, wsum2 + parity * 16, &n_tile);
    uint16_t* th = L.hdr + (size_t)tile * (size_t)(P + 1);
    for (int i = q0; i < q1; ++i) {
      toff[i] = run;
      th[i] = (uint16_t)run;
      run += hist[i];
    }
    if (tid == 0) th[P] = (uint16_t)n_tile;
    lds_barrier();
    // PACK: this tile records its entries' rows in tile (PartLaunch::rit; uniform)
    const bool with_rit = PACK && tile < L.rit_tiles;
    // stage the tile sorted by partition
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t rit0 = (uint32_t)(k * CH) + (uint32_t)tid * kRowsPerThread;  // row in tile
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (!(pass[k] & (1u << r))) continue;
        if (PACK) {
          const uint32_t pos = toff[part[k][r] >> 16] + (part[k][r] & 0xFFFFu);
          smeta[pos] = low[k][r];
          if (with_rit) srit[pos] = (uint16_t)(rit0 + r);
          continue;
        }
        const uint32_t pos = toff[part[k][r]] + rank[k][r];
        smeta[pos] = ((rit0 + r) << L.wbits) | low[k][r];
#pragma unroll
        for (int s = 0; s < NS; ++s)
          if (s < nsum) {
            if (NARROW) sval32[(size_t)s * TR + pos] = part_enc(p, L, s, sv[s][k][r]);
            else sval[(size_t)s * TR + pos] = sv[s][k][r];
          }
      }
    }
    lds_barrier();
    // linear copy-out: K 16-byte stores of meta and 2K per summed column, every thread
#pragma unroll
    for (int k = 0; k < K; ++k)
      st_nt16(L.meta + obase + 4 * (tid + k * T), smeta + 4 * (tid + k * T));
    if (with_rit)
      for (int i = tid; i < TR / 8; i += T)
        st_nt16(L.rit + obase + 8 * i, srit + 8 * i);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (PACK || s >= nsum) break;
      if (NARROW) {
        uint32_t* dv = reinterpret_cast<uint32_t*>(L.vals) + (size_t)s * L.capacity + obase;
        const uint32_t* lv = sval32 + (size_t)s * TR;
#pragma unroll
        for (int k = 0; k < K; ++k)
          *reinterpret_cast<uint4*>(dv + 4 * (tid + k * T)) = *reinterpret_cast<const uint4*>(lv + 4 * (tid + k * T));
      } else {
        unsigned long long* dv = L.vals + (size_t)s * L.capacity + obase;
        const unsigned long long* lv = sval + (size_t)s * TR;
#pragma unroll
        for (int k = 0; k < 2 * K; ++k)
          *reinterpret_cast<uint4*>(dv + 2 * (tid + k * T)) = *reinterpret_cast<const uint4*>(lv + 2 * (tid + k * T));
      }
    }
    for (int i = q0; i < q1; ++i) hist[i] = 0;
  }
  }
}

// First rows of the PACK path: a slot's first row lies in its first tile, and the aggregate
// marks every slot's first tile (tile_mark) and keeps its low 8 bits per slot (first_tag);
// the marked tiles are read again -- their key / filter columns, through the scan's own row ->
// slot code -- and a passing row whose slot's tag matches the tile's takes part in an
// atomicMin on the slot's first row (the combine set every slot to kNoRow): the slot's true
// first row is among them, and any other row that passes the 8-bit check is later, so it
// cannot win.  The per-row check reads a 1-byte tag (the array stays in L2) instead of
// issuing a memory-side atomic per row.  On random keys the marked tiles are mostly a prefix
// (each slot's first appearance falls early: ~10-15 % of the tiles at C3's 1 M groups); on
// sorted keys every tile is marked.
// Work unit: one 4096-row quarter of a tile (kFirstRowsBlock threads x 16 rows, every load of
// the unit issued before the first is used); the grid strides over the units of the marked
// tiles' list, so the marked tiles spread over every CU instead of queueing behind one large
// workgroup each.  With the rows in tile recorded where first appearances fall
// (PartLaunch::rit) the list is usually empty and the pass ends at once.
constexpr int kFirstRowsBlock = 256;
constexpr int kFirstRowsUnit = kFirstRowsBlock * 16;
template <int NC>
__device__ __forceinline__ void part_first_rows_body(const ScanParams& p, const PartLaunch& L, const SlotArrays& sa) {
  // only the key, term and mask columns are read (the others re-read one line per wave)
  uint32_t need = p.mask_col >= 0 ? 1u << p.mask_col : 0u;
  for (int k = 0; k < p.nkeys; ++k) need |= 1u << p.keys[k].col;
  for (int i = 0; i < p.nterms; ++i) need |= 1u << p.terms[i].col;
  const int64_t TR = L.tile_rows;
  const int64_t per_tile = (TR + kFirstRowsUnit - 1) / kFirstRowsUnit;
  // the marked tiles' list (k_part_aggregate / k_part_combine append each tile once): empty
  // when every slot's first row came from the rows in tile (PartLaunch::rit)
  const int64_t units = (int64_t)*L.nmarked * per_tile;
  for (int64_t u = blockIdx.x; u < units; u += gridDim.x) {
    const int64_t t = L.marked[u / per_tile];
    const unsigned char tag = (unsigned char)t;
    const int64_t base = t * TR + (u % per_tile) * kFirstRowsUnit;
    const int64_t end = min(min(p.nrows, (t + 1) * TR), base + kFirstRowsUnit);
    Chunk raw[4][NC];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      load_rows4_clamped<NC>(p, base + ((int64_t)threadIdx.x + k * kFirstRowsBlock) * kRowsPerThread, end, raw[k], need, base);
    // every row's slot first, then all 16 tag loads (independent: issued together), then the
    // atomics of the matching rows -- a tag load per row waited for one at a time (behind the
    // previous row's atomic) made the pass latency-bound
    uint32_t slot[4][4], pass[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t row0 = base + ((int64_t)threadIdx.x + k * kFirstRowsBlock) * kRowsPerThread;
      uint64_t v[NC][4], code[4];
      decode_all<NC, 4>(p, raw[k], v);
      const int64_t rem = end - row0;
      pass[k] = rem >= 4 ? 0xFu : (rem > 0 ? ((1u << rem) - 1u) : 0u);
      pass[k] &= vals_pass<NC, 4, false>(p, row0, v);
      vals_code<NC, 4>(p, v, code);
#pragma unroll
      for (int r = 0; r < 4; ++r) slot[k][r] = ((pass[k] >> r) & 1u) ? (uint32_t)code[r] : 0u;
    }
    unsigned char tg[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) tg[k][r] = L.first_tag[slot[k][r]];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t row0 = base + ((int64_t)threadIdx.x + k * kFirstRowsBlock) * kRowsPerThread;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (((pass[k] >> r) & 1u) && tg[k][r] == tag) atomicMin(&sa.fst[slot[k][r]], (uint32_t)(row0 + r));
    }
  }
}

}  // namespace bqg
