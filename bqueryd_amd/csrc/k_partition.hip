// k_partition.hip -- partitioned aggregation for large dense slot spaces (config C3: ~1 M
// groups), and a multi-workgroup exclusive scan.
//
// Per-row device atomics on a 1 M-slot table are random 8-byte memory-side operations
// (MI355X_MICROARCH.md §Global float atomics: they execute past L2).  Instead:
//   scatter:   each workgroup owns a contiguous range of whole tiles; a tile is counting-
//              sorted by partition p = slot >> wbits in LDS and written back linearly to the
//              tile's own entry range, with a header of P + 1 16-bit partition offsets
//              (partition.h);
//   aggregate: workgroups per partition walk a range of tiles, read the partition's segment
//              of each (16-bit header -> 4-byte meta + 8-byte values), aggregate the entries
//              in an LDS table of 2^wbits slots and flush the occupied slots.
// Traffic per row (C3, one f64 sum): 16 read + 12 written + 12 read back (segments of ~32
// entries: partial edge lines, shared by neighbouring partitions through the XCD's L2).
// Measured (tools/micro/part_micro.hip): the segment reads run at ~3.4 TB/s -- a loads-only
// probe of the aggregate takes as long as the whole kernel -- and storing each segment as one
// run of 12-byte {meta, value} entries instead of two runs read no faster.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "partition.h"

namespace bqg {

template <int NC, int K, bool NARROW, bool PACK>
__global__ __launch_bounds__(kPartBlock) void k_part_scatter(ScanParams p, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  part_scatter_body<NC, K, NARROW, PACK>(p, L, smem);
}

// Aggregate over the tile layout.  Workgroup (partition, split): the split's tile range.  A
// wave takes groups of G consecutive tiles; lane j < G holds tile j's segment bounds, a wave
// scan of the segment lengths flattens the group, and each of U wave-wide loads reads 64
// consecutive entries of the flattened group: an entry finds its tile with G - 1 compares
// against wave-uniform segment starts and takes that tile's first index with one lane
// shuffle.  Software-pipelined: while a group's entries are aggregated, the next group's
// entries and the header of the group after it are in flight (two register sets used in
// turn, so no copy waits on a pending load).  Measured (tools/micro/part_micro.hip, C3
// shape): with loads only and no LDS atomics the unpipelined loop took as long as the whole
// aggregate -- it waited on each group's loads.  Workgroups are mapped XCD-aware: the
// workgroups of one XCD (blockIdx % 8) take consecutive partitions over the same tile range,
// so the edge lines their segments share are read once into that XCD's L2.
//
// PACK entries (PartLaunch::pack): one 32-bit word {code16, slot_low}; the slot table is one
// packed 64-bit accumulator (count << sbits | code16 sum: ONE LDS atomic per entry) and the
// slot's first-appearance key (PartLaunch::rit: the exact first row where the tile recorded its
// rows, else the first tile), and the combine leaves the rest to k_part_first_rows.
// One split's record of a slot: count, first row (PACK: first-appearance key), sums (PACK: 64-bit count
// c64 and the code16 sum a[0]).
// the exact int64 code of a summed float value of a wide entry (ScanParams::sum_enc)
__device__ __forceinline__ long long part_sum_code(const ScanParams& p, int q, uint64_t v) {
  const double d = value_f64(v, p.sum_conv[q]) * p.sum_mul[q];
  return (long long)(p.sum_enc[q] == 1 ? d : rint(d));
}

template <int NV>
struct PartRec {
  unsigned long long a[NV];
  unsigned long long x[NV][kFxWords];  // fixed-point sums: limbs 1, 2, non-finite flags (a holds limb 0)
  unsigned long long c64;  // PACK: count
  uint32_t c, f;
};

// The final values of slot gs from its S split records (rec(o, r) fills split o's), added in
// split order, written to the slot arrays.
template <int NSUM, bool NARROW, bool PACK, typename Rec>
__device__ __forceinline__ void part_finish_slot(const ScanParams& p, const PartLaunch& L, const SlotArrays& sa,
                                                 uint64_t gs, int S, Rec rec) {
  constexpr int NV = NSUM > 0 ? NSUM : 1;
  constexpr int nsum = NSUM;
  if (PACK) {
    // split records hold the unpacked count (c64) and code16 sum (a[0]); exact code sum =
    // sum of code16 + count x enc_base16
    unsigned long long c = 0, cs = 0;
    uint32_t f = kNoRow;
    for (int o = 0; o < S; ++o) {
      PartRec<NV> r;
      rec(o, r);
      c += r.c64;
      cs += r.a[0];
      f = r.f < f ? r.f : f;
    }
    sa.cnt[gs] = c;
    // f: the least first-appearance key (PartLaunch::rit): an exact row when its tile recorded
    // rows in tile, else the first tile's last row -- then k_part_first_rows finds the row
    const uint32_t ft = f == kNoRow ? kNoRow : f / (uint32_t)L.tile_rows;
    sa.fst[gs] = (f != kNoRow && (int64_t)ft < L.rit_tiles) ? f : kNoRow;
    if (f != kNoRow && (int64_t)ft >= L.rit_tiles) {
      // a few hundred marked tiles take ~1 M marks (random keys without row records): a read
      // first (an L2 hit once the XCD has seen the line) instead of 1 M contended byte stores
      // each marked tile joins the first-row pass's list once
      if (!L.tile_mark[ft] && atomicCAS(&L.tile_mark[ft], 0u, 1u) == 0u) L.marked[atomicAdd(L.nmarked, 1u)] = ft;
      L.first_tag[gs] = (unsigned char)ft;
    }
    if (nsum) {
      unsigned long long tot = cs + c * (unsigned long long)L.enc_base16;
      if (L.enc_kind[0] == 3) tot += c * (unsigned long long)L.enc_off[0];
      else tot = as_u64((double)(long long)tot / L.enc_mul[0]);
      sa.acc[gs] = tot;
    }
    return;
  }
  uint32_t c = 0, f = kNoRow;
  unsigned long long a[NV], x[NV][kFxWords];
#pragma unroll
  for (int q = 0; q < NV; ++q) a[q] = x[q][0] = x[q][1] = x[q][2] = 0;
  for (int o = 0; o < S; ++o) {
    PartRec<NV> r;
    rec(o, r);
    c += r.c;
    f = r.f < f ? r.f : f;
#pragma unroll
    for (int q = 0; q < nsum; ++q) {
      if (!NARROW && p.sum_is_float[q] && !p.sum_enc[q]) a[q] = as_u64(as_f64(a[q]) + as_f64(r.a[q]));
      else a[q] += r.a[q];
      x[q][0] += r.x[q][0];
      x[q][1] += r.x[q][1];
      x[q][2] |= r.x[q][2];
    }
  }
  sa.cnt[gs] = c;
  sa.fst[gs] = f;
#pragma unroll
  for (int q = 0; q < nsum; ++q) {
    // narrow: the exact sum of the codes, scaled back once (dyadic: exact below 2^53), or
    // shifted back by count x offset (integers, modulo 2^64 like the 64-bit accumulator)
    if (NARROW) {
      if (L.enc_kind[q] == 3) a[q] += (unsigned long long)c * (unsigned long long)L.enc_off[q];
      else a[q] = as_u64((double)(long long)a[q] / L.enc_mul[q]);
    } else if (p.sum_is_float[q] && p.sum_enc[q] == 3) {
      a[q] = as_u64(x[q][2] ? fx_nonfinite(x[q][2])
                            : fx_value((long long)a[q], (long long)x[q][0], (long long)x[q][1], fx_shift(p, q, gs)));
    } else if (p.sum_is_float[q] && p.sum_enc[q]) {
      a[q] = as_u64((double)(long long)a[q] / p.sum_mul[q]);
    }
    sa.acc[(size_t)q * p.nslots + gs] = a[q];
  }
}

template <int U, int AH, int NSUM, bool NARROW, bool PACK>
__global__ __launch_bounds__(1024) void k_part_aggregate(ScanParams p, PartLaunch L, SlotArrays sa) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int P = L.nparts;
  const int per_x = (P + 7) / 8;
  const int bx = (int)(blockIdx.x & 7u), bi = (int)(blockIdx.x >> 3);
  const int part = bx * per_x + bi % per_x, split = bi / per_x;
  if (part >= P || split >= L.splits) return;  // the whole workgroup
  const int W = 1 << L.wbits;
  constexpr int nsum = NSUM;
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem);  // [nsum][W] (PACK: [W] packed)
  uint32_t* cnt = reinterpret_cast<uint32_t*>(acc + (size_t)(PACK ? 1 : nsum) * W);  // [W] (PACK: unused)
  uint32_t* fst = PACK ? cnt : cnt + W;                                    // [W] first row (PACK: first-appearance key)
  // fixed-point sums (L.fx): limbs 1, 2 and flags [nsum][kFxWords][W] after the table (limb 0 is acc)
  const bool fx = !PACK && !NARROW && L.fx;
  unsigned long long* fxl = reinterpret_cast<unsigned long long*>(smem + part_agg_lds(L.wbits, nsum, PACK));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, NW = (int)(blockDim.x >> 6);
  for (int i = tid; i < W; i += blockDim.x) {
    if (!PACK) cnt[i] = 0;
    fst[i] = kNoRow;
  }
  for (int i = tid; i < (PACK ? 1 : nsum) * W; i += blockDim.x) acc[i] = 0;
  if (fx)
    for (int i = tid; i < kFxWords * nsum * W; i += blockDim.x) fxl[i] = 0;
  const unsigned long long inc = PACK ? 1ull << L.sbits : 0ull;  // one row in the packed count field
  const uint32_t inc_hi = (uint32_t)(inc >> 32);                  // (sbits >= 32)
  __syncthreads();
  const int64_t nt = L.ntiles;
  // (splits <= ntiles: every split's tile range is non-empty, and every split must reach the
  // combine below)
  const int64_t t_lo = nt * split / L.splits, t_hi = nt * (split + 1) / L.splits;
  const uint32_t lowmask = (uint32_t)W - 1u;
  const uint32_t TR = (uint32_t)L.tile_rows;
  constexpr int NV = NSUM > 0 ? NSUM : 1;
  // Entries are read in 16-byte granules (4 entries, a lane's one load; a segment's edge
  // granules also hold neighbouring partitions' entries, masked off by their index in the tile):
  // 4-byte loads kept too few bytes in flight -- a loads-only probe of the 4-byte version took
  // 0.178 of the aggregate's 0.195 ms.  The window's tiles, in LDS, one 16-byte record each
  // (wT[j] = {F, B, E, AB}): flattened granule start F, global granule base B (granule = B +
  // flattened position), E (entry index in the tile of a flattened granule's first entry = E +
  // 4 x position) and the segment's entry range AB = a | b << 16; K + 1 sentinels past the
  // last tile.  A granule's lane finds its tile by comparing against the chunk's K tile starts
  // (read once per chunk) and fetches that tile's record with one 16-byte LDS read.
  const int WIN = L.win;  // <= kAggWinMax: the header loads below are 4 tiles per thread at most
  uint4* wT = reinterpret_cast<uint4*>(smem + part_agg_lds(L.wbits, nsum, PACK, !PACK && L.fx));
  const uint32_t TG = TR >> 2;  // granules per tile
  // one chunk of at most U x 64 consecutive granules of a wave's range, spanning at most K
  // tiles: per granule its 4 entries, its tile (global index; kNoRow past the chunk), the tile
  // index of its first entry and the segment's entry range
  struct Ent {
    uint4 m[U];
    uint2 rr[PACK ? U : 1];  // PACK: the granule's 4 rows in tile (tiles below L.rit_tiles)
    uint32_t t[U], e0[U], ab[U];
    unsigned long long v[U][4][NV];
  };
  const uint32_t rit_tiles = (uint32_t)min(L.rit_tiles, (int64_t)0xFFFFFFFF);
  // PACK: the packed accumulator's fields hold L.pack_flush entries (count < 2^(64 - sbits),
  // code16 sum < 2^sbits); a window holds at most that many entries (4 per granule), and before
  // a window that would pass it the accumulators are flushed (unpacked, added) into the
  // workgroup's own split record -- never at C3's ~400 K entries per workgroup, only for
  // partitions with many millions of rows in one split (skewed keys)
  unsigned long long* rec_cnt = nullptr;
  unsigned long long* rec_sum = nullptr;
  uint32_t* rec_fst = nullptr;
  if (PACK) {
    rec_cnt = reinterpret_cast<unsigned long long*>(L.partial + ((size_t)part * L.splits + split) * L.partial_bytes);
    rec_sum = rec_cnt + W;
    rec_fst = reinterpret_cast<uint32_t*>(rec_sum + W);
  }
  const unsigned long long smask = PACK ? (1ull << L.sbits) - 1ull : 0ull;
  bool flushed = false;
  uint64_t since = 0;
  auto flush = [&]() {
    for (int sl = tid; sl < W; sl += blockDim.x) {
      const unsigned long long a = acc[sl];
      const unsigned long long c = a >> L.sbits, sm = a & smask;
      rec_cnt[sl] = flushed ? rec_cnt[sl] + c : c;
      rec_sum[sl] = flushed ? rec_sum[sl] + sm : sm;
      acc[sl] = 0ull;
    }
    flushed = true;
    lds_barrier();
  };
  const uint32_t gflush = (uint32_t)(L.pack_flush >> 2);  // granules between flushes
  for (int64_t w0 = t_lo; w0 < t_hi;) {
    int nw = (int)min((int64_t)WIN, t_hi - w0);
    // headers of the window's tiles (up to four per thread, contiguous for the scan; every
    // load issued before the first is used)
    constexpr int kHdr = kAggWinMax / 1024;
    const int per = (nw + (int)blockDim.x - 1) / (int)blockDim.x;  // 1 .. kHdr, uniform
    uint32_t glen[kHdr], ga[kHdr], ab[kHdr];
#pragma unroll
    for (int k = 0; k < kHdr; ++k) {
      const int j = per * tid + k;
      glen[k] = ga[k] = ab[k] = 0;
      if (k < per && j < nw) {
        const uint16_t* th = L.hdr + (size_t)(w0 + j) * (size_t)(P + 1) + part;
        const uint32_t a = th[0], b = th[1];
        ga[k] = a >> 2;
        glen[k] = b > a ? ((b + 3u) >> 2) - ga[k] : 0u;
        ab[k] = a | (b << 16);
      }
    }
    uint32_t tot, mine = 0;
#pragma unroll
    for (int k = 0; k < kHdr; ++k) mine += glen[k];
    uint32_t fj = block_excl_scan_1024(mine, &tot);
#pragma unroll
    for (int k = 0; k < kHdr; ++k) {
      const int j = per * tid + k;
      if (k < per && j < nw) wT[j] = make_uint4(fj, (uint32_t)(w0 + j) * TG + ga[k] - fj, 4u * ga[k] - 4u * fj, ab[k]);
      fj += glen[k];
    }
    lds_barrier();
    if (PACK && tot > gflush) {
      // cut the window at the last tile boundary within pack_flush entries (one tile holds at
      // most tile_rows / 4 + 1 granules, and tile_rows + 4 <= pack_flush)
      int lo = 1, hi = nw;  // largest j with F[j] <= gflush
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (wT[mid].x <= gflush) lo = mid; else hi = mid;
      }
      tot = wT[lo].x;
      nw = lo;
      lds_barrier();
    }
    for (int j = nw + tid; j <= nw + kAggK; j += blockDim.x) wT[j] = make_uint4(tot, 0u, 0u, 0u);
    lds_barrier();
    if (PACK) {
      if (since + tot > gflush) {
        flush();
        since = 0;
      }
      since += tot;
    }
    // the wave's equal share of the window's granules, and the tile of its first granule
    const uint32_t e_lo = (uint32_t)((uint64_t)tot * wave / NW), e_hi = (uint32_t)((uint64_t)tot * (wave + 1) / NW);
    int jlo = 0, jhi = nw;  // largest j < nw with F[j] <= e_lo
    while (jhi - jlo > 1) {
      const int mid = (jlo + jhi) >> 1;
      if (wT[mid].x <= e_lo) jlo = mid; else jhi = mid;
    }
    uint32_t f_next = e_lo;
    int j_next = __builtin_amdgcn_readfirstlane(jlo);
    // issue the next chunk into `en`: lanes 0..K read the chunk's tile starts, the chunk ends
    // at U x 64 granules, the wave's range end or the K-th tile boundary
    // (RIT: the chunk's tiles may hold row records -- a window past PartLaunch::rit_tiles runs
    // the variant that loads none: a uniform choice per window, so the counted waits stay)
    auto issue = [&](Ent& en, auto rit_c) {
      constexpr bool RIT = decltype(rit_c)::value;
      const uint32_t lf = wT[j_next + min(lane, kAggK)].x;
      uint32_t Fk[kAggK + 1];
#pragma unroll
      for (int k = 0; k <= kAggK; ++k) Fk[k] = (uint32_t)__builtin_amdgcn_readlane((int)lf, k);
      const uint32_t fe = min(min(f_next + 64u * U, e_hi), max(Fk[kAggK], f_next));
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t f = f_next + u * 64u + lane;
        const bool valid = f < fe;
        const uint32_t fc = valid ? f : f_next;
        // the granule's tile: the last of the chunk's tiles starting at or before it
        uint32_t j = 0;
#pragma unroll
        for (int k = 1; k < kAggK; ++k) j += fc >= Fk[k] ? 1u : 0u;
        const uint4 tr = wT[j_next + j];
        const uint32_t gidx = f_next < fe ? tr.y + fc : 0u;
        en.t[u] = (uint32_t)w0 + (uint32_t)j_next + j;
        en.e0[u] = tr.z + 4u * fc;
        en.ab[u] = valid ? tr.w : 0u;  // an empty entry range past the chunk
        en.m[u] = reinterpret_cast<const uint4*>(L.meta)[gidx];
        if (PACK) {
          // rows in tile where the tile recorded them; the other lanes re-read word 0 (the
          // same number of loads on every path: counted waits, no drain)
          const uint32_t tt = (uint32_t)w0 + (uint32_t)j_next + j;
          en.rr[u] = RIT ? reinterpret_cast<const uint2*>(L.rit)[(valid && tt < rit_tiles) ? gidx : 0u] : make_uint2(0u, 0u);
          continue;
        }
#pragma unroll
        for (int q = 0; q < NV; ++q) {
          if (NARROW) {  // the exact 32-bit codes: float codes signed, integer offsets unsigned
            const uint4 c4 = reinterpret_cast<const uint4*>(reinterpret_cast<const uint32_t*>(L.vals) + (size_t)q * L.capacity)[gidx];
            const uint32_t cc[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
              en.v[u][e][q] = L.enc_kind[q] == 3 ? (unsigned long long)cc[e] : (unsigned long long)(long long)(int32_t)cc[e];
          } else {
            const uint4* vp = reinterpret_cast<const uint4*>(L.vals + (size_t)q * L.capacity) + 2 * (size_t)gidx;
            const uint4 v0 = vp[0], v1 = vp[1];
            en.v[u][0][q] = ((unsigned long long)v0.y << 32) | v0.x;
            en.v[u][1][q] = ((unsigned long long)v0.w << 32) | v0.z;
            en.v[u][2][q] = ((unsigned long long)v1.y << 32) | v1.x;
            en.v[u][3][q] = ((unsigned long long)v1.w << 32) | v1.z;
          }
        }
      }
      // the next chunk starts in the last tile whose start is <= fe (empty tiles skipped)
      int adv = 0;
#pragma unroll
      for (int k = 1; k <= kAggK; ++k) adv += Fk[k] <= fe ? 1 : 0;
      j_next = min(j_next + adv, nw);
      f_next = fe;
    };
    auto consume = [&](const Ent& en) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // entry e of the granule is the segment's iff a <= e0 + e < b: (e0 - a) + e < b - a
        // unsigned (an entry below a wraps past it); granules past the chunk have a = b = 0
        const uint32_t a = en.ab[u] & 0xFFFFu, b = en.ab[u] >> 16;
        const uint32_t d = en.e0[u] - a, n = b - a;
        const uint32_t mm[4] = {en.m[u].x, en.m[u].y, en.m[u].z, en.m[u].w};
        // PACK: the first-appearance key is the exact row in a tile with row records, else the
        // tile's last row (per granule: the base key, and the rows in tile or zero)
        const bool hr = en.t[u] < rit_tiles;
        const uint32_t kb = en.t[u] * TR + (hr ? 0u : TR - 1u);
        const uint32_t r01 = PACK && hr ? en.rr[u].x : 0u, r23 = PACK && hr ? en.rr[u].y : 0u;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (d + (uint32_t)e >= n) continue;  // a neighbouring partition's entry
          const uint32_t sl = mm[e] & lowmask;
          if (PACK) {
            // fire-and-forget LDS atomics: nothing in the loop waits on the LDS
            const uint32_t rw = e < 2 ? r01 : r23;
            const uint32_t key = kb + ((e & 1) ? rw >> 16 : rw & 0xFFFFu);
            // count field + code16 (inc has no low bits, code16 < 2^16: an OR, one shift)
            atomicAdd(&acc[sl], ((unsigned long long)inc_hi << 32) | (mm[e] >> 16));
            atomicMin(&fst[sl], key);
            continue;
          }
          const uint32_t row = en.t[u] * TR + (mm[e] >> L.wbits);
          atomicAdd(&cnt[sl], 1u);
          atomicMin(&fst[sl], row);
#pragma unroll
          for (int q = 0; q < nsum; ++q) {
            // wide entries of an int64-codable float column (ScanParams::sum_enc): integer
            // code sums, the same whatever order the entries arrive in
            if (!NARROW && p.sum_is_float[q] && p.sum_enc[q] == 3) {
              // fixed-point limbs: integer sums, the same whatever order the entries arrive in
              const double xv = value_f64(en.v[u][e][q], p.sum_conv[q]);
              if (fx_finite(xv)) {
                long long l[3];
                fx_limbs(xv, fx_shift(p, q, ((uint64_t)part << L.wbits) + sl), l);
                atomicAdd(&acc[(size_t)q * W + sl], (unsigned long long)l[0]);
                atomicAdd(&fxl[(size_t)(kFxWords * q) * W + sl], (unsigned long long)l[1]);
                atomicAdd(&fxl[(size_t)(kFxWords * q + 1) * W + sl], (unsigned long long)l[2]);
              } else {
                atomicOr(&fxl[(size_t)(kFxWords * q + 2) * W + sl], fx_flag(xv));
              }
            } else if (!NARROW && p.sum_is_float[q] && p.sum_enc[q]) atomicAdd(&acc[(size_t)q * W + sl], (unsigned long long)part_sum_code(p, q, en.v[u][e][q]));
            else if (!NARROW && p.sum_is_float[q]) unsafeAtomicAdd(reinterpret_cast<double*>(&acc[(size_t)q * W + sl]), value_f64(en.v[u][e][q], p.sum_conv[q]));
            else atomicAdd(&acc[(size_t)q * W + sl], en.v[u][e][q]);
          }
        }
      }
    };
    // AH chunks in flight: each ring slot is consumed, then refilled in place (no exit
    // inside the body: a copy of a pending load would wait for every load in flight)
    auto run = [&](auto rit_c) {
      Ent ring[AH];
      uint32_t cstart[AH];
#pragma unroll
      for (int a = 0; a < AH; ++a) {
        cstart[a] = f_next;
        issue(ring[a], rit_c);
      }
      while (cstart[0] < e_hi) {
#pragma unroll
        for (int a = 0; a < AH; ++a) {
          consume(ring[a]);
          cstart[a] = f_next;
          issue(ring[a], rit_c);
        }
      }
    };
    // (C3: the row-record tiles are the first ~18 %; a window past them loads no row records --
    // 0.135 -> 0.122 ms for the aggregate with none at all, r5al)
    if (PACK && w0 >= (int64_t)rit_tiles) run(std::false_type{});
    else run(std::true_type{});
    lds_barrier();  // every wave is done with this window's bounds
    w0 += nw;
  }
  __syncthreads();
  // Split tables: with several splits per partition every workgroup stores its table to its own
  // partial record and k_part_combine adds the records in split order (the same sums whatever
  // the order the workgroups ran in); with one split the workgroup finishes its slots itself.
  // (An in-kernel hand-off -- the last split to arrive adds the others' records after an agent
  // release / acquire -- cost ~130 us at C3: every workgroup's release writes back its XCD's L2.)
  const uint64_t slot0 = (uint64_t)part << L.wbits;
  const int nvalid = (int)((uint64_t)W < p.nslots - slot0 ? (uint64_t)W : p.nslots - slot0);
  if (PACK) {
    // the workgroup's totals (flushed + LDS), unpacked: [W] counts, [W] code16 sums, [W] first
    // tiles; one split finishes its slots itself
    for (int s = tid; s < nvalid; s += blockDim.x) {
      const unsigned long long a = acc[s];
      unsigned long long c = a >> L.sbits, sm = a & smask;
      if (flushed) {
        c += rec_cnt[s];
        sm += rec_sum[s];
      }
      if (L.splits > 1) {
        rec_cnt[s] = c;
        rec_sum[s] = sm;
        rec_fst[s] = fst[s];
      } else {
        PartRec<NV> r;
        r.c64 = c;
        r.a[0] = sm;
        r.f = fst[s];
        part_finish_slot<NSUM, NARROW, PACK>(p, L, sa, slot0 + s, 1, [&](int, PartRec<NV>& o) { o = r; });
      }
    }
    return;
  }
  if (L.splits > 1) {
    unsigned char* rec = L.partial + ((size_t)part * L.splits + split) * L.partial_bytes;
    {  // [W] counts, [W] first rows, then [nsum][W] sums (fx: then [nsum][kFxWords][W] limbs / flags)
      uint32_t* pc = reinterpret_cast<uint32_t*>(rec);
      uint32_t* pf = pc + W;
      unsigned long long* pa = reinterpret_cast<unsigned long long*>(pf + W);
      for (int s = tid; s < nvalid; s += blockDim.x) {
        pc[s] = cnt[s];
        pf[s] = fst[s];
#pragma unroll
        for (int q = 0; q < nsum; ++q) pa[(size_t)q * W + s] = acc[(size_t)q * W + s];
        if (fx)
          for (int h = 0; h < kFxWords * nsum; ++h) pa[(size_t)(nsum + h) * W + s] = fxl[(size_t)h * W + s];
      }
    }
    return;
  }
  for (int s = tid; s < nvalid; s += blockDim.x) {
    PartRec<NV> r;
    r.f = fst[s];
    r.c = PACK ? 0u : cnt[s];
#pragma unroll
    for (int q = 0; q < (PACK ? 1 : nsum); ++q) {
      r.a[q] = acc[(size_t)q * W + s];
      r.x[q][0] = fx ? fxl[(size_t)(kFxWords * q) * W + s] : 0ull;
      r.x[q][1] = fx ? fxl[(size_t)(kFxWords * q + 1) * W + s] : 0ull;
      r.x[q][2] = fx ? fxl[(size_t)(kFxWords * q + 2) * W + s] : 0ull;
    }
    part_finish_slot<NSUM, NARROW, PACK>(p, L, sa, slot0 + s, 1, [&](int, PartRec<NV>& o) { o = r; });
  }
}

// The split records of a partition added in split order, one thread per slot (coalesced).
template <int NSUM, bool NARROW, bool PACK>
__global__ __launch_bounds__(256) void k_part_combine(ScanParams p, PartLaunch L, SlotArrays sa) {
  constexpr int NV = NSUM > 0 ? NSUM : 1;
  const int W = 1 << L.wbits, S = L.splits;
  for (uint64_t gs = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; gs < p.nslots; gs += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t part = gs >> L.wbits;
    const int s = (int)(gs & (uint64_t)(W - 1));
    part_finish_slot<NSUM, NARROW, PACK>(p, L, sa, gs, S, [&](int o, PartRec<NV>& r) {
      const unsigned char* rec = L.partial + ((size_t)part * S + o) * L.partial_bytes;
      if (PACK) {
        const unsigned long long* pc = reinterpret_cast<const unsigned long long*>(rec);
        r.c64 = pc[s];
        r.a[0] = pc[W + s];
        r.f = reinterpret_cast<const uint32_t*>(pc + 2 * W)[s];
      } else {
        const uint32_t* pc = reinterpret_cast<const uint32_t*>(rec);
        const unsigned long long* pa = reinterpret_cast<const unsigned long long*>(pc + 2 * W);
        r.c = pc[s];
        r.f = pc[W + s];
        const bool fx = !NARROW && L.fx;
#pragma unroll
        for (int q = 0; q < NSUM; ++q) {
          r.a[q] = pa[(size_t)q * W + s];
          r.x[q][0] = fx ? pa[(size_t)(NSUM + kFxWords * q) * W + s] : 0ull;
          r.x[q][1] = fx ? pa[(size_t)(NSUM + kFxWords * q + 1) * W + s] : 0ull;
          r.x[q][2] = fx ? pa[(size_t)(NSUM + kFxWords * q + 2) * W + s] : 0ull;
        }
      }
    });
  }
}

template <int NC>
__global__ __launch_bounds__(kFirstRowsBlock) void k_part_first_rows(ScanParams p, PartLaunch L, SlotArrays sa) {
  part_first_rows_body<NC>(p, L, sa);
}

// ------------------------------------------------------------------------------------
// Multi-workgroup exclusive scan of uint32 (3 launches): per-1024-segment scan with segment
// totals, scan of the totals (recursively small), add-back.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_scan_seg(uint32_t* v, uint64_t n, uint32_t* seg_totals) {
  const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  const uint32_t x = i < n ? v[i] : 0u;
  uint32_t tot;
  const uint32_t e = block_excl_scan_1024(x, &tot);
  if (i < n) v[i] = e;
  if (threadIdx.x == 0) seg_totals[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_scan_add(uint32_t* v, uint64_t n, const uint32_t* seg_offsets) {
  const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  if (i < n) v[i] += seg_offsets[blockIdx.x];
}

void launch_exclusive_scan_u32(uint32_t* v, uint64_t n, uint32_t* scratch, hipStream_t st) {
  // scratch: >= 2 * ceil(n / 1024) + 2048 words
  if (n == 0) return;
  const uint64_t segs = (n + 1023) / 1024;
  uint32_t* totals = scratch;
  hipLaunchKernelGGL(k_scan_seg, dim3((unsigned)segs), dim3(1024), 0, st, v, n, totals);
  if (segs > 1) {
    launch_exclusive_scan_u32(totals, segs, scratch + segs + 1, st);
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)segs), dim3(1024), 0, st, v, n, totals);
  }
}

#ifndef BQG_PART_MICRO  // tools/micro/part_micro.hip includes this file for the aggregate kernel
void launch_partitioned(const ScanParams& p, const SlotArrays& s, const PartLaunch& L, hipStream_t st,
                        hipFunction_t fscatter, hipFunction_t ffirst) {
  const size_t scatter_lds = part_scatter_lds(L.nparts, L.threads, p.nsum, L.k, L.narrow != 0, L.pack != 0);
  if (fscatter) {
    PartLaunch Lc = L;
    ScanParams pc = p;
    void* args[] = {(void*)&pc, (void*)&Lc};
    (void)hipModuleLaunchKernel(fscatter, (unsigned)L.blocks, 1, 1, (unsigned)L.threads, 1, 1, (unsigned)scatter_lds,
                                st, args, nullptr);
  } else {
#define BQG_SCATTER(K, NW, PK) BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_part_scatter<NC, K, NW, PK>), dim3(L.blocks), dim3(L.threads), scatter_lds, st, p, L))
    if (L.k == 4) {
      BQG_SCATTER(4, true, true);  // 16384-row tiles: packed entries only (LDS)
    } else if (L.k == 2) {
      if (L.pack) {
        BQG_SCATTER(2, true, true);
      } else if (L.narrow) {
        BQG_SCATTER(2, true, false);
      } else {
        BQG_SCATTER(2, false, false);
      }
    } else {
      if (L.pack) {
        BQG_SCATTER(1, true, true);
      } else if (L.narrow) {
        BQG_SCATTER(1, true, false);
      } else {
        BQG_SCATTER(1, false, false);
      }
    }
#undef BQG_SCATTER
  }
  const size_t agg_lds = part_agg_lds_launch(L.wbits, p.nsum, L.pack != 0, L.win, L.fx != 0);
  const unsigned grid = (unsigned)(((L.nparts + 7) / 8) * 8 * L.splits);
  const unsigned cgrid = (unsigned)std::min<uint64_t>((p.nslots + 255) / 256, 4096);
  if (L.pack) {
    // (the tile marks and the list's length are zeroed by the scatter)
#define BQG_AGGP(NS) hipLaunchKernelGGL((k_part_aggregate<2, 2, NS, true, true>), dim3(grid), dim3(1024), agg_lds, st, p, L, s)
    if (p.nsum == 0) BQG_AGGP(0); else BQG_AGGP(1);
#undef BQG_AGGP
    if (L.splits > 1) {
      if (p.nsum == 0) hipLaunchKernelGGL((k_part_combine<0, true, true>), dim3(cgrid), dim3(256), 0, st, p, L, s);
      else hipLaunchKernelGGL((k_part_combine<1, true, true>), dim3(cgrid), dim3(256), 0, st, p, L, s);
    }
    // grid-stride over 4096-row units of the tiles (the marked ones are mostly a prefix on
    // random keys)
    // (grid-stride over the marked tiles' units; the list's length is read on the device)
    const int64_t funits = L.ntiles * ((L.tile_rows + kFirstRowsUnit - 1) / kFirstRowsUnit);
    const unsigned fgrid = (unsigned)std::min<int64_t>(funits, 512);
    if (ffirst) {
      PartLaunch Lc = L;
      ScanParams pc = p;
      SlotArrays sc = s;
      void* args[] = {(void*)&pc, (void*)&Lc, (void*)&sc};
      (void)hipModuleLaunchKernel(ffirst, fgrid, 1, 1, kFirstRowsBlock, 1, 1, 0, st, args, nullptr);
    } else {
      BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_part_first_rows<NC>), dim3(fgrid), dim3(kFirstRowsBlock), 0, st, p, L, s));
    }
    return;
  }
#define BQG_AGG2(U, NS, NW) do { \
    hipLaunchKernelGGL((k_part_aggregate<U, 2, NS, NW, false>), dim3(grid), dim3(1024), agg_lds, st, p, L, s); \
    if (L.splits > 1) hipLaunchKernelGGL((k_part_combine<NS, NW, false>), dim3(cgrid), dim3(256), 0, st, p, L, s); \
  } while (0)
#define BQG_AGG(U, NS) do { if (L.narrow) BQG_AGG2(U, NS, true); else BQG_AGG2(U, NS, false); } while (0)
  switch (p.nsum) {
    case 0: BQG_AGG2(2, 0, false); break;
    case 1: BQG_AGG(2, 1); break;
    case 2: BQG_AGG(1, 2); break;
    case 3: BQG_AGG(1, 3); break;
    default: BQG_AGG(1, 4); break;
  }
#undef BQG_AGG
#undef BQG_AGG2
}
#endif

}  // namespace bqg
