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
// slot's first tile, and the combine leaves first rows to k_part_first_rows.
template <int G, int U, int NSUM, bool NARROW, bool PACK = false>
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
  uint32_t* fst = PACK ? cnt : cnt + W;                                    // [W] first row (PACK: first tile)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, NW = (int)(blockDim.x >> 6);
  for (int i = tid; i < W; i += blockDim.x) {
    if (!PACK) cnt[i] = 0;
    fst[i] = kNoRow;
  }
  for (int i = tid; i < (PACK ? 1 : nsum) * W; i += blockDim.x) acc[i] = 0;
  const unsigned long long inc = PACK ? 1ull << L.sbits : 0ull;  // one row in the packed count field
  __syncthreads();
  const int64_t nt = L.ntiles;
  // (splits <= ntiles: every split's tile range is non-empty, and every split must reach the
  // combine below)
  const int64_t t_lo = nt * split / L.splits, t_hi = nt * (split + 1) / L.splits;
  const uint32_t lowmask = (uint32_t)W - 1u;
  const uint32_t TR = (uint32_t)L.tile_rows;
  auto hload = [&](int64_t tg, uint32_t& s0, uint32_t& s1) {
    const int64_t t = tg + lane;
    const bool valid = lane < G && t < t_hi;
    const uint16_t* th = L.hdr + (size_t)(valid ? t : t_lo) * (size_t)(P + 1) + part;
    const uint32_t a = th[0], b = th[1];
    s0 = valid ? a : 0u;
    s1 = valid ? b : 0u;
  };
  constexpr int NV = NSUM > 0 ? NSUM : 1;
  // one group of G tiles: flattened segment starts (wave-uniform), the per-lane index base
  // (lane j: entry index of tile j's segment start minus its flattened position) and the total
  struct Grp {
    uint32_t ex[G];
    uint32_t dl, total;
    size_t gbase;
    uint32_t tile0;
  };
  // one U x 64-entry load of a group
  struct Ent {
    uint32_t m[U], rowb[U];
    unsigned long long v[U][NV];
  };
  auto prep = [&](int64_t tg, uint32_t s0, uint32_t s1, Grp& g) {
    const uint32_t len = s1 - s0;
    const uint32_t incl = wave_incl_scan_u32(len, lane);
    const uint32_t excl = incl - len;
    g.total = (uint32_t)__builtin_amdgcn_readlane((int)incl, G - 1);
#pragma unroll
    for (int j = 0; j < G; ++j) g.ex[j] = (uint32_t)__builtin_amdgcn_readlane((int)excl, j);
    g.dl = (uint32_t)lane * TR + s0 - excl;
    g.gbase = (size_t)tg * TR;
    g.tile0 = (uint32_t)tg;
  };
  // unconditional loads (an empty group -- past the range -- reads entry 0; the value array
  // exists even without a summed column): the same loads on every path, so the compiler
  // waits for exactly the set it consumes
  auto issue = [&](const Grp& g, uint32_t e0, Ent& en) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t e = e0 + u * 64u + lane;
      const uint32_t ec = e < g.total ? e : (g.total ? g.total - 1u : 0u);
      uint32_t j0 = 0;
#pragma unroll
      for (int j = 1; j < G; ++j) j0 += ec >= g.ex[j] ? 1u : 0u;
      size_t idx = g.gbase + (uint32_t)__shfl((int)g.dl, (int)j0, 64) + ec;
      idx = g.total ? idx : 0;
      en.rowb[u] = PACK ? g.tile0 + j0 : (uint32_t)g.gbase + j0 * TR;  // PACK: the tile
      en.m[u] = L.meta[idx];
      if (PACK) continue;
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        if (NARROW) {  // the exact 32-bit code: float codes signed, integer offsets unsigned
          const uint32_t code = reinterpret_cast<const uint32_t*>(L.vals)[(size_t)q * L.capacity + idx];
          en.v[u][q] = L.enc_kind[q] == 3 ? (unsigned long long)code : (unsigned long long)(long long)(int32_t)code;
        }
        else
          en.v[u][q] = L.vals[(size_t)q * L.capacity + idx];
      }
    }
  };
  auto consume = [&](const Grp& g, uint32_t e0, const Ent& en) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t e = e0 + u * 64u + lane;
      if (e >= g.total) continue;
      const uint32_t sl = en.m[u] & lowmask;
      if (PACK) {
        atomicAdd(&acc[sl], inc + (unsigned long long)(en.m[u] >> 16));
        if (fst[sl] > en.rowb[u]) atomicMin(&fst[sl], en.rowb[u]);
        continue;
      }
      const uint32_t row = en.rowb[u] + (en.m[u] >> L.wbits);
      atomicAdd(&cnt[sl], 1u);
      if (fst[sl] > row) atomicMin(&fst[sl], row);
#pragma unroll
      for (int q = 0; q < nsum; ++q) {
        if (!NARROW && p.sum_is_float[q]) unsafeAtomicAdd(reinterpret_cast<double*>(&acc[(size_t)q * W + sl]), value_f64(en.v[u][q], p.sum_conv[q]));
        else atomicAdd(&acc[(size_t)q * W + sl], en.v[u][q]);
      }
    }
  };
  // entries of a group beyond its first U x 64 (segments longer than the typical tile share)
  auto rest = [&](const Grp& g, Ent& en) {
    for (uint32_t e0 = 64u * U; e0 < g.total; e0 += 64u * U) {
      issue(g, e0, en);
      consume(g, e0, en);
    }
  };
  const int64_t stride = (int64_t)NW * G;
  int64_t tg = t_lo + (int64_t)wave * G;
  uint32_t ha0, ha1, hb0, hb1;  // headers of the groups two and three ahead, in turn
  Grp ga, gb;
  Ent ea, eb;
  hload(tg, ha0, ha1);
  hload(tg + stride, hb0, hb1);
  prep(tg, ha0, ha1, ga);
  issue(ga, 0, ea);
  hload(tg + 2 * stride, ha0, ha1);
  for (; tg < t_hi; tg += 2 * stride) {
    // group tg in (ga, ea); group tg + stride's header in hb
    prep(tg + stride, hb0, hb1, gb);
    issue(gb, 0, eb);
    hload(tg + 3 * stride, hb0, hb1);
    consume(ga, 0, ea);
    rest(ga, ea);
    if (tg + stride >= t_hi) break;
    // group tg + stride in (gb, eb); group tg + 2 * stride's header in ha
    prep(tg + 2 * stride, ha0, ha1, ga);
    issue(ga, 0, ea);
    hload(tg + 4 * stride, ha0, ha1);
    consume(gb, 0, eb);
    rest(gb, eb);
  }
  __syncthreads();
  // Combine the partition's split tables without device atomics (and without a slot-array
  // initialisation pass): every split stores its table to its own partial record, the last
  // split to arrive (one agent-scope counter per partition, zeroed before the launch) adds the
  // records in split order -- the same sums whatever the arrival order -- and writes every slot
  // of the partition, empty ones included.  Hand-off: plain stores, each wave drains, barrier,
  // one lane's agent release, then the counter; the last arriver acquires before reading
  // (cdna_hip_programming.md Guideline 16).  Nobody waits: no spin, no residency assumption.
  const uint64_t slot0 = (uint64_t)part << L.wbits;
  const int nvalid = (int)((uint64_t)W < p.nslots - slot0 ? (uint64_t)W : p.nslots - slot0);
  const int S = L.splits;
  __shared__ unsigned int s_last;
  if (S > 1) {
    uint32_t* pc = reinterpret_cast<uint32_t*>(L.partial + ((size_t)part * S + split) * L.partial_bytes);
    if (PACK) {  // [W] packed accumulators, then [W] first tiles
      unsigned long long* pa = reinterpret_cast<unsigned long long*>(pc);
      uint32_t* pf = reinterpret_cast<uint32_t*>(pa + W);
      for (int s = tid; s < W; s += blockDim.x) {
        pa[s] = acc[s];
        pf[s] = fst[s];
      }
    }
    uint32_t* pf = pc + W;
    unsigned long long* pa = reinterpret_cast<unsigned long long*>(pf + W);
    for (int s = tid; !PACK && s < W; s += blockDim.x) {
      pc[s] = cnt[s];
      pf[s] = fst[s];
#pragma unroll
      for (int q = 0; q < nsum; ++q) pa[(size_t)q * W + s] = acc[(size_t)q * W + s];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned int old = __hip_atomic_fetch_add(&L.arrive[part], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = old == (unsigned int)(S - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      s_last = last ? 1u : 0u;
    }
    __syncthreads();
    if (!s_last) return;
  }
  if (PACK) {
    // unpack every split's accumulator before adding (the packed fields of a sum over splits
    // could carry into each other); exact code sum = sum of code16 + count x enc_base16
    const unsigned long long smask = (1ull << L.sbits) - 1ull;
    for (int s = tid; s < nvalid; s += blockDim.x) {
      unsigned long long c = 0, cs = 0;
      uint32_t f = kNoRow;
      for (int o = 0; o < S; ++o) {
        unsigned long long a;
        uint32_t of;
        if (o == split) {
          a = acc[s];
          of = fst[s];
        } else {
          const unsigned long long* pa =
              reinterpret_cast<const unsigned long long*>(L.partial + ((size_t)part * S + o) * L.partial_bytes);
          a = pa[s];
          of = reinterpret_cast<const uint32_t*>(pa + W)[s];
        }
        c += a >> L.sbits;
        cs += a & smask;
        f = of < f ? of : f;
      }
      const uint64_t gs = slot0 + s;
      sa.cnt[gs] = c;
      sa.fst[gs] = kNoRow;  // k_part_first_rows
      if (f != kNoRow) {
        L.tile_mark[f] = 1;
        L.first_tag[gs] = (unsigned char)f;
      }
      if (nsum) {
        unsigned long long tot = cs + c * (unsigned long long)L.enc_base16;
        if (L.enc_kind[0] == 3) tot += c * (unsigned long long)L.enc_off[0];
        else tot = as_u64((double)(long long)tot / L.enc_mul[0]);
        sa.acc[gs] = tot;
      }
    }
    return;
  }
  for (int s = tid; s < nvalid; s += blockDim.x) {
    uint32_t c = 0, f = kNoRow;
    unsigned long long a[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) a[q] = 0;
    for (int o = 0; o < S; ++o) {
      uint32_t oc, of;
      unsigned long long oa[NV];
      if (o == split) {
        oc = cnt[s];
        of = fst[s];
#pragma unroll
        for (int q = 0; q < nsum; ++q) oa[q] = acc[(size_t)q * W + s];
      } else {
        const uint32_t* pc = reinterpret_cast<const uint32_t*>(L.partial + ((size_t)part * S + o) * L.partial_bytes);
        const unsigned long long* pa = reinterpret_cast<const unsigned long long*>(pc + 2 * W);
        oc = pc[s];
        of = pc[W + s];
#pragma unroll
        for (int q = 0; q < nsum; ++q) oa[q] = pa[(size_t)q * W + s];
      }
      c += oc;
      f = of < f ? of : f;
#pragma unroll
      for (int q = 0; q < nsum; ++q) {
        if (!NARROW && p.sum_is_float[q]) a[q] = as_u64(as_f64(a[q]) + as_f64(oa[q]));
        else a[q] += oa[q];
      }
    }
    const uint64_t gs = slot0 + s;
    sa.cnt[gs] = c;
    sa.fst[gs] = f;
#pragma unroll
    for (int q = 0; q < nsum; ++q) {
      // narrow: the exact sum of the codes, scaled back once (dyadic: exact below 2^53), or
      // shifted back by count x offset (integers, modulo 2^64 like the 64-bit accumulator)
      if (NARROW) {
        if (L.enc_kind[q] == 3) a[q] += (unsigned long long)c * (unsigned long long)L.enc_off[q];
        else a[q] = as_u64((double)(long long)a[q] / L.enc_mul[q]);
      }
      sa.acc[(size_t)q * p.nslots + gs] = a[q];
    }
  }
}

template <int NC>
__global__ __launch_bounds__(1024) void k_part_first_rows(ScanParams p, PartLaunch L, SlotArrays sa) {
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
  const size_t agg_lds = part_agg_lds(L.wbits, p.nsum, L.pack != 0);
  const unsigned grid = (unsigned)(((L.nparts + 7) / 8) * 8 * L.splits);
  if (L.pack) {
    (void)hipMemsetAsync(L.tile_mark, 0, (size_t)L.ntiles, st);
#define BQG_AGGP(G, U, NS) hipLaunchKernelGGL((k_part_aggregate<G, U, NS, true, true>), dim3(grid), dim3(1024), agg_lds, st, p, L, s)
    const bool big = L.tile_rows > 4096;
    if (p.nsum == 0) {
      if (big) BQG_AGGP(4, 4, 0); else BQG_AGGP(8, 4, 0);
    } else {
      if (big) BQG_AGGP(4, 4, 1); else BQG_AGGP(8, 4, 1);
    }
#undef BQG_AGGP
    // grid-stride over the tiles (the marked ones are mostly a prefix on random keys)
    const unsigned fgrid = (unsigned)std::min<int64_t>(L.ntiles, 2048);
    if (ffirst) {
      PartLaunch Lc = L;
      ScanParams pc = p;
      SlotArrays sc = s;
      void* args[] = {(void*)&pc, (void*)&Lc, (void*)&sc};
      (void)hipModuleLaunchKernel(ffirst, fgrid, 1, 1, 1024, 1, 1, 0, st, args, nullptr);
    } else {
      BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_part_first_rows<NC>), dim3(fgrid), dim3(1024), 0, st, p, L, s));
    }
    return;
  }
  // G tiles per wave group: ~8 x 4096 rows of segments whichever the tile size
#define BQG_AGG2(G, U, NS, NW) hipLaunchKernelGGL((k_part_aggregate<G, U, NS, NW>), dim3(grid), dim3(1024), agg_lds, st, p, L, s)
#define BQG_AGG(G, U, NS) do { if (L.narrow) BQG_AGG2(G, U, NS, true); else BQG_AGG2(G, U, NS, false); } while (0)
  const bool big = L.tile_rows > 4096;
  switch (p.nsum) {
    case 0: if (big) BQG_AGG2(4, 4, 0, false); else BQG_AGG2(8, 4, 0, false); break;
    case 1: if (big) BQG_AGG(4, 4, 1); else BQG_AGG(8, 4, 1); break;
    case 2: if (big) BQG_AGG(4, 4, 2); else BQG_AGG(8, 4, 2); break;
    case 3: if (big) BQG_AGG(4, 2, 3); else BQG_AGG(8, 2, 3); break;
    default: if (big) BQG_AGG(4, 2, 4); else BQG_AGG(8, 2, 4); break;
  }
#undef BQG_AGG
#undef BQG_AGG2
}
#endif

}  // namespace bqg
