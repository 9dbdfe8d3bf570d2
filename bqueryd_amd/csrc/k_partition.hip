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
#include <hip/hip_runtime.h>

#include <algorithm>

#include "partition.h"

namespace bqg {

template <int NC>
__global__ __launch_bounds__(kPartBlock) void k_part_scatter(ScanParams p, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  part_scatter_body<NC>(p, L, smem);
}

// Aggregate over the tile layout.  Workgroup (partition, split): the split's tile range.  A
// wave takes groups of G consecutive tiles; lane j < G holds tile j's segment bounds (the
// headers of the next two groups are in flight while a group is aggregated), a wave scan of
// the segment lengths flattens the group, and each of U wave-wide iterations in flight reads
// 64 consecutive entries of the flattened group: an entry finds its tile with G - 1 compares
// against wave-uniform segment starts and takes that tile's first index with one lane
// shuffle.  Workgroups are mapped XCD-aware: the workgroups of one XCD (blockIdx % 8) take
// consecutive partitions over the same tile range, so the edge lines their segments share
// are read once into that XCD's L2.
template <int G, int U, int NSUM>
__global__ __launch_bounds__(1024) void k_part_aggregate(ScanParams p, PartLaunch L, SlotArrays sa) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int P = L.nparts;
  const int per_x = (P + 7) / 8;
  const int bx = (int)(blockIdx.x & 7u), bi = (int)(blockIdx.x >> 3);
  const int part = bx * per_x + bi % per_x, split = bi / per_x;
  if (part >= P || split >= L.splits) return;  // the whole workgroup
  const int W = 1 << L.wbits;
  constexpr int nsum = NSUM;
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem);  // [nsum][W]
  uint32_t* cnt = reinterpret_cast<uint32_t*>(acc + (size_t)nsum * W);    // [W]
  uint32_t* fst = cnt + W;                                                 // [W]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, NW = (int)(blockDim.x >> 6);
  for (int i = tid; i < W; i += blockDim.x) {
    cnt[i] = 0;
    fst[i] = kNoRow;
  }
  for (int i = tid; i < nsum * W; i += blockDim.x) acc[i] = 0;
  __syncthreads();
  const int64_t nt = L.ntiles;
  const int64_t t_lo = nt * split / L.splits, t_hi = nt * (split + 1) / L.splits;
  if (t_lo >= t_hi) return;  // the whole workgroup: an empty tile range leaves the table empty
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
  const int64_t stride = (int64_t)NW * G;
  int64_t tg = t_lo + (int64_t)wave * G;
  uint32_t a0, a1, b0, b1;
  hload(tg, a0, a1);
  hload(tg + stride, b0, b1);
  for (; tg < t_hi; tg += stride) {
    const uint32_t s0 = a0, s1 = a1;
    a0 = b0;
    a1 = b1;
    hload(tg + 2 * stride, b0, b1);
    const uint32_t len = s1 - s0;
    const uint32_t incl = wave_incl_scan_u32(len, lane);
    const uint32_t excl = incl - len;
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, G - 1);
    uint32_t ex[G];
#pragma unroll
    for (int j = 0; j < G; ++j) ex[j] = (uint32_t)__builtin_amdgcn_readlane((int)excl, j);
    // lane j: entry index of tile j's segment start minus the segment's flattened position
    // (relative to the group's first tile): entry index = that + flattened position
    const uint32_t dl = (uint32_t)lane * TR + s0 - excl;
    const size_t gbase = (size_t)tg * TR;
    for (uint32_t e0 = 0; e0 < total; e0 += 64u * U) {
      constexpr int NV = NSUM > 0 ? NSUM : 1;
      uint32_t m[U], rowb[U];
      unsigned long long v[U][NV];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = e0 + u * 64u + lane;
        const uint32_t ec = e < total ? e : total - 1u;
        uint32_t j0 = 0;
#pragma unroll
        for (int j = 1; j < G; ++j) j0 += ec >= ex[j] ? 1u : 0u;
        const size_t idx = gbase + (uint32_t)__shfl((int)dl, (int)j0, 64) + ec;
        rowb[u] = (uint32_t)gbase + j0 * TR;
        // unconditional loads (the value array exists even without a summed column): the
        // same loads on every path, so the next group's headers stay in flight
        m[u] = L.meta[idx];
#pragma unroll
        for (int q = 0; q < NV; ++q) v[u][q] = L.vals[(size_t)q * L.capacity + idx];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = e0 + u * 64u + lane;
        if (e >= total) continue;
        const uint32_t sl = m[u] & lowmask;
        const uint32_t row = rowb[u] + (m[u] >> L.wbits);
        atomicAdd(&cnt[sl], 1u);
        if (fst[sl] > row) atomicMin(&fst[sl], row);
#pragma unroll
        for (int q = 0; q < nsum; ++q) {
          if (p.sum_is_float[q]) unsafeAtomicAdd(reinterpret_cast<double*>(&acc[(size_t)q * W + sl]), value_f64(v[u][q], p.sum_conv[q]));
          else atomicAdd(&acc[(size_t)q * W + sl], v[u][q]);
        }
      }
    }
  }
  __syncthreads();
  const uint64_t slot0 = (uint64_t)part << L.wbits;
  for (int s = tid; s < W; s += blockDim.x) {
    const uint32_t c = cnt[s];
    if (c == 0) continue;
    const uint64_t gs = slot0 + s;
    atomicAdd(&sa.cnt[gs], (unsigned long long)c);
    atomicMin(&sa.fst[gs], fst[s]);
#pragma unroll
    for (int q = 0; q < nsum; ++q) {
      const unsigned long long a = acc[(size_t)q * W + s];
      if (p.sum_is_float[q]) unsafeAtomicAdd(reinterpret_cast<double*>(&sa.acc[(size_t)q * p.nslots + gs]), as_f64(a));
      else atomicAdd(&sa.acc[(size_t)q * p.nslots + gs], a);
    }
  }
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
                        hipFunction_t fscatter) {
  const size_t scatter_lds = part_scatter_lds(L.nparts, L.threads, p.nsum);
  if (fscatter) {
    PartLaunch Lc = L;
    ScanParams pc = p;
    void* args[] = {(void*)&pc, (void*)&Lc};
    (void)hipModuleLaunchKernel(fscatter, (unsigned)L.blocks, 1, 1, (unsigned)L.threads, 1, 1, (unsigned)scatter_lds,
                                st, args, nullptr);
  } else {
    BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_part_scatter<NC>), dim3(L.blocks), dim3(L.threads), scatter_lds, st, p, L));
  }
  const size_t agg_lds = ((size_t)1 << L.wbits) * (8 + 8 * (size_t)p.nsum);
  const unsigned grid = (unsigned)(((L.nparts + 7) / 8) * 8 * L.splits);
  switch (p.nsum) {
    case 0: hipLaunchKernelGGL((k_part_aggregate<8, 4, 0>), dim3(grid), dim3(1024), agg_lds, st, p, L, s); break;
    case 1: hipLaunchKernelGGL((k_part_aggregate<8, 4, 1>), dim3(grid), dim3(1024), agg_lds, st, p, L, s); break;
    case 2: hipLaunchKernelGGL((k_part_aggregate<8, 4, 2>), dim3(grid), dim3(1024), agg_lds, st, p, L, s); break;
    case 3: hipLaunchKernelGGL((k_part_aggregate<8, 2, 3>), dim3(grid), dim3(1024), agg_lds, st, p, L, s); break;
    default: hipLaunchKernelGGL((k_part_aggregate<8, 2, 4>), dim3(grid), dim3(1024), agg_lds, st, p, L, s); break;
  }
}
#endif

}  // namespace bqg
