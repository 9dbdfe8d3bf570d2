// k_partition.hip -- partitioned aggregation for large dense slot spaces (config C3: ~1 M
// groups), and a multi-workgroup exclusive scan.
//
// Per-row device atomics on a 1 M-slot table are random 8-byte memory-side operations
// (MI355X_MICROARCH.md §Global float atomics: they execute past L2).  Instead:
//   count:     each workgroup owns a contiguous row range and histograms its passing rows by
//              partition p = slot >> wbits (LDS atomics) -> counts[p][block]; it reads only
//              the key / filter columns;
//   scan:      exclusive scan of counts in [p][block] order -> the offset of every
//              (partition, workgroup) region; partitions are contiguous in the entry arrays;
//   scatter:   the workgroup re-reads its rows one tile at a time, counting-sorts the tile by
//              partition in LDS and copies the sorted tile out as runs (consecutive lanes
//              write consecutive entries of one region: whole cache lines, no write-allocate
//              of half-written lines);
//   aggregate: workgroups per partition walk its regions, aggregate the entries in an LDS
//              table of 2^wbits slots and flush the occupied slots.
// Entries are structure-of-arrays: a 32-bit meta word ((row - block begin) << wbits |
// slot_low; the region identifies the block) and one 64-bit value per summed column.
// Traffic per row (C3, one f64 sum): keys 8 (count) + 16 (scatter read) + 12 written + 12
// read back = 48 bytes against the 16 algorithmic bytes.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "partition.h"

namespace bqg {

template <int NC>
__global__ __launch_bounds__(kPartBlock) void k_part_count(ScanParams p, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  part_count_body<NC>(p, L, smem);
}

template <int NC>
__global__ __launch_bounds__(kPartBlock) void k_part_scatter(ScanParams p, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  part_scatter_body<NC>(p, L, smem);
}

// One workgroup per (partition, split): the split's share of the partition's entries, four
// consecutive entries per thread (16-byte loads), the block of each entry -- hence its row --
// from the partition's region starts in LDS.
__global__ __launch_bounds__(1024) void k_part_aggregate(ScanParams p, PartLaunch L, SlotArrays sa) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int W = 1 << L.wbits;
  const int nsum = p.nsum;
  const int B = L.blocks;
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem);  // [nsum][W]
  uint32_t* cnt = reinterpret_cast<uint32_t*>(acc + (size_t)nsum * W);    // [W]
  uint32_t* fst = cnt + W;                                                 // [W]
  uint32_t* rs = fst + W;                                                  // [B + 1] region starts
  const int tid = threadIdx.x;
  const int part = blockIdx.x / L.splits, split = blockIdx.x % L.splits;
  for (int i = tid; i < W; i += blockDim.x) {
    cnt[i] = 0;
    fst[i] = kNoRow;
  }
  for (int i = tid; i < nsum * W; i += blockDim.x) acc[i] = 0;
  for (int i = tid; i <= B; i += blockDim.x) rs[i] = L.counts[(size_t)part * B + i];
  __syncthreads();
  const uint32_t pbeg = rs[0], pend = rs[B];
  const uint64_t len = pend - pbeg;
  const uint32_t lo = pbeg + (uint32_t)(len * split / L.splits);
  const uint32_t hi = pbeg + (uint32_t)(len * (split + 1) / L.splits);
  const uint32_t lowmask = (uint32_t)W - 1u;
  const uint32_t c4e = (hi + 3u) >> 2;
  uint32_t c4 = (lo >> 2) + tid;
  // entries are visited in increasing order: the region of a thread's next entry is found by
  // walking forward from its last one (a few LDS reads), falling back to a binary search
  int b = 0;
  auto region_of = [&](uint32_t key) {  // largest b with rs[b] <= key
    for (int k = 0; k < 8; ++k) {
      if (rs[b + 1] > key) return;
      ++b;
    }
    int e = B - 1;
    while (b < e) {
      const int mid = (b + e + 1) >> 1;
      if (rs[mid] <= key) b = mid;
      else e = mid - 1;
    }
  };
  // two iterations' meta and first summed column are in flight while one is aggregated
  // (clamped to the last group of the range: the same loads on every path, so the compiler
  // waits for the oldest group with vmcnt(N) instead of draining)
  const bool pre_v = nsum > 0;
  const unsigned char* v0 = reinterpret_cast<const unsigned char*>(L.vals);
  struct Grp {
    uint4 m, v01, v23;
  };
  auto fetch = [&](uint32_t cc) {
    Grp g;
    cc = cc < c4e ? cc : (c4e > 0u ? c4e - 1u : 0u);
    g.m = load_stream16(reinterpret_cast<const unsigned char*>(L.meta + ((size_t)cc << 2)));
    if (pre_v) {
      g.v01 = load_stream16(v0 + ((size_t)cc << 5));
      g.v23 = load_stream16(v0 + ((size_t)cc << 5) + 16);
    } else {
      g.v01 = g.m;
      g.v23 = g.m;
    }
    return g;
  };
  auto consume = [&](const Grp& g, uint32_t cc) {
    const uint32_t i0 = cc << 2;
    if (i0 >= hi) return;
    region_of(max(i0, lo));
    const uint32_t mm[4] = {g.m.x, g.m.y, g.m.z, g.m.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t i = i0 + k;
      if (i < lo || i >= hi) continue;
      while (i >= rs[b + 1]) ++b;
      const uint32_t s = mm[k] & lowmask;
      const uint32_t row = (uint32_t)(L.row_base + (int64_t)b * L.rows_per_block) + (mm[k] >> L.wbits);
      atomicAdd(&cnt[s], 1u);
      if (fst[s] > row) atomicMin(&fst[s], row);
    }
    for (int q = 0; q < nsum; ++q) {
      const unsigned char* vp = reinterpret_cast<const unsigned char*>(L.vals + (size_t)q * L.capacity + i0);
      const uint4 x01 = q == 0 ? g.v01 : load_stream16(vp), x23 = q == 0 ? g.v23 : load_stream16(vp + 16);
      const unsigned long long xs[4] = {((unsigned long long)x01.y << 32) | x01.x, ((unsigned long long)x01.w << 32) | x01.z,
                                        ((unsigned long long)x23.y << 32) | x23.x, ((unsigned long long)x23.w << 32) | x23.z};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t i = i0 + k;
        if (i < lo || i >= hi) continue;
        const uint32_t s = mm[k] & lowmask;
        if (p.sum_is_float[q]) unsafeAtomicAdd(reinterpret_cast<double*>(&acc[(size_t)q * W + s]), value_f64(xs[k], p.sum_conv[q]));
        else atomicAdd(&acc[(size_t)q * W + s], xs[k]);
      }
    }
  };
  if (c4 < c4e) {
    const uint32_t T = blockDim.x;
    Grp ga = fetch(c4), gb = fetch(c4 + T);
    for (; c4 < c4e; c4 += 2u * T) {
      const Grp a = ga;
      ga = fetch(c4 + 2u * T);
      consume(a, c4);
      const Grp bb = gb;
      gb = fetch(c4 + 3u * T);
      consume(bb, c4 + T);
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

void launch_partitioned(const ScanParams& p, const SlotArrays& s, PartLaunch L, uint32_t* scan_scratch,
                        hipStream_t st, hipFunction_t fcount, hipFunction_t fscatter) {
  const size_t hist_lds = (size_t)L.nparts * 4;
  void* args[] = {(void*)&p, (void*)&L};
  if (fcount) {
    (void)hipModuleLaunchKernel(fcount, (unsigned)L.blocks, 1, 1, (unsigned)L.threads, 1, 1, (unsigned)hist_lds, st,
                                args, nullptr);
  } else {
    BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_part_count<NC>), dim3(L.blocks), dim3(L.threads), hist_lds, st, p, L));
  }
  // counts has one extra zero word at the end: after the scan it holds the total
  const uint64_t n = (uint64_t)L.nparts * L.blocks + 1;
  launch_exclusive_scan_u32(L.counts, n, scan_scratch, st);
  const size_t scatter_lds = part_scatter_lds(L.nparts, L.threads, p.nsum, fscatter ? L.chunks : 1);
  if (fscatter) {
    (void)hipModuleLaunchKernel(fscatter, (unsigned)L.blocks, 1, 1, (unsigned)L.threads, 1, 1, (unsigned)scatter_lds,
                                st, args, nullptr);
  } else {
    BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_part_scatter<NC>), dim3(L.blocks), dim3(L.threads), scatter_lds, st, p, L));
  }
  const size_t agg_lds = ((size_t)1 << L.wbits) * (8 + 8 * (size_t)p.nsum) + ((size_t)L.blocks + 1) * 4;
  hipLaunchKernelGGL(k_part_aggregate, dim3(L.nparts * L.splits), dim3(1024), agg_lds, st, p, L, s);
}

}  // namespace bqg
