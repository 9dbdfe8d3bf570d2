// k_partition.hip -- partitioned aggregation for large dense slot spaces (config C3: ~1 M
// groups), and a multi-workgroup exclusive scan.
//
// Per-row device atomics on a 1 M-slot table are random 8-byte memory-side operations
// (MI355X_MICROARCH.md: ~17x below the streaming rate).  Instead:
//   count:    each workgroup owns a contiguous row range and histograms the passing rows by
//             partition p = slot >> wbits (LDS atomics) -> counts[p][block];
//   scan:     exclusive scan of counts in [p][block] order -> every (partition, workgroup)
//             region's offset; partitions are contiguous in the entry buffers;
//   scatter:  the workgroup re-reads its rows and writes (row << 32 | slot_low, values) into
//             its regions (LDS cursors, no global atomics);
//   aggregate: one or more workgroups per partition aggregate its entries in an LDS table of
//             2^wbits slots and flush the occupied slots (contiguous, coalesced atomics).
// Traffic per row: keys + filters (count) + all columns (scatter) + the entry written and
// read back once.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device.h"

namespace bqg {

// count / scatter run as one 1024-thread workgroup per CU over a contiguous row range: the
// (workgroup, partition) regions being filled at any time total ~256 x nparts cache lines,
// small enough to stay in the XCDs' L2 until each line is complete (write combining).
constexpr int kPartBlock = 1024;
constexpr int kPartTile = kPartBlock * kRowsPerThread;

template <int NC>
__device__ __forceinline__ uint32_t part_rows(const ScanParams& p, int64_t row0, int64_t end, const Chunk (&raw)[NC],
                                              uint64_t (&v)[NC][4], uint64_t (&code)[4]) {
  decode_all<NC, 4>(p, raw, v);
  uint32_t pass = vals_pass<NC, 4>(p, row0, v);
  if (end - row0 < 4) pass &= (end - row0 > 0) ? ((1u << (end - row0)) - 1u) : 0u;
  vals_code<NC, 4>(p, v, code);
  return pass;
}

template <int NC>
__global__ __launch_bounds__(kPartBlock) void k_part_count(ScanParams p, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);
  const int tid = threadIdx.x;
  for (int i = tid; i < L.nparts; i += kPartBlock) hist[i] = 0;
  __syncthreads();
  const int64_t begin = (int64_t)blockIdx.x * L.rows_per_block;
  const int64_t end = std::min<int64_t>(p.nrows, begin + L.rows_per_block);
  Chunk raw[NC];
  if (begin < end) load_rows4<NC>(p, begin + (int64_t)tid * kRowsPerThread, raw);
  for (int64_t base = begin; base < end; base += kPartTile) {
    const int64_t row0 = base + (int64_t)tid * kRowsPerThread;
    uint64_t v[NC][4], code[4];
    decode_all<NC, 4>(p, raw, v);
    if (base + kPartTile < end) load_rows4<NC>(p, row0 + kPartTile, raw);
    uint32_t pass = vals_pass<NC, 4>(p, row0, v);
    if (end - row0 < 4) pass &= (end - row0 > 0) ? ((1u << (end - row0)) - 1u) : 0u;
    vals_code<NC, 4>(p, v, code);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (pass & (1u << r)) atomicAdd(&hist[(uint32_t)(code[r] >> L.wbits)], 1u);
  }
  __syncthreads();
  for (int i = tid; i < L.nparts; i += kPartBlock) L.counts[(size_t)i * gridDim.x + blockIdx.x] = hist[i];
}

// entries are array-of-structs: {u32 slot_low, u32 row, u64 value[nsum]} (16 bytes for one
// summed column: a single 16-byte store per passing row)
template <int NC>
__global__ __launch_bounds__(kPartBlock) void k_part_scatter(ScanParams p, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* cursor = reinterpret_cast<uint32_t*>(smem);
  const int tid = threadIdx.x;
  for (int i = tid; i < L.nparts; i += kPartBlock) cursor[i] = L.counts[(size_t)i * gridDim.x + blockIdx.x];
  __syncthreads();
  const int64_t begin = (int64_t)blockIdx.x * L.rows_per_block;
  const int64_t end = std::min<int64_t>(p.nrows, begin + L.rows_per_block);
  const uint64_t lowmask = (1ull << L.wbits) - 1ull;
  const int nsum = p.nsum;
  const int words = 1 + nsum;  // 8-byte words per entry
  Chunk raw[NC];
  if (begin < end) load_rows4<NC>(p, begin + (int64_t)tid * kRowsPerThread, raw);
  for (int64_t base = begin; base < end; base += kPartTile) {
    const int64_t row0 = base + (int64_t)tid * kRowsPerThread;
    uint64_t v[NC][4], code[4];
    decode_all<NC, 4>(p, raw, v);
    if (base + kPartTile < end) load_rows4<NC>(p, row0 + kPartTile, raw);
    uint32_t pass = vals_pass<NC, 4>(p, row0, v);
    if (end - row0 < 4) pass &= (end - row0 > 0) ? ((1u << (end - row0)) - 1u) : 0u;
    vals_code<NC, 4>(p, v, code);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (pass & (1u << r)) {
        const uint32_t pos = atomicAdd(&cursor[(uint32_t)(code[r] >> L.wbits)], 1u);
        const unsigned long long meta = ((unsigned long long)(uint32_t)(row0 + r) << 32) | (code[r] & lowmask);
        unsigned long long* e = L.entries + (size_t)pos * words;
        if (nsum == 1) {
          *reinterpret_cast<ulonglong2*>(e) = make_ulonglong2(meta, v[0][r]);
        } else {
          e[0] = meta;
#pragma unroll
          for (int s = 0; s < (NC < kMaxSums ? NC : kMaxSums); ++s)
            if (s < nsum) e[1 + s] = v[s][r];
        }
      }
    }
  }
}

__global__ __launch_bounds__(1024) void k_part_aggregate(ScanParams p, PartLaunch L, SlotArrays sa) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int W = 1 << L.wbits;
  const int nsum = p.nsum;
  const int words = 1 + nsum;
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem);  // [nsum][W]
  uint32_t* cnt = reinterpret_cast<uint32_t*>(acc + (size_t)nsum * W);    // [W]
  uint32_t* fst = cnt + W;                                                 // [W]
  const int tid = threadIdx.x;
  for (int i = tid; i < W; i += blockDim.x) {
    cnt[i] = 0;
    fst[i] = kNoRow;
  }
  for (int i = tid; i < nsum * W; i += blockDim.x) acc[i] = 0;
  __syncthreads();
  const int part = blockIdx.x / L.splits, split = blockIdx.x % L.splits;
  const uint32_t pbeg = L.part_start[part];
  const uint32_t pend = L.part_start[part + 1];
  const uint64_t len = pend - pbeg;
  const uint32_t beg = pbeg + (uint32_t)(len * split / L.splits);
  const uint32_t fin = pbeg + (uint32_t)(len * (split + 1) / L.splits);
  for (uint32_t i = beg + tid; i < fin; i += blockDim.x) {
    const unsigned long long* e = L.entries + (size_t)i * words;
    unsigned long long m, x0;
    if (nsum == 1) {
      const ulonglong2 t = *reinterpret_cast<const ulonglong2*>(e);
      m = t.x;
      x0 = t.y;
    } else {
      m = e[0];
      x0 = nsum ? e[1] : 0ull;
    }
    const uint32_t s = (uint32_t)(m & 0xFFFFFFFFull);
    const uint32_t row = (uint32_t)(m >> 32);
    atomicAdd(&cnt[s], 1u);
    if (fst[s] > row) atomicMin(&fst[s], row);
    for (int q = 0; q < nsum; ++q) {
      const unsigned long long x = q == 0 ? x0 : e[1 + q];
      if (p.sum_is_float[q]) unsafeAtomicAdd(reinterpret_cast<double*>(&acc[(size_t)q * W + s]), value_f64(x, p.sum_conv[q]));
      else atomicAdd(&acc[(size_t)q * W + s], x);
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
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ uint32_t block_excl_scan_1024(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan_u32(v, lane);
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  if (wave == 0) {
    const uint32_t w = lane < (int)(blockDim.x >> 6) ? wsum[lane] : 0u;
    const uint32_t wi = wave_incl_scan_u32(w, lane);
    if (lane < 16) wsum[lane] = wi - w;
    if (lane == 63 && total) *total = wi;
  }
  __syncthreads();
  const uint32_t r = wsum[wave] + incl - v;
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(1024) void k_scan_seg(uint32_t* v, uint64_t n, uint32_t* seg_totals) {
  const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  const uint32_t x = i < n ? v[i] : 0u;
  __shared__ uint32_t tot;
  const uint32_t e = block_excl_scan_1024(x, &tot);
  if (i < n) v[i] = e;
  __syncthreads();
  if (threadIdx.x == 0) seg_totals[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_scan_add(uint32_t* v, uint64_t n, const uint32_t* seg_offsets) {
  const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  if (i < n) v[i] += seg_offsets[blockIdx.x];
}

// part_start[p] = offsets[p * B] (first region of partition p); part_start[P] = total
__global__ void k_part_starts(const uint32_t* offsets, int nparts, int blocks, uint32_t* starts) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i <= nparts; i += gridDim.x * blockDim.x)
    starts[i] = offsets[(size_t)i * blocks];  // i == nparts: the trailing total word
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
                        hipStream_t st) {
  const size_t hist_lds = (size_t)L.nparts * 4;
  BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_part_count<NC>), dim3(L.blocks), dim3(kPartBlock), hist_lds, st, p, L));
  // counts has one extra zero word at the end: after the scan it holds the total
  const uint64_t n = (uint64_t)L.nparts * L.blocks + 1;
  launch_exclusive_scan_u32(L.counts, n, scan_scratch, st);
  hipLaunchKernelGGL(k_part_starts, dim3((L.nparts + 256) / 256), dim3(256), 0, st, L.counts, L.nparts, L.blocks,
                     L.part_start);
  BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_part_scatter<NC>), dim3(L.blocks), dim3(kPartBlock), hist_lds, st, p, L));
  const size_t agg_lds = ((size_t)1 << L.wbits) * (8 + 8 * (size_t)p.nsum);
  hipLaunchKernelGGL(k_part_aggregate, dim3(L.nparts * L.splits), dim3(1024), agg_lds, st, p, L, s);
}

}  // namespace bqg
