// partition.h -- bodies of the partitioned-aggregation count and scatter passes (config C3),
// shared by the precompiled kernels (k_partition.hip) and the query-specialised JIT kernels
// (jit_kernels.h): with the query shape folded into constants the per-row dtype / operator
// dispatch of the generic bodies disappears.
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

// count / scatter: workgroups of up to 1024 threads, each over a contiguous row range
constexpr int kPartBlock = 1024;

// A thread's 4-row chunk of the columns in `mask`, loaded unconditionally: a chunk at or past
// `end` re-reads the block's last chunk (its rows are masked off by the caller), and a column
// outside `mask` re-reads its own first chunk at `home` (one cache line for the whole wave:
// no HBM traffic to speak of).  Every path keeps the same number of loads in flight, so the
// compiler waits for exactly the chunk it consumes (vmcnt(N)) instead of draining the
// prefetch (vmcnt(0)).
template <int NC>
__device__ __forceinline__ void load_rows4_clamped(const ScanParams& p, int64_t row0, int64_t end, Chunk (&raw)[NC],
                                                   uint32_t mask, int64_t home) {
  const int64_t r = row0 < end ? row0 : ((end - 1) & ~(int64_t)(kRowsPerThread - 1));
#pragma unroll
  for (int c = 0; c < NC; ++c) load_chunk(raw[c], p.cols[c], ((mask >> c) & 1u) ? r : home);
}

// Each thread keeps kCountChunks 4-row chunks of the key columns in flight (16 rows), so a
// workgroup has ~128 KiB of key bytes outstanding while it histograms the previous group.
constexpr int kCountChunks = 4;

template <int NC>
__device__ __forceinline__ void part_count_body(const ScanParams& p, const PartLaunch& L, unsigned char* smem) {
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);
  const int tid = threadIdx.x, T = blockDim.x;
  const int step = T * kRowsPerThread;  // rows of one chunk slice of the workgroup
  const int tile = step * kCountChunks;
  for (int i = tid; i < L.nparts; i += T) hist[i] = 0;
  lds_barrier();
  const int64_t begin = (int64_t)blockIdx.x * L.rows_per_block;
  const int64_t end = (p.nrows < begin + L.rows_per_block ? p.nrows : begin + L.rows_per_block);
  if (begin >= end) {
    for (int i = tid; i < L.nparts; i += T) L.counts[(size_t)i * gridDim.x + blockIdx.x] = 0u;
    return;
  }
  const int64_t home = begin;
  Chunk raw[kCountChunks][NC];
#pragma unroll
  for (int u = 0; u < kCountChunks; ++u)
    load_rows4_clamped<NC>(p, begin + (int64_t)u * step + (int64_t)tid * kRowsPerThread, end, raw[u], L.load_mask, home);
  for (int64_t base = begin; base < end; base += tile) {
    uint32_t part[kCountChunks][4], pass[kCountChunks];
#pragma unroll
    for (int u = 0; u < kCountChunks; ++u) {
      const int64_t row0 = base + (int64_t)u * step + (int64_t)tid * kRowsPerThread;
      uint64_t v[NC][4], code[4];
      decode_all<NC, 4>(p, raw[u], v);
      pass[u] = vals_pass<NC, 4>(p, row0, v);
      const int64_t rem = end - row0;
      pass[u] &= rem >= 4 ? 0xFu : (rem > 0 ? ((1u << rem) - 1u) : 0u);
      vals_code<NC, 4>(p, v, code);
#pragma unroll
      for (int r = 0; r < 4; ++r) part[u][r] = (uint32_t)(code[r] >> L.wbits);
    }
#pragma unroll
    for (int u = 0; u < kCountChunks; ++u)
      load_rows4_clamped<NC>(p, base + tile + (int64_t)u * step + (int64_t)tid * kRowsPerThread, end, raw[u],
                             L.load_mask, home);
#pragma unroll
    for (int u = 0; u < kCountChunks; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (pass[u] & (1u << r)) atomicAdd(&hist[part[u][r]], 1u);
  }
  lds_barrier();
  for (int i = tid; i < L.nparts; i += T) L.counts[(size_t)i * gridDim.x + blockIdx.x] = hist[i];
}

// Single-buffered tile staging (64 KiB for one summed column at 1024 threads and CH = 1: two
// scatter workgroups fit on a CU, which measured faster than double buffering at one per CU);
// the scan's wave totals alternate between two buffers so the scan needs one barrier.  CH
// 4-row chunks per thread make a tile of CH * 4 * T rows (each chunk slice coalesced): longer
// runs per partition and fewer barriers per row, at CH times the staging LDS.
template <int NC, int CH = 1>
__device__ __forceinline__ void part_scatter_body(const ScanParams& p, const PartLaunch& L, unsigned char* smem) {
  const int T = blockDim.x, tid = threadIdx.x;
  const int P = L.nparts;
  const int slice = T * kRowsPerThread;
  const int tile = slice * CH;
  const int nsum = p.nsum;
  unsigned long long* sval = reinterpret_cast<unsigned long long*>(smem);             // [nsum][tile]
  uint32_t* smeta = reinterpret_cast<uint32_t*>(sval + (size_t)nsum * tile);          // [tile]
  uint32_t* sdst = smeta + tile;                                                       // [tile] destinations
  uint32_t* hist2 = sdst + tile;                                                       // [2][P] tile counts
  uint32_t* toff = hist2 + 2 * P;                                                      // [P] tile offsets
  uint32_t* cur = toff + P;                                                            // [P] region cursors
  uint32_t* wsum2 = cur + P;                                                           // [2][16] scan totals
  for (int i = tid; i < P; i += T) {
    hist2[i] = 0;
    hist2[P + i] = 0;
    cur[i] = L.counts[(size_t)i * gridDim.x + blockIdx.x];
  }
  lds_barrier();
  const int64_t begin = (int64_t)blockIdx.x * L.rows_per_block;
  const int64_t end = (p.nrows < begin + L.rows_per_block ? p.nrows : begin + L.rows_per_block);
  const uint64_t lowmask = (1ull << L.wbits) - 1ull;
  const int per = (P + T - 1) / T;  // partitions per thread in the tile scan
  const int q0 = tid * per;
  const int q1 = min(P, q0 + per);
  const uint32_t all = (1u << NC) - 1u;
  constexpr int NS = NC < kMaxSums ? NC : kMaxSums;
  Chunk raw[CH][NC];
  if (begin < end) {
#pragma unroll
    for (int u = 0; u < CH; ++u)
      load_rows4_clamped<NC>(p, begin + (int64_t)u * slice + (int64_t)tid * kRowsPerThread, end, raw[u], all, begin);
  }
  int parity = 0;
  for (int64_t base = begin; base < end; base += tile, parity ^= 1) {
    // the tile histogram alternates between two buffers: the one this tile zeroes at its end
    // is next counted into two tiles later, past this tile's barriers, so the loop needs no
    // trailing barrier (tile t+1's first phase touches neither the staging area nor `cur`)
    uint32_t* hist = hist2 + parity * P;
    uint32_t pass[CH], part[CH][4], rank[CH][4], low[CH][4];
    uint64_t sv[CH][NS][4];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int64_t row0 = base + (int64_t)u * slice + (int64_t)tid * kRowsPerThread;
      uint64_t v[NC][4], code[4];
      decode_all<NC, 4>(p, raw[u], v);
      load_rows4_clamped<NC>(p, row0 + tile, end, raw[u], all, begin);
      pass[u] = vals_pass<NC, 4>(p, row0, v);
      const int64_t rem = end - row0;
      pass[u] &= rem >= 4 ? 0xFu : (rem > 0 ? ((1u << rem) - 1u) : 0u);
      vals_code<NC, 4>(p, v, code);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        part[u][r] = (uint32_t)(code[r] >> L.wbits);
        low[u][r] = (uint32_t)(code[r] & lowmask);
#pragma unroll
        for (int s = 0; s < NS; ++s) sv[u][s][r] = v[s][r];
      }
    }
#pragma unroll
    for (int u = 0; u < CH; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) rank[u][r] = (pass[u] & (1u << r)) ? atomicAdd(&hist[part[u][r]], 1u) : 0u;
    lds_barrier();
    // tile offsets: exclusive scan of the tile histogram
    uint32_t local = 0;
    for (int i = q0; i < q1; ++i) local += hist[i];
    uint32_t n_tile;
    uint32_t run = block_excl_scan_1b(local, wsum2 + parity * 16, &n_tile);
    for (int i = q0; i < q1; ++i) {
      toff[i] = run;
      run += hist[i];
    }
    lds_barrier();
    // stage the tile sorted by partition, with each entry's destination (region cursor + rank)
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int64_t row0 = base + (int64_t)u * slice + (int64_t)tid * kRowsPerThread;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (!(pass[u] & (1u << r))) continue;
        const uint32_t pos = toff[part[u][r]] + rank[u][r];
        smeta[pos] = ((uint32_t)(row0 + r - begin) << L.wbits) | low[u][r];
        sdst[pos] = cur[part[u][r]] + rank[u][r];
#pragma unroll
        for (int s = 0; s < NS; ++s)
          if (s < nsum) sval[(size_t)s * tile + pos] = sv[u][s][r];
      }
    }
    lds_barrier();
    // copy out: consecutive lanes -> consecutive entries of one region (whole lines)
#pragma unroll
    for (int k = 0; k < kRowsPerThread * CH; ++k) {
      const uint32_t i = (uint32_t)(tid + k * T);
      if (i < n_tile) {
        const uint32_t dst = sdst[i];
        L.meta[dst] = smeta[i];
#pragma unroll
        for (int s = 0; s < NS; ++s)
          if (s < nsum) L.vals[(size_t)s * L.capacity + dst] = sval[(size_t)s * tile + i];
      }
    }
    for (int i = q0; i < q1; ++i) {
      cur[i] += hist[i];
      hist[i] = 0;
    }
  }
}

}  // namespace bqg
