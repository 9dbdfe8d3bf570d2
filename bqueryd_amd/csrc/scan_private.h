// scan_private.h -- body of the private-LDS fused scan (config C2's hot loop), shared by the
// precompiled kernel (k_scan_private.hip) and the query-specialised JIT kernel (jit.hip).
#pragma once

#include "device.h"

namespace bqg {

#ifndef BQ_PRIV_AHEAD
#define BQ_PRIV_AHEAD 1
#endif
constexpr int kPrivAhead = BQ_PRIV_AHEAD;  // tiles loaded ahead of the one being aggregated

// Every lane owns a private accumulator row per slot in LDS, laid out [slot][lane]: nothing
// contends, so the per-row updates are LDS atomics without return (no read-modify-write
// chains).  Rows of a lane are processed in increasing order, so the minimum of its rows in a
// slot is that slot's first row for the lane.  A workgroup streams tiles of 1024 rows (4 per
// lane; one load per column: 16 bytes of a 4-byte column, exactly the lane's 4 or 8 bytes of
// a 1- or 2-byte column in specialised kernels) and prefetches the next tile while it
// aggregates the current one.
template <int NC>
__device__ __forceinline__ void scan_private_body(const ScanParams& p, const PrivateLaunch& L, unsigned char* smem) {
  const int S = (int)p.nslots;
  const int tid = threadIdx.x;
  const int nsum = p.nsum;
  // [S][256] {count, first row} word pairs (one address per row for both), then the sums
  // [nsum][S][256]
  uint32_t* cf = reinterpret_cast<uint32_t*>(smem);
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem + (size_t)S * kBlock * 8);
  for (int s = 0; s < S; ++s)
    reinterpret_cast<unsigned long long*>(cf)[s * kBlock + tid] = (unsigned long long)kNoRow << 32;
  for (int i = 0; i < nsum * S; ++i) acc[i * kBlock + tid] = 0;

  const int64_t ntiles = (p.nrows + kTileRows - 1) / kTileRows;
  const int64_t grid = gridDim.x;
  const int64_t lane_row = (int64_t)tid * kRowsPerThread;
  // kPrivAhead tiles in flight per workgroup while one is aggregated (a ring of registers).
  // Loads are unconditional: past the last tile a lane re-reads the tile it is consuming (an
  // L2 hit), so every path has the same loads in flight and the compiler waits with
  // vmcnt(N) for exactly the oldest tile.
  Chunk ring[kPrivAhead][NC];
  if (blockIdx.x < ntiles) {
#pragma unroll
    for (int a = 0; a < kPrivAhead; ++a) {
      const int64_t t = blockIdx.x + a * grid;
      load_rows4<NC>(p, (t < ntiles ? t : (int64_t)blockIdx.x) * kTileRows + lane_row, ring[a]);
    }
  }
  for (int64_t tbase = blockIdx.x; tbase < ntiles; tbase += kPrivAhead * grid) {
#pragma unroll
  for (int a = 0; a < kPrivAhead; ++a) {
    const int64_t tile = tbase + a * grid;
    if (tile >= ntiles) break;
    const int64_t row0 = tile * kTileRows + lane_row;
    uint64_t v[NC][4];
    decode_all<NC, 4>(p, ring[a], v);
    const int64_t next = tile + kPrivAhead * grid;
    load_rows4<NC>(p, (next < ntiles ? next : tile) * kTileRows + lane_row, ring[a]);
    // the row bound only on the last tile (wave-uniform branch): full tiles skip its 64-bit
    // compares
    uint32_t pass = 0xFu;
    if (tile == ntiles - 1) {
      const int64_t rem = p.nrows - row0;
      pass = rem >= 4 ? 0xFu : (rem > 0 ? ((1u << rem) - 1u) : 0u);
    }
    pass &= vals_pass<NC, 4, false>(p, row0, v);
    uint64_t code[4];
    vals_code<NC, 4>(p, v, code);
    // count, first row and integer sums as LDS atomics whose results are unused (ds_add /
    // ds_min without return): the slot rows are lane-private, so nothing contends, and no row
    // waits for a read of the row before it (a read-modify-write chain per row stalled the
    // wave on two LDS round trips).  Rows are visited in increasing order, so min = first.
    // Float sums keep the ordered read-modify-write (row-order float64 additions per lane).
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (pass & (1u << r)) {
        const int idx = (int)code[r] * kBlock + tid;
        atomicAdd(&cf[2 * idx], 1u);
        atomicMin(&cf[2 * idx + 1], (uint32_t)(row0 + r));
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
              atomicAdd(a, (unsigned long long)v[s][r]);
            }
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
      c += cf[2 * (s * kBlock + lane + 64 * j)];
      f = min(f, cf[2 * (s * kBlock + lane + 64 * j) + 1]);
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

}  // namespace bqg
