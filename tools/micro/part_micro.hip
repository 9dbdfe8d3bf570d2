// part_micro.hip -- C3-shaped partitioned aggregation (100 M rows, pickup_location x vendor_id,
// ~1 M dense slots, one f64 sum + count) outside the library: the library's count / scan /
// scatter / aggregate kernels (k_partition.hip, specialised like the JIT build) against
// experimental variants, each timed with events and checked slot by slot against the
// library pipeline.  Phase counters (clock64 on lane 0 of each workgroup) split the scatter.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I bqueryd_amd/csrc
//        -I include tools/micro/part_micro.hip -o build/part_micro
#define BQ_NC 3
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "partition.h"

namespace bqg {
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

}  // namespace bqg

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

using namespace bqg;

__device__ __forceinline__ void specialize(ScanParams& p) {
  p.ncols = 3;
  p.cols[0].dtype = BQG_F64; p.cols[0].lg = 3;
  p.cols[1].dtype = BQG_I32; p.cols[1].lg = 2;
  p.cols[2].dtype = BQG_I32; p.cols[2].lg = 2;
  p.nterms = 0;
  p.nkeys = 2;
  p.keys[0].col = 1; p.keys[0].is_float = 0;
  p.keys[1].col = 2; p.keys[1].is_float = 0; p.keys[1].stride = 1ull;
  p.nsum = 1;
  p.sum_is_float[0] = 1; p.sum_conv[0] = 0; p.sum_centered[0] = 0;
  p.mask_col = -1;
  p.hash = 0;
}

__device__ unsigned long long g_phase[8];
__device__ unsigned int g_err[4];  // bounds-check hits: [0] scatter part/pos, [1] header, [2] aggregate entry index

__global__ void k_gen(int64_t n, double* fare, int32_t* pl, int32_t* ven) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = mix64((uint64_t)i * 0x9E3779B97F4A7C15ull + 12345);
    pl[i] = (int32_t)((h >> 8) % 500000u);
    ven[i] = 1 + (int32_t)((h >> 40) & 1u);
    fare[i] = 2.5 + (double)((h >> 44) % 30000u) / 64.0;
  }
}

__global__ __launch_bounds__(1024) void k_count_lib(ScanParams pin, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  ScanParams p = pin;
  specialize(p);
  part_count_body<3>(p, L, smem);
}

__global__ __launch_bounds__(1024) void k_scatter_lib(ScanParams pin, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  ScanParams p = pin;
  specialize(p);
  part_scatter_body<3>(p, L, smem);
}

// the library scatter body with phase counters on thread 0
__global__ __launch_bounds__(1024) void k_scatter_prof(ScanParams pin, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  ScanParams p = pin;
  specialize(p);
  constexpr int NC = 3, CH = 1;
  const int T = blockDim.x, tid = threadIdx.x;
  const int P = L.nparts;
  const int slice = T * kRowsPerThread;
  const int tile = slice * CH;
  const int nsum = p.nsum;
  unsigned long long* sval = reinterpret_cast<unsigned long long*>(smem);
  uint32_t* smeta = reinterpret_cast<uint32_t*>(sval + (size_t)nsum * tile);
  uint32_t* sdst = smeta + tile;
  uint32_t* hist2 = sdst + tile;
  uint32_t* toff = hist2 + 2 * P;
  uint32_t* cur = toff + P;
  uint32_t* wsum2 = cur + P;
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long t0 = clock64();
  for (int i = tid; i < P; i += T) {
    hist2[i] = 0;
    hist2[P + i] = 0;
    cur[i] = L.counts[(size_t)i * gridDim.x + blockIdx.x];
  }
  lds_barrier();
  const int64_t begin = (int64_t)blockIdx.x * L.rows_per_block;
  const int64_t end = (p.nrows < begin + L.rows_per_block ? p.nrows : begin + L.rows_per_block);
  const uint64_t lowmask = (1ull << L.wbits) - 1ull;
  const int per = (P + T - 1) / T;
  const int q0 = tid * per;
  const int q1 = min(P, q0 + per);
  const uint32_t all = (1u << NC) - 1u;
  constexpr int NS = 1;
  Chunk raw[CH][NC];
  if (begin < end) {
    for (int u = 0; u < CH; ++u)
      load_rows4_clamped<NC>(p, begin + (int64_t)u * slice + (int64_t)tid * kRowsPerThread, end, raw[u], all, begin);
  }
  int parity = 0;
  unsigned long long t1 = clock64();
  ph[0] += t1 - t0;
  for (int64_t base = begin; base < end; base += tile, parity ^= 1) {
    uint32_t* hist = hist2 + parity * P;
    uint32_t pass[CH], part[CH][4], rank[CH][4], low[CH][4];
    uint64_t sv[CH][NS][4];
    t0 = clock64();
    for (int u = 0; u < CH; ++u) {
      const int64_t row0 = base + (int64_t)u * slice + (int64_t)tid * kRowsPerThread;
      uint64_t v[NC][4], code[4];
      decode_all<NC, 4>(p, raw[u], v);
      load_rows4_clamped<NC>(p, row0 + tile, end, raw[u], all, begin);
      pass[u] = vals_pass<NC, 4>(p, row0, v);
      const int64_t rem = end - row0;
      pass[u] &= rem >= 4 ? 0xFu : (rem > 0 ? ((1u << rem) - 1u) : 0u);
      vals_code<NC, 4>(p, v, code);
      for (int r = 0; r < 4; ++r) {
        part[u][r] = (uint32_t)(code[r] >> L.wbits);
        low[u][r] = (uint32_t)(code[r] & lowmask);
        sv[u][0][r] = v[0][r];
      }
    }
    t1 = clock64();
    ph[1] += t1 - t0;
    for (int u = 0; u < CH; ++u)
      for (int r = 0; r < 4; ++r) rank[u][r] = (pass[u] & (1u << r)) ? atomicAdd(&hist[part[u][r]], 1u) : 0u;
    lds_barrier();
    t0 = clock64();
    ph[2] += t0 - t1;
    uint32_t local = 0;
    for (int i = q0; i < q1; ++i) local += hist[i];
    uint32_t n_tile;
    uint32_t run = block_excl_scan_1b(local, wsum2 + parity * 16, &n_tile);
    for (int i = q0; i < q1; ++i) {
      toff[i] = run;
      run += hist[i];
    }
    lds_barrier();
    t1 = clock64();
    ph[3] += t1 - t0;
    for (int u = 0; u < CH; ++u) {
      const int64_t row0 = base + (int64_t)u * slice + (int64_t)tid * kRowsPerThread;
      for (int r = 0; r < 4; ++r) {
        if (!(pass[u] & (1u << r))) continue;
        const uint32_t pos = toff[part[u][r]] + rank[u][r];
        smeta[pos] = ((uint32_t)(row0 + r - begin) << L.wbits) | low[u][r];
        sdst[pos] = cur[part[u][r]] + rank[u][r];
        sval[pos] = sv[u][0][r];
      }
    }
    lds_barrier();
    t0 = clock64();
    ph[4] += t0 - t1;
    for (int k = 0; k < kRowsPerThread * CH; ++k) {
      const uint32_t i = (uint32_t)(tid + k * T);
      if (i < n_tile) {
        const uint32_t dst = sdst[i];
        L.meta[dst] = smeta[i];
        L.vals[dst] = sval[i];
      }
    }
    for (int i = q0; i < q1; ++i) {
      cur[i] += hist[i];
      hist[i] = 0;
    }
    t1 = clock64();
    ph[5] += t1 - t0;
  }
  if (tid == 0)
    for (int i = 0; i < 6; ++i) atomicAdd(&g_phase[i], ph[i]);
}


// Variant v2: PD tiles of loads in flight (register ring, loop unrolled by PD so every ring
// index is static) and a static store count per tile (lanes past the tile's entry count
// store to a junk entry at index `capacity`), so the back-edge waits with vmcnt(N) for the
// oldest tile's loads instead of draining every load and store.
template <int PD>
__global__ __launch_bounds__(1024) void k_scatter_v2(ScanParams pin, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  ScanParams p = pin;
  specialize(p);
  constexpr int NC = 3;
  const int T = blockDim.x, tid = threadIdx.x;
  const int P = L.nparts;
  const int tile = T * kRowsPerThread;
  unsigned long long* sval = reinterpret_cast<unsigned long long*>(smem);
  uint32_t* smeta = reinterpret_cast<uint32_t*>(sval + tile);
  uint32_t* sdst = smeta + tile;
  uint32_t* hist2 = sdst + tile;
  uint32_t* toff = hist2 + 2 * P;
  uint32_t* cur = toff + P;
  uint32_t* wsum2 = cur + P;
  for (int i = tid; i < P; i += T) {
    hist2[i] = 0;
    hist2[P + i] = 0;
    cur[i] = L.counts[(size_t)i * gridDim.x + blockIdx.x];
  }
  lds_barrier();
  const int64_t begin = (int64_t)blockIdx.x * L.rows_per_block;
  const int64_t end = (p.nrows < begin + L.rows_per_block ? p.nrows : begin + L.rows_per_block);
  if (begin >= end) return;
  const uint64_t lowmask = (1ull << L.wbits) - 1ull;
  const int per = (P + T - 1) / T;
  const int q0 = tid * per;
  const int q1 = min(P, q0 + per);
  const uint32_t all = (1u << NC) - 1u;
  const uint32_t junk = (uint32_t)L.capacity;
  Chunk raw[PD][NC];
#pragma unroll
  for (int d = 0; d < PD; ++d)
    load_rows4_clamped<NC>(p, begin + (int64_t)d * tile + (int64_t)tid * kRowsPerThread, end, raw[d], all, begin);
  for (int64_t base0 = begin; base0 < end; base0 += (int64_t)PD * tile) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const int64_t base = base0 + (int64_t)d * tile;
      uint32_t* hist = hist2 + (d & 1) * P;
      uint32_t part[4], rank[4], low[4];
      uint64_t sv[4];
      const int64_t row0 = base + (int64_t)tid * kRowsPerThread;
      uint32_t pass;
      {
        uint64_t v[NC][4], code[4];
        decode_all<NC, 4>(p, raw[d], v);
        load_rows4_clamped<NC>(p, row0 + (int64_t)PD * tile, end, raw[d], all, begin);
        pass = vals_pass<NC, 4>(p, row0, v);
        const int64_t rem = end - row0;
        pass &= rem >= 4 ? 0xFu : (rem > 0 ? ((1u << rem) - 1u) : 0u);
        vals_code<NC, 4>(p, v, code);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          part[r] = (uint32_t)(code[r] >> L.wbits);
          low[r] = (uint32_t)(code[r] & lowmask);
          sv[r] = v[0][r];
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) rank[r] = (pass & (1u << r)) ? atomicAdd(&hist[part[r]], 1u) : 0u;
      lds_barrier();
      uint32_t local = 0;
      for (int i = q0; i < q1; ++i) local += hist[i];
      uint32_t n_tile;
      uint32_t run = block_excl_scan_1b(local, wsum2 + (d & 1) * 16, &n_tile);
      for (int i = q0; i < q1; ++i) {
        toff[i] = run;
        run += hist[i];
      }
      lds_barrier();
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (!(pass & (1u << r))) continue;
        const uint32_t pos = toff[part[r]] + rank[r];
        smeta[pos] = ((uint32_t)(row0 + r - begin) << L.wbits) | low[r];
        sdst[pos] = cur[part[r]] + rank[r];
        sval[pos] = sv[r];
      }
      lds_barrier();
#pragma unroll
      for (int k = 0; k < kRowsPerThread; ++k) {
        const uint32_t i = (uint32_t)(tid + k * T);
        const uint32_t dst = i < n_tile ? sdst[i] : junk;
        L.meta[dst] = smeta[i];
        L.vals[dst] = sval[i];
      }
      for (int i = q0; i < q1; ++i) {
        cur[i] += hist[i];
        hist[i] = 0;
      }
    }
  }
}


// Variant v3: wave-private tile histograms (hw[wave][partition]): a tile's 4096 LDS atomics
// spread over 16 x P addresses instead of P, so same-address read-modify-write chains are
// ~16x shorter; the per-(partition, wave) offsets come from one pass over the histograms.
template <int LINEAR>
__global__ __launch_bounds__(1024) void k_scatter_v3(ScanParams pin, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  ScanParams p = pin;
  specialize(p);
  constexpr int NC = 3;
  const int T = blockDim.x, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, NW = T >> 6;
  const int P = L.nparts;
  const int tile = T * kRowsPerThread;
  unsigned long long* sval = reinterpret_cast<unsigned long long*>(smem);
  uint32_t* smeta = reinterpret_cast<uint32_t*>(sval + tile);
  uint32_t* sdst = smeta + tile;
  uint32_t* hw2 = sdst + tile;        // [2][NW][P]
  uint32_t* tdst = hw2 + 2 * NW * P;  // [NW][P] destination of each (wave, partition) run's first entry
  uint32_t* cur = tdst + NW * P;      // [P]
  uint32_t* wsum2 = cur + P;          // [2][16]
  for (int i = tid; i < 2 * NW * P; i += T) hw2[i] = 0;
  for (int i = tid; i < P; i += T) cur[i] = L.counts[(size_t)i * gridDim.x + blockIdx.x];
  lds_barrier();
  const int64_t begin = (int64_t)blockIdx.x * L.rows_per_block;
  const int64_t end = (p.nrows < begin + L.rows_per_block ? p.nrows : begin + L.rows_per_block);
  if (begin >= end) return;
  const uint64_t lowmask = (1ull << L.wbits) - 1ull;
  const uint32_t all = (1u << NC) - 1u;
  const uint32_t junk = (uint32_t)L.capacity;
  Chunk raw[NC];
  load_rows4_clamped<NC>(p, begin + (int64_t)tid * kRowsPerThread, end, raw, all, begin);
  int parity = 0;
  for (int64_t base = begin; base < end; base += tile, parity ^= 1) {
    uint32_t* hw = hw2 + parity * NW * P;
    uint32_t part[4], rank[4], low[4];
    uint64_t sv[4];
    const int64_t row0 = base + (int64_t)tid * kRowsPerThread;
    uint32_t pass;
    {
      uint64_t v[NC][4], code[4];
      decode_all<NC, 4>(p, raw, v);
      load_rows4_clamped<NC>(p, row0 + tile, end, raw, all, begin);
      pass = vals_pass<NC, 4>(p, row0, v);
      const int64_t rem = end - row0;
      pass &= rem >= 4 ? 0xFu : (rem > 0 ? ((1u << rem) - 1u) : 0u);
      vals_code<NC, 4>(p, v, code);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        part[r] = (uint32_t)(code[r] >> L.wbits);
        low[r] = (uint32_t)(code[r] & lowmask);
        sv[r] = v[0][r];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) rank[r] = (pass & (1u << r)) ? atomicAdd(&hw[wave * P + part[r]], 1u) : 0u;
    lds_barrier();
    // partition q's runs: waves in order; thread q sums its column, the block scans the totals
    uint32_t colsum = 0;
    if (tid < P)
      for (int w = 0; w < NW; ++w) colsum += hw[w * P + tid];
    uint32_t n_tile;
    const uint32_t tb = block_excl_scan_1b(colsum, wsum2 + parity * 16, &n_tile);
    if (tid < P) {
      uint32_t o = tb, d = cur[tid];
      for (int w = 0; w < NW; ++w) {
        const uint32_t c = hw[w * P + tid];
        hw[w * P + tid] = o;       // tile position of (w, q)'s run
        tdst[w * P + tid] = d;     // region destination of its first entry
        o += c;
        d += c;
      }
      cur[tid] = d;
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (!(pass & (1u << r))) continue;
      const uint32_t pos = hw[wave * P + part[r]] + rank[r];
      smeta[pos] = ((uint32_t)(row0 + r - begin) << L.wbits) | low[r];
      sdst[pos] = tdst[wave * P + part[r]] + rank[r];
      sval[pos] = sv[r];
    }
    lds_barrier();
#pragma unroll
    for (int k = 0; k < kRowsPerThread; ++k) {
      const uint32_t i = (uint32_t)(tid + k * T);
      const uint32_t dst = LINEAR ? (uint32_t)(base + i) : (i < n_tile ? sdst[i] : junk);
      L.meta[dst] = smeta[i];
      L.vals[dst] = sval[i];
    }
    // this tile's histogram buffer is counted into again two tiles later, past the next
    // tile's barriers
    for (int i = tid; i < NW * P; i += T) hw[i] = 0;
  }
}


// Variant v5 ("tile layout"): no count pass.  Each 4096-row tile is counting-sorted by
// partition in LDS and written back linearly at the tile's own entry range [tile * 4096,
// +4096) (whole lines, static store count), with a header of P + 1 16-bit offsets: entries of
// partition q in tile t are [hdr[t][q], hdr[t][q + 1]).  Meta = row-in-tile << wbits | low.
__global__ __launch_bounds__(1024) void k_scatter_v5(ScanParams pin, PartLaunch L, uint16_t* hdr) {
  extern __shared__ __align__(16) unsigned char smem[];
  ScanParams p = pin;
  specialize(p);
  constexpr int NC = 3;
  const int T = blockDim.x, tid = threadIdx.x;
  const int wave = tid >> 6, NW = T >> 6;
  const int P = L.nparts;
  const int tile = T * kRowsPerThread;
  unsigned long long* sval = reinterpret_cast<unsigned long long*>(smem);
  uint32_t* smeta = reinterpret_cast<uint32_t*>(sval + tile);
  uint32_t* hw2 = smeta + tile;       // [2][NW][P]
  uint32_t* wsum2 = hw2 + 2 * NW * P; // [2][16]
  for (int i = tid; i < 2 * NW * P; i += T) hw2[i] = 0;
  lds_barrier();
  const int64_t begin = (int64_t)blockIdx.x * L.rows_per_block;
  const int64_t end = (p.nrows < begin + L.rows_per_block ? p.nrows : begin + L.rows_per_block);
  if (begin >= end) return;
  const uint64_t lowmask = (1ull << L.wbits) - 1ull;
  const uint32_t all = (1u << NC) - 1u;
  Chunk raw[NC];
  load_rows4_clamped<NC>(p, begin + (int64_t)tid * kRowsPerThread, end, raw, all, begin);
  int parity = 0;
  for (int64_t base = begin; base < end; base += tile, parity ^= 1) {
    uint32_t* hw = hw2 + parity * NW * P;
    uint32_t part[4], rank[4], low[4];
    uint64_t sv[4];
    const int64_t row0 = base + (int64_t)tid * kRowsPerThread;
    uint32_t pass;
    {
      uint64_t v[NC][4], code[4];
      decode_all<NC, 4>(p, raw, v);
      load_rows4_clamped<NC>(p, row0 + tile, end, raw, all, begin);
      pass = vals_pass<NC, 4>(p, row0, v);
      const int64_t rem = end - row0;
      pass &= rem >= 4 ? 0xFu : (rem > 0 ? ((1u << rem) - 1u) : 0u);
      vals_code<NC, 4>(p, v, code);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        part[r] = (uint32_t)(code[r] >> L.wbits);
        low[r] = (uint32_t)(code[r] & lowmask);
        sv[r] = v[0][r];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (part[r] >= (uint32_t)P) {
        atomicOr(&g_err[0], 1u);
        pass &= ~(1u << r);
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) rank[r] = (pass & (1u << r)) ? atomicAdd(&hw[wave * P + part[r]], 1u) : 0u;
    lds_barrier();
    uint32_t colsum = 0;
    if (tid < P)
      for (int w = 0; w < NW; ++w) colsum += hw[w * P + tid];
    uint32_t n_tile;
    const uint32_t tb = block_excl_scan_1b(colsum, wsum2 + parity * 16, &n_tile);
    const bool hbad = n_tile > (uint32_t)tile || (size_t)(base / tile) >= (size_t)((p.nrows + tile - 1) / tile);
    if (hbad) atomicOr(&g_err[1], 1u);
    uint16_t* th = hdr + (size_t)(hbad ? 0 : base / tile) * (P + 1);
    if (tid < P) {
      uint32_t o = tb;
      if (!hbad) th[tid] = (uint16_t)tb;
      for (int w = 0; w < NW; ++w) {
        const uint32_t c = hw[w * P + tid];
        hw[w * P + tid] = o;
        o += c;
      }
    }
    if (tid == 0 && !hbad) th[P] = (uint16_t)n_tile;
    lds_barrier();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (!(pass & (1u << r))) continue;
      const uint32_t pos = hw[wave * P + part[r]] + rank[r];
      smeta[pos] = ((uint32_t)(row0 + r - base) << L.wbits) | low[r];
      sval[pos] = sv[r];
    }
    lds_barrier();
    const bool inb = (uint64_t)(base + tile) <= L.capacity + 16384u;
    if (!inb) atomicOr(&g_err[0], 2u);
#pragma unroll
    for (int k = 0; k < kRowsPerThread; ++k) {
      const uint32_t i = (uint32_t)(tid + k * T);
      if (inb) {
        L.meta[base + i] = smeta[i];
        L.vals[base + i] = sval[i];
      }
    }
    for (int i = tid; i < NW * P; i += T) hw[i] = 0;
  }
}

// Aggregate over the tile layout: workgroup (partition, split) walks its tiles in groups of
// G per wave; a group's segments are flattened (wave scan of the segment lengths) and read
// 64 entries per wave instruction, U instructions' loads in flight.
template <int G, int U>
__global__ __launch_bounds__(1024) void k_agg_v5(ScanParams p, PartLaunch L, SlotArrays sa, const uint16_t* hdr,
                                                 int ntiles) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int W = 1 << L.wbits;
  const int P = L.nparts;
  double* acc = reinterpret_cast<double*>(smem);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(acc + W);
  uint32_t* fst = cnt + W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, NW = blockDim.x >> 6;
  for (int i = tid; i < W; i += blockDim.x) {
    cnt[i] = 0;
    fst[i] = kNoRow;
    acc[i] = 0.0;
  }
  __syncthreads();
  const int part = blockIdx.x / L.splits, split = blockIdx.x % L.splits;
  const int t_lo = (int)((int64_t)ntiles * split / L.splits), t_hi = (int)((int64_t)ntiles * (split + 1) / L.splits);
  const uint32_t lowmask = (uint32_t)W - 1u;
  constexpr int TR = 4096;
  for (int tg = t_lo + wave * G; tg < t_hi; tg += NW * G) {
    const int l = lane < G ? lane : G - 1;
    const int t = tg + l;
    const bool valid = lane < G && t < t_hi;
    const uint16_t* th = hdr + (size_t)(valid ? t : tg) * (P + 1) + part;
    const uint32_t s0 = valid ? th[0] : 0u, s1 = valid ? th[1] : 0u;
    const uint32_t len = s1 - s0;
    const uint32_t incl = wave_incl_scan_u32(len, lane);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, G - 1);
    uint32_t ex[G], st[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      ex[j] = (uint32_t)__builtin_amdgcn_readlane((int)(incl - len), j);
      st[j] = (uint32_t)__builtin_amdgcn_readlane((int)((uint32_t)(tg + j) * TR + s0), j);
    }
    for (uint32_t e0 = 0; e0 < total; e0 += 64u * U) {
      uint32_t m[U], rowb[U];
      unsigned long long v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = e0 + u * 64u + lane;
        const uint32_t ec = e < total ? e : total - 1u;
        uint32_t idx = st[0] + ec, tb = (uint32_t)tg * TR;
#pragma unroll
        for (int j = 1; j < G; ++j)
          if (ec >= ex[j]) {
            idx = st[j] + (ec - ex[j]);
            tb = (uint32_t)(tg + j) * TR;
          }
        rowb[u] = tb;
        if (idx >= (uint32_t)L.capacity + 16384u) { atomicOr(&g_err[2], 1u); idx = 0; }
        m[u] = L.meta[idx];
        v[u] = L.vals[idx];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = e0 + u * 64u + lane;
        if (e >= total) continue;
        const uint32_t sl = m[u] & lowmask;
        const uint32_t row = rowb[u] + (m[u] >> L.wbits);
        atomicAdd(&cnt[sl], 1u);
        if (fst[sl] > row) atomicMin(&fst[sl], row);
        unsafeAtomicAdd(&acc[sl], as_f64(v[u]));
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
    unsafeAtomicAdd(reinterpret_cast<double*>(&sa.acc[gs]), acc[s]);
  }
}


// Variant F ("fused"): one persistent workgroup per CU produces AND consumes.  Workgroup x
// owns partition x (W = 2^wbits slots in LDS for the whole launch).  Rows go in batches of
// TB = G * K tiles: each workgroup counting-sorts its K tiles of batch b by partition (as v5)
// and stores each sorted tile write-through (sc1 16-byte buffer stores) into the tile's own
// block [vals | meta | header]; then signals done[b].  It then consumes batch b - 1: waits for
// done[b - 1] == G, acquires, and aggregates partition x's segment of every tile of that
// batch into its LDS table.  Entry blocks are never reused within a launch.  At the end the
// table is stored (each slot has exactly one owner: plain stores).  Every wait is bounded: a
// timeout sets *abort and every workgroup leaves; the host then runs the two-kernel path.
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
struct FusedArgs {
  unsigned char* blocks;   // [ntiles][tile_bytes]
  unsigned int* done;      // [nbatches] zeroed before launch
  unsigned int* abort_;    // zeroed before launch
  int ntiles, nbatches, k; // tiles per workgroup per batch
  int tile_bytes;          // vals (TR*8) + meta (TR*4) + header (1 KiB)
};
constexpr int kTR = 4096;
constexpr int kHdrOff = kTR * 12;

__device__ __forceinline__ bool wait_count(unsigned int* w, unsigned int target, unsigned int* abort_) {
  const unsigned long long t0 = wall_clock64();
  for (unsigned spins = 0;; ++spins) {
    if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    if (__hip_atomic_load(abort_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return false;
    if (wall_clock64() - t0 > 2000000ull) {  // 20 ms at 100 MHz
      __hip_atomic_store(abort_, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

__global__ __launch_bounds__(1024) void k_fused(ScanParams pin, PartLaunch L, SlotArrays sa, FusedArgs F) {
  extern __shared__ __align__(16) unsigned char smem[];
  ScanParams p = pin;
  specialize(p);
  constexpr int NC = 3;
  const int T = blockDim.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, NW = T >> 6;
  const int P = L.nparts, G = gridDim.x, x = blockIdx.x;
  const int W = 1 << L.wbits;
  // LDS: table | staging vals | staging meta | header (u16, 512) | hist [2][P] | wsum [2][16] | flag
  double* tacc = reinterpret_cast<double*>(smem);
  uint32_t* tcnt = reinterpret_cast<uint32_t*>(tacc + W);
  uint32_t* tfst = tcnt + W;
  unsigned long long* sval = reinterpret_cast<unsigned long long*>(tfst + W);
  uint32_t* smeta = reinterpret_cast<uint32_t*>(sval + kTR);
  uint16_t* shdr = reinterpret_cast<uint16_t*>(smeta + kTR);
  uint32_t* hist2 = reinterpret_cast<uint32_t*>(shdr + 512);
  uint32_t* wsum2 = hist2 + 2 * P;
  uint32_t* sflag = wsum2 + 32;
  for (int i = tid; i < W; i += T) {
    tacc[i] = 0.0;
    tcnt[i] = 0;
    tfst[i] = kNoRow;
  }
  for (int i = tid; i < 2 * P; i += T) hist2[i] = 0;
  for (int i = tid; i < 512; i += T) shdr[i] = 0;
  lds_barrier();
  const uint64_t lowmask = (1ull << L.wbits) - 1ull;
  const uint32_t all = (1u << NC) - 1u;
  const int TB = G * F.k;
  // this workgroup's j-th tile of batch b
  auto tile_of = [&](int b, int j) { return b * TB + x * F.k + j; };
  auto tile_rows = [&](int t, int64_t& b0, int64_t& e0) {
    b0 = (int64_t)t * kTR;
    e0 = min(p.nrows, b0 + kTR);
  };
  Chunk raw[NC];
  {
    int64_t b0, e0;
    tile_rows(tile_of(0, 0), b0, e0);
    if (b0 < p.nrows) load_rows4_clamped<NC>(p, b0 + (int64_t)tid * kRowsPerThread, e0, raw, all, b0);
    else load_rows4_clamped<NC>(p, (int64_t)tid * kRowsPerThread, kTR, raw, all, 0);
  }
  int parity = 0;
  bool ok = true;
  for (int b = 0; b <= F.nbatches && ok; ++b) {
    if (b < F.nbatches) {
      for (int j = 0; j < F.k; ++j, parity ^= 1) {
        const int t = tile_of(b, j);
        int64_t base, end;
        tile_rows(t, base, end);
        // next tile to produce (prefetch)
        const int tn = j + 1 < F.k ? t + 1 : tile_of(b + 1, 0);
        int64_t nb0, ne0;
        tile_rows(tn, nb0, ne0);
        if (nb0 >= p.nrows) { nb0 = 0; ne0 = kTR; }
        uint32_t* hist = hist2 + parity * P;
        uint32_t part[4], rank[4], low[4];
        uint64_t sv[4];
        const int64_t row0 = base + (int64_t)tid * kRowsPerThread;
        uint32_t pass;
        {
          uint64_t v[NC][4], code[4];
          decode_all<NC, 4>(p, raw, v);
          load_rows4_clamped<NC>(p, nb0 + (int64_t)tid * kRowsPerThread, ne0, raw, all, nb0);
          pass = vals_pass<NC, 4>(p, row0, v);
          const int64_t rem = end - row0;
          pass &= rem >= 4 ? 0xFu : (rem > 0 ? ((1u << rem) - 1u) : 0u);
          vals_code<NC, 4>(p, v, code);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            part[r] = (uint32_t)(code[r] >> L.wbits);
            low[r] = (uint32_t)(code[r] & lowmask);
            sv[r] = v[0][r];
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) rank[r] = (pass & (1u << r)) ? atomicAdd(&hist[part[r]], 1u) : 0u;
        lds_barrier();
        const uint32_t mine = tid < P ? hist[tid] : 0u;
        uint32_t n_tile;
        const uint32_t off = block_excl_scan_1b(mine, wsum2 + parity * 16, &n_tile);
        if (tid < P) shdr[tid] = (uint16_t)off;
        if (tid == 0) shdr[P] = (uint16_t)n_tile;
        lds_barrier();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (!(pass & (1u << r))) continue;
          const uint32_t pos = shdr[part[r]] + rank[r];
          smeta[pos] = ((uint32_t)(row0 + r - base) << L.wbits) | low[r];
          sval[pos] = sv[r];
        }
        lds_barrier();
        if (t < F.ntiles) {
          __amdgpu_buffer_rsrc_t rs =
              __builtin_amdgcn_make_buffer_rsrc(F.blocks + (size_t)t * F.tile_bytes, 0, F.tile_bytes, 0x00020000);
          const u32x4v* lv = reinterpret_cast<const u32x4v*>(sval);
          const u32x4v* lm = reinterpret_cast<const u32x4v*>(smeta);
          __builtin_amdgcn_raw_buffer_store_b128(lv[tid], rs, tid * 16, 0, 16);
          __builtin_amdgcn_raw_buffer_store_b128(lv[tid + 1024], rs, (tid + 1024) * 16, 0, 16);
          __builtin_amdgcn_raw_buffer_store_b128(lm[tid], rs, kTR * 8 + tid * 16, 0, 16);
          if (tid < 64) {
            const u32x4v* lh = reinterpret_cast<const u32x4v*>(shdr);
            __builtin_amdgcn_raw_buffer_store_b128(lh[tid], rs, kHdrOff + tid * 16, 0, 16);
          }
        }
        if (tid < P) hist[tid] = 0;
      }
      // publish batch b: every storing wave drains, then one lane counts the workgroup in
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(&F.done[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (b >= 1) {
      const int cb = b - 1;
      if (tid == 0) {
        const bool got = wait_count(&F.done[cb], (unsigned)G, F.abort_);
        sflag[0] = got ? 1u : 0u;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      ok = sflag[0] != 0u;
      if (!ok) break;
      if (x < P) {
        const int t_lo = cb * TB, t_hi = min(F.ntiles, (cb + 1) * TB);
        constexpr int GG = 8, U = 2;
        for (int tg = t_lo + wave * GG; tg < t_hi; tg += NW * GG) {
          const int l = lane < GG ? lane : GG - 1;
          const int t = tg + l;
          const bool valid = lane < GG && t < t_hi;
          const uint16_t* th = reinterpret_cast<const uint16_t*>(F.blocks + (size_t)(valid ? t : tg) * F.tile_bytes + kHdrOff) + x;
          const uint32_t s0 = valid ? th[0] : 0u, s1 = valid ? th[1] : 0u;
          const uint32_t len = s1 - s0;
          const uint32_t incl = wave_incl_scan_u32(len, lane);
          const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, GG - 1);
          uint32_t ex[GG], st[GG];
#pragma unroll
          for (int j = 0; j < GG; ++j) {
            ex[j] = (uint32_t)__builtin_amdgcn_readlane((int)(incl - len), j);
            st[j] = (uint32_t)__builtin_amdgcn_readlane((int)s0, j);
          }
          for (uint32_t e0 = 0; e0 < total; e0 += 64u * U) {
            uint32_t m[U], rowb[U];
            unsigned long long v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const uint32_t e = e0 + u * 64u + lane;
              const uint32_t ec = e < total ? e : total - 1u;
              uint32_t j0 = 0;
#pragma unroll
              for (int j = 1; j < GG; ++j) j0 += ec >= ex[j] ? 1u : 0u;
              uint32_t exj = ex[0], stj = st[0];
#pragma unroll
              for (int j = 1; j < GG; ++j)
                if (j0 == (uint32_t)j) { exj = ex[j]; stj = st[j]; }
              uint32_t tt = (uint32_t)tg + j0;
              uint32_t pos = stj + (ec - exj);
              if (pos >= (uint32_t)kTR || tt >= (uint32_t)F.ntiles) { atomicOr(&g_err[3], 1u); pos = 0; tt = 0; }
              const unsigned char* blk = F.blocks + (size_t)tt * F.tile_bytes;
              rowb[u] = tt * kTR;
              m[u] = reinterpret_cast<const uint32_t*>(blk + kTR * 8)[pos];
              v[u] = reinterpret_cast<const unsigned long long*>(blk)[pos];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const uint32_t e = e0 + u * 64u + lane;
              if (e >= total) continue;
              const uint32_t sl = m[u] & (uint32_t)lowmask;
              const uint32_t row = rowb[u] + (m[u] >> L.wbits);
              atomicAdd(&tcnt[sl], 1u);
              if (tfst[sl] > row) atomicMin(&tfst[sl], row);
              unsafeAtomicAdd(&tacc[sl], as_f64(v[u]));
            }
          }
        }
      }
    }
  }
  if (!ok || x >= P) return;
  __syncthreads();
  const uint64_t slot0 = (uint64_t)x << L.wbits;
  for (int s = tid; s < W; s += T) {
    const uint64_t gs = slot0 + s;
    if (gs >= p.nslots) break;
    sa.cnt[gs] = tcnt[s];
    sa.fst[gs] = tfst[s];
    sa.acc[gs] = as_u64(tacc[s]);
  }
}


// Aggregate v6 over the tile layout: headers of the next two tile groups prefetched while a
// group is aggregated; an entry finds its tile by G compares against wave-uniform segment
// starts and takes the tile's start / first index with two lane shuffles; workgroups of one
// XCD take consecutive partitions over the same tile range (their segments share edge lines
// in that XCD's L2).
template <int G, int U>
__global__ __launch_bounds__(1024) void k_agg_v6(ScanParams p, PartLaunch L, SlotArrays sa, const uint16_t* hdr,
                                                 int ntiles) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int W = 1 << L.wbits;
  const int P = L.nparts;
  double* acc = reinterpret_cast<double*>(smem);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(acc + W);
  uint32_t* fst = cnt + W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, NW = blockDim.x >> 6;
  for (int i = tid; i < W; i += blockDim.x) {
    cnt[i] = 0;
    fst[i] = kNoRow;
    acc[i] = 0.0;
  }
  __syncthreads();
  // XCD-aware (partition, split)
  const int nx = 8;
  const int per_x = (P + nx - 1) / nx;
  const int bx = blockIdx.x % nx, bi = blockIdx.x / nx;
  const int part = bx * per_x + bi % per_x, split = bi / per_x;
  if (part >= P || split >= L.splits) return;
  const int t_lo = (int)((int64_t)ntiles * split / L.splits), t_hi = (int)((int64_t)ntiles * (split + 1) / L.splits);
  const uint32_t lowmask = (uint32_t)W - 1u;
  constexpr int TR = 4096;
  auto hload = [&](int tg, uint32_t& s0, uint32_t& s1) {
    const int t = tg + lane;
    const bool valid = lane < G && t < t_hi;
    const uint16_t* th = hdr + (size_t)(valid ? t : t_lo) * (P + 1) + part;
    const uint32_t a = th[0], b = th[1];
    s0 = valid ? a : 0u;
    s1 = valid ? b : 0u;
  };
  int tg = t_lo + wave * G;
  const int stride = NW * G;
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
    const uint32_t stl = (uint32_t)(tg + lane) * TR + s0;  // lane j: first entry index of tile j's segment
    for (uint32_t e0 = 0; e0 < total; e0 += 64u * U) {
      uint32_t m[U], rowb[U];
      unsigned long long v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = e0 + u * 64u + lane;
        const uint32_t ec = e < total ? e : total - 1u;
        int j0 = 0;
#pragma unroll
        for (int j = 1; j < G; ++j) j0 += ec >= ex[j] ? 1 : 0;
        const uint32_t exj = (uint32_t)__shfl((int)excl, j0, 64);
        const uint32_t stj = (uint32_t)__shfl((int)stl, j0, 64);
        uint32_t idx = stj + (ec - exj);
        if (idx >= (uint32_t)L.capacity + 16384u) { atomicOr(&g_err[2], 2u); idx = 0; }
        rowb[u] = (uint32_t)(tg + j0) * TR;
        m[u] = L.meta[idx];
        v[u] = L.vals[idx];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = e0 + u * 64u + lane;
        if (e >= total) continue;
        const uint32_t sl = m[u] & lowmask;
        const uint32_t row = rowb[u] + (m[u] >> L.wbits);
        atomicAdd(&cnt[sl], 1u);
        if (fst[sl] > row) atomicMin(&fst[sl], row);
        unsafeAtomicAdd(&acc[sl], as_f64(v[u]));
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
    unsafeAtomicAdd(reinterpret_cast<double*>(&sa.acc[gs]), acc[s]);
  }
}

// ------------------------------------------------------------------------------------
struct Bufs {
  int64_t n;
  double* fare;
  int32_t *pl, *ven;
  ScanParams p;
  SlotArrays sa;
  unsigned long long *cnt, *acc;
  uint32_t* fst;
  uint32_t* counts;
  uint32_t* scratch;
  uint32_t* meta;
  unsigned long long* vals;
};

static PartLaunch make_launch(Bufs& b, int cu, int threads, int per_cu) {
  PartLaunch L{};
  L.wbits = 13;
  L.nparts = (int)((b.p.nslots + (1ull << L.wbits) - 1) >> L.wbits);
  L.threads = threads;
  L.chunks = 1;
  L.load_mask = 1u << 1;  // the count pass reads pickup_location only
  const int64_t ptile = 4096;
  const int64_t ptiles = (b.n + ptile - 1) / ptile;
  L.blocks = (int)std::min<int64_t>((int64_t)cu * per_cu, ptiles);
  L.rows_per_block = ((ptiles + L.blocks - 1) / L.blocks) * ptile;
  L.splits = 2;
  L.row_base = 0;
  L.capacity = ((uint64_t)b.n + 3) & ~3ull;
  L.counts = b.counts;
  L.meta = b.meta;
  L.vals = b.vals;
  return L;
}

static void init_slots(Bufs& b) {
  CK(hipMemsetAsync(b.cnt, 0, b.p.nslots * 8, 0));
  CK(hipMemsetAsync(b.fst, 0xFF, b.p.nslots * 4, 0));
  CK(hipMemsetAsync(b.acc, 0, b.p.nslots * 8, 0));
}

struct Res {
  std::vector<unsigned long long> cnt, acc;
  std::vector<uint32_t> fst;
};
static Res fetch(Bufs& b) {
  Res r;
  r.cnt.resize(b.p.nslots);
  r.acc.resize(b.p.nslots);
  r.fst.resize(b.p.nslots);
  CK(hipMemcpy(r.cnt.data(), b.cnt, b.p.nslots * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r.acc.data(), b.acc, b.p.nslots * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r.fst.data(), b.fst, b.p.nslots * 4, hipMemcpyDeviceToHost));
  return r;
}
static bool same(const Res& a, const Res& b, const char* what) {
  size_t bad = 0;
  for (size_t i = 0; i < a.cnt.size(); ++i)
    if (a.cnt[i] != b.cnt[i] || a.acc[i] != b.acc[i] || a.fst[i] != b.fst[i]) {
      if (bad < 3) fprintf(stderr, "%s: slot %zu cnt %llu/%llu fst %u/%u\n", what, i, a.cnt[i], b.cnt[i], a.fst[i], b.fst[i]);
      ++bad;
    }
  printf("%s: %s (%zu bad slots)\n", what, bad ? "MISMATCH" : "match", bad);
  return bad == 0;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000ll;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  int cu = 0;
  CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
  Bufs b{};
  b.n = n;
  const size_t pad = 65536;
  CK(hipMalloc(&b.fare, n * 8 + pad));
  CK(hipMalloc(&b.pl, n * 4 + pad));
  CK(hipMalloc(&b.ven, n * 4 + pad));
  k_gen<<<4096, 256>>>(n, b.fare, b.pl, b.ven);
  b.p.nrows = n;
  b.p.ncols = 3;
  b.p.cols[0] = {reinterpret_cast<const unsigned char*>(b.fare), BQG_F64, 3};
  b.p.cols[1] = {reinterpret_cast<const unsigned char*>(b.pl), BQG_I32, 2};
  b.p.cols[2] = {reinterpret_cast<const unsigned char*>(b.ven), BQG_I32, 2};
  b.p.nkeys = 2;
  b.p.keys[0] = {1, 0, 0, 2, 500000};
  b.p.keys[1] = {2, 0, 1, 1, 2};
  b.p.nsum = 1;
  b.p.sum_is_float[0] = 1;
  b.p.mask_col = -1;
  b.p.nslots = 1000000;
  CK(hipMalloc(&b.cnt, b.p.nslots * 8));
  CK(hipMalloc(&b.acc, b.p.nslots * 8));
  CK(hipMalloc(&b.fst, b.p.nslots * 4));
  b.sa.cnt = b.cnt;
  b.sa.acc = b.acc;
  b.sa.fst = b.fst;
  CK(hipMalloc(&b.counts, (size_t)4096 * 2048 * 4 + 4096));
  CK(hipMalloc(&b.scratch, 1 << 22));
  CK(hipMalloc(&b.meta, n * 4 + pad));
  CK(hipMalloc(&b.vals, n * 8 + pad));
  hipEvent_t ev[8];
  for (auto& e : ev) CK(hipEventCreate(&e));
  printf("rows %lld cus %d\n", (long long)n, cu);

  // ---- library pipeline (reference + timing)
  PartLaunch L = make_launch(b, cu, 1024, 2);
  auto lib_pipeline = [&](bool prof) {
    init_slots(b);
    CK(hipMemsetAsync(L.counts + (size_t)L.nparts * L.blocks, 0, 4, 0));
    CK(hipEventRecord(ev[0], 0));
    k_count_lib<<<L.blocks, L.threads, L.nparts * 4>>>(b.p, L);
    CK(hipEventRecord(ev[1], 0));
    launch_exclusive_scan_u32(L.counts, (uint64_t)L.nparts * L.blocks + 1, b.scratch, 0);
    CK(hipEventRecord(ev[2], 0));
    const size_t slds = part_scatter_lds(L.nparts, L.threads, 1);
    if (prof) k_scatter_prof<<<L.blocks, L.threads, slds>>>(b.p, L);
    else k_scatter_lib<<<L.blocks, L.threads, slds>>>(b.p, L);
    CK(hipEventRecord(ev[3], 0));
    const size_t agg_lds = ((size_t)1 << L.wbits) * 16 + ((size_t)L.blocks + 1) * 4;
    k_part_aggregate<<<L.nparts * L.splits, 1024, agg_lds>>>(b.p, L, b.sa);
    CK(hipEventRecord(ev[4], 0));
    CK(hipEventSynchronize(ev[4]));
    float t[4];
    for (int i = 0; i < 4; ++i) CK(hipEventElapsedTime(&t[i], ev[i], ev[i + 1]));
    printf("lib%s: count %.3f scan %.3f scatter %.3f aggregate %.3f total %.3f ms\n", prof ? "(prof)" : "", t[0], t[1],
           t[2], t[3], t[0] + t[1] + t[2] + t[3]);
  };
  for (int r = 0; r < reps; ++r) lib_pipeline(false);
  const Res ref = fetch(b);
  // launch-shape sweep of the library bodies
  {
    const int shapes[][2] = {{1024, 1}, {1024, 2}};
    for (auto& sh : shapes) {
      L = make_launch(b, cu, sh[0], sh[1]);
      printf("threads %d per_cu %d blocks %d rows/block %lld\n", sh[0], sh[1], L.blocks, (long long)L.rows_per_block);
      for (int r = 0; r < 2; ++r) lib_pipeline(false);
      same(ref, fetch(b), "shape");
    }
    L = make_launch(b, cu, 1024, 2);
  }
  auto v2 = [&](auto kern, const char* what, int per_cu, int pd) {
    PartLaunch L2 = make_launch(b, cu, 1024, per_cu);
    // whole groups of pd tiles per block
    const int64_t g = 4096 * pd;
    L2.rows_per_block = (L2.rows_per_block + g - 1) / g * g;
    L2.blocks = (int)((b.n + L2.rows_per_block - 1) / L2.rows_per_block);
    for (int r = 0; r < 3; ++r) {
      init_slots(b);
      CK(hipMemsetAsync(L2.counts + (size_t)L2.nparts * L2.blocks, 0, 4, 0));
      CK(hipEventRecord(ev[0], 0));
      k_count_lib<<<L2.blocks, 1024, L2.nparts * 4>>>(b.p, L2);
      CK(hipEventRecord(ev[1], 0));
      launch_exclusive_scan_u32(L2.counts, (uint64_t)L2.nparts * L2.blocks + 1, b.scratch, 0);
      CK(hipEventRecord(ev[2], 0));
      kern<<<L2.blocks, 1024, part_scatter_lds(L2.nparts, 1024, 1) + 3 * 16 * L2.nparts * 4>>>(b.p, L2);
      CK(hipEventRecord(ev[3], 0));
      k_part_aggregate<<<L2.nparts * L2.splits, 1024, ((size_t)1 << L2.wbits) * 16 + ((size_t)L2.blocks + 1) * 4>>>(b.p, L2, b.sa);
      CK(hipEventRecord(ev[4], 0));
      CK(hipEventSynchronize(ev[4]));
      float t[4];
      for (int i = 0; i < 4; ++i) CK(hipEventElapsedTime(&t[i], ev[i], ev[i + 1]));
      printf("%s per_cu %d: count %.3f scan %.3f scatter %.3f aggregate %.3f total %.3f ms\n", what, per_cu, t[0], t[1], t[2], t[3],
             t[0] + t[1] + t[2] + t[3]);
    }
    same(ref, fetch(b), what);
  };
  v2(k_scatter_v3<0>, "v3 wave-hist", 2, 1);
  {
    uint16_t* hdr;
    const int ntiles = (int)((b.n + 4095) / 4096);
    CK(hipMalloc(&hdr, (size_t)ntiles * 130 * 2 + 4096));
    auto v5 = [&](auto agg, const char* what, int splits) {
      PartLaunch L5 = make_launch(b, cu, 1024, 2);
      L5.splits = splits;
      const size_t slds = (size_t)4096 * 12 + 2 * 16 * L5.nparts * 4 + 256;
      for (int r = 0; r < 3; ++r) {
        init_slots(b);
        CK(hipEventRecord(ev[0], 0));
        k_scatter_v5<<<L5.blocks, 1024, slds>>>(b.p, L5, hdr);
        CK(hipEventRecord(ev[1], 0));
        agg<<<((L5.nparts + 7) / 8) * 8 * L5.splits, 1024, ((size_t)1 << L5.wbits) * 16>>>(b.p, L5, b.sa, hdr, ntiles);
        CK(hipEventRecord(ev[2], 0));
        CK(hipEventSynchronize(ev[2]));
        float t[2];
        for (int i = 0; i < 2; ++i) CK(hipEventElapsedTime(&t[i], ev[i], ev[i + 1]));
        printf("%s splits %d: scatter %.3f aggregate %.3f total %.3f ms\n", what, splits, t[0], t[1], t[0] + t[1]);
      }
      same(ref, fetch(b), what);
      unsigned int er[4];
      CK(hipMemcpyFromSymbol(er, g_err, sizeof er));
      printf("%s: bounds flags %u %u %u\n", what, er[0], er[1], er[2]);
    };
    CK(hipFuncSetAttribute((const void*)k_scatter_v5, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    v5(k_agg_v5<8, 2>, "v5 tile-layout G8 U2", 2);
    v5(k_agg_v6<8, 4>, "v6 G8 U4", 2);
    v5(k_agg_v6<16, 4>, "v6 G16 U4", 2);
    v5(k_agg_v6<16, 2>, "v6 G16 U2", 2);
    v5(k_agg_v6<32, 4>, "v6 G32 U4", 2);
    v5(k_agg_v6<16, 4>, "v6 G16 U4", 1);
  }
  if (argc > 3 && atoi(argv[3]) == 1) {
    PartLaunch LF = make_launch(b, cu, 1024, 1);
    LF.wbits = 12;
    LF.nparts = (int)((b.p.nslots + 4095) >> 12);
    FusedArgs F{};
    F.ntiles = (int)((b.n + kTR - 1) / kTR);
    F.tile_bytes = kTR * 12 + 1024;
    const size_t lds = (size_t)4096 * 16 + kTR * 12 + 1024 + 2 * LF.nparts * 4 + 32 * 4 + 64;
    CK(hipFuncSetAttribute((const void*)k_fused, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_fused, 1024, lds));
    unsigned char* blocks;
    CK(hipMalloc(&blocks, (size_t)F.ntiles * F.tile_bytes + 4096));
    unsigned int* flags;
    CK(hipMalloc(&flags, 4096 * 4));
    F.blocks = blocks;
    F.done = flags + 1;
    F.abort_ = flags;
    for (int kk : {8}) {
      F.k = kk;
      F.nbatches = (F.ntiles + cu * kk - 1) / (cu * kk);
      printf("fused: occupancy %d/CU, lds %zu, k %d, batches %d\n", occ, lds, kk, F.nbatches);
      for (int r = 0; r < 3; ++r) {
        init_slots(b);
        CK(hipMemsetAsync(flags, 0, 4096 * 4, 0));
        CK(hipEventRecord(ev[0], 0));
        k_fused<<<cu, 1024, lds>>>(b.p, LF, b.sa, F);
        CK(hipEventRecord(ev[1], 0));
        CK(hipEventSynchronize(ev[1]));
        float t;
        CK(hipEventElapsedTime(&t, ev[0], ev[1]));
        unsigned int ab = 0;
        CK(hipMemcpy(&ab, flags, 4, hipMemcpyDeviceToHost));
        unsigned int er[4];
        CK(hipMemcpyFromSymbol(er, g_err, sizeof er));
        printf("fused k=%d: %.3f ms abort=%u bounds %u\n", kk, t, ab, er[3]);
      }
      same(ref, fetch(b), "fused");
    }
  }


  unsigned long long z[8] = {0};
  CK(hipMemcpyToSymbol(g_phase, z, sizeof z));
  lib_pipeline(true);
  same(ref, fetch(b), "lib(prof)");
  unsigned long long ph[8];
  CK(hipMemcpyFromSymbol(ph, g_phase, sizeof ph));
  const char* names[6] = {"setup", "decode+wait", "hist+bar", "scan+bar", "stage+bar", "copyout"};
  double tot = 0;
  for (int i = 0; i < 6; ++i) tot += (double)ph[i];
  for (int i = 0; i < 6; ++i) printf("  %-12s %5.1f %%  %.0f cyc/block\n", names[i], 100.0 * ph[i] / tot, (double)ph[i] / L.blocks);
  return 0;
}
