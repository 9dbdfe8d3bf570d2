// part_micro.hip -- C3-shaped partitioned aggregation (100 M rows, pickup_location x vendor_id,
// ~1 M dense slots, one f64 sum + count) outside the library: the library's tile scatter body
// (partition.h, specialised like the JIT build) with the library aggregate (k_partition.hip) and a fused
// persistent producer / consumer kernel, each timed with events and checked slot by slot
// against a per-row global-atomics reference (exact: the values are dyadic).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I bqueryd_amd/csrc
//        -I include tools/micro/part_micro.hip -o build/part_micro
// run:   part_micro [rows] [reps] [fused 0/1]
#define BQ_NC 3
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define BQG_PART_MICRO
#include "k_partition.hip"

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

__device__ unsigned int g_err[4];  // bounds-check hits: [2] aggregate entry index, [3] fused entry index

__global__ void k_gen(int64_t n, double* fare, int32_t* pl, int32_t* ven) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = mix64((uint64_t)i * 0x9E3779B97F4A7C15ull + 12345);
    pl[i] = (int32_t)((h >> 8) % 500000u);
    ven[i] = 1 + (int32_t)((h >> 40) & 1u);
    fare[i] = 2.5 + (double)((h >> 44) % 30000u) / 64.0;
  }
}

// reference: one global atomic per row and state
__global__ void k_ref(int64_t n, const double* fare, const int32_t* pl, const int32_t* ven, SlotArrays sa) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t s = (uint64_t)pl[i] * 2u + (uint64_t)(ven[i] - 1);
    atomicAdd(&sa.cnt[s], 1ull);
    atomicMin(&sa.fst[s], (uint32_t)i);
    unsafeAtomicAdd(reinterpret_cast<double*>(&sa.acc[s]), fare[i]);
  }
}

__global__ __launch_bounds__(1024) void k_scatter_lib(ScanParams pin, PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  ScanParams p = pin;
  specialize(p);
  part_scatter_body<3>(p, L, smem);
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


template <int G, int U, int NSUM, int MODE>
__global__ __launch_bounds__(1024) void k_agg_probe(ScanParams p, PartLaunch L, SlotArrays sa) {
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
  uint32_t sink = 0;
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
        if (MODE == 2) {
          m[u] = (uint32_t)(idx * 2654435761u) & 0x1FFFu;
#pragma unroll
          for (int q = 0; q < NV; ++q) v[u][q] = 0x4000000000000000ull;
        } else {
          m[u] = L.meta[idx];
#pragma unroll
          for (int q = 0; q < NV; ++q) v[u][q] = L.vals[(size_t)q * L.capacity + idx];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = e0 + u * 64u + lane;
        if (e >= total) continue;
        const uint32_t sl = m[u] & lowmask;
        const uint32_t row = rowb[u] + (m[u] >> L.wbits);
        if (MODE == 1) {
          sink ^= m[u] ^ (uint32_t)v[u][0] ^ row;
          continue;
        }
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
  if (MODE == 1 && sink == 0x12345u) cnt[0] = sink;
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
struct Bufs {
  int64_t n;
  double* fare;
  int32_t *pl, *ven;
  ScanParams p;
  SlotArrays sa;
  unsigned long long *cnt, *acc;
  uint32_t* fst;
};

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
  unsigned int er[4];
  CK(hipMemcpyFromSymbol(er, g_err, sizeof er));
  printf("%s: %s (%zu bad slots) bounds flags %u %u\n", what, bad ? "MISMATCH" : "match", bad, er[2], er[3]);
  return bad == 0;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000ll;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
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
  hipEvent_t ev[8];
  for (auto& e : ev) CK(hipEventCreate(&e));
  printf("rows %lld cus %d\n", (long long)n, cu);
  init_slots(b);
  k_ref<<<4096, 256>>>(n, b.fare, b.pl, b.ven, b.sa);
  CK(hipDeviceSynchronize());
  const Res ref = fetch(b);

  // the library's launch shape (api.hip, partitioned mode)
  PartLaunch L{};
  L.wbits = 13;
  L.nparts = (int)((b.p.nslots + (1ull << L.wbits) - 1) >> L.wbits);
  L.threads = 1024;
  L.tile_rows = 4096;
  L.ntiles = (n + 4095) / 4096;
  L.blocks = (int)std::min<int64_t>((int64_t)cu * 2, L.ntiles);
  L.rows_per_block = ((L.ntiles + L.blocks - 1) / L.blocks) * 4096;
  L.blocks = (int)((n + L.rows_per_block - 1) / L.rows_per_block);
  L.splits = 2;
  L.win = kAggWin;
  L.capacity = (uint64_t)L.ntiles * 4096;
  CK(hipMalloc(&L.hdr, (size_t)L.ntiles * (L.nparts + 1) * 2 + 256));
  CK(hipMalloc(&L.meta, L.capacity * 4 + 256));
  CK(hipMalloc(&L.vals, L.capacity * 8 + 256));
  L.partial_bytes = ((size_t)1 << L.wbits) * 16;
  CK(hipMalloc(&L.partial, (size_t)L.nparts * 8 * L.partial_bytes + 256));

  const size_t slds = part_scatter_lds(L.nparts, L.threads, 1);
  CK(hipFuncSetAttribute((const void*)k_scatter_lib, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  auto agg_run = [&](auto agg, const char* what, int splits) {
    L.splits = splits;
    const unsigned grid = (unsigned)(((L.nparts + 7) / 8) * 8 * splits);
    for (int r = 0; r < reps; ++r) {
      init_slots(b);
      CK(hipEventRecord(ev[0], 0));
      k_scatter_lib<<<L.blocks, L.threads, slds>>>(b.p, L);
      CK(hipEventRecord(ev[1], 0));
      agg<<<grid, 1024, part_agg_lds_launch(L.wbits, 1, false)>>>(b.p, L, b.sa);
      CK(hipEventRecord(ev[2], 0));
      CK(hipEventSynchronize(ev[2]));
      float t[2];
      for (int i = 0; i < 2; ++i) CK(hipEventElapsedTime(&t[i], ev[i], ev[i + 1]));
      printf("%s splits %d: scatter %.3f aggregate %.3f total %.3f ms\n", what, splits, t[0], t[1], t[0] + t[1]);
    }
    same(ref, fetch(b), what);
  };
  agg_run(k_part_aggregate<2, 2, 1, false, false>, "agg U2 granules (library; splits > 1 need k_part_combine)", 1);

  agg_run(k_agg_probe<8, 4, 1, 1>, "probe: loads only (no LDS atomics)", 2);
  agg_run(k_agg_probe<8, 4, 1, 2>, "probe: LDS atomics only (no entry loads)", 2);

  if (argc > 3 && atoi(argv[3]) == 1) {
    PartLaunch LF = L;
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
    for (int kk : {4, 8}) {
      F.k = kk;
      F.nbatches = (F.ntiles + cu * kk - 1) / (cu * kk);
      printf("fused: occupancy %d/CU, lds %zu, k %d, batches %d\n", occ, lds, kk, F.nbatches);
      for (int r = 0; r < reps; ++r) {
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
        printf("fused k=%d: %.3f ms abort=%u\n", kk, t, ab);
      }
      same(ref, fetch(b), "fused");
    }
  }
  return 0;
}
