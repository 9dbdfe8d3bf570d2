// k_misc.hip -- emit, stats, where_terms mask, row selection, basket expansion
#include <hip/hip_runtime.h>

#include <algorithm>

#include "partition.h"  // device.h + block_excl_scan_1024

namespace bqg {

// ------------------------------------------------------------------------------------
// Emit: occupied slots -> first-appearance order -> output columns
// ------------------------------------------------------------------------------------
// Occupied slots -> (first row, slot) list in slot order: per-workgroup counts, an exclusive
// scan of the counts, then an ordered write (deterministic, no shared counter).
constexpr int kCompactBlock = 1024;
constexpr int kCompactSlots = kCompactBlock * 4;

__global__ __launch_bounds__(kCompactBlock) void k_compact_count(SlotArrays sa, uint64_t nslots, uint32_t* block_counts,
                                                                 unsigned long long* total) {
  const uint64_t base = (uint64_t)blockIdx.x * kCompactSlots + (uint64_t)threadIdx.x * 4;
  unsigned int c = 0;
  unsigned long long rows = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint64_t s = base + r;
    const unsigned long long n = s < nslots ? sa.cnt[s] : 0ull;
    c += n > 0 ? 1u : 0u;
    rows += n;
  }
  __shared__ unsigned int wc[kCompactBlock / 64];
  __shared__ unsigned long long wr[kCompactBlock / 64];
  const unsigned int cw = (unsigned int)wave_sum_u64(c);
  const unsigned long long rw = wave_sum_u64(rows);
  if ((threadIdx.x & 63) == 0) {
    wc[threadIdx.x >> 6] = cw;
    wr[threadIdx.x >> 6] = rw;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned int t = 0;
    unsigned long long tr = 0;
    for (int q = 0; q < kCompactBlock / 64; ++q) {
      t += wc[q];
      tr += wr[q];
    }
    block_counts[blockIdx.x] = t;
    if (tr) atomicAdd(total, tr);
  }
}

__global__ __launch_bounds__(kCompactBlock) void k_compact_write(SlotArrays sa, uint64_t nslots, const uint32_t* block_offsets,
                                                                 uint32_t* list_fst, uint32_t* list_slot) {
  const uint64_t base = (uint64_t)blockIdx.x * kCompactSlots + (uint64_t)threadIdx.x * 4;
  uint32_t occ = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint64_t s = base + r;
    if (s < nslots && sa.cnt[s] > 0) occ |= 1u << r;
  }
  __shared__ unsigned int wsum[kCompactBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned int v = (unsigned int)__popc(occ), incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned int t = (unsigned int)__shfl_up((int)incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  unsigned int before = 0;
  for (int q = 0; q < wave; ++q) before += wsum[q];
  unsigned int pos = block_offsets[blockIdx.x] + before + incl - v;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (occ & (1u << r)) {
      list_fst[pos] = sa.fst[base + r];
      list_slot[pos] = (uint32_t)(base + r);
      ++pos;
    }
  }
}

// single-workgroup bitonic sort of up to 8192 (first_row, slot) pairs by first_row
__global__ __launch_bounds__(1024) void k_sort_small(const uint32_t* list_fst, const uint32_t* list_slot,
                                                     unsigned int n, uint32_t* order) {
  __shared__ uint32_t kf[8192];
  __shared__ uint32_t ks[8192];
  unsigned int m = 1;
  while (m < n) m <<= 1;
  for (unsigned int i = threadIdx.x; i < m; i += blockDim.x) {
    kf[i] = i < n ? list_fst[i] : kNoRow;
    ks[i] = i < n ? list_slot[i] : 0u;
  }
  __syncthreads();
  for (unsigned int k = 2; k <= m; k <<= 1) {
    for (unsigned int j = k >> 1; j > 0; j >>= 1) {
      for (unsigned int i = threadIdx.x; i < m; i += blockDim.x) {
        const unsigned int ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const uint32_t a = kf[i], b = kf[ixj];
          if ((a > b) == up) {
            kf[i] = b; kf[ixj] = a;
            const uint32_t t = ks[i]; ks[i] = ks[ixj]; ks[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  for (unsigned int i = threadIdx.x; i < n; i += blockDim.x) order[i] = ks[i];
}

// rank of each group = number of groups whose first row precedes its first row, read off a
// bitmap of first rows (N bits) with a two-level popcount prefix.
__global__ void k_setbits(const uint32_t* list_fst, unsigned int n, unsigned int* bitmap) {
  for (unsigned int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t f = list_fst[i];
    atomicOr(&bitmap[f >> 5], 1u << (f & 31));
  }
}

__global__ __launch_bounds__(1024) void k_word_scan(const unsigned int* bitmap, uint64_t nwords,
                                                    unsigned int* word_prefix, unsigned int* block_sum) {
  // the block scan of wave scans (one barrier; a 20-barrier LDS ladder took 17 us for the
  // 3 M words of a 100 M-row bitmap)
  const uint64_t w = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  const unsigned int c = w < nwords ? (unsigned int)__popc(bitmap[w]) : 0u;
  unsigned int tot;
  const unsigned int e = block_excl_scan_1024(c, &tot);
  if (w < nwords) word_prefix[w] = e;
  if (threadIdx.x == 0) block_sum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_block_scan(unsigned int* block_sum, uint64_t nblocks) {
  __shared__ unsigned int sh[1024];
  __shared__ unsigned int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t base = 0; base < nblocks; base += 1024) {
    const uint64_t i = base + threadIdx.x;
    const unsigned int c = i < nblocks ? block_sum[i] : 0u;
    sh[threadIdx.x] = c;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const unsigned int t = threadIdx.x >= (unsigned)o ? sh[threadIdx.x - o] : 0u;
      __syncthreads();
      sh[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < nblocks) block_sum[i] = carry + sh[threadIdx.x] - c;
    __syncthreads();
    if (threadIdx.x == 1023) carry += sh[1023];
    __syncthreads();
  }
}

__global__ void k_rank(const uint32_t* list_fst, const uint32_t* list_slot, unsigned int n,
                       const unsigned int* bitmap, const unsigned int* word_prefix,
                       const unsigned int* block_prefix, uint32_t* order) {
  for (unsigned int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t f = list_fst[i];
    const uint32_t w = f >> 5;
    const unsigned int r = block_prefix[w >> 10] + word_prefix[w] +
                           (unsigned int)__popc(bitmap[w] & ((1u << (f & 31)) - 1u));
    order[r] = list_slot[i];
  }
}

__global__ void k_emit(EmitParams e, SlotArrays sa, const uint32_t* order, unsigned int n, int nsum,
                       uint64_t nslots) {
  for (unsigned int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t s = order[i];
    const SlotRef t = slot_ref(sa, s, nslots, sa.cnt[s], sa.fst[s]);
    const uint64_t code = e.hash ? (uint64_t)sa.keys[s] : (uint64_t)s;
    emit_slot(e, s, code, i, t);
  }
}

// Large results: rank (first-row bitmap popcount) and emit in one pass over the compacted
// list, which is in slot order -- the slot totals are read coalesced and each group's output
// row is written at its rank (scatter-by-rank), instead of a rank pass writing `order` and an
// emit pass gathering the totals of random slots (~100 bytes of line traffic per 8-byte read).
__global__ void k_rank_emit(EmitParams e, SlotArrays sa, const uint32_t* list_fst, const uint32_t* list_slot,
                            unsigned int n, int nsum, uint64_t nslots, const unsigned int* bitmap,
                            const unsigned int* word_prefix, const unsigned int* block_prefix) {
  for (unsigned int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t f = list_fst[i];
    const uint32_t w = f >> 5;
    const unsigned int r = block_prefix[w >> 10] + word_prefix[w] +
                           (unsigned int)__popc(bitmap[w] & ((1u << (f & 31)) - 1u));
    const uint32_t s = list_slot[i];
    const SlotRef t = slot_ref(sa, s, nslots, sa.cnt[s], f);
    const uint64_t code = e.hash ? (uint64_t)sa.keys[s] : (uint64_t)s;
    emit_slot(e, s, code, r, t);
  }
}

// Large slot spaces without the compaction and its host round trip (round 6): the first-row
// bitmap is set straight from the slot arrays (an occupied slot has cnt > 0), the rank scan
// leaves the group count G on the device -- the emit lays the output columns out by it -- and
// mirrors G and the passing rows into page-locked host memory, which the host reads after an
// event while the emit runs; the copy of the G rows follows.
__global__ __launch_bounds__(1024) void k_setbits_slots(SlotArrays sa, uint64_t nslots, unsigned int* bitmap,
                                                        unsigned long long* rows_total) {
  unsigned long long rows = 0;
  for (uint64_t s = (uint64_t)blockIdx.x * 1024 + threadIdx.x; s < nslots; s += (uint64_t)gridDim.x * 1024) {
    const unsigned long long n = sa.cnt[s];
    if (n) {
      const uint32_t f = sa.fst[s];
      atomicOr(&bitmap[f >> 5], 1u << (f & 31));
      rows += n;
    }
  }
  __shared__ unsigned long long wr[16];
  rows = wave_sum_u64(rows);
  if ((threadIdx.x & 63) == 0) wr[threadIdx.x >> 6] = rows;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int q = 0; q < 16; ++q) t += wr[q];
    if (t) atomicAdd(rows_total, t);
  }
}

// The same marks without atomics (round 6): one byte per row, set to the query's epoch (1..255)
// with a plain store -- distinct groups have distinct first rows, so no two stores meet -- and
// read back as "byte == epoch"; the map is cleared only when the epoch wraps.  1 M random bit
// atomics took 43 us at C3 (the atomic unit's rate), the byte stores and the 100 MB read-back
// a fraction of that, and no bitmap fill.
__global__ __launch_bounds__(1024) void k_mark_rows(SlotArrays sa, uint64_t nslots, unsigned char* map,
                                                    unsigned char epoch, unsigned long long* rows_part) {
  unsigned long long rows = 0;
  for (uint64_t s = (uint64_t)blockIdx.x * 1024 + threadIdx.x; s < nslots; s += (uint64_t)gridDim.x * 1024) {
    const unsigned long long n = sa.cnt[s];
    if (n) {
      map[sa.fst[s]] = epoch;
      rows += n;
    }
  }
  __shared__ unsigned long long wr[16];
  rows = wave_sum_u64(rows);
  if ((threadIdx.x & 63) == 0) wr[threadIdx.x >> 6] = rows;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int q = 0; q < 16; ++q) t += wr[q];
    rows_part[blockIdx.x] = t;  // every workgroup: no zeroing, no atomics
  }
}

// 4 bytes -> 4 flag bits (byte == epoch), exact (no borrow between bytes)
__device__ __forceinline__ unsigned int epoch_bits4(unsigned int d, unsigned int ep4) {
  const unsigned int t = d ^ ep4;
  const unsigned int nz = ((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t;  // high bit: byte != epoch
  const unsigned int hi = ~nz & 0x80808080u;
  return ((hi >> 7) & 1u) | ((hi >> 14) & 2u) | ((hi >> 21) & 4u) | ((hi >> 28) & 8u);
}

// the row map's 32-row words (32 bytes per thread, two 16-byte loads) as bitmap words:
// per word its exclusive popcount prefix in its 1024-word block and the word (k_word_scan_pairs)
__global__ __launch_bounds__(1024) void k_map_scan_pairs(const unsigned char* map, uint64_t nwords, unsigned char epoch,
                                                         unsigned long long* word_pair, unsigned int* block_sum) {
  const uint64_t w = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  unsigned int b = 0;
  if (w < nwords) {
    const uint4 lo = load_stream16(map + w * 32), hi = load_stream16(map + w * 32 + 16);
    const unsigned int ep4 = 0x01010101u * epoch;
    b = epoch_bits4(lo.x, ep4) | epoch_bits4(lo.y, ep4) << 4 | epoch_bits4(lo.z, ep4) << 8 |
        epoch_bits4(lo.w, ep4) << 12 | epoch_bits4(hi.x, ep4) << 16 | epoch_bits4(hi.y, ep4) << 20 |
        epoch_bits4(hi.z, ep4) << 24 | epoch_bits4(hi.w, ep4) << 28;
  }
  unsigned int tot;
  const unsigned int e = block_excl_scan_1024((unsigned int)__popc(b), &tot);
  if (w < nwords) word_pair[w] = ((unsigned long long)e << 32) | b;
  if (threadIdx.x == 0) block_sum[blockIdx.x] = tot;
}

// exclusive scan of the bitmap's block totals in one workgroup (each thread a run of
// consecutive blocks, one block-wide scan); hdr[0] = G, host[0] = G, host[1] = hdr[1]
__global__ __launch_bounds__(1024) void k_block_scan_groups(unsigned int* block_sum, uint64_t nblocks,
                                                            const unsigned long long* rows_part, int nrp,
                                                            unsigned long long* hdr, unsigned long long* host) {
  // passing rows: the marking workgroups' counts (rows_part), or hdr[1] from the bitmap pass
  __shared__ unsigned long long rsum[16];
  unsigned long long rp = rows_part && (int)threadIdx.x < nrp ? rows_part[threadIdx.x] : 0ull;
  rp = wave_sum_u64(rp);
  if ((threadIdx.x & 63) == 0) rsum[threadIdx.x >> 6] = rp;
  const uint64_t per = (nblocks + 1023) / 1024;
  const uint64_t b0 = (uint64_t)threadIdx.x * per, b1 = min(b0 + per, nblocks);
  unsigned int s = 0;
  for (uint64_t i = b0; i < b1; ++i) s += block_sum[i];
  unsigned int tot;
  unsigned int e = block_excl_scan_1024(s, &tot);
  for (uint64_t i = b0; i < b1; ++i) {
    const unsigned int c = block_sum[i];
    block_sum[i] = e;
    e += c;
  }
  if (threadIdx.x == 0) {
    unsigned long long rows = 0;
    for (int q = 0; q < 16; ++q) rows += rsum[q];
    if (rows_part) hdr[1] = rows;
    else rows = hdr[1];
    hdr[0] = tot;
    host[0] = tot;
    host[1] = rows;
  }
}

// per bitmap word: its exclusive popcount prefix within its 1024-word block (high half) and
// the word itself (low half) -- the emit's rank is then one 8-byte read per group
__global__ __launch_bounds__(1024) void k_word_scan_pairs(const unsigned int* bitmap, uint64_t nwords,
                                                          unsigned long long* word_pair, unsigned int* block_sum) {
  const uint64_t w = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  const unsigned int b = w < nwords ? bitmap[w] : 0u;
  unsigned int tot;
  const unsigned int e = block_excl_scan_1024((unsigned int)__popc(b), &tot);
  if (w < nwords) word_pair[w] = ((unsigned long long)e << 32) | b;
  if (threadIdx.x == 0) block_sum[blockIdx.x] = tot;
}

// The emit with the columns outermost: K slots per thread (slot = block base + k * 256 + tid,
// coalesced per k), their counts, first rows, rank words and keys loaded together, then per
// output column -- its descriptor read once for the K slots, the K values computed (their
// loads issued together), then stored.  (Per slot, each column's descriptor fields are a chain
// of dependent scalar loads: the one-slot emit spent ~2/3 of its wave cycles waiting and took
// 54-56 us at C3.)
// The stores at random ranks are ~3/4 of the pass (C3: 52.6 us; 13.8 without them, 20.9 with
// them in slot order) and are bound by their number, not their lines: REC (option slot_emit 2)
// writes each group's values into its record (ncols 8-byte words at rec + rank * ncols, one
// line or two) and k_aos_columns the columns in rank order -- 59 + 12.9 us, slower.
template <int K, bool REC>
__global__ __launch_bounds__(256) void k_rank_emit_cols(EmitParams e, SlotArrays sa, uint64_t nslots,
                                                        const unsigned long long* word_pair,
                                                        const unsigned int* block_prefix, const unsigned long long* hdr,
                                                        unsigned char* out) {
  const uint64_t G = hdr[0];
  for (uint64_t base = (uint64_t)blockIdx.x * 256 * K; base < nslots; base += (uint64_t)gridDim.x * 256 * K) {
    uint64_t s[K], code[K];
    unsigned long long n[K];
    uint32_t f[K];
    unsigned int r[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      s[k] = base + (uint64_t)k * 256 + threadIdx.x;
      n[k] = s[k] < nslots ? sa.cnt[s[k]] : 0ull;
      f[k] = s[k] < nslots ? sa.fst[s[k]] : 0u;
      code[k] = (e.hash && n[k]) ? (uint64_t)sa.keys[s[k]] : s[k];
    }
    unsigned long long pw[K];
    unsigned int bp[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t w = f[k] >> 5;
      pw[k] = n[k] ? word_pair[w] : 0ull;
      bp[k] = n[k] ? block_prefix[w >> 10] : 0u;
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
      r[k] = bp[k] + (unsigned int)(pw[k] >> 32) + (unsigned int)__popc((unsigned int)pw[k] & ((1u << (f[k] & 31)) - 1u));
    size_t goff = 0;
    for (int j = 0; j < e.ncols; ++j) {
      const EmitCol c = e.cols[j];
      uint64_t bits[K];
#pragma unroll
      for (int k = 0; k < K; ++k)
        bits[k] = n[k] ? column_bits(e, c, s[k], code[k], r[k], slot_ref(sa, s[k], nslots, n[k], f[k])) : 0ull;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (!n[k]) continue;
        if (REC) reinterpret_cast<unsigned long long*>(out)[(size_t)r[k] * e.ncols + j] = bits[k];
        else store_elem(out + goff, c.out_dtype, r[k], bits[k]);
      }
      goff += (((size_t)G << dtype_lg(c.out_dtype)) + 255) & ~size_t(255);
    }
  }
}

// the group records (emit_slot OUT 2) -> the output columns, in rank order: reads and writes
// coalesced; column j at out + the 256-byte aligned sizes of columns 0..j-1 at G rows
__global__ void k_aos_columns(EmitParams e, const unsigned long long* rec, unsigned char* out,
                              const unsigned long long* hdr) {
  const uint64_t G = hdr[0];
  const int nc = e.ncols;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < G; r += (uint64_t)gridDim.x * blockDim.x) {
    size_t off = 0;
    for (int j = 0; j < nc; ++j) {
      const int dt = e.cols[j].out_dtype;
      store_elem(out + off, dt, r, rec[r * nc + j]);
      off += (((size_t)G << dtype_lg(dt)) + 255) & ~size_t(255);
    }
  }
}

// Small slot spaces (<= kSmallEmitSlots): compaction, first-appearance ordering and emit in
// one workgroup, with the group count and passing rows written to hdr[0], hdr[1] -- no host
// round trip between the compaction and the emit.  Up to 1024 groups are ranked by counting
// (each thread compares its group's first row with every other one, LDS broadcast reads);
// more are bitonic-sorted in LDS.
__global__ __launch_bounds__(1024) void k_emit_small(EmitParams e, SlotArrays sa, uint32_t nslots, int nsum,
                                                     unsigned long long* hdr) {
  __shared__ uint32_t kf[kSmallEmitSlots];
  __shared__ uint32_t ks[kSmallEmitSlots];
  __shared__ unsigned int wsum[16];
  __shared__ unsigned long long wrows[16];
  constexpr int kPer = kSmallEmitSlots / 1024;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t occ = 0;
  unsigned long long rows = 0;
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint32_t s = threadIdx.x * kPer + r;
    const unsigned long long n = s < nslots ? sa.cnt[s] : 0ull;
    occ |= (n > 0 ? 1u : 0u) << r;
    rows += n;
  }
  const unsigned int v = (unsigned int)__popc(occ);
  unsigned int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned int t = (unsigned int)__shfl_up((int)incl, o, 64);
    if (lane >= o) incl += t;
  }
  const unsigned long long rw = wave_sum_u64(rows);
  if (lane == 63) wsum[wave] = incl;
  if (lane == 0) wrows[wave] = rw;
  __syncthreads();
  unsigned int before = 0, G = 0;
  unsigned long long total = 0;
  for (int q = 0; q < 16; ++q) {
    before += q < wave ? wsum[q] : 0u;
    G += wsum[q];
    total += wrows[q];
  }
  unsigned int pos = before + incl - v;
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    if (occ & (1u << r)) {
      const uint32_t s = threadIdx.x * kPer + r;
      kf[pos] = sa.fst[s];
      ks[pos] = s;
      ++pos;
    }
  }
  if (threadIdx.x == 0) {
    hdr[0] = G;
    hdr[1] = total;
  }
  auto emit_one = [&](uint32_t s, unsigned int row) {
    const SlotRef t = slot_ref(sa, s, nslots, sa.cnt[s], sa.fst[s]);
    const uint64_t code = e.hash ? (uint64_t)sa.keys[s] : (uint64_t)s;
    emit_slot(e, s, code, row, t);
  };
  if (G <= 1024) {
    // the first rows of distinct groups are distinct: rank = groups whose first row is earlier
    __syncthreads();
    uint32_t f = kNoRow, s = 0;
    if (threadIdx.x < G) {
      f = kf[threadIdx.x];
      s = ks[threadIdx.x];
    }
    unsigned int rank = 0;
    for (unsigned int j = 0; j < G; ++j) rank += kf[j] < f ? 1u : 0u;
    // (outputs in pinned host memory are read after hipStreamSynchronize: no system fence)
    if (threadIdx.x < G) emit_one(s, rank);
    return;
  }
  unsigned int m = 1;
  while (m < G) m <<= 1;
  for (unsigned int i = G + threadIdx.x; i < m; i += blockDim.x) kf[i] = kNoRow;
  __syncthreads();
  for (unsigned int k = 2; k <= m; k <<= 1) {
    for (unsigned int j = k >> 1; j > 0; j >>= 1) {
      for (unsigned int i = threadIdx.x; i < m; i += blockDim.x) {
        const unsigned int ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const uint32_t a = kf[i], b = kf[ixj];
          if ((a > b) == up) {
            kf[i] = b; kf[ixj] = a;
            const uint32_t t = ks[i]; ks[i] = ks[ixj]; ks[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  for (unsigned int i = threadIdx.x; i < G; i += blockDim.x) emit_one(ks[i], i);
}

// ------------------------------------------------------------------------------------
// Column statistics: order-preserving 64-bit keys, min/max by atomics
// ------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long ord_key_i(int64_t x) { return (unsigned long long)x ^ 0x8000000000000000ull; }
__device__ __forceinline__ unsigned long long ord_key_f(double d) {
  const unsigned long long u = as_u64(d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

// out[0] / out[1]: min / max order key; out[2]: NaN seen; float columns also get the facts
// that decide an exact 32-bit code for partitioned sums (api.hip, narrow entries):
// out[3]: min over non-zero values of (exponent of the lowest set mantissa bit + 4096), so
// every value is an integer multiple of 2^(out[3] - 4096); out[4]: bit 0 -- some value is
// subnormal or infinite (no dyadic code), bit 1 -- some value is not a whole number of
// hundredths (rint(v * 100) / 100 != v, or |v * 100| > 2^53: no cents code).  The code's
// width bounds (32-bit codes, or int64 sums that cannot overflow) are the host's.
// Four 4-row chunks per thread in flight (every load of a round issued before the first is
// used; rows past the end re-read the last chunk and are masked off): one chunk at a time left
// the pass latency-bound at ~2.3 TB/s (r4 trace: 0.17 ms per 400 MB column).
constexpr int kStatsAhead = 4;

// A 4-row chunk of a column of compile-time width (no branch between its loads: a runtime
// width split the loads and drained vmcnt at the join)
template <int DT>
__device__ __forceinline__ void load_chunk_dt(Chunk& c, const unsigned char* ptr, int64_t row0) {
  constexpr int LG = DT == BQG_BOOL || DT == BQG_I8 || DT == BQG_U8 ? 0
                     : DT == BQG_I16 || DT == BQG_U16              ? 1
                     : DT == BQG_I32 || DT == BQG_U32 || DT == BQG_F32 ? 2 : 3;
  const int64_t off = row0 << LG;
  const unsigned char* p = ptr + (off & ~int64_t(15));
  c.a = load_stream16(p);
  if (LG == 3) c.b = load_stream16(p + 16);
  c.sh = (uint32_t)(off & 15) >> 2;
}

template <int DT>
__global__ __launch_bounds__(kBlock) void k_stats(DevCol c, int64_t nrows, unsigned long long* partial) {
  unsigned long long mn = ~0ull, mx = 0ull, nan = 0ull, lsb = ~0ull, enc = 0ull;
  // floats: the largest finite magnitude (its bits: nonnegative doubles order as their bits)
  // and flags (bit 0: a subnormal value)
  unsigned long long fab = 0ull, flg = 0ull;
  constexpr bool isf = DT == BQG_F32 || DT == BQG_F64;
  constexpr bool u64 = DT == BQG_U64;
  const int64_t stride = (int64_t)gridDim.x * kBlock * 4;
  const int64_t last = (nrows - 1) & ~(int64_t)3;
  for (int64_t r0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4; r0 < nrows; r0 += stride * kStatsAhead) {
    Chunk ch[kStatsAhead];
#pragma unroll
    for (int a = 0; a < kStatsAhead; ++a) {
      const int64_t row0 = r0 + a * stride;
      load_chunk_dt<DT>(ch[a], c.ptr, row0 < nrows ? row0 : last);
    }
#pragma unroll
    for (int a = 0; a < kStatsAhead; ++a) {
      const int64_t row0 = r0 + a * stride;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (row0 + r >= nrows) break;
        unsigned long long k;
        if (isf) {
          const double d = chunk_f64(ch[a], DT, r);
          if (d != d) { nan = 1; continue; }
          k = ord_key_f(d + 0.0);
          const unsigned long long b = (unsigned long long)__double_as_longlong(d);
          const unsigned int ex = (unsigned int)(b >> 52) & 0x7FFu;
          // -0.0 codes as 0: bquery's sum starts at +0.0 and +0.0 + -0.0 == +0.0, so a sum
          // never keeps the sign of a zero either way
          const bool zero = (b << 1) == 0ull;
          if (ex != 0x7FFu) fab = max(fab, b & 0x7FFFFFFFFFFFFFFFull);
          if (ex == 0u && !zero) flg |= 1ull;
          if (ex == 0x7FFu || (ex == 0u && !zero)) {
            enc |= 1ull;
          } else if (!zero) {
            const unsigned long long m = (b & 0xFFFFFFFFFFFFFull) | 0x10000000000000ull;
            lsb = min(lsb, (unsigned long long)((int)ex - 1075 + __builtin_ctzll(m) + 4096));
          }
          // (the cents test divides: skipped once this lane has seen a value that is not
          // whole hundredths)
          if (!(enc & 2ull)) {
            const double n = rint(d * 100.0);
            if (n / 100.0 != d || fabs(n) > 9007199254740992.0) enc |= 2ull;
          }
        } else if (u64) {
          k = (unsigned long long)chunk_i64(ch[a], DT, r);
        } else {
          k = ord_key_i(chunk_i64(ch[a], DT, r));
        }
        mn = min(mn, k);
        mx = max(mx, k);
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    mn = min(mn, (unsigned long long)__shfl_xor(mn, o, 64));
    mx = max(mx, (unsigned long long)__shfl_xor(mx, o, 64));
    nan |= (unsigned long long)__shfl_xor(nan, o, 64);
    lsb = min(lsb, (unsigned long long)__shfl_xor(lsb, o, 64));
    enc |= (unsigned long long)__shfl_xor(enc, o, 64);
    fab = max(fab, (unsigned long long)__shfl_xor(fab, o, 64));
    flg |= (unsigned long long)__shfl_xor(flg, o, 64);
  }
  __shared__ unsigned long long smn[kBlock / 64], smx[kBlock / 64], snan[kBlock / 64], slsb[kBlock / 64], senc[kBlock / 64],
      sfab[kBlock / 64], sflg[kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    smn[threadIdx.x >> 6] = mn;
    smx[threadIdx.x >> 6] = mx;
    snan[threadIdx.x >> 6] = nan;
    slsb[threadIdx.x >> 6] = lsb;
    senc[threadIdx.x >> 6] = enc;
    sfab[threadIdx.x >> 6] = fab;
    sflg[threadIdx.x >> 6] = flg;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < kBlock / 64; ++q) {
      mn = min(mn, smn[q]);
      mx = max(mx, smx[q]);
      nan |= snan[q];
      lsb = min(lsb, slsb[q]);
      enc |= senc[q];
      fab = max(fab, sfab[q]);
      flg |= sflg[q];
    }
    // the block's partial (k_stats_final reduces them: ~1000 blocks' same-address device
    // atomics on these words serialised at the memory side, 25 us and more per column)
    unsigned long long* o = partial + (size_t)blockIdx.x * kStatsWords;
    o[0] = mn;
    o[1] = mx;
    o[2] = nan;
    o[3] = lsb;
    o[4] = enc;
    o[5] = fab;
    o[6] = flg;
  }
}

__global__ __launch_bounds__(kBlock) void k_stats_final(const unsigned long long* partial, int blocks,
                                                        unsigned long long* out) {
  unsigned long long mn = ~0ull, mx = 0ull, nan = 0ull, lsb = ~0ull, enc = 0ull, fab = 0ull, flg = 0ull;
  for (int b = threadIdx.x; b < blocks; b += kBlock) {
    const unsigned long long* o = partial + (size_t)b * kStatsWords;
    mn = min(mn, o[0]);
    mx = max(mx, o[1]);
    nan |= o[2];
    lsb = min(lsb, o[3]);
    enc |= o[4];
    fab = max(fab, o[5]);
    flg |= o[6];
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    mn = min(mn, (unsigned long long)__shfl_xor(mn, o, 64));
    mx = max(mx, (unsigned long long)__shfl_xor(mx, o, 64));
    nan |= (unsigned long long)__shfl_xor(nan, o, 64);
    lsb = min(lsb, (unsigned long long)__shfl_xor(lsb, o, 64));
    enc |= (unsigned long long)__shfl_xor(enc, o, 64);
    fab = max(fab, (unsigned long long)__shfl_xor(fab, o, 64));
    flg |= (unsigned long long)__shfl_xor(flg, o, 64);
  }
  __shared__ unsigned long long s[kStatsWords][kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    s[0][threadIdx.x >> 6] = mn;
    s[1][threadIdx.x >> 6] = mx;
    s[2][threadIdx.x >> 6] = nan;
    s[3][threadIdx.x >> 6] = lsb;
    s[4][threadIdx.x >> 6] = enc;
    s[5][threadIdx.x >> 6] = fab;
    s[6][threadIdx.x >> 6] = flg;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < kBlock / 64; ++q) {
      mn = min(mn, s[0][q]);
      mx = max(mx, s[1][q]);
      nan |= s[2][q];
      lsb = min(lsb, s[3][q]);
      enc |= s[4][q];
      fab = max(fab, s[5][q]);
      flg |= s[6][q];
    }
    out[0] = min(out[0], mn);
    out[1] = max(out[1], mx);
    out[2] |= nan ? 1ull : 0ull;
    out[3] = min(out[3], lsb);
    out[4] |= enc;
    out[5] = max(out[5], fab);
    out[6] |= flg;
  }
}

// ------------------------------------------------------------------------------------
// where_terms -> uint8 mask (worker.py:303), counting passing rows
// ------------------------------------------------------------------------------------
template <int NC>
__global__ __launch_bounds__(kBlock) void k_where(ScanParams p, unsigned char* out, unsigned long long* npass) {
  unsigned long long cnt = 0;
  const int64_t ntiles = (p.nrows + kTileRows - 1) / kTileRows;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t row0 = tile * kTileRows + (int64_t)threadIdx.x * kRowsPerThread;
    if (row0 >= p.nrows) continue;
    Chunk raw[NC];
    load_rows4<NC>(p, row0, raw);
    uint64_t v[NC][4];
    decode_all<NC, 4>(p, raw, v);
    const uint32_t pass = vals_pass<NC, 4>(p, row0, v);
    const uint32_t bytes = (pass & 1u) | ((pass & 2u) << 7) | ((pass & 4u) << 14) | ((pass & 8u) << 21);
    *reinterpret_cast<uint32_t*>(out + row0) = bytes;  // mask buffer is padded
    cnt += (unsigned long long)__popc(pass);
  }
  cnt = wave_sum_u64(cnt);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(npass, cnt);
}

// ------------------------------------------------------------------------------------
// Tile scans for selection and basket expansion (tiles of 1024 rows, 4 per lane)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned int block_excl_scan(unsigned int v, unsigned int* total) {
  __shared__ unsigned int sh[kBlock];
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int o = 1; o < kBlock; o <<= 1) {
    const unsigned int t = threadIdx.x >= (unsigned)o ? sh[threadIdx.x - o] : 0u;
    __syncthreads();
    sh[threadIdx.x] += t;
    __syncthreads();
  }
  const unsigned int incl = sh[threadIdx.x];
  if (total) *total = sh[kBlock - 1];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(kBlock) void k_select_count(const unsigned char* mask, int64_t nrows,
                                                         unsigned int* tile_counts) {
  const int64_t row0 = (int64_t)blockIdx.x * kTileRows + threadIdx.x * 4;
  unsigned int c = 0;
  if (row0 < nrows) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(mask + row0);
#pragma unroll
    for (int r = 0; r < 4; ++r) c += (row0 + r < nrows && ((w >> (8 * r)) & 0xFF)) ? 1u : 0u;
  }
  c = (unsigned int)wave_sum_u64(c);
  __shared__ unsigned int sw[kBlock / 64];
  if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = sw[0] + sw[1] + sw[2] + sw[3];
}

struct GatherCols {
  DevCol cols[kMaxKeys + kMaxAggs];
  void* outs[kMaxKeys + kMaxAggs];
  int ncols;
};

__global__ __launch_bounds__(kBlock) void k_select_gather(const unsigned char* mask, int64_t nrows,
                                                          const unsigned int* tile_offsets, GatherCols g) {
  const int64_t row0 = (int64_t)blockIdx.x * kTileRows + threadIdx.x * 4;
  uint32_t pass = 0;
  if (row0 < nrows) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(mask + row0);
#pragma unroll
    for (int r = 0; r < 4; ++r) pass |= (row0 + r < nrows && ((w >> (8 * r)) & 0xFF)) ? (1u << r) : 0u;
  }
  const unsigned int off = tile_offsets[blockIdx.x] + block_excl_scan((unsigned int)__popc(pass), nullptr);
  unsigned int k = 0;
  for (int r = 0; r < 4; ++r) {
    if (!(pass & (1u << r))) continue;
    const int64_t row = row0 + r;
    for (int c = 0; c < g.ncols; ++c) {
      const DevCol& col = g.cols[c];
      switch (col.lg) {
        case 0: reinterpret_cast<uint8_t*>(g.outs[c])[off + k] = col.ptr[row]; break;
        case 1: reinterpret_cast<uint16_t*>(g.outs[c])[off + k] = reinterpret_cast<const uint16_t*>(col.ptr)[row]; break;
        case 2: reinterpret_cast<uint32_t*>(g.outs[c])[off + k] = reinterpret_cast<const uint32_t*>(col.ptr)[row]; break;
        default: reinterpret_cast<unsigned long long*>(g.outs[c])[off + k] = reinterpret_cast<const unsigned long long*>(col.ptr)[row]; break;
      }
    }
    ++k;
  }
}

// basket runs: boundary where basket[i] != basket[i-1]; run id = inclusive boundary count - 1
__device__ __forceinline__ bool basket_differs(const Chunk& a, int ra, const Chunk& b, int rb, int dt) {
  if (dtype_is_float(dt)) return chunk_f64(a, dt, ra) != chunk_f64(b, dt, rb);
  return chunk_i64(a, dt, ra) != chunk_i64(b, dt, rb);
}

__device__ __forceinline__ uint32_t run_starts(const DevCol& b, int64_t row0, int64_t nrows) {
  Chunk cur, pc;
  load_chunk(cur, b, row0);
  if (row0 > 0) load_one(pc, b, row0 - 1);
  uint32_t st = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (row0 + r >= nrows) break;
    bool start;
    if (r == 0) start = (row0 == 0) || basket_differs(cur, 0, pc, 0, b.dtype);
    else start = basket_differs(cur, r, cur, r - 1, b.dtype);
    if (start) st |= 1u << r;
  }
  return st;
}

__global__ __launch_bounds__(kBlock) void k_runs_count(DevCol b, int64_t nrows, unsigned int* tile_counts) {
  const int64_t row0 = (int64_t)blockIdx.x * kTileRows + threadIdx.x * 4;
  const unsigned int c = row0 < nrows ? (unsigned int)__popc(run_starts(b, row0, nrows)) : 0u;
  unsigned int total;
  block_excl_scan(c, &total);
  if (threadIdx.x == 0) tile_counts[blockIdx.x] = total;
}

template <bool APPLY>
__global__ __launch_bounds__(kBlock) void k_runs_mark(DevCol b, int64_t nrows, const unsigned int* tile_offsets,
                                                      const unsigned char* mask, unsigned char* out,
                                                      unsigned char* run_any) {
  const int64_t row0 = (int64_t)blockIdx.x * kTileRows + threadIdx.x * 4;
  const uint32_t st = row0 < nrows ? run_starts(b, row0, nrows) : 0u;
  const unsigned int before = tile_offsets[blockIdx.x] + block_excl_scan((unsigned int)__popc(st), nullptr);
  if (row0 >= nrows) return;
  unsigned int id = before;  // inclusive count of starts up to row r, minus one
  for (int r = 0; r < 4; ++r) {
    const int64_t row = row0 + r;
    if (row >= nrows) break;
    if (st & (1u << r)) ++id;
    const unsigned int run = id - 1;
    if (!APPLY) {
      if (mask[row]) run_any[run] = 1;
    } else {
      out[row] = run_any[run];
    }
  }
}

void launch_compact(const SlotArrays& s, uint64_t nslots, uint32_t* list_fst, uint32_t* list_slot,
                    unsigned int* count, unsigned long long* total, uint32_t* scratch, hipStream_t st) {
  const uint64_t blocks = std::max<uint64_t>(1, (nslots + kCompactSlots - 1) / kCompactSlots);
  uint32_t* counts = scratch;  // [blocks + 1], scanned in place; counts[blocks] = groups
  hipLaunchKernelGGL(k_compact_count, dim3((unsigned)blocks), dim3(kCompactBlock), 0, st, s, nslots, counts, total);
  (void)hipMemsetAsync(counts + blocks, 0, 4, st);
  launch_exclusive_scan_u32(counts, blocks + 1, scratch + blocks + 1, st);
  hipLaunchKernelGGL(k_compact_write, dim3((unsigned)blocks), dim3(kCompactBlock), 0, st, s, nslots, counts, list_fst,
                     list_slot);
  (void)hipMemcpyAsync(count, counts + blocks, 4, hipMemcpyDeviceToDevice, st);
}
void launch_sort_small(uint32_t* list_fst, uint32_t* list_slot, unsigned int n, uint32_t* order, hipStream_t st) {
  hipLaunchKernelGGL(k_sort_small, dim3(1), dim3(1024), 0, st, list_fst, list_slot, n, order);
}
void launch_rank_bitmap(const uint32_t* list_fst, const uint32_t* list_slot, unsigned int n, int64_t nrows,
                        unsigned int* bitmap, unsigned int* word_prefix, unsigned int* block_prefix,
                        uint32_t* order, hipStream_t st) {
  const uint64_t nwords = ((uint64_t)nrows + 31) / 32;
  const uint64_t nblocks = (nwords + 1023) / 1024;
  (void)hipMemsetAsync(bitmap, 0, nwords * 4, st);
  const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_setbits, dim3(g ? g : 1), dim3(256), 0, st, list_fst, n, bitmap);
  hipLaunchKernelGGL(k_word_scan, dim3((unsigned)nblocks), dim3(1024), 0, st, bitmap, nwords, word_prefix, block_prefix);
  hipLaunchKernelGGL(k_block_scan, dim3(1), dim3(1024), 0, st, block_prefix, nblocks);
  hipLaunchKernelGGL(k_rank, dim3(g ? g : 1), dim3(256), 0, st, list_fst, list_slot, n, bitmap, word_prefix,
                     block_prefix, order);
}
void launch_rank_emit_bitmap(const EmitParams& e, const SlotArrays& s, const uint32_t* list_fst,
                             const uint32_t* list_slot, unsigned int n, int nsum, uint64_t nslots, int64_t nrows,
                             unsigned int* bitmap, unsigned int* word_prefix, unsigned int* block_prefix,
                             hipStream_t st) {
  const uint64_t nwords = ((uint64_t)nrows + 31) / 32;
  const uint64_t nblocks = (nwords + 1023) / 1024;
  (void)hipMemsetAsync(bitmap, 0, nwords * 4, st);
  const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_setbits, dim3(g ? g : 1), dim3(256), 0, st, list_fst, n, bitmap);
  hipLaunchKernelGGL(k_word_scan, dim3((unsigned)nblocks), dim3(1024), 0, st, bitmap, nwords, word_prefix, block_prefix);
  hipLaunchKernelGGL(k_block_scan, dim3(1), dim3(1024), 0, st, block_prefix, nblocks);
  hipLaunchKernelGGL(k_rank_emit, dim3(g ? g : 1), dim3(256), 0, st, e, s, list_fst, list_slot, n, nsum, nslots,
                     bitmap, word_prefix, block_prefix);
}
void launch_slot_emit(const EmitParams& e, const SlotArrays& s, uint64_t nslots, int64_t nrows,
                      unsigned int* bitmap, unsigned char* row_map, unsigned char epoch,
                      unsigned long long* word_pair, unsigned int* block_prefix,
                      unsigned long long* rows_part, unsigned long long* hdr,
                      unsigned long long* host_hdr, hipEvent_t ev_groups, unsigned char* out,
                      unsigned long long* rec, hipStream_t st) {
  const uint64_t nwords = ((uint64_t)nrows + 31) / 32;
  const uint64_t nblocks = (nwords + 1023) / 1024;
  const unsigned gs = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nslots + 1023) / 1024, 1024));
  if (row_map) {
    hipLaunchKernelGGL(k_mark_rows, dim3(gs), dim3(1024), 0, st, s, nslots, row_map, epoch, rows_part);
    if (nwords)
      hipLaunchKernelGGL(k_map_scan_pairs, dim3((unsigned)nblocks), dim3(1024), 0, st, row_map, nwords, epoch,
                         word_pair, block_prefix);
  } else {
    // hdr follows the bitmap: one fill zeroes both
    (void)hipMemsetAsync(bitmap, 0, (size_t)((char*)hdr - (char*)bitmap) + 16, st);
    hipLaunchKernelGGL(k_setbits_slots, dim3(gs), dim3(1024), 0, st, s, nslots, bitmap, hdr + 1);
    if (nwords)
      hipLaunchKernelGGL(k_word_scan_pairs, dim3((unsigned)nblocks), dim3(1024), 0, st, bitmap, nwords, word_pair,
                         block_prefix);
  }
  hipLaunchKernelGGL(k_block_scan_groups, dim3(1), dim3(1024), 0, st, block_prefix, nblocks,
                     (const unsigned long long*)(row_map ? rows_part : nullptr), (int)gs, hdr, host_hdr);
  (void)hipEventRecord(ev_groups, st);
  const unsigned gk = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nslots + 1023) / 1024, 4096));
  if (rec) {
    hipLaunchKernelGGL((k_rank_emit_cols<4, true>), dim3(gk), dim3(256), 0, st, e, s, nslots, word_pair, block_prefix,
                       hdr, (unsigned char*)rec);
    const unsigned ga = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nslots + 255) / 256, 4096));
    hipLaunchKernelGGL(k_aos_columns, dim3(ga), dim3(256), 0, st, e, rec, out, hdr);
  } else {
    hipLaunchKernelGGL((k_rank_emit_cols<4, false>), dim3(gk), dim3(256), 0, st, e, s, nslots, word_pair, block_prefix,
                       hdr, out);
  }
}
__global__ void k_column_copies(ColumnCopies cc) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (int j = 0; j < cc.n; ++j) {
    const uint64_t used = cc.used[j], units = cc.cap[j] / 16;
    uint4* d = reinterpret_cast<uint4*>(cc.dst[j]);
    const uint4* src = reinterpret_cast<const uint4*>(cc.src[j]);
    for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += stride) {
      const uint64_t b = u * 16;
      if (b + 16 <= used) {
        d[u] = src[u];
      } else if (b >= used) {
        d[u] = make_uint4(0u, 0u, 0u, 0u);
      } else {  // the unit holding the last rows: their bytes, then zeros (no read past them)
        unsigned char tmp[16];
        for (int k = 0; k < 16; ++k) tmp[k] = b + k < used ? cc.src[j][b + k] : (unsigned char)0;
        uint4 v;
        __builtin_memcpy(&v, tmp, 16);
        d[u] = v;
      }
    }
  }
}
void launch_column_copies(const ColumnCopies& cc, hipStream_t st) {
  uint64_t units = 0;
  for (int j = 0; j < cc.n; ++j) units = std::max<uint64_t>(units, cc.cap[j] / 16);
  const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((units + 255) / 256, 2048));
  hipLaunchKernelGGL(k_column_copies, dim3(g), dim3(256), 0, st, cc);
}
__global__ void k_zero_ranges(ZeroRanges z) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (int r = 0; r < z.n; ++r)
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < z.words[r]; i += stride) z.p[r][i] = 0u;
}
void launch_zero_ranges(const ZeroRanges& z, hipStream_t st) {
  uint64_t most = 1;
  for (int r = 0; r < z.n; ++r) most = std::max<uint64_t>(most, z.words[r]);
  const unsigned g = (unsigned)std::min<uint64_t>((most + 255) / 256, 1024);
  hipLaunchKernelGGL(k_zero_ranges, dim3(g), dim3(256), 0, st, z);
}
void launch_emit(const EmitParams& e, const SlotArrays& s, const uint32_t* order, unsigned int n, int nsum,
                 uint64_t nslots, hipStream_t st) {
  const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_emit, dim3(g ? g : 1), dim3(256), 0, st, e, s, order, n, nsum, nslots);
}
void launch_emit_small(const EmitParams& e, const SlotArrays& s, uint32_t nslots, int nsum, unsigned long long* hdr,
                       hipStream_t st) {
  hipLaunchKernelGGL(k_emit_small, dim3(1), dim3(1024), 0, st, e, s, nslots, nsum, hdr);
}
constexpr uint32_t kHashPartLds = 8192;
// ------------------------------------------------------------------------------------
// Hash partition of rows by their key VALUES (not codes: codes depend on per-shard
// statistics), for the cross-rank merge: partition = mix(canonical key bits) mod nparts.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t row_partition(const PartitionCols& k, int64_t row, uint32_t nparts) {
  return (uint32_t)(key_hash_row(k, row) % nparts);
}

__global__ __launch_bounds__(kBlock) void k_hash_partition(PartitionCols k, int64_t nrows, uint32_t nparts,
                                                           uint32_t* out, unsigned long long* counts) {
  // per-workgroup LDS histogram (a single hot partition -- world size 1 or skewed keys --
  // would otherwise serialize every row on one device atomic)
  extern __shared__ unsigned int hist[];
  const bool lds = nparts <= kHashPartLds;
  if (lds)
    for (uint32_t i = threadIdx.x; i < nparts; i += kBlock) hist[i] = 0;
  __syncthreads();
  for (int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x; row < nrows; row += (int64_t)gridDim.x * kBlock) {
    const uint32_t p = row_partition(k, row, nparts);
    out[row] = p;
    if (lds)
      atomicAdd(&hist[p], 1u);
    else
      atomicAdd(&counts[p], 1ull);
  }
  if (lds) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nparts; i += kBlock)
      if (hist[i]) atomicAdd(&counts[i], (unsigned long long)hist[i]);
  }
}

// ------------------------------------------------------------------------------------
// Cross-rank merge, send side: every row of a rank's reduced table goes straight into its
// destination rank's packed block (the block's columns one after another, each 16-byte
// aligned, rows in table order).  A stable counting partition in three launches: per-workgroup
// destination histograms (each row's destination kept as one byte), an exclusive scan over
// the workgroups per destination plus the block layout, then the ordered scatter.  It
// replaces one row-selection pass per destination and a copy per column and destination.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_mpack_hist(MergePack m) {
  __shared__ unsigned int hist[kMergeMaxRanks];
  for (int i = threadIdx.x; i < m.nranks; i += kBlock) hist[i] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * m.rows_per_block;
  const int64_t r1 = min(m.nrows, r0 + m.rows_per_block);
  for (int64_t row = r0 + threadIdx.x; row < r1; row += kBlock) {
    const uint32_t d = row_partition(m.keys, row, (uint32_t)m.nranks);
    m.dest[row] = (unsigned char)d;
    atomicAdd(&hist[d], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < m.nranks; i += kBlock) m.block_hist[(size_t)blockIdx.x * m.nranks + i] = hist[i];
}

__global__ __launch_bounds__(kBlock) void k_mpack_scan(MergePack m) {
  // thread (c, d): destination d over the c-th run of workgroups (kBlock / nranks runs)
  __shared__ unsigned int part[kBlock];
  __shared__ unsigned long long tot[kMergeMaxRanks];
  const int W = m.nranks;
  const int C = kBlock / W;
  const int per = (m.nblocks + C - 1) / C;
  const int d = threadIdx.x % W, c = threadIdx.x / W;
  const bool on = c < C;
  const int b0 = c * per, b1 = min(m.nblocks, (c + 1) * per);
  unsigned int s = 0;
  if (on)
    for (int b = b0; b < b1; ++b) s += m.block_hist[(size_t)b * W + d];
  part[threadIdx.x] = s;
  __syncthreads();
  if (on) {
    unsigned int run = 0;
    for (int c2 = 0; c2 < c; ++c2) run += part[c2 * W + d];
    if (c == C - 1) {
      tot[d] = run + s;
      m.to_peer[d] = run + s;
    }
    for (int b = b0; b < b1; ++b) {
      const size_t i = (size_t)b * W + d;
      const unsigned int v = m.block_hist[i];
      m.block_hist[i] = run;
      run += v;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long off = 0;
    for (int dd = 0; dd < W; ++dd)
      for (int j = 0; j < m.ncols; ++j) {
        m.colbase[dd * m.ncols + j] = off;
        off += ((tot[dd] << m.lg[j]) + 15) & ~15ull;
      }
  }
}

__global__ __launch_bounds__(kBlock) void k_mpack_scatter(MergePack m) {
  __shared__ unsigned int next[kMergeMaxRanks];               // next position of each destination
  __shared__ unsigned int wcnt[kBlock / 64][kMergeMaxRanks];  // rows per (wave, destination) of a step
  const int W = m.nranks;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < W; i += kBlock) next[i] = m.block_hist[(size_t)blockIdx.x * W + i];
  const int64_t r0 = (int64_t)blockIdx.x * m.rows_per_block;
  const int64_t r1 = min(m.nrows, r0 + m.rows_per_block);
  for (int64_t c0 = r0; c0 < r1; c0 += kBlock) {
    for (int i = threadIdx.x; i < (kBlock / 64) * W; i += kBlock) wcnt[i / W][i % W] = 0;
    __syncthreads();
    const int64_t row = c0 + threadIdx.x;
    const bool valid = row < r1;
    const uint32_t d = valid ? m.dest[row] : 0u;
    // rank among the wave's rows of the same destination: one ballot per distinct destination
    uint64_t todo = __ballot(valid);
    uint32_t rank = 0;
    while (todo) {
      const int leader = __ffsll((unsigned long long)todo) - 1;
      const uint32_t dd = (uint32_t)__shfl((int)d, leader);
      const uint64_t same = __ballot(valid && d == dd);
      if (valid && d == dd) rank = (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
      if (lane == leader) wcnt[wave][dd] = (unsigned int)__popcll(same);
      todo &= ~same;
    }
    __syncthreads();
    if (valid) {
      uint32_t pos = next[d] + rank;
      for (int w = 0; w < wave; ++w) pos += wcnt[w][d];
      const unsigned long long* cb = m.colbase + (size_t)d * m.ncols;
      for (int j = 0; j < m.ncols; ++j) {
        unsigned char* dst = m.send + cb[j];
        switch (m.lg[j]) {
          case 0: dst[pos] = m.cols[j][row]; break;
          case 1: ((uint16_t*)dst)[pos] = ((const uint16_t*)m.cols[j])[row]; break;
          case 2: ((uint32_t*)dst)[pos] = ((const uint32_t*)m.cols[j])[row]; break;
          default: ((uint64_t*)dst)[pos] = ((const uint64_t*)m.cols[j])[row]; break;
        }
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < W; i += kBlock) {
      unsigned int add = 0;
      for (int w = 0; w < kBlock / 64; ++w) add += wcnt[w][i];
      next[i] += add;
    }
    __syncthreads();
  }
}

// Compact resident copies (Column::shadow).  Integer source: its canonical value minus `off`,
// stored in 1 / 2 / 4 bytes; float64 source: the exact int32 code of every value (the column
// statistics guarantee one exists and the decode divides it back exactly).
// 16 rows per thread and round (four 4-row chunks loaded together, one 4 / 8 / 16-byte store
// of the narrow values per chunk): a row per thread kept a few KB in flight per CU and ran at
// ~2.3 TB/s (r4 trace: 0.18-0.22 ms per 100 M-row column).  Rows past the end are not written
// (the caller zeroes the copy's padding).
template <int DT>
__global__ __launch_bounds__(kBlock) void k_shadow(DevCol src, int64_t n, int kind, double mul, int64_t off,
                                                    unsigned char* dst, int dst_lg) {
  constexpr bool CODE = DT == BQG_F64;
  const int64_t stride = (int64_t)gridDim.x * kBlock * 4;
  const int64_t last = (n - 1) & ~(int64_t)3;
  for (int64_t r0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4; r0 < n; r0 += stride * 4) {
    Chunk ch[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int64_t row0 = r0 + a * stride;
      load_chunk_dt<DT>(ch[a], src.ptr, row0 < n ? row0 : last);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int64_t row0 = r0 + a * stride;
      if (row0 >= n) break;
      uint32_t u[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int64_t v;
        if (CODE) {
          const double d = chunk_f64(ch[a], BQG_F64, r) * mul;
          v = (int64_t)(kind == 1 ? d : rint(d));
          if (dst_lg != 2) v -= off;  // int32 codes are stored as they are
        } else {
          v = chunk_i64(ch[a], DT, r) - off;
        }
        u[r] = (uint32_t)v;
      }
      if (row0 + 4 <= n) {
        if (dst_lg == 0) {
          *reinterpret_cast<uint32_t*>(dst + row0) = (u[0] & 0xFFu) | (u[1] & 0xFFu) << 8 | (u[2] & 0xFFu) << 16 | u[3] << 24;
        } else if (dst_lg == 1) {
          *reinterpret_cast<uint2*>(dst + 2 * row0) = make_uint2((u[0] & 0xFFFFu) | u[1] << 16, (u[2] & 0xFFFFu) | u[3] << 16);
        } else {
          *reinterpret_cast<uint4*>(dst + 4 * row0) = make_uint4(u[0], u[1], u[2], u[3]);
        }
      } else {
        for (int r = 0; r < 4 && row0 + r < n; ++r) {
          if (dst_lg == 0) dst[row0 + r] = (uint8_t)u[r];
          else if (dst_lg == 1) reinterpret_cast<uint16_t*>(dst)[row0 + r] = (uint16_t)u[r];
          else reinterpret_cast<uint32_t*>(dst)[row0 + r] = u[r];
        }
      }
    }
  }
}

static unsigned shadow_grid(int64_t nrows) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((nrows + 4 * kBlock - 1) / (4 * kBlock), (int64_t)device_cu_count() * 8));
}

void launch_shadow_int(const DevCol& src, int64_t nrows, int64_t off, void* dst, int dst_lg, hipStream_t st) {
  if (nrows <= 0) return;
#define BQG_SHADOW(DTV) hipLaunchKernelGGL((k_shadow<DTV>), dim3(shadow_grid(nrows)), dim3(kBlock), 0, st, src, nrows, 0, 0.0, \
                                           off, (unsigned char*)dst, dst_lg)
  switch (src.dtype) {
    case BQG_I8: BQG_SHADOW(BQG_I8); break;
    case BQG_I16: BQG_SHADOW(BQG_I16); break;
    case BQG_I32: BQG_SHADOW(BQG_I32); break;
    case BQG_U8: BQG_SHADOW(BQG_U8); break;
    case BQG_U16: BQG_SHADOW(BQG_U16); break;
    case BQG_U32: BQG_SHADOW(BQG_U32); break;
    default: BQG_SHADOW(BQG_I64); break;  // (uint64 columns have no compact copy)
  }
#undef BQG_SHADOW
}

void launch_shadow_code(const double* src, int64_t nrows, int kind, double mul, int64_t off, void* dst, int dst_lg,
                        hipStream_t st) {
  if (nrows <= 0) return;
  const DevCol c{(const unsigned char*)src, BQG_F64, 3};
  hipLaunchKernelGGL(k_shadow<BQG_F64>, dim3(shadow_grid(nrows)), dim3(kBlock), 0, st, c, nrows, kind, mul, off,
                     (unsigned char*)dst, dst_lg);
}

// std pass 2 centers: the mean of every slot of every std column, from pass 1's count and sum
// (conv: 0 float bits, 1 signed, 2 unsigned integer sum), written where pass 2 reads them --
// no host round trip between the passes
__global__ __launch_bounds__(kBlock) void k_std_centers(const unsigned long long* cnt, const unsigned long long* acc,
                                                        StdCenters sc, uint64_t nslots, double* centers) {
  const uint64_t total = (uint64_t)sc.n * nslots;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += (uint64_t)gridDim.x * kBlock) {
    const int k = (int)(i / nslots);
    const uint64_t s = i - (uint64_t)k * nslots;
    const unsigned long long a = acc[(size_t)sc.state[k] * nslots + s];
    const double sum = sc.conv[k] == 0   ? as_f64(a)
                       : sc.conv[k] == 2 ? (double)a
                       : sc.conv[k] == 3 ? (double)(long long)a / sc.dec[k]
                                         : (double)(long long)a;
    const unsigned long long c = cnt[s];
    centers[i] = c ? sum / (double)c : 0.0;
  }
}

void launch_std_centers(const unsigned long long* cnt, const unsigned long long* acc, const StdCenters& sc,
                        uint64_t nslots, double* centers, hipStream_t st) {
  const uint64_t total = (uint64_t)sc.n * nslots;
  if (!total) return;
  const unsigned g = (unsigned)std::min<uint64_t>((total + kBlock - 1) / kBlock, 4096);
  hipLaunchKernelGGL(k_std_centers, dim3(g), dim3(kBlock), 0, st, cnt, acc, sc, nslots, centers);
}

void merge_pack_grid(int64_t nrows, int32_t* nblocks, int64_t* rows_per_block) {
  int64_t nb = std::max<int64_t>(1, std::min<int64_t>(256, (nrows + 4095) / 4096));
  int64_t rpb = (nrows + nb - 1) / nb;
  rpb = std::max<int64_t>(kBlock, (rpb + kBlock - 1) / kBlock * kBlock);
  nb = std::max<int64_t>(1, (nrows + rpb - 1) / rpb);
  *nblocks = (int32_t)nb;
  *rows_per_block = rpb;
}

void launch_merge_pack(const MergePack& m, hipStream_t st) {
  if (m.nrows > 0) hipLaunchKernelGGL(k_mpack_hist, dim3(m.nblocks), dim3(kBlock), 0, st, m);
  else (void)hipMemsetAsync(m.block_hist, 0, (size_t)m.nblocks * m.nranks * 4, st);
  hipLaunchKernelGGL(k_mpack_scan, dim3(1), dim3(kBlock), 0, st, m);
  if (m.nrows > 0) hipLaunchKernelGGL(k_mpack_scatter, dim3(m.nblocks), dim3(kBlock), 0, st, m);
}

// ------------------------------------------------------------------------------------
// Cross-rank merge, receive side (MergeReduce, kernels.h): the received rows summed by key.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mred_val(const unsigned char* col, int dt, int64_t row) {
  const DevCol c{col, dt, dtype_lg(dt)};
  Chunk ch;
  row_word_to_chunk(ch, c, row, load_row_word(c, row));
  uint64_t v[1];
  decode<1>(ch, dt, v);
  return v[0];
}

__device__ __forceinline__ bool mred_same_keys(const PartitionCols& k, int64_t a, int64_t b) {
  bool same = true;
  for (int j = 0; j < k.nkeys; ++j) {
    const bool f = dtype_is_float(k.cols[j].dtype);
    same &= key_at_row(k.cols[j], f, (uint32_t)a) == key_at_row(k.cols[j], f, (uint32_t)b);
  }
  return same;
}

// one source block [row0, row1): claim or find each row's slot and add its values to the
// slot's sums -- atomics on zero-initialised sums for tables that may repeat a key (a rank's
// input tables: a launch adds at most once per slot when they do not, so the sums come out in
// source order whatever the atomics' timing), plain stores and adds for sources known to hold
// each key once (the reduced partitions a rank receives).
__global__ __launch_bounds__(kBlock) void k_mred_insert(MergeReduce m) {
  for (int64_t row = m.row0 + (int64_t)blockIdx.x * kBlock + threadIdx.x; row < m.row1;
       row += (int64_t)gridDim.x * kBlock) {
    const uint64_t h = key_hash_row(m.keys, row);
    const uint32_t hi = (uint32_t)(h >> 32);
    // the table position from a second mix: the rows of one rank share h mod nranks
    uint64_t pos = mix64(h ^ 0x9E3779B97F4A7C15ull) & m.mask;
    bool fresh = false;  // this row claimed the slot: it represents the key
    uint64_t i = 0;
    for (; i <= m.mask; ++i) {
      unsigned long long w = m.table[pos];
      if (w == kEmpty) {
        const unsigned long long mine = ((unsigned long long)hi << 32) | (uint32_t)row;
        const unsigned long long prev = atomicCAS(&m.table[pos], kEmpty, mine);
        if (prev == kEmpty) {
          fresh = true;
          break;
        }
        w = prev;
      }
      if ((uint32_t)(w >> 32) == hi && mred_same_keys(m.keys, (int64_t)(uint32_t)w, row)) break;
      pos = (pos + 1) & m.mask;
    }
    if (i > m.mask) {
      atomicOr(m.overflow, 1u);
      continue;
    }
    if (fresh) atomicOr(&m.rep_bits[row >> 5], 1u << (row & 31));
    for (int j = 0; j < m.nvals; ++j) {
      const int dt = m.vdt[j];
      const uint64_t v = mred_val(m.vals[j], dt, row);
      unsigned long long* a = m.acc + (size_t)j * (m.mask + 1) + pos;
      if (m.unique_sources) {
        // no other row of this launch has this key: the first source stores, later ones add
        if (fresh) *a = v;
        else if (dtype_is_float(dt)) *a = as_u64(as_f64(*a) + as_f64(v));
        else *a += v;  // two's complement: wraps at the output width
      } else if (dtype_is_float(dt)) {
        atomicAdd(reinterpret_cast<double*>(a), as_f64(v));
      } else {
        atomicAdd(a, (unsigned long long)v);
      }
    }
  }
}

// Rank scan of a row bitmap (the merge reduce's representative rows, the byte encoder's first
// rows): exclusive popcount prefix per word inside blocks of 1024 words, block totals, then an
// exclusive scan of the block totals in one workgroup with the bit count in *total.
__global__ __launch_bounds__(1024) void k_rank_word_scan(const unsigned int* bits, uint64_t nwords,
                                                         unsigned int* word_prefix, unsigned int* block_sum) {
  const uint64_t w = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  const unsigned int c = w < nwords ? (unsigned int)__popc(bits[w]) : 0u;
  unsigned int tot;
  const unsigned int e = block_excl_scan_1024(c, &tot);
  if (w < nwords) word_prefix[w] = e;
  if (threadIdx.x == 0) block_sum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_rank_block_scan(unsigned int* block_sum, uint64_t nblocks,
                                                          unsigned long long* total) {
  __shared__ unsigned int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t base = 0; base < nblocks; base += 1024) {
    const uint64_t i = base + threadIdx.x;
    const unsigned int c = i < nblocks ? block_sum[i] : 0u;
    unsigned int tot;
    const unsigned int e = block_excl_scan_1024(c, &tot);
    if (i < nblocks) block_sum[i] = carry + e;
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

// number of set bits of the scanned bitmap before bit r
__device__ __forceinline__ uint64_t bit_rank(const unsigned int* bits, const unsigned int* word_prefix,
                                             const unsigned int* block_sum, uint32_t r) {
  const uint32_t wi = r >> 5;
  return (uint64_t)block_sum[wi >> 10] + word_prefix[wi] + (unsigned int)__popc(bits[wi] & ((1u << (r & 31)) - 1u));
}

static void launch_rank_scan(const unsigned int* bits, int64_t nrows, unsigned int* word_prefix, unsigned int* block_sum,
                             unsigned long long* total, hipStream_t st) {
  const uint64_t nwords = ((uint64_t)nrows + 31) / 32, nblocks = (nwords + 1023) / 1024;
  if (nwords) hipLaunchKernelGGL(k_rank_word_scan, dim3((unsigned)nblocks), dim3(1024), 0, st, bits, nwords, word_prefix, block_sum);
  hipLaunchKernelGGL(k_rank_block_scan, dim3(1), dim3(1024), 0, st, block_sum, nblocks, total);
}

// every occupied slot writes its output row at the rank of its representative row: keys as
// stored at that row, sums converted to the column's dtype (integers wrap, float32 rounds once)
__global__ __launch_bounds__(kBlock) void k_mred_emit(MergeReduce m) {
  const uint64_t cap = m.mask + 1;
  for (uint64_t pos = (uint64_t)blockIdx.x * kBlock + threadIdx.x; pos < cap; pos += (uint64_t)gridDim.x * kBlock) {
    const unsigned long long w = m.table[pos];
    if (w == kEmpty) continue;
    const uint32_t rep = (uint32_t)w;
    const uint64_t r = bit_rank(m.rep_bits, m.word_prefix, m.block_sum, rep);
    for (int k = 0; k < m.keys.nkeys; ++k) {
      const DevCol& c = m.keys.cols[k];
      switch (c.lg) {
        case 0: m.out_keys[k][r] = c.ptr[rep]; break;
        case 1: reinterpret_cast<uint16_t*>(m.out_keys[k])[r] = reinterpret_cast<const uint16_t*>(c.ptr)[rep]; break;
        case 2: reinterpret_cast<uint32_t*>(m.out_keys[k])[r] = reinterpret_cast<const uint32_t*>(c.ptr)[rep]; break;
        default: reinterpret_cast<uint64_t*>(m.out_keys[k])[r] = reinterpret_cast<const uint64_t*>(c.ptr)[rep]; break;
      }
    }
    for (int j = 0; j < m.nvals; ++j) {
      unsigned long long a = m.acc[(size_t)j * cap + pos];
      if (m.vdt[j] == BQG_F32) a = __float_as_uint((float)as_f64(a));
      store_elem(m.out_vals[j], m.vdt[j], r, a);
    }
  }
}

void launch_merge_reduce(MergeReduce m, const int64_t* src_off, int nsrc, hipStream_t st) {
  const uint64_t cap = m.mask + 1;
  const uint64_t nwords = ((uint64_t)m.nrows + 31) / 32;
  (void)hipMemsetAsync(m.table, 0xFF, cap * 8, st);
  if (!m.unique_sources) (void)hipMemsetAsync(m.acc, 0, cap * 8 * (size_t)std::max(1, m.nvals), st);
  (void)hipMemsetAsync(m.rep_bits, 0, nwords * 4 + 4, st);
  for (int s = 0; s < nsrc; ++s) {
    m.row0 = src_off[s];
    m.row1 = src_off[s + 1];
    if (m.row1 <= m.row0) continue;
    const unsigned g = (unsigned)std::min<int64_t>((m.row1 - m.row0 + kBlock - 1) / kBlock, 2048);
    hipLaunchKernelGGL(k_mred_insert, dim3(g), dim3(kBlock), 0, st, m);
  }
  launch_rank_scan(m.rep_bits, m.nrows, m.word_prefix, m.block_sum, m.groups, st);
  const unsigned ge = (unsigned)std::min<uint64_t>((cap + kBlock - 1) / kBlock, 4096);
  hipLaunchKernelGGL(k_mred_emit, dim3(ge), dim3(kBlock), 0, st, m);
}

// ------------------------------------------------------------------------------------
// Fixed-width byte strings (numpy 'S<n>' / 'U<n>', bqg_encode_bytes): dictionary codes in
// first-appearance order.  A row's value is its `width` bytes (trailing zero bytes are
// numpy's padding and take part like any other byte: equal strings have equal bytes).
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t bytes_word(const unsigned char* p, int avail) {
  uint64_t w = 0;
  for (int b = 0; b < 8 && b < avail; ++b) w |= (uint64_t)p[b] << (8 * b);
  return w;
}

__device__ __forceinline__ uint64_t bytes_hash(const unsigned char* p, int width) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)width;
  for (int i = 0; i < width; i += 8) h = mix64(h ^ (bytes_word(p + i, width - i) + (uint64_t)i));
  return h;
}

__device__ __forceinline__ bool bytes_equal(const unsigned char* a, const unsigned char* b, int width) {
  for (int i = 0; i < width; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

__global__ __launch_bounds__(kBlock) void k_bytes_insert(BytesEncode e) {
  for (int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x; row < e.n; row += (int64_t)gridDim.x * kBlock) {
    const unsigned char* mine = e.data + (size_t)row * e.width;
    const uint64_t h = bytes_hash(mine, e.width);
    const uint32_t hi = (uint32_t)(h >> 32);
    uint64_t pos = h & e.mask;
    uint64_t i = 0;
    for (; i <= e.mask; ++i) {
      unsigned long long w = e.table[pos];
      if (w == kEmpty) {
        const unsigned long long prev = atomicCAS(&e.table[pos], kEmpty, ((unsigned long long)hi << 32) | (uint32_t)row);
        if (prev == kEmpty) break;
        w = prev;
      }
      if ((uint32_t)(w >> 32) == hi && bytes_equal(e.data + (size_t)(uint32_t)w * e.width, mine, e.width)) break;
      pos = (pos + 1) & e.mask;
    }
    if (i > e.mask) {
      atomicOr(e.overflow, 1u);
      continue;
    }
    e.row_slot[row] = (uint32_t)pos;
    atomicMin(&e.first[pos], (uint32_t)row);
  }
}

// the first row of every value, as a bit of the row bitmap
__global__ __launch_bounds__(kBlock) void k_bytes_mark(BytesEncode e) {
  const uint64_t cap = e.mask + 1;
  for (uint64_t pos = (uint64_t)blockIdx.x * kBlock + threadIdx.x; pos < cap; pos += (uint64_t)gridDim.x * kBlock) {
    const uint32_t f = e.first[pos];
    if (f != 0xFFFFFFFFu) atomicOr(&e.rep_bits[f >> 5], 1u << (f & 31));
  }
}

// code = 1 + first-appearance rank (0 for the empty string: all zero bytes); first rows write
// their value into the dictionary at their rank
__global__ __launch_bounds__(kBlock) void k_bytes_codes(BytesEncode e) {
  for (int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x; row < e.n; row += (int64_t)gridDim.x * kBlock) {
    const unsigned char* mine = e.data + (size_t)row * e.width;
    const uint32_t f = e.first[e.row_slot[row]];
    const uint64_t r = bit_rank(e.rep_bits, e.word_prefix, e.block_sum, f);
    bool empty = true;
    for (int b = 0; b < e.width; ++b) empty &= mine[b] == 0;
    e.codes[row] = empty ? 0 : (int32_t)(r + 1);
    if ((int64_t)f == row)
      for (int b = 0; b < e.width; ++b) e.values[r * e.width + b] = mine[b];
  }
}

void launch_bytes_encode(BytesEncode e, hipStream_t st) {
  const uint64_t cap = e.mask + 1;
  (void)hipMemsetAsync(e.table, 0xFF, cap * 8, st);
  (void)hipMemsetAsync(e.first, 0xFF, cap * 4, st);
  (void)hipMemsetAsync(e.rep_bits, 0, ((uint64_t)e.n + 31) / 32 * 4 + 4, st);
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((e.n + kBlock - 1) / kBlock, 4096));
  hipLaunchKernelGGL(k_bytes_insert, dim3(g), dim3(kBlock), 0, st, e);
  const unsigned gm = (unsigned)std::min<uint64_t>((cap + kBlock - 1) / kBlock, 4096);
  hipLaunchKernelGGL(k_bytes_mark, dim3(gm), dim3(kBlock), 0, st, e);
  launch_rank_scan(e.rep_bits, e.n, e.word_prefix, e.block_sum, e.groups, st);
  hipLaunchKernelGGL(k_bytes_codes, dim3(g), dim3(kBlock), 0, st, e);
}

// value runs: rows whose value differs from the previous row's (canonical bits: a float
// column's -0.0 / +0.0 and NaN count as one value, like a group key)
__global__ __launch_bounds__(kBlock) void k_runs(DevCol c, int64_t nrows, unsigned long long* out) {
  unsigned long long n = 0;
  for (int64_t row = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kRowsPerThread; row < nrows;
       row += (int64_t)gridDim.x * kBlock * kRowsPerThread) {
    Chunk ch;
    load_chunk(ch, c, row);
    uint64_t v[4];
    decode<4>(ch, c.dtype, v);
    uint64_t prev = 0;
    if (row > 0) {
      Chunk pc;
      row_word_to_chunk(pc, c, row - 1, load_row_word(c, row - 1));
      uint64_t pv[1];
      decode<1>(pc, c.dtype, pv);
      prev = pv[0];
    }
    const bool isf = dtype_is_float(c.dtype);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint64_t x = isf ? canon_f64_bits(v[r]) : v[r];
      const uint64_t y = isf ? canon_f64_bits(prev) : prev;
      if (row + r < nrows && row + r > 0 && x != y) ++n;
      prev = v[r];
    }
  }
  n = wave_sum_u64(n);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(out, n);
}

void launch_runs(const DevCol& c, int64_t nrows, unsigned long long* out, hipStream_t st) {
  int64_t blocks = (nrows + kTileRows - 1) / kTileRows;
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, 2048));
  if (nrows > 0) hipLaunchKernelGGL(k_runs, dim3((unsigned)blocks), dim3(kBlock), 0, st, c, nrows, out);
}

void launch_stats(const DevCol& c, int64_t nrows, unsigned long long* out4, unsigned long long* scratch,
                  hipStream_t st) {  // out4: kStatsWords words; scratch: kStatsMaxBlocks x kStatsWords words
  int64_t blocks = (nrows + kTileRows - 1) / kTileRows;
  if (blocks > kStatsMaxBlocks) blocks = kStatsMaxBlocks;
  if (blocks < 1) blocks = 1;
#define BQG_STATS(DTV) hipLaunchKernelGGL((k_stats<DTV>), dim3((unsigned)blocks), dim3(kBlock), 0, st, c, nrows, scratch)
  switch (c.dtype) {
    case BQG_BOOL: BQG_STATS(BQG_BOOL); break;
    case BQG_I8: BQG_STATS(BQG_I8); break;
    case BQG_I16: BQG_STATS(BQG_I16); break;
    case BQG_I32: BQG_STATS(BQG_I32); break;
    case BQG_I64: BQG_STATS(BQG_I64); break;
    case BQG_U8: BQG_STATS(BQG_U8); break;
    case BQG_U16: BQG_STATS(BQG_U16); break;
    case BQG_U32: BQG_STATS(BQG_U32); break;
    case BQG_U64: BQG_STATS(BQG_U64); break;
    case BQG_F32: BQG_STATS(BQG_F32); break;
    default: BQG_STATS(BQG_F64); break;
  }
#undef BQG_STATS
  hipLaunchKernelGGL(k_stats_final, dim3(1), dim3(kBlock), 0, st, scratch, (int)blocks, out4);
}
void launch_where(const ScanParams& p, unsigned char* out_mask, unsigned long long* npass, int blocks, hipStream_t st) {
  BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_where<NC>), dim3(blocks), dim3(kBlock), 0, st, p, out_mask, npass));
}
void launch_select_count(const unsigned char* mask, int64_t nrows, unsigned int* tile_counts, hipStream_t st) {
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  if (tiles > 0) hipLaunchKernelGGL(k_select_count, dim3((unsigned)tiles), dim3(kBlock), 0, st, mask, nrows, tile_counts);
}
void launch_select_scan(unsigned int* tile_counts, int64_t ntiles, unsigned int* scratch, hipStream_t st) {
  if (ntiles > 0) launch_exclusive_scan_u32(tile_counts, (uint64_t)ntiles, scratch, st);
}
void launch_select_gather(const unsigned char* mask, int64_t nrows, const unsigned int* tile_offsets,
                          const DevCol* cols, int ncols, void* const* outs, hipStream_t st) {
  GatherCols g;
  g.ncols = ncols;
  for (int c = 0; c < ncols; ++c) {
    g.cols[c] = cols[c];
    g.outs[c] = outs[c];
  }
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  if (tiles > 0) hipLaunchKernelGGL(k_select_gather, dim3((unsigned)tiles), dim3(kBlock), 0, st, mask, nrows, tile_offsets, g);
}
void launch_expand_subgroups(const DevCol& basket, const unsigned char* mask, unsigned char* out, int64_t nrows,
                             int blocks, unsigned int* scratch, hipStream_t st) {
  (void)blocks;
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  if (tiles <= 0) return;
  unsigned int* tile_counts = scratch;
  unsigned int* scan_scratch = scratch + tiles + 1;
  const int64_t scan_words = 2 * (tiles / 1024 + 2) + 4096;
  unsigned char* run_any = reinterpret_cast<unsigned char*>(scan_scratch + scan_words);
  hipLaunchKernelGGL(k_runs_count, dim3((unsigned)tiles), dim3(kBlock), 0, st, basket, nrows, tile_counts);
  launch_exclusive_scan_u32(tile_counts, (uint64_t)tiles, scan_scratch, st);
  (void)hipMemsetAsync(run_any, 0, (size_t)nrows, st);
  hipLaunchKernelGGL((k_runs_mark<false>), dim3((unsigned)tiles), dim3(kBlock), 0, st, basket, nrows, tile_counts,
                     mask, out, run_any);
  hipLaunchKernelGGL((k_runs_mark<true>), dim3((unsigned)tiles), dim3(kBlock), 0, st, basket, nrows, tile_counts,
                     mask, out, run_any);
}

// ------------------------------------------------------------------------------------
// bquery's factor cache (auto_cache, worker.py:291): label of every row = first-appearance
// rank of its value.  `vals` holds the distinct values in label order (a groupby over the
// column); lut[v - vmin] = label, then one gather per row.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_factor_lut(DevCol vals, int64_t n, int64_t vmin, int32_t* lut) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    Chunk c;
    row_word_to_chunk(c, vals, i, load_row_word(vals, i));
    uint64_t v[1];
    decode<1>(c, vals.dtype, v);
    lut[v[0] - (uint64_t)vmin] = (int32_t)i;
  }
}

__global__ __launch_bounds__(kBlock) void k_factor_labels(DevCol col, int64_t n, int64_t vmin, const int32_t* lut,
                                                          long long* out) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    Chunk c;
    row_word_to_chunk(c, col, i, load_row_word(col, i));
    uint64_t v[1];
    decode<1>(c, col.dtype, v);
    out[i] = (long long)lut[v[0] - (uint64_t)vmin];
  }
}

// Factor caches of any key column -- floats (khash identity: -0.0 == +0.0, NaN == NaN, the
// canonical bits of the groupby's key), bools and integers spanning more than a lookup table
// allows: an open-addressing table from the distinct values' canonical bits to their labels
// (inserted without collisions between equal keys: the values are distinct), then one probe
// per row.  labs[] holds label + 1 (0 = empty slot).
__device__ __forceinline__ uint64_t factor_bits(const DevCol& c, int64_t i) {
  Chunk ch;
  row_word_to_chunk(ch, c, i, load_row_word(c, i));
  uint64_t v[1];
  decode<1>(ch, c.dtype, v);
  return dtype_is_float(c.dtype) ? canon_f64_bits(v[0]) : v[0];
}

__global__ __launch_bounds__(kBlock) void k_factor_hash_build(DevCol vals, int64_t n, uint64_t mask,
                                                              unsigned long long* keys, uint32_t* labs) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const uint64_t bits = factor_bits(vals, i);
    for (uint64_t h = mix64(bits) & mask;; h = (h + 1) & mask)
      if (atomicCAS(&labs[h], 0u, (uint32_t)(i + 1)) == 0u) {
        keys[h] = bits;
        break;
      }
  }
}

__global__ __launch_bounds__(kBlock) void k_factor_hash_labels(DevCol col, int64_t n, uint64_t mask,
                                                               const unsigned long long* keys, const uint32_t* labs,
                                                               long long* out) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const uint64_t bits = factor_bits(col, i);
    long long lab = -1;  // every row's value is among the distinct values: not reached
    for (uint64_t h = mix64(bits) & mask;; h = (h + 1) & mask) {
      const uint32_t l = labs[h];
      if (l == 0u) break;
      if (keys[h] == bits) {
        lab = (long long)l - 1;
        break;
      }
    }
    out[i] = lab;
  }
}

void launch_factor_hash_labels(const DevCol& vals, int64_t nvals, const DevCol& col, int64_t nrows, uint64_t cap,
                               unsigned long long* keys, uint32_t* labs, long long* out, hipStream_t st) {
  auto grid = [](int64_t n) {
    int64_t b = (n + kBlock - 1) / kBlock;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(b, 8192));
  };
  (void)hipMemsetAsync(labs, 0, cap * 4, st);
  if (nvals > 0) hipLaunchKernelGGL(k_factor_hash_build, dim3(grid(nvals)), dim3(kBlock), 0, st, vals, nvals, cap - 1, keys, labs);
  if (nrows > 0)
    hipLaunchKernelGGL(k_factor_hash_labels, dim3(grid(nrows)), dim3(kBlock), 0, st, col, nrows, cap - 1, keys, labs, out);
}

void launch_factor_labels(const DevCol& vals, int64_t nvals, const DevCol& col, int64_t nrows, int64_t vmin,
                          int32_t* lut, long long* out, hipStream_t st) {
  auto grid = [](int64_t n) {
    int64_t b = (n + kBlock - 1) / kBlock;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(b, 8192));
  };
  if (nvals > 0) hipLaunchKernelGGL(k_factor_lut, dim3(grid(nvals)), dim3(kBlock), 0, st, vals, nvals, vmin, lut);
  if (nrows > 0) hipLaunchKernelGGL(k_factor_labels, dim3(grid(nrows)), dim3(kBlock), 0, st, col, nrows, vmin, lut, out);
}

int device_cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 256;
  return n;
}


void launch_hash_partition(const PartitionCols& k, int64_t nrows, uint32_t nparts, uint32_t* out,
                           unsigned long long* counts, hipStream_t st) {
  int64_t blocks = (nrows + kBlock - 1) / kBlock;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  const size_t lds = nparts <= kHashPartLds ? (size_t)nparts * 4 : 0;
  hipLaunchKernelGGL(k_hash_partition, dim3((unsigned)blocks), dim3(kBlock), lds, st, k, nrows, nparts, out, counts);
}

}  // namespace bqg
