// device.h -- device-side building blocks shared by the libbqgpu kernel translation units.
//
// Row prologue ("decode once"): every column of a 4-row chunk is loaded with one vector
// load, then decoded ONCE into canonical 64-bit values -- two's-complement int64 for integer
// and bool columns, the raw bits for uint64, IEEE double bits for float32/float64.  Terms,
// key coding and aggregation then work on those values without further dtype dispatch.
#pragma once

#include "kernels.h"

namespace bqg {

// Loops over a query's terms / keys: in a query-specialised (JIT) build the bound is the
// array size and the loop unrolls, so every ScanParams access has a constant index and the
// specialised parameter copy stays in registers (a dynamic index would put the whole struct
// in scratch memory and re-read it after every workgroup barrier).
#ifdef BQ_NC
#define BQ_LOOP_BOUND(n, maxn) (maxn)
#else
#define BQ_LOOP_BOUND(n, maxn) (n)
#endif

// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup-scope fence on all
// address spaces: it waits for every outstanding global load and store (vmcnt(0)), which
// drains a tile's prefetched loads and streaming stores at each barrier.  Kernels whose
// workgroups exchange data through LDS only use this instead (s_waitcnt lgkmcnt(0) +
// s_barrier).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ------------------------------------------------------------------------------------
// wave64 reductions (fixed butterfly order: bitwise deterministic)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

__device__ __forceinline__ double as_f64(unsigned long long u) { return __longlong_as_double((long long)u); }
__device__ __forceinline__ unsigned long long as_u64(double d) { return (unsigned long long)__double_as_longlong(d); }

// canonical identity of a double (khash equality: NaN == NaN, -0.0 == +0.0)
__device__ __forceinline__ uint64_t canon_f64_bits(uint64_t bits) {
  const double d = as_f64(bits);
  if (d != d) return 0x7ff8000000000000ull;
  return as_u64(d + 0.0);
}

// ------------------------------------------------------------------------------------
// loads and decode
// ------------------------------------------------------------------------------------
template <int NC>
__device__ __forceinline__ void load_rows4(const ScanParams& p, int64_t row0, Chunk (&raw)[NC]) {
#pragma unroll
  for (int c = 0; c < NC; ++c) load_chunk(raw[c], p.cols[c], row0);
}

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

__device__ __forceinline__ void load_one(Chunk& c, const DevCol& col, int64_t row) {
  c.sh = 0;
  switch (col.lg) {
    case 0: c.a.x = col.ptr[row]; break;
    case 1: c.a.x = reinterpret_cast<const uint16_t*>(col.ptr)[row]; break;
    case 2: c.a.x = reinterpret_cast<const uint32_t*>(col.ptr)[row]; break;
    default: {
      const uint2 t = reinterpret_cast<const uint2*>(col.ptr)[row];
      c.a.x = t.x;
      c.a.y = t.y;
    }
  }
}

// Branch-free single-row load: the aligned 8-byte word holding the row (any width <= 8; the
// column allocations are padded, so the word never leaves the buffer).
__device__ __forceinline__ uint2 load_row_word(const DevCol& col, int64_t row) {
  const int64_t off = row << col.lg;
  return *reinterpret_cast<const uint2*>(col.ptr + (off & ~(int64_t)7));
}
__device__ __forceinline__ void row_word_to_chunk(Chunk& c, const DevCol& col, int64_t row, uint2 w) {
  const int64_t off = row << col.lg;
  const uint64_t x = (((uint64_t)w.y << 32) | w.x) >> ((off & 7) * 8);
  c.a = make_uint4((uint32_t)x, (uint32_t)(x >> 32), 0u, 0u);
  c.b = make_uint4(0u, 0u, 0u, 0u);
  c.sh = 0;
}

template <int NC>
__device__ __forceinline__ void load_rows1(const ScanParams& p, int64_t row, Chunk (&raw)[NC]) {
#pragma unroll
  for (int c = 0; c < NC; ++c) load_one(raw[c], p.cols[c], row);
}

template <int R>
__device__ __forceinline__ void decode(const Chunk& c, int dt, uint64_t (&v)[R]) {
  switch (dt) {
    case BQG_BOOL:
    case BQG_U8: {
      const uint32_t w = chunk_word_dyn(c, 0);
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = (w >> (8 * r)) & 0xFFu;
    } break;
    case BQG_I8: {
      const uint32_t w = chunk_word_dyn(c, 0);
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = (uint64_t)(int64_t)(int8_t)((w >> (8 * r)) & 0xFFu);
    } break;
    case BQG_U16:
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = (chunk_word_dyn(c, r >> 1) >> (16 * (r & 1))) & 0xFFFFu;
      break;
    case BQG_I16:
#pragma unroll
      for (int r = 0; r < R; ++r)
        v[r] = (uint64_t)(int64_t)(int16_t)((chunk_word_dyn(c, r >> 1) >> (16 * (r & 1))) & 0xFFFFu);
      break;
    case BQG_I32:
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = (uint64_t)(int64_t)(int32_t)chunk_u32(c, r);
      break;
    case BQG_U32:
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = chunk_u32(c, r);
      break;
    case BQG_F32:
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = as_u64((double)__uint_as_float(chunk_u32(c, r)));
      break;
    default:  // I64, U64, F64: raw 64-bit pattern
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = ((uint64_t)chunk_u32(c, 2 * r + 1) << 32) | chunk_u32(c, 2 * r);
      break;
  }
}

// float64 value of an aggregation input held as a canonical value
__device__ __forceinline__ double value_f64(uint64_t v, int conv) {
  return conv == 0 ? as_f64(v) : (conv == 1 ? (double)(int64_t)v : (double)v);
}

// Fixed-point limbs of a finite float64 (ScanParams::sum_enc 3): X = |x| * 2^shift, truncated to
// an integer (below 2^95 by the choice of shift), split into three 32-bit limbs that carry x's
// sign.  Limb sums of fewer than 2^31 rows fit int64; integer adds make the total independent of
// the order the rows arrive in.
// Non-finite values of a fixed-point sum are flags beside its limbs (SlotArrays::fx word 2):
// 1 NaN, 2 +inf, 4 -inf, ORed in any order; the sum is then NaN (a NaN, or both infinities)
// or the one infinity -- what float64 addition gives in any order
__device__ __forceinline__ bool fx_finite(double x) { return (as_u64(x) & 0x7FF0000000000000ull) != 0x7FF0000000000000ull; }
__device__ __forceinline__ unsigned long long fx_flag(double x) { return x != x ? 1ull : (x > 0 ? 2ull : 4ull); }
__device__ __forceinline__ double fx_nonfinite(unsigned long long fl) {
  if ((fl & 1ull) || (fl & 6ull) == 6ull) return __longlong_as_double(0x7FF8000000000000ll);
  return (fl & 2ull) ? __longlong_as_double(0x7FF0000000000000ll) : __longlong_as_double((long long)0xFFF0000000000000ull);
}

// the fixed-point shift of state q at a slot: the column's, or the slot's own (fx_emax)
__device__ __forceinline__ int fx_shift(const ScanParams& p, int q, uint64_t s) {
  if (!p.fx_emax[q]) return p.sum_fx_shift[q];
  const int32_t e = p.fx_emax[q][s];
  return e ? 95 - (e - 2048) : 0;
}
// 2048 + e for a finite nonzero |x| < 2^e (its exponent field + 1 - 1023; subnormals as 2^-1022)
__device__ __forceinline__ int32_t fx_exp_key(double x) {
  const int ex = (int)((as_u64(x) >> 52) & 0x7FFu);
  return (ex ? ex : 1) - 1022 + 2048;
}

__device__ __forceinline__ void fx_limbs(double x, int shift, long long (&l)[3]) {
  const uint64_t b = as_u64(x);
  const int ex = (int)((b >> 52) & 0x7FFu);
  const uint64_t mant = (b & 0xFFFFFFFFFFFFFull) | (ex ? (1ull << 52) : 0ull);
  const int k = (ex ? ex - 1075 : -1074) + shift;  // X = mant * 2^k, k <= 42
  uint64_t lo, hi;
  if (k >= 64) {
    lo = 0;
    hi = mant << (k - 64);
  } else if (k > 0) {
    lo = mant << k;
    hi = mant >> (64 - k);
  } else {
    lo = k > -64 ? mant >> -k : 0ull;
    hi = 0;
  }
  const long long sg = (b >> 63) ? -1ll : 1ll;
  l[0] = sg * (long long)(lo & 0xFFFFFFFFull);
  l[1] = sg * (long long)(lo >> 32);
  l[2] = sg * (long long)(hi & 0xFFFFFFFFull);
}

// The float64 nearest the exact limb total (s0 + s1 * 2^32 + s2 * 2^64) * 2^-shift: the limb
// sums are combined exactly in 128 bits (|s2| < 2^62, so the total stays below 2^127) and
// rounded once
__device__ __forceinline__ double fx_value(long long s0, long long s1, long long s2, int shift) {
  const __int128 t = (((__int128)s2 << 32) + (__int128)s1) * ((__int128)1 << 32) + (__int128)s0;
  return ldexp((double)t, -shift);
}

template <int NC, int R>
__device__ __forceinline__ void decode_all(const ScanParams& p, const Chunk (&raw)[NC], uint64_t (&v)[NC][R]) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    decode<R>(raw[c], p.cols[c].dtype, v[c]);
    if (p.cols[c].enc == 1) {  // compact copy: offset back to the canonical value
#pragma unroll
      for (int r = 0; r < R; ++r) v[c][r] += (uint64_t)p.cols[c].off;
    }
  }
}

// ------------------------------------------------------------------------------------
// where-terms on canonical values
// ------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ bool sorted_contains(const T* vals, int n, T x) {
  if (n <= 8) {
    bool hit = false;
    for (int i = 0; i < n; ++i) hit |= (vals[i] == x);
    return hit;
  }
  int lo = 0, hi = n - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const T m = vals[mid];
    if (m == x) return true;
    if (m < x) lo = mid + 1;
    else hi = mid - 1;
  }
  return false;
}

template <typename T>
__device__ __forceinline__ bool cmp_op(int op, T x, T v) {
  switch (op) {
    case BQG_T_EQ: return x == v;
    case BQG_T_NE: return x != v;
    case BQG_T_GT: return x > v;
    case BQG_T_GE: return x >= v;
    case BQG_T_LT: return x < v;
    default: return x <= v;
  }
}

// A scalar comparison of values known to lie in [0, 2^32) (a compact copy's stored offsets,
// compile-time in a specialised kernel): the int64 constant folds into a 32-bit bound once
// (uniform), so each row costs one 32-bit compare instead of a 64-bit one
template <int R>
__device__ __forceinline__ uint32_t eval_term_u32(int op, int64_t c, const uint64_t (&v)[R]) {
  // ge: v >= lo (lo in [0, 2^32]); lt: v < lo; eq / ne: v == c when c is in range
  const int64_t lo64 = (op == BQG_T_GT || op == BQG_T_LE) ? (c == (int64_t)0x7FFFFFFFFFFFFFFFll ? c : c + 1) : c;
  const bool lo_neg = lo64 <= 0, lo_big = lo64 > (int64_t)0xFFFFFFFFll;
  const uint32_t lo = lo_neg ? 0u : (uint32_t)lo64;
  const bool in_range = c >= 0 && c <= (int64_t)0xFFFFFFFFll;
  uint32_t m = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t x = (uint32_t)v[r];
    bool hit;
    switch (op) {
      case BQG_T_GE:
      case BQG_T_GT: hit = !lo_big && x >= lo; break;
      case BQG_T_LT:
      case BQG_T_LE: hit = lo_big || (!lo_neg && x < lo); break;
      case BQG_T_EQ: hit = in_range && x == (uint32_t)c; break;
      default: hit = !in_range || x != (uint32_t)c; break;  // NE
    }
    m |= (uint32_t)hit << r;
  }
  return m;
}

template <int R>
__device__ __forceinline__ uint32_t eval_term(const DevTerm& t, const uint64_t (&v)[R], bool uns, bool u32 = false) {
  const int op = t.op;
  if (op == BQG_T_TRUE) return (1u << R) - 1u;
  if (op == BQG_T_FALSE) return 0u;
  uint32_t m = 0;
  const bool list = (op == BQG_T_IN || op == BQG_T_NIN);
  if (u32 && !list && !t.is_float) return eval_term_u32<R>(op, t.iv0, v);
  if (t.is_float) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double x = as_f64(v[r]);
      bool hit = list ? (sorted_contains<double>(t.fvals, t.nvals, x) == (op == BQG_T_IN)) : cmp_op<double>(op, x, t.fv0);
      m |= (uint32_t)hit << r;
    }
  } else if (uns) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      bool hit = list ? (sorted_contains<uint64_t>(reinterpret_cast<const uint64_t*>(t.ivals), t.nvals, v[r]) ==
                         (op == BQG_T_IN))
                      : cmp_op<uint64_t>(op, v[r], (uint64_t)t.iv0);
      m |= (uint32_t)hit << r;
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t x = (int64_t)v[r];
      bool hit = list ? (sorted_contains<int64_t>(t.ivals, t.nvals, x) == (op == BQG_T_IN)) : cmp_op<int64_t>(op, x, t.iv0);
      m |= (uint32_t)hit << r;
    }
  }
  return m;
}

// R-bit pass mask of the rows starting at row0 (BOUND = false: the caller has already masked
// rows past the end, and only the where terms and the mask column are applied)
template <int NC, int R, bool BOUND = true>
__device__ __forceinline__ uint32_t vals_pass(const ScanParams& p, int64_t row0, const uint64_t (&v)[NC][R]) {
  uint32_t pass = (1u << R) - 1u;
  if (BOUND) {
    const int64_t rem = p.nrows - row0;
    pass = rem >= R ? ((1u << R) - 1u) : (rem > 0 ? ((1u << rem) - 1u) : 0u);
  }
#pragma unroll
  for (int t = 0; t < BQ_LOOP_BOUND(p.nterms, kMaxTerms); ++t) {
    if (t >= p.nterms) break;
    const DevTerm& tm = p.terms[t];
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (tm.col == c)
        pass &= eval_term<R>(tm, v[c], p.cols[c].dtype == BQG_U64,
                             p.cols[c].enc == 0 && (p.cols[c].dtype == BQG_U8 || p.cols[c].dtype == BQG_U16 ||
                                                    p.cols[c].dtype == BQG_U32));
  }
  if (p.mask_col >= 0) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (p.mask_col == c) {
        uint32_t m = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) m |= (v[c][r] != 0) ? (1u << r) : 0u;
        pass &= m;
      }
  }
  return pass;
}

// canonical 64-bit identity of a key value (float keys: NaN == NaN, -0.0 == +0.0)
__device__ __forceinline__ uint64_t key_identity(uint64_t v, bool is_float) {
  return is_float ? canon_f64_bits(v) : v;
}

// dense mixed-radix (or packed, hash mode 1) group code of each row; hash mode 2 (wide
// keys: key spaces over 63 bits, float columns in a multi-column key): a 64-bit hash of the
// keys' canonical values, resolved against the stored representative row (slot_lookup)
template <int NC, int R>
__device__ __forceinline__ void vals_code(const ScanParams& p, const uint64_t (&v)[NC][R], uint64_t (&code)[R]) {
#pragma unroll
  for (int r = 0; r < R; ++r) code[r] = 0;
  if (p.hash == 2) {
#pragma unroll
    for (int r = 0; r < R; ++r) code[r] = 0x243F6A8885A308D3ull;
#pragma unroll
    for (int k = 0; k < BQ_LOOP_BOUND(p.nkeys, kMaxKeys); ++k) {
      if (k >= p.nkeys) break;
      const DevKey& key = p.keys[k];
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (key.col == c) {
#pragma unroll
          for (int r = 0; r < R; ++r) code[r] = mix64(code[r] ^ (key_identity(v[c][r], key.is_float) + (uint64_t)k));
        }
    }
    return;
  }
  if (p.hash == 0) {
    // dense slot spaces (< 2^27 slots, integer keys only): every term (v - min) * stride and
    // their sum are below the slot count, so 32-bit arithmetic gives the exact code -- a third
    // of the 64-bit sub / mul / add chain per key and row
    uint32_t c32[R];
#pragma unroll
    for (int r = 0; r < R; ++r) c32[r] = 0;
#pragma unroll
    for (int k = 0; k < BQ_LOOP_BOUND(p.nkeys, kMaxKeys); ++k) {
      if (k >= p.nkeys) break;
      const DevKey& key = p.keys[k];
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (key.col == c) {
#pragma unroll
          for (int r = 0; r < R; ++r) c32[r] += ((uint32_t)v[c][r] - (uint32_t)key.min) * (uint32_t)key.stride;
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) code[r] = c32[r];
    return;
  }
#pragma unroll
  for (int k = 0; k < BQ_LOOP_BOUND(p.nkeys, kMaxKeys); ++k) {
    if (k >= p.nkeys) break;
    const DevKey& key = p.keys[k];
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (key.col == c) {
        if (key.is_float) {
#pragma unroll
          for (int r = 0; r < R; ++r) code[r] += canon_f64_bits(v[c][r]) * key.stride;
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r) code[r] += (v[c][r] - (uint64_t)key.min) * key.stride;
        }
      }
  }
}

// open-addressing hash of packed key codes -> table position (the slot)
__device__ __forceinline__ uint64_t hash_slot(const SlotArrays& sa, uint64_t mask, uint64_t code, bool insert) {
  uint64_t pos = mix64(code) & mask;
  for (uint64_t i = 0; i <= mask; ++i) {
    const unsigned long long k = sa.keys[pos];
    if (k == code) return pos;
    if (k == kEmpty) {
      if (!insert) return kEmpty;
      const unsigned long long prev = atomicCAS(&sa.keys[pos], kEmpty, (unsigned long long)code);
      if (prev == kEmpty) {
        const unsigned int f = atomicAdd(sa.hash_fill, 1u);
        if ((uint64_t)(f + 1) * 2 > mask + 1) atomicOr(sa.overflow, 1u);
        return pos;
      }
      if (prev == code) return pos;
    }
    pos = (pos + 1) & mask;
  }
  atomicOr(sa.overflow, 1u);
  return kEmpty;
}

// canonical value of column `kc` at `row` (floats: float64 bits)
__device__ __forceinline__ uint64_t value_at_row(const DevCol& kc, uint32_t row) {
  Chunk c;
  row_word_to_chunk(c, kc, row, load_row_word(kc, row));
  uint64_t v[1];
  decode<1>(c, kc.dtype, v);
  return v[0];
}

// key value of column `kc` at `row` (a slot's representative row), canonical
__device__ __forceinline__ uint64_t key_at_row(const DevCol& kc, bool is_float, uint32_t row) {
  return key_identity(value_at_row(kc, row), is_float);
}

// Slot of row r's key: hash modes 1 (packed code stored in the table) and 2 (wide keys: the
// table word is hash_hi32 << 32 | representative row; a candidate with the same hash half
// matches only when every key value at its representative row equals this row's).  The
// representative is the inserting row, written with the claim itself (one 64-bit CAS), so a
// reader never sees a half-built entry.  kEmpty: absent (lookup) or table full.
template <int NC, int R>
__device__ __forceinline__ uint64_t slot_lookup(const ScanParams& p, const SlotArrays& sa, uint64_t mask,
                                                const uint64_t (&v)[NC][R], const uint64_t (&code)[R], int r,
                                                uint32_t row, bool insert) {
  if (p.hash != 2) return hash_slot(sa, mask, code[r], insert);
  const uint32_t hi = (uint32_t)(code[r] >> 32);
  uint64_t pos = code[r] & mask;
  for (uint64_t i = 0; i <= mask; ++i) {
    unsigned long long w = sa.keys[pos];
    if (w == kEmpty) {
      if (!insert) return kEmpty;
      const unsigned long long mine = ((unsigned long long)hi << 32) | row;
      const unsigned long long prev = atomicCAS(&sa.keys[pos], kEmpty, mine);
      if (prev == kEmpty) {
        const unsigned int f = atomicAdd(sa.hash_fill, 1u);
        if ((uint64_t)(f + 1) * 2 > mask + 1) atomicOr(sa.overflow, 1u);
        return pos;
      }
      w = prev;
    }
    if ((uint32_t)(w >> 32) == hi) {
      const uint32_t rep = (uint32_t)w;
      bool same = true;
#pragma unroll
      for (int k = 0; k < BQ_LOOP_BOUND(p.nkeys, kMaxKeys); ++k) {
        if (k >= p.nkeys) break;
        const DevKey& key = p.keys[k];
#pragma unroll
        for (int c = 0; c < NC; ++c)
          if (key.col == c) same &= key_at_row(p.cols[c], key.is_float, rep) == key_identity(v[c][r], key.is_float);
      }
      if (same) return pos;
    }
    pos = (pos + 1) & mask;
  }
  atomicOr(sa.overflow, 1u);
  return kEmpty;
}

// 64-bit hash of the canonical key VALUES of a row (not codes: codes depend on per-table
// statistics) -- the cross-rank merge's partition function (mod nranks) and its reduce table
__device__ __forceinline__ uint64_t key_hash_row(const PartitionCols& k, int64_t row) {
  uint64_t h = 0x243F6A8885A308D3ull;
  for (int j = 0; j < k.nkeys; ++j) {
    Chunk c;
    row_word_to_chunk(c, k.cols[j], row, load_row_word(k.cols[j], row));
    uint64_t v[1];
    decode<1>(c, k.cols[j].dtype, v);
    const uint64_t bits = dtype_is_float(k.cols[j].dtype) ? canon_f64_bits(v[0]) : v[0];
    h = mix64(h ^ mix64(bits + (uint64_t)j));
  }
  return h;
}

// ------------------------------------------------------------------------------------
// Emit helpers (shared by the private finish kernel and the generic emit kernel)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void store_elem(void* base, int dt, uint64_t idx, uint64_t bits) {
  switch (dtype_lg(dt)) {
    case 0: reinterpret_cast<uint8_t*>(base)[idx] = (uint8_t)bits; break;
    case 1: reinterpret_cast<uint16_t*>(base)[idx] = (uint16_t)bits; break;
    case 2: reinterpret_cast<uint32_t*>(base)[idx] = (uint32_t)bits; break;
    default: reinterpret_cast<unsigned long long*>(base)[idx] = bits; break;
  }
}

// a dense key's offset in its range from its slot code: 32-bit division when code, stride and
// range fit (dense slot spaces stay below 2^27) -- a 64-bit division is a long software
// sequence, and two keys' division and modulo were most of a 1 M-group emit's time
__device__ __forceinline__ uint64_t key_offset(uint64_t code, const DevKey& k) {
  if (((code | k.stride | k.range) >> 32) == 0) return (uint32_t)code / (uint32_t)k.stride % (uint32_t)k.range;
  return (code / k.stride) % k.range;
}

struct SlotTotals {
  unsigned long long cnt;
  uint32_t fst;
  unsigned long long acc[kMaxSums];
  unsigned long long acc2[kMaxSums];  // centered second moments (std pass 2)
  __device__ unsigned long long sum(int q) const { return acc[q]; }
  __device__ unsigned long long m2(int q) const { return acc2[q]; }
};

// A slot's totals read where they lie (the emit kernels): a sum state is picked by the
// column's runtime state index, and an array of all of them in registers would be indexed
// dynamically -- which the compiler turns into an LDS array sized for 1024 threads (80 KB per
// workgroup: one or two workgroups per CU, the 1 M-group emit latency-bound at ~1.5 waves per
// SIMD; round 6)
struct SlotRef {
  unsigned long long cnt;
  uint32_t fst;
  const unsigned long long* acc;   // &sa.acc[s]: state q at acc[q * stride]
  const unsigned long long* acc2;  // &sa.acc2[s] (std states) or nullptr
  uint64_t stride;
  __device__ unsigned long long sum(int q) const { return acc[(size_t)q * stride]; }
  __device__ unsigned long long m2(int q) const { return acc2[(size_t)q * stride]; }
};
__device__ __forceinline__ SlotRef slot_ref(const SlotArrays& sa, uint64_t s, uint64_t nslots, unsigned long long cnt,
                                            uint32_t fst) {
  SlotRef t;
  t.cnt = cnt;
  t.fst = fst;
  t.acc = sa.acc ? sa.acc + s : nullptr;
  t.acc2 = sa.acc2 ? sa.acc2 + s : nullptr;
  t.stride = nslots;
  return t;
}

// one output column's value for one group (emit_slot's column loop body)
template <typename T>
__device__ __forceinline__ uint64_t column_bits(const EmitParams& e, const EmitCol& c, uint64_t slot, uint64_t code,
                                               unsigned int rank, const T& t) {
  uint64_t bits = 0;
  if (c.kind == 0) {
    const DevKey& k = e.keys[c.key];
    if (e.hash == 2) {  // wide keys: the value at the slot's representative row
      bits = key_at_row(e.key_cols[c.key], k.is_float, (uint32_t)code);
      if (c.out_dtype == BQG_F32) bits = __float_as_uint((float)as_f64(bits));
    } else if (k.is_float) {
      bits = code;
      if (c.out_dtype == BQG_F32) bits = __float_as_uint((float)as_f64(code));
    } else {
      const uint64_t off = key_offset(code, k);
      bits = (uint64_t)k.min + off;
    }
  } else {
    switch (c.op) {
      case BQG_SUM: {
        unsigned long long a = t.sum(c.state);
        if (c.in_float && e.sum_dec[c.state] != 0.0) a = as_u64((double)(long long)a / e.sum_dec[c.state]);
        if (c.in_float) bits = (c.out_dtype == BQG_F32) ? (uint64_t)__float_as_uint((float)as_f64(a)) : a;
        else bits = a;  // wrap-around to the output width happens in store_elem
      } break;
      case BQG_COUNT: bits = t.cnt; break;
      case BQG_MEAN: {
        const unsigned long long a = t.sum(c.state);
        const double s = c.in_float ? (e.sum_dec[c.state] != 0.0 ? (double)(long long)a / e.sum_dec[c.state] : as_f64(a))
                                    : (c.in_dtype == BQG_U64 ? (double)(uint64_t)a : (double)(long long)a);
        bits = as_u64(s / (double)t.cnt);
        if (e.nf_cnt[c.sum_state]) {
          // bquery's m += (x - m) / c: an infinity stays only as the group's last row and its
          // one non-finite value (the next row makes inf - inf); NaN otherwise
          const uint32_t k = e.nf_cnt[c.sum_state][slot];
          if (k) {
            double m = __builtin_nan("");
            if (k == 1 && e.nf_row[c.sum_state][slot] == e.nf_last[slot]) {
              const double x = as_f64(value_at_row(e.nf_col[c.sum_state], e.nf_row[c.sum_state][slot]));
              if (__builtin_isinf(x)) m = x;
            }
            bits = as_u64(m);
          }
        }
      } break;
      case BQG_STD: {
        const double m2 = as_f64(t.m2(c.state));
        bits = as_u64(t.cnt ? sqrt(m2 / (double)t.cnt) : __builtin_nan(""));
        // Welford: d * (x - mean) is inf * (inf - inf) at the first non-finite value
        if (e.nf_cnt[c.sum_state] && e.nf_cnt[c.sum_state][slot]) bits = as_u64(__builtin_nan(""));
      } break;
      case BQG_COUNT_DISTINCT: bits = e.cd[c.state][slot]; break;
      case BQG_SORTED_COUNT_DISTINCT: {
        // bquery rule: the first processed row initialises slot 0 (counts 1 only when that
        // row has label 0, i.e. row 0 passes); every other group's first value is compared
        // with the zero-initialised last value.
        unsigned long long ch = e.scd_changes[c.state][slot];
        const unsigned long long fv = e.scd_first[c.state][slot];
        const bool first_differs = c.in_float ? !(as_f64(fv) == 0.0) : (fv != 0ull);
        if (rank == 0) ch += (t.fst == 0u) ? 1ull : 0ull;
        else ch += first_differs ? 1ull : 0ull;
        bits = ch;
      } break;
    }
  }
  return bits;
}

template <typename T>
__device__ __forceinline__ void emit_slot(const EmitParams& e, uint64_t slot, uint64_t code, unsigned int rank,
                                       const T& t) {
  for (int j = 0; j < e.ncols; ++j) {
    const EmitCol& c = e.cols[j];
    store_elem(c.out, c.out_dtype, rank, column_bits(e, c, slot, code, rank, t));
  }
}

#define BQG_DISPATCH_NC(NCV, ...)                       \
  switch (NCV) {                                        \
    case 1: { constexpr int NC = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int NC = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int NC = 3; __VA_ARGS__; } break; \
    case 4: { constexpr int NC = 4; __VA_ARGS__; } break; \
    case 5: { constexpr int NC = 5; __VA_ARGS__; } break; \
    default: { constexpr int NC = 6; __VA_ARGS__; } break; \
  }

}  // namespace bqg
