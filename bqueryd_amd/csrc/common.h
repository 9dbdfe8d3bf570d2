// common.h -- shared host/device definitions for libbqgpu (gfx950 only).
#pragma once

#ifndef __HIPCC_RTC__  // the JIT (hiprtc) provides the HIP runtime and fixed-width types
#include <hip/hip_runtime.h>
#include <stdint.h>
#else
typedef struct ihipStream_t* hipStream_t;  // host launchers are declared, never defined, in JIT code
typedef struct ihipModuleSymbol_t* hipFunction_t;
typedef struct ihipEvent_t* hipEvent_t;
#endif

#include "../../include/bqgpu.h"

namespace bqg {

constexpr int kMaxCols = 6;    // distinct input columns one scan kernel streams
constexpr int kMaxTerms = 8;   // where terms fused into one scan
constexpr int kMaxKeys = 4;    // groupby columns
constexpr int kMaxSums = 4;    // summed value columns per scan
constexpr int kMaxAggs = 16;   // aggregations per query
constexpr int kBlock = 256;    // threads per workgroup of the scan kernels (4 wave64)
constexpr int kRowsPerThread = 4;
constexpr int kTileRows = kBlock * kRowsPerThread;  // rows per workgroup iteration
constexpr uint32_t kNoRow = 0xFFFFFFFFu;
constexpr uint64_t kEmpty = ~0ull;  // empty hash slot

__host__ __device__ inline int dtype_lg(int dt) {
  switch (dt) {
    case BQG_BOOL: case BQG_I8: case BQG_U8: return 0;
    case BQG_I16: case BQG_U16: return 1;
    case BQG_I32: case BQG_U32: case BQG_F32: return 2;
    default: return 3;
  }
}
__host__ __device__ inline bool dtype_is_float(int dt) { return dt == BQG_F32 || dt == BQG_F64; }
__host__ __device__ inline bool dtype_is_unsigned(int dt) {
  return dt == BQG_BOOL || dt == BQG_U8 || dt == BQG_U16 || dt == BQG_U32 || dt == BQG_U64;
}

// ------------------------------------------------------------------------------------
// Kernel parameter block (passed by value; < 4 KiB).
// ------------------------------------------------------------------------------------
struct DevCol {
  const unsigned char* ptr;
  int32_t dtype;  // the STORED element type (a compact copy's narrow type, see enc)
  int32_t lg;
  // compact resident copy (api.hip Column::shadow): enc 1 -- an integer column stored as an
  // unsigned offset from `off` in fewer bytes; the decode adds `off` back, so every consumer
  // sees the column's canonical int64 value.  (A float64 column stored as its exact int32
  // codes carries enc 0: its canonical value IS the code, and only code-aware sum states read it.)
  int32_t enc;
  int32_t pad_;
  int64_t off;
};

struct DevTerm {
  int32_t col;       // index into ScanParams::cols
  int32_t op;        // bqg_term_op
  int32_t is_float;
  int32_t nvals;
  int64_t iv0;       // first value (scalar ops)
  double fv0;
  const int64_t* ivals;  // sorted list for IN / NIN (device)
  const double* fvals;
};

struct DevKey {
  int32_t col;       // index into ScanParams::cols
  int32_t is_float;  // float key: code = canonical bits (single-key hash mode)
  int64_t min;       // code = (v - min) * stride
  uint64_t stride;
  uint64_t range;
};

struct ScanParams {
  int64_t nrows;
  int32_t ncols;
  int32_t nterms;
  int32_t nkeys;
  int32_t nsum;      // sum states = cols[0 .. nsum-1]
  int32_t mask_col;  // index into cols of a BOOL mask column, or -1
  int32_t hash;      // 1: slot = hash-table position of the packed key code
  uint64_t nslots;   // dense slot space (or hash capacity)
  DevCol cols[kMaxCols];
  DevTerm terms[kMaxTerms];
  DevKey keys[kMaxKeys];
  int32_t sum_is_float[kMaxSums];      // accumulate in float64 (else int64)
  int32_t sum_conv[kMaxSums];          // input: 0 float bits, 1 signed int, 2 uint64
  int32_t sum_centered[kMaxSums];      // accumulate (v - center[slot])^2 (std pass 2)
  const double* centers[kMaxSums];
  // shared / global modes: a float sum whose column has an exact 32-bit integer code for every
  // value (column statistics) accumulates the codes as int64 -- 1 dyadic, code = v * sum_mul;
  // 2 cents, code = rint(v * sum_mul); 0 = float64 arrival-order sum.  Integer atomics make the
  // sum independent of the arrival order (bit-reproducible); EmitParams::sum_dec scales it back.
  int32_t sum_enc[kMaxSums];
  double sum_mul[kMaxSums];
  // sum_enc 3 (the atomic modes' float sums without an exact code): each value as a
  // fixed-point integer |x| * 2^sum_fx_shift (< 2^95; the shift from the column statistics'
  // largest magnitude) in three 32-bit limbs carrying x's sign, each limb summed as an int64 --
  // integer atomics, so the sum no longer depends on the arrival order (k_fx_finalize rounds it
  // to float64 once)
  int32_t sum_fx_shift[kMaxSums];
  // ... or, for a column the column-wide shift would truncate (values spanning more than ~2^42
  // in magnitude), a shift per slot from the slot's own largest magnitude: fx_emax[q][slot] =
  // 2048 + e for the slot's largest finite |x| < 2^e (0: none; k_fx_emax fills it before the
  // sums), the slot's shift 95 - e (fx_shift)
  const int32_t* fx_emax[kMaxSums];
};

// words per fixed-point sum state beside its limb 0 (SlotArrays::fx): limbs 1, 2, flags
constexpr int kFxWords = 3;

// Per-slot aggregation state in device memory (global modes, and the target of the
// private/shared modes' block flush).
struct SlotArrays {
  unsigned long long* cnt;   // [nslots]
  uint32_t* fst;             // [nslots]  first passing row (kNoRow = none)
  unsigned long long* acc;   // [nsum][nslots]  f64 or i64 bit patterns
  unsigned long long* acc2;  // [nsum2][nslots] centered second moments (std), or null
  unsigned long long* fx;    // [nsum][kFxWords][nslots]: limbs 1 and 2 of fixed-point sums
                             // (sum_enc 3; limb 0 is acc) and their non-finite flags, or null
  unsigned long long* keys;  // hash mode: [nslots] packed key code or kEmpty
  unsigned int* hash_fill;   // hash mode: number of occupied positions
  unsigned int* overflow;    // hash mode: set when the table is over-full
};

// ------------------------------------------------------------------------------------
// Device helpers: 4-row column chunks.
// ------------------------------------------------------------------------------------
struct Chunk {
  uint4 a, b;    // up to 32 bytes = 4 rows x 8 bytes
  uint32_t sh;   // word offset of row0 inside `a` (1- and 2-byte columns)
};

// Branch-free chunk load: 1- to 4-byte columns read the aligned 16-byte block that holds the
// lane's 4 rows (one global_load_dwordx4; neighbouring lanes share the block, so HBM traffic
// is unchanged), 8-byte columns read 32 bytes.  A runtime switch on the width here made the
// compiler split the loads and drain vmcnt at every join.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// Column streams are read once per query: non-temporal 16-byte loads (measured on MI355X,
// tools/membench.hip: three C2-shaped streams 6.55-6.7 TB/s nt vs 5.8-5.9 TB/s default policy)
__device__ __forceinline__ uint4 load_stream16(const unsigned char* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void load_chunk(Chunk& c, const DevCol& col, int64_t row0) {
  const int64_t off = row0 << col.lg;
#ifdef BQ_NC
  // query-specialised build: the width is a constant, so a 1- / 2-byte column loads exactly
  // its lane's 4 rows (one dword / dwordx2 at the 4-row-aligned row0; the wave's loads stay
  // contiguous) -- no 16-byte block to pick the lane's word out of at decode
  if (col.lg == 0) {
    c.a = make_uint4(__builtin_nontemporal_load(reinterpret_cast<const unsigned int*>(col.ptr + off)), 0u, 0u, 0u);
    c.sh = 0;
    return;
  }
  if (col.lg == 1) {
    const u32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(col.ptr + off));
    c.a = make_uint4(v.x, v.y, 0u, 0u);
    c.sh = 0;
    return;
  }
#endif
  const unsigned char* p = col.ptr + (off & ~int64_t(15));
  c.a = load_stream16(p);
  if (col.lg == 3) c.b = load_stream16(p + 16);
  c.sh = (uint32_t)(off & 15) >> 2;
}

__device__ __forceinline__ uint32_t chunk_u32(const Chunk& c, int i) {
  // i in [0, 8): 32-bit word i of the 32-byte chunk (i is a compile-time constant after unroll)
  switch (i) {
    case 0: return c.a.x; case 1: return c.a.y; case 2: return c.a.z; case 3: return c.a.w;
    case 4: return c.b.x; case 5: return c.b.y; case 6: return c.b.z; default: return c.b.w;
  }
}

// word (sh + i) of `a`, sh a per-lane runtime offset (narrow columns)
__device__ __forceinline__ uint32_t chunk_word_dyn(const Chunk& c, uint32_t i) {
  const uint32_t w = c.sh + i;
  const uint32_t lo = (w & 1u) ? c.a.y : c.a.x;
  const uint32_t hi = (w & 1u) ? c.a.w : c.a.z;
  return (w & 2u) ? hi : lo;
}

// element r (0..3) of the chunk as raw 64-bit pattern, sign/zero-extended as int64
__device__ __forceinline__ int64_t chunk_i64(const Chunk& c, int dt, int r) {
  switch (dt) {
    case BQG_BOOL: case BQG_U8: return (int64_t)((chunk_word_dyn(c, 0) >> (8 * r)) & 0xFF);
    case BQG_I8: return (int64_t)(int8_t)((chunk_word_dyn(c, 0) >> (8 * r)) & 0xFF);
    case BQG_U16: return (int64_t)((chunk_word_dyn(c, r >> 1) >> (16 * (r & 1))) & 0xFFFF);
    case BQG_I16: return (int64_t)(int16_t)((chunk_word_dyn(c, r >> 1) >> (16 * (r & 1))) & 0xFFFF);
    case BQG_I32: return (int64_t)(int32_t)chunk_u32(c, r);
    case BQG_U32: return (int64_t)chunk_u32(c, r);
    case BQG_F32: return (int64_t)__uint_as_float(chunk_u32(c, r));
    case BQG_F64: {
      const uint64_t u = ((uint64_t)chunk_u32(c, 2 * r + 1) << 32) | chunk_u32(c, 2 * r);
      return (int64_t)__longlong_as_double((long long)u);
    }
    default:  // I64, U64
      return (int64_t)(((uint64_t)chunk_u32(c, 2 * r + 1) << 32) | chunk_u32(c, 2 * r));
  }
}

__device__ __forceinline__ double chunk_f64(const Chunk& c, int dt, int r) {
  switch (dt) {
    case BQG_F32: return (double)__uint_as_float(chunk_u32(c, r));
    case BQG_F64: {
      const uint64_t u = ((uint64_t)chunk_u32(c, 2 * r + 1) << 32) | chunk_u32(c, 2 * r);
      return __longlong_as_double((long long)u);
    }
    case BQG_U64: return (double)(uint64_t)chunk_i64(c, dt, r);
    default: return (double)chunk_i64(c, dt, r);
  }
}

// canonical 64-bit identity (khash equality: NaN == NaN, -0.0 == +0.0)
__device__ __forceinline__ uint64_t chunk_bits(const Chunk& c, int dt, int r) {
  if (dtype_is_float(dt)) {
    double d = chunk_f64(c, dt, r);
    if (d != d) return 0x7ff8000000000000ull;
    d += 0.0;
    return (uint64_t)__double_as_longlong(d);
  }
  return (uint64_t)chunk_i64(c, dt, r);
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

}  // namespace bqg
