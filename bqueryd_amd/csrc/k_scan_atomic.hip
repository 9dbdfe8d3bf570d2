// k_scan_atomic.hip -- shared-LDS and global (dense / hashed) fused scans.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device.h"

namespace bqg {

// the exact integer code of a summed float value (ScanParams::sum_enc)
__device__ __forceinline__ long long sum_code(const ScanParams& p, int q, uint64_t v) {
  const double d = value_f64(v, p.sum_conv[q]) * p.sum_mul[q];
  return (long long)(p.sum_enc[q] == 1 ? d : rint(d));
}

// SHARED mode: one LDS table per workgroup updated with LDS atomics (ds_add_u32/ds_min_u32/
// ds_add_f64/ds_add_u64), flushed to the per-slot HBM arrays with device-scope atomics.
// Used for mid-size dense slot spaces (e.g. config C4's 265 pickup locations).
template <int NC>
__global__ __launch_bounds__(kBlock, 2) void k_scan_shared(ScanParams p, SlotArrays sa) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int S = (int)p.nslots;
  const int tid = threadIdx.x;
  const int nsum = p.nsum;
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem);  // [nsum][S]
  uint32_t* cnt = reinterpret_cast<uint32_t*>(acc + (size_t)nsum * S);    // [S]
  uint32_t* fst = cnt + S;                                                 // [S]
  // fixed-point sums (sum_enc 3): limbs 1, 2 and the non-finite flags [nsum][3][S] after the
  // table (sa.fx set; 8-byte aligned: the table is 8 (nsum + 1) S bytes)
  unsigned long long* fxl = reinterpret_cast<unsigned long long*>(fst + S);
  for (int i = tid; i < S; i += kBlock) {
    cnt[i] = 0;
    fst[i] = kNoRow;
  }
  for (int i = tid; i < nsum * S; i += kBlock) acc[i] = 0;
  if (sa.fx)
    for (int i = tid; i < kFxWords * nsum * S; i += kBlock) fxl[i] = 0;
  __syncthreads();

  const int64_t ntiles = (p.nrows + kTileRows - 1) / kTileRows;
  int64_t tile = blockIdx.x;
  Chunk raw[NC];
  if (tile < ntiles) load_rows4<NC>(p, tile * kTileRows + (int64_t)tid * kRowsPerThread, raw);
  for (; tile < ntiles; tile += gridDim.x) {
    const int64_t row0 = tile * kTileRows + (int64_t)tid * kRowsPerThread;
    uint64_t v[NC][4];
    decode_all<NC, 4>(p, raw, v);
    const int64_t next = tile + gridDim.x;
    if (next < ntiles) load_rows4<NC>(p, next * kTileRows + (int64_t)tid * kRowsPerThread, raw);
    const uint32_t pass = vals_pass<NC, 4>(p, row0, v);
    uint64_t code[4];
    vals_code<NC, 4>(p, v, code);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (pass & (1u << r)) {
        const int s = (int)code[r];
        const uint32_t row = (uint32_t)(row0 + r);
        atomicAdd(&cnt[s], 1u);
        if (fst[s] > row) atomicMin(&fst[s], row);
#pragma unroll
        for (int q = 0; q < (NC < kMaxSums ? NC : kMaxSums); ++q) {
          if (q < nsum) {
            if (p.sum_is_float[q] && p.sum_enc[q] == 3) {
              double x = value_f64(v[q][r], p.sum_conv[q]);
              if (p.sum_centered[q]) {
                const double d = x - p.centers[q][s];
                x = d * d;
              }
              if (fx_finite(x)) {
                long long l[3];
                fx_limbs(x, fx_shift(p, q, (uint64_t)s), l);
                atomicAdd(&acc[(size_t)q * S + s], (unsigned long long)l[0]);
                atomicAdd(&fxl[(size_t)(kFxWords * q) * S + s], (unsigned long long)l[1]);
                atomicAdd(&fxl[(size_t)(kFxWords * q + 1) * S + s], (unsigned long long)l[2]);
              } else {
                atomicOr(&fxl[(size_t)(kFxWords * q + 2) * S + s], fx_flag(x));
              }
            } else if (p.sum_is_float[q] && p.sum_enc[q]) {
              atomicAdd(&acc[(size_t)q * S + s], (unsigned long long)sum_code(p, q, v[q][r]));
            } else if (p.sum_is_float[q]) {
              double x = value_f64(v[q][r], p.sum_conv[q]);
              if (p.sum_centered[q]) {
                const double d = x - p.centers[q][s];
                x = d * d;
              }
              unsafeAtomicAdd(reinterpret_cast<double*>(&acc[(size_t)q * S + s]), x);
            } else {
              atomicAdd(&acc[(size_t)q * S + s], (unsigned long long)v[q][r]);
            }
          }
        }
      }
    }
  }
  __syncthreads();
  for (int s = tid; s < S; s += kBlock) {
    const uint32_t c = cnt[s];
    if (c == 0) continue;
    atomicAdd(&sa.cnt[s], (unsigned long long)c);
    atomicMin(&sa.fst[s], fst[s]);
    for (int q = 0; q < nsum; ++q) {
      const unsigned long long a = acc[(size_t)q * S + s];
      if (p.sum_is_float[q] && !p.sum_enc[q]) unsafeAtomicAdd(reinterpret_cast<double*>(&sa.acc[(size_t)q * p.nslots + s]), as_f64(a));
      else atomicAdd(&sa.acc[(size_t)q * p.nslots + s], a);
      if (p.sum_is_float[q] && p.sum_enc[q] == 3) {
        for (int h = 0; h < 2; ++h)
          atomicAdd(&sa.fx[(size_t)(kFxWords * q + h) * p.nslots + s], fxl[(size_t)(kFxWords * q + h) * S + s]);
        const unsigned long long fl = fxl[(size_t)(kFxWords * q + 2) * S + s];
        if (fl) atomicOr(&sa.fx[(size_t)(kFxWords * q + 2) * p.nslots + s], fl);
      }
    }
  }
}

// GLOBAL mode: per-slot arrays in HBM updated with device-scope atomics (large dense slot
// spaces, and the hashed key mode where the slot is the hash-table position).
template <int NC, bool HASH>
__global__ __launch_bounds__(kBlock, 4) void k_scan_global(ScanParams p, SlotArrays sa) {
  const int tid = threadIdx.x;
  const int nsum = p.nsum;
  const uint64_t hmask = p.nslots - 1;
  const int64_t ntiles = (p.nrows + kTileRows - 1) / kTileRows;
  int64_t tile = blockIdx.x;
  Chunk raw[NC];
  if (tile < ntiles) load_rows4<NC>(p, tile * kTileRows + (int64_t)tid * kRowsPerThread, raw);
  for (; tile < ntiles; tile += gridDim.x) {
    const int64_t row0 = tile * kTileRows + (int64_t)tid * kRowsPerThread;
    uint64_t v[NC][4];
    decode_all<NC, 4>(p, raw, v);
    const int64_t next = tile + gridDim.x;
    if (next < ntiles) load_rows4<NC>(p, next * kTileRows + (int64_t)tid * kRowsPerThread, raw);
    const uint32_t pass = vals_pass<NC, 4>(p, row0, v);
    uint64_t code[4];
    vals_code<NC, 4>(p, v, code);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (pass & (1u << r)) {
        uint64_t s = code[r];
        const uint32_t row = (uint32_t)(row0 + r);
        if (HASH) {
          s = slot_lookup<NC, 4>(p, sa, hmask, v, code, r, row, true);
          if (s == kEmpty) continue;
        }
        atomicAdd(&sa.cnt[s], 1ull);
        if (sa.fst[s] > row) atomicMin(&sa.fst[s], row);
#pragma unroll
        for (int q = 0; q < (NC < kMaxSums ? NC : kMaxSums); ++q) {
          if (q < nsum) {
            if (p.sum_is_float[q] && p.sum_enc[q] == 3) {
              double x = value_f64(v[q][r], p.sum_conv[q]);
              if (p.sum_centered[q]) {
                const double d = x - p.centers[q][s];
                x = d * d;
              }
              if (fx_finite(x)) {
                long long l[3];
                fx_limbs(x, fx_shift(p, q, s), l);
                atomicAdd(&sa.acc[(size_t)q * p.nslots + s], (unsigned long long)l[0]);
                atomicAdd(&sa.fx[(size_t)(kFxWords * q) * p.nslots + s], (unsigned long long)l[1]);
                atomicAdd(&sa.fx[(size_t)(kFxWords * q + 1) * p.nslots + s], (unsigned long long)l[2]);
              } else {
                atomicOr(&sa.fx[(size_t)(kFxWords * q + 2) * p.nslots + s], fx_flag(x));
              }
            } else if (p.sum_is_float[q] && p.sum_enc[q]) {
              atomicAdd(&sa.acc[(size_t)q * p.nslots + s], (unsigned long long)sum_code(p, q, v[q][r]));
            } else if (p.sum_is_float[q]) {
              double x = value_f64(v[q][r], p.sum_conv[q]);
              if (p.sum_centered[q]) {
                const double d = x - p.centers[q][s];
                x = d * d;
              }
              unsafeAtomicAdd(reinterpret_cast<double*>(&sa.acc[(size_t)q * p.nslots + s]), x);
            } else {
              atomicAdd(&sa.acc[(size_t)q * p.nslots + s], (unsigned long long)v[q][r]);
            }
          }
        }
      }
    }
  }
}

// The nonfinite pass (kernels.h NonfiniteLaunch): the same rows, terms and slots as pass 1;
// per slot the last passing row (an LDS table per workgroup when the slot space is small, one
// atomicMax per slot at the end), per checked sum state the count and last row of its
// non-finite values (rare: global atomics).
template <int NC, bool HASH>
__global__ __launch_bounds__(kBlock) void k_nonfinite(ScanParams p, SlotArrays sa, NonfiniteLaunch nf) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t* slast = reinterpret_cast<uint32_t*>(smem);
  const int tid = threadIdx.x;
  const uint64_t hmask = p.nslots - 1;
  if (nf.lds) {
    for (uint64_t i = tid; i < p.nslots; i += kBlock) slast[i] = 0;
    __syncthreads();
  }
  const int64_t ntiles = (p.nrows + kTileRows - 1) / kTileRows;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t row0 = tile * kTileRows + (int64_t)tid * kRowsPerThread;
    Chunk raw[NC];
    load_rows4<NC>(p, row0, raw);
    uint64_t v[NC][4];
    decode_all<NC, 4>(p, raw, v);
    const uint32_t pass = vals_pass<NC, 4>(p, row0, v);
    uint64_t code[4];
    vals_code<NC, 4>(p, v, code);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (!(pass & (1u << r))) continue;
      uint64_t s = code[r];
      const uint32_t row = (uint32_t)(row0 + r);
      if (HASH) {
        s = slot_lookup<NC, 4>(p, sa, hmask, v, code, r, row, false);
        if (s == kEmpty) continue;
      }
      if (nf.lds) atomicMax(&slast[s], row);
      else if (nf.last_row[s] < row) atomicMax(&nf.last_row[s], row);
#pragma unroll
      for (int q = 0; q < (NC < kMaxSums ? NC : kMaxSums); ++q) {
        if (!((nf.states >> q) & 1)) continue;
        const double x = value_f64(v[q][r], p.sum_conv[q]);
        if (!__builtin_isfinite(x)) {
          atomicAdd(&nf.cnt[q][s], 1u);
          atomicMax(&nf.row[q][s], row);
        }
      }
    }
  }
  if (nf.lds) {
    __syncthreads();
    for (uint64_t i = tid; i < p.nslots; i += kBlock)
      if (slast[i]) atomicMax(&nf.last_row[i], slast[i]);
  }
}

// Per-slot fixed-point shifts (ScanParams::fx_emax): before the sums, the same rows, terms and
// slots (hash mode: inserting, as pass 1 will) -- per slot and state the largest exponent of a
// finite nonzero value, one integer atomicMax (order-free)
template <int NC, bool HASH>
__global__ __launch_bounds__(kBlock) void k_fx_emax(ScanParams p, SlotArrays sa, FxEmaxLaunch fe) {
  const int tid = threadIdx.x;
  const uint64_t hmask = p.nslots - 1;
  const int64_t ntiles = (p.nrows + kTileRows - 1) / kTileRows;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t row0 = tile * kTileRows + (int64_t)tid * kRowsPerThread;
    Chunk raw[NC];
    load_rows4<NC>(p, row0, raw);
    uint64_t v[NC][4];
    decode_all<NC, 4>(p, raw, v);
    const uint32_t pass = vals_pass<NC, 4>(p, row0, v);
    uint64_t code[4];
    vals_code<NC, 4>(p, v, code);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (!(pass & (1u << r))) continue;
      uint64_t s = code[r];
      if (HASH) {
        s = slot_lookup<NC, 4>(p, sa, hmask, v, code, r, (uint32_t)(row0 + r), true);
        if (s == kEmpty) continue;
      }
#pragma unroll
      for (int q = 0; q < (NC < kMaxSums ? NC : kMaxSums); ++q) {
        if (!fe.emax[q]) continue;
        const double x = value_f64(v[q][r], p.sum_conv[q]);
        if (x == 0.0 || !fx_finite(x)) continue;
        const int32_t k = fx_exp_key(x);
        if (fe.emax[q][s] < k) atomicMax(&fe.emax[q][s], k);
      }
    }
  }
}

void launch_fx_emax(const ScanParams& p, const SlotArrays& s, const FxEmaxLaunch& fe, int blocks, hipStream_t st) {
  if (p.hash) {
    BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_fx_emax<NC, true>), dim3(blocks), dim3(kBlock), 0, st, p, s, fe));
  } else {
    BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_fx_emax<NC, false>), dim3(blocks), dim3(kBlock), 0, st, p, s, fe));
  }
}

void launch_nonfinite(const ScanParams& p, const SlotArrays& s, const NonfiniteLaunch& nf, int blocks,
                      hipStream_t st) {
  const size_t lds = nf.lds ? (size_t)p.nslots * 4 : 0;
  if (p.hash) {
    BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_nonfinite<NC, true>), dim3(blocks), dim3(kBlock), lds, st, p, s, nf));
  } else {
    BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_nonfinite<NC, false>), dim3(blocks), dim3(kBlock), lds, st, p, s, nf));
  }
}

__global__ void k_init_slots(SlotArrays sa, int nsum, uint64_t nslots) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * blockDim.x) {
    sa.cnt[i] = 0;
    sa.fst[i] = kNoRow;
    for (int v = 0; v < nsum; ++v) sa.acc[(size_t)v * nslots + i] = 0;
    if (sa.fx)
      for (int v = 0; v < kFxWords * nsum; ++v) sa.fx[(size_t)v * nslots + i] = 0;
    if (sa.keys) sa.keys[i] = kEmpty;
  }
}

// Fixed-point sums (sum_enc 3) to float64 bits in place: acc[q][s] = the nearest double of the
// limbs' exact total (one rounding; fx_value), for every state q in `states`.  Order-free
// integer limbs, one deterministic rounding: the same bits on every run.
__global__ void k_fx_finalize(unsigned long long* acc, const unsigned long long* fx, int nsum, int states,
                              FxShifts sh, uint64_t nslots) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * blockDim.x)
    for (int q = 0; q < nsum; ++q) {
      if (!((states >> q) & 1)) continue;
      const long long s0 = (long long)acc[(size_t)q * nslots + i];
      const long long s1 = (long long)fx[(size_t)(kFxWords * q) * nslots + i];
      const long long s2 = (long long)fx[(size_t)(kFxWords * q + 1) * nslots + i];
      const unsigned long long fl = fx[(size_t)(kFxWords * q + 2) * nslots + i];
      const int shift = sh.emax[q] ? (sh.emax[q][i] ? 95 - (sh.emax[q][i] - 2048) : 0) : sh.shift[q];
      acc[(size_t)q * nslots + i] = as_u64(fl ? fx_nonfinite(fl) : fx_value(s0, s1, s2, shift));
    }
}

void launch_fx_finalize(unsigned long long* acc, const unsigned long long* fx, int nsum, int states, const FxShifts& sh,
                        uint64_t nslots, hipStream_t st) {
  if (!states || !nslots) return;
  uint64_t blocks = (nslots + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_fx_finalize, dim3((unsigned)blocks), dim3(kBlock), 0, st, acc, fx, nsum, states, sh, nslots);
}

void launch_scan_shared(const ScanParams& p, const SlotArrays& s, int blocks, size_t lds, hipStream_t st) {
  BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scan_shared<NC>), dim3(blocks), dim3(kBlock), lds, st, p, s));
}

void launch_scan_global(const ScanParams& p, const SlotArrays& s, int blocks, hipStream_t st) {
  if (p.hash) {
    BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scan_global<NC, true>), dim3(blocks), dim3(kBlock), 0, st, p, s));
  } else {
    BQG_DISPATCH_NC(p.ncols, hipLaunchKernelGGL((k_scan_global<NC, false>), dim3(blocks), dim3(kBlock), 0, st, p, s));
  }
}

void launch_init_slots(const SlotArrays& s, int nsum, uint64_t nslots, hipStream_t st) {
  uint64_t blocks = (nslots + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_init_slots, dim3((unsigned)blocks), dim3(kBlock), 0, st, s, nsum, nslots);
}

}  // namespace bqg
