// jit_kernels.h -- query-specialised kernel entry points, compiled at run time by hiprtc
// (jit.hip).  The host prepends `#define BQ_NC <n>` and `#define BQ_SPEC <assignments>`:
// the query's shape (column dtypes and widths, term columns and operators, key columns,
// summed-column kinds, mask / hash flags) becomes compile-time constants, so every dtype and
// operator dispatch of the generic kernels folds away; pointers, values, key minima and
// strides stay run-time parameters.  The bodies are the precompiled kernels' own
// (scan_private.h), so both paths compute the same thing.
#pragma once

#include "partition.h"
#include "scd.h"
#include "scan_private.h"

#ifndef BQ_PART_K
#define BQ_PART_K 1
#endif
#ifndef BQ_PART_NARROW
#define BQ_PART_NARROW 0
#endif
#ifndef BQ_PART_PACK
#define BQ_PART_PACK 0
#endif
#ifndef BQ_PART_RING
#define BQ_PART_RING 1
#endif

namespace bqg {
__device__ __forceinline__ void jit_specialize(ScanParams& p) { BQ_SPEC }
}  // namespace bqg

extern "C" __global__ __launch_bounds__(256, 4) void bq_jit_scan_private(bqg::ScanParams pin, bqg::PrivateLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  bqg::ScanParams p = pin;
  bqg::jit_specialize(p);
  bqg::scan_private_body<BQ_NC>(p, L, smem);
}

#ifndef BQ_PART_THREADS
#define BQ_PART_THREADS 1024
#endif
extern "C" __global__ __launch_bounds__(BQ_PART_THREADS) void bq_jit_part_scatter(bqg::ScanParams pin, bqg::PartLaunch L) {
  extern __shared__ __align__(16) unsigned char smem[];
  bqg::ScanParams p = pin;
  bqg::jit_specialize(p);
  bqg::part_scatter_body<BQ_NC, BQ_PART_K, BQ_PART_NARROW != 0, BQ_PART_PACK != 0, BQ_PART_RING>(p, L, smem);
}

extern "C" __global__ __launch_bounds__(bqg::kFirstRowsBlock) void bq_jit_part_first_rows(bqg::ScanParams pin, bqg::PartLaunch L,
                                                                        bqg::SlotArrays sa) {
  bqg::ScanParams p = pin;
  bqg::jit_specialize(p);
  bqg::part_first_rows_body<BQ_NC>(p, L, sa);
}

extern "C" __global__ __launch_bounds__(256) void bq_jit_scd_fused(bqg::ScanParams pin, bqg::ScdLaunch d) {
  extern __shared__ __align__(16) unsigned char smem[];
  bqg::ScanParams p = pin;
  bqg::jit_specialize(p);
  bqg::scd_fused_body<BQ_NC, false>(p, d, smem);
}

extern "C" __global__ __launch_bounds__(256) void bq_jit_scd_fused32(bqg::ScanParams pin, bqg::ScdLaunch d) {
  extern __shared__ __align__(16) unsigned char smem[];
  bqg::ScanParams p = pin;
  bqg::jit_specialize(p);
  bqg::scd_fused_body<BQ_NC, true>(p, d, smem);
}

extern "C" __global__ __launch_bounds__(256) void bq_jit_scd_runs32(bqg::ScanParams pin, bqg::ScdLaunch d) {
  extern __shared__ __align__(16) unsigned char smem[];
  bqg::ScanParams p = pin;
  bqg::jit_specialize(p);
  bqg::scd_fused_body<BQ_NC, true, true>(p, d, smem);
}
