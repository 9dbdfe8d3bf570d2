// jit.h -- run-time specialisation of the hot scan kernels (hiprtc).
//
// A query's shape (column dtypes, term operators, key / sum layout) is turned into
// compile-time constants of the same kernel bodies the library precompiles, compiled once
// per shape for gfx950 with hiprtc and cached in memory and on disk.  hiprtc is loaded with
// dlopen on first use; without it (or with BQGPU_JIT=0) the precompiled generic kernels run.
#pragma once

#include <string>

#include "kernels.h"

namespace bqg {

// the BQ_NC / BQ_SPEC prologue for a ScanParams (see jit_kernels.h)
std::string jit_spec(const ScanParams& p);

// module function `kernel` specialised by `spec` for the current device, or nullptr when the
// JIT is unavailable / disabled / failed (the failure is remembered, not retried)
hipFunction_t jit_function(const char* kernel, const std::string& spec);

// rows from which a scan is worth specialising (BQGPU_JIT_MIN_ROWS, default 4 Mi rows)
int64_t jit_min_rows();

}  // namespace bqg
