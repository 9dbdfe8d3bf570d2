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
// JIT is unavailable or failed (the failure is remembered, not retried); whether to use it at
// all is the caller's choice (context options "jit" / "jit_min_rows", api.hip)
hipFunction_t jit_function(const char* kernel, const std::string& spec);

// jit_function(kernel, jit_spec(p) + extra), looked up first by the binary image of p's
// specialised fields (the per-query path: no prologue text is built for a known shape)
hipFunction_t jit_function_for(const char* kernel, const ScanParams& p, const std::string& extra = std::string());

}  // namespace bqg
