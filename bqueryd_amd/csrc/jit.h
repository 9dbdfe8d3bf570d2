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
// `async`: a shape in neither the memory nor the disk cache is queued for a background
// compile and nullptr returned (*final_answer = false) -- the caller runs the generic kernel
// this time and gets the specialised one on a later call, so no query waits for hiprtc
hipFunction_t jit_function(const char* kernel, const std::string& spec, bool async = false,
                           bool* final_answer = nullptr);

// jit_function(kernel, jit_spec(p) + extra), looked up first by the binary image of p's
// specialised fields (the per-query path: no prologue text is built for a known shape)
hipFunction_t jit_function_for(const char* kernel, const ScanParams& p, const std::string& extra = std::string(),
                               bool async = false);

// wait until no background compile is queued or running (timeout_ms < 0: no limit); false on
// timeout.  compiled / failed (optional): background compiles finished so far, per outcome.
bool jit_wait(double timeout_ms, int64_t* compiled, int64_t* failed);

}  // namespace bqg
