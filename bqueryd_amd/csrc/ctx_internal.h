// ctx_internal.h -- what the library's other host translation units (comm.hip) need from a
// context, without exposing its layout: its device, its stream, and the per-context error
// message that bqg_last_error returns.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/bqgpu.h"

int bqg_internal_device(bqg_ctx* c);
hipStream_t bqg_internal_stream(bqg_ctx* c);
// bqg_enable_timing is on: the merge also waits for each rank's own device work at the end of
// its local phase, so every phase's time is that rank's alone (on a one-GPU rehearsal of
// several ranks, the ranks' kernels would otherwise be charged to the first collective)
bool bqg_internal_timing(bqg_ctx* c);
void bqg_internal_set_error(bqg_ctx* c, const std::string& msg);
// comm.hip: drop the context's RCCL communicator, if any (called by bqg_destroy)
void bqg_internal_comm_release(bqg_ctx* c);
