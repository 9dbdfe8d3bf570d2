// ctx_internal.h -- what the library's other host translation units (comm.hip) need from a
// context, without exposing its layout: its device, its stream, and the per-context error
// message that bqg_last_error returns.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

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
// comm.hip: lower a library table's row count to n <= its rows (the merge emits into a table
// sized by an upper bound); the column memory is kept
int bqg_internal_table_set_rows(bqg_table* t, int64_t n);
// a host result of n rows of the given dtypes in one pinned block of the context's pool
// (device-mapped); cols[j] receives column j's host address (BQG_OK or an error code, with
// the context's message set)
int bqg_internal_host_result(bqg_ctx* c, int64_t n, const std::vector<int32_t>& dts, std::vector<void*>& cols,
                             bqg_result** out);
