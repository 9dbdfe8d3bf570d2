// blosc_gpu.h -- launches of the on-GPU blosc1 decode (k_blosc.hip); its task lists are built on
// the host by blosc_plan.h from the frames' headers.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "blosc_plan.h"

namespace bqg {

// pad the compressed staging buffer by this many bytes (the decode reads whole windows)
constexpr size_t kBloscPad = 2048;

void launch_blosc_decode(const unsigned char* comp, const BloscSplit* tasks, int ntasks, unsigned int* bad,
                         hipStream_t st);
void launch_blosc_unshuffle(const BloscBlock* blocks, int nblocks, hipStream_t st);

}  // namespace bqg
