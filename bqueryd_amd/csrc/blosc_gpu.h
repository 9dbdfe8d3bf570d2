// blosc_gpu.h -- task lists of the on-GPU blosc1 decode (k_blosc.hip), built on the host by
// ingest.hip from the frames' headers.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bqg {

enum { kSplitRaw = -1, kSplitBloscLz = 0, kSplitLz4 = 1 };

// one compressed stream -> dsize bytes at device address dst
struct BloscSplit {
  uint64_t src;    // offset of the stream in the compressed staging buffer
  uint64_t dst;    // device address of its output
  uint32_t csize;  // compressed bytes
  uint32_t dsize;  // decoded bytes
  int32_t codec;   // kSplitRaw / kSplitBloscLz / kSplitLz4
  int32_t pad;
};

// one byte-shuffled block: device address tmp (typesize planes) -> dst (elements)
struct BloscBlock {
  uint64_t tmp;
  uint64_t dst;
  uint32_t bytes;
  uint32_t typesize;
};

// pad the compressed staging buffer by this many bytes (the decode reads whole windows)
constexpr size_t kBloscPad = 2048;

void launch_blosc_decode(const unsigned char* comp, const BloscSplit* tasks, int ntasks, unsigned int* bad,
                         hipStream_t st);
void launch_blosc_unshuffle(const BloscBlock* blocks, int nblocks, hipStream_t st);

}  // namespace bqg
