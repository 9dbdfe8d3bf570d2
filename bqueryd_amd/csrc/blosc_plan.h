// blosc_plan.h -- host-side parsing of bcolz chunk files (bloscpack header + one blosc1
// frame) into the on-GPU decoder's task lists (k_blosc.hip), and the task records themselves.
//
// Pure host C++ (no HIP): ingest.hip includes it through blosc_gpu.h, and
// tests/blosc_plan_check.cpp compiles it with g++ -fsanitize=address,undefined and feeds it
// truncated, oversized and corrupted headers -- every malformed file must come back as an
// error or a host fallback, never as an out-of-bounds read or a task that reaches outside the
// file / the chunk's place in the column.  The frame layout is c-blosc 1.x's (the format bcolz
// writes for the chunks bqueryd's worker opens, bqueryd/worker.py:291): a 16-byte header
// {version, versionlz, flags, typesize, int32 nbytes, int32 blocksize, int32 cbytes}, an int32
// start offset per block, then per block `nsplits` streams of {int32 csize, csize bytes}.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

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

constexpr size_t kBloscpackHeader = 16;         // 'blpk', version, 3 reserved bytes, int64 nchunks
constexpr size_t kBloscHeader = 16;             // the blosc1 frame header
constexpr size_t kRawPiece = size_t(64) << 10;  // stored-raw bytes per copy task

inline int32_t le32(const unsigned char* p) {
  int32_t v;
  memcpy(&v, p, 4);
  return v;
}

struct ChunkFile {
  int job;      // column (index into the jobs)
  int64_t index;
  size_t off;   // of the file in the slot's host buffer
  size_t size;  // file bytes
};

enum class Plan { kTasks, kFallback, kError };

// Task lists for one chunk file (bloscpack header + blosc1 frame) already in the host buffer
// at f.off.  dst / tmp: the chunk's place in the column / in the slot's shuffle scratch.
inline Plan plan_chunk(const unsigned char* file, const ChunkFile& f, uint64_t dst, uint64_t tmp, size_t want,
                size_t chunk_bytes, const std::string& dir, std::vector<BloscSplit>& splits,
                std::vector<BloscBlock>& blocks, std::string& err) {
  const std::string where = "chunk " + std::to_string(f.index) + " of " + dir;
  if (f.size < kBloscpackHeader + kBloscHeader || memcmp(file, "blpk", 4) != 0) {
    err = where + " is not a bloscpack chunk";
    return Plan::kError;
  }
  const unsigned char* frame = file + kBloscpackHeader;
  const size_t avail = f.size - kBloscpackHeader;
  const unsigned flags = frame[2], ts = frame[3];
  const int64_t nbytes = le32(frame + 4), blocksize = le32(frame + 8), cbytes = le32(frame + 12);
  if (cbytes < (int64_t)kBloscHeader || (size_t)cbytes > avail || nbytes < (int64_t)want ||
      nbytes > (int64_t)chunk_bytes) {
    err = where + ": frame holds " + std::to_string(nbytes) + " bytes, expected " + std::to_string(want);
    return Plan::kError;
  }
  if ((size_t)nbytes != want) return Plan::kFallback;  // a padded last frame: host copies `want`
  if (nbytes == 0) return Plan::kTasks;
  // flag bits the device decoder does not implement go to host libblosc: 0x8 (the delta
  // filter of newer c-blosc 1.x) and the reserved 0x40 / 0x80 bits of non-codec use
  if (flags & 0x8) return Plan::kFallback;
  const uint64_t frame_src = f.off + kBloscpackHeader;
  if (flags & 0x2) {  // memcpyed: the items follow the header as they are
    if (kBloscHeader + (size_t)nbytes > (size_t)cbytes) {
      err = where + ": truncated memcpyed frame";
      return Plan::kError;
    }
    for (size_t k = 0; k < (size_t)nbytes; k += kRawPiece) {
      const uint32_t n = (uint32_t)std::min(kRawPiece, (size_t)nbytes - k);
      splits.push_back({frame_src + kBloscHeader + k, dst + k, n, n, kSplitRaw, 0});
    }
    return Plan::kTasks;
  }
  const int codec = (int)(flags >> 5);
  if ((flags & 0x4) || (codec != kSplitBloscLz && codec != kSplitLz4) || ts == 0) return Plan::kFallback;
  if (blocksize <= 0) {
    err = where + ": bad blocksize";
    return Plan::kError;
  }
  const int64_t nblocks = (nbytes + blocksize - 1) / blocksize;
  const int64_t leftover = nbytes % blocksize;
  if ((int64_t)kBloscHeader + 4 * nblocks > cbytes) {
    err = where + ": truncated block table";
    return Plan::kError;
  }
  const bool shuffle = (flags & 0x1) && ts > 1;
  const uint64_t out = shuffle ? tmp : dst;
  const size_t splits0 = splits.size(), blocks0 = blocks.size();
  for (int64_t b = 0; b < nblocks; ++b) {
    const bool last_partial = b == nblocks - 1 && leftover != 0;
    const int64_t bsize = last_partial ? leftover : blocksize;
    const int64_t nsplits =
        (!(flags & 0x10) && ts <= 16 && blocksize / (int64_t)ts >= 128 && !last_partial) ? (int64_t)ts : 1;
    if (bsize % nsplits != 0) {
      splits.resize(splits0);
      blocks.resize(blocks0);
      return Plan::kFallback;
    }
    const int64_t neblock = bsize / nsplits;
    int64_t p = le32(frame + kBloscHeader + 4 * b);
    const uint64_t boff = (uint64_t)(b * blocksize);
    for (int64_t j = 0; j < nsplits; ++j) {
      if (p < 0 || p + 4 > cbytes) {
        err = where + ": block " + std::to_string(b) + " out of the frame";
        return Plan::kError;
      }
      const int64_t csize = le32(frame + p);
      p += 4;
      if (csize < 0 || p + csize > cbytes) {
        err = where + ": block " + std::to_string(b) + " out of the frame";
        return Plan::kError;
      }
      splits.push_back({frame_src + (uint64_t)p, out + boff + (uint64_t)(j * neblock), (uint32_t)csize,
                        (uint32_t)neblock, csize == neblock ? (int32_t)kSplitRaw : (int32_t)codec, 0});
      p += csize;
    }
    if (shuffle) blocks.push_back({tmp + boff, dst + boff, (uint32_t)bsize, ts});
  }
  return Plan::kTasks;
}

}  // namespace bqg
