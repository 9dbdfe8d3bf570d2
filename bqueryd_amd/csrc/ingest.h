// ingest.h -- host-side bcolz carray -> HBM column loader (ingest.hip), used by
// bqg_table_load_carray (api.hip).
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

namespace bqg {

struct IngestJob {
  int device;              // HIP device of the destination column
  void* dev_dst;           // device column (>= nrows * itemsize bytes)
  std::string carray_dir;  // bcolz carray rootdir (holds data/__<i>.blp)
  int64_t nrows;           // items of the carray
  int itemsize;            // bytes per item
  int64_t chunklen;        // items per chunk (meta/storage "chunklen")
  int nthreads;            // host file-read / decode threads (<= 0: 8)
  bool device_decode;      // decode the blosc frames on the GPU (ingest_carray_device)
  hipStream_t stream;      // the device decode's stream (the context's)
};

// Reusable per-worker resources (HIP stream, two page-locked staging buffers, their events):
// created on first use and kept by the context, so repeated ingests pay no pinned allocation.
struct IngestWorker {
  hipStream_t stream = nullptr;
  void* pinned[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  size_t cap = 0;
};
// Staging of the on-GPU decode, double-buffered by batch: page-locked compressed bytes + task
// lists, their device copy, and the shuffled-block scratch.
struct DecodeSlot {
  void* host = nullptr;  // page-locked: compressed chunk files, then the task lists
  size_t host_cap = 0;
  void* dev = nullptr;   // device copy of `host`
  size_t dev_cap = 0;
  void* tmp = nullptr;   // device: decoded byte-shuffled blocks before the un-shuffle
  size_t tmp_cap = 0;
  hipEvent_t copied = nullptr;  // the slot's host-to-device copy has finished (host reusable)
  hipEvent_t done = nullptr;    // the slot's kernels have finished (device buffers reusable)
  hipStream_t stream = nullptr; // the slot's decode kernels: batches decode concurrently
};
constexpr int kDecodeSlots = 3;
struct IngestPool {
  int device = -1;
  std::vector<IngestWorker> workers;
  DecodeSlot slots[kDecodeSlots];
  hipStream_t copy_stream = nullptr;  // host-to-device copies of the batches, in order
  unsigned int* bad = nullptr;  // device flag: a split failed to decode
  ~IngestPool();
};

struct IngestStats {
  int64_t chunks = 0;
  int64_t compressed_bytes = 0;
  int64_t bytes = 0;
  int threads = 0;
  int64_t device_splits = 0;     // streams decoded on the GPU
  int64_t host_fallback = 0;     // chunks the GPU decoder does not handle (host libblosc)
};

// Decodes every chunk into dev_dst; returns 0, or -1 with a message in err.  Synchronous:
// the column is complete in HBM when it returns.
int ingest_carray(const IngestJob& job, IngestPool& pool, IngestStats* stats, std::string& err);

// The same with the frames decoded on the GPU (k_blosc.hip): host threads only read the chunk
// files into page-locked memory; the compressed bytes cross PCIe; BloscLZ and LZ4 streams (the
// bcolz defaults) and byte shuffle are decoded by kernels; chunks with another codec, bit
// shuffle or a short last frame are decoded by host libblosc as in ingest_carray.
int ingest_carray_device(const IngestJob& job, IngestPool& pool, IngestStats* stats, std::string& err);
// Several columns at once (one table's, one device and stream): the chunks of all of them form
// one sequence of batches, so one column's file reads overlap the previous one's kernels.
int ingest_carrays_device(const std::vector<IngestJob>& jobs, IngestPool& pool, std::vector<IngestStats>& stats,
                          std::string& err);

}  // namespace bqg
