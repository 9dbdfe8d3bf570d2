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
  int nthreads;            // host decode threads (<= 0: 8)
};

// Reusable per-worker resources (HIP stream, two page-locked staging buffers, their events):
// created on first use and kept by the context, so repeated ingests pay no pinned allocation.
struct IngestWorker {
  hipStream_t stream = nullptr;
  void* pinned[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  size_t cap = 0;
};
struct IngestPool {
  int device = -1;
  std::vector<IngestWorker> workers;
  ~IngestPool();
};

struct IngestStats {
  int64_t chunks = 0;
  int64_t compressed_bytes = 0;
  int64_t bytes = 0;
  int threads = 0;
};

// Decodes every chunk into dev_dst; returns 0, or -1 with a message in err.  Synchronous:
// the column is complete in HBM when it returns.
int ingest_carray(const IngestJob& job, IngestPool& pool, IngestStats* stats, std::string& err);

}  // namespace bqg
