// ingest.hip -- cold-path ingest of one bcolz carray straight into an HBM column.
//
// bqueryd's worker opens each shard with bquery.ctable(rootdir, mode='r', auto_cache=True)
// (bqueryd/worker.py:291) and bquery/bcolz then decompress every touched chunk on ONE thread
// (bcolz.set_nthreads(1), worker.py:40).  Here the chunks of a column are spread over host
// threads; each thread reads a chunk file, blosc-decompresses it straight into one of its
// two page-locked staging buffers and DMAs the buffer to the chunk's place in the device
// column with hipMemcpyAsync on the thread's own stream, then decodes its next chunk into the
// other buffer while that copy runs (double buffering per thread).
//
// On-disk layout [ext-bcolz, unverified: bcolz is not vendored, SURVEY.md §8c]:
// <carray>/data/__<i>.blp = 16-byte bloscpack header ('blpk', version, 3 reserved bytes,
// int64 nchunks) + one blosc1 frame of `chunklen` items (the last chunk: the remainder).
// The blosc frames are decoded by the system c-blosc 1.x (libblosc.so.1, loaded with dlopen:
// every codec bcolz can write -- blosclz / lz4 / zstd / zlib / snappy -- decodes).
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ingest.h"

namespace bqg {
namespace {

struct BloscApi {
  int (*decompress_ctx)(const void* src, void* dest, size_t destsize, int nthreads) = nullptr;
  void (*cbuffer_sizes)(const void* cbuffer, size_t* nbytes, size_t* cbytes, size_t* blocksize) = nullptr;
  std::string err;
};

const BloscApi& blosc_api() {
  static BloscApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    std::vector<std::string> cands;
    if (const char* ev = getenv("BQGPU_BLOSC")) cands.push_back(ev);
    for (const char* c : {"libblosc.so.1", "/opt/conda/lib/libblosc.so.1", "libblosc.so", "/opt/conda/lib/libblosc.so"})
      cands.push_back(c);
    void* h = nullptr;
    for (const std::string& c : cands)
      if ((h = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!h) {
      api.err = "libblosc (c-blosc 1.x) not found (set BQGPU_BLOSC)";
      return;
    }
    api.decompress_ctx = reinterpret_cast<int (*)(const void*, void*, size_t, int)>(dlsym(h, "blosc_decompress_ctx"));
    api.cbuffer_sizes =
        reinterpret_cast<void (*)(const void*, size_t*, size_t*, size_t*)>(dlsym(h, "blosc_cbuffer_sizes"));
    if (!api.decompress_ctx || !api.cbuffer_sizes) api.err = "libblosc lacks blosc_decompress_ctx / blosc_cbuffer_sizes";
  });
  return api;
}

constexpr size_t kBloscpackHeader = 16;
constexpr size_t kBloscHeader = 16;

bool read_file(const std::string& path, std::vector<unsigned char>& buf, std::string& err) {
  const int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    err = "cannot open " + path;
    return false;
  }
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    err = "cannot stat " + path;
    return false;
  }
  buf.resize((size_t)st.st_size);
  size_t got = 0;
  while (got < buf.size()) {
    const ssize_t n = pread(fd, buf.data() + got, buf.size() - got, (off_t)got);
    if (n <= 0) {
      close(fd);
      err = "short read of " + path;
      return false;
    }
    got += (size_t)n;
  }
  close(fd);
  return true;
}

}  // namespace

IngestPool::~IngestPool() {
  for (IngestWorker& w : workers) {
    if (w.stream) (void)hipStreamSynchronize(w.stream);
    for (int k = 0; k < 2; ++k) {
      if (w.ev[k]) (void)hipEventDestroy(w.ev[k]);
      if (w.pinned[k]) (void)hipHostFree(w.pinned[k]);
    }
    if (w.stream) (void)hipStreamDestroy(w.stream);
  }
}

namespace {
// worker resources with staging buffers of at least `bytes` (called on the calling thread)
bool prepare_workers(IngestPool& pool, int device, int n, size_t bytes, std::string& err) {
  if (pool.device != device) {
    pool.workers.clear();
    pool.device = device;
  }
  while ((int)pool.workers.size() < n) pool.workers.emplace_back();
  for (int i = 0; i < n; ++i) {
    IngestWorker& w = pool.workers[i];
    if (!w.stream && hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking) != hipSuccess) {
      err = "ingest: HIP stream creation failed";
      return false;
    }
    for (int k = 0; k < 2; ++k)
      if (!w.ev[k] && hipEventCreateWithFlags(&w.ev[k], hipEventDisableTiming) != hipSuccess) {
        err = "ingest: HIP event creation failed";
        return false;
      }
    if (w.cap < bytes) {
      for (int k = 0; k < 2; ++k) {
        if (w.pinned[k]) {
          (void)hipEventSynchronize(w.ev[k]);
          (void)hipHostFree(w.pinned[k]);
          w.pinned[k] = nullptr;
        }
        if (hipHostMalloc(&w.pinned[k], bytes, hipHostMallocDefault) != hipSuccess) {
          w.pinned[k] = nullptr;
          w.cap = 0;
          err = "ingest: pinned staging allocation failed";
          return false;
        }
      }
      w.cap = bytes;
    }
  }
  return true;
}
}  // namespace

int ingest_carray(const IngestJob& job, IngestPool& pool, IngestStats* stats, std::string& err) {
  const BloscApi& bl = blosc_api();
  if (!bl.err.empty()) {
    err = bl.err;
    return -1;
  }
  if (job.nrows < 0 || job.itemsize <= 0 || job.chunklen <= 0) {
    err = "bad carray geometry";
    return -1;
  }
  const int64_t nchunks = job.nrows ? (job.nrows + job.chunklen - 1) / job.chunklen : 0;
  if (nchunks == 0) return 0;
  const size_t chunk_bytes = (size_t)job.chunklen * (size_t)job.itemsize;
  int nthreads = job.nthreads > 0 ? job.nthreads : 8;
  nthreads = (int)std::min<int64_t>(nthreads, nchunks);

  if (!prepare_workers(pool, job.device, nthreads, chunk_bytes + kBloscHeader, err)) return -1;

  std::atomic<int64_t> next{0};
  std::atomic<bool> failed{false};
  std::atomic<int64_t> comp_bytes{0};
  std::mutex mu;
  std::string first_err;
  auto set_err = [&](const std::string& e) {
    std::lock_guard<std::mutex> lk(mu);
    if (first_err.empty()) first_err = e;
    failed = true;
  };

  auto worker = [&](IngestWorker& res) {
    hipStream_t s = res.stream;
    std::vector<unsigned char> file;
    std::string e;
    if (hipSetDevice(job.device) != hipSuccess) {
      set_err("ingest: hipSetDevice failed");
      return;
    }
    int slot = 0;
    while (!failed.load(std::memory_order_relaxed)) {
      const int64_t i = next.fetch_add(1);
      if (i >= nchunks) break;
      char name[64];
      snprintf(name, sizeof(name), "/data/__%lld.blp", (long long)i);
      if (!read_file(job.carray_dir + std::string(name), file, e)) {
        set_err("ingest: " + e);
        break;
      }
      if (file.size() < kBloscpackHeader + kBloscHeader || memcmp(file.data(), "blpk", 4) != 0) {
        set_err("ingest: chunk " + std::to_string(i) + " of " + job.carray_dir + " is not a bloscpack chunk");
        break;
      }
      const unsigned char* frame = file.data() + kBloscpackHeader;
      size_t nbytes = 0, cbytes = 0, bsize = 0;
      bl.cbuffer_sizes(frame, &nbytes, &cbytes, &bsize);
      const int64_t rows_here = std::min<int64_t>(job.chunklen, job.nrows - i * job.chunklen);
      const size_t want = (size_t)rows_here * (size_t)job.itemsize;
      if (cbytes > file.size() - kBloscpackHeader || nbytes < want || nbytes > chunk_bytes) {
        set_err("ingest: chunk " + std::to_string(i) + " of " + job.carray_dir + ": frame holds " +
                std::to_string(nbytes) + " bytes, expected " + std::to_string(want));
        break;
      }
      // the staging buffer's previous copy must have drained before it is overwritten
      if (hipEventSynchronize(res.ev[slot]) != hipSuccess) {
        set_err("ingest: HIP event wait failed");
        break;
      }
      const int got = bl.decompress_ctx(frame, res.pinned[slot], chunk_bytes + kBloscHeader, 1);
      if (got < 0 || (size_t)got != nbytes) {
        set_err("ingest: blosc decompression of chunk " + std::to_string(i) + " of " + job.carray_dir + " failed");
        break;
      }
      unsigned char* dst = static_cast<unsigned char*>(job.dev_dst) + (size_t)i * chunk_bytes;
      if (hipMemcpyAsync(dst, res.pinned[slot], want, hipMemcpyHostToDevice, s) != hipSuccess ||
          hipEventRecord(res.ev[slot], s) != hipSuccess) {
        set_err("ingest: host-to-device copy failed");
        break;
      }
      comp_bytes += (int64_t)file.size();
      slot ^= 1;
    }
    (void)hipStreamSynchronize(s);
  };

  std::vector<std::thread> threads;
  threads.reserve(nthreads);
  for (int t = 0; t < nthreads; ++t) threads.emplace_back(worker, std::ref(pool.workers[t]));
  for (std::thread& t : threads) t.join();
  if (failed) {
    err = first_err;
    return -1;
  }
  if (stats) {
    stats->chunks = nchunks;
    stats->compressed_bytes = comp_bytes.load();
    stats->bytes = (int64_t)job.nrows * job.itemsize;
    stats->threads = nthreads;
  }
  return 0;
}

}  // namespace bqg
