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
#include <chrono>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "blosc_gpu.h"
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

// drops the on-GPU decode's staging (its streams' work first)
void release_decode(IngestPool& pool) {
  if (pool.copy_stream) (void)hipStreamSynchronize(pool.copy_stream);
  for (DecodeSlot& d : pool.slots)
    if (d.stream) (void)hipStreamSynchronize(d.stream);
  for (DecodeSlot& d : pool.slots) {
    if (d.host) (void)hipHostFree(d.host);
    if (d.dev) (void)hipFree(d.dev);
    if (d.tmp) (void)hipFree(d.tmp);
    if (d.copied) (void)hipEventDestroy(d.copied);
    if (d.done) (void)hipEventDestroy(d.done);
    if (d.stream) (void)hipStreamDestroy(d.stream);
    d = DecodeSlot();
  }
  if (pool.bad) (void)hipFree(pool.bad);
  pool.bad = nullptr;
  if (pool.copy_stream) (void)hipStreamDestroy(pool.copy_stream);
  pool.copy_stream = nullptr;
}

IngestPool::~IngestPool() {
  release_decode(*this);
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

// ---------------------------------------------------------------------------------------
// On-GPU decode.  Per batch of chunks (about kBatchBytes decoded): host threads pread the
// chunk files into a page-locked buffer (16-byte aligned frames), the host parses the frame
// headers into split / block task lists, one DMA carries the compressed bytes and the tasks,
// k_blosc_decode writes every stream to its place in the column (byte-shuffled blocks to a
// scratch buffer first) and k_blosc_unshuffle finishes those.  Two slots alternate, so the
// file reads of batch b+1 overlap the copy and kernels of batch b.

namespace {

// decoded bytes per batch (BQGPU_INGEST_BATCH_MB overrides; tools/bench_ingest.py)
size_t batch_bytes() {
  static const size_t b = [] {
    const char* e = getenv("BQGPU_INGEST_BATCH_MB");
    const long mb = e ? atol(e) : 256;
    return (size_t)(mb > 0 ? mb : 256) << 20;
  }();
  return b;
}

bool grow_host(void*& p, size_t& cap, size_t want) {
  if (cap >= want) return true;
  if (p) (void)hipHostFree(p);
  p = nullptr;
  cap = 0;
  want += want / 4;
  if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
    p = nullptr;
    return false;
  }
  cap = want;
  return true;
}

bool grow_dev(void*& p, size_t& cap, size_t want) {
  if (cap >= want) return true;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  want += want / 4;
  if (hipMalloc(&p, want) != hipSuccess) {
    p = nullptr;
    return false;
  }
  cap = want;
  return true;
}

// host libblosc decode of one chunk file already in memory, `want` bytes to dst (synchronous)
bool host_decode_chunk(const BloscApi& bl, const unsigned char* file, size_t chunk_bytes, size_t want, void* dst,
                       hipStream_t st, std::vector<unsigned char>& buf, std::string& err) {
  buf.resize(chunk_bytes + kBloscHeader);
  const int got = bl.decompress_ctx(file + kBloscpackHeader, buf.data(), buf.size(), 1);
  if (got < 0 || (size_t)got < want) {
    err = "blosc decompression failed";
    return false;
  }
  if (hipMemcpyAsync(dst, buf.data(), want, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    err = "host-to-device copy failed";
    return false;
  }
  return true;
}

}  // namespace

int ingest_carrays_device(const std::vector<IngestJob>& jobs, IngestPool& pool, std::vector<IngestStats>& stats,
                          std::string& err) {
  stats.assign(jobs.size(), IngestStats());
  if (jobs.empty()) return 0;
  // every chunk of every column, in order: batches may span columns, so the file reads of
  // one column overlap the kernels of the previous one
  struct ChunkRef {
    int job;
    int64_t index;
  };
  std::vector<ChunkRef> chunks;
  std::vector<size_t> chunk_bytes(jobs.size());
  for (size_t j = 0; j < jobs.size(); ++j) {
    const IngestJob& job = jobs[j];
    if (job.nrows < 0 || job.itemsize <= 0 || job.chunklen <= 0) {
      err = "bad carray geometry";
      return -1;
    }
    chunk_bytes[j] = (size_t)job.chunklen * (size_t)job.itemsize;
    if (chunk_bytes[j] > (size_t)INT32_MAX) {
      err = "chunk larger than a blosc1 frame";
      return -1;
    }
    const int64_t n = job.nrows ? (job.nrows + job.chunklen - 1) / job.chunklen : 0;
    for (int64_t i = 0; i < n; ++i) chunks.push_back({(int)j, i});
    stats[j].chunks = n;
    stats[j].bytes = job.nrows * job.itemsize;
    stats[j].threads = job.nthreads > 0 ? job.nthreads : 8;
  }
  if (chunks.empty()) return 0;
  const IngestJob& job0 = jobs[0];
  if (pool.device != job0.device) {
    // resources of another device: drop them (re-created below)
    pool.workers.clear();
    release_decode(pool);
    pool.device = job0.device;
  }
  if (!pool.copy_stream && hipStreamCreateWithFlags(&pool.copy_stream, hipStreamNonBlocking) != hipSuccess) {
    err = "ingest: HIP stream creation failed";
    return -1;
  }
  for (DecodeSlot& d : pool.slots)
    if ((!d.done && hipEventCreateWithFlags(&d.done, hipEventDisableTiming) != hipSuccess) ||
        (!d.copied && hipEventCreateWithFlags(&d.copied, hipEventDisableTiming) != hipSuccess) ||
        (!d.stream && hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess)) {
      err = "ingest: HIP event / stream creation failed";
      return -1;
    }
  hipStream_t cs = pool.copy_stream;
  // every exit waits for the call's copies and kernels: an error return must not leave a
  // kernel running that could still raise `bad` during the next call
  struct Drain {
    IngestPool& p;
    ~Drain() {
      if (p.copy_stream) (void)hipStreamSynchronize(p.copy_stream);
      for (DecodeSlot& d : p.slots)
        if (d.stream) (void)hipStreamSynchronize(d.stream);
    }
  } drain{pool};
  if (!pool.bad && hipMalloc(&pool.bad, sizeof(unsigned int)) != hipSuccess) {
    pool.bad = nullptr;
    err = "ingest: device allocation failed";
    return -1;
  }
  // on the copy stream: every decode kernel follows its batch's copy, so this clear too
  if (hipMemsetAsync(pool.bad, 0, sizeof(unsigned int), cs) != hipSuccess) {
    err = "ingest: device memset failed";
    return -1;
  }
  const int nthreads = job0.nthreads > 0 ? job0.nthreads : 8;
  // BQGPU_INGEST_TRACE=1: per-batch host phase times on stderr (tools/bench_ingest.py)
  static const bool trace = getenv("BQGPU_INGEST_TRACE") != nullptr;
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); };
  std::vector<BloscSplit> splits;
  std::vector<BloscBlock> blocks;
  std::vector<ChunkFile> files;
  std::vector<unsigned char> hostbuf;
  auto chunk_path = [&](int j, int64_t i) {
    char name[64];
    snprintf(name, sizeof(name), "/data/__%lld.blp", (long long)i);
    return jobs[j].carray_dir + name;
  };

  for (size_t c0 = 0, b = 0; c0 < chunks.size(); ++b) {
    // the batch: chunks up to kBatchBytes decoded (at least one)
    size_t c1 = c0, batch_out = 0;
    while (c1 < chunks.size() && (c1 == c0 || batch_out + chunk_bytes[chunks[c1].job] <= batch_bytes()))
      batch_out += chunk_bytes[chunks[c1++].job];
    // three slots in turn: batch b's file reads overlap batch b-1's copy and b-2's kernels
    DecodeSlot& slot = pool.slots[b % kDecodeSlots];
    hipStream_t st = slot.stream;
    const clk::time_point t_wait = clk::now();
    if (hipEventSynchronize(slot.copied) != hipSuccess) {  // the slot's host buffer is free
      err = "ingest: HIP event wait failed";
      return -1;
    }
    const double wait_ms = ms_since(t_wait);
    const clk::time_point t_read = clk::now();
    // file sizes -> 16-byte aligned places in the slot's host buffer
    files.clear();
    size_t total = 0;
    for (size_t c = c0; c < c1; ++c) {
      struct stat sb;
      const std::string path = chunk_path(chunks[c].job, chunks[c].index);
      if (stat(path.c_str(), &sb) != 0) {
        err = "ingest: cannot open " + path;
        return -1;
      }
      files.push_back({chunks[c].job, chunks[c].index, total, (size_t)sb.st_size});
      total += ((size_t)sb.st_size + 15) & ~(size_t)15;
    }
    const size_t comp_bytes = total + kBloscPad;
    // device buffers of the slot are reallocated only once its previous kernels are done
    if ((slot.dev_cap < comp_bytes || slot.tmp_cap < batch_out) && hipEventSynchronize(slot.done) != hipSuccess) {
      err = "ingest: HIP event wait failed";
      return -1;
    }
    // sized once for a full batch (page-locked allocations cost ~0.1 ms per MB): compressed
    // bytes are at most the decoded bytes plus the frame headers and the alignment
    // (sized for the batch's decoded bytes, so a small call does not pin a full batch)
    const size_t slot_bytes = std::max(comp_bytes, batch_out + batch_out / 16 + kBloscPad);
    if (!grow_host(slot.host, slot.host_cap, slot_bytes) || !grow_dev(slot.dev, slot.dev_cap, slot_bytes)) {
      err = "ingest: staging allocation failed";
      return -1;
    }
    unsigned char* hbase = static_cast<unsigned char*>(slot.host);
    memset(hbase + total, 0, kBloscPad);
    // parallel reads (host threads do nothing else)
    {
      std::atomic<size_t> next{0};
      std::atomic<bool> failed{false};
      std::mutex mu;
      std::string first;
      auto reader = [&] {
        for (;;) {
          const size_t k = next.fetch_add(1);
          if (k >= files.size() || failed.load(std::memory_order_relaxed)) return;
          const ChunkFile& f = files[k];
          const std::string path = chunk_path(f.job, f.index);
          const int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
          size_t got = 0;
          if (fd >= 0) {
            while (got < f.size) {
              const ssize_t n = pread(fd, hbase + f.off + got, f.size - got, (off_t)got);
              if (n <= 0) break;
              got += (size_t)n;
            }
            close(fd);
          }
          if (got != f.size) {
            std::lock_guard<std::mutex> lk(mu);
            if (first.empty()) first = (fd < 0 ? "ingest: cannot open " : "ingest: short read of ") + path;
            failed = true;
            return;
          }
        }
      };
      const int nt = (int)std::min<size_t>((size_t)nthreads, files.size());
      std::vector<std::thread> th;
      for (int t = 1; t < nt; ++t) th.emplace_back(reader);
      reader();
      for (std::thread& t : th) t.join();
      if (failed) {
        err = first;
        return -1;
      }
    }
    const double read_ms = ms_since(t_read);
    const clk::time_point t_plan = clk::now();
    // tasks (byte-shuffled blocks decode into the slot's scratch, then un-shuffle)
    if (!grow_dev(slot.tmp, slot.tmp_cap, batch_out)) {
      err = "ingest: shuffle scratch allocation failed";
      return -1;
    }
    splits.clear();
    blocks.clear();
    std::vector<size_t> fallback;
    uint64_t tmp_at = reinterpret_cast<uint64_t>(slot.tmp);
    for (size_t k = 0; k < files.size(); ++k) {
      const ChunkFile& f = files[k];
      const IngestJob& job = jobs[f.job];
      const size_t cb = chunk_bytes[f.job];
      const size_t want = (size_t)std::min<int64_t>(job.chunklen, job.nrows - f.index * job.chunklen) * job.itemsize;
      const uint64_t dst = reinterpret_cast<uint64_t>(job.dev_dst) + (uint64_t)f.index * cb;
      const size_t ns0 = splits.size();
      std::string e;
      const Plan pl = plan_chunk(hbase + f.off, f, dst, tmp_at, want, cb, job.carray_dir, splits, blocks, e);
      tmp_at += cb;
      if (pl == Plan::kError) {
        err = "ingest: " + e;
        return -1;
      }
      if (pl == Plan::kFallback) fallback.push_back(k);
      stats[f.job].compressed_bytes += (int64_t)f.size;
      stats[f.job].device_splits += (int64_t)(splits.size() - ns0);
    }
    // heaviest streams first (compressed size; stored-raw copies last): the long serial decodes
    // start in the first dispatch wave, spread over the CUs, instead of doubling up on SIMDs
    std::stable_sort(splits.begin(), splits.end(), [](const BloscSplit& x, const BloscSplit& y) {
      const uint32_t kx = x.codec == kSplitRaw ? 0 : x.csize, ky = y.codec == kSplitRaw ? 0 : y.csize;
      return kx > ky;
    });
    // task lists after the compressed bytes, one DMA for all
    const size_t split_off = (comp_bytes + 15) & ~(size_t)15;
    const size_t block_off = split_off + splits.size() * sizeof(BloscSplit);
    const size_t all = block_off + blocks.size() * sizeof(BloscBlock);
    if (all > slot.host_cap || all > slot.dev_cap) {
      // tasks did not fit the slack: grow both, keeping the compressed bytes
      if (hipEventSynchronize(slot.done) != hipSuccess) {
        err = "ingest: HIP event wait failed";
        return -1;
      }
      std::vector<unsigned char> keep(hbase, hbase + comp_bytes);
      if (!grow_host(slot.host, slot.host_cap, all) || !grow_dev(slot.dev, slot.dev_cap, all)) {
        err = "ingest: staging allocation failed";
        return -1;
      }
      hbase = static_cast<unsigned char*>(slot.host);
      memcpy(hbase, keep.data(), comp_bytes);
    }
    if (!splits.empty()) memcpy(hbase + split_off, splits.data(), splits.size() * sizeof(BloscSplit));
    if (!blocks.empty()) memcpy(hbase + block_off, blocks.data(), blocks.size() * sizeof(BloscBlock));
    unsigned char* dbase = static_cast<unsigned char*>(slot.dev);
    // copy stream: after the slot's previous kernels; decode stream: after this copy
    if (hipStreamWaitEvent(cs, slot.done, 0) != hipSuccess ||
        hipMemcpyAsync(dbase, hbase, all, hipMemcpyHostToDevice, cs) != hipSuccess ||
        hipEventRecord(slot.copied, cs) != hipSuccess || hipStreamWaitEvent(st, slot.copied, 0) != hipSuccess) {
      err = "ingest: host-to-device copy failed";
      return -1;
    }
    launch_blosc_decode(dbase, reinterpret_cast<const BloscSplit*>(dbase + split_off), (int)splits.size(), pool.bad,
                        st);
    launch_blosc_unshuffle(reinterpret_cast<const BloscBlock*>(dbase + block_off), (int)blocks.size(), st);
    if (hipGetLastError() != hipSuccess || hipEventRecord(slot.done, st) != hipSuccess) {
      err = "ingest: blosc decode launch failed";
      return -1;
    }
    if (trace)
      fprintf(stderr, "[ingest] batch %zu: %zu chunks, %.1f MB -> %.1f MB, %zu splits; wait %.2f ms, read %.2f ms, plan+launch %.2f ms\n",
              b, c1 - c0, total / 1e6, batch_out / 1e6, splits.size(), wait_ms, read_ms, ms_since(t_plan));
    for (size_t k : fallback) {
      const ChunkFile& f = files[k];
      const IngestJob& job = jobs[f.job];
      const BloscApi& bl = blosc_api();
      if (!bl.err.empty()) {
        err = bl.err;
        return -1;
      }
      const size_t cb = chunk_bytes[f.job];
      const size_t want = (size_t)std::min<int64_t>(job.chunklen, job.nrows - f.index * job.chunklen) * job.itemsize;
      std::string e;
      if (!host_decode_chunk(bl, hbase + f.off, cb, want, static_cast<unsigned char*>(job.dev_dst) + (size_t)f.index * cb,
                             st, hostbuf, e)) {
        err = "ingest: chunk " + std::to_string(f.index) + " of " + job.carray_dir + ": " + e;
        return -1;
      }
      stats[f.job].host_fallback += 1;
    }
    c0 = c1;
  }
  unsigned int bad = 0;
  const clk::time_point t_tail = clk::now();
  bool ok = hipStreamSynchronize(cs) == hipSuccess;
  for (DecodeSlot& d : pool.slots) ok = ok && hipStreamSynchronize(d.stream) == hipSuccess;
  if (!ok || hipMemcpy(&bad, pool.bad, sizeof(bad), hipMemcpyDeviceToHost) != hipSuccess) {
    err = "ingest: device decode failed";
    return -1;
  }
  if (trace) fprintf(stderr, "[ingest] tail wait %.2f ms\n", ms_since(t_tail));
  if (bad) {
    std::string dirs;
    for (const IngestJob& j : jobs) dirs += (dirs.empty() ? "" : ", ") + j.carray_dir;
    err = "ingest: on-GPU blosc decode of " + dirs + " failed (corrupt stream)";
    return -1;
  }
  return 0;
}

int ingest_carray_device(const IngestJob& job, IngestPool& pool, IngestStats* stats, std::string& err) {
  std::vector<IngestStats> st;
  const int rc = ingest_carrays_device(std::vector<IngestJob>{job}, pool, st, err);
  if (rc == 0 && stats) *stats = st[0];
  return rc;
}

}  // namespace bqg
