// comm.hip -- multi-GPU merge of co-located shard results over RCCL (xGMI), C ABI
// bqg_comm_* / bqg_merge* of include/bqgpu.h.
//
// bqueryd merges shard results on the client: every shard's finalized table is appended and
// re-grouped with `sum` of every column ("we can only sum now", bqueryd/rpc.py:164-173).  For
// shards that live on one node's GPUs the same merge runs here, on device buffers:
//   1. local:     this rank's shard tables are concatenated (device to device) and summed by
//                 key (MergeReduce: one hash table, tables in order) -- skipped when the
//                 caller's one table is already reduced (a co-located one-pass groupby);
//   2. partition: every row goes to rank hash(key values) mod nranks (the partition function
//                 of bqg_hash_partition: a pure function of the values, identical on every
//                 rank) -- one stable scatter (k_mpack_*) writes each row straight into its
//                 destination's packed block, whose row counts land on the device;
//   3. exchange:  the [nranks x nranks] row-count matrix (ncclAllGather, then the one host
//                 read of the exchange), then the payload (grouped ncclSend / ncclRecv, one
//                 message per peer and column, self included) straight into the receiving
//                 rank's table columns;
//   4. reduce:    the received rows are summed by key again (MergeReduce, sources in rank
//                 order; keys are disjoint across ranks);
//   5. output:    the reduced partitions travel to rank 0 column by column (grouped send /
//                 recv), straight into the result table, in rank order -- or, when one process
//                 drives every rank and wants host memory (bqg_merge_group_host), each rank
//                 copies its partition straight into its slice of one pinned host result.
// Only the row counts cross to the host (to size buffers).  librccl is loaded with dlopen on
// first use, so libbqgpu itself loads where RCCL is absent; every entry here then fails with
// a message instead.
//
// The merge is built from the library's own public entry points (table create, push) plus the
// pack and reduce kernels (k_misc.hip); this file adds the communicator and the exchange.  It runs any number of
// local ranks from ONE host thread: bqg_merge drives one rank of a multi-process job (one
// process per GPU), bqg_merge_group every rank of a process that owns several GPUs, with the
// collective calls of all of them inside one ncclGroupStart / ncclGroupEnd.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "ctx_internal.h"
#include "kernels.h"
#include "merge_schedule.h"

namespace {

struct CommError {
  int code;
  std::string msg;
};

[[noreturn]] void comm_fail(int code, const std::string& msg) { throw CommError{code, msg}; }

// ------------------------------------------------------------------------------------
// librccl, resolved at first use
// ------------------------------------------------------------------------------------
struct Rccl {
  bool loaded = false;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!h) {
      r.err = std::string("librccl could not be loaded: ") + dlerror();
      return;
    }
    bool ok = true;
    auto sym = [&](const char* name) {
      void* p = dlsym(h, name);
      if (!p) ok = false;
      return p;
    };
    r.GetUniqueId = (decltype(r.GetUniqueId))sym("ncclGetUniqueId");
    r.CommInitRank = (decltype(r.CommInitRank))sym("ncclCommInitRank");
    r.CommInitAll = (decltype(r.CommInitAll))sym("ncclCommInitAll");
    r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
    r.Send = (decltype(r.Send))sym("ncclSend");
    r.Recv = (decltype(r.Recv))sym("ncclRecv");
    r.AllGather = (decltype(r.AllGather))sym("ncclAllGather");
    r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
    r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
    r.GetErrorString = (decltype(r.GetErrorString))sym("ncclGetErrorString");
    if (!ok) r.err = "librccl lacks a required symbol";
    r.loaded = ok;
  });
  if (!r.loaded) comm_fail(BQG_E_UNSUPPORTED, r.err);
  return r;
}

#define NCCLCHECK(x)                                                                         \
  do {                                                                                       \
    ncclResult_t _r = (x);                                                                   \
    if (_r != ncclSuccess)                                                                   \
      comm_fail(BQG_E_HIP, std::string("RCCL error in " #x ": ") + rccl().GetErrorString(_r)); \
  } while (0)

#define HIPCK(x)                                                                              \
  do {                                                                                        \
    hipError_t _e = (x);                                                                      \
    if (_e != hipSuccess) comm_fail(BQG_E_HIP, std::string("HIP error in " #x ": ") + hipGetErrorString(_e)); \
  } while (0)

// growable device buffer (stream-ordered use; freed only at communicator teardown)
struct Buf {
  void* p = nullptr;
  size_t cap = 0;
  void* ensure(size_t bytes) {
    bytes = std::max<size_t>(bytes, 256);
    if (bytes > cap) {
      const size_t c = std::max(bytes, cap + cap / 2);
      if (p) HIPCK(hipFree(p));
      p = nullptr;
      cap = 0;
      if (hipMalloc(&p, c) != hipSuccess) comm_fail(BQG_E_OOM, "device allocation for the merge exchange failed");
      cap = c;
    }
    return p;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

constexpr int kMergePhases = 6;  // bqg_comm_last_phases
struct CommState {
  ncclComm_t comm = nullptr;  // RCCL transport; nullptr = in-process transport (see below)
  int rank = 0, nranks = 1;
  Buf send, scratch, counts;  // packed send blocks, pack scratch, row counts
  Buf reduce;                 // receive-side reduce: hash table, sums, rank bitmap
  void* hcnt = nullptr;       // page-locked staging of the reduce's key count (async D2H)
  void* hcounts() {
    if (!hcnt && hipHostMalloc(&hcnt, 64, hipHostMallocDefault) != hipSuccess) {
      hcnt = nullptr;
      comm_fail(BQG_E_OOM, "pinned staging for the merge counts failed");
    }
    return hcnt;
  }
  double phase_ms[kMergePhases] = {};  // host wall time of this rank's part of the last merge
  // bqg_comm_progress (read from another host thread while a merge runs, e.g. a watchdog
  // naming the collective a hung rank waits in): the phase entered last, -1 between merges
  std::atomic<int32_t> cur_phase{-1};
  std::atomic<int64_t> merges_started{0}, merges_done{0};
  // the shared host result block of bqg_merge_shared_host, page-locked once (hipHostRegister)
  // and kept registered while the caller keeps passing the same block
  void* reg = nullptr;
  size_t reg_bytes = 0;
  void register_host(void* base, size_t bytes) {
    if (reg == base && reg_bytes >= bytes) return;
    if (reg) (void)hipHostUnregister(reg);
    reg = nullptr;
    reg_bytes = 0;
    const hipError_t e = hipHostRegister(base, bytes, hipHostRegisterDefault);
    if (e == hipErrorHostMemoryAlreadyRegistered) {
      (void)hipGetLastError();  // the caller pinned it: use it as it is
      return;
    }
    if (e != hipSuccess) comm_fail(BQG_E_OOM, std::string("hipHostRegister of the shared merge result: ") + hipGetErrorString(e));
    reg = base;
    reg_bytes = bytes;
  }
  // in-process transport: an event on this rank's stream, and (rank 0) the copy descriptors
  // of a transfer step -- page-locked staging, its reuse guarded by desc_ev -- and their
  // device copy
  hipEvent_t ev = nullptr, desc_ev = nullptr;
  void* hdesc = nullptr;
  size_t hdesc_cap = 0;
  Buf ddesc;
};

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

std::mutex g_mu;
std::map<bqg_ctx*, CommState*> g_comms;

CommState* state_of(bqg_ctx* c) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_comms.find(c);
  if (it == g_comms.end()) comm_fail(BQG_E_STATE, "no communicator on this context (bqg_comm_init first)");
  return it->second;
}

void destroy_state(CommState* s) {
  if (!s) return;
  if (s->comm) (void)rccl().CommDestroy(s->comm);
  if (s->comm == nullptr) (void)hipDeviceSynchronize();  // in-process copies may target its buffers
  s->send.release();
  s->scratch.release();
  s->counts.release();
  s->reduce.release();
  s->ddesc.release();
  if (s->hcnt) (void)hipHostFree(s->hcnt);
  if (s->hdesc) (void)hipHostFree(s->hdesc);
  if (s->reg) (void)hipHostUnregister(s->reg);
  if (s->ev) (void)hipEventDestroy(s->ev);
  if (s->desc_ev) (void)hipEventDestroy(s->desc_ev);
  delete s;
}

template <typename F>
int comm_guard(bqg_ctx* ctx, F&& f) {
  try {
    f();
    return BQG_OK;
  } catch (const CommError& e) {
    bqg_internal_set_error(ctx, e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    bqg_internal_set_error(ctx, "host out of memory");
    return BQG_E_OOM;
  }
}

// a public entry point of this library, failing with its message
void ck(bqg_ctx* c, int rc) {
  if (rc != BQG_OK) comm_fail(rc, bqg_last_error(c));
}

size_t dt_size(int dt) {
  switch (dt) {
    case BQG_BOOL: case BQG_I8: case BQG_U8: return 1;
    case BQG_I16: case BQG_U16: return 2;
    case BQG_I32: case BQG_U32: case BQG_F32: return 4;
    default: return 8;
  }
}

size_t align16(size_t n) { return (n + 15) & ~size_t(15); }

int64_t nrows_of(bqg_ctx* c, bqg_table* t) {
  int64_t n = 0;
  ck(c, bqg_table_nrows(t, &n));
  return n;
}

void* col_ptr(bqg_ctx* c, bqg_table* t, int col) {
  void* p = nullptr;
  ck(c, bqg_table_column_ptr(t, col, &p));
  return p;
}

struct TableOwner {  // destroys a library table on scope exit
  bqg_table* t = nullptr;
  TableOwner() = default;
  TableOwner(const TableOwner&) = delete;
  TableOwner& operator=(const TableOwner&) = delete;
  ~TableOwner() { reset(); }
  void reset() {
    if (t) (void)bqg_table_destroy(t);
    t = nullptr;
  }
  bqg_table* release() {
    bqg_table* r = t;
    t = nullptr;
    return r;
  }
};

// Row-concatenation of device tables (device-to-device copies) with statistics computed.
bqg_table* concat_tables(bqg_ctx* c, const std::vector<bqg_table*>& parts, const std::vector<int32_t>& dts) {
  int64_t total = 0;
  for (bqg_table* p : parts) total += nrows_of(c, p);
  TableOwner out;
  ck(c, bqg_table_create(c, total, (int32_t)dts.size(), dts.data(), &out.t));
  int64_t off = 0;
  for (bqg_table* p : parts) {
    const int64_t n = nrows_of(c, p);
    if (n)
      for (int j = 0; j < (int)dts.size(); ++j) ck(c, bqg_push_chunk(out.t, j, col_ptr(c, p, j), n, off));
    off += n;
  }
  // no bqg_table_sync: the copies are ordered on the context's stream before anything that
  // reads the table
  return out.release();
}

struct Local {
  bqg_ctx* ctx = nullptr;
  std::vector<bqg_table*> tables;
  CommState* st = nullptr;
  hipStream_t stream = nullptr;
  TableOwner L;                   // this rank's reduced rows (when the caller's are not)
  bqg_table* Lv = nullptr;        // the table whose rows this rank sends (L, or the caller's)
  int64_t nl = 0;                 // rows of Lv
  std::vector<int64_t> to_peer;   // rows for each destination rank
  std::vector<int64_t> from_peer; // rows from each source rank
  TableOwner R;                   // rows received from every rank, then reduced
  bqg_table** out = nullptr;
};

int lg_of(int32_t dt) {
  switch (dt_size(dt)) {
    case 1: return 0;
    case 2: return 1;
    case 4: return 2;
    default: return 3;
  }
}

// one 64-bit count into device memory without a host round trip (two 32-bit fills)
void put_count(int64_t* dst, int64_t v, hipStream_t st) {
  HIPCK(hipMemsetD32Async((hipDeviceptr_t)dst, (int)(uint32_t)(uint64_t)v, 1, st));
  HIPCK(hipMemsetD32Async((hipDeviceptr_t)((uint32_t*)dst + 1), (int)(uint32_t)((uint64_t)v >> 32), 1, st));
}


// ------------------------------------------------------------------------------------
// transport: RCCL, or in-process copies when every rank of the communicator is a local rank
// of this call (bqg_comm_init_local: one process driving several contexts, possibly on one
// GPU -- the test harness for the exchange logic on a one-GPU machine)
// ------------------------------------------------------------------------------------
// one message (merge_schedule.h); the messages between one (sender, receiver) pair are
// matched in the order they are posted, as RCCL matches grouped send / receive operations with
// the same peer
using bqg_sched::P2P;

void sync_all(std::vector<Local>& ranks) {
  for (Local& l : ranks) {
    HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
    HIPCK(hipStreamSynchronize(l.stream));
  }
}

Local& by_rank(std::vector<Local>& ranks, int r) {
  for (Local& l : ranks)
    if (l.st->rank == r) return l;
  comm_fail(BQG_E_STATE, "in-process transport: a rank of the communicator is not part of this merge call");
}

// In-process transport on one GPU: every copy of a transfer step in ONE kernel launch (a
// descriptor per copy; 16-, 4- or 1-byte moves by alignment) instead of one hipMemcpyAsync
// per (rank, peer, column) -- the host cost of hundreds of small copies would otherwise swamp
// the exchange being measured.
struct CopyDesc {
  const unsigned char* src;
  unsigned char* dst;
  unsigned long long bytes;
};

// A rank's slice of every column into the node-shared host result (bqg_merge_shared_host),
// one launch instead of one DMA copy per column (each copy past the first costs ~8-10 us,
// profiles/r6aq_d2h_chunks_micro.txt): 16-byte stores at 16-byte aligned host addresses (PCIe
// writes of whole units, ~50 GB/s, profiles/r6s_host_write_micro.txt); the unit at each end of
// a slice is written byte by byte, since the neighbouring rank's rows share it.
struct SliceCopies {
  int n;
  const unsigned char* src[bqg::kMergeMaxCols];
  unsigned char* dst[bqg::kMergeMaxCols];  // device mapping of the host block
  unsigned long long bytes[bqg::kMergeMaxCols];
};

__global__ __launch_bounds__(256) void k_slices_to_host(SliceCopies s) {
  const int j = blockIdx.y;
  const unsigned char* src = s.src[j];
  const uintptr_t d0 = (uintptr_t)s.dst[j], d1 = d0 + s.bytes[j];
  const uintptr_t a0 = d0 & ~(uintptr_t)15, a1 = (d1 + 15) & ~(uintptr_t)15;
  const bool agree4 = (((uintptr_t)src - d0) & 3) == 0;
  for (uintptr_t a = a0 + ((uintptr_t)blockIdx.x * 256 + threadIdx.x) * 16; a < a1; a += (uintptr_t)gridDim.x * 256 * 16) {
    if (a >= d0 && a + 16 <= d1) {
      const unsigned char* p = src + (a - d0);
      uint4 v;
      if (((uintptr_t)p & 15) == 0) {
        v = *reinterpret_cast<const uint4*>(p);
      } else if (agree4) {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
        v = make_uint4(q[0], q[1], q[2], q[3]);
      } else {
        unsigned char t[16];
        for (int k = 0; k < 16; ++k) t[k] = p[k];
        __builtin_memcpy(&v, t, 16);
      }
      *reinterpret_cast<uint4*>(a) = v;
    } else {
      for (int k = 0; k < 16; ++k)
        if (a + k >= d0 && a + k < d1) *reinterpret_cast<unsigned char*>(a + k) = src[a + k - d0];
    }
  }
}

__global__ __launch_bounds__(256) void k_batch_copy(const CopyDesc* d) {
  const CopyDesc c = d[blockIdx.y];
  const unsigned long long stride = (unsigned long long)gridDim.x * 256;
  const uintptr_t al = (uintptr_t)c.src | (uintptr_t)c.dst | (uintptr_t)c.bytes;
  if ((al & 15) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(c.src);
    uint4* d4 = reinterpret_cast<uint4*>(c.dst);
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < c.bytes / 16; i += stride)
      d4[i] = s4[i];
  } else if ((al & 3) == 0) {
    const uint32_t* s1 = reinterpret_cast<const uint32_t*>(c.src);
    uint32_t* d1 = reinterpret_cast<uint32_t*>(c.dst);
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < c.bytes / 4; i += stride)
      d1[i] = s1[i];
  } else {
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < c.bytes; i += stride)
      c.dst[i] = c.src[i];
  }
}

bool one_device(std::vector<Local>& ranks) {
  for (Local& l : ranks)
    if (bqg_internal_device(l.ctx) != bqg_internal_device(ranks[0].ctx)) return false;
  return true;
}

hipEvent_t event_of(CommState* st, hipEvent_t CommState::*which) {
  if (!(st->*which)) HIPCK(hipEventCreateWithFlags(&(st->*which), hipEventDisableTiming));
  return st->*which;
}

// The copies of one in-process transfer step, ordered on the ranks' streams the way RCCL
// orders a collective, with no host synchronisation: rank 0's stream waits for every rank's
// work so far, runs all the copies in one kernel, and every rank's stream waits for that
// kernel.  Contexts on different GPUs fall back to one copy per message on the receiver's
// stream between full synchronisations.
void batch_copies(std::vector<Local>& ranks, const std::vector<std::pair<size_t, CopyDesc>>& copies) {
  if (!one_device(ranks)) {
    sync_all(ranks);
    for (const auto& rc : copies) {
      Local& d = ranks[rc.first];
      HIPCK(hipSetDevice(bqg_internal_device(d.ctx)));
      HIPCK(hipMemcpyAsync(rc.second.dst, rc.second.src, rc.second.bytes, hipMemcpyDefault, d.stream));
    }
    sync_all(ranks);
    return;
  }
  if (copies.empty()) return;
  Local& l = ranks[0];
  HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
  for (size_t i = 1; i < ranks.size(); ++i) {
    hipEvent_t e = event_of(ranks[i].st, &CommState::ev);
    HIPCK(hipEventRecord(e, ranks[i].stream));
    HIPCK(hipStreamWaitEvent(l.stream, e, 0));
  }
  CommState* st = l.st;
  const size_t bytes = sizeof(CopyDesc) * copies.size();
  hipEvent_t de = event_of(st, &CommState::desc_ev);
  HIPCK(hipEventSynchronize(de));  // the previous step's descriptor upload has read the staging
  if (bytes > st->hdesc_cap) {
    if (st->hdesc) HIPCK(hipHostFree(st->hdesc));
    st->hdesc = nullptr;
    st->hdesc_cap = 0;
    HIPCK(hipHostMalloc(&st->hdesc, std::max<size_t>(bytes, 4096), hipHostMallocDefault));
    st->hdesc_cap = std::max<size_t>(bytes, 4096);
  }
  CopyDesc* h = (CopyDesc*)st->hdesc;
  unsigned long long most = 0;
  for (size_t i = 0; i < copies.size(); ++i) {
    h[i] = copies[i].second;
    most = std::max<unsigned long long>(most, h[i].bytes);
  }
  CopyDesc* dd = (CopyDesc*)st->ddesc.ensure(bytes);
  HIPCK(hipMemcpyAsync(dd, h, bytes, hipMemcpyHostToDevice, l.stream));
  HIPCK(hipEventRecord(de, l.stream));
  const unsigned gx = (unsigned)std::max<unsigned long long>(1, std::min<unsigned long long>(512, (most / 16 + 255) / 256));
  for (size_t i0 = 0; i0 < copies.size(); i0 += 65535) {
    const size_t n = std::min<size_t>(65535, copies.size() - i0);
    hipLaunchKernelGGL(k_batch_copy, dim3(gx, (unsigned)n), dim3(256), 0, l.stream, dd + i0);
    HIPCK(hipGetLastError());
  }
  hipEvent_t done = event_of(st, &CommState::ev);
  HIPCK(hipEventRecord(done, l.stream));
  for (size_t i = 1; i < ranks.size(); ++i) HIPCK(hipStreamWaitEvent(ranks[i].stream, done, 0));
}

// every rank: `count` int64 at counts.p -> [nranks][count] at counts.p + nranks
void xfer_allgather_i64(std::vector<Local>& ranks, size_t count) {
  const int W = ranks[0].st->nranks;
  if (ranks[0].st->comm) {
    Rccl& R = rccl();
    NCCLCHECK(R.GroupStart());
    for (Local& l : ranks) {
      int64_t* cnt = (int64_t*)l.st->counts.p;
      NCCLCHECK(R.AllGather(cnt, cnt + W, count, ncclInt64, l.st->comm, l.stream));
    }
    NCCLCHECK(R.GroupEnd());
    return;
  }
  if ((int)ranks.size() != W) comm_fail(BQG_E_STATE, "in-process transport needs every rank in one merge call");
  std::vector<std::pair<size_t, CopyDesc>> copies;
  for (size_t i = 0; i < ranks.size(); ++i) {
    Local& d = ranks[i];
    for (int s = 0; s < W; ++s) {
      Local& src = by_rank(ranks, s);
      copies.push_back({i, CopyDesc{(const unsigned char*)src.st->counts.p,
                                    (unsigned char*)((int64_t*)d.st->counts.p + W + (size_t)s * count),
                                    count * sizeof(int64_t)}});
    }
  }
  batch_copies(ranks, copies);
}

// grouped point-to-point: sends[i] / recvs[i] of local rank i (matching lists on both sides)
void xfer_p2p(std::vector<Local>& ranks, const std::vector<std::vector<P2P>>& sends,
              const std::vector<std::vector<P2P>>& recvs) {
  if (ranks[0].st->comm) {
    Rccl& R = rccl();
    NCCLCHECK(R.GroupStart());
    for (size_t i = 0; i < ranks.size(); ++i) {
      Local& l = ranks[i];
      for (const P2P& x : sends[i]) NCCLCHECK(R.Send(x.ptr, x.bytes, ncclUint8, x.peer, l.st->comm, l.stream));
      for (const P2P& x : recvs[i]) NCCLCHECK(R.Recv(x.ptr, x.bytes, ncclUint8, x.peer, l.st->comm, l.stream));
    }
    NCCLCHECK(R.GroupEnd());
    return;
  }
  std::vector<std::pair<size_t, CopyDesc>> copies;
  for (size_t i = 0; i < ranks.size(); ++i) {
    Local& d = ranks[i];
    std::vector<size_t> taken(ranks.size(), 0);  // messages of each sender matched so far
    for (const P2P& x : recvs[i]) {
      size_t j = 0;
      while (j < ranks.size() && ranks[j].st->rank != x.peer) ++j;
      if (j == ranks.size()) comm_fail(BQG_E_STATE, "in-process transport: peer rank not in this merge call");
      const P2P* m = nullptr;
      size_t k = 0;
      for (const P2P& y : sends[j])
        if (y.peer == d.st->rank && k++ == taken[j]) {
          m = &y;
          break;
        }
      ++taken[j];
      if (!m || m->bytes != x.bytes) comm_fail(BQG_E_STATE, "in-process transport: unmatched send / receive");
      copies.push_back({i, CopyDesc{(const unsigned char*)m->ptr, (unsigned char*)x.ptr, x.bytes}});
    }
  }
  batch_copies(ranks, copies);
}

// where the merged table goes: a new device table on rank 0 (bqg_merge / bqg_merge_group), a
// host result on rank 0 after the gather (bqg_merge_host), or a host result that every rank
// fills with its own partition (bqg_merge_group_host driving every rank: no gather)
// ... or (bqg_merge_shared_host, one process per GPU) host memory every rank's process maps:
// each rank copies its partition into its slice over its own link (no gather to rank 0)
enum class MergeOut { kDeviceRoot, kHostRoot, kHostDirect, kSharedHost };

// the caller's shared block: column j at sum_{j' < j} align256(capacity << lg[j']) bytes,
// rank r's rows after every lower rank's
struct SharedOut {
  unsigned char* base;
  int64_t capacity;
  int64_t* rows;
};

size_t shared_col_bytes(int64_t capacity, int lg) { return (((size_t)capacity << lg) + 255) & ~size_t(255); }

// sum by key (MergeReduce, kernels.h) of the table `in` whose rows come from several sources
// (row blocks [src_off[s], src_off[s + 1]), each unique by key) into `out` (capacity: every
// row), launched on the rank's stream; the key count is copied to st->hcounts() (the caller
// syncs, then lowers out's row count to it)
void queue_reduce(Local& l, bqg_table* in, const std::vector<int64_t>& src_off, int n_keys,
                  const std::vector<int32_t>& dts, const std::vector<int>& lg, TableOwner& out, bool unique_sources) {
  const int ncols = (int)dts.size();
  const int64_t n = nrows_of(l.ctx, in);
  ck(l.ctx, bqg_table_create(l.ctx, n, ncols, dts.data(), &out.t));
  bqg::MergeReduce m{};
  m.keys.nkeys = n_keys;
  for (int k = 0; k < n_keys; ++k) {
    m.keys.cols[k] = bqg::DevCol{(const unsigned char*)col_ptr(l.ctx, in, k), dts[k], lg[k]};
    m.out_keys[k] = (unsigned char*)col_ptr(l.ctx, out.t, k);
  }
  m.nvals = ncols - n_keys;
  for (int j = 0; j < m.nvals; ++j) {
    m.vals[j] = (const unsigned char*)col_ptr(l.ctx, in, n_keys + j);
    m.vdt[j] = dts[n_keys + j];
    m.out_vals[j] = (unsigned char*)col_ptr(l.ctx, out.t, n_keys + j);
  }
  m.nrows = n;
  m.unique_sources = unique_sources ? 1 : 0;
  const uint64_t cap = bqg::merge_reduce_cap(n);
  m.mask = cap - 1;
  const uint64_t nwords = ((uint64_t)n + 31) / 32, nblocks = (nwords + 1023) / 1024;
  const size_t o_acc = align16(cap * 8), o_bits = o_acc + align16(cap * 8 * (size_t)std::max(1, m.nvals)),
               o_wp = o_bits + align16(nwords * 4 + 4), o_bs = o_wp + align16(nwords * 4 + 4),
               total = o_bs + align16(nblocks * 4 + 4);
  unsigned char* b = (unsigned char*)l.st->reduce.ensure(total);
  m.table = (unsigned long long*)b;
  m.acc = (unsigned long long*)(b + o_acc);
  m.rep_bits = (unsigned int*)(b + o_bits);
  m.word_prefix = (unsigned int*)(b + o_wp);
  m.block_sum = (unsigned int*)(b + o_bs);
  int64_t* cnt = (int64_t*)l.st->counts.p;
  m.groups = (unsigned long long*)cnt;                 // [0]: keys found
  m.overflow = (unsigned int*)(cnt + 1);               // [1]: probe overflow flag
  HIPCK(hipMemsetAsync(cnt + 1, 0, 8, l.stream));
  bqg::launch_merge_reduce(m, src_off.data(), (int)src_off.size() - 1, l.stream);
  HIPCK(hipGetLastError());
  HIPCK(hipMemcpyAsync(l.st->hcounts(), cnt, 16, hipMemcpyDeviceToHost, l.stream));
}

// after queue_reduce and a sync of the rank's stream: the reduced table, its rows set
void finish_reduce(Local& l, TableOwner& out) {
  const int64_t* hc = (const int64_t*)l.st->hcounts();
  if (hc[1] & 0xFFFFFFFFll) comm_fail(BQG_E_HIP, "merge reduce: hash table overflow");
  ck(l.ctx, bqg_internal_table_set_rows(out.t, hc[0]));
}

void merge_impl(std::vector<Local>& ranks, int n_keys, const std::vector<int32_t>& dts, int reduced, MergeOut mode,
                bqg_result** host_out, const SharedOut* sh) {
  const int ncols = (int)dts.size();
  if (n_keys < 1 || n_keys > ncols || n_keys > bqg::kMaxKeys) comm_fail(BQG_E_INVALID, "merge needs 1..4 key columns");
  if (ncols > bqg::kMergeMaxCols) comm_fail(BQG_E_UNSUPPORTED, "merge schema has too many columns");
  const int W = ranks[0].st->nranks;
  if (W > bqg::kMergeMaxRanks) comm_fail(BQG_E_UNSUPPORTED, "merge across more than 256 ranks");
  for (Local& l : ranks) {
    if (l.st->nranks != W) comm_fail(BQG_E_INVALID, "local ranks of one merge must share a communicator size");
    for (bqg_table* t : l.tables) {
      int32_t nc = 0;
      ck(l.ctx, bqg_table_ncols(t, &nc));
      if (nc < ncols) comm_fail(BQG_E_INVALID, "merge input table has fewer columns than the merge schema");
      for (int j = 0; j < ncols; ++j) {
        int32_t dt = 0;
        ck(l.ctx, bqg_table_dtype(t, j, &dt));
        if (dt != dts[j]) comm_fail(BQG_E_INVALID, "merge input column dtype differs from the merge schema");
      }
    }
  }
  const bool all_local = (int)ranks.size() == W;
  if (mode == MergeOut::kHostDirect && !all_local) mode = MergeOut::kHostRoot;
  const bool timing = bqg_internal_timing(ranks[0].ctx);
  std::vector<int> lg(ncols);
  size_t row_bytes = 0;
  for (int j = 0; j < ncols; ++j) {
    lg[j] = lg_of(dts[j]);
    row_bytes += dt_size(dts[j]);
  }
  // byte offset of column j of destination d's packed block (k_mpack_scan's layout)
  auto packed_base = [&](const std::vector<int64_t>& rows, int d, int j) {
    size_t off = 0;
    for (int dd = 0; dd <= d; ++dd)
      for (int jj = 0; jj < ncols; ++jj) {
        if (dd == d && jj == j) return off;
        off += align16((size_t)rows[dd] << lg[jj]);
      }
    return off;
  };
  // phases (bqg_comm_last_phases): 0 local re-group + pack, 1 count exchange, 2 payload
  // exchange, 3 reduce, 4 gather counts, 5 gather + final sync; a collective step's time is
  // charged to every rank of the call (with timing on, after its device work has finished)
  for (Local& l : ranks)
    for (double& x : l.st->phase_ms) x = 0.0;
  auto enter = [&](int ph) {
    for (Local& l : ranks) l.st->cur_phase.store(ph, std::memory_order_relaxed);
  };
  enter(0);
  auto collective = [&](int ph, double t0) {
    if (timing) sync_all(ranks);
    const double dt = now_ms() - t0;
    for (Local& l : ranks) l.st->phase_ms[ph] += dt;
  };
  // a host result with the merged rows of every local rank's table `src` (rank order), each
  // rank's slice copied on its own stream: per-rank phase 5 with timing (each copy alone)
  auto to_host = [&](std::vector<bqg_table*> src) {
    std::vector<int64_t> rows(ranks.size(), 0);
    std::vector<size_t> order(ranks.size());  // slices in rank order
    int64_t total = 0;
    for (size_t i = 0; i < ranks.size(); ++i) {
      rows[i] = src[i] ? nrows_of(ranks[i].ctx, src[i]) : 0;
      total += rows[i];
      order[i] = i;
    }
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return ranks[a].st->rank < ranks[b].st->rank; });
    std::vector<void*> cols;
    bqg_result* r = nullptr;
    ck(ranks[0].ctx, bqg_internal_host_result(ranks[0].ctx, total, dts, cols, &r));
    std::unique_ptr<bqg_result, int (*)(bqg_result*)> own(r, bqg_result_free);
    int64_t off = 0;
    for (size_t i : order) {
      Local& l = ranks[i];
      const double t0 = now_ms();
      HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
      for (int j = 0; rows[i] && j < ncols; ++j)
        HIPCK(hipMemcpyAsync((unsigned char*)cols[j] + ((size_t)off << lg[j]), col_ptr(l.ctx, src[i], j),
                             (size_t)rows[i] << lg[j], hipMemcpyDeviceToHost, l.stream));
      if (timing) {
        HIPCK(hipStreamSynchronize(l.stream));
        l.st->phase_ms[5] += now_ms() - t0;
      }
      off += rows[i];
    }
    sync_all(ranks);
    *host_out = own.release();
  };
  // the shared host result: every rank's row count (an all-gather), each rank's slice copied
  // from its own GPU into the block every process maps, then an all-gather queued behind every
  // rank's copies -- when it completes, every slice has landed (stream order on each rank)
  auto to_shared = [&](std::vector<bqg_table*> src) {
    enter(4);
    double t0 = now_ms();
    std::vector<int64_t> part_rows(W, 0);
    if (W > 1) {
      for (size_t i = 0; i < ranks.size(); ++i) {
        HIPCK(hipSetDevice(bqg_internal_device(ranks[i].ctx)));
        put_count((int64_t*)ranks[i].st->counts.p, src[i] ? nrows_of(ranks[i].ctx, src[i]) : 0, ranks[i].stream);
      }
      xfer_allgather_i64(ranks, 1);
      Local& l0 = ranks[0];
      HIPCK(hipSetDevice(bqg_internal_device(l0.ctx)));
      HIPCK(hipMemcpyAsync(part_rows.data(), (int64_t*)l0.st->counts.p + W, sizeof(int64_t) * W, hipMemcpyDeviceToHost,
                           l0.stream));
      HIPCK(hipStreamSynchronize(l0.stream));
    } else {
      part_rows[0] = src[0] ? nrows_of(ranks[0].ctx, src[0]) : 0;
    }
    collective(4, t0);
    int64_t total = 0;
    for (int64_t r : part_rows) total += r;
    *sh->rows = total;  // (every rank sees the same total, so every rank fails alike below)
    if (total > sh->capacity)
      comm_fail(BQG_E_INVALID, "shared merge result holds " + std::to_string(sh->capacity) + " rows, the merge has " +
                                   std::to_string(total) + " (grow it to *rows and merge again)");
    enter(5);
    t0 = now_ms();
    std::vector<size_t> coff(ncols + 1, 0);
    for (int j = 0; j < ncols; ++j) coff[j + 1] = coff[j] + shared_col_bytes(sh->capacity, lg[j]);
    for (size_t i = 0; i < ranks.size(); ++i) {
      Local& l = ranks[i];
      HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
      l.st->register_host(sh->base, coff[ncols]);
      int64_t off = 0;
      for (int s2 = 0; s2 < l.st->rank; ++s2) off += part_rows[s2];
      const int64_t n = part_rows[l.st->rank];
      void* hdev = nullptr;
      if (n && ncols <= bqg::kMergeMaxCols && hipHostGetDevicePointer(&hdev, sh->base, 0) == hipSuccess && hdev) {
        SliceCopies sc{};
        sc.n = ncols;
        unsigned long long most = 0;
        for (int j = 0; j < ncols; ++j) {
          sc.src[j] = (const unsigned char*)col_ptr(l.ctx, src[i], j);
          sc.dst[j] = (unsigned char*)hdev + coff[j] + ((size_t)off << lg[j]);
          sc.bytes[j] = (unsigned long long)n << lg[j];
          most = std::max(most, sc.bytes[j]);
        }
        const unsigned gx = (unsigned)std::max<unsigned long long>(1, std::min<unsigned long long>((most / 16 + 2 + 255) / 256, 1024));
        hipLaunchKernelGGL(k_slices_to_host, dim3(gx, (unsigned)ncols), dim3(256), 0, l.stream, sc);
        HIPCK(hipGetLastError());
      } else {
        (void)hipGetLastError();
        for (int j = 0; n && j < ncols; ++j)
          HIPCK(hipMemcpyAsync(sh->base + coff[j] + ((size_t)off << lg[j]), col_ptr(l.ctx, src[i], j), (size_t)n << lg[j],
                               hipMemcpyDeviceToHost, l.stream));
      }
    }
    if (W > 1) xfer_allgather_i64(ranks, 1);
    sync_all(ranks);
    collective(5, t0);
  };
  // 1. local reduce: the rank's tables summed by key (one hash reduce over their row-
  // concatenation, tables in order: the client's first-appearance order), unless the caller's
  // one table is already reduced
  {
    std::vector<TableOwner> cat(ranks.size()), red(ranks.size());
    for (size_t i = 0; i < ranks.size(); ++i) {
      Local& l = ranks[i];
      const double t0 = now_ms();
      HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
      l.st->counts.ensure(sizeof(int64_t) * ((size_t)W * (W + 1) + 2));  // counts, reduce key count
      std::vector<bqg_table*> parts;
      for (bqg_table* t : l.tables)
        if (nrows_of(l.ctx, t) > 0) parts.push_back(t);
      if (parts.size() == 1 && reduced) {
        l.Lv = parts[0];  // keys already unique (a one-pass groupby over the rank's shards)
      } else if (!parts.empty()) {
        std::vector<int64_t> off(1, 0);
        for (bqg_table* t : parts) off.push_back(off.back() + nrows_of(l.ctx, t));
        cat[i].t = concat_tables(l.ctx, parts, dts);
        // a rank's tables (per-shard results) may repeat a key: atomic sums
        queue_reduce(l, cat[i].t, off, n_keys, dts, lg, red[i], false);
      }
      if (timing) HIPCK(hipStreamSynchronize(l.stream));
      l.st->phase_ms[0] += now_ms() - t0;
    }
    for (size_t i = 0; i < ranks.size(); ++i) {
      if (!red[i].t) continue;
      Local& l = ranks[i];
      const double t0 = now_ms();
      HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
      HIPCK(hipStreamSynchronize(l.stream));
      finish_reduce(l, red[i]);
      l.L.t = red[i].release();
      l.Lv = l.L.t;
      l.st->phase_ms[0] += now_ms() - t0;
    }
  }
  // 2. every row straight into its destination's packed block
  for (Local& l : ranks) {
    const double t0 = now_ms();
    HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
    l.nl = l.Lv ? nrows_of(l.ctx, l.Lv) : 0;
    int64_t* cnt = (int64_t*)l.st->counts.ensure(sizeof(int64_t) * ((size_t)W * (W + 1) + 2));
    if (W == 1) {
      put_count(cnt, l.nl, l.stream);  // one rank: every row goes to itself, sent as it is
    } else if (l.nl == 0) {
      HIPCK(hipMemsetAsync(cnt, 0, sizeof(int64_t) * W, l.stream));
    } else {
      bqg::MergePack m{};
      m.keys.nkeys = n_keys;
      for (int k = 0; k < n_keys; ++k)
        m.keys.cols[k] = bqg::DevCol{(const unsigned char*)col_ptr(l.ctx, l.Lv, k), dts[k], lg[k]};
      for (int j = 0; j < ncols; ++j) {
        m.cols[j] = (const unsigned char*)col_ptr(l.ctx, l.Lv, j);
        m.lg[j] = lg[j];
      }
      m.ncols = ncols;
      m.nranks = W;
      m.nrows = l.nl;
      bqg::merge_pack_grid(l.nl, &m.nblocks, &m.rows_per_block);
      const size_t dest_b = align16((size_t)l.nl), hist_b = align16((size_t)m.nblocks * W * 4);
      unsigned char* scr = (unsigned char*)l.st->scratch.ensure(dest_b + hist_b + (size_t)W * ncols * 8);
      m.dest = scr;
      m.block_hist = (uint32_t*)(scr + dest_b);
      m.colbase = (unsigned long long*)(scr + dest_b + hist_b);
      m.to_peer = (unsigned long long*)cnt;
      m.send = (unsigned char*)l.st->send.ensure((size_t)l.nl * row_bytes + (size_t)W * ncols * 16);
      bqg::launch_merge_pack(m, l.stream);
      HIPCK(hipGetLastError());
    }
    if (timing) HIPCK(hipStreamSynchronize(l.stream));
    l.st->phase_ms[0] += now_ms() - t0;
  }
  // world 1 with a host result: the rank's reduced rows are the answer (no exchange)
  if (W == 1 && mode == MergeOut::kSharedHost) {
    to_shared({ranks[0].Lv});
    for (Local& l : ranks) l.L.reset();
    return;
  }
  if (W == 1 && mode != MergeOut::kDeviceRoot) {
    enter(5);
    to_host({ranks[0].Lv});
    for (Local& l : ranks) l.L.reset();
    return;
  }
  // 3a. count matrix: every rank's row counts per destination
  enter(1);
  double tc = now_ms();
  xfer_allgather_i64(ranks, (size_t)W);
  collective(1, tc);
  for (Local& l : ranks) {
    const double t0 = now_ms();
    HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
    std::vector<int64_t> m((size_t)W * W);
    HIPCK(hipMemcpyAsync(m.data(), (int64_t*)l.st->counts.p + W, sizeof(int64_t) * W * W, hipMemcpyDeviceToHost,
                         l.stream));
    HIPCK(hipStreamSynchronize(l.stream));
    l.to_peer.assign(m.begin() + (size_t)l.st->rank * W, m.begin() + (size_t)(l.st->rank + 1) * W);
    l.from_peer.assign(W, 0);
    for (int s = 0; s < W; ++s) l.from_peer[s] = m[(size_t)s * W + l.st->rank];
    l.st->phase_ms[1] += now_ms() - t0;
  }
  // 3b. payload: column by column, straight into the receiving rank's table
  {
    std::vector<std::vector<P2P>> sends(ranks.size()), recvs(ranks.size());
    for (size_t i = 0; i < ranks.size(); ++i) {
      Local& l = ranks[i];
      HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
      int64_t total = 0;
      for (int s = 0; s < W; ++s) total += l.from_peer[s];
      if (total) ck(l.ctx, bqg_table_create(l.ctx, total, ncols, dts.data(), &l.R.t));
      std::vector<void*> dst(ncols);
      for (int j = 0; j < ncols; ++j) dst[j] = total ? col_ptr(l.ctx, l.R.t, j) : nullptr;
      bqg_sched::exchange_schedule(W, ncols, lg, l.to_peer, l.from_peer, [&](int d, int j) {
        return W == 1 ? col_ptr(l.ctx, l.Lv, j) : (void*)((unsigned char*)l.st->send.p + packed_base(l.to_peer, d, j));
      }, dst, sends[i], recvs[i]);
    }
    enter(2);
    tc = now_ms();
    xfer_p2p(ranks, sends, recvs);
    collective(2, tc);
  }
  // 4. reduce the received rows: one source's rows are already unique by key, rows from two or
  // more sources are summed by key (MergeReduce: one hash table, source order)
  enter(3);
  {
    std::vector<TableOwner> red(ranks.size());
    for (size_t i = 0; i < ranks.size(); ++i) {
      Local& l = ranks[i];
      const double t0 = now_ms();
      HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
      int sources = 0;
      for (int s = 0; s < W; ++s) sources += l.from_peer[s] > 0;
      if (sources > 1) {
        std::vector<int64_t> off(W + 1, 0);
        for (int s = 0; s < W; ++s) off[s + 1] = off[s] + l.from_peer[s];
        // every source sent a block of its reduced table: each key once per source
        queue_reduce(l, l.R.t, off, n_keys, dts, lg, red[i], true);
      }
      if (timing) HIPCK(hipStreamSynchronize(l.stream));
      l.st->phase_ms[3] += now_ms() - t0;
    }
    for (size_t i = 0; i < ranks.size(); ++i) {
      Local& l = ranks[i];
      const double t0 = now_ms();
      HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
      HIPCK(hipStreamSynchronize(l.stream));
      l.L.reset();  // sent (stream-ordered before any later use of its memory)
      l.Lv = nullptr;
      if (red[i].t) {
        finish_reduce(l, red[i]);
        l.R.reset();
        l.R.t = red[i].release();
      }
      l.st->phase_ms[3] += now_ms() - t0;
    }
  }
  if (mode == MergeOut::kSharedHost) {
    // 5. every rank's partition straight into its slice of the shared host block
    std::vector<bqg_table*> src;
    for (Local& l : ranks) src.push_back(l.R.t);
    to_shared(src);
    for (Local& l : ranks) l.R.reset();
    return;
  }
  if (mode == MergeOut::kHostDirect) {
    // 5. every rank's partition straight into its slice of the host result
    enter(5);
    std::vector<bqg_table*> src;
    for (Local& l : ranks) src.push_back(l.R.t);
    to_host(src);
    for (Local& l : ranks) l.R.reset();
    return;
  }
  // 5. gather to rank 0: the partitions' row counts (all-local: known here; else an
  // all-gather), then the reduced partitions column by column
  std::vector<int64_t> part_rows(W, 0);
  enter(4);
  tc = now_ms();
  if (all_local) {
    for (Local& l : ranks) part_rows[l.st->rank] = l.R.t ? nrows_of(l.ctx, l.R.t) : 0;
  } else {
    for (Local& l : ranks) put_count((int64_t*)l.st->counts.p, l.R.t ? nrows_of(l.ctx, l.R.t) : 0, l.stream);
    xfer_allgather_i64(ranks, 1);
    for (Local& l : ranks)
      if (l.st->rank == 0) {
        HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
        HIPCK(hipMemcpyAsync(part_rows.data(), (int64_t*)l.st->counts.p + W, sizeof(int64_t) * W,
                             hipMemcpyDeviceToHost, l.stream));
        HIPCK(hipStreamSynchronize(l.stream));
      }
    // non-root ranks learn the gather sizes they need (their own) locally
    for (Local& l : ranks)
      if (l.st->rank != 0) part_rows[l.st->rank] = l.R.t ? nrows_of(l.ctx, l.R.t) : 0;
  }
  collective(4, tc);
  enter(5);
  tc = now_ms();
  int64_t others = 0;
  for (int s = 1; s < W; ++s) others += part_rows[s];
  {
    std::vector<std::vector<P2P>> sends(ranks.size()), recvs(ranks.size());
    for (size_t i = 0; i < ranks.size(); ++i) {
      Local& l = ranks[i];
      HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
      std::vector<void*> src(ncols, nullptr), dst(ncols, nullptr);
      if (l.st->rank != 0) {
        for (int j = 0; l.R.t && j < ncols; ++j) src[j] = col_ptr(l.ctx, l.R.t, j);
        bqg_sched::gather_schedule(l.st->rank, W, ncols, lg, part_rows, src, dst, sends[i], recvs[i]);
        continue;
      }
      if (others == 0) continue;  // every merged row is in rank 0's own partition
      int64_t total = 0;
      for (int s = 0; s < W; ++s) total += part_rows[s];
      TableOwner res;
      ck(l.ctx, bqg_table_create(l.ctx, total, ncols, dts.data(), &res.t));
      if (part_rows[0])
        for (int j = 0; j < ncols; ++j) ck(l.ctx, bqg_push_chunk(res.t, j, col_ptr(l.ctx, l.R.t, j), part_rows[0], 0));
      for (int j = 0; j < ncols; ++j) dst[j] = col_ptr(l.ctx, res.t, j);
      bqg_sched::gather_schedule(0, W, ncols, lg, part_rows, src, dst, sends[i], recvs[i]);
      l.R.reset();
      l.R.t = res.release();
    }
    xfer_p2p(ranks, sends, recvs);
  }
  for (Local& l : ranks) {
    HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
    HIPCK(hipStreamSynchronize(l.stream));  // sends complete before their tables are released
    if (l.st->rank == 0 && !l.R.t) ck(l.ctx, bqg_table_create(l.ctx, 0, ncols, dts.data(), &l.R.t));  // no rows anywhere
  }
  collective(5, tc);
  if (mode == MergeOut::kHostRoot) {
    for (Local& l : ranks)
      if (l.st->rank == 0) {
        const double t0 = now_ms();
        // the gathered table to host memory on rank 0's stream
        std::vector<void*> cols;
        bqg_result* r = nullptr;
        const int64_t n = nrows_of(l.ctx, l.R.t);
        ck(l.ctx, bqg_internal_host_result(l.ctx, n, dts, cols, &r));
        std::unique_ptr<bqg_result, int (*)(bqg_result*)> own(r, bqg_result_free);
        HIPCK(hipSetDevice(bqg_internal_device(l.ctx)));
        for (int j = 0; n && j < ncols; ++j)
          HIPCK(hipMemcpyAsync(cols[j], col_ptr(l.ctx, l.R.t, j), (size_t)n << lg[j], hipMemcpyDeviceToHost, l.stream));
        HIPCK(hipStreamSynchronize(l.stream));
        *host_out = own.release();
        l.st->phase_ms[4] += now_ms() - t0;
      }
    for (Local& l : ranks) {
      l.R.reset();
      *l.out = nullptr;
    }
    return;
  }
  for (Local& l : ranks) {
    if (l.st->rank == 0) *l.out = l.R.release();
    else *l.out = nullptr;
    l.R.reset();
  }
}

int merge_entry(int32_t n_local, bqg_ctx* const* ctxs, const int32_t* n_tables, bqg_table* const* tables,
                int32_t n_keys, int32_t n_cols, const int32_t* dtypes, int32_t reduced, bqg_table** out,
                MergeOut mode, bqg_result** host_out, const SharedOut* sh = nullptr) {
  bqg_ctx* c0 = n_local > 0 && ctxs ? ctxs[0] : nullptr;
  return comm_guard(c0, [&] {
    const bool host_mode = mode == MergeOut::kHostRoot || mode == MergeOut::kHostDirect;
    if (n_local < 1 || !ctxs || !n_tables || !out || !dtypes || n_cols < 1 || (host_mode && !host_out) ||
        (mode == MergeOut::kSharedHost && (!sh || !sh->base || !sh->rows || sh->capacity < 0)))
      comm_fail(BQG_E_INVALID, "bad merge arguments");
    if (host_out) *host_out = nullptr;
    std::vector<int32_t> dts(dtypes, dtypes + n_cols);
    for (int32_t dt : dts)
      if (dt < BQG_BOOL || dt > BQG_F64) comm_fail(BQG_E_INVALID, "unknown dtype in the merge schema");
    std::vector<Local> ranks(n_local);
    size_t k = 0;
    for (int i = 0; i < n_local; ++i) {
      ranks[i].ctx = ctxs[i];
      ranks[i].st = state_of(ctxs[i]);
      ranks[i].stream = bqg_internal_stream(ctxs[i]);
      ranks[i].out = &out[i];
      out[i] = nullptr;
      if (n_tables[i] < 0) comm_fail(BQG_E_INVALID, "negative table count");
      for (int j = 0; j < n_tables[i]; ++j) ranks[i].tables.push_back(tables[k++]);
    }
    // progress marks (bqg_comm_progress): started now; idle and done at every exit
    struct Progress {
      std::vector<Local>& r;
      ~Progress() {
        for (Local& l : r) {
          l.st->cur_phase.store(-1, std::memory_order_relaxed);
          l.st->merges_done.fetch_add(1, std::memory_order_relaxed);
        }
      }
    } progress{ranks};
    for (Local& l : ranks) l.st->merges_started.fetch_add(1, std::memory_order_relaxed);
    merge_impl(ranks, n_keys, dts, reduced, mode, host_out, sh);
  });
}

}  // namespace

void bqg_internal_comm_release(bqg_ctx* c) {
  CommState* s = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comms.find(c);
    if (it == g_comms.end()) return;
    s = it->second;
    g_comms.erase(it);
  }
  try {
    destroy_state(s);
  } catch (...) {
  }
}

extern "C" {

int bqg_comm_unique_id(void* out) {
  return comm_guard(nullptr, [&] {
    if (!out) comm_fail(BQG_E_INVALID, "null output");
    ncclUniqueId id;
    NCCLCHECK(rccl().GetUniqueId(&id));
    memcpy(out, &id, sizeof(id));
  });
}

int bqg_comm_init(bqg_ctx* ctx, int32_t rank, int32_t nranks, const void* unique_id) {
  return comm_guard(ctx, [&] {
    if (!ctx || !unique_id) comm_fail(BQG_E_INVALID, "null context or unique id");
    if (nranks < 1 || rank < 0 || rank >= nranks) comm_fail(BQG_E_INVALID, "rank out of range");
    bqg_internal_comm_release(ctx);
    HIPCK(hipSetDevice(bqg_internal_device(ctx)));
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    CommState* s = new CommState();
    s->rank = rank;
    s->nranks = nranks;
    const ncclResult_t r = rccl().CommInitRank(&s->comm, nranks, id, rank);
    if (r != ncclSuccess) {
      delete s;
      comm_fail(BQG_E_HIP, std::string("ncclCommInitRank: ") + rccl().GetErrorString(r));
    }
    std::lock_guard<std::mutex> lk(g_mu);
    g_comms[ctx] = s;
  });
}

int bqg_comm_init_all(int32_t n, bqg_ctx* const* ctxs) {
  return comm_guard(n > 0 && ctxs ? ctxs[0] : nullptr, [&] {
    if (n < 1 || !ctxs) comm_fail(BQG_E_INVALID, "need at least one context");
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) {
      devs[i] = bqg_internal_device(ctxs[i]);
      for (int j = 0; j < i; ++j)
        if (devs[j] == devs[i]) comm_fail(BQG_E_INVALID, "one context per GPU");
    }
    for (int i = 0; i < n; ++i) bqg_internal_comm_release(ctxs[i]);
    std::vector<ncclComm_t> comms(n, nullptr);
    NCCLCHECK(rccl().CommInitAll(comms.data(), n, devs.data()));
    std::lock_guard<std::mutex> lk(g_mu);
    for (int i = 0; i < n; ++i) {
      CommState* s = new CommState();
      s->comm = comms[i];
      s->rank = i;
      s->nranks = n;
      g_comms[ctxs[i]] = s;
    }
  });
}

int bqg_comm_init_local(int32_t n, bqg_ctx* const* ctxs) {
  return comm_guard(n > 0 && ctxs ? ctxs[0] : nullptr, [&] {
    if (n < 1 || !ctxs) comm_fail(BQG_E_INVALID, "need at least one context");
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < i; ++j)
        if (ctxs[i] == ctxs[j]) comm_fail(BQG_E_INVALID, "one context per rank");
    for (int i = 0; i < n; ++i) bqg_internal_comm_release(ctxs[i]);
    std::lock_guard<std::mutex> lk(g_mu);
    for (int i = 0; i < n; ++i) {
      CommState* s = new CommState();
      s->rank = i;
      s->nranks = n;
      g_comms[ctxs[i]] = s;
    }
  });
}

int bqg_comm_destroy(bqg_ctx* ctx) {
  return comm_guard(ctx, [&] { bqg_internal_comm_release(ctx); });
}

int bqg_comm_info(bqg_ctx* ctx, int32_t* rank, int32_t* nranks) {
  return comm_guard(ctx, [&] {
    CommState* s = state_of(ctx);
    if (rank) *rank = s->rank;
    if (nranks) *nranks = s->nranks;
  });
}

int bqg_comm_last_phases(bqg_ctx* ctx, double* ms, int32_t n) {
  return comm_guard(ctx, [&] {
    if (!ms || n < 0) comm_fail(BQG_E_INVALID, "null output");
    CommState* s = state_of(ctx);
    for (int i = 0; i < n && i < kMergePhases; ++i) ms[i] = s->phase_ms[i];
  });
}

int bqg_comm_progress(bqg_ctx* ctx, int32_t* phase, int64_t* started, int64_t* done) {
  return comm_guard(ctx, [&] {
    CommState* s = state_of(ctx);
    if (phase) *phase = s->cur_phase.load(std::memory_order_relaxed);
    if (started) *started = s->merges_started.load(std::memory_order_relaxed);
    if (done) *done = s->merges_done.load(std::memory_order_relaxed);
  });
}

int bqg_merge(bqg_ctx* ctx, int32_t n_tables, bqg_table* const* tables, int32_t n_keys, int32_t n_cols,
              const int32_t* dtypes, int32_t reduced, bqg_table** out) {
  return bqg_merge_group(1, &ctx, &n_tables, tables, n_keys, n_cols, dtypes, reduced, out);
}

int bqg_merge_group(int32_t n_local, bqg_ctx* const* ctxs, const int32_t* n_tables, bqg_table* const* tables,
                    int32_t n_keys, int32_t n_cols, const int32_t* dtypes, int32_t reduced, bqg_table** out) {
  return merge_entry(n_local, ctxs, n_tables, tables, n_keys, n_cols, dtypes, reduced, out, MergeOut::kDeviceRoot,
                     nullptr);
}

int bqg_merge_host(bqg_ctx* ctx, int32_t n_tables, bqg_table* const* tables, int32_t n_keys, int32_t n_cols,
                   const int32_t* dtypes, int32_t reduced, bqg_result** out) {
  bqg_table* unused = nullptr;
  return merge_entry(1, &ctx, &n_tables, tables, n_keys, n_cols, dtypes, reduced, &unused, MergeOut::kHostRoot, out);
}

int bqg_merge_shared_host(bqg_ctx* ctx, int32_t n_tables, bqg_table* const* tables, int32_t n_keys, int32_t n_cols,
                          const int32_t* dtypes, int32_t reduced, void* host, int64_t capacity_rows, int64_t* rows) {
  bqg_table* unused = nullptr;
  const SharedOut sh{(unsigned char*)host, capacity_rows, rows};
  return merge_entry(1, &ctx, &n_tables, tables, n_keys, n_cols, dtypes, reduced, &unused, MergeOut::kSharedHost,
                     nullptr, &sh);
}

int bqg_merge_group_host(int32_t n_local, bqg_ctx* const* ctxs, const int32_t* n_tables, bqg_table* const* tables,
                         int32_t n_keys, int32_t n_cols, const int32_t* dtypes, int32_t reduced, bqg_result** out) {
  std::vector<bqg_table*> unused((size_t)std::max(n_local, 1), nullptr);
  return merge_entry(n_local, ctxs, n_tables, tables, n_keys, n_cols, dtypes, reduced, unused.data(),
                     MergeOut::kHostDirect, out);
}

}  // extern "C"
