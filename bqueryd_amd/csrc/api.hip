// api.hip -- host runtime of libbqgpu: contexts, device-resident shard tables, the query
// planner and the C ABI declared in include/bqgpu.h.
//
// The planner maps one bquery ctable.groupby call (bqueryd/worker.py:313) onto:
//   1. key coding: every key column is coded as (v - min) from the column statistics, and
//      the codes are combined mixed-radix into one dense slot id; sparse key spaces fall back
//      to an open-addressing hash of the packed code (float keys: canonical bits);
//   2. one fused scan over the columns (where-terms + slot + sums/counts/first row), in the
//      private-LDS, shared-LDS or global-atomic flavour by slot-space size;
//   3. extra ordered passes only for std (centered second moments), count_distinct and
//      sorted_count_distinct;
//   4. emit in first-appearance order of the passing rows (bquery's group order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "kernels.h"
#include "jit.h"
#include "ingest.h"
#include "ctx_internal.h"

using namespace bqg;

namespace {

struct HipError {
  hipError_t e;
  const char* what;
  int line;
};
struct ApiError {
  int code;
  std::string msg;
};
// A hash table (group keys) or count_distinct set of `slots` slots filled past half during a
// query: the query is re-run with twice the slots (run_groupby_grow).
struct TableOverflow {
  bool distinct;
  uint64_t slots;
};

#define HIPCHECK(x)                                 \
  do {                                              \
    hipError_t _e = (x);                            \
    if (_e != hipSuccess) throw HipError{_e, #x, __LINE__}; \
  } while (0)

[[noreturn]] void fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  throw ApiError{code, buf};
}

thread_local std::string g_err;

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  void* ensure(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (bytes > cap) {
      if (p) HIPCHECK(hipFree(p));
      p = nullptr;
      size_t c = std::max<size_t>(bytes, cap + cap / 2);
      c = (c + 255) & ~size_t(255);
      if (hipMalloc(&p, c) != hipSuccess) {
        p = nullptr;
        cap = 0;
        fail(BQG_E_OOM, "device allocation of %zu bytes failed", c);
      }
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

struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  void* ensure(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (bytes > cap) {
      if (p) HIPCHECK(hipHostFree(p));
      p = nullptr;
      size_t c = std::max<size_t>(bytes, cap + cap / 2);
      if (hipHostMalloc(&p, c, hipHostMallocDefault) != hipSuccess) {
        p = nullptr;
        cap = 0;
        fail(BQG_E_OOM, "pinned allocation of %zu bytes failed", c);
      }
      cap = c;
    }
    return p;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

size_t dtype_size(int dt) { return size_t(1) << dtype_lg(dt); }

// Column allocations cover whole 1024-row tiles plus 4096 rows plus 256 bytes: every lane of
// the last (partial) tile issues its full-width load in bounds, and so does a prefetch of up
// to 4096 rows that starts before the last row, so the scans need no tail branch.
size_t column_bytes(int64_t nrows, int dtype) {
  const size_t rows = ((size_t)nrows + kTileRows - 1) / kTileRows * kTileRows + 4096;
  return (rows << dtype_lg(dtype)) + 256;
}

}  // namespace

struct ColStats {
  bool valid = false;
  bool empty = true;
  int64_t imin = 0, imax = 0;
  double fmin = 0, fmax = 0;
  bool has_nan = false;
  // float columns: an exact 32-bit integer code for every value (partitioned sums travel as
  // codes): 1 = dyadic, code = v * 2^enc_k; 2 = cents, code = rint(v * 100); 0 = none
  int enc = 0;
  int enc_k = 0;
  // the same codes where the sum of every row's |code| stays below 2^63 (int64 sums that
  // cannot overflow; the atomic modes and the wide partitioned entries): a superset of enc
  int enc64 = 0;
  int enc64_k = 0;
  // float columns: the weight 2^lsb_exp of the lowest set bit over every finite nonzero value
  // (INT_MAX: none), and whether a subnormal occurs -- a fixed-point sum at shift s is exact iff
  // lsb_exp >= -s and no subnormal
  int lsb_exp = INT_MAX;
  bool subnormal = false;
  double fmaxabs = 0;  // the largest finite magnitude (0: none)
  int64_t runs = -1;  // value runs (rows differing from the row before + 1), -1 = not measured
};

// A compact resident copy of a column for the HBM-bound scans: an integer column as its
// offset from the minimum in the fewest of 1 / 2 / 4 bytes that hold its range, a float64
// column as its exact integer codes (ColStats::enc) -- as offsets from the smallest code in 1
// or 2 bytes when the codes span fewer than 2^16, else as int32 codes.  Built on first use by a scan that can read
// it, rebuilt when the column's statistics are (its data changed); every other path reads the
// column itself.
struct Shadow {
  unsigned char* dev = nullptr;
  size_t bytes = 0;
  bool valid = false;
  int dtype = 0;    // stored type
  int enc = 0;      // 1: integer offset (DevCol::enc), 2: float64 as integer codes
  int64_t off = 0;  // stored = value - off (enc 1), code - off (enc 2 with a 1 / 2-byte type)
  double mul = 0;   // enc 2: code = v * mul (value = code / mul)
};

struct Column {
  int dtype = 0;
  unsigned char* dev = nullptr;
  size_t bytes = 0;
  ColStats stats;
  Shadow shadow;
};

struct bqg_table {
  bqg_ctx* ctx = nullptr;
  int64_t nrows = 0;
  std::vector<Column> cols;
};

// A result's columns live in one pinned host block taken from the context's pool (the D2H
// copies land there directly; Python wraps the columns zero-copy) or, for tiny synthesized
// results, in `small`.
struct PinnedBlock {
  void* p = nullptr;
  size_t cap = 0;
  void* dev = nullptr;  // the block's device address (kernels write results into it directly)
};

struct PinnedPool {
  std::mutex mu;
  std::vector<PinnedBlock> free;
  ~PinnedPool() {
    for (PinnedBlock& b : free) (void)hipHostFree(b.p);
  }
  PinnedBlock get(size_t bytes) {
    bytes = std::max<size_t>(bytes, 4096);
    {
      std::lock_guard<std::mutex> lk(mu);
      size_t best = (size_t)-1;
      for (size_t i = 0; i < free.size(); ++i)
        if (free[i].cap >= bytes && (best == (size_t)-1 || free[i].cap < free[best].cap)) best = i;
      if (best != (size_t)-1) {
        PinnedBlock b = free[best];
        free.erase(free.begin() + best);
        return b;
      }
    }
    size_t cap = 4096;
    while (cap < bytes) cap <<= 1;
    PinnedBlock b;
    if (hipHostMalloc(&b.p, cap, hipHostMallocDefault) != hipSuccess) {
      b.p = nullptr;
      throw ApiError{BQG_E_OOM, "pinned result block allocation failed"};
    }
    b.cap = cap;
    if (hipHostGetDevicePointer(&b.dev, b.p, 0) != hipSuccess || !b.dev) {
      (void)hipHostFree(b.p);
      throw ApiError{BQG_E_HIP, "pinned result block is not device-mapped"};
    }
    return b;
  }
  void put(PinnedBlock b) {
    if (!b.p) return;
    std::lock_guard<std::mutex> lk(mu);
    free.push_back(b);
    // bounded (a multi-shard step keeps one block per shard result alive at once):
    // at most kMaxBlocks blocks, dropping the smallest, and kMaxBytes, dropping the largest
    constexpr size_t kMaxBlocks = 32, kMaxBytes = size_t(2) << 30;
    while (free.size() > kMaxBlocks) {
      size_t sm = 0;
      for (size_t i = 1; i < free.size(); ++i)
        if (free[i].cap < free[sm].cap) sm = i;
      (void)hipHostFree(free[sm].p);
      free.erase(free.begin() + sm);
    }
    for (;;) {
      size_t tot = 0, lg = 0;
      for (size_t i = 0; i < free.size(); ++i) {
        tot += free[i].cap;
        if (free[i].cap > free[lg].cap) lg = i;
      }
      if (tot <= kMaxBytes || free.empty()) break;
      (void)hipHostFree(free[lg].p);
      free.erase(free.begin() + lg);
    }
  }
};

// Owns a pool block until a result takes it over (release()); an exception that unwinds the
// call first (a JIT or launch failure, a HIP error) returns the block to the pool.
struct BlockGuard {
  std::shared_ptr<PinnedPool> pool;
  PinnedBlock b{};
  BlockGuard() = default;
  BlockGuard(const BlockGuard&) = delete;
  BlockGuard& operator=(const BlockGuard&) = delete;
  void reset(const std::shared_ptr<PinnedPool>& p, PinnedBlock blk) {
    if (b.p && pool) pool->put(b);
    pool = p;
    b = blk;
  }
  PinnedBlock release() {
    PinnedBlock r = b;
    b = PinnedBlock{};
    return r;
  }
  ~BlockGuard() {
    if (b.p && pool) pool->put(b);
  }
};

struct bqg_result {
  std::shared_ptr<PinnedPool> pool;
  PinnedBlock block;
  int64_t n_rows = 0;
  int32_t filtered = 0;
  std::vector<int32_t> dtypes;
  std::vector<std::vector<unsigned char>> small;
  std::vector<const void*> ptrs;
};

// Column memory of short-lived tables (query results kept in HBM, merge inputs, masks) is
// recycled instead of hipMalloc/hipFree per table (hipFree synchronises the device): freed
// blocks wait in size order, at most kMaxIdle bytes of them.
struct ColumnPool {
  std::multimap<size_t, void*> idle;  // capacity -> block
  size_t idle_bytes = 0;
  static constexpr size_t kMaxIdle = size_t(8) << 30;
  // column memory held from the device (handed out + idle), and the context's budget for it
  // (option mem_cap_mb; 0 = the device's memory): past the budget an allocation fails as an
  // out-of-memory hipMalloc would
  size_t allocated = 0;
  size_t budget = 0;
  void* get(size_t bytes, size_t* cap) {
    auto it = idle.lower_bound(bytes);
    if (it != idle.end() && it->first <= bytes + bytes / 2 + (size_t(1) << 20)) {
      void* p = it->second;
      *cap = it->first;
      idle_bytes -= it->first;
      idle.erase(it);
      return p;
    }
    void* p = nullptr;
    if (budget && allocated + bytes > budget) {
      release();
      if (allocated + bytes > budget) return nullptr;
    }
    if (hipMalloc(&p, bytes) != hipSuccess) {
      // release the idle blocks and retry once
      release();
      if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    }
    allocated += bytes;
    *cap = bytes;
    return p;
  }
  void put(void* p, size_t cap) {
    if (!p) return;
    idle.emplace(cap, p);
    idle_bytes += cap;
    while (idle_bytes > kMaxIdle && !idle.empty()) {
      auto last = std::prev(idle.end());
      idle_bytes -= last->first;
      allocated -= last->first;
      (void)hipFree(last->second);
      idle.erase(last);
    }
  }
  void release() {
    for (auto& kv : idle) (void)hipFree(kv.second);
    idle.clear();
    allocated -= idle_bytes;
    idle_bytes = 0;
  }
};

// Engine options: launch shapes and path choices the planner otherwise makes by itself.  Set
// per context with bqg_set_option (tests, profiling), or once at context creation from the
// environment (BQGPU_OPTIONS="name=value,..."; BQGPU_JIT / BQGPU_JIT_MIN_ROWS as before).
// Nothing on the query path reads the environment.  The list is documented in bqgpu.h and
// every non-default value is exercised against the oracle by tests/test_gpu_parity.py.
enum Opt {
  kOptJit, kOptJitMinRows, kOptPartition, kOptPartWbits, kOptPartK, kOptPartThreads, kOptPartPerCu,
  kOptPartSplits, kOptPartNarrow, kOptFusedScd, kOptScdCompact, kOptScdPack16, kOptPrivAhead,
  kOptPrivatePerCu, kOptSmallEmit, kOptHashSlots, kOptDistinctSlots, kOptPartPack, kOptScdRuns, kOptPartWin, kOptCompact, kOptPartFirst, kOptFxSums, kOptMemCap, kOptPartRing, kOptJitAsync, kOptWarm, kOptSlotEmit, kNumOpts
};
struct OptDef {
  const char* name;
  int64_t def, lo, hi;
};
constexpr OptDef kOptDefs[kNumOpts] = {
    {"jit", 1, 0, 1},                       // run-time specialised (hiprtc) scans
    {"jit_min_rows", 4ll << 20, 0, INT64_MAX},  // ... for tables of at least this many rows
    {"partition", 1, 0, 1},                 // partitioned aggregation for large dense slot spaces
    {"part_wbits", 0, 0, 13},               // slots per partition 2^wbits (0: auto, else 6..13)
    {"part_k", 0, 0, 4},                    // 4-row chunks per scatter thread (0: auto; 4: packed entries only)
    {"part_threads", 0, 0, 1024},           // scatter workgroup size (0: auto; 256, 512, 1024)
    {"part_per_cu", 0, 0, 8},               // scatter workgroups per CU (0: auto)
    {"part_splits", 0, 0, 1 << 20},         // aggregate workgroups per partition (0: auto)
    {"part_narrow", 1, 0, 1},               // exact 32-bit value codes in partition entries
    {"fused_scd", 1, 0, 1},                 // one fused pass for count / distinct queries
    {"scd_compact", 1, 0, 1},               // ... with 32-bit value codes when they fit
    {"scd_pack16", 1, 0, 1},                // ... first value and row in one LDS word
    {"priv_ahead", 0, 0, 4},                // private scan: tiles in flight (0: kernel default)
    {"private_per_cu", 0, 0, 8},            // private scan: workgroups per CU cap (0: auto)
    {"small_emit", 1, 0, 1},                // one-workgroup emit for <= 8192 slots
    {"hash_slots", 0, 0, 1ll << 31},        // initial hash-table slots (0: from the row count)
    {"distinct_slots", 0, 0, 1ll << 31},    // initial count_distinct set slots (0: from rows)
    {"part_pack", 1, 0, 1},                 // packed 4-byte partition entries when they fit
    {"scd_runs", 1, 0, 1},                  // fused distinct pass: 256-row steps for clustered keys
    {"part_win", 0, 0, 4096},               // partitioned aggregate: tiles per window (0: auto; 64..4096)
    {"compact", 1, 0, 2},                   // private / shared / dense global scans read compact column copies
    {"part_first", 0, 0, 2},                // packed partitioned path: rows in tile recorded for 0 auto / 1 no / 2 every tile
    {"fx_sums", 1, 0, 2},                   // atomic modes: fixed-point float sums (bit-reproducible; 2: per-slot shifts)
    {"mem_cap_mb", 0, 0, 1ll << 24},        // column memory budget of the context in MiB (0: the device's)
    {"part_ring", 0, 0, 2},                 // packed scatter (JIT): tiles of row loads in flight (0: 1)
    {"jit_async", 1, 0, 1},                 // a shape not compiled yet runs the generic kernel while hiprtc compiles it
    {"warm", 1, 0, 1},                      // bqg_create runs one small query (read at context creation only)
    {"slot_emit", 1, 0, 3},                 // large slot spaces: emit without the compaction and its host round trip (2: via group records, 3: first-row bitmap atomics)
};

static int opt_index(const char* name) {
  for (int i = 0; i < kNumOpts; ++i)
    if (name && strcmp(name, kOptDefs[i].name) == 0) return i;
  return -1;
}

static bool opt_valid(int i, int64_t v) {
  if (v < kOptDefs[i].lo || v > kOptDefs[i].hi) return false;
  if (i == kOptPartWbits) return v == 0 || v >= 6;
  if (i == kOptPartThreads) return v == 0 || v == 256 || v == 512 || v == 1024;
  if (i == kOptPartWin) return v == 0 || v >= 64;
  return true;
}

struct bqg_ctx {
  int device = 0;
  int64_t opt[kNumOpts];
  // hash / count_distinct tables grown after an overflow (the query is re-run with them)
  uint64_t hash_grow = 0, distinct_grow = 0;
  int32_t last_regrows = 0;  // re-runs of the last query after a table overflow
  ColumnPool colpool;
  IngestPool ingest;  // cold-path staging: streams + pinned double buffers per decode thread
  int cu = 256;
  // LDS one workgroup may take: the device's hipDeviceAttributeMaxSharedMemoryPerBlock, read at
  // bqg_create (gfx950: 160 KiB, tools/micro/lds_attrs.hip on MI355X); the planner sizes
  // workgroups per CU from it and check_launch refuses shapes past it
  size_t max_lds = 160 * 1024;
  int64_t jit_min_rows() const { return opt[kOptJitMinRows]; }
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  // staging for pushes
  static constexpr size_t kStage = 8u << 20;
  void* stage[2] = {nullptr, nullptr};
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  int stage_i = 0;
  // scratch
  DevBuf partials, counter, hdr, slots, terms, outcols, lists, bitmap, prefix, cdbuf, scdbuf, mask, misc, done;
  DevBuf strings;  // bqg_encode_bytes: the staged bytes and the dictionary's work arrays
  DevBuf nfbuf;    // the nonfinite pass's per-slot rows and counts
  // the large-result emit's row map (one byte per row; a query's first rows hold its epoch)
  DevBuf rowmap;
  unsigned char rowmap_epoch = 0;
  HostBuf hhdr, hout;
  // pinned blocks for results (returned by bqg_result_free); shared with outstanding results
  // so a result may outlive its context
  std::shared_ptr<PinnedPool> pool = std::make_shared<PinnedPool>();
  PinnedBlock pool_get(size_t bytes) { return pool->get(bytes); }
  // set by bqg_groupby_table / bqg_select_rows_table: the result becomes a new device table
  // (device-to-device copies of the output columns) instead of a host result
  bqg_table** dev_target = nullptr;
  // timing
  int timing = 0;  // 1: query window and scan window events, 2: the scan window only
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // timing level 1: the first and last compact-copy build of the current query
  hipEvent_t ev_sh[2] = {nullptr, nullptr};
  // timing level 1: the start of the result's copy to host memory (large results)
  hipEvent_t ev_copy = nullptr;
  bool copy_timed = false;
  // the large-result emit: the group count has reached page-locked host memory
  hipEvent_t ev_groups = nullptr;
  bool sh_timed = false;
  bqg_timing last{};
  double scan_ms_sum = 0;  // since timing was last enabled
  int64_t timed_queries = 0;
  // the context's live tables: an allocation that fails releases their compact copies (a
  // derived, rebuildable cache) and retries before it reports OOM
  std::vector<bqg_table*> tables;
};

namespace {

void set_stream_device(bqg_ctx* c) { HIPCHECK(hipSetDevice(c->device)); }

// Release every compact resident copy of one table (their memory back to the pool); they are
// rebuilt by the next query that reads them.  Returns whether any was held.
bool drop_shadows(bqg_ctx* c, bqg_table* t) {
  bool any = false;
  for (Column& col : t->cols) {
    if (!col.shadow.dev) continue;
    c->colpool.put(col.shadow.dev, col.shadow.bytes);
    col.shadow = Shadow{};
    any = true;
  }
  return any;
}

// Column memory from the pool.  A failed hipMalloc leaves its error as the thread's last HIP
// error: it is cleared here (an expected failure must not fail the next launch check), and
// before giving up the compact copies of every table of the context are released -- they are
// a rebuildable cache, the base columns are not.
void* col_alloc(bqg_ctx* c, size_t need, size_t* cap, bool may_drop_shadows = true) {
  c->colpool.budget = (size_t)c->opt[kOptMemCap] << 20;
  void* p = c->colpool.get(need, cap);
  if (p) return p;
  (void)hipGetLastError();
  if (!may_drop_shadows) return nullptr;
  bool any = false;
  for (bqg_table* t : c->tables) any |= drop_shadows(c, t);
  if (!any) return nullptr;
  c->colpool.release();  // hipFree synchronises: the released copies are no longer read
  p = c->colpool.get(need, cap);
  if (!p) (void)hipGetLastError();
  return p;
}

template <typename F>
int guard(bqg_ctx* ctx, F&& f) {
  try {
    if (ctx) set_stream_device(ctx);
    f();
    return BQG_OK;
  } catch (const ApiError& e) {
    if (ctx) ctx->err = e.msg;
    g_err = e.msg;
    return e.code;
  } catch (const HipError& e) {
    char buf[512];
    snprintf(buf, sizeof(buf), "HIP error %d (%s) in %s (api.hip:%d)", (int)e.e, hipGetErrorString(e.e), e.what,
             e.line);
    if (ctx) ctx->err = buf;
    g_err = buf;
    return BQG_E_HIP;
  } catch (const std::bad_alloc&) {
    if (ctx) ctx->err = "host out of memory";
    g_err = "host out of memory";
    return BQG_E_OOM;
  }
}

// ------------------------------------------------------------------------------------
// statistics
// ------------------------------------------------------------------------------------
// the k_stats result words of one column -> its ColStats (min / max / NaN / exact codes)
void finish_stats(Column& k, const unsigned long long* r, int64_t nrows) {
  const unsigned long long mn = r[0], mx = r[1], lsb = r[3], enc = r[4];
  k.stats.has_nan = r[2] != 0;
  k.stats.empty = mn > mx;
  if (!k.stats.empty) {
    if (dtype_is_float(k.dtype)) {
      auto dec = [](unsigned long long u) {
        u = (u & 0x8000000000000000ull) ? (u & ~0x8000000000000000ull) : ~u;
        double d;
        memcpy(&d, &u, 8);
        return d;
      };
      k.stats.fmin = dec(mn);
      k.stats.fmax = dec(mx);
      // exact 32-bit codes (k_stats): dyadic first (the code's sum times 2^-k is the exact sum
      // whenever it is below 2^53), else whole hundredths; |code| < 2^31 for every value
      const double maxabs = std::max(std::fabs(k.stats.fmin), std::fabs(k.stats.fmax));
      k.stats.lsb_exp = lsb == ~0ull ? INT_MAX : (int)lsb - 4096;
      k.stats.subnormal = (r[6] & 1ull) != 0;
      memcpy(&k.stats.fmaxabs, &r[5], 8);
      if (!k.stats.has_nan) {
        const int kk = lsb == ~0ull ? 0 : std::max(0, 4096 - (int)lsb);
        if (!(enc & 1ull) && kk <= 62 && std::ldexp(maxabs, kk) < 2147483647.0) {
          k.stats.enc = 1;
          k.stats.enc_k = kk;
        } else if (!(enc & 2ull) && maxabs * 100.0 < 2147483647.0) {
          k.stats.enc = 2;
        }
        const double rows = (double)std::max<int64_t>(nrows, 1);
        if (!(enc & 1ull) && kk <= 1000 && std::ldexp(maxabs, kk) * rows < 9.2e18) {
          k.stats.enc64 = 1;
          k.stats.enc64_k = kk;
        } else if (!(enc & 2ull) && maxabs * 100.0 * rows < 9.2e18) {
          k.stats.enc64 = 2;
        }
        if (k.stats.enc) {  // the 32-bit code's kind wins (same kind, same scale)
          k.stats.enc64 = k.stats.enc;
          k.stats.enc64_k = k.stats.enc_k;
        }
      }
    } else if (k.dtype == BQG_U64) {
      k.stats.imin = (int64_t)mn;
      k.stats.imax = (int64_t)mx;
    } else {
      k.stats.imin = (int64_t)(mn ^ 0x8000000000000000ull);
      k.stats.imax = (int64_t)(mx ^ 0x8000000000000000ull);
    }
  }
  k.stats.valid = true;
}

// Statistics of several columns in one round trip: one k_stats launch per column without
// valid statistics, then ONE copy back and ONE synchronisation (a re-group of a merge's
// received rows otherwise paid a host round trip per column).
void compute_stats_many(bqg_table* t, const std::vector<int>& cols) {
  bqg_ctx* c = t->ctx;
  std::vector<int> todo;
  for (int col : cols)
    if (col >= 0 && col < (int)t->cols.size() && !t->cols[col].stats.valid &&
        std::find(todo.begin(), todo.end(), col) == todo.end())
      todo.push_back(col);
  if (todo.empty()) return;
  const size_t n = todo.size();
  // results [n][8] words, then one column's per-block partials at a time (the launches of
  // one stream run in order)
  unsigned long long* d = (unsigned long long*)c->misc.ensure((n * 8 + (size_t)kStatsMaxBlocks * kStatsWords) *
                                                              sizeof(unsigned long long));
  unsigned long long* h = (unsigned long long*)c->hhdr.ensure(2 * n * 8 * sizeof(unsigned long long));
  static const unsigned long long init[8] = {~0ull, 0ull, 0ull, ~0ull, 0ull, 0ull, 0ull, 0ull};
  for (size_t i = 0; i < n; ++i) memcpy(h + 8 * i, init, sizeof(init));
  HIPCHECK(hipMemcpyAsync(d, h, n * sizeof(init), hipMemcpyHostToDevice, c->stream));
  for (size_t i = 0; i < n; ++i) {
    Column& k = t->cols[todo[i]];
    k.stats.runs = -1;  // measured again on demand (column_runs)
    k.shadow.valid = false;  // the data changed: the compact copy is rebuilt on demand
    DevCol dc{k.dev, k.dtype, dtype_lg(k.dtype)};
    if (t->nrows > 0) launch_stats(dc, t->nrows, d + 8 * i, d + 8 * n, c->stream);
  }
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipMemcpyAsync(h + 8 * n, d, n * sizeof(init), hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < n; ++i) finish_stats(t->cols[todo[i]], h + 8 * n + 8 * i, t->nrows);
}

void compute_stats(bqg_table* t, int col) {
  if (t->cols[col].stats.valid) return;
  compute_stats_many(t, std::vector<int>{col});
}

// value runs of a column (count_runs: one pass, cached with the statistics; a push or a
// chunk load invalidates both)
int64_t column_runs(bqg_table* t, int col) {
  bqg_ctx* c = t->ctx;
  Column& k = t->cols[col];
  compute_stats(t, col);
  if (k.stats.runs >= 0) return k.stats.runs;
  unsigned long long* d = (unsigned long long*)c->misc.ensure(64);
  HIPCHECK(hipMemsetAsync(d, 0, 8, c->stream));
  launch_runs(DevCol{k.dev, k.dtype, dtype_lg(k.dtype)}, t->nrows, d, c->stream);
  HIPCHECK(hipGetLastError());
  unsigned long long* h = (unsigned long long*)c->hhdr.ensure(128);
  HIPCHECK(hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  k.stats.runs = t->nrows > 0 ? (int64_t)h[0] + 1 : 0;
  return k.stats.runs;
}

// ------------------------------------------------------------------------------------
// query planning
// ------------------------------------------------------------------------------------
enum Mode { kPrivate = 0, kShared = 1, kGlobalDense = 2, kGlobalHash = 3, kPartitioned = 4 };

struct Plan {
  ScanParams p{};
  std::vector<int> tcol;       // table column of each scan column
  int mode = kGlobalDense;
  uint64_t nslots = 1;
  int nsum = 0;                // sum states (SUM / MEAN)
  std::vector<int> std_cols;   // scan columns needing a centered pass (subset of sum states)
  int32_t agg_state[kMaxAggs];
  int wbits = 12;
  bool has_filter = false;
  int64_t alg_bytes = 0;       // the query's distinct columns at their stored widths
  int64_t read_bytes = 0;      // what the scan reads of them (compact copies: fewer)
  bool dummy_col = false;      // the one scan column of a plan that reads none (not in alg_bytes)
  // mean / std states whose float column holds NaN or infinities (column statistics): bquery's
  // row-order update turns such a group's mean into NaN unless its only non-finite value is its
  // last row, which the extra nonfinite pass decides per slot
  int nf_states = 0;           // bit q: sum state q needs it
  // float sum states the atomic / partitioned modes accumulate as fixed-point limbs
  // (ScanParams::sum_enc 3): finite columns without an exact int64 code (fx_states, pass 1),
  // and the std pass's centred squares (fx2_states, bit i: the i-th std column)
  int fx_states = 0;
  int fx2_states = 0;
  // ... of those, the states that take their shift per slot (ScanParams::fx_emax): columns whose
  // values span more than the 2^42 a column-wide shift keeps exact (option fx_sums=2: all)
  int fx_slot_states = 0;
  int32_t fx2_shift[kMaxSums] = {};
};

// the fixed-point shift of values of magnitude at most m: m * 2^shift < 2^95 (ScanParams::
// sum_fx_shift; limbs of 32 bits, three of them)
int fx_shift_for(double m) {
  if (!(m > 0.0)) return 0;
  int e;
  std::frexp(m, &e);  // m < 2^e
  return 95 - e;
}

// bytes of one workgroup's shared-mode LDS table (k_scan_shared): [nsum][S] sums, [S] counts,
// [S] first rows, then with fixed-point sums [nsum][kFxWords][S] limbs and flags
size_t shared_lds(uint64_t S, int nsum, bool fx) {
  return (size_t)S * (8 + 8 * (size_t)nsum) + (fx ? 8 * kFxWords * (size_t)nsum * S : 0);
}

int scan_col(Plan& pl, int tc) {
  for (size_t i = 0; i < pl.tcol.size(); ++i)
    if (pl.tcol[i] == tc) return (int)i;
  if ((int)pl.tcol.size() >= kMaxCols)
    fail(BQG_E_UNSUPPORTED, "query touches more than %d distinct columns", kMaxCols);
  pl.tcol.push_back(tc);
  return (int)pl.tcol.size() - 1;
}

uint64_t bits_for(uint64_t range) {  // bits needed to code values 0..range-1
  uint64_t b = 0;
  while (b < 64 && (range - 1) >> b) ++b;
  return b;
}

void build_terms(bqg_ctx* c, bqg_table* t, Plan& pl, int n_terms, const bqg_term* terms) {
  if (n_terms > kMaxTerms) fail(BQG_E_UNSUPPORTED, "more than %d where terms", kMaxTerms);
  size_t need = 0;
  for (int i = 0; i < n_terms; ++i)
    if (terms[i].op == BQG_T_IN || terms[i].op == BQG_T_NIN) need += (size_t)terms[i].nvals * 8;
  unsigned char* dv = (unsigned char*)c->terms.ensure(need + 64);
  std::vector<unsigned char> host(need + 64);
  size_t off = 0;
  pl.p.nterms = n_terms;
  for (int i = 0; i < n_terms; ++i) {
    const bqg_term& tm = terms[i];
    if (tm.col < 0 || tm.col >= (int)t->cols.size()) fail(BQG_E_INVALID, "where term column %d out of range", tm.col);
    if (tm.op < BQG_T_FALSE || tm.op > BQG_T_LE) fail(BQG_E_INVALID, "unknown where operator code %d", tm.op);
    DevTerm& d = pl.p.terms[i];
    d.col = scan_col(pl, tm.col);
    d.op = tm.op;
    d.is_float = dtype_is_float(t->cols[tm.col].dtype);
    d.nvals = (int32_t)tm.nvals;
    d.ivals = nullptr;
    d.fvals = nullptr;
    d.iv0 = 0;
    d.fv0 = 0;
    if (tm.op == BQG_T_TRUE || tm.op == BQG_T_FALSE) continue;
    if (tm.nvals < 1) fail(BQG_E_INVALID, "where term without values");
    if (d.is_float) {
      if (!tm.fvals) fail(BQG_E_INVALID, "float where term without fvals");
      d.fv0 = tm.fvals[0];
    } else {
      if (!tm.ivals) fail(BQG_E_INVALID, "integer where term without ivals");
      d.iv0 = tm.ivals[0];
    }
    if (tm.op == BQG_T_IN || tm.op == BQG_T_NIN) {
      const void* src = d.is_float ? (const void*)tm.fvals : (const void*)tm.ivals;
      memcpy(host.data() + off, src, (size_t)tm.nvals * 8);
      if (d.is_float) d.fvals = (const double*)(dv + off);
      else d.ivals = (const int64_t*)(dv + off);
      off += (size_t)tm.nvals * 8;
    }
  }
  if (off) HIPCHECK(hipMemcpyAsync(dv, host.data(), off, hipMemcpyHostToDevice, c->stream));
  // the staging vector must outlive the async copy: synchronise (tiny, once per query)
  if (off) HIPCHECK(hipStreamSynchronize(c->stream));
}

void plan_query(bqg_ctx* c, bqg_table* t, const bqg_query* q, Plan& pl) {
  const int ncols_t = (int)t->cols.size();
  if (q->n_keys < 0 || q->n_keys > kMaxKeys) fail(BQG_E_UNSUPPORTED, "at most %d groupby columns", kMaxKeys);
  if (q->n_aggs < 0 || q->n_aggs > kMaxAggs) fail(BQG_E_UNSUPPORTED, "at most %d aggregations", kMaxAggs);
  for (int i = 0; i < q->n_keys; ++i)
    if (q->key_cols[i] < 0 || q->key_cols[i] >= ncols_t) fail(BQG_E_INVALID, "groupby column %d out of range", q->key_cols[i]);
  // 1. sum states (value columns first), deduplicated by column
  for (int a = 0; a < q->n_aggs; ++a) {
    const bqg_agg& g = q->aggs[a];
    if (g.col < 0 || g.col >= ncols_t) fail(BQG_E_INVALID, "aggregation column %d out of range", g.col);
    if (g.op < BQG_SUM || g.op > BQG_STD) fail(BQG_E_INVALID, "unknown aggregation op %d", g.op);
    pl.agg_state[a] = -1;
    if (g.op == BQG_SUM || g.op == BQG_MEAN || g.op == BQG_STD) {
      const int dt = t->cols[g.col].dtype;
      if (dt == BQG_BOOL) fail(BQG_E_UNSUPPORTED, "sum/mean/std of a bool column");
      // mean / std of a 64-bit integer column whose sum can leave the 64-bit accumulator: a
      // float64 sum state of its own (bquery's incremental mean runs in float64 and never
      // wraps; the sum keeps its wrapping integer state)
      bool fview = false;
      if ((g.op == BQG_MEAN || g.op == BQG_STD) && (dt == BQG_I64 || dt == BQG_U64)) {
        compute_stats(t, g.col);
        const ColStats& cs = t->cols[g.col].stats;
        const double rows = (double)std::max<int64_t>(t->nrows, 1);
        const double mx = dt == BQG_U64 ? (double)(uint64_t)cs.imax
                                        : std::max(std::fabs((double)cs.imin), std::fabs((double)cs.imax));
        fview = !cs.empty && mx * rows >= (dt == BQG_U64 ? 1.8e19 : 9.2e18);
      }
      int st = -1;
      for (int s = 0; s < (int)pl.tcol.size(); ++s)
        if (pl.tcol[s] == g.col && (pl.p.sum_is_float[s] != 0) == (dtype_is_float(dt) || fview)) st = s;
      if (st < 0) {
        if ((int)pl.tcol.size() >= kMaxSums) fail(BQG_E_UNSUPPORTED, "more than %d summed columns", kMaxSums);
        pl.tcol.push_back(g.col);
        st = (int)pl.tcol.size() - 1;
        pl.p.sum_is_float[st] = dtype_is_float(dt) || fview;
        pl.p.sum_conv[st] = dtype_is_float(dt) ? 0 : (dt == BQG_U64 ? 2 : 1);
        pl.p.sum_centered[st] = 0;
        pl.p.centers[st] = nullptr;
      }
      pl.agg_state[a] = st;
      if (g.op == BQG_STD && std::find(pl.std_cols.begin(), pl.std_cols.end(), st) == pl.std_cols.end())
        pl.std_cols.push_back(st);
    }
  }
  pl.nsum = (int)pl.tcol.size();
  pl.p.nsum = pl.nsum;
  // 2. where terms and mask
  build_terms(c, t, pl, q->n_terms, q->terms);
  pl.p.mask_col = -1;
  if (q->mask_col >= 0) {
    if (q->mask_col >= ncols_t || t->cols[q->mask_col].dtype != BQG_BOOL)
      fail(BQG_E_INVALID, "mask column must be a BOOL column");
    pl.p.mask_col = scan_col(pl, q->mask_col);
  }
  pl.has_filter = q->n_terms > 0 || q->mask_col >= 0;
  {
    // the statistics this plan reads (key ranges, value codes of summed and distinct columns),
    // in one device round trip
    std::vector<int> sc;
    for (int k = 0; k < q->n_keys; ++k) sc.push_back(q->key_cols[k]);
    for (int a = 0; a < q->n_aggs; ++a)
      if (q->aggs[a].op != BQG_COUNT) sc.push_back(q->aggs[a].col);
    compute_stats_many(t, sc);
  }
  // mean / std of a float column holding NaN or an infinity: the nonfinite pass decides those
  // groups' values the way bquery's row-order update does
  for (int a = 0; a < q->n_aggs; ++a) {
    const bqg_agg& g = q->aggs[a];
    if ((g.op != BQG_MEAN && g.op != BQG_STD) || !dtype_is_float(t->cols[g.col].dtype)) continue;
    const ColStats& cs = t->cols[g.col].stats;
    if (cs.has_nan || (!cs.empty && (std::isinf(cs.fmin) || std::isinf(cs.fmax)))) pl.nf_states |= 1 << pl.agg_state[a];
  }
  // float sums the atomic / partitioned modes cannot keep as exact integer codes: fixed-point
  // limbs, summed as integers whatever the arrival order (bit-reproducible); the
  // column finite, below 2^31 rows (the int64 limb sums cannot wrap)
  if (c->opt[kOptFxSums] && t->nrows < ((int64_t)1 << 31)) {
    for (int q = 0; q < pl.nsum; ++q) {
      if (!pl.p.sum_is_float[q] || pl.p.sum_conv[q] != 0) continue;
      const ColStats& cs = t->cols[pl.tcol[q]].stats;
      if (cs.empty) continue;
      // (NaN / infinities are flags beside the limbs: a group's sum is NaN or +-inf whatever
      // the order its values arrive in; the shift follows the finite values)
      pl.p.sum_fx_shift[q] = fx_shift_for(cs.fmaxabs);
      if (cs.enc64 && c->opt[kOptPartNarrow] != 0) continue;  // integer codes already (set_sum_codes)
      // only where every value is a multiple of 2^-shift: the limb sums are then the EXACT sums
      // (one rounding at the end) -- a column whose values span more than 2^42 in magnitude
      // (an outlier beside small values) keeps the float64 atomics, whose error is relative
      if (cs.subnormal) continue;
      // (an outlier beside small values: a shift per slot, from the slot's own largest value --
      // exact again unless one slot holds both; within 2^-95 of that slot's largest magnitude
      // per value otherwise, and the same bits on every run)
      if (c->opt[kOptFxSums] == 2 || (cs.lsb_exp != INT_MAX && cs.lsb_exp < -pl.p.sum_fx_shift[q])) pl.fx_slot_states |= 1 << q;
      pl.fx_states |= 1 << q;
    }
    // the std pass's (x - mean)^2 <= (max - min)^2
    for (size_t i = 0; i < pl.std_cols.size(); ++i) {
      const int q = pl.std_cols[i];
      if (!pl.p.sum_is_float[q] || pl.p.sum_conv[q] != 0) continue;
      const ColStats& cs = t->cols[pl.tcol[q]].stats;
      if (cs.empty) continue;
      // the centre is a rounded float mean: it may sit an ulp or two of the column's magnitude
      // outside [min, max], so |x - centre| <= span + 4 ulp(magnitude); squared with a factor 2
      // of headroom (timestamp-like columns, whose span is far below their magnitude,
      // could reach 2^e at the old 1.0000001 margin and lose the limbs' top bits).  A column
      // holding NaN or infinities: its finite values lie within +-fmaxabs; a group with a
      // non-finite value has a non-finite centre, its squares land in the limbs' flags and its
      // std is NaN anyway (the nonfinite pass) -- so these columns keep the limbs too (round 6:
      // they took float64 atomics, whose sums depend on the arrival order)
      const bool nonfinite = cs.has_nan || std::isinf(cs.fmin) || std::isinf(cs.fmax);
      const double mag = nonfinite ? cs.fmaxabs : std::max(std::fabs(cs.fmin), std::fabs(cs.fmax));
      const double span = nonfinite ? 2.0 * cs.fmaxabs : cs.fmax - cs.fmin;
      const double dev = span + 4.0 * std::ldexp(mag, -52), sq = dev * dev * 2.0;
      if (!std::isfinite(sq)) continue;
      pl.fx2_states |= 1 << i;
      pl.fx2_shift[i] = fx_shift_for(sq);
    }
  }
  // 3. keys
  pl.p.nkeys = q->n_keys;
  bool any_float = false;
  unsigned __int128 space = 1;
  uint64_t bits = 0;
  for (int k = 0; k < q->n_keys; ++k) {
    const int tc = q->key_cols[k];
    Column& col = t->cols[tc];
    compute_stats(t, tc);
    DevKey& dk = pl.p.keys[k];
    dk.col = scan_col(pl, tc);
    dk.is_float = dtype_is_float(col.dtype);
    if (dk.is_float) {
      any_float = true;
      dk.min = 0;
      dk.range = 0;
      continue;
    }
    if (col.stats.empty) {
      dk.min = 0;
      dk.range = 1;
    } else {
      dk.min = col.stats.imin;
      const uint64_t r = (uint64_t)col.stats.imax - (uint64_t)col.stats.imin;  // may wrap to 2^64-1
      dk.range = r + 1;                                                       // 0 means 2^64
    }
    const unsigned __int128 rr = dk.range ? (unsigned __int128)dk.range : ((unsigned __int128)1 << 64);
    // saturate at 2^100 before the product can wrap (two full-range 64-bit keys: 2^128)
    const unsigned __int128 cap100 = (unsigned __int128)1 << 100;
    space = space > cap100 / rr ? cap100 : space * rr;
    bits += dk.range ? bits_for(dk.range) : 64;
  }
  pl.p.ncols = (int)pl.tcol.size();
  for (int i = 0; i < pl.p.ncols; ++i) {
    const Column& col = t->cols[pl.tcol[i]];
    pl.p.cols[i] = DevCol{col.dev, col.dtype, dtype_lg(col.dtype)};
  }
  // algorithmic bytes: every distinct input column the query reads, once --
  // keys, where-term / mask columns and aggregated columns (count_distinct and
  // sorted_count_distinct value columns are not scan columns of the main pass)
  {
    std::vector<int> distinct(pl.tcol.begin(), pl.tcol.end());
    for (int a = 0; a < q->n_aggs; ++a)
      if ((q->aggs[a].op == BQG_COUNT_DISTINCT || q->aggs[a].op == BQG_SORTED_COUNT_DISTINCT) &&
          std::find(distinct.begin(), distinct.end(), q->aggs[a].col) == distinct.end())
        distinct.push_back(q->aggs[a].col);
    for (int tc : distinct) pl.alg_bytes += (int64_t)dtype_size(t->cols[tc].dtype) * t->nrows;
    pl.read_bytes = pl.alg_bytes;
  }
  if (pl.tcol.empty()) {
    // no keys, terms, mask or summed columns (e.g. groupby([], count / count_distinct)): the
    // scan kernels stream at least one column (NC >= 1) -- the first aggregation's, whose rows
    // the count covers (not counted in alg_bytes: nothing is read from it)
    if (ncols_t < 1) fail(BQG_E_INVALID, "table has no columns");
    const int tc = q->n_aggs > 0 ? q->aggs[0].col : 0;
    scan_col(pl, tc);
    pl.p.ncols = 1;
    pl.dummy_col = true;
    const Column& col = t->cols[tc];
    pl.p.cols[0] = DevCol{col.dev, col.dtype, dtype_lg(col.dtype)};
  }
  if (pl.p.ncols < 1 || pl.p.ncols > kMaxCols) fail(BQG_E_INVALID, "scan plan with %d columns", pl.p.ncols);
  pl.p.nrows = t->nrows;
  // 4. mode
  const uint64_t kDenseMax = std::max<uint64_t>(1ull << 24, std::min<uint64_t>(2ull * (uint64_t)t->nrows, 1ull << 27));
  bool hash = any_float || space > kDenseMax;
  if (hash) {
    // wide keys (hash mode 2): float columns in a multi-column key, or packed codes over 63
    // bits (e.g. a full-range int64 / uint64 key): the table holds a hash half and a
    // representative row whose key values are compared in full
    const bool wide = (any_float && q->n_keys > 1) || (!any_float && bits > 63);
    // packed power-of-two strides: last key in the low bits
    uint64_t shift = 0;
    for (int k = wide ? -1 : q->n_keys - 1; k >= 0; --k) {
      DevKey& dk = pl.p.keys[k];
      if (dk.is_float) {
        dk.stride = 1;
        dk.range = 0;
        continue;
      }
      // the field of a packed key is a power of two wide: emit decodes (code / stride) % range
      const uint64_t b = bits_for(dk.range);
      dk.stride = 1ull << shift;
      dk.range = 1ull << b;
      shift += b;
    }
    uint64_t est = std::min<uint64_t>((uint64_t)std::max<int64_t>(t->nrows, 1), 1ull << 26);
    uint64_t cap = 1024;
    if (c->opt[kOptHashSlots]) est = (uint64_t)c->opt[kOptHashSlots] / 2;
    while (cap < 2 * est) cap <<= 1;
    // a table that overflowed on this query grows (run_groupby_grow re-runs the query)
    if (c->hash_grow > cap) cap = c->hash_grow;
    pl.nslots = cap;
    pl.mode = kGlobalHash;
    pl.p.hash = wide ? 2 : 1;
    if (wide)
      for (int k = 0; k < q->n_keys; ++k) {
        pl.p.keys[k].stride = 1;
        pl.p.keys[k].range = 0;
      }
  } else {
    uint64_t stride = 1;
    for (int k = q->n_keys - 1; k >= 0; --k) {
      DevKey& dk = pl.p.keys[k];
      dk.stride = stride;
      stride *= dk.range;
    }
    pl.nslots = (uint64_t)space;
    pl.p.hash = 0;
    const size_t per_slot_private = 8 + 8 * (size_t)pl.nsum;  // bytes per lane per slot
    const size_t per_slot_shared = 8 + 8 * (size_t)pl.nsum + (pl.fx_states ? 8 * kFxWords * (size_t)pl.nsum : 0);
    if (pl.nslots <= (uint64_t)kMaxPrivateSlots && pl.nslots * per_slot_private * kBlock <= 80 * 1024)
      pl.mode = kPrivate;
    else if (pl.nslots * per_slot_shared <= 64 * 1024) pl.mode = kShared;
    else {
      // partitioned aggregation: 2^wbits slots of LDS state per partition (64 KiB: two
      // aggregate workgroups per CU; up to 128 KiB when the slot space needs it), at most
      // kPartMaxParts partitions
      const size_t per_slot = 8 + 8 * (size_t)pl.nsum + (pl.fx_states ? 8 * kFxWords * (size_t)pl.nsum : 0);
      int wbits = 12;
      if (c->opt[kOptPartWbits]) wbits = (int)c->opt[kOptPartWbits];
      while (wbits > 6 && ((size_t)1 << wbits) * per_slot > 128 * 1024) --wbits;
      if (!c->opt[kOptPartWbits] && ((size_t)2 << wbits) * per_slot <= 128 * 1024) ++wbits;  // fewer, longer runs
      while (((pl.nslots + (1ull << wbits) - 1) >> wbits) > (uint64_t)kPartMaxParts &&
             ((size_t)2 << wbits) * per_slot <= 128 * 1024)
        ++wbits;
      pl.wbits = wbits;
      const uint64_t parts = (pl.nslots + (1ull << wbits) - 1) >> wbits;
      pl.mode = (parts <= (uint64_t)kPartMaxParts && part_scatter_lds((int)parts, 256, pl.nsum) <= 150 * 1024 &&
                 c->opt[kOptPartition] != 0)
                    ? kPartitioned
                    : kGlobalDense;
    }
  }
  pl.p.nslots = pl.nslots;
}

// ------------------------------------------------------------------------------------
// emit description
// ------------------------------------------------------------------------------------
int agg_out_dtype(int op, int in_dt) {
  if (op == BQG_COUNT || op == BQG_COUNT_DISTINCT || op == BQG_SORTED_COUNT_DISTINCT) return BQG_I64;
  if (op == BQG_MEAN || op == BQG_STD) return BQG_F64;
  return in_dt;
}

// The compact copy of table column `tc` (Column::shadow), built if needed: kind 1 for an
// integer column whose range fits fewer bytes, kind 2 for a float64 column with exact int32
// codes; returns false when the column has none of the wanted kind.
bool ensure_shadow(bqg_ctx* c, bqg_table* t, int tc, int kind) {
  Column& col = t->cols[tc];
  compute_stats(t, tc);
  const ColStats& cs = col.stats;
  Shadow& sh = col.shadow;
  int dtype = 0, enc = 0;
  int64_t off = 0;
  double mul = 0;
  if (kind == 1) {
    if (dtype_is_float(col.dtype) || col.dtype == BQG_BOOL || col.dtype == BQG_U64 || cs.empty) return false;
    const uint64_t range = (uint64_t)cs.imax - (uint64_t)cs.imin;
    const int lg = range < 0x100ull ? 0 : range < 0x10000ull ? 1 : range < 0x100000000ull ? 2 : 3;
    if (lg >= dtype_lg(col.dtype)) return false;  // no narrower
    dtype = lg == 0 ? BQG_U8 : lg == 1 ? BQG_U16 : BQG_U32;
    enc = 1;
    off = cs.imin;
  } else {
    if (col.dtype != BQG_F64 || !cs.enc || cs.empty) return false;
    enc = 2;
    mul = cs.enc == 1 ? std::ldexp(1.0, cs.enc_k) : 100.0;
    // the codes' range (exact products for dyadic codes, rint is monotonic for cents)
    const int64_t cmin = (int64_t)(cs.enc == 1 ? cs.fmin * mul : std::rint(cs.fmin * mul));
    const int64_t cmax = (int64_t)(cs.enc == 1 ? cs.fmax * mul : std::rint(cs.fmax * mul));
    const uint64_t span = (uint64_t)cmax - (uint64_t)cmin;
    dtype = span < 0x100ull ? BQG_U8 : span < 0x10000ull ? BQG_U16 : BQG_I32;
    if (c->opt[kOptCompact] == 2) dtype = BQG_I32;  // option compact=2: int32 codes only
    off = dtype == BQG_I32 ? 0 : cmin;
  }
  if (sh.valid && sh.dtype == dtype && sh.enc == enc && sh.off == off && sh.mul == mul) return true;
  const size_t need = column_bytes(t->nrows, dtype);
  if (sh.bytes < need) {
    c->colpool.put(sh.dev, sh.bytes);
    size_t cap = 0;
    // no other table's copy is dropped for this one (a scan being planned may already read it)
    sh.dev = (unsigned char*)col_alloc(c, need, &cap, false);
    sh.bytes = sh.dev ? cap : 0;
    if (!sh.dev) {  // no room: the scan reads the column itself
      sh = Shadow{};
      return false;
    }
  }
  if (c->timing == 1 && !c->sh_timed) HIPCHECK(hipEventRecord(c->ev_sh[0], c->stream));
  // zero padding past the last row (the scans' vector loads read it), then the rows
  const size_t used = (size_t)t->nrows * dtype_size(dtype);
  HIPCHECK(hipMemsetAsync(sh.dev + used, 0, sh.bytes - used, c->stream));
  if (enc == 1) launch_shadow_int(DevCol{col.dev, col.dtype, dtype_lg(col.dtype)}, t->nrows, off, sh.dev, dtype_lg(dtype), c->stream);
  else launch_shadow_code((const double*)col.dev, t->nrows, cs.enc, mul, off, sh.dev, dtype_lg(dtype), c->stream);
  HIPCHECK(hipGetLastError());
  if (c->timing == 1) {
    HIPCHECK(hipEventRecord(c->ev_sh[1], c->stream));
    c->sh_timed = true;
  }
  sh.valid = true;
  sh.dtype = dtype;
  sh.enc = enc;
  sh.off = off;
  sh.mul = mul;
  return true;
}

// The scan parameters with the columns' compact resident copies where they have one (option
// compact; private, shared and dense global scans): integer keys / terms / sums as narrow
// offsets (the decode restores the canonical value), float64 columns that are only summed as
// their exact int32 codes, summed as integers and scaled back once at emit (EmitParams::
// sum_dec) -- fewer HBM bytes for the same rows.  pl.alg_bytes follows the bytes read.
ScanParams compact_scan(bqg_ctx* c, bqg_table* t, Plan& pl, EmitParams& e) {
  ScanParams sp = pl.p;
  if (!c->opt[kOptCompact] || pl.p.hash) return sp;
  const int64_t N = t->nrows;
  for (int i = 0; i < sp.ncols; ++i) {
    const int tc = pl.tcol[i];
    Column& col = t->cols[tc];
    bool other = i == sp.mask_col;  // used as anything but a plain sum state
    for (int k = 0; k < sp.nkeys; ++k) other |= sp.keys[k].col == i;
    for (int k = 0; k < sp.nterms; ++k) other |= sp.terms[k].col == i;
    const bool sum_only = i < pl.nsum && !other &&
                          std::find(pl.std_cols.begin(), pl.std_cols.end(), i) == pl.std_cols.end();
    if (ensure_shadow(c, t, tc, 1)) {
      sp.cols[i] = DevCol{col.shadow.dev, col.shadow.dtype, dtype_lg(col.shadow.dtype), 1, 0, col.shadow.off};
    } else if (sum_only && ensure_shadow(c, t, tc, 2)) {
      // int32 codes as they are; 1 / 2-byte codes as offsets (the decode adds the smallest back)
      const Shadow& sh = col.shadow;
      sp.cols[i] = DevCol{sh.dev, sh.dtype, dtype_lg(sh.dtype), sh.dtype == BQG_I32 ? 0 : 1, 0, sh.off};
      sp.sum_is_float[i] = 0;
      sp.sum_conv[i] = 1;
      sp.sum_enc[i] = 0;
      e.sum_dec[i] = col.shadow.mul;
      // the state now sums integer codes: it is no fixed-point limb sum (with part_narrow=0 the
      // plan may have made it one), so k_fx_finalize must leave its accumulator alone
      pl.fx_states &= ~(1 << i);
      pl.fx_slot_states &= ~(1 << i);
    }
    // bytes read (the algorithmic bytes keep the stored width)
    if (!pl.dummy_col) pl.read_bytes -= ((int64_t)dtype_size(col.dtype) - ((int64_t)1 << sp.cols[i].lg)) * N;
    // a key / term column that is not summed works in its copy's own domain (stored = value
    // - off): key minima and scalar term constants shift by -off instead of every row adding
    // off back (an `in` / `nin` list keeps the decode offset; its values stay canonical)
    if (sp.cols[i].enc != 1 || i < pl.nsum) continue;
    bool list = false;
    for (int k = 0; k < sp.nterms; ++k)
      list |= sp.terms[k].col == i && (sp.terms[k].op == BQG_T_IN || sp.terms[k].op == BQG_T_NIN);
    if (list) continue;
    const int64_t off = sp.cols[i].off;
    for (int k = 0; k < sp.nkeys; ++k)
      if (sp.keys[k].col == i) sp.keys[k].min = (int64_t)((uint64_t)sp.keys[k].min - (uint64_t)off);
    for (int k = 0; k < sp.nterms; ++k) {
      DevTerm& tm = sp.terms[k];
      if (tm.col != i || tm.op < BQG_T_EQ || tm.op > BQG_T_LE) continue;
      // stored values lie in [0, 2^32): a constant clamped into int64 compares the same
      const __int128 v = (__int128)tm.iv0 - off;
      tm.iv0 = v < (__int128)INT64_MIN ? INT64_MIN : v > (__int128)INT64_MAX ? INT64_MAX : (int64_t)v;
    }
    sp.cols[i].enc = 0;
    sp.cols[i].off = 0;
  }
  return sp;
}

// Float sum states whose column has an exact int64 code for every value (ColStats::enc64) and
// is not centred: ScanParams::sum_enc / sum_mul for the kernels, and (atomic modes, whose
// accumulators keep the codes to the emit) EmitParams::sum_dec
void set_sum_codes(bqg_table* t, Plan& pl, EmitParams* e) {
  for (int q = 0; q < pl.nsum; ++q) {
    if (!pl.p.sum_is_float[q] || pl.p.sum_centered[q]) continue;
    compute_stats(t, pl.tcol[q]);
    const ColStats& cs = t->cols[pl.tcol[q]].stats;
    if (!cs.enc64) continue;
    pl.p.sum_enc[q] = cs.enc64;
    pl.p.sum_mul[q] = cs.enc64 == 1 ? std::ldexp(1.0, cs.enc64_k) : 100.0;
    if (e) e->sum_dec[q] = pl.p.sum_mul[q];
  }
}

// The fixed-point states of pass 1 (Plan::fx_states; the atomic / partitioned-wide modes, after
// set_sum_codes): ScanParams::sum_enc 3, the shift set by plan_query
void set_sum_fx(Plan& pl) {
  for (int q = 0; q < pl.nsum; ++q)
    if ((pl.fx_states >> q) & 1) pl.p.sum_enc[q] = 3;
}

void build_emit(bqg_table* t, const bqg_query* q, const Plan& pl, EmitParams& e, std::vector<int>& out_dt) {
  memset(&e, 0, sizeof(e));
  e.nkeys = q->n_keys;
  e.hash = pl.p.hash;
  e.ncols = q->n_keys + q->n_aggs;
  for (int k = 0; k < q->n_keys; ++k) {
    e.keys[k] = pl.p.keys[k];
    e.key_dtype[k] = t->cols[q->key_cols[k]].dtype;
    const Column& kc = t->cols[q->key_cols[k]];
    e.key_cols[k] = DevCol{kc.dev, kc.dtype, dtype_lg(kc.dtype)};
    EmitCol& ec = e.cols[k];
    ec.kind = 0;
    ec.key = k;
    ec.out_dtype = e.key_dtype[k];
    out_dt.push_back(ec.out_dtype);
  }
  int ncd = 0, nscd = 0;
  for (int a = 0; a < q->n_aggs; ++a) {
    const bqg_agg& g = q->aggs[a];
    EmitCol& ec = e.cols[q->n_keys + a];
    const int in_dt = t->cols[g.col].dtype;
    ec.kind = 1;
    ec.op = g.op;
    ec.in_dtype = in_dt;
    ec.in_float = dtype_is_float(in_dt);
    ec.out_dtype = agg_out_dtype(g.op, in_dt);
    // a mean over an integer column's float64 sum state (plan_query: 64-bit sums that can wrap)
    if (g.op == BQG_MEAN) ec.in_float = pl.p.sum_is_float[pl.agg_state[a]];
    if (g.op == BQG_MEAN || g.op == BQG_STD) ec.sum_state = pl.agg_state[a];
    if (g.op == BQG_SUM || g.op == BQG_MEAN) ec.state = pl.agg_state[a];
    else if (g.op == BQG_STD) {
      int idx = 0;
      for (size_t i = 0; i < pl.std_cols.size(); ++i)
        if (pl.std_cols[i] == pl.agg_state[a]) idx = (int)i;
      ec.state = idx;
    } else if (g.op == BQG_COUNT_DISTINCT) ec.state = ncd++;
    else if (g.op == BQG_SORTED_COUNT_DISTINCT) ec.state = nscd++;
    out_dt.push_back(ec.out_dtype);
  }
  e.nsum2 = (int)pl.std_cols.size();
}

// workgroups per CU for the private-LDS scan (tools/membench.hip: 2-4 per CU stream best
// with non-temporal loads; the grid still strides over >= 97 k tiles at C2 size)
constexpr size_t kPrivatePerCu = 4;

int scan_blocks(bqg_ctx* c, int64_t nrows, int per_cu) {
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  int64_t b = (int64_t)c->cu * per_cu;
  if (b > tiles) b = tiles;
  if (b < 1) b = 1;
  return (int)b;
}

// Every planned launch is checked against the device's limits before it is issued: a shape the
// planner (or an engine option) gets wrong fails the query with BQG_E_INVALID and a message
// instead of surfacing as a launch failure from hipGetLastError.
void check_launch(bqg_ctx* c, const char* what, size_t lds, int64_t blocks, int threads = kBlock) {
  if (lds > c->max_lds)
    fail(BQG_E_INVALID, "%s: %zu bytes of LDS per workgroup exceed the device's %zu", what, lds, c->max_lds);
  if (blocks < 1 || blocks > 0x7FFFFFFFll) fail(BQG_E_INVALID, "%s: grid of %lld workgroups", what, (long long)blocks);
  if (threads < 64 || threads > 1024 || threads % 64) fail(BQG_E_INVALID, "%s: %d threads per workgroup", what, threads);
}

bqg_result* empty_result(const std::vector<int>& dts, int filtered) {
  bqg_result* r = new bqg_result();
  r->n_rows = 0;
  r->filtered = filtered;
  for (int dt : dts) {
    r->dtypes.push_back(dt);
    r->small.emplace_back(8);
  }
  for (auto& d : r->small) r->ptrs.push_back(d.data());
  return r;
}

// result over a pinned block: column j at base + offsets[j]
bqg_result* block_result(bqg_ctx* c, PinnedBlock b, int64_t n, int filtered, const std::vector<int>& dts,
                         const std::vector<size_t>& offsets) {
  bqg_result* r = new bqg_result();
  r->pool = c->pool;
  r->block = b;
  r->n_rows = n;
  r->filtered = filtered;
  for (size_t j = 0; j < dts.size(); ++j) {
    r->dtypes.push_back(dts[j]);
    r->ptrs.push_back((const unsigned char*)b.p + offsets[j]);
  }
  return r;
}

// Column storage from the context's pool; zero_all: zero the whole allocation (public table
// creation), else only the padding past the last row (the caller fills the rows).
void alloc_column(bqg_ctx* c, Column& col, int64_t nrows, bool zero_all) {
  const size_t need = column_bytes(nrows, col.dtype);
  size_t cap = 0;
  col.dev = (unsigned char*)col_alloc(c, need, &cap);
  if (!col.dev) fail(BQG_E_OOM, "device allocation of a column (%zu bytes) failed", need);
  col.bytes = cap;
  const size_t used = zero_all ? 0 : (size_t)nrows * dtype_size(col.dtype);
  HIPCHECK(hipMemsetAsync(col.dev + used, 0, cap - used, c->stream));
}

// Result as a new device table: device-to-device copies of the output columns (dev_target).
void table_from_device(bqg_ctx* c, const std::vector<int>& dts, const std::vector<const void*>& src, int64_t n) {
  std::unique_ptr<bqg_table> t(new bqg_table());
  t->ctx = c;
  t->nrows = n;
  for (int dt : dts) {
    Column col;
    col.dtype = dt;
    t->cols.push_back(col);
  }
  struct Undo {
    bqg_table* t;
    ~Undo() {
      if (t)
        for (Column& col : t->cols) t->ctx->colpool.put(col.dev, col.bytes);
    }
  } undo{t.get()};
  // one kernel copies the rows and zeroes every column's tail (a fill and a copy per column
  // cost ~10 us each: ~40 us of C5's shard pass); per-column calls when a pointer or size is
  // not 16-byte aligned
  for (Column& col : t->cols) {
    size_t cap = 0;
    col.dev = (unsigned char*)col_alloc(c, column_bytes(n, col.dtype), &cap);
    if (!col.dev) fail(BQG_E_OOM, "device allocation of a column (%zu bytes) failed", column_bytes(n, col.dtype));
    col.bytes = cap;
  }
  bool one = dts.size() <= (size_t)kMaxCopyCols;
  for (size_t j = 0; j < dts.size() && one; ++j)
    one = ((uintptr_t)src[j] & 15) == 0 && ((uintptr_t)t->cols[j].dev & 15) == 0 && (t->cols[j].bytes & 15) == 0;
  if (one) {
    ColumnCopies cc{};
    cc.n = (int)dts.size();
    for (size_t j = 0; j < dts.size(); ++j) {
      cc.dst[j] = t->cols[j].dev;
      cc.src[j] = (const unsigned char*)src[j];
      cc.used[j] = (uint64_t)n * dtype_size(dts[j]);
      cc.cap[j] = t->cols[j].bytes;
    }
    launch_column_copies(cc, c->stream);
    HIPCHECK(hipGetLastError());
  } else {
    for (size_t j = 0; j < dts.size(); ++j) {
      Column& col = t->cols[j];
      const size_t used = (size_t)n * dtype_size(dts[j]);
      HIPCHECK(hipMemsetAsync(col.dev + used, 0, col.bytes - used, c->stream));
      if (n > 0) HIPCHECK(hipMemcpyAsync(col.dev, src[j], used, hipMemcpyDeviceToDevice, c->stream));
    }
  }
  HIPCHECK(hipStreamSynchronize(c->stream));
  undo.t = nullptr;
  c->tables.push_back(t.get());
  *c->dev_target = t.release();
}

// Small host result (empty tables, the zero-key 'Total' row) as a new device table.
void table_from_host_result(bqg_ctx* c, bqg_result* r) {
  std::unique_ptr<bqg_result> own(r);
  bqg_table* t = nullptr;
  const int rc = bqg_table_create(c, r->n_rows, (int32_t)r->dtypes.size(), r->dtypes.data(), &t);
  if (rc != BQG_OK) throw ApiError{rc, c->err};
  for (size_t j = 0; j < r->dtypes.size(); ++j)
    if (r->n_rows > 0)
      HIPCHECK(hipMemcpyAsync(t->cols[j].dev, r->ptrs[j], (size_t)r->n_rows * dtype_size(r->dtypes[j]), hipMemcpyHostToDevice,
                              c->stream));
  HIPCHECK(hipStreamSynchronize(c->stream));
  *c->dev_target = t;
}

// After the query's last synchronisation: the byte counts of the last call (algorithmic and
// read, each + the G x ncols output) and, with timing on, its HIP-event times
void finish_query(bqg_ctx* c, const Plan& pl, int64_t G, int ncols) {
  const int64_t out = G * (int64_t)ncols * 8;
  c->last.bytes = pl.alg_bytes + out;
  c->last.bytes_read = pl.read_bytes + out;
  c->last.compact_ms = NAN;
  c->last.copy_ms = NAN;
  if (!c->timing) return;
  float ms = 0;
  HIPCHECK(hipEventElapsedTime(&ms, c->ev[1], c->ev[2]));
  c->last.scan_ms = ms;
  c->scan_ms_sum += ms;
  ++c->timed_queries;
  c->last.total_ms = NAN;
  if (c->timing == 1) {
    HIPCHECK(hipEventElapsedTime(&ms, c->ev[0], c->ev[3]));
    c->last.total_ms = ms;
    c->last.compact_ms = 0.0;
    if (c->sh_timed) {
      HIPCHECK(hipEventElapsedTime(&ms, c->ev_sh[0], c->ev_sh[1]));
      c->last.compact_ms = ms;
    }
    c->last.copy_ms = 0.0;
    if (c->copy_timed) {
      HIPCHECK(hipEventElapsedTime(&ms, c->ev_copy, c->ev[3]));
      c->last.copy_ms = ms;
    }
  }
}

// Runs the passes of one groupby; returns the device output columns through `res`.
void run_groupby(bqg_ctx* c, bqg_table* t, const bqg_query* q, bqg_result** out) {
  c->sh_timed = false;
  c->copy_timed = false;
  Plan pl;
  plan_query(c, t, q, pl);
  EmitParams e;
  std::vector<int> out_dt;
  build_emit(t, q, pl, e, out_dt);
  const int64_t N = t->nrows;
  c->last = bqg_timing{};
  c->last.rows = N;
  c->last.mode = pl.mode;
  c->last.scan_launches = pl.mode == kPartitioned ? 2 : 1;

  // bquery's zero-key, unfiltered, empty-table case yields one 'Total' row of zeros
  if (N == 0) {
    if (q->n_keys == 0 && !pl.has_filter) {
      bqg_result* r = new bqg_result();
      r->n_rows = 1;
      for (size_t j = 0; j < out_dt.size(); ++j) {
        r->dtypes.push_back(out_dt[j]);
        r->small.emplace_back(8, 0);
        const bqg_agg& g = q->aggs[j];
        if (g.op == BQG_STD) {
          const double nan = NAN;
          memcpy(r->small.back().data(), &nan, 8);
        }
      }
      for (auto& d : r->small) r->ptrs.push_back(d.data());
      *out = r;
    } else {
      *out = empty_result(out_dt, 0);
    }
    return;
  }

  bool distinct_ops = false;
  for (int a = 0; a < q->n_aggs; ++a)
    if (q->aggs[a].op == BQG_COUNT_DISTINCT || q->aggs[a].op == BQG_SORTED_COUNT_DISTINCT) distinct_ops = true;
  const bool need_generic = distinct_ops || !pl.std_cols.empty() || pl.mode != kPrivate || pl.nf_states != 0;

  const uint64_t S = pl.nslots;
  const int nsum = pl.nsum;
  const int nsum2 = (int)pl.std_cols.size();
  // slot arrays: cnt | fst | acc | acc2 | keys | hash counters | fixed-point limbs (pass 1, std pass)
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  const size_t o_cnt = carve(S * 8), o_fst = carve(S * 4), o_acc = carve(S * 8 * std::max(nsum, 1)),
               o_acc2 = carve(S * 8 * std::max(nsum2, 1)), o_keys = carve(pl.p.hash ? S * 8 : 8),
               o_hc = carve(16);
  const bool atomic_mode = pl.mode != kPrivate;
  // (the std pass's shared table with limbs: one workgroup per CU at most; past the LDS its
  // centred squares keep the float64 atomics)
  const bool fx1 = atomic_mode && pl.fx_states != 0,
             fx2 = atomic_mode && pl.fx2_states != 0 && !(pl.mode == kShared && shared_lds(S, nsum2, true) > c->max_lds);
  const size_t o_fx = fx1 ? carve(S * 8 * kFxWords * (size_t)nsum) : 0,
               o_fx2 = fx2 ? carve(S * 8 * kFxWords * (size_t)nsum2) : 0,
               o_fxe = fx1 && pl.fx_slot_states ? carve(S * 4 * (size_t)nsum) : 0;
  unsigned char* sbase = (unsigned char*)c->slots.ensure(off);
  SlotArrays sa{};
  sa.cnt = (unsigned long long*)(sbase + o_cnt);
  sa.fst = (uint32_t*)(sbase + o_fst);
  sa.acc = (unsigned long long*)(sbase + o_acc);
  sa.acc2 = nsum2 ? (unsigned long long*)(sbase + o_acc2) : nullptr;
  sa.keys = pl.p.hash ? (unsigned long long*)(sbase + o_keys) : nullptr;
  sa.hash_fill = (unsigned int*)(sbase + o_hc);
  sa.overflow = sa.hash_fill + 1;
  sa.fx = fx1 ? (unsigned long long*)(sbase + o_fx) : nullptr;

  // output columns (device), capacity S rows (private) or G rows (generic, sized later)
  hipStream_t st = c->stream;
  if (c->timing == 1) HIPCHECK(hipEventRecord(c->ev[0], st));

  // count / distinct-only queries on a small dense slot space: one fused pass
  // (k_scd_fused) produces rows, first rows, sorted_count_distinct and one count_distinct
  int ncd = 0, nscd = 0;
  for (int a = 0; a < q->n_aggs; ++a) ncd += q->aggs[a].op == BQG_COUNT_DISTINCT, nscd += q->aggs[a].op == BQG_SORTED_COUNT_DISTINCT;
  bool fused = !pl.p.hash && nsum == 0 && nsum2 == 0 && nscd == 1 && ncd <= 1 && N < (int64_t)kNoRow &&
               (kBlock / 64) * scd_fused_wave_lds(S) <= kScdFusedMaxLds && c->opt[kOptFusedScd] != 0;
  if (fused && ncd == 1) {
    for (int a = 0; a < q->n_aggs; ++a) {
      if (q->aggs[a].op != BQG_COUNT_DISTINCT) continue;
      Column& col = t->cols[q->aggs[a].col];
      compute_stats(t, q->aggs[a].col);
      if (dtype_is_float(col.dtype)) {
        fused = false;
      } else {
        const uint64_t vr = col.stats.empty ? 1 : (uint64_t)col.stats.imax - (uint64_t)col.stats.imin + 1;
        if (vr == 0 || (unsigned __int128)S * vr > ((unsigned __int128)1 << 30)) fused = false;
      }
    }
  }

  if (fused) {
    // the scan is the fused distinct pass below
    c->last.mode = 5;
  } else if (pl.mode == kPrivate) {
    // the scan's columns as their compact resident copies where they have one (option
    // compact): integer keys / terms / sums as narrow offsets (the decode restores the
    // canonical value), float64 columns that are only summed as their exact int32 codes,
    // summed as integers and scaled back once at emit -- fewer HBM bytes for the same rows
    ScanParams sp = compact_scan(c, t, pl, e);
    int row_bytes = 0;
    for (int i = 0; i < sp.ncols; ++i) row_bytes += 1 << sp.cols[i].lg;
    const size_t lds = (size_t)S * kBlock * (8 + 8 * (size_t)nsum);
    // workgroups per CU: 3 when a row reads more than 4 bytes (C2 as stored, 16 B/row: 0.2441 ->
    // 0.2363 ms against 4, profiles/r5g_c2_launch_sweep.txt), 4 for the narrow compact rows
    int per_cu = (int)std::min<size_t>(row_bytes > 4 ? 3 : kPrivatePerCu, c->max_lds / std::max<size_t>(lds, 1));
    if (c->opt[kOptPrivatePerCu]) per_cu = std::min<int>((int)(c->max_lds / std::max<size_t>(lds, 1)), (int)c->opt[kOptPrivatePerCu]);
    if (per_cu < 1) per_cu = 1;
    PrivateLaunch L{};
    L.blocks = scan_blocks(c, N, per_cu);
    L.lds_bytes = lds;
    L.partials = (unsigned long long*)c->partials.ensure((size_t)(2 + nsum) * L.blocks * S * 8);
    FinishParams F{};
    F.nslots = (int)S;
    F.blocks = L.blocks;
    F.nsum = nsum;
    for (int i = 0; i < kMaxSums; ++i) F.sum_is_float[i] = sp.sum_is_float[i];
    F.partials = L.partials;
    F.out_hdr = (unsigned long long*)c->hdr.ensure(64);
    F.totals = (unsigned long long*)c->counter.ensure((size_t)(2 + kMaxSums) * kMaxPrivateSlots * 8);
    F.done = (unsigned int*)c->done.p;
    F.emit_inline = need_generic ? 0 : 1;
    // host result: the finish step writes [64-byte header | columns of S rows] straight into
    // a pooled pinned block (device-mapped host memory: no copy); device result: into HBM
    BlockGuard hblk;
    const size_t colbytes = (size_t)e.ncols * S * 8;
    if (F.emit_inline) {
      unsigned char* ob;
      if (!c->dev_target) {
        hblk.reset(c->pool, c->pool_get(colbytes + 64));
        ob = (unsigned char*)hblk.b.dev;
      } else {
        ob = (unsigned char*)c->outcols.ensure(64 + colbytes + 256);
      }
      F.out_hdr = (unsigned long long*)ob;
      for (int j = 0; j < e.ncols; ++j) e.cols[j].out = ob + 64 + (size_t)j * S * 8;
    }
    hipFunction_t jfn = nullptr;
    if (c->opt[kOptJit] && N >= c->jit_min_rows()) {
      // tiles in flight per workgroup (profiling option; default in scan_private.h)
      // (default: 3 when the scan reads at most 4 bytes per row -- compact copies: each tile is
      // small, and one in flight leaves the waves parked on memory; r4x8: C2 0.072 -> 0.069
      // ms -- else the kernel's 1)
      const int64_t ahead = c->opt[kOptPrivAhead] ? c->opt[kOptPrivAhead] : (row_bytes <= 4 ? 3 : 0);
      std::string extra;
      if (ahead) extra = std::string("#define BQ_PRIV_AHEAD ") + std::to_string(ahead) + "\n";
      jfn = jit_function_for("bq_jit_scan_private", sp, extra, c->opt[kOptJitAsync] != 0);
    }
    check_launch(c, "private scan", L.lds_bytes, L.blocks);
    if (c->timing) HIPCHECK(hipEventRecord(c->ev[1], st));
    if (jfn) {
      void* args[] = {(void*)&sp, (void*)&L};
      HIPCHECK(hipModuleLaunchKernel(jfn, (unsigned)L.blocks, 1, 1, kBlock, 1, 1, (unsigned)L.lds_bytes, st, args,
                                     nullptr));
      c->last.specialized = 1;
    } else {
      launch_scan_private(sp, L, st);
    }
    HIPCHECK(hipGetLastError());
    if (c->timing) HIPCHECK(hipEventRecord(c->ev[2], st));
    launch_private_finish(F, sa, e, st);
    HIPCHECK(hipGetLastError());
    if (!need_generic && c->dev_target) {
      unsigned long long* hh = (unsigned long long*)c->hhdr.ensure(64);
      HIPCHECK(hipMemcpyAsync(hh, F.out_hdr, 16, hipMemcpyDeviceToHost, st));
      if (c->timing == 1) HIPCHECK(hipEventRecord(c->ev[3], st));
      HIPCHECK(hipStreamSynchronize(st));
      std::vector<const void*> src;
      for (int j = 0; j < e.ncols; ++j) src.push_back(e.cols[j].out);
      table_from_device(c, out_dt, src, (int64_t)hh[0]);
      finish_query(c, pl, (int64_t)hh[0], e.ncols);
      return;
    }
    if (!need_generic) {
      unsigned char* h = (unsigned char*)hblk.b.p;
      if (c->timing == 1) HIPCHECK(hipEventRecord(c->ev[3], st));
      HIPCHECK(hipStreamSynchronize(st));
      const unsigned long long G = ((unsigned long long*)h)[0], total = ((unsigned long long*)h)[1];
      std::vector<size_t> offs;
      for (int j = 0; j < e.ncols; ++j) offs.push_back(64 + (size_t)j * S * 8);
      bqg_result* r = block_result(c, hblk.release(), (int64_t)G, pl.has_filter && (int64_t)total < N, out_dt, offs);
      finish_query(c, pl, (int64_t)G, e.ncols);
      *out = r;
      return;
    }
  } else {
    // the partitioned aggregate writes every slot itself (no initialisation pass)
    if (pl.mode != kPartitioned) launch_init_slots(sa, nsum, S, st);
    // atomic modes: float sums of exactly codable columns accumulate integer codes (the same
    // column statistics as the partitioned narrow entries) -- bit-reproducible sums; the emit
    // scales them back
    if (pl.mode != kPartitioned && c->opt[kOptPartNarrow] != 0) set_sum_codes(t, pl, &e);
    // the other float sums as fixed-point limbs (the same bits on every run)
    if (pl.mode != kPartitioned) set_sum_fx(pl);
    if (pl.p.hash) HIPCHECK(hipMemsetAsync(sa.hash_fill, 0, 8, st));  // (+ overflow flag)
    // fixed-point states with per-slot shifts: each slot's largest exponent first (one pass over
    // the same rows; the hash modes insert their keys here already)
    auto fx_emax_pass = [&]() {
      if (!fx1 || !pl.fx_slot_states) return;
      FxEmaxLaunch fe{};
      int32_t* em = (int32_t*)(sbase + o_fxe);
      HIPCHECK(hipMemsetAsync(em, 0, S * 4 * (size_t)nsum, st));
      for (int q = 0; q < nsum; ++q)
        if ((pl.fx_slot_states >> q) & 1) pl.p.fx_emax[q] = fe.emax[q] = em + (size_t)q * S;
      launch_fx_emax(pl.p, sa, fe, scan_blocks(c, N, 8), st);
      HIPCHECK(hipGetLastError());
    };
    if (pl.mode != kPartitioned) fx_emax_pass();
    // shared / dense global scans read the columns' compact copies (after set_sum_codes: a
    // code-copy column's state sums the codes as integers)
    ScanParams sp = pl.mode == kPartitioned ? pl.p : compact_scan(c, t, pl, e);
    if (c->timing) HIPCHECK(hipEventRecord(c->ev[1], st));
    if (pl.mode == kShared) {
      const size_t lds = shared_lds(S, nsum, fx1);
      int per_cu = (int)std::min<size_t>(8, c->max_lds / std::max<size_t>(lds, 1));
      check_launch(c, "shared scan", lds, scan_blocks(c, N, std::max(per_cu, 1)));
      launch_scan_shared(sp, sa, scan_blocks(c, N, std::max(per_cu, 1)), lds, st);
    } else if (pl.mode == kPartitioned) {
      PartLaunch L{};
      L.wbits = pl.wbits;
      L.nparts = (int)((S + (1ull << pl.wbits) - 1) >> pl.wbits);
      // narrow entries: every summed column is a float column whose values all have an exact
      // 32-bit integer code (column statistics): 8-byte instead of 12-byte C3 entries, and the
      // sums are exact integer sums scaled back once (option part_narrow=0 turns it off)
      L.narrow = nsum > 0 && c->opt[kOptPartNarrow] != 0;
      for (int q = 0; q < nsum && L.narrow; ++q) {
        compute_stats(t, pl.tcol[q]);
        const Column& col = t->cols[pl.tcol[q]];
        const ColStats& cs = col.stats;
        if (pl.p.sum_centered[q]) {
          L.narrow = 0;
        } else if (pl.p.sum_is_float[q]) {
          L.narrow = cs.enc != 0;
          L.enc_kind[q] = cs.enc;
          L.enc_mul[q] = cs.enc == 1 ? std::ldexp(1.0, cs.enc_k) : 100.0;
        } else {
          // integers (not uint64) whose values span fewer than 2^32: code = v - min
          L.narrow = col.dtype != BQG_U64 && pl.p.sum_conv[q] == 1 &&
                     (cs.empty || (uint64_t)cs.imax - (uint64_t)cs.imin <= 0xFFFFFFFFull);
          L.enc_kind[q] = 3;
          L.enc_off[q] = cs.empty ? 0 : cs.imin;
        }
      }
      // wide entries: float sums of int64-codable columns add codes (deterministic); the
      // combine scales them back
      if (!L.narrow && c->opt[kOptPartNarrow] != 0) set_sum_codes(t, pl, nullptr);
      // ... and the other float sums of wide entries as fixed-point limbs
      if (!L.narrow) set_sum_fx(pl);
      L.fx = !L.narrow && pl.fx_states != 0;
      if (L.fx) fx_emax_pass();
      // packed 4-byte entries (option part_pack): no summed column, or one narrow-coded
      // column whose codes span at most 2^16 values -- {code16, slot_low} per entry
      L.pack = 0;
      uint64_t span16 = 0;
      // (packed entries key first appearances by 32-bit tile x tile rows: tables below 2^32 - 2^14 rows)
      if (c->opt[kOptPartPack] && pl.wbits <= 16 && (nsum == 0 || (nsum == 1 && L.narrow)) &&
          N < (int64_t)0xFFFFFFFFll - 16384) {
        L.pack = 1;
        L.enc_base16 = 0;
        const ColStats& cs = nsum ? t->cols[pl.tcol[0]].stats : ColStats{};
        if (nsum && !cs.empty) {
          if (L.enc_kind[0] == 3) {
            span16 = (uint64_t)cs.imax - (uint64_t)cs.imin;  // codes are v - min already
          } else {
            // the device's code of a value is monotonic in it: the codes of min and max bound all
            const double lo = cs.fmin * L.enc_mul[0], hi = cs.fmax * L.enc_mul[0];
            const int64_t clo = (int64_t)(L.enc_kind[0] == 1 ? lo : std::rint(lo));
            const int64_t chi = (int64_t)(L.enc_kind[0] == 1 ? hi : std::rint(hi));
            span16 = (uint64_t)(chi - clo);
            L.enc_base16 = clo;
          }
          if (span16 > 0xFFFFull) L.pack = 0;
        }
      }
      // launch shape: tile size, scatter grid, aggregate splits
      auto shape = [&]() {
        const bool nw = L.narrow != 0, pk = L.pack != 0;
        // scatter workgroup: the widest whose staged tile fits in LDS (option part_threads caps it)
        L.threads = c->opt[kOptPartThreads] ? (int)c->opt[kOptPartThreads] : 1024;
        while (L.threads > 256 && part_scatter_lds(L.nparts, L.threads, nsum, 1, nw, pk) > 150 * 1024) L.threads >>= 1;
        // 8192-row tiles (two 4-row chunks per thread) when the staged tile fits: the aggregate's
        // per-tile partition segments are twice as long (option part_k=1|2 forces the choice)
        L.k = (L.threads == 1024 && part_scatter_lds(L.nparts, L.threads, nsum, 2, nw, pk) <= 150 * 1024) ? 2 : 1;
        if (c->opt[kOptPartK]) {
          // 1, 2 or (packed entries: 16384-row tiles) 4 chunks, the most that fit
          int want = c->opt[kOptPartK] >= 4 ? 4 : (int)c->opt[kOptPartK];
          while (want > 1 && !(L.threads == 1024 && (want != 4 || pk) &&
                               part_scatter_lds(L.nparts, L.threads, nsum, want, nw, pk) <= 150 * 1024))
            want >>= 1;
          L.k = want;
        }
        L.tile_rows = L.threads * kRowsPerThread * L.k;
        const int64_t tr = L.tile_rows;
        L.ntiles = (N + tr - 1) / tr;
        // contiguous whole-tile row ranges, as many scatter workgroups per CU as fit in LDS
        // (2-chunk tiles: three workgroups per CU in turn -- one fits at a time (VGPRs), the
        // shorter ranges balance the tail: scatter 0.420 -> 0.396 ms at C3, r5k)
        int per_cu = L.k == 2 ? 3 : 2;
        if (c->opt[kOptPartPerCu]) per_cu = (int)c->opt[kOptPartPerCu];
        L.blocks = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)c->cu * per_cu, L.ntiles));
        L.rows_per_block = ((L.ntiles + L.blocks - 1) / L.blocks) * tr;
        L.blocks = (int)((N + L.rows_per_block - 1) / L.rows_per_block);
        // aggregate window: the tile bounds of as many tiles as the LDS left beside the slot
        // table holds (up to kAggWinMax, in 1024-tile steps; option part_win) -- fewer windows,
        // fewer header-scan prologues; workgroups per CU stay what the slot table allows
        {
          const size_t table = part_agg_lds(L.wbits, nsum, pk, L.fx);
          const int per_cu_agg = std::max(1, (int)(c->max_lds / part_agg_lds_launch(L.wbits, nsum, pk, kAggWin, L.fx)));
          const size_t budget = c->max_lds / per_cu_agg - 1024;  // static LDS of the scans
          L.win = kAggWin;
          while (L.win + 1024 <= kAggWinMax && table + 16 * (size_t)(L.win + 1024 + kAggK + 1) <= budget) L.win += 1024;
          if (c->opt[kOptPartWin]) {
            // as asked, but no wider than the LDS beside the slot table holds
            L.win = (int)std::min<int64_t>(kAggWinMax, c->opt[kOptPartWin]);
            while (L.win > 64 && table + 16 * (size_t)(L.win + kAggK + 1) > (160 - 1) * 1024) L.win -= 64;
          }
        }
        // aggregate workgroups per partition: one round of workgroups over the CUs (a 128 KiB
        // slot table allows one per CU)
        const size_t agg_lds = part_agg_lds_launch(L.wbits, nsum, pk, L.win, L.fx);
        const int fit = std::max(1, (int)(c->max_lds / agg_lds));
        L.splits = std::max(1, (int)std::min<int64_t>(L.ntiles, (c->cu * fit + L.nparts / 2) / L.nparts));
        if (c->opt[kOptPartSplits]) L.splits = std::max(1, (int)std::min<int64_t>(L.ntiles, c->opt[kOptPartSplits]));
        if (pk) {
          // the packed accumulator: count << 40 | code16 sum, flushed every 2^23 entries (a
          // count below 2^24, a sum below 2^23 x 65535 < 2^40) -- fixed widths, so the packing
          // does not constrain the splits
          L.sbits = 40;
          L.pack_flush = 1ll << 23;
        }
      };
      shape();
      const bool nw = L.narrow != 0, pk = L.pack != 0;
      c->last.narrow = pk ? 2 : L.narrow;
      const int64_t tr = L.tile_rows;
      L.capacity = (uint64_t)L.ntiles * (uint64_t)tr;
      // (+ one spare tile of header and entry words: the packed scatter's ring writes a block's
      // tiles past its rows there, partition.h)
      L.hdr = (uint16_t*)c->prefix.ensure((size_t)(L.ntiles + 1) * (size_t)(L.nparts + 1) * 2 + 256);
      // one scratch block: entry values | entry meta | split partial tables
      // (| pack: first tile tags, tile marks)
      const size_t vbytes = pk ? 0 : ((size_t)L.capacity * (nw ? 4 : 8) * (size_t)std::max(nsum, 1) + 255) & ~size_t(255);
      const size_t mbytes = (((size_t)L.capacity + (size_t)tr) * 4 + 255) & ~size_t(255);
      // split records: [W] counts, [W] sums ([W] first rows / tiles); packed entries always
      // have one (an aggregate that flushes its accumulators adds into it)
      L.partial_bytes = ((pk ? ((size_t)1 << L.wbits) * 20 : part_agg_lds(L.wbits, nsum, pk, L.fx)) + 255) & ~size_t(255);
      const size_t pbytes = (L.splits > 1 || pk) ? (size_t)L.nparts * L.splits * L.partial_bytes : 0;
      const size_t tbytes = pk ? (((size_t)L.nparts << L.wbits) + 255) & ~size_t(255) : 0;
      // rows in tile (PartLaunch::rit) for the tiles where first appearances fall: on uniform
      // keys over S slots a slot's first row is ~exponential with mean N / (rows per slot) and
      // the last first appearance comes near S (ln S + 4) rows (C3: 1 M slots -> the first 18 %
      // of the rows); those tiles' entries then carry their exact rows into the aggregate and
      // the first-row pass only re-reads the tiles of slots first seen later (option
      // part_first: 1 none, 2 every tile)
      L.rit_tiles = 0;
      if (pk) {
        const double S = (double)std::max<uint64_t>(pl.nslots, 2);
        const double rows = std::min<double>((double)N, S * (std::log(S) + 4.0));
        L.rit_tiles = c->opt[kOptPartFirst] == 1 ? 0
                      : c->opt[kOptPartFirst] == 2 ? L.ntiles
                                                   : std::min<int64_t>(L.ntiles, (int64_t)std::ceil(rows / (double)tr));
      }
      const size_t rbytes = pk ? (((size_t)std::max<int64_t>(L.rit_tiles, 1) * (size_t)tr * 2) + 255) & ~size_t(255) : 0;
      // packed: first tags | tile marks + marked count [ntiles + 64] u32 | marked list [ntiles] u32 | rit
      const size_t kbytes = pk ? (((size_t)L.ntiles + 64) * 4 + 255) & ~size_t(255) : 0;
      const size_t lbytes = pk ? ((size_t)L.ntiles * 4 + 255) & ~size_t(255) : 0;
      unsigned char* eb = (unsigned char*)c->bitmap.ensure(vbytes + mbytes + pbytes + tbytes + kbytes + lbytes + rbytes + 256);
      L.vals = (unsigned long long*)eb;
      L.meta = (uint32_t*)(eb + vbytes);
      L.partial = eb + vbytes + mbytes;
      if (pk) {
        L.first_tag = eb + vbytes + mbytes + pbytes;
        L.tile_mark = (uint32_t*)(L.first_tag + tbytes);
        L.nmarked = L.tile_mark + L.ntiles;
        L.marked = (uint32_t*)(L.first_tag + tbytes + kbytes);
        L.rit = (uint16_t*)(L.first_tag + tbytes + kbytes + lbytes);
      }
      hipFunction_t fs = nullptr, ff = nullptr;
      if (c->opt[kOptJit] && N >= c->jit_min_rows()) {
        std::string extra = "#define BQ_PART_K " + std::to_string(L.k) + "\n#define BQ_PART_NARROW " +
                            std::to_string(L.narrow) + "\n#define BQ_PART_PACK " + std::to_string(L.pack) + "\n";
        // packed entries: tiles of row loads in flight per scatter workgroup (option part_ring)
        if (pk && c->opt[kOptPartRing] > 1) extra += "#define BQ_PART_RING " + std::to_string(c->opt[kOptPartRing]) + "\n";
        if (L.narrow) {  // the summed columns' code kinds (partition.h part_kind)
          extra += "#define BQ_PART_ENC ";
          for (int q = 0; q < kMaxSums; ++q) extra += std::to_string(q < nsum ? L.enc_kind[q] : 0) + (q + 1 < kMaxSums ? "," : "\n");
        }
        fs = jit_function_for("bq_jit_part_scatter", pl.p, extra, c->opt[kOptJitAsync] != 0);
        if (pk) ff = jit_function_for("bq_jit_part_first_rows", pl.p, extra, c->opt[kOptJitAsync] != 0);
        c->last.specialized = fs ? 1 : 0;
      }
      check_launch(c, "partitioned scatter", part_scatter_lds(L.nparts, L.threads, nsum, L.k, nw, pk), L.blocks, L.threads);
      check_launch(c, "partitioned aggregate", part_agg_lds_launch(L.wbits, nsum, pk, L.win, L.fx),
                   (int64_t)L.nparts * L.splits, 1024);
      launch_partitioned(pl.p, sa, L, st, fs, ff);
    } else {
      launch_scan_global(sp, sa, scan_blocks(c, N, 8), st);
    }
    HIPCHECK(hipGetLastError());
    // fixed-point sums to float64 (the partitioned path's combine rounds them itself)
    if (fx1 && pl.mode != kPartitioned) {
      FxShifts sh{};
      for (int q = 0; q < nsum; ++q) sh.shift[q] = pl.p.sum_fx_shift[q], sh.emax[q] = pl.p.fx_emax[q];
      launch_fx_finalize(sa.acc, sa.fx, nsum, pl.fx_states, sh, S, st);
      HIPCHECK(hipGetLastError());
    }
    if (c->timing) HIPCHECK(hipEventRecord(c->ev[2], st));
    if (pl.p.hash) {
      unsigned int hc[2];
      HIPCHECK(hipMemcpyAsync(hc, sa.hash_fill, 8, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      if (hc[1]) throw TableOverflow{false, S};  // run_groupby_grow re-runs with a bigger table
    }
  }

  // ---- std: centered second moments
  if (nsum2) {
    // means per slot, on device: centers[i][s] = acc[v][s] / cnt[s] for the i-th std column v
    double* centers = (double*)c->misc.ensure((size_t)nsum2 * S * 8 + 64);
    StdCenters sc{};
    sc.n = nsum2;
    if (nsum2 > kMaxSums) fail(BQG_E_UNSUPPORTED, "more than %d std columns", kMaxSums);
    for (int i = 0; i < nsum2; ++i) {
      const int v = pl.std_cols[i];
      const int dt = t->cols[pl.tcol[v]].dtype;
      sc.state[i] = v;
      // the pass-1 accumulator: int64 codes (atomic modes, e.sum_dec), float64 bits (float
      // columns, float64 sum states of integer columns, the partitioned path's finished
      // codes) or an integer sum
      sc.conv[i] = e.sum_dec[v] != 0.0 ? 3 : pl.p.sum_is_float[v] ? 0 : dt == BQG_U64 ? 2 : 1;
      sc.dec[i] = e.sum_dec[v];
    }
    launch_std_centers(sa.cnt, sa.acc, sc, S, centers, st);
    HIPCHECK(hipGetLastError());
    Plan p2 = pl;
    // sum states of pass 2: the std columns, centered, in std order (they are the first
    // nsum2 scan columns after re-ordering)
    std::vector<int> order;
    for (int v : pl.std_cols) order.push_back(v);
    for (int i = 0; i < pl.p.ncols; ++i)
      if (std::find(order.begin(), order.end(), i) == order.end()) order.push_back(i);
    ScanParams& q2 = p2.p;
    for (int i = 0; i < pl.p.ncols; ++i) q2.cols[i] = pl.p.cols[order[i]];
    auto remap = [&](int oldc) { return (int)(std::find(order.begin(), order.end(), oldc) - order.begin()); };
    for (int i = 0; i < q2.nterms; ++i) q2.terms[i].col = remap(pl.p.terms[i].col);
    for (int k = 0; k < q2.nkeys; ++k) q2.keys[k].col = remap(pl.p.keys[k].col);
    if (q2.mask_col >= 0) q2.mask_col = remap(pl.p.mask_col);
    q2.nsum = nsum2;
    for (int i = 0; i < kMaxSums; ++i) q2.fx_emax[i] = nullptr;  // (pass 2: column-wide shifts)
    for (int i = 0; i < nsum2; ++i) {
      q2.sum_is_float[i] = 1;
      q2.sum_conv[i] = pl.p.sum_conv[pl.std_cols[i]];
      q2.sum_centered[i] = 1;
      // atomic modes: the centred squares as fixed-point limbs (bit-reproducible)
      q2.sum_enc[i] = fx2 && ((pl.fx2_states >> i) & 1) ? 3 : 0;
      q2.sum_fx_shift[i] = pl.fx2_shift[i];
      q2.centers[i] = centers + (size_t)i * S;
    }
    SlotArrays sa2 = sa;
    sa2.acc = sa.acc2;
    sa2.fx = fx2 ? (unsigned long long*)(sbase + o_fx2) : nullptr;
    // pass 2 recomputes cnt/fst identically into scratch copies
    unsigned char* b2 = (unsigned char*)c->cdbuf.ensure(S * 12 + 512);
    sa2.cnt = (unsigned long long*)b2;
    sa2.fst = (uint32_t*)(b2 + ((S * 8 + 255) & ~size_t(255)));
    if (pl.mode == kPrivate) {
      const size_t lds = (size_t)S * kBlock * (8 + 8 * (size_t)nsum2);
      int per_cu = (int)std::min<size_t>(8, c->max_lds / std::max<size_t>(lds, 1));
      PrivateLaunch L{};
      L.blocks = scan_blocks(c, N, std::max(per_cu, 1));
      L.lds_bytes = lds;
      L.partials = (unsigned long long*)c->partials.ensure((size_t)(2 + nsum2) * L.blocks * S * 8);
      FinishParams F{};
      F.nslots = (int)S;
      F.blocks = L.blocks;
      F.nsum = nsum2;
      for (int i = 0; i < kMaxSums; ++i) F.sum_is_float[i] = q2.sum_is_float[i];
      F.partials = L.partials;
      F.out_hdr = (unsigned long long*)c->hdr.ensure(64);
      F.totals = (unsigned long long*)c->counter.ensure((size_t)(2 + kMaxSums) * kMaxPrivateSlots * 8);
      F.done = (unsigned int*)c->done.p;
      F.emit_inline = 0;
      launch_scan_private(q2, L, st);
      launch_private_finish(F, sa2, e, st);
    } else {
      sa2.keys = nullptr;  // keep the hash table built by pass 1: init only the accumulators
      launch_init_slots(sa2, nsum2, S, st);
      sa2.keys = sa.keys;
      if (pl.mode == kShared) {
        const size_t lds = shared_lds(S, nsum2, fx2);
        int per_cu = (int)std::min<size_t>(8, c->max_lds / std::max<size_t>(lds, 1));
        check_launch(c, "shared scan (std pass)", lds, scan_blocks(c, N, std::max(per_cu, 1)));
        launch_scan_shared(q2, sa2, scan_blocks(c, N, std::max(per_cu, 1)), lds, st);
      } else {
        launch_scan_global(q2, sa2, scan_blocks(c, N, 8), st);
      }
      if (fx2) {
        FxShifts sh{};
        for (int i = 0; i < nsum2; ++i) sh.shift[i] = q2.sum_fx_shift[i];
        launch_fx_finalize(sa2.acc, sa2.fx, nsum2, pl.fx2_states, sh, S, st);
      }
    }
    HIPCHECK(hipGetLastError());
  }

  // ---- nonfinite pass: mean / std of float columns holding NaN or infinities
  if (pl.nf_states) {
    int nst = 0;
    for (int q = 0; q < nsum; ++q) nst += (pl.nf_states >> q) & 1;
    const size_t words = (size_t)S * (1 + 2 * (size_t)nst);
    uint32_t* nb = (uint32_t*)c->nfbuf.ensure(words * 4 + 256);
    HIPCHECK(hipMemsetAsync(nb, 0, words * 4, st));
    NonfiniteLaunch nf{};
    nf.states = pl.nf_states;
    nf.lds = S <= kNonfiniteLdsSlots ? 1 : 0;
    nf.last_row = nb;
    e.nf_last = nb;
    int k = 0;
    for (int q = 0; q < nsum; ++q) {
      if (!((pl.nf_states >> q) & 1)) continue;
      nf.cnt[q] = nb + (size_t)S * (1 + 2 * k);
      nf.row[q] = nf.cnt[q] + S;
      e.nf_cnt[q] = nf.cnt[q];
      e.nf_row[q] = nf.row[q];
      e.nf_col[q] = pl.p.cols[q];
      ++k;
    }
    launch_nonfinite(pl.p, sa, nf, scan_blocks(c, N, 8), st);
    HIPCHECK(hipGetLastError());
  }

  // ---- count_distinct
  DistinctLaunch fused_cd{};
  std::vector<DevBuf> tmp_bufs;  // per-op scratch
  unsigned long long* cd_out = nullptr;
  if (ncd) cd_out = (unsigned long long*)c->cdbuf.ensure((size_t)ncd * S * 8 + (nsum2 ? 0 : 0));
  // note: cdbuf is reused by std pass 2 above only before this point
  // the fused distinct pass's zeroed buffers (its count_distinct outputs and pair bitmap) are
  // cleared by one kernel before it: two fills and their host calls cost ~10 us of a C4 query
  ZeroRanges zr{};
  auto zero_async = [&](void* p, size_t bytes) {
    if (fused && zr.n < kZeroRanges && bytes % 4 == 0) {
      zr.p[zr.n] = (unsigned int*)p;
      zr.words[zr.n++] = bytes / 4;
    } else {
      HIPCHECK(hipMemsetAsync(p, 0, bytes, st));
    }
  };
  if (ncd) {
    zero_async(cd_out, (size_t)ncd * S * 8);
    int i = 0;
    for (int a = 0; a < q->n_aggs; ++a) {
      if (q->aggs[a].op != BQG_COUNT_DISTINCT) continue;
      const int tc = q->aggs[a].col;
      Column& col = t->cols[tc];
      compute_stats(t, tc);
      Plan pc = pl;
      DistinctLaunch d{};
      d.vcol = scan_col(pc, tc);
      pc.p.ncols = (int)pc.tcol.size();
      pc.p.cols[d.vcol] = DevCol{col.dev, col.dtype, dtype_lg(col.dtype)};
      d.out = cd_out + (size_t)i * S;
      // pair identity: (slot, value code) packed into one 64-bit set key when the pair space
      // allows (a bitmap when it is small), else slot << 32 | representative row (pair_rows)
      const bool isf = dtype_is_float(col.dtype);
      unsigned __int128 pairs;
      if (isf) {
        d.vmin = 0;
        d.vrange = 1;  // S == 1: key = canonical value bits
        d.pair_rows = S != 1;
        pairs = (unsigned __int128)1 << 64;
      } else {
        d.vmin = col.stats.empty ? 0 : col.stats.imin;
        d.vrange = col.stats.empty ? 1 : (uint64_t)col.stats.imax - (uint64_t)col.stats.imin + 1;
        pairs = (unsigned __int128)S * (d.vrange ? d.vrange : ((unsigned __int128)1 << 64));
        // a full-range 64-bit column (vrange wraps to 0) or S x range >= 2^63
        if (pairs >= ((unsigned __int128)1 << 63)) {
          d.pair_rows = 1;
          d.vmin = 0;
        }
      }
      if (!isf && pairs <= ((unsigned __int128)1 << 30)) {
        const size_t words = (size_t)((pairs + 31) / 32);
        d.bitmap = (unsigned int*)c->bitmap.ensure(words * 4);
        zero_async(d.bitmap, words * 4);
        d.lds_bitmap_words = words * 4 <= 32 * 1024 ? (int)words : 0;
      } else {
        if (d.pair_rows && (S >= 0xFFFFFFFFull || N > (int64_t)0xFFFFFFFFll))
          fail(BQG_E_UNSUPPORTED, "count_distinct pair set: slot or row index beyond 32 bits");
        uint64_t cap = 1024;
        uint64_t est = std::min<uint64_t>((uint64_t)N, 1ull << 27);
        if (c->opt[kOptDistinctSlots]) est = (uint64_t)c->opt[kOptDistinctSlots] / 2;
        while (cap < 2 * est) cap <<= 1;
        if (c->distinct_grow > cap) cap = c->distinct_grow;
        unsigned char* sb = (unsigned char*)c->bitmap.ensure(cap * 8 + 256);
        d.set = (unsigned long long*)sb;
        d.set_mask = cap - 1;
        d.set_fill = (unsigned int*)(sb + cap * 8);
        d.overflow = d.set_fill + 1;
        HIPCHECK(hipMemsetAsync(d.set, 0xFF, cap * 8, st));
        HIPCHECK(hipMemsetAsync(d.set_fill, 0, 8, st));
      }
      if (fused) {
        fused_cd = d;  // folded into k_scd_fused (bitmap mode: checked above)
        e.cd[i] = d.out;
        ++i;
        continue;
      }
      launch_count_distinct(pc.p, sa, d, scan_blocks(c, N, 8), st);
      HIPCHECK(hipGetLastError());
      if (d.set) {
        unsigned int hc[2];
        HIPCHECK(hipMemcpyAsync(hc, d.set_fill, 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        if (hc[1]) throw TableOverflow{true, d.set_mask + 1};
      }
      e.cd[i] = d.out;
      ++i;
    }
  }

  if (zr.n) {
    launch_zero_ranges(zr, st);
    HIPCHECK(hipGetLastError());
  }

  // ---- sorted_count_distinct
  if (nscd) {
    unsigned long long* so = (unsigned long long*)c->scdbuf.ensure((size_t)nscd * S * 16 + 256);
    int i = 0;
    for (int a = 0; a < q->n_aggs; ++a) {
      if (q->aggs[a].op != BQG_SORTED_COUNT_DISTINCT) continue;
      const int tc = q->aggs[a].col;
      Column& col = t->cols[tc];
      Plan pc = pl;
      ScdLaunch d{};
      d.vcol = scan_col(pc, tc);
      pc.p.ncols = (int)pc.tcol.size();
      pc.p.cols[d.vcol] = DevCol{col.dev, col.dtype, dtype_lg(col.dtype)};
      if (fused && fused_cd.bitmap) {
        // the count_distinct column joins this pass's column set
        for (int b2 = 0; b2 < q->n_aggs; ++b2) {
          if (q->aggs[b2].op != BQG_COUNT_DISTINCT) continue;
          const int cc = q->aggs[b2].col;
          fused_cd.vcol = scan_col(pc, cc);
          pc.p.ncols = (int)pc.tcol.size();
          pc.p.cols[fused_cd.vcol] = DevCol{t->cols[cc].dev, t->cols[cc].dtype, dtype_lg(t->cols[cc].dtype)};
        }
      }
      const uint64_t budget = 1ull << 30;
      uint64_t waves = (uint64_t)c->cu * 16;
      const uint64_t grain = fused ? 256 : 64;  // fused: 256-row groups, 4 rows per lane
      if (fused) {
        d.fused = 1;
        // compact 32-bit value codes for integer value columns spanning < 2^32
        compute_stats(t, tc);
        if (!dtype_is_float(col.dtype) && c->opt[kOptScdCompact]) {
          const uint64_t vr = col.stats.empty ? 1 : (uint64_t)col.stats.imax - (uint64_t)col.stats.imin + 1;
          if (vr != 0 && vr <= 0xFFFFFFFFull) {
            d.compact = 1;
            d.vmin = col.stats.empty ? 0 : col.stats.imin;
            // value codes below 2^16 (compact chunks are below 2^16 rows): first value and
            // first row share one LDS word
            d.pack16 = vr <= 0x10000ull && c->opt[kOptScdPack16] ? 1 : 0;
          }
        }
        d.wave_lds = scd_fused_wave_lds(S, d.compact != 0, d.pack16 != 0);
        d.cd = fused_cd;
        const size_t blk_lds = (kBlock / 64) * d.wave_lds + (size_t)fused_cd.lds_bitmap_words * 4;
        if (blk_lds > kScdFusedMaxLds) d.cd.lds_bitmap_words = 0;  // no LDS pre-filter
        const size_t lds = (kBlock / 64) * d.wave_lds + (size_t)d.cd.lds_bitmap_words * 4;
        const uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>(8, c->max_lds / lds));
        waves = (uint64_t)c->cu * per_cu * (kBlock / 64);
      }
      const uint64_t needg = ((uint64_t)N + grain - 1) / grain;
      if (waves > needg) waves = needg;
      while (waves > 64 && waves * S * 28 > budget) waves /= 2;
      if (waves < 1) waves = 1;
      if (fused && d.compact) {
        // 16-bit per-slot row counts: at most kScdCompactMaxRows rows per wave chunk
        const uint64_t need = ((uint64_t)N + kScdCompactMaxRows - 1) / kScdCompactMaxRows;
        if (need * S * 28 > budget) {
          d.compact = 0;  // that many chunk states do not fit: the wide pass (32-bit counts)
          d.pack16 = 0;
          d.wave_lds = scd_fused_wave_lds(S, false);
        } else if (waves < need) {
          waves = need;
        }
      }
      // clustered keys (runs of 512 rows and more on average in the first key column) and no
      // row filter: the RUNS loop (256-row steps)
      if (fused && d.compact && c->opt[kOptScdRuns] && pc.p.nterms == 0 && pc.p.mask_col < 0 && q->n_keys > 0 &&
          column_runs(t, q->key_cols[0]) * 512 <= N)
        d.runs = 1;
      d.waves = (int)waves;
      d.chunk_rows = (((int64_t)((N + waves - 1) / waves)) + grain - 1) / grain * grain;
      d.lds_state = (S * 24 * (kBlock / 64) <= 64 * 1024) ? 1 : 0;
      d.slot_bits = 0;
      while (d.slot_bits < 63 && (S - 1) >> d.slot_bits) ++d.slot_bits;
      unsigned char* b = (unsigned char*)c->prefix.ensure(waves * S * 28 + 1024);
      d.st_first = (unsigned long long*)b;
      d.st_last = d.st_first + waves * S;
      d.st_first_row = (uint32_t*)(d.st_last + waves * S);
      d.st_changes = d.st_first_row + waves * S;
      d.st_count = fused ? d.st_changes + waves * S : nullptr;
      if (!d.lds_state && !fused) {
        HIPCHECK(hipMemsetAsync(d.st_first_row, 0xFF, waves * S * 4, st));
        HIPCHECK(hipMemsetAsync(d.st_changes, 0, waves * S * 4, st));
      }
      if (fused) {
        d.slot_cnt = sa.cnt;
        d.slot_fst = sa.fst;
      }
      d.out_changes = so + (size_t)i * S * 2;
      d.out_first = d.out_changes + S;
      if (fused && d.runs && c->opt[kOptCompact]) {
        // the RUNS loop (clustered keys, 16-byte loads of 4 rows per lane) reads the integer
        // columns' compact copies (narrow offsets; the decode restores canonical values, so
        // keys, value runs and distinct pairs are unchanged): C4 sorted 0.284 -> 0.145 ms.  The
        // random-order loop loads one row per lane -- an 8-byte word per row of a narrow column
        // -- and is compute-bound: its copies measured slower (0.475 -> 0.505 ms), so it reads
        // the columns as stored
        for (int ci = 0; ci < pc.p.ncols; ++ci) {
          const int tc2 = pc.tcol[ci];
          Column& k2 = t->cols[tc2];
          if (!ensure_shadow(c, t, tc2, 1)) continue;
          pc.p.cols[ci] = DevCol{k2.shadow.dev, k2.shadow.dtype, dtype_lg(k2.shadow.dtype), 1, 0, k2.shadow.off};
          if (!pl.dummy_col) pl.read_bytes -= ((int64_t)dtype_size(k2.dtype) - (int64_t)dtype_size(k2.shadow.dtype)) * N;
        }
      }
      hipFunction_t sfn = nullptr;
      if (fused && c->opt[kOptJit] && N >= c->jit_min_rows()) {
        const int cd_mode = d.cd.bitmap == nullptr ? 0 : (d.cd.lds_bitmap_words > 0 ? 1 : 2);
        // the value columns as constants (the same choice as the generic body's column loop)
        const int nc = pc.p.ncols;
        const int vc = d.vcol >= 0 && d.vcol < nc ? d.vcol : 0;
        const int cc = d.cd.vcol >= 0 && d.cd.vcol < nc ? d.cd.vcol : 0;
        const std::string extra = "#define BQ_SCD_CD " + std::to_string(cd_mode) + "\n#define BQ_SCD_VC " +
                                  std::to_string(vc) + "\n#define BQ_SCD_CC " + std::to_string(cc) +
                                  "\n#define BQ_SCD_P16 " + std::to_string(d.pack16) + "\n";
        sfn = jit_function_for(d.runs ? "bq_jit_scd_runs32" : d.compact ? "bq_jit_scd_fused32" : "bq_jit_scd_fused",
                               pc.p, extra, c->opt[kOptJitAsync] != 0);
        c->last.specialized = sfn ? 1 : 0;
      }
      if (fused && c->timing) HIPCHECK(hipEventRecord(c->ev[1], st));
      // timing brackets the pass itself (the chunk combine follows it)
      launch_scd(pc.p, sa, d, st, sfn, fused && c->timing ? c->ev[2] : nullptr);
      HIPCHECK(hipGetLastError());
      e.scd_changes[i] = d.out_changes;
      e.scd_first[i] = d.out_first;
      ++i;
    }
  }

  // ---- small slot spaces: compaction + ordering + emit in one workgroup; the header and the
  // columns (capacity S) come back in one copy, with no host round trip in between
  if (S <= kSmallEmitSlots && c->opt[kOptSmallEmit]) {
    std::vector<size_t> offs;
    size_t obytes = 256;  // header: groups, passing rows
    for (int j = 0; j < e.ncols; ++j) {
      offs.push_back(obytes);
      obytes += ((size_t)S * dtype_size(out_dt[j]) + 255) & ~size_t(255);
    }
    // host result: written straight into a pooled pinned block (device-mapped, no copy)
    BlockGuard blk;
    if (!c->dev_target) blk.reset(c->pool, c->pool_get(obytes + 64));
    unsigned char* ob = c->dev_target ? (unsigned char*)c->outcols.ensure(obytes + 256) : (unsigned char*)blk.b.dev;
    for (int j = 0; j < e.ncols; ++j) e.cols[j].out = ob + offs[j];
    launch_emit_small(e, sa, (uint32_t)S, nsum, (unsigned long long*)ob, st);
    HIPCHECK(hipGetLastError());
    const unsigned long long* hh;
    if (c->dev_target) {
      hh = (const unsigned long long*)c->hhdr.ensure(64);
      HIPCHECK(hipMemcpyAsync((void*)hh, ob, 16, hipMemcpyDeviceToHost, st));
    } else {
      hh = (const unsigned long long*)blk.b.p;
    }
    if (c->timing == 1) HIPCHECK(hipEventRecord(c->ev[3], st));
    HIPCHECK(hipStreamSynchronize(st));
    const int64_t G = (int64_t)hh[0];
    const int filtered = pl.has_filter && (int64_t)hh[1] < N;
    finish_query(c, pl, (int64_t)G, e.ncols);
    if (G == 0) {
      *out = empty_result(out_dt, filtered);  // the guard returns the block
    } else if (c->dev_target) {
      std::vector<const void*> src;
      for (int j = 0; j < e.ncols; ++j) src.push_back(e.cols[j].out);
      table_from_device(c, out_dt, src, G);
    } else {
      *out = block_result(c, blk.release(), G, filtered, out_dt, offs);
    }
    return;
  }

  // ---- large slot spaces: no compaction, no host round trip before the emit (the group count
  // is read from page-locked memory while the emit runs)
  if (S > kSmallEmitSlots && c->opt[kOptSlotEmit]) {
    const uint64_t nwords = ((uint64_t)N + 31) / 32;
    const uint64_t nblocks = (nwords + 1023) / 1024;
    // bitmap [nwords] u32 | hdr (256 B) | word pairs [nwords] u64 | block prefixes [nblocks] u32
    const size_t bm_bytes = (nwords * 4 + 255) & ~size_t(255);
    unsigned char* pb = (unsigned char*)c->prefix.ensure(bm_bytes + 256 + nwords * 8 + nblocks * 4 + 1024 + 8192);
    unsigned int* bitmap = (unsigned int*)pb;
    unsigned long long* hdev = (unsigned long long*)(pb + bm_bytes);
    unsigned long long* wpair = (unsigned long long*)(pb + bm_bytes + 256);
    unsigned int* bprefix = (unsigned int*)(wpair + nwords);
    // the marking pass's per-workgroup passing rows (up to 1024 workgroups)
    unsigned long long* rows_part = (unsigned long long*)(pb + ((bm_bytes + 256 + nwords * 8 + nblocks * 4 + 255) & ~size_t(255)));
    unsigned long long* hh = (unsigned long long*)c->hhdr.ensure(64);
    void* hh_dev = nullptr;
    HIPCHECK(hipHostGetDevicePointer(&hh_dev, hh, 0));
    // output columns at capacity S, laid out by the group count on the device (+ with
    // slot_emit 2 the group records, S x ncols words)
    size_t ocap = 0;
    for (int j = 0; j < e.ncols; ++j) ocap += ((size_t)S * dtype_size(out_dt[j]) + 255) & ~size_t(255);
    const bool aos = c->opt[kOptSlotEmit] == 2;
    unsigned char* ob = (unsigned char*)c->outcols.ensure(ocap + 256 + (aos ? (size_t)S * e.ncols * 8 : 0));
    // first rows marked in the row map (one byte per row, the query's epoch) up to 2^30 rows,
    // else by bitmap atomics
    unsigned char* row_map = nullptr;
    unsigned char epoch = 0;
    if ((uint64_t)N <= (1ull << 30) && c->opt[kOptSlotEmit] != 3) {
      const size_t need = nwords * 32 + 256;
      const void* before = c->rowmap.p;
      const size_t cap_before = c->rowmap.cap;
      row_map = (unsigned char*)c->rowmap.ensure(need);
      if (row_map != before || c->rowmap.cap != cap_before || c->rowmap_epoch == 255) {
        HIPCHECK(hipMemsetAsync(row_map, 0, c->rowmap.cap, st));
        c->rowmap_epoch = 0;
      }
      epoch = ++c->rowmap_epoch;
    }
    launch_slot_emit(e, sa, S, N, bitmap, row_map, epoch, wpair, bprefix, rows_part, hdev, (unsigned long long*)hh_dev,
                     c->ev_groups, ob, aos ? (unsigned long long*)(ob + ocap + 256) : nullptr, st);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventSynchronize(c->ev_groups));
    const uint64_t G = hh[0];
    const unsigned long long total = hh[1];
    const int filtered = pl.has_filter && (int64_t)total < N;
    std::vector<size_t> offs;
    size_t obytes = 0;
    for (int j = 0; j < e.ncols; ++j) {
      offs.push_back(obytes);
      obytes += ((size_t)G * dtype_size(out_dt[j]) + 255) & ~size_t(255);
    }
    if (G == 0) {
      HIPCHECK(hipStreamSynchronize(st));
      finish_query(c, pl, 0, e.ncols);
      *out = empty_result(out_dt, filtered);
      return;
    }
    if (c->dev_target) {
      if (c->timing == 1) HIPCHECK(hipEventRecord(c->ev[3], st));
      std::vector<const void*> src;
      for (int j = 0; j < e.ncols; ++j) src.push_back(ob + offs[j]);
      table_from_device(c, out_dt, src, (int64_t)G);
      finish_query(c, pl, (int64_t)G, e.ncols);
      return;
    }
    BlockGuard blk;
    blk.reset(c->pool, c->pool_get(obytes + 64));
    if (c->timing == 1) {
      HIPCHECK(hipEventRecord(c->ev_copy, st));
      c->copy_timed = true;
    }
    HIPCHECK(hipMemcpyAsync(blk.b.p, ob, obytes, hipMemcpyDeviceToHost, st));
    if (c->timing == 1) HIPCHECK(hipEventRecord(c->ev[3], st));
    HIPCHECK(hipStreamSynchronize(st));
    bqg_result* r = block_result(c, blk.release(), (int64_t)G, filtered, out_dt, offs);
    finish_query(c, pl, (int64_t)G, e.ncols);
    *out = r;
    return;
  }

  // ---- generic emit
  const uint64_t cblocks = (S + 4095) / 4096 + 1;
  unsigned char* lb = (unsigned char*)c->lists.ensure(S * 8 + (2 * cblocks + 4096) * 8 + 256);
  uint32_t* list_fst = (uint32_t*)lb;
  uint32_t* list_slot = list_fst + S;
  uint32_t* compact_scratch = list_slot + S;
  unsigned char* hb = (unsigned char*)c->hdr.ensure(64);
  unsigned int* gcount = (unsigned int*)hb;
  unsigned long long* gtotal = (unsigned long long*)(hb + 8);
  HIPCHECK(hipMemsetAsync(hb, 0, 16, st));
  launch_compact(sa, S, list_fst, list_slot, gcount, gtotal, compact_scratch, st);
  HIPCHECK(hipGetLastError());
  unsigned char* hh = (unsigned char*)c->hhdr.ensure(64);
  HIPCHECK(hipMemcpyAsync(hh, hb, 16, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  const unsigned int G = *(unsigned int*)hh;
  const unsigned long long total = *(unsigned long long*)(hh + 8);
  if (G == 0) {
    *out = empty_result(out_dt, pl.has_filter && (int64_t)total < N);
    return;
  }
  uint32_t* order = nullptr;
  if (G <= 8192) {
    order = (uint32_t*)c->misc.ensure((size_t)G * 4 + 256);
    launch_sort_small(list_fst, list_slot, G, order, st);
  }
  HIPCHECK(hipGetLastError());
  size_t obytes = 0;
  for (int j = 0; j < e.ncols; ++j) obytes += ((size_t)G * dtype_size(out_dt[j]) + 255) & ~size_t(255);
  unsigned char* ob = (unsigned char*)c->outcols.ensure(obytes + 256);
  {
    size_t o = 0;
    for (int j = 0; j < e.ncols; ++j) {
      e.cols[j].out = ob + o;
      o += ((size_t)G * dtype_size(out_dt[j]) + 255) & ~size_t(255);
    }
  }
  if (order) {
    launch_emit(e, sa, order, G, nsum, S, st);
  } else {
    // more groups: rank by a bitmap of first rows, emit each group at its rank in one pass
    const uint64_t nwords = ((uint64_t)N + 31) / 32;
    const uint64_t nblocks = (nwords + 1023) / 1024;
    unsigned char* pb = (unsigned char*)c->prefix.ensure(nwords * 8 + nblocks * 4 + 1024);
    unsigned int* bitmap = (unsigned int*)pb;
    unsigned int* wprefix = bitmap + nwords;
    unsigned int* bprefix = wprefix + nwords;
    launch_rank_emit_bitmap(e, sa, list_fst, list_slot, G, nsum, S, N, bitmap, wprefix, bprefix, st);
  }
  HIPCHECK(hipGetLastError());
  if (c->dev_target) {
    if (c->timing == 1) HIPCHECK(hipEventRecord(c->ev[3], st));
    std::vector<const void*> src;
    for (int j = 0; j < e.ncols; ++j) src.push_back(e.cols[j].out);
    table_from_device(c, out_dt, src, (int64_t)G);
    finish_query(c, pl, (int64_t)G, e.ncols);
    return;
  }
  BlockGuard blk;
  blk.reset(c->pool, c->pool_get(obytes + 64));
  if (c->timing == 1) {
    HIPCHECK(hipEventRecord(c->ev_copy, st));
    c->copy_timed = true;
  }
  HIPCHECK(hipMemcpyAsync(blk.b.p, ob, obytes, hipMemcpyDeviceToHost, st));
  if (c->timing == 1) HIPCHECK(hipEventRecord(c->ev[3], st));
  HIPCHECK(hipStreamSynchronize(st));
  std::vector<size_t> offs;
  {
    size_t o = 0;
    for (int j = 0; j < e.ncols; ++j) {
      offs.push_back(o);
      o += ((size_t)G * dtype_size(out_dt[j]) + 255) & ~size_t(255);
    }
  }
  bqg_result* r = block_result(c, blk.release(), G, pl.has_filter && (int64_t)total < N, out_dt, offs);
  finish_query(c, pl, (int64_t)G, e.ncols);
  *out = r;
}

// run_groupby, growing an over-full hash table or count_distinct set and re-running the query
// (bquery's khash factorize has no cardinality ceiling, worker.py:313).  Slot ids stay below
// 2^31 (32-bit slot lists and first rows on device).
void run_groupby_grow(bqg_ctx* c, bqg_table* t, const bqg_query* q, bqg_result** out) {
  struct Reset {
    bqg_ctx* c;
    ~Reset() { c->hash_grow = c->distinct_grow = 0; }
  } reset{c};
  c->hash_grow = c->distinct_grow = 0;
  for (;;) {
    try {
      run_groupby(c, t, q, out);
      return;
    } catch (const TableOverflow& o) {
      if (o.slots >= (1ull << 31))
        fail(BQG_E_OOM, "%s would need more than 2^31 slots", o.distinct ? "count_distinct set" : "group hash table");
      (o.distinct ? c->distinct_grow : c->hash_grow) = o.slots * 2;
      ++c->last_regrows;
    }
  }
}

}  // namespace

int bqg_internal_device(bqg_ctx* c) { return c->device; }
hipStream_t bqg_internal_stream(bqg_ctx* c) { return c->stream; }
bool bqg_internal_timing(bqg_ctx* c) { return c->timing != 0; }
void bqg_internal_set_error(bqg_ctx* c, const std::string& msg) {
  if (c) c->err = msg;
  g_err = msg;
}
int bqg_internal_table_set_rows(bqg_table* t, int64_t n) {
  if (!t || n < 0 || n > t->nrows) return BQG_E_INVALID;
  t->nrows = n;
  for (Column& col : t->cols) col.stats.valid = false;
  return BQG_OK;
}
int bqg_internal_host_result(bqg_ctx* c, int64_t n, const std::vector<int32_t>& dts, std::vector<void*>& cols,
                             bqg_result** out) {
  *out = nullptr;
  try {
    std::vector<size_t> offs;
    size_t off = 0;
    for (int32_t dt : dts) {
      offs.push_back(off);
      off += ((size_t)n * dtype_size(dt) + 255) & ~size_t(255);
    }
    BlockGuard blk;
    blk.reset(c->pool, c->pool_get(off + 256));
    std::vector<int> d(dts.begin(), dts.end());
    bqg_result* r = block_result(c, blk.b, n, 0, d, offs);
    blk.release();
    cols.clear();
    for (size_t j = 0; j < dts.size(); ++j) cols.push_back((unsigned char*)r->block.p + offs[j]);
    *out = r;
    return BQG_OK;
  } catch (const ApiError& e) {
    c->err = e.msg;
    return e.code;
  } catch (const std::bad_alloc&) {
    c->err = "host out of memory";
    return BQG_E_OOM;
  }
}

// ======================================================================================
// C ABI
// ======================================================================================
extern "C" {

int bqg_abi_version(void) { return BQG_ABI_VERSION; }

int bqg_jit_wait(bqg_ctx* ctx, double timeout_ms, int32_t* idle, int64_t* compiled, int64_t* failed) {
  return guard(ctx, [&] {
    const bool done = jit_wait(timeout_ms, compiled, failed);
    if (idle) *idle = done ? 1 : 0;
  });
}

int bqg_device_count(int* n) {
  return guard(nullptr, [&] {
    int k = 0;
    HIPCHECK(hipGetDeviceCount(&k));
    *n = k;
  });
}

// defaults, then the environment (read once per context, never on the query path)
static void load_options(bqg_ctx* c) {
  for (int i = 0; i < kNumOpts; ++i) c->opt[i] = kOptDefs[i].def;
  if (const char* e = getenv("BQGPU_JIT")) c->opt[kOptJit] = strcmp(e, "0") == 0 ? 0 : 1;
  if (const char* e = getenv("BQGPU_JIT_MIN_ROWS")) c->opt[kOptJitMinRows] = std::max<int64_t>(0, atoll(e));
  if (const char* e = getenv("BQGPU_OPTIONS")) {
    std::string all(e);
    size_t pos = 0;
    while (pos <= all.size()) {
      size_t end = all.find(',', pos);
      if (end == std::string::npos) end = all.size();
      const std::string item = all.substr(pos, end - pos);
      pos = end + 1;
      if (item.empty()) continue;
      const size_t eq = item.find('=');
      const std::string name = item.substr(0, eq);
      const int i = opt_index(name.c_str());
      char* tail = nullptr;
      const long long v = eq == std::string::npos ? 0 : strtoll(item.c_str() + eq + 1, &tail, 0);
      if (i < 0 || eq == std::string::npos || !tail || *tail || !opt_valid(i, v))
        fail(BQG_E_INVALID, "BQGPU_OPTIONS: bad item '%s'", item.c_str());
      c->opt[i] = v;
    }
  }
}

int bqg_set_option(bqg_ctx* c, const char* name, int64_t value) {
  return guard(c, [&] {
    if (!c) fail(BQG_E_INVALID, "null context");
    const int i = opt_index(name);
    if (i < 0) fail(BQG_E_INVALID, "unknown option '%s'", name ? name : "(null)");
    if (!opt_valid(i, value)) fail(BQG_E_INVALID, "option %s: value %lld out of range", name, (long long)value);
    c->opt[i] = value;
  });
}

int bqg_get_option(bqg_ctx* c, const char* name, int64_t* value) {
  return guard(c, [&] {
    if (!c || !value) fail(BQG_E_INVALID, "null argument");
    const int i = opt_index(name);
    if (i < 0) fail(BQG_E_INVALID, "unknown option '%s'", name ? name : "(null)");
    *value = c->opt[i];
  });
}

int bqg_reset_options(bqg_ctx* c) {
  return guard(c, [&] {
    if (!c) fail(BQG_E_INVALID, "null context");
    load_options(c);
  });
}

// Start-up work a worker's first query would otherwise pay (option warm, at context creation):
// the first launch from the library's code object loads it (~0.7 ms, measured: a cold C2
// query's generic scan 1.04 ms against 0.36 ms steady, profiles/r6b_cold_probe.json), each
// kernel's first launch resolves its symbol, and the private scan's partials / the pooled
// pinned result blocks are allocated on first use.  One small C2-shaped query -- 3 columns, a
// filter, sum / mean / count over 10 groups, 768 tiles so the partials reach their steady size
// on a 256-CU device -- does all of it once, and a C3- and a C4-shaped query launch the
// partition / large-emit and distinct kernels once; the table is freed before bqg_create returns.
static void warm_context(bqg_ctx* c) {
  const int64_t n = (int64_t)std::max(c->cu, 1) * 3 * 1024;
  const int32_t dts[4] = {BQG_I32, BQG_F64, BQG_I8, BQG_I32};
  std::vector<int32_t> k((size_t)n), k2((size_t)n);
  std::vector<double> v((size_t)n);
  std::vector<int8_t> f((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    k[(size_t)i] = (int32_t)(i % 10);
    v[(size_t)i] = (double)(i % 97) * 0.25;
    f[(size_t)i] = (int8_t)(i % 5);
    k2[(size_t)i] = (int32_t)(i % 100000);
  }
  bqg_table* t = nullptr;
  auto ok = [&](int rc) {
    if (rc != BQG_OK) fail(rc, "context warm-up query failed: %s", bqg_last_error(c));
  };
  ok(bqg_table_create(c, n, 4, dts, &t));
  std::unique_ptr<bqg_table, int (*)(bqg_table*)> own(t, bqg_table_destroy);
  ok(bqg_push_chunk(t, 0, k.data(), n, 0));
  ok(bqg_push_chunk(t, 1, v.data(), n, 0));
  ok(bqg_push_chunk(t, 2, f.data(), n, 0));
  ok(bqg_push_chunk(t, 3, k2.data(), n, 0));
  ok(bqg_table_sync(t));
  const int64_t two = 2;
  const bqg_term term{2, BQG_T_GE, 1, &two, nullptr};
  const int32_t key = 0;
  const bqg_agg aggs[3] = {{1, BQG_SUM}, {1, BQG_MEAN}, {1, BQG_COUNT}};
  const bqg_query q{1, &key, 1, &term, -1, 3, aggs};
  for (int64_t compact = 0; compact <= 1; ++compact) {  // the scan over the columns as stored, then over copies
    const int64_t saved = c->opt[kOptCompact];
    c->opt[kOptCompact] = compact ? saved : 0;
    bqg_result* r = nullptr;
    const int rc = bqg_groupby(c, t, &q, &r);
    c->opt[kOptCompact] = saved;
    ok(rc);
    bqg_result_free(r);
  }
  // best effort (a failure here only leaves those kernels cold): the partitioned path with its
  // large-result emit (C3's shape: two keys over 10^6 slots, 10^5 groups) and the fused
  // distinct pass (C4's aggregations)
  {
    const int32_t keys2[2] = {3, 0};
    const bqg_agg a3[2] = {{1, BQG_SUM}, {1, BQG_COUNT}};
    const bqg_query q3{2, keys2, 0, nullptr, -1, 2, a3};
    const bqg_agg a4[2] = {{2, BQG_COUNT_DISTINCT}, {2, BQG_SORTED_COUNT_DISTINCT}};
    const bqg_query q4{1, &key, 0, nullptr, -1, 2, a4};
    for (const bqg_query* qq : {&q3, &q4}) {
      bqg_result* r = nullptr;
      if (bqg_groupby(c, t, qq, &r) == BQG_OK) bqg_result_free(r);
    }
    c->err.clear();
  }
  own.reset();
  HIPCHECK(hipStreamSynchronize(c->stream));
  // the warm-up table's column blocks leave the context: no idle block of it may later stand in
  // for an allocation that the column budget (option mem_cap_mb) would refuse
  c->colpool.release();
  c->last = bqg_timing{};
}

int bqg_create(int device_ordinal, bqg_ctx** out) {
  bqg_ctx* c = nullptr;
  int rc = guard(nullptr, [&] {
    if (!out) fail(BQG_E_INVALID, "null output pointer");
    int n = 0;
    HIPCHECK(hipGetDeviceCount(&n));
    if (device_ordinal < 0 || device_ordinal >= n) fail(BQG_E_INVALID, "device %d not present (%d devices)", device_ordinal, n);
    HIPCHECK(hipSetDevice(device_ordinal));
    c = new bqg_ctx();
    c->device = device_ordinal;
    load_options(c);
    HIPCHECK(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
    c->stream = c->own;
    c->cu = device_cu_count();
    {
      int lds = 0;
      if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device_ordinal) == hipSuccess && lds > 0)
        c->max_lds = (size_t)lds;
    }
    for (int i = 0; i < 2; ++i) {
      HIPCHECK(hipHostMalloc(&c->stage[i], bqg_ctx::kStage, hipHostMallocDefault));
      HIPCHECK(hipEventCreateWithFlags(&c->stage_ev[i], hipEventDisableTiming));
    }
    // timing-only events: no system-scope fence (cache writeback) at each record
    for (int i = 0; i < 4; ++i) HIPCHECK(hipEventCreateWithFlags(&c->ev[i], hipEventDisableSystemFence));
    for (int i = 0; i < 2; ++i) HIPCHECK(hipEventCreateWithFlags(&c->ev_sh[i], hipEventDisableSystemFence));
    HIPCHECK(hipEventCreateWithFlags(&c->ev_groups, hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&c->ev_copy, hipEventDisableSystemFence));
    // last-workgroup-done counters of the finish kernels (each reset by its last workgroup)
    HIPCHECK(hipMemset(c->done.ensure(256), 0, 256));
    if (c->opt[kOptWarm]) warm_context(c);
    *out = c;
  });
  if (rc != BQG_OK && c) {
    delete c;
    *out = nullptr;
  }
  return rc;
}

int bqg_destroy(bqg_ctx* c) {
  if (!c) return BQG_OK;
  bqg_internal_comm_release(c);
  int rc = guard(c, [&] {
    HIPCHECK(hipStreamSynchronize(c->stream));
    for (DevBuf* b : {&c->partials, &c->counter, &c->hdr, &c->slots, &c->terms, &c->outcols, &c->lists,
                      &c->bitmap, &c->prefix, &c->cdbuf, &c->scdbuf, &c->mask, &c->misc, &c->done, &c->strings, &c->nfbuf, &c->rowmap})
      b->release();
    c->hhdr.release();
    c->hout.release();
    c->colpool.release();
    c->pool.reset();
    for (int i = 0; i < 2; ++i) {
      if (c->stage[i]) (void)hipHostFree(c->stage[i]);
      if (c->stage_ev[i]) (void)hipEventDestroy(c->stage_ev[i]);
    }
    for (int i = 0; i < 4; ++i)
      if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    for (int i = 0; i < 2; ++i)
      if (c->ev_sh[i]) (void)hipEventDestroy(c->ev_sh[i]);
    if (c->ev_groups) (void)hipEventDestroy(c->ev_groups);
    if (c->ev_copy) (void)hipEventDestroy(c->ev_copy);
    if (c->own) (void)hipStreamDestroy(c->own);
  });
  delete c;
  return rc;
}

const char* bqg_last_error(bqg_ctx* c) { return c ? c->err.c_str() : g_err.c_str(); }

int bqg_set_stream(bqg_ctx* c, void* s) {
  return guard(c, [&] { c->stream = s ? (hipStream_t)s : c->own; });
}

int bqg_synchronize(bqg_ctx* c) {
  return guard(c, [&] { HIPCHECK(hipStreamSynchronize(c->stream)); });
}

int bqg_enable_timing(bqg_ctx* c, int on) {
  return guard(c, [&] {
    c->timing = on == 2 ? 2 : (on != 0 ? 1 : 0);
    c->scan_ms_sum = 0;
    c->timed_queries = 0;
  });
}

int bqg_last_timing(bqg_ctx* c, bqg_timing* out) {
  return guard(c, [&] {
    *out = c->last;
    out->regrows = c->last_regrows;
    out->scan_ms_sum = c->scan_ms_sum;
    out->timed_queries = c->timed_queries;
  });
}

int bqg_alloc_pinned(bqg_ctx* c, size_t bytes, void** out) {
  return guard(c, [&] {
    if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) fail(BQG_E_OOM, "pinned allocation failed");
  });
}

int bqg_free_pinned(bqg_ctx* c, void* p) {
  return guard(c, [&] { HIPCHECK(hipHostFree(p)); });
}

int bqg_table_create(bqg_ctx* c, int64_t nrows, int32_t ncols, const int32_t* dtypes, bqg_table** out) {
  bqg_table* t = nullptr;
  int rc = guard(c, [&] {
    if (nrows < 0 || nrows >= (int64_t)0xFFFFFFFF) fail(BQG_E_INVALID, "table rows must be in [0, 2^32-1)");
    if (ncols < 0) fail(BQG_E_INVALID, "negative column count");
    t = new bqg_table();
    t->ctx = c;
    t->nrows = nrows;
    for (int i = 0; i < ncols; ++i) {
      int32_t slot;
      if (dtypes[i] < BQG_BOOL || dtypes[i] > BQG_F64) fail(BQG_E_INVALID, "unknown dtype %d", dtypes[i]);
      Column col;
      col.dtype = dtypes[i];
      t->cols.push_back(col);
      (void)slot;
    }
    for (Column& col : t->cols) alloc_column(c, col, nrows, true);
    c->tables.push_back(t);
    *out = t;
  });
  if (rc != BQG_OK && t) {
    for (Column& col : t->cols) c->colpool.put(col.dev, col.bytes);
    delete t;
  }
  return rc;
}

int bqg_table_destroy(bqg_table* t) {
  if (!t) return BQG_OK;
  int rc = guard(t->ctx, [&] {
    HIPCHECK(hipStreamSynchronize(t->ctx->stream));
    for (Column& col : t->cols) {
      t->ctx->colpool.put(col.dev, col.bytes);
      t->ctx->colpool.put(col.shadow.dev, col.shadow.bytes);
    }
  });
  auto& v = t->ctx->tables;
  v.erase(std::remove(v.begin(), v.end(), t), v.end());
  delete t;
  return rc;
}

int bqg_table_device_bytes(bqg_table* t, int64_t* bytes) {
  if (!t || !bytes) return BQG_E_INVALID;
  return guard(t->ctx, [&] {
    int64_t b = 0;
    for (const Column& col : t->cols) b += (int64_t)col.bytes + (int64_t)col.shadow.bytes;
    *bytes = b;
  });
}

int bqg_table_build_compact(bqg_table* t, int32_t n, const int32_t* cols, int32_t* built) {
  if (!t) return BQG_E_INVALID;
  return guard(t->ctx, [&] {
    if (n < 0 || (n && !cols)) fail(BQG_E_INVALID, "bad column list");
    int32_t k = 0;
    for (int i = 0; i < n; ++i) {
      if (cols[i] < 0 || cols[i] >= (int)t->cols.size()) fail(BQG_E_INVALID, "column %d out of range", cols[i]);
      // an integer column's narrow offsets, else a float64 column's exact codes
      if (ensure_shadow(t->ctx, t, cols[i], 1) || ensure_shadow(t->ctx, t, cols[i], 2)) ++k;
    }
    HIPCHECK(hipStreamSynchronize(t->ctx->stream));
    if (built) *built = k;
  });
}

int bqg_table_drop_compact(bqg_table* t) {
  if (!t) return BQG_E_INVALID;
  return guard(t->ctx, [&] {
    HIPCHECK(hipStreamSynchronize(t->ctx->stream));
    drop_shadows(t->ctx, t);
  });
}

int bqg_table_add_column(bqg_table* t, int32_t dtype, int32_t* slot_out) {
  return guard(t->ctx, [&] {
    if (dtype < BQG_BOOL || dtype > BQG_F64) fail(BQG_E_INVALID, "unknown dtype %d", dtype);
    Column col;
    col.dtype = dtype;
    alloc_column(t->ctx, col, t->nrows, true);
    t->cols.push_back(col);
    *slot_out = (int32_t)t->cols.size() - 1;
  });
}

// 0: pageable host memory, 1: page-locked host memory, 2: device memory
static int mem_kind(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return a.type == hipMemoryTypeDevice ? 2 : (a.type == hipMemoryTypeHost ? 1 : 0);
}

int bqg_push_chunk(bqg_table* t, int32_t col, const void* host, int64_t nrows, int64_t row_offset) {
  bqg_ctx* c = t->ctx;
  return guard(c, [&] {
    if (col < 0 || col >= (int)t->cols.size()) fail(BQG_E_INVALID, "column %d out of range", col);
    if (row_offset < 0 || nrows < 0 || row_offset + nrows > t->nrows) fail(BQG_E_INVALID, "rows out of range");
    Column& k = t->cols[col];
    k.stats.valid = false;
    const size_t isz = dtype_size(k.dtype);
    const unsigned char* src = (const unsigned char*)host;
    size_t left = (size_t)nrows * isz;
    unsigned char* dst = k.dev + (size_t)row_offset * isz;
    const int kind = mem_kind(src);
    if (kind == 2) {
      // device memory (another table's column, a collective's receive buffer): D2D copy,
      // stream-ordered; complete by the next bqg_table_sync / synchronising call
      HIPCHECK(hipMemcpyAsync(dst, src, left, hipMemcpyDeviceToDevice, c->stream));
      return;
    }
    if (left >= (1u << 20) && kind == 1) {
      // page-locked source (e.g. another query's result block): one DMA, no staging memcpy;
      // synchronous like the staged path, so the caller may reuse the buffer on return
      HIPCHECK(hipMemcpyAsync(dst, src, left, hipMemcpyHostToDevice, c->stream));
      HIPCHECK(hipStreamSynchronize(c->stream));
      return;
    }
    while (left) {
      const size_t n = std::min(left, bqg_ctx::kStage);
      const int i = c->stage_i;
      c->stage_i ^= 1;
      HIPCHECK(hipEventSynchronize(c->stage_ev[i]));
      memcpy(c->stage[i], src, n);
      HIPCHECK(hipMemcpyAsync(dst, c->stage[i], n, hipMemcpyHostToDevice, c->stream));
      HIPCHECK(hipEventRecord(c->stage_ev[i], c->stream));
      src += n;
      dst += n;
      left -= n;
    }
  });
}

int bqg_table_load_carrays(bqg_table* t, int32_t n, const int32_t* cols, const char* const* carray_dirs,
                           const int64_t* chunklens, int32_t nthreads, int32_t decode, bqg_ingest_stats* stats) {
  bqg_ctx* c = t->ctx;
  return guard(c, [&] {
    if (n < 0 || (n && (!cols || !carray_dirs || !chunklens))) fail(BQG_E_INVALID, "bad column list");
    if (decode < BQG_DECODE_AUTO || decode > BQG_DECODE_DEVICE) fail(BQG_E_INVALID, "unknown decoder %d", decode);
    std::vector<IngestJob> jobs(n);
    for (int i = 0; i < n; ++i) {
      const int32_t col = cols[i];
      if (col < 0 || col >= (int)t->cols.size()) fail(BQG_E_INVALID, "column %d out of range", col);
      if (!carray_dirs[i]) fail(BQG_E_INVALID, "null carray directory");
      if (chunklens[i] <= 0) fail(BQG_E_INVALID, "chunklen must be positive");
      for (int k = 0; k < i; ++k)
        if (cols[k] == col) fail(BQG_E_INVALID, "column %d listed twice", col);
      Column& k = t->cols[col];
      k.stats.valid = false;
      IngestJob& job = jobs[i];
      job.device = c->device;
      job.dev_dst = k.dev;
      job.carray_dir = carray_dirs[i];
      job.nrows = t->nrows;
      job.itemsize = (int)dtype_size(k.dtype);
      job.chunklen = chunklens[i];
      job.nthreads = nthreads;
      job.stream = c->stream;
    }
    // AUTO: the device decoder for large calls; below ~128 MB decoded the host threads win (a
    // batch costs the device path at least one long serial stream decode, ~3 ms)
    int64_t total = 0;
    for (const IngestJob& j : jobs) total += j.nrows * j.itemsize;
    const bool dev = decode == BQG_DECODE_DEVICE || (decode == BQG_DECODE_AUTO && total >= (int64_t(128) << 20));
    for (IngestJob& j : jobs) j.device_decode = dev;
    HIPCHECK(hipStreamSynchronize(c->stream));  // the columns' zero-fill has landed
    std::vector<IngestStats> st(n);
    std::string err;
    if (dev) {
      if (ingest_carrays_device(jobs, c->ingest, st, err) != 0) fail(BQG_E_INVALID, "%s", err.c_str());
    } else {
      for (int i = 0; i < n; ++i)
        if (ingest_carray(jobs[i], c->ingest, &st[i], err) != 0) fail(BQG_E_INVALID, "%s", err.c_str());
    }
    if (stats)
      for (int i = 0; i < n; ++i) {
        stats[i].chunks = st[i].chunks;
        stats[i].compressed_bytes = st[i].compressed_bytes;
        stats[i].bytes = st[i].bytes;
        stats[i].device_splits = st[i].device_splits;
        stats[i].host_chunks = dev ? st[i].host_fallback : st[i].chunks;
        stats[i].decoder = dev ? BQG_DECODE_DEVICE : BQG_DECODE_HOST;
      }
  });
}

int bqg_table_load_carray_ex(bqg_table* t, int32_t col, const char* carray_dir, int64_t chunklen, int32_t nthreads,
                             int32_t decode, bqg_ingest_stats* stats) {
  return bqg_table_load_carrays(t, 1, &col, &carray_dir, &chunklen, nthreads, decode, stats);
}

int bqg_table_load_carray(bqg_table* t, int32_t col, const char* carray_dir, int64_t chunklen, int32_t nthreads) {
  return bqg_table_load_carray_ex(t, col, carray_dir, chunklen, nthreads, BQG_DECODE_AUTO, nullptr);
}

int bqg_table_sync(bqg_table* t) {
  return guard(t->ctx, [&] {
    HIPCHECK(hipStreamSynchronize(t->ctx->stream));
    for (int i = 0; i < (int)t->cols.size(); ++i) compute_stats(t, i);
  });
}

int bqg_table_nrows(bqg_table* t, int64_t* nrows) {
  if (!t) return BQG_E_INVALID;
  return guard(t->ctx, [&] { *nrows = t->nrows; });
}

int bqg_table_ncols(bqg_table* t, int32_t* ncols) {
  if (!t) return BQG_E_INVALID;
  return guard(t->ctx, [&] { *ncols = (int32_t)t->cols.size(); });
}

int bqg_table_dtype(bqg_table* t, int32_t col, int32_t* dtype) {
  if (!t) return BQG_E_INVALID;
  return guard(t->ctx, [&] {
    if (col < 0 || col >= (int)t->cols.size()) fail(BQG_E_INVALID, "column %d out of range", col);
    *dtype = t->cols[col].dtype;
  });
}

int bqg_table_column_ptr(bqg_table* t, int32_t col, void** dev_ptr) {
  if (!t) return BQG_E_INVALID;
  return guard(t->ctx, [&] {
    if (col < 0 || col >= (int)t->cols.size()) fail(BQG_E_INVALID, "column %d out of range", col);
    *dev_ptr = t->cols[col].dev;
  });
}

int bqg_table_stats(bqg_table* t, int32_t col, int64_t* imin, int64_t* imax, double* fmin, double* fmax,
                    int32_t* has_nan) {
  return guard(t->ctx, [&] {
    if (col < 0 || col >= (int)t->cols.size()) fail(BQG_E_INVALID, "column %d out of range", col);
    compute_stats(t, col);
    const ColStats& s = t->cols[col].stats;
    if (imin) *imin = s.imin;
    if (imax) *imax = s.imax;
    if (fmin) *fmin = s.fmin;
    if (fmax) *fmax = s.fmax;
    if (has_nan) *has_nan = s.has_nan ? 1 : (s.empty ? -1 : 0);
  });
}

int bqg_table_read(bqg_table* t, int32_t col, void* host, int64_t nrows, int64_t row_offset) {
  return guard(t->ctx, [&] {
    if (col < 0 || col >= (int)t->cols.size()) fail(BQG_E_INVALID, "column %d out of range", col);
    if (row_offset < 0 || nrows < 0 || row_offset + nrows > t->nrows) fail(BQG_E_INVALID, "rows out of range");
    const size_t isz = dtype_size(t->cols[col].dtype);
    HIPCHECK(hipMemcpyAsync(host, t->cols[col].dev + (size_t)row_offset * isz, (size_t)nrows * isz,
                            mem_kind(host) == 2 ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, t->ctx->stream));
    HIPCHECK(hipStreamSynchronize(t->ctx->stream));
  });
}

int bqg_where(bqg_ctx* c, bqg_table* t, int32_t n_terms, const bqg_term* terms, int32_t out_mask_col,
              int64_t* n_pass) {
  return guard(c, [&] {
    if (out_mask_col < 0 || out_mask_col >= (int)t->cols.size() || t->cols[out_mask_col].dtype != BQG_BOOL)
      fail(BQG_E_INVALID, "where output must be a BOOL column");
    Plan pl;
    build_terms(c, t, pl, n_terms, terms);
    if (pl.tcol.empty()) scan_col(pl, out_mask_col);  // no terms: every row passes
    pl.p.ncols = (int)pl.tcol.size();
    for (int i = 0; i < pl.p.ncols; ++i) {
      const Column& col = t->cols[pl.tcol[i]];
      pl.p.cols[i] = DevCol{col.dev, col.dtype, dtype_lg(col.dtype)};
    }
    pl.p.nrows = t->nrows;
    pl.p.mask_col = -1;
    unsigned long long* d = (unsigned long long*)c->hdr.ensure(64);
    HIPCHECK(hipMemsetAsync(d, 0, 8, c->stream));
    if (t->nrows > 0) launch_where(pl.p, t->cols[out_mask_col].dev, d, scan_blocks(c, t->nrows, 8), c->stream);
    HIPCHECK(hipGetLastError());
    unsigned long long* h = (unsigned long long*)c->hhdr.ensure(64);
    HIPCHECK(hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    t->cols[out_mask_col].stats.valid = false;
    if (n_pass) *n_pass = (int64_t)h[0];
  });
}

int bqg_expand_subgroups(bqg_ctx* c, bqg_table* t, int32_t basket_col, int32_t mask_col, int32_t out_mask_col) {
  return guard(c, [&] {
    const int nc = (int)t->cols.size();
    if (basket_col < 0 || basket_col >= nc) fail(BQG_E_INVALID, "basket column out of range");
    if (mask_col < 0 || mask_col >= nc || t->cols[mask_col].dtype != BQG_BOOL) fail(BQG_E_INVALID, "mask must be BOOL");
    if (out_mask_col < 0 || out_mask_col >= nc || t->cols[out_mask_col].dtype != BQG_BOOL)
      fail(BQG_E_INVALID, "output mask must be BOOL");
    if (out_mask_col == mask_col) fail(BQG_E_INVALID, "output mask must differ from the input mask");
    const int64_t N = t->nrows;
    if (N == 0) return;
    const int64_t tiles = (N + kTileRows - 1) / kTileRows;
    unsigned int* scratch = (unsigned int*)c->misc.ensure((size_t)(tiles + 1) * 4 + (2 * (tiles / 1024 + 2) + 4096) * 4 +
                                                          (size_t)N + 256);
    const Column& b = t->cols[basket_col];
    DevCol bc{b.dev, b.dtype, dtype_lg(b.dtype)};
    launch_expand_subgroups(bc, t->cols[mask_col].dev, t->cols[out_mask_col].dev, N, 0, scratch, c->stream);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(c->stream));
    t->cols[out_mask_col].stats.valid = false;
  });
}

int bqg_groupby(bqg_ctx* c, bqg_table* t, const bqg_query* q, bqg_result** out) {
  return guard(c, [&] {
    if (!q || !out) fail(BQG_E_INVALID, "null query/output");
    *out = nullptr;
    c->dev_target = nullptr;
    c->last_regrows = 0;
    run_groupby_grow(c, t, q, out);
  });
}

int bqg_groupby_table(bqg_ctx* c, bqg_table* t, const bqg_query* q, bqg_table** out) {
  return guard(c, [&] {
    if (!q || !out) fail(BQG_E_INVALID, "null query/output");
    *out = nullptr;
    struct Reset {
      bqg_ctx* c;
      ~Reset() { c->dev_target = nullptr; }
    } reset{c};
    c->dev_target = out;
    bqg_result* r = nullptr;
    c->last_regrows = 0;
    run_groupby_grow(c, t, q, &r);
    if (r) table_from_host_result(c, r);  // empty / synthesized results: host-built
  });
}

int bqg_select_rows_table(bqg_ctx* c, bqg_table* t, const bqg_query* q, int32_t n_cols, const int32_t* cols,
                          bqg_table** out) {
  if (!out) return guard(c, [&] { fail(BQG_E_INVALID, "null output"); });
  *out = nullptr;
  c->dev_target = out;
  bqg_result* r = nullptr;
  const int rc = bqg_select_rows(c, t, q, n_cols, cols, &r);
  c->dev_target = nullptr;
  if (r) bqg_result_free(r);
  return rc;
}

int bqg_select_rows(bqg_ctx* c, bqg_table* t, const bqg_query* q, int32_t n_cols, const int32_t* cols,
                    bqg_result** out) {
  return guard(c, [&] {
    if (n_cols < 0 || n_cols > kMaxKeys + kMaxAggs) fail(BQG_E_UNSUPPORTED, "too many selected columns");
    for (int i = 0; i < n_cols; ++i)
      if (cols[i] < 0 || cols[i] >= (int)t->cols.size()) fail(BQG_E_INVALID, "column %d out of range", cols[i]);
    const int64_t N = t->nrows;
    const int64_t tiles = (N + kTileRows - 1) / kTileRows;
    // mask: precomputed column, fused terms, or all rows
    unsigned char* mask = nullptr;
    if (q && q->n_terms > 0) {
      Plan pl;
      build_terms(c, t, pl, q->n_terms, q->terms);
      pl.p.ncols = (int)pl.tcol.size();
      for (int i = 0; i < pl.p.ncols; ++i) {
        const Column& col = t->cols[pl.tcol[i]];
        pl.p.cols[i] = DevCol{col.dev, col.dtype, dtype_lg(col.dtype)};
      }
      pl.p.nrows = N;
      pl.p.mask_col = -1;
      if (q->mask_col >= 0) {
        pl.p.mask_col = scan_col(pl, q->mask_col);
        pl.p.ncols = (int)pl.tcol.size();
        const Column& col = t->cols[q->mask_col];
        pl.p.cols[pl.p.mask_col] = DevCol{col.dev, col.dtype, 0};
      }
      mask = (unsigned char*)c->mask.ensure(column_bytes(N, BQG_U8));
      unsigned long long* d = (unsigned long long*)c->hdr.ensure(64);
      HIPCHECK(hipMemsetAsync(d, 0, 8, c->stream));
      if (N > 0) launch_where(pl.p, mask, d, scan_blocks(c, N, 8), c->stream);
    } else if (q && q->mask_col >= 0) {
      if (t->cols[q->mask_col].dtype != BQG_BOOL) fail(BQG_E_INVALID, "mask must be BOOL");
      mask = t->cols[q->mask_col].dev;
    } else {
      mask = (unsigned char*)c->mask.ensure(column_bytes(N, BQG_U8));
      HIPCHECK(hipMemsetAsync(mask, 1, (size_t)N + 4, c->stream));
    }
    bqg_result* r = new bqg_result();
    std::unique_ptr<bqg_result> guard_r(r);
    unsigned int* tc = (unsigned int*)c->lists.ensure((size_t)(tiles + 1) * 4 + (2 * (tiles / 1024 + 2) + 4096) * 4 + 256);
    int64_t total = 0;
    if (N > 0) {
      launch_select_count(mask, N, tc, c->stream);
      launch_select_scan(tc, tiles, tc + tiles + 1, c->stream);
      // total = offset of the last tile + its count: recount on host from the mask tail
      unsigned int* hc = (unsigned int*)c->hhdr.ensure(64);
      HIPCHECK(hipMemcpyAsync(hc, tc + tiles - 1, 4, hipMemcpyDeviceToHost, c->stream));
      std::vector<unsigned char> tail((size_t)(N - (tiles - 1) * kTileRows));
      HIPCHECK(hipMemcpyAsync(tail.data(), mask + (tiles - 1) * kTileRows, tail.size(), hipMemcpyDeviceToHost, c->stream));
      HIPCHECK(hipStreamSynchronize(c->stream));
      total = hc[0];
      for (unsigned char v : tail) total += v ? 1 : 0;
    }
    r->n_rows = total;
    r->filtered = total < N;
    std::vector<DevCol> dcs;
    std::vector<void*> outs;
    size_t obytes = 0;
    std::vector<size_t> offs;
    for (int i = 0; i < n_cols; ++i) {
      const Column& col = t->cols[cols[i]];
      dcs.push_back(DevCol{col.dev, col.dtype, dtype_lg(col.dtype)});
      offs.push_back(obytes);
      obytes += ((size_t)total * dtype_size(col.dtype) + 255) & ~size_t(255);
    }
    unsigned char* ob = (unsigned char*)c->outcols.ensure(obytes + 256);
    for (int i = 0; i < n_cols; ++i) outs.push_back(ob + offs[i]);
    if (total > 0) launch_select_gather(mask, N, tc, dcs.data(), n_cols, outs.data(), c->stream);
    HIPCHECK(hipGetLastError());
    if (c->dev_target) {
      std::vector<int> dts;
      std::vector<const void*> src;
      for (int i = 0; i < n_cols; ++i) {
        dts.push_back(t->cols[cols[i]].dtype);
        src.push_back(outs[i]);
      }
      table_from_device(c, dts, src, total);
      return;
    }
    BlockGuard blk;
    blk.reset(c->pool, c->pool_get(obytes + 64));
    if (obytes) HIPCHECK(hipMemcpyAsync(blk.b.p, ob, obytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    r->pool = c->pool;
    r->block = blk.release();
    for (int i = 0; i < n_cols; ++i) {
      r->dtypes.push_back(t->cols[cols[i]].dtype);
      r->ptrs.push_back((const unsigned char*)r->block.p + offs[i]);
    }
    *out = guard_r.release();
  });
}

int bqg_hash_partition(bqg_ctx* c, bqg_table* t, int32_t n_keys, const int32_t* key_cols, int32_t nparts,
                       int32_t out_col, int64_t* counts) {
  return guard(c, [&] {
    if (n_keys < 1 || n_keys > kMaxKeys) fail(BQG_E_UNSUPPORTED, "1..%d key columns", kMaxKeys);
    if (nparts < 1) fail(BQG_E_INVALID, "nparts must be >= 1");
    if (out_col < 0 || out_col >= (int)t->cols.size() || t->cols[out_col].dtype != BQG_U32)
      fail(BQG_E_INVALID, "partition output must be a U32 column");
    PartitionCols k{};
    k.nkeys = n_keys;
    for (int i = 0; i < n_keys; ++i) {
      if (key_cols[i] < 0 || key_cols[i] >= (int)t->cols.size()) fail(BQG_E_INVALID, "key column out of range");
      const Column& col = t->cols[key_cols[i]];
      k.cols[i] = DevCol{col.dev, col.dtype, dtype_lg(col.dtype)};
    }
    unsigned long long* d = (unsigned long long*)c->misc.ensure((size_t)nparts * 8 + 64);
    HIPCHECK(hipMemsetAsync(d, 0, (size_t)nparts * 8, c->stream));
    if (t->nrows > 0) launch_hash_partition(k, t->nrows, (uint32_t)nparts, (uint32_t*)t->cols[out_col].dev, d, c->stream);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(counts, d, (size_t)nparts * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    t->cols[out_col].stats.valid = false;
  });
}

int bqg_encode_bytes(bqg_ctx* c, bqg_table* t, int32_t out_col, const void* bytes, int32_t width, void* values,
                     int64_t values_cap, int64_t* n_values) {
  return guard(c, [&] {
    if (!t || out_col < 0 || out_col >= (int)t->cols.size() || t->cols[out_col].dtype != BQG_I32)
      fail(BQG_E_INVALID, "bqg_encode_bytes: output must be an INT32 column of the table");
    if (width < 1 || width > 4096) fail(BQG_E_INVALID, "bqg_encode_bytes: width %d out of range", width);
    if (!n_values || (t->nrows > 0 && !bytes)) fail(BQG_E_INVALID, "bqg_encode_bytes: null argument");
    const int64_t n = t->nrows;
    *n_values = 0;
    Column& out = t->cols[out_col];
    out.stats.valid = false;
    if (n == 0) return;
    if ((uint64_t)n >= 0xFFFFFFFFull) fail(BQG_E_UNSUPPORTED, "bqg_encode_bytes: 2^32 rows or more");
    uint64_t cap = 1024;
    while (cap < 2 * (uint64_t)n) cap <<= 1;
    const uint64_t nwords = ((uint64_t)n + 31) / 32, nblocks = (nwords + 1023) / 1024;
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t o_data = 0, o_table = al((size_t)n * width), o_first = o_table + al(cap * 8),
                 o_slot = o_first + al(cap * 4), o_bits = o_slot + al((size_t)n * 4),
                 o_wp = o_bits + al(nwords * 4 + 4), o_bs = o_wp + al(nwords * 4 + 4),
                 o_cnt = o_bs + al(nblocks * 4 + 4), o_vals = o_cnt + 256, total = o_vals + al((size_t)n * width);
    // the staging (raw bytes, table, per-row slots, values: ~2 x n x width) is released when
    // the call returns, however it returns -- a 100 M-row 'U8' column would otherwise keep
    // 7 GB of HBM for the context's lifetime
    struct Release {
      bqg_ctx* c;
      ~Release() {
        (void)hipStreamSynchronize(c->stream);
        c->strings.release();
      }
    } release{c};
    unsigned char* b = (unsigned char*)c->strings.ensure(total);
    hipStream_t st = c->stream;
    HIPCHECK(hipMemcpyAsync(b + o_data, bytes, (size_t)n * width,
                            mem_kind(bytes) == 2 ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    BytesEncode e{};
    e.data = b + o_data;
    e.n = n;
    e.width = width;
    e.table = (unsigned long long*)(b + o_table);
    e.mask = cap - 1;
    e.first = (uint32_t*)(b + o_first);
    e.row_slot = (uint32_t*)(b + o_slot);
    e.rep_bits = (unsigned int*)(b + o_bits);
    e.word_prefix = (unsigned int*)(b + o_wp);
    e.block_sum = (unsigned int*)(b + o_bs);
    e.groups = (unsigned long long*)(b + o_cnt);
    e.overflow = (unsigned int*)(b + o_cnt + 8);
    e.codes = (int32_t*)out.dev;
    e.values = b + o_vals;
    HIPCHECK(hipMemsetAsync(e.overflow, 0, 8, st));
    launch_bytes_encode(e, st);
    HIPCHECK(hipGetLastError());
    unsigned long long* h = (unsigned long long*)c->hhdr.ensure(64);
    HIPCHECK(hipMemcpyAsync(h, e.groups, 16, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    if (h[1] & 0xFFFFFFFFull) fail(BQG_E_HIP, "bqg_encode_bytes: dictionary table overflow");
    const int64_t G = (int64_t)h[0];
    *n_values = G;
    if (values) {
      if (G > values_cap) fail(BQG_E_INVALID, "values buffer holds %lld, column has %lld distinct values",
                               (long long)values_cap, (long long)G);
      HIPCHECK(hipMemcpyAsync(values, e.values, (size_t)G * width,
                              mem_kind(values) == 2 ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
    }
  });
}

int bqg_factorize(bqg_ctx* c, bqg_table* t, int32_t col, int64_t* labels, void* values, int64_t values_cap,
                  int64_t* n_values) {
  return guard(c, [&] {
    if (col < 0 || col >= (int)t->cols.size()) fail(BQG_E_INVALID, "column %d out of range", col);
    if (!n_values) fail(BQG_E_INVALID, "null n_values");
    Column& k = t->cols[col];
    compute_stats(t, col);
    // labels by a lookup table lut[v - min] for integer columns spanning at most 2^27 values,
    // else (floats, bools, wider spans) by a hash of the canonical key bits
    const bool integer = !dtype_is_float(k.dtype) && k.dtype != BQG_BOOL;
    const uint64_t range = (!integer || k.stats.empty) ? 1 : (uint64_t)k.stats.imax - (uint64_t)k.stats.imin + 1;
    const bool use_lut = integer && range != 0 && range <= (1ull << 27);
    // distinct values in first-appearance order: a groupby over the column with no aggregation
    bqg_table* vt = nullptr;
    {
      const int32_t key = col;
      bqg_query q{};
      q.n_keys = 1;
      q.key_cols = &key;
      q.mask_col = -1;
      struct Reset {
        bqg_ctx* c;
        ~Reset() { c->dev_target = nullptr; }
      } reset{c};
      c->dev_target = &vt;
      bqg_result* r = nullptr;
      run_groupby_grow(c, t, &q, &r);
      if (r) table_from_host_result(c, r);
    }
    std::unique_ptr<bqg_table, int (*)(bqg_table*)> vown(vt, bqg_table_destroy);
    const int64_t G = vt->nrows;
    *n_values = G;
    if (values && G > values_cap) fail(BQG_E_INVALID, "values buffer holds %lld, column has %lld distinct values",
                                       (long long)values_cap, (long long)G);
    const int64_t vmin = (!integer || k.stats.empty) ? 0 : k.stats.imin;
    const bool dev_out = labels && mem_kind(labels) == 2;
    long long* out = nullptr;
    if (labels) out = dev_out ? (long long*)labels : (long long*)c->outcols.ensure((size_t)t->nrows * 8 + 256);
    const Column& vc = vt->cols[0];
    if (labels) {
      const DevCol dvals{vc.dev, vc.dtype, dtype_lg(vc.dtype)}, dcol{k.dev, k.dtype, dtype_lg(k.dtype)};
      if (use_lut) {
        int32_t* lut = (int32_t*)c->misc.ensure(range * 4 + 256);
        launch_factor_labels(dvals, G, dcol, t->nrows, vmin, lut, out, c->stream);
      } else {
        uint64_t cap = 64;
        while (cap < 2 * (uint64_t)G) cap <<= 1;
        unsigned char* hb = (unsigned char*)c->misc.ensure(cap * 12 + 256);
        launch_factor_hash_labels(dvals, G, dcol, t->nrows, cap, (unsigned long long*)hb, (uint32_t*)(hb + cap * 8), out,
                                  c->stream);
      }
      HIPCHECK(hipGetLastError());
      if (!dev_out && t->nrows)
        HIPCHECK(hipMemcpyAsync(labels, out, (size_t)t->nrows * 8, hipMemcpyDeviceToHost, c->stream));
    }
    if (values && G)
      HIPCHECK(hipMemcpyAsync(values, vc.dev, (size_t)G * dtype_size(vc.dtype),
                              mem_kind(values) == 2 ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
  });
}

int bqg_result_view_get(bqg_result* r, bqg_result_view* out) {
  if (!r || !out) return BQG_E_INVALID;
  out->n_rows = r->n_rows;
  out->n_cols = (int32_t)r->dtypes.size();
  out->dtypes = r->dtypes.data();
  out->cols = r->ptrs.data();
  out->filtered = r->filtered;
  return BQG_OK;
}

int bqg_result_free(bqg_result* r) {
  if (!r) return BQG_OK;
  if (r->pool && r->block.p) r->pool->put(r->block);
  delete r;
  return BQG_OK;
}

}  // extern "C"
