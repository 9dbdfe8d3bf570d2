/*
 * bqgpu.h -- C ABI of libbqgpu, the MI355X (gfx950) shard-groupby engine.
 *
 * This is the drop-in boundary for bqueryd's per-shard calc path.  It replaces the block
 * of WorkerNode.handle_work that calls bquery (bqueryd/worker.py:291-323):
 *
 *   worker.py:291  ct = bquery.ctable(rootdir, mode='r', auto_cache=True)
 *                    -> bqg_table_create + bqg_push_chunk (+ bqg_table_sync)
 *   worker.py:298  ct.where_terms_factorization_check(terms)
 *                    -> host layer (bqueryd_amd/ctable.py) over the <col>.values caches
 *   worker.py:303  bool_arr = ct.where_terms(terms, cache=True)
 *                    -> bqg_where (device mask column) -- or fused into bqg_groupby
 *   worker.py:307  ct.is_in_ordered_subgroups(basket_col, bool_arr)
 *                    -> bqg_expand_subgroups
 *   worker.py:313  ct.groupby(groupby_cols, agg_list, bool_arr=bool_arr, rootdir=tmp_dir)
 *                    -> bqg_groupby
 *   worker.py:319  bcolz.fromiter(ct[cols].where(bool_arr), ...)   (aggregate=False)
 *                    -> bqg_select_rows
 * and the co-located cross-shard merge that the client does at bqueryd/rpc.py:164-173
 * ("we can only sum now") -> bqg_comm_init* + bqg_merge / bqg_merge_group (local re-group,
 * hash partition, RCCL exchange over xGMI, re-group, gather to rank 0; all on device).
 *
 * Conventions
 *  - Every function returns 0 on success and a negative BQG_E_* code on failure; the
 *    message is available from bqg_last_error(ctx) (per-context; ctx may be NULL for
 *    errors raised before a context exists).  The Python layer turns it into
 *    RuntimeError / KeyError / NotImplementedError so that the worker's ErrorMessage path
 *    (worker.py:171-176) is unchanged.
 *  - One context per device per host thread; a context is not re-entrant.
 *  - Host buffers passed to bqg_push_chunk are owned by the caller and may be reused as
 *    soon as the call returns (the library stages them through its own pinned buffers).
 *  - Result memory (bqg_result) is owned by the library until bqg_result_free.
 *  - Row counts of one table must be < 2^32 (row indices are carried as uint32 on device).
 */
#ifndef BQGPU_H
#define BQGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history: 5 -- bqg_timing.narrow (exact 32-bit codes on the partitioned path);
 * 6 -- bqg_timing.narrow == 2 (packed entries) and the engine options (bqg_set_option);
 * 7 -- bqg_merge_host / bqg_merge_group_host (merged table straight to host memory),
 *      bqg_encode_bytes (string columns as dictionary codes);
 * 8 -- bqg_timing.bytes is always the algorithmic bytes (the query's columns at
 *      their stored widths) and bqg_timing.bytes_read the bytes the scan actually read (less
 *      when it read compact resident copies); bqg_table_device_bytes, bqg_table_build_compact,
 *      bqg_table_drop_compact (the compact copies' HBM, built and released explicitly);
 * 9 -- bqg_comm_progress (the merge phase a rank is in, readable while it runs); option
 *      jit_async and bqg_jit_wait (no query waits for a run-time compile); option warm;
 *      bqg_merge_shared_host (the merged rows straight into node-shared host memory);
 * 10 -- bqg_timing.copy_ms (the result's copy to host memory inside total_ms); option
 *      slot_emit (the large-result emit without compaction or host round trip). */
#define BQG_ABI_VERSION 10

/* error codes */
#define BQG_OK 0
#define BQG_E_INVALID (-1)      /* bad argument / unknown column (KeyError/ValueError) */
#define BQG_E_UNSUPPORTED (-2)  /* query shape not supported (NotImplementedError) */
#define BQG_E_HIP (-3)          /* HIP runtime error */
#define BQG_E_OOM (-4)          /* device or pinned allocation failed */
#define BQG_E_STATE (-5)        /* call out of sequence */

/* column dtypes (numpy kinds: ?, i1, i2, i4, i8, u1, u2, u4, u8, f4, f8) */
enum bqg_dtype {
  BQG_BOOL = 0, BQG_I8, BQG_I16, BQG_I32, BQG_I64,
  BQG_U8, BQG_U16, BQG_U32, BQG_U64, BQG_F32, BQG_F64
};

/* aggregation ops, as accepted by bquery's create_agg_ctable */
enum bqg_agg_op {
  BQG_SUM = 0, BQG_COUNT, BQG_COUNT_DISTINCT, BQG_SORTED_COUNT_DISTINCT, BQG_MEAN, BQG_STD
};

/* where-term ops: bquery's codes 1..8 (==, !=, in, nin, >, >=, <, <=) plus two folded
 * constants produced by the host normaliser (e.g. int_col == 2.5 -> BQG_T_FALSE) */
enum bqg_term_op {
  BQG_T_FALSE = -1, BQG_T_TRUE = 0,
  BQG_T_EQ = 1, BQG_T_NE, BQG_T_IN, BQG_T_NIN, BQG_T_GT, BQG_T_GE, BQG_T_LT, BQG_T_LE
};

typedef struct bqg_ctx bqg_ctx;
typedef struct bqg_table bqg_table;
typedef struct bqg_result bqg_result;

/* One normalised where-term.  Integer/bool columns compare against ivals (uint64 columns:
 * the bit pattern), float columns against fvals (after promotion to float64).  For
 * IN/NIN the value list must be sorted ascending and duplicate-free. */
typedef struct {
  int32_t col;
  int32_t op;
  int64_t nvals;
  const int64_t* ivals;
  const double* fvals;
} bqg_term;

typedef struct {
  int32_t col;  /* input column */
  int32_t op;   /* enum bqg_agg_op */
} bqg_agg;

typedef struct {
  int32_t n_keys;
  const int32_t* key_cols;  /* groupby_col_list, in order */
  int32_t n_terms;
  const bqg_term* terms;    /* where_terms_list, AND-ed */
  int32_t mask_col;         /* -1, or a BOOL column holding a precomputed bool_arr */
  int32_t n_aggs;
  const bqg_agg* aggs;      /* aggregation_list, in order */
} bqg_query;

/* Read-only view of a result.  Columns: groupby keys (input dtypes) then one column per
 * aggregation (dtype per create_agg_ctable: sum keeps the input dtype, count /
 * count_distinct / sorted_count_distinct are int64, mean / std are float64).  Groups are
 * in first-appearance order of the passing rows, exactly as bquery emits them. */
typedef struct {
  int64_t n_rows;
  int32_t n_cols;
  const int32_t* dtypes;
  const void* const* cols;  /* host pointers, n_rows elements each */
  int32_t filtered;         /* 1 when the filter removed at least one row */
} bqg_result_view;

/* Per-query device timing of the dominant scan kernel (HIP events on the library stream). */
typedef struct {
  double scan_ms;        /* summed duration of the row-scan kernel launches of the last call */
  int32_t scan_launches;
  double total_ms;       /* all device work of the last call */
  int64_t rows;          /* input rows scanned */
  int64_t bytes;         /* algorithmic bytes: distinct input columns x their stored
                            itemsize x rows + output -- the same whichever copy the scan read */
  int32_t mode;          /* 0 private-LDS, 1 shared-LDS, 2 global dense, 3 global hash,
                            4 partitioned, 5 fused distinct pass (sorted_count_distinct) */
  int32_t specialized;   /* 1: the scan ran a query-specialised (run-time compiled) kernel */
  int32_t narrow;        /* partitioned mode: 1 when the summed values travelled as exact 32-bit
                            integer codes (ABI 5); 2 when the entries were packed 32-bit words
                            {16-bit value code, slot} (no or one summed column) */
  int32_t regrows;       /* times the last query was re-run after its group hash table or
                            count_distinct set filled past half, each time with twice the slots
                            (ABI 6) */
  int64_t bytes_read;    /* the column bytes the scan read + output (ABI 8): `bytes` unless it
                            read compact resident copies (option compact), then fewer */
  double compact_ms;     /* device time of the compact copies this query built on first use
                            (0 when none was built; timing level 1 only, else NaN) (ABI 8) */
  double scan_ms_sum;    /* scan_ms summed over every query since timing was (re-)enabled, and */
  int64_t timed_queries; /* how many (ABI 8): a benchmark loop reads them once at its end */
  double copy_ms;        /* the part of total_ms spent copying the result to host memory (large
                            results; 0 when the emit wrote it there directly; timing level 1
                            only, else NaN) (ABI 10) */
} bqg_timing;

/* ---------------- lifecycle ---------------- */
int bqg_abi_version(void);
int bqg_device_count(int* n);
int bqg_create(int device_ordinal, bqg_ctx** out);
int bqg_destroy(bqg_ctx* ctx);
const char* bqg_last_error(bqg_ctx* ctx);
/* Run library work on an external HIP stream (e.g. torch's current stream); NULL restores
 * the library's own stream. */
int bqg_set_stream(bqg_ctx* ctx, void* hip_stream);
int bqg_synchronize(bqg_ctx* ctx);
/* on: 0 off; 1 (any other non-zero) HIP events around the scan kernels (scan_ms) and the whole
 * query (total_ms); 2 the scan events only (total_ms NaN: two fewer event records per query).
 * Every call resets the running sums (bqg_timing.scan_ms_sum / timed_queries). */
int bqg_enable_timing(bqg_ctx* ctx, int on);
int bqg_last_timing(bqg_ctx* ctx, bqg_timing* out);

/* Engine options (ABI 6): launch shapes and path choices the planner otherwise makes by
 * itself -- for tests and profiling; every value gives the same results.  Per context; read
 * once from the environment when the context is created (BQGPU_OPTIONS="name=value,...";
 * BQGPU_JIT=0 and BQGPU_JIT_MIN_ROWS=<n> set "jit" / "jit_min_rows"), never on the query path.
 *   jit            1  run-time specialised (hiprtc) scans            0 | 1
 *   jit_min_rows   4Mi  ... for tables of at least this many rows
 *   partition      1  partitioned aggregation for large dense slot spaces   0 | 1
 *   part_wbits     0  slots per partition 2^wbits (0: auto)           0 | 6..13
 *   part_k         0  4-row chunks per scatter thread (0: auto)        0 | 1 | 2 | 4 (packed)
 *   part_threads   0  scatter workgroup size (0: auto)                 0 | 256 | 512 | 1024
 *   part_per_cu    0  scatter workgroups per CU (0: auto)              0..8
 *   part_splits    0  aggregate workgroups per partition (0: auto)
 *   part_narrow    1  exact 32-bit value codes of float sums: partition     0 | 1
 *                     entries, and integer (order-independent) sums in the
 *                     shared / global atomic modes
 *   fused_scd      1  one fused pass for count / distinct queries       0 | 1
 *   scd_compact    1  ... with 32-bit value codes when they fit         0 | 1
 *   scd_pack16     1  ... first value and first row in one LDS word     0 | 1
 *   priv_ahead     0  private scan: tiles in flight (0: default)       0..4
 *   private_per_cu 0  private scan: workgroups per CU (0: auto, 3 or 4) 0..8
 *   small_emit     1  one-workgroup emit for <= 8192 slots              0 | 1
 *   hash_slots     0  initial group hash-table slots (0: from rows)    0..2^31
 *   distinct_slots 0  initial count_distinct set slots (0: from rows)  0..2^31
 *   part_pack      1  packed 4-byte partition entries when they fit    0 | 1
 *   scd_runs       1  fused distinct pass in 256-row steps for clustered keys  0 | 1
 *   part_win       0  partitioned aggregate: tiles of bounds per LDS window   0 (auto) | 64..4096
 *   compact        1  private / shared / dense global scans read compact  0 | 1 | 2
 *                     resident copies of their columns (narrow integer
 *                     offsets; exact integer codes of float64 columns that
 *                     are only summed, as 1 / 2-byte offsets when they span
 *                     < 2^16, else int32; 2: int32 codes only)
 *   part_first     0  packed partitioned path: tiles whose entries also   0 (auto) | 1 none | 2 all
 *                     record their rows in tile (exact first rows in the
 *                     aggregate; auto: the tiles where first appearances
 *                     fall on uniform keys), the rest by the first-row pass
 *   fx_sums        1  shared / global / hash / partitioned-wide modes:     0 | 1 | 2
 *                     float sums of columns without an exact int64 code,
 *                     and the std pass's centred squares, as fixed-point
 *                     limbs in integer atomics -- the same bits on every
 *                     run (NaN / infinities are flags beside the limbs).
 *                     The shift is the column's when its finite values are
 *                     all multiples of 2^-shift (exact sums), else each
 *                     slot's own from its largest value (an extra pass;
 *                     2: per-slot shifts for every such column;
 *                     0: float64 atomics)
 *   mem_cap_mb     0  the context's budget for resident column memory     0 | MiB
 *                     (tables' columns and compact copies, pooled blocks
 *                     included; 0: the device's memory).  Past it a copy is
 *                     not built (the scan reads the column as stored) and a
 *                     column allocation first releases every table's
 *                     copies, then fails with BQG_E_OOM
 *   part_ring      0  packed partitioned scatter (query-specialised): tiles 0 (1) | 1 | 2
 *                     of row loads in flight per workgroup
 *   jit_async      1  a query shape whose specialised kernel is in neither  0 | 1
 *                     the memory nor the disk cache runs the precompiled
 *                     generic kernel while a background host thread compiles
 *                     it with hiprtc; later queries of the shape run it
 *                     (0: the query compiles and waits, seconds on a cold
 *                     cache).  Both kernels give the same bits
 *   warm           1  bqg_create runs one small query, so that a worker's    0 | 1
 *                     first query does not pay the library's start-up (code
 *                     object load, first launches, buffer sizing; read from
 *                     BQGPU_OPTIONS at context creation only)
 *   slot_emit      1  slot spaces above 8192: the first-appearance ranks     0 .. 3
 *                     come from the groups' first rows marked straight from
 *                     the slot arrays (a byte per row holding the query's
 *                     epoch, up to 2^30 rows; bitmap atomics beyond) and the
 *                     group count stays on the device for the emit (no
 *                     compaction pass, no host round trip before the emit);
 *                     2: the same, the emit writing one record per group and
 *                     a second pass the columns in rank order; 3: bitmap
 *                     atomics at every size; 0: compaction, count read back,
 *                     then the emit.  All give the same result
 * An unknown name or out-of-range value fails with BQG_E_INVALID.  bqg_reset_options restores
 * the defaults (then the environment's values). */
int bqg_set_option(bqg_ctx* ctx, const char* name, int64_t value);
int bqg_get_option(bqg_ctx* ctx, const char* name, int64_t* value);
int bqg_reset_options(bqg_ctx* ctx);
/* Wait for the background compiles of query-specialised kernels (option jit_async; ABI 9):
 * until none is queued or running, or timeout_ms (< 0: no limit).  *idle 1 when none is left
 * (0 on timeout); *compiled / *failed the background jobs (a compile, or a load of a code object
 * another process compiled into the disk cache) finished so far in this process.
 * Any out pointer may be NULL.  A benchmark calls it before its timed loop; a worker never
 * needs to. */
int bqg_jit_wait(bqg_ctx* ctx, double timeout_ms, int32_t* idle, int64_t* compiled, int64_t* failed);

/* ---------------- pinned host memory ---------------- */
int bqg_alloc_pinned(bqg_ctx* ctx, size_t bytes, void** out);
int bqg_free_pinned(bqg_ctx* ctx, void* p);

/* ---------------- device-resident shard tables ---------------- */
int bqg_table_create(bqg_ctx* ctx, int64_t nrows, int32_t ncols, const int32_t* dtypes,
                     bqg_table** out);
int bqg_table_destroy(bqg_table* t);
int bqg_table_add_column(bqg_table* t, int32_t dtype, int32_t* slot_out);
/* Copy rows [row_offset, row_offset + nrows) of column `col` from host memory (or from
 * device memory: another table's column, a collective's receive buffer -- a D2D copy that
 * is stream-ordered and complete at the next bqg_table_sync; keep the source alive until
 * then). */
int bqg_push_chunk(bqg_table* t, int32_t col, const void* host, int64_t nrows,
                   int64_t row_offset);
/* Cold-path ingest (worker.py:291 bquery.ctable(rootdir) + bcolz's per-chunk blosc decode,
 * which bqueryd runs on one thread, worker.py:40): decode the bcolz carray directory
 * `carray_dir` (data/__<i>.blp, one blosc frame of `chunklen` items each) straight into
 * column `col` -- `nthreads` host threads decompress chunks into page-locked double buffers
 * and DMA them with hipMemcpyAsync while the next chunk decodes.  The carray must hold the
 * table's row count of items of the column's dtype.  Synchronous; statistics are recomputed
 * by the next bqg_table_sync. */
int bqg_table_load_carray(bqg_table* t, int32_t col, const char* carray_dir, int64_t chunklen,
                          int32_t nthreads);
/* The same with a choice of decoder and a report.  BQG_DECODE_DEVICE: the host threads only
 * read the chunk files into page-locked memory, the compressed bytes cross PCIe, and the
 * blosc1 frames are decoded on the GPU (BloscLZ and LZ4 streams, byte shuffle, memcpyed
 * frames; a chunk with another codec -- zstd, zlib, snappy -- or bit shuffle is decoded by
 * host libblosc as in the host path).  BQG_DECODE_AUTO picks the device decoder for calls of
 * 128 MB decoded or more (C2 shard: 97 GB/s decoded into HBM vs 43 GB/s for 16 host decode
 * threads) and the host decoder below (a device batch costs at least one serial stream decode,
 * ~3 ms).  A corrupt stream fails the call (BQG_E_INVALID) on either path. */
enum bqg_decode { BQG_DECODE_AUTO = 0, BQG_DECODE_HOST = 1, BQG_DECODE_DEVICE = 2 };
typedef struct {
  int64_t chunks;
  int64_t compressed_bytes;  /* chunk file bytes read */
  int64_t bytes;             /* decoded bytes written to the column */
  int64_t device_splits;     /* compressed streams decoded on the GPU */
  int64_t host_chunks;       /* chunks decoded by host libblosc */
  int32_t decoder;           /* BQG_DECODE_HOST / BQG_DECODE_DEVICE: the one that ran */
} bqg_ingest_stats;
int bqg_table_load_carray_ex(bqg_table* t, int32_t col, const char* carray_dir, int64_t chunklen,
                             int32_t nthreads, int32_t decode, bqg_ingest_stats* stats);
/* Several columns in one call (the columns a query touches, ctable._ensure_device): with the
 * device decoder their chunks form one stream of batches, so one column's file reads overlap
 * the previous column's kernels.  stats: NULL or n entries. */
int bqg_table_load_carrays(bqg_table* t, int32_t n, const int32_t* cols, const char* const* carray_dirs,
                           const int64_t* chunklens, int32_t nthreads, int32_t decode,
                           bqg_ingest_stats* stats);
/* Wait for pushes and compute per-column statistics (min / max / has_nan). */
int bqg_table_sync(bqg_table* t);
int bqg_table_column_ptr(bqg_table* t, int32_t col, void** dev_ptr);
int bqg_table_stats(bqg_table* t, int32_t col, int64_t* imin, int64_t* imax, double* fmin,
                    double* fmax, int32_t* has_nan);
/* Copy rows of a device column back to host memory (or into device memory). */
int bqg_table_read(bqg_table* t, int32_t col, void* host, int64_t nrows, int64_t row_offset);
/* HBM held by the table (ABI 8): every column allocation plus its compact resident copy, if
 * one was built -- what a shard cache's byte budget has to count. */
int bqg_table_device_bytes(bqg_table* t, int64_t* bytes);
/* Compact resident copies (option compact) of columns `cols[0..n)` built now
 * instead of on the first query that reads them: an integer column whose range fits fewer
 * bytes as its offset from the minimum, a float64 column with exact integer codes as those
 * codes.  *built (optional) receives the copies built.  A column without a narrower form is
 * skipped.  bqg_table_drop_compact releases every copy of the table (a cache under memory
 * pressure; the next query that wants one builds it again). */
int bqg_table_build_compact(bqg_table* t, int32_t n, const int32_t* cols, int32_t* built);
int bqg_table_drop_compact(bqg_table* t);
int bqg_table_nrows(bqg_table* t, int64_t* nrows);
int bqg_table_ncols(bqg_table* t, int32_t* ncols);
int bqg_table_dtype(bqg_table* t, int32_t col, int32_t* dtype);

/* ---------------- calc path ---------------- */
/* where_terms: AND of the terms -> BOOL column `out_mask_col` (device); *n_pass receives the
 * number of passing rows.  (worker.py:303) */
int bqg_where(bqg_ctx* ctx, bqg_table* t, int32_t n_terms, const bqg_term* terms,
              int32_t out_mask_col, int64_t* n_pass);
/* is_in_ordered_subgroups: widen mask to whole runs of equal basket values that contain a
 * passing row.  (worker.py:306-307) */
int bqg_expand_subgroups(bqg_ctx* ctx, bqg_table* t, int32_t basket_col, int32_t mask_col,
                         int32_t out_mask_col);
/* groupby with the predicate fused into the scan.  (worker.py:313-314) */
int bqg_groupby(bqg_ctx* ctx, bqg_table* t, const bqg_query* q, bqg_result** out);
/* aggregate=False: the passing rows of `cols`, in row order.  (worker.py:316-323) */
int bqg_select_rows(bqg_ctx* ctx, bqg_table* t, const bqg_query* q, int32_t n_cols,
                    const int32_t* cols, bqg_result** out);
/* The same two calls with the result kept in HBM as a new table (columns as in
 * bqg_result_view; free with bqg_table_destroy): the co-located aggregate=True merge
 * (rpc.py:164-173 restated on the GPU, bqueryd_amd/dist.py) chains them without host copies. */
int bqg_groupby_table(bqg_ctx* ctx, bqg_table* t, const bqg_query* q, bqg_table** out);
int bqg_select_rows_table(bqg_ctx* ctx, bqg_table* t, const bqg_query* q, int32_t n_cols,
                          const int32_t* cols, bqg_table** out);
int bqg_result_view_get(bqg_result* r, bqg_result_view* out);

/* ---------------- co-located merge (replaces the client re-group, rpc.py:164-173) --------
 * Partition id (hash of the key VALUES mod nparts) of every row into the U32 column
 * `out_col`; counts[nparts] receives the rows per partition.  Identical on every rank, so
 * partials of one key meet on one rank after the all-to-all exchange. */
int bqg_hash_partition(bqg_ctx* ctx, bqg_table* t, int32_t n_keys, const int32_t* key_cols,
                       int32_t nparts, int32_t out_col, int64_t* counts);
int bqg_result_free(bqg_result* r);

/* ---------------- fixed-width byte / string columns ----------------
 * bquery factorizes string key columns and compares them in where_terms [ext-bquery]; here a
 * string column lives on the device as dictionary codes.  bqg_encode_bytes encodes t->nrows
 * fixed-width values (`width` bytes each: numpy 'S<n>' bytes, or the UCS-4 bytes of 'U<n>';
 * host or device memory) into the INT32 column `out_col`: code = 1 + the value's rank in order
 * of first appearance, and 0 for the empty string (all zero bytes: numpy's padding), so a
 * zero-initialised code compares like bquery's zero-initialised string.  values (NULL to
 * skip; at most values_cap values of `width` bytes) receives the distinct values in order of
 * first appearance, *n_values their count (BQG_E_INVALID when values_cap is too small).  On
 * the GPU: a hash of each row's bytes into a table of representative rows with a full byte
 * compare, the first row of each value, a rank scan of the first-row bitmap.  (ABI 7) */
int bqg_encode_bytes(bqg_ctx* ctx, bqg_table* t, int32_t out_col, const void* bytes, int32_t width, void* values,
                     int64_t values_cap, int64_t* n_values);

/* ---------------- factor caches (bquery auto_cache, worker.py:291) ----------------
 * The <col>.factor / <col>.values carrays bquery writes next to a shard's columns the first
 * time it groups by `col` (read back by where_terms_factorization_check, worker.py:298):
 * labels[nrows] (int64, host or device memory; NULL to skip) = first-appearance rank of each
 * row's value over ALL rows; values[*n_values] (column dtype; NULL to skip; at most
 * values_cap) = the distinct values in label order.  Every column dtype: integer columns
 * spanning at most 2^27 values through a lookup table, any other column (floats with khash
 * identity -0.0 == +0.0 and NaN == NaN, bools, wider integer spans) through a hash of its
 * canonical bits.  BQG_E_INVALID when `values` holds fewer than the distinct values. */
int bqg_factorize(bqg_ctx* ctx, bqg_table* t, int32_t col, int64_t* labels, void* values, int64_t values_cap,
                  int64_t* n_values);

/* ---------------- multi-GPU: RCCL over xGMI ----------------
 * The aggregate=True merge of co-located shards: the client's re-group of every shard's
 * finalized table with `sum` of every column (rpc.py:164-173), run across the node's GPUs on
 * device buffers.  One communicator per context; librccl is loaded on first use.
 *   bqg_comm_unique_id   ncclGetUniqueId: called once (rank 0); the host layer hands the
 *                        BQG_UNIQUE_ID_BYTES bytes to every rank (any side channel)
 *   bqg_comm_init        one rank per process (ncclCommInitRank on the context's GPU)
 *   bqg_comm_init_all    every rank in this process: one context per GPU (ncclCommInitAll)
 *   bqg_comm_init_local  every rank in this process, exchanging by device copies instead of
 *                        RCCL (contexts may share a GPU: the exchange logic on one GPU)
 *   bqg_merge            collective: every rank calls it with its partial tables (columns:
 *                        n_keys key columns, then the finalized aggregations, dtypes as
 *                        given); the merged table (sum of every non-key column by key) is
 *                        returned on rank 0 as a new device table, NULL elsewhere.
 *                        `reduced`: this rank's one table already has unique keys (a
 *                        co-located one-pass groupby), so the local re-group is skipped.
 *                        Rows of the merged table come grouped by key hash, not in the
 *                        client's first-appearance order (which is file-system order in the
 *                        reference, rpc.py:151); compare after sorting by the keys.
 *   bqg_merge_group      the same for n_local ranks driven from one host thread (a process
 *                        owning several GPUs, after bqg_comm_init_all); n_tables[i] tables
 *                        of rank i follow each other in `tables`; out[i] per rank.
 *   bqg_merge_host       bqg_merge with the merged table returned as a host result (rank 0;
 *                        NULL elsewhere): the gather to rank 0, then one copy to host memory.
 *   bqg_merge_group_host bqg_merge_group with a host result: when every rank of the
 *                        communicator is driven by this call, each rank copies its reduced
 *                        partition straight into its slice of one pinned host result over
 *                        its own link (no gather to rank 0); rows come in rank order.
 *   bqg_merge_shared_host (ABI 9) bqg_merge for one process per GPU, with the merged rows
 *                        written into host memory that every rank's process maps (shared
 *                        memory of the node): after the reduce each rank copies its partition
 *                        into its slice over its own PCIe link -- no gather to rank 0 and no
 *                        single 24 MB copy behind one link.  Layout of `host`: column j (schema
 *                        order) at byte sum over j' < j of align256(capacity_rows x itemsize(j'));
 *                        rank r's rows follow every lower rank's.  Every rank passes its own
 *                        mapping of the same block (page-locked by the library on first use and
 *                        kept registered while the same block is passed); *rows receives the
 *                        merged rows on every rank; when they exceed capacity_rows every rank
 *                        fails with BQG_E_INVALID (grow the block to *rows and merge again).
 *                        When the call returns on any rank, every rank's slice has landed.
 * The receive-side reduce sums each key's partials in source-rank order (deterministic), and
 * a rank's rows come in first-appearance order of the rows it received. */
#define BQG_UNIQUE_ID_BYTES 128
int bqg_comm_unique_id(void* out);
int bqg_comm_init(bqg_ctx* ctx, int32_t rank, int32_t nranks, const void* unique_id);
int bqg_comm_init_all(int32_t n, bqg_ctx* const* ctxs);
int bqg_comm_init_local(int32_t n, bqg_ctx* const* ctxs);
int bqg_comm_destroy(bqg_ctx* ctx);
int bqg_comm_info(bqg_ctx* ctx, int32_t* rank, int32_t* nranks);
/* Profiling: host wall time (ms) of this rank's part of the last merge, per phase -- 0 local
 * re-group + pack, 1 count exchange, 2 payload exchange, 3 reduce, 4 gather counts, 5 gather
 * to rank 0 (host results: 5 is this rank's copy to host memory, 4 the copy of the gathered
 * table); a collective step is charged to every rank of the call.  With bqg_enable_timing
 * every step waits for the device work it queued, so each phase holds its own device time.
 * Up to n values. */
int bqg_comm_last_phases(bqg_ctx* ctx, double* ms, int32_t n);
/* Progress of this rank's merges (ABI 9), safe to call from another host thread while a merge
 * runs -- a watchdog naming the step a hung collective waits in: *phase the merge phase entered
 * last (numbered as above) or -1 between merges, *started / *done the merges begun / ended
 * (done counts failures too).  Any pointer may be NULL. */
int bqg_comm_progress(bqg_ctx* ctx, int32_t* phase, int64_t* started, int64_t* done);
int bqg_merge(bqg_ctx* ctx, int32_t n_tables, bqg_table* const* tables, int32_t n_keys, int32_t n_cols,
              const int32_t* dtypes, int32_t reduced, bqg_table** out);
int bqg_merge_group(int32_t n_local, bqg_ctx* const* ctxs, const int32_t* n_tables, bqg_table* const* tables,
                    int32_t n_keys, int32_t n_cols, const int32_t* dtypes, int32_t reduced, bqg_table** out);
int bqg_merge_host(bqg_ctx* ctx, int32_t n_tables, bqg_table* const* tables, int32_t n_keys, int32_t n_cols,
                   const int32_t* dtypes, int32_t reduced, bqg_result** out);
int bqg_merge_group_host(int32_t n_local, bqg_ctx* const* ctxs, const int32_t* n_tables, bqg_table* const* tables,
                         int32_t n_keys, int32_t n_cols, const int32_t* dtypes, int32_t reduced, bqg_result** out);
int bqg_merge_shared_host(bqg_ctx* ctx, int32_t n_tables, bqg_table* const* tables, int32_t n_keys, int32_t n_cols,
                          const int32_t* dtypes, int32_t reduced, void* host, int64_t capacity_rows, int64_t* rows);

#ifdef __cplusplus
}
#endif
#endif /* BQGPU_H */
