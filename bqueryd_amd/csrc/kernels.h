// kernels.h -- launch interface between the host planner (api.hip) and the gfx950 kernels.
#pragma once

#include "common.h"

namespace bqg {

// Output column of the emit step (keys first, then aggregations).
struct EmitCol {
  int32_t kind;       // 0 = key, 1 = aggregation
  int32_t out_dtype;  // bqg_dtype of the output column
  int32_t op;         // bqg_agg_op (aggregations)
  int32_t state;      // sum-state index (SUM / MEAN / STD) or distinct-state index (CD / SCD)
  int32_t key;        // key index (keys)
  int32_t in_float;   // aggregation input column is float
  int32_t in_dtype;   // aggregation input dtype
  int32_t sum_state;  // MEAN / STD: the sum-state index of the input column (nonfinite pass)
  void* out;          // device output array (capacity >= groups)
};

struct EmitParams {
  int32_t ncols;
  int32_t nkeys;
  int32_t hash;
  int32_t nsum2;  // std second-moment states in SlotArrays::acc2
  DevKey keys[kMaxKeys];
  int32_t key_dtype[kMaxKeys];
  DevCol key_cols[kMaxKeys];  // hash mode 2: key columns, read at each slot's representative row
  EmitCol cols[kMaxKeys + kMaxAggs];
  const unsigned long long* cd[kMaxAggs];        // count_distinct per slot
  const unsigned long long* scd_changes[kMaxAggs];
  const unsigned long long* scd_first[kMaxAggs]; // first value bits per slot
  double sum_dec[kMaxSums];  // != 0: sum state q holds int64 codes, value = code / sum_dec[q]
  // nonfinite pass (a mean / std over a float column holding NaN or infinities): per slot the
  // last passing row, and per such sum state q its non-finite values' count and last row; the
  // value column is read at that row (bquery's row-order mean keeps an infinity only when it is
  // the group's one non-finite value and its last row)
  const uint32_t* nf_last;
  const uint32_t* nf_cnt[kMaxSums];
  const uint32_t* nf_row[kMaxSums];
  DevCol nf_col[kMaxSums];
};

// Private-LDS mode (small dense slot spaces): the scan writes per-workgroup partials, the
// single-workgroup finish kernel combines them and either emits the groups itself
// (emit_inline) or stores per-slot totals into SlotArrays for the generic emit path.
constexpr int kMaxPrivateSlots = 40;

struct PrivateLaunch {
  int blocks;
  size_t lds_bytes;
  unsigned long long* partials;   // [(2 + nsum)][nslots][blocks]
};

struct FinishParams {
  int nslots;
  int blocks;
  int nsum;
  int emit_inline;
  int32_t sum_is_float[kMaxSums];
  const unsigned long long* partials;
  unsigned long long* totals;     // [(2 + nsum) * nslots] scratch
  unsigned long long* out_hdr;    // [0] = groups, [1] = passing rows
  unsigned int* done;             // zero-initialised counter: the last reduce workgroup finishes
};

void launch_scan_private(const ScanParams& p, const PrivateLaunch& l, hipStream_t st);
void launch_private_finish(const FinishParams& f, const SlotArrays& s, const EmitParams& e,
                           hipStream_t st);
void launch_scan_shared(const ScanParams& p, const SlotArrays& s, int blocks, size_t lds_bytes,
                        hipStream_t st);
void launch_scan_global(const ScanParams& p, const SlotArrays& s, int blocks, hipStream_t st);
void launch_init_slots(const SlotArrays& s, int nsum, uint64_t nslots, hipStream_t st);
// fixed-point float sums (ScanParams::sum_enc 3) of the states in `states` to float64 bits in acc
struct FxShifts {
  int32_t shift[kMaxSums];
  const int32_t* emax[kMaxSums];  // per-slot shifts (ScanParams::fx_emax), or null
};
// the per-slot exponent pass of fixed-point sums with per-slot shifts (ScanParams::fx_emax)
struct FxEmaxLaunch {
  int32_t* emax[kMaxSums];  // [nslots] for the states that have them, else null
};
void launch_fx_emax(const ScanParams& p, const SlotArrays& s, const FxEmaxLaunch& fe, int blocks, hipStream_t st);
void launch_fx_finalize(unsigned long long* acc, const unsigned long long* fx, int nsum, int states, const FxShifts& sh,
                        uint64_t nslots, hipStream_t st);

// The nonfinite pass (EmitParams::nf_*): one scan over the rows with the query's terms and key
// coding (hash modes look the slot up in pass 1's table), recording per slot the last passing
// row and, for each sum state in `states`, the count and last row of its non-finite values.
// Arrays zeroed by the caller.  lds: slot space small enough for a per-workgroup LDS table of
// last rows (flushed with one atomicMax per slot).
constexpr uint64_t kNonfiniteLdsSlots = 16384;
struct NonfiniteLaunch {
  int32_t states;           // bit q: sum state q (ScanParams::cols[q]) is checked
  int32_t lds;
  uint32_t* last_row;       // [nslots]
  uint32_t* cnt[kMaxSums];  // [nslots] per checked state
  uint32_t* row[kMaxSums];  // [nslots] per checked state
};
void launch_nonfinite(const ScanParams& p, const SlotArrays& s, const NonfiniteLaunch& nf, int blocks,
                      hipStream_t st);

// count_distinct: pair (slot, value-code) set; bitmap when bitmap != nullptr, else hash set
struct DistinctLaunch {
  int vcol;                 // index into ScanParams::cols of the value column
  int64_t vmin;             // value code = v - vmin (ints) or canonical bits (floats)
  uint64_t vrange;          // value code space (bitmap mode)
  unsigned int* bitmap;     // [ceil(nslots * vrange / 32)]
  unsigned long long* set;  // hash set of packed (slot, vcode) keys (bitmap == nullptr)
  uint64_t set_mask;
  unsigned int* set_fill;
  unsigned int* overflow;
  unsigned long long* out;  // [nslots] distinct counts
  int lds_bitmap_words;     // > 0: per-workgroup LDS pre-filter of this many words
  // pair_rows (float values with group keys, integer pair spaces of 2^63 and more): set
  // entries are slot << 32 | representative row, probed at hash(slot, canonical value) and
  // matched by re-reading the value column at the representative row (full compare)
  int pair_rows;
};
void launch_count_distinct(const ScanParams& p, const SlotArrays& s, const DistinctLaunch& d,
                           int blocks, hipStream_t st);

// sorted_count_distinct: per-wave contiguous chunks, ordered monoid per slot
struct ScdLaunch {
  int vcol;
  int waves;                         // number of row chunks (one wave each)
  int64_t chunk_rows;                // rows per chunk (multiple of 64)
  int lds_state;                     // 1: per-wave state staged in LDS
  int slot_bits;                     // bits of a slot id (ballots per 64-row step)
  uint32_t* st_first_row;            // [waves][nslots]   (kNoRow = absent)
  unsigned long long* st_first;      // [waves][nslots]   first value bits
  unsigned long long* st_last;       // [waves][nslots]
  uint32_t* st_changes;              // [waves][nslots]
  unsigned long long* out_changes;   // [nslots]
  unsigned long long* out_first;     // [nslots]
  // fused variant (k_scd_fused: dense slots, small slot space): LDS match masks instead of
  // slot-bit ballots, per-slot row counts, optional count_distinct folded into the same pass
  int fused;                         // 1: k_scd_fused
  size_t wave_lds;                   // bytes of LDS per wave (16-byte multiple)
  uint32_t* st_count;                // [waves][nslots] rows per chunk (fused)
  unsigned long long* slot_cnt;      // fused + write_slots: SlotArrays::cnt to fill
  uint32_t* slot_fst;                // fused + write_slots: SlotArrays::fst to fill
  DistinctLaunch cd;                 // fused: cd.bitmap != nullptr -> count_distinct too
  int compact;                       // fused: 32-bit value codes (integer values, range < 2^32)
  int pack16;                        // compact: value codes < 2^16, first value + first row in one word
  int64_t vmin;                      // compact: value code = v - vmin
  int runs;                          // compact: the RUNS loop (clustered keys, no terms / mask)
};
// LDS bytes per wave of k_scd_fused for a slot space of nslots: a 32-byte state per slot (20
// bytes with compact 32-bit value codes) plus an 8-byte lane mask per slot
inline size_t scd_fused_wave_lds(uint64_t nslots, bool compact = false, bool pack16 = false) {
  // compact: 8-byte states + first values + first rows (pack16: one word for both); wide:
  // 32-byte states; then the 8-byte lane masks
  const size_t state = compact ? (((size_t)nslots * (pack16 ? 12 : 16) + 7) & ~size_t(7)) : (size_t)nslots * 32;
  return (state + (size_t)nslots * 8 + 15) & ~size_t(15);
}
constexpr int64_t kScdCompactMaxRows = 65280;  // rows per wave chunk of the compact pass (16-bit counts)
constexpr size_t kScdFusedMaxLds = 80 * 1024;  // per workgroup (4 waves + shared cd filter)
// fused_fn: query-specialised (JIT) k_scd_fused, or nullptr for the precompiled kernel
// pass_done (optional): recorded between the pass and the chunk combine (kernel timing)
void launch_scd(const ScanParams& p, const SlotArrays& s, const ScdLaunch& d, hipStream_t st,
                hipFunction_t fused_fn = nullptr, hipEvent_t pass_done = nullptr);

// emit: occupied slots -> first-appearance order -> finalised output columns
void launch_compact(const SlotArrays& s, uint64_t nslots, uint32_t* list_fst,
                    uint32_t* list_slot, unsigned int* count, unsigned long long* total,
                    uint32_t* scratch, hipStream_t st);
void launch_sort_small(uint32_t* list_fst, uint32_t* list_slot, unsigned int n,
                       uint32_t* order, hipStream_t st);
void launch_rank_bitmap(const uint32_t* list_fst, const uint32_t* list_slot, unsigned int n,
                        int64_t nrows, unsigned int* bitmap, unsigned int* word_prefix,
                        unsigned int* block_prefix, uint32_t* order, hipStream_t st);
// rank by the first-row bitmap and emit each group at its rank, in one pass (> 8192 groups)
void launch_rank_emit_bitmap(const EmitParams& e, const SlotArrays& s, const uint32_t* list_fst,
                             const uint32_t* list_slot, unsigned int n, int nsum, uint64_t nslots, int64_t nrows,
                             unsigned int* bitmap, unsigned int* word_prefix, unsigned int* block_prefix,
                             hipStream_t st);
void launch_emit(const EmitParams& e, const SlotArrays& s, const uint32_t* order,
                 unsigned int n, int nsum, uint64_t nslots, hipStream_t st);
// large slot spaces, no compaction and no host round trip before the emit: the groups' first
// rows marked -- in row_map (one byte per row, = epoch; cleared by the caller when the epoch
// wraps; the marking workgroups' passing rows in rows_part [1024], summed by the rank scan) or,
// with row_map null, in the bitmap by atomics (hdr then sits after the bitmap and is zeroed
// with it) -- their rank scan with the group count in hdr[0] (passing rows in hdr[1];
// both mirrored to host_hdr, page-locked, device-mapped, readable once ev_groups has
// completed), then the emit over the slots with the output columns at `out` laid out by that
// count (column j after the 256-byte aligned sizes of columns 0..j-1); with `rec` (capacity
// nslots x ncols 8-byte words) the emit writes one record per group and a second pass writes
// the columns from them in rank order (without, it stores the columns at the ranks)
void launch_slot_emit(const EmitParams& e, const SlotArrays& s, uint64_t nslots, int64_t nrows,
                      unsigned int* bitmap, unsigned char* row_map, unsigned char epoch,
                      unsigned long long* word_pair, unsigned int* block_prefix,
                      unsigned long long* rows_part, unsigned long long* hdr,
                      unsigned long long* host_hdr, hipEvent_t ev_groups, unsigned char* out,
                      unsigned long long* rec, hipStream_t st);
// slot spaces up to kSmallEmitSlots: compaction + ordering + emit in one workgroup (output
// columns of capacity nslots); hdr[0] = groups, hdr[1] = passing rows
constexpr uint32_t kSmallEmitSlots = 8192;
// a result's columns copied into a new device table's columns, each column's tail past its
// rows zeroed, in one kernel launch (table_from_device: a fill and a copy per column cost ~10 us
// each)
constexpr int kMaxCopyCols = kMaxKeys + kMaxAggs;
struct ColumnCopies {
  int n;
  unsigned char* dst[kMaxCopyCols];      // 16-byte aligned, cap bytes
  const unsigned char* src[kMaxCopyCols];  // 16-byte aligned, used bytes
  uint64_t used[kMaxCopyCols];
  uint64_t cap[kMaxCopyCols];            // a multiple of 16
};
void launch_column_copies(const ColumnCopies& cc, hipStream_t st);
// up to kZeroRanges word ranges zeroed by one kernel launch
constexpr int kZeroRanges = 4;
struct ZeroRanges {
  int n;
  unsigned int* p[kZeroRanges];
  uint64_t words[kZeroRanges];
};
void launch_zero_ranges(const ZeroRanges& z, hipStream_t st);
void launch_emit_small(const EmitParams& e, const SlotArrays& s, uint32_t nslots, int nsum,
                       unsigned long long* hdr, hipStream_t st);

// column statistics (min / max / nan) of one column
constexpr int kStatsMaxBlocks = 2048;
constexpr int kStatsWords = 7;  // min, max, NaN, lowest set bit, code flags, finite |max| bits, flags
void launch_stats(const DevCol& c, int64_t nrows, unsigned long long* out4, unsigned long long* scratch,
                  hipStream_t st);
// value runs of one column: rows whose value differs from the row before (out: one counter,
// zeroed by the caller)
void launch_runs(const DevCol& c, int64_t nrows, unsigned long long* out, hipStream_t st);

// where_terms -> uint8 mask column, passing-row count
void launch_where(const ScanParams& p, unsigned char* out_mask, unsigned long long* npass,
                  int blocks, hipStream_t st);
// is_in_ordered_subgroups
void launch_expand_subgroups(const DevCol& basket, const unsigned char* mask,
                             unsigned char* out, int64_t nrows, int blocks,
                             unsigned int* run_any_scratch, hipStream_t st);
// aggregate=False row selection: per-tile pass counts, then ordered compaction
void launch_select_count(const unsigned char* mask, int64_t nrows, unsigned int* tile_counts,
                         hipStream_t st);
void launch_select_scan(unsigned int* tile_counts, int64_t ntiles, unsigned int* scratch, hipStream_t st);
void launch_select_gather(const unsigned char* mask, int64_t nrows,
                          const unsigned int* tile_offsets, const DevCol* cols, int ncols,
                          void* const* outs, hipStream_t st);

// Partitioned aggregation (large dense slot spaces): tile scatter -> aggregate
constexpr int kPartMaxParts = 4096;
struct PartLaunch {
  int wbits;                 // slots per partition = 2^wbits
  int nparts;                // <= kPartMaxParts
  int blocks;                // workgroups of the scatter pass
  int splits;                // aggregate workgroups per partition (tile ranges)
  int threads;               // threads of a scatter workgroup: tiles of threads * 4 rows
  int tile_rows;             // threads * 4 * k
  int k;                     // 4-row chunks per scatter thread and tile (1 or 2)
  int64_t rows_per_block;    // contiguous rows per scatter workgroup, whole tiles
  int64_t ntiles;            // ceil(nrows / tile_rows)
  uint64_t capacity;         // entries per array = ntiles * tile_rows
  uint16_t* hdr;             // [ntiles][nparts + 1]: partition offsets in each sorted tile
  uint32_t* meta;            // [capacity]: row-in-tile << wbits | slot_low
  unsigned long long* vals;  // [nsum][capacity]: summed values (canonical 64-bit), or with
                             // narrow: uint32_t [nsum][capacity] exact integer codes
  // narrow entries: every summed column has an exact 32-bit code -- floats (ColStats::enc):
  // code = v * enc_mul (dyadic: 2^k) or rint(v * enc_mul) (cents: 100), summed in int64, total
  // = sum * 2^-k or sum / 100; integers with max - min < 2^32: code = v - enc_off (unsigned),
  // summed in uint64, total = sum + count * enc_off (mod 2^64, as the 64-bit path)
  int narrow;
  int32_t enc_kind[kMaxSums];  // 1 dyadic, 2 cents, 3 integer offset
  double enc_mul[kMaxSums];
  int64_t enc_off[kMaxSums];
  // packed entries (at most one summed column, its narrow codes spanning at most 2^16 values):
  // one 32-bit word per entry, code16 = code - enc_base16 above the 16-bit slot_low; the
  // aggregate's per-slot accumulator is count << sbits | sum of code16 (one 64-bit LDS atomic
  // per entry; flushed into the split record every pack_flush entries so neither field can
  // overflow), and it
  // marks each slot's first TILE: tile_mark [ntiles] (1 = some slot's first tile, zeroed
  // before the aggregate; each marked tile appended once to marked [nmarked]) and first_tag
  // [nslots] (its low 8 bits), then k_part_first_rows re-reads only the marked tiles for the
  // exact first rows
  int pack;
  int sbits;
  int64_t pack_flush;  // entries between flushes of the packed accumulators
  int64_t enc_base16;
  uint32_t* tile_mark;
  uint32_t* nmarked;  // tile_mark + ntiles (zeroed with it)
  uint32_t* marked;
  unsigned char* first_tag;
  // PACK: the tiles [0, rit_tiles) also store each entry's row in the tile (rit [rit_tiles x
  // tile_rows] u16, at the entry's own position): the aggregate keys a slot's first appearance
  // by t * tile_rows + rit -- the exact first row of every slot seen in those tiles (where
  // first appearances fall on random keys) -- and by t * tile_rows + tile_rows - 1 in later
  // tiles (its first tile only: k_part_first_rows re-reads the tiles marked for such slots)
  int64_t rit_tiles;
  uint16_t* rit;
  // splits > 1: [nparts][splits] split tables of partial_bytes each, added by k_part_combine
  unsigned char* partial;
  size_t partial_bytes;      // 2^wbits * (8 + 8 * nsum) (+ 24 * nsum with fx)
  int win;                   // aggregate window: tiles whose bounds are staged in LDS at once
  // wide entries with fixed-point float sums (ScanParams::sum_enc 3): the slot table and split
  // records carry limbs 1, 2 and the non-finite flags of every sum state ([nsum][3][W] after
  // the table)
  int fx;
};
// LDS bytes of a scatter workgroup: the staged tile (values, meta), tile counts (two
// buffers) / offsets and two sets of scan totals
inline size_t part_scatter_lds(int nparts, int threads, int nsum, int k = 1, bool narrow = false, bool pack = false) {
  // pack: + the tile's rows in tile (u16) staged beside the entry words
  return (size_t)threads * 4 * k * (4 + (pack ? 2 : (narrow ? 4 : 8) * (size_t)nsum)) + (size_t)nparts * 12 + 2 * 16 * 4;
}
// LDS bytes of an aggregate workgroup's slot table: count + first row + 8-byte sums (+ two
// 8-byte limbs and a flags word per sum with fixed-point sums), or (pack) the packed 8-byte
// accumulator + first tile
__host__ __device__ inline size_t part_agg_lds(int wbits, int nsum, bool pack, bool fx = false) {
  return ((size_t)1 << wbits) * (pack ? 12 : 8 + 8 * (size_t)nsum + (fx ? 8 * kFxWords * (size_t)nsum : 0));
}
// the aggregate walks its split's tiles in windows of PartLaunch::win tiles (four words of
// bounds per tile in LDS, up to kAggWinMax); a chunk of entry granules spans at most kAggK tiles
constexpr int kAggWin = 1024;     // the default window (option part_win = 0 and no room for more)
constexpr int kAggWinMax = 4096;  // 1024 threads x 4 tiles of header loads
constexpr int kAggK = 8;
inline size_t part_agg_lds_launch(int wbits, int nsum, bool pack, int win = kAggWin, bool fx = false) {
  return part_agg_lds(wbits, nsum, pack, fx) + 4 * (size_t)(win + kAggK + 1) * 4;
}
// fscatter: the query-specialised (JIT) scatter kernel, or nullptr for the precompiled one
// ffirst: the query-specialised (JIT) first-row pass of packed entries, or nullptr
void launch_partitioned(const ScanParams& p, const SlotArrays& s, const PartLaunch& L, hipStream_t st,
                        hipFunction_t fscatter = nullptr, hipFunction_t ffirst = nullptr);
void launch_exclusive_scan_u32(uint32_t* v, uint64_t n, uint32_t* scratch, hipStream_t st);

// cross-rank merge: partition id of every row from its key values
struct PartitionCols {
  DevCol cols[kMaxKeys];
  int nkeys;
};
void launch_hash_partition(const PartitionCols& k, int64_t nrows, uint32_t nparts, uint32_t* out,
                           unsigned long long* counts, hipStream_t st);

// cross-rank merge, send side: rows -> destination rank hash(key values) mod nranks (the
// partition of launch_hash_partition), packed per destination in one stable scatter
constexpr int kMergeMaxRanks = 256;  // destinations are kept as one byte per row
constexpr int kMergeMaxCols = kMaxKeys + kMaxAggs;
struct MergePack {
  PartitionCols keys;
  const unsigned char* cols[kMergeMaxCols];  // every column of the table (keys included)
  int32_t lg[kMergeMaxCols];                 // log2 of the element size
  int32_t ncols;
  int32_t nranks;
  int32_t nblocks;                           // merge_pack_grid
  int64_t nrows;
  int64_t rows_per_block;
  unsigned char* dest;                       // [nrows] scratch
  uint32_t* block_hist;                      // [nblocks][nranks] scratch
  unsigned long long* to_peer;               // [nranks] out: rows per destination
  unsigned long long* colbase;               // [nranks][ncols] out: byte offset of each packed column
  unsigned char* send;                       // packed blocks, destination order
};
void merge_pack_grid(int64_t nrows, int32_t* nblocks, int64_t* rows_per_block);
void launch_merge_pack(const MergePack& m, hipStream_t st);

// cross-rank merge: rows from several sources (the tables of one rank's shards, or the rows a
// rank received from every source rank), each source's rows unique by key, summed by key in
// one hash table -- no statistics, no planner, no first-appearance sort.  Sources are
// inserted one launch each, in source order, so every key's sums are added in source order
// (deterministic: a launch adds at most once per slot).  The table word is hash_hi32 << 32 |
// representative row (the key's first row, in the lowest source holding it); keys compare in
// full at the representative row.  Output rows come in representative-row order: first
// appearance in the concatenated sources, the client's order for a rank's shard tables.
constexpr int kMergeMaxVals = kMergeMaxCols;
struct MergeReduce {
  PartitionCols keys;                         // key columns of the received table
  const unsigned char* vals[kMergeMaxVals];   // value (sum) columns
  int32_t vdt[kMergeMaxVals];                 // their dtypes (the output dtype too)
  int32_t nvals;
  int64_t nrows;                              // received rows
  int64_t row0, row1;                         // this launch's source block
  unsigned long long* table;                  // [cap] kEmpty or hash_hi32 << 32 | rep row
  uint64_t mask;                              // cap - 1
  unsigned long long* acc;                    // [nvals][cap] 64-bit sums (f64 bits for floats)
  unsigned int* rep_bits;                     // [ceil(nrows / 32)] rows that represent a key
  unsigned int* word_prefix;                  // [ceil(nrows / 32)] rank-scan scratch
  unsigned int* block_sum;                    // [ceil(nrows / 32768)] rank-scan scratch
  unsigned int* overflow;                     // a probe ran past the table (cannot at load <= 1/2)
  int32_t unique_sources;                     // 1: every source holds each key at most once
                                              // (reduced partitions): plain stores / adds, no
                                              // zero-initialised sums
  unsigned long long* groups;                 // out: keys found
  unsigned char* out_keys[kMaxKeys];          // out columns, capacity nrows
  unsigned char* out_vals[kMergeMaxVals];
};
// table capacity for `rows` received rows (load <= 1/2)
inline uint64_t merge_reduce_cap(int64_t rows) {
  uint64_t cap = 1024;
  while (cap < 2 * (uint64_t)rows) cap <<= 1;
  return cap;
}
// every launch of the reduce on `st`: table init, one insert per non-empty source block
// (src_off[0..nsrc]), rank scan, emit; `groups` receives the key count on the device
void launch_merge_reduce(MergeReduce m, const int64_t* src_off, int nsrc, hipStream_t st);

// fixed-width byte strings (numpy 'S<n>' / 'U<n>') -> INT32 dictionary codes: 1 + the value's
// first-appearance rank, 0 for the empty string (bqg_encode_bytes)
struct BytesEncode {
  const unsigned char* data;  // [n][width] on the device
  int64_t n;
  int32_t width;
  unsigned long long* table;  // [cap] kEmpty or hash_hi32 << 32 | a row holding the value
  uint64_t mask;              // cap - 1
  uint32_t* first;            // [cap] first row of each slot's value
  uint32_t* row_slot;         // [n] each row's slot
  unsigned int* rep_bits;     // [ceil(n / 32)] first rows
  unsigned int* word_prefix;  // [ceil(n / 32)]
  unsigned int* block_sum;    // [ceil(n / 32768)]
  unsigned long long* groups; // out: distinct values
  unsigned int* overflow;     // a probe ran past the table (cannot at load <= 1/2)
  int32_t* codes;             // [n] out
  unsigned char* values;      // [distinct][width] out, first-appearance order
};
void launch_bytes_encode(BytesEncode e, hipStream_t st);

// std: per-slot means of the std columns (pass 1 totals -> pass 2 centers), on device
struct StdCenters {
  int32_t n;                // std columns
  int32_t state[kMaxSums];  // their sum-state index in SlotArrays::acc
  int32_t conv[kMaxSums];   // 0 float bits, 1 signed integer, 2 unsigned integer, 3 int64 codes / dec
  double dec[kMaxSums];
};
// compact resident copies (api.hip Column::shadow): an integer column as (v - off) in 1, 2 or 4
// bytes (dst_lg), a float64 column as its exact integer codes (kind 1 dyadic v * mul, 2 cents
// rint(v * mul)): code - off in 1 / 2 bytes (dst_lg 0 / 1), or the int32 code (dst_lg 2)
void launch_shadow_int(const DevCol& src, int64_t nrows, int64_t off, void* dst, int dst_lg, hipStream_t st);
void launch_shadow_code(const double* src, int64_t nrows, int kind, double mul, int64_t off, void* dst, int dst_lg,
                        hipStream_t st);
void launch_std_centers(const unsigned long long* cnt, const unsigned long long* acc, const StdCenters& sc,
                        uint64_t nslots, double* centers, hipStream_t st);

// factor cache labels (bquery auto_cache): lut [range] scratch, out [nrows] int64 labels
void launch_factor_labels(const DevCol& vals, int64_t nvals, const DevCol& col, int64_t nrows, int64_t vmin,
                          int32_t* lut, long long* out, hipStream_t st);

// ... any key column (floats, bools, wide integer spans): hash of canonical bits -> label;
// cap a power of two >= 2 * nvals, keys [cap] / labs [cap] scratch
void launch_factor_hash_labels(const DevCol& vals, int64_t nvals, const DevCol& col, int64_t nrows, uint64_t cap,
                               unsigned long long* keys, uint32_t* labs, long long* out, hipStream_t st);

int device_cu_count();

}  // namespace bqg
