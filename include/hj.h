/*
 * hj.h — C ABI of the MI355X-native parallel hash join (build + inner probe).
 *
 * This is the drop-in boundary for the hot path of jamesfer/datafusion-parallelism
 * (paths below are relative to that repository). Every entry point names the
 * reference interface it replaces. Plain pointers and sizes only; no torch or HIP
 * types appear here (a stream is an opaque `void*` that is a hipStream_t, NULL =
 * the null stream).
 *
 * Semantics (canonical parity contract):
 *   * build_row_idx  = position of the row in the concatenation of all appended
 *                      build rows in (partition 0 appends in order, partition 1, ...)
 *                      order; or the caller's explicit id when `ids` is given.
 *   * probe_row_idx  = position of the row inside the probe call (the reference's
 *                      per-batch u32 index, src/shared/shared.rs:32-41).
 *   * pair order     = probe ascending, then build index DESCENDING within a probe
 *                      row (the reference's newest-first chain order at parallelism 1,
 *                      src/utils/concurrent_self_hash_join_map.rs:223-249).
 *   * null keys never match (src/shared/datafusion_private.rs:18-38 with
 *     null_equals_null = false, src/operator/probe_lookup_implementation/inner.rs:101-108).
 *   * pairs are those of get_matching_indices + equal_rows_arr
 *     (src/shared/shared.rs:29-47, src/shared/datafusion_private.rs:40-80): exact key
 *     equality, independent of the hash function.
 */
#ifndef DFP_HJ_H
#define DFP_HJ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum hj_status {
    HJ_OK = 0,
    HJ_ERR_INVALID = 1,   /* bad argument / state (DataFusionError::Internal) */
    HJ_ERR_OOM = 2,       /* device allocation failed */
    HJ_ERR_HIP = 3,       /* HIP runtime error */
    HJ_ERR_RCCL = 4,      /* RCCL failure in a multi-process step (hj_comm_*, hj_dist_*) */
    HJ_ERR_CAPACITY = 5,  /* output buffer too small; *count holds the size needed */
    HJ_ERR_NO_DEVICE = 6  /* no GPU: the HIP path cannot run (there is no CPU fallback) */
} hj_status;

typedef enum hj_key_type { HJ_INT32 = 0, HJ_INT64 = 1 } hj_key_type;

/* flags for hj_build_append / hj_probe */
enum {
    HJ_INPUT_DEVICE = 1u << 0, /* pointers are device memory (else host memory, copied) */
    HJ_BORROW = 1u << 1,       /* device input is not copied: caller keeps it alive until
                                  hj_build_finish returns on every partition */
    HJ_OUTPUT_HOST = 1u << 2,  /* hj_probe: return pairs in host memory (else device) */
    HJ_IDS_U31 = 1u << 3,      /* hj_build_append: the explicit ids are < 2^31 and ascend in
                                  canonical row order; when every id batch says so the table
                                  stores the ids in place of row numbers (pairs carry them
                                  with no id gather at probe time) */
    HJ_BORROW_KEEP = 1u << 4   /* with HJ_BORROW: the caller keeps the buffers alive and
                                  unmodified until hj_table_free, so hj_build_finish may return
                                  before the device build is done (it stays ordered before
                                  every later use of the table) */
};

typedef struct hj_table hj_table; /* opaque, device resident */

/* Match pairs of one probe call (ProbeBuildIndices, src/shared/shared.rs:24-27).
 * Owned by the library; release with hj_pairs_free. */
typedef struct hj_pairs {
    uint64_t* build_idx;   /* UInt64 build indices (length count) */
    uint32_t* probe_idx;   /* UInt32 probe indices (length count) */
    int64_t count;
    int device_resident;   /* 1: pointers are device memory; 0: host memory */
} hj_pairs;

/* Build statistics, filled by hj_table_stats after the build barrier. */
typedef struct hj_table_stats {
    int64_t build_rows;     /* rows appended (incl. null rows) */
    int64_t inserted_rows;  /* non-null rows inserted */
    int64_t distinct_keys;  /* occupied slots */
    int64_t dup_keys;       /* keys with > 1 row */
    int64_t dup_rows;       /* rows belonging to keys with > 1 row */
    int64_t max_key_rows;   /* largest chain length */
    int64_t buckets;        /* 64-byte buckets of 5 slots (0: direct-addressed table) */
    int64_t table_bytes;    /* device bytes of the bucket / direct-addressed table */
    int64_t build_ns;       /* device time of the last build (HIP events) */
} hj_table_stats;

/* ---- library ------------------------------------------------------------ */

/* Last error text of the calling thread ("" if none). */
const char* hj_last_error(void);
/* Version string; "gfx950" code object target is baked in. */
const char* hj_version(void);
/* Number of visible GPUs (0 on a machine without one). */
int hj_device_count(void);

/* ---- build: replaces BuildImplementation::new / build_side
 *      (src/operator/build_implementation.rs:34-48, 50-112) and the v10 insert
 *      path (src/operator/version10/parallel_join_execution_state.rs:91-133,
 *      src/operator/version10/new_map_3/fixed_table.rs:560-672). ----------------- */

/* Create a table for `parallelism` build partitions on GPU `device`.
 * `expected_rows` sizes the staging (a hint; 0 is fine). */
hj_status hj_build_begin(int device, int parallelism, hj_key_type key_type,
                         int64_t expected_rows, hj_table** out);

/* Multi-GPU table plans (hj_build_begin_multi). */
enum { HJ_MULTI_AUTO = 0, HJ_MULTI_BROADCAST = 1, HJ_MULTI_RADIX = 2 };

/* A table whose shards live on the GPUs `devices[0..ngpu)` (repeats allowed), behind the
 * same append / finish / probe / pairs / free ABI as a one-GPU table: the drop-in for a
 * process that drives a node of GPUs, as the reference's one process drives its
 * `parallelism` partitions. plan HJ_MULTI_BROADCAST: every GPU builds the whole build
 * side and a probe batch is split into contiguous row ranges, one per GPU (cheaper while
 * build rows x GPUs < build + probe rows); HJ_MULTI_RADIX (ngpu a power
 * of two <= 64): the build side is sharded by key hash (the hj_partition_rows map), a
 * probe batch is partitioned the same way, every piece probed by its owner over
 * device-to-device copies, and the pieces' pairs merged back into canonical order;
 * HJ_MULTI_AUTO: broadcast for build sides up to 2^27 rows, else radix. Pairs carry
 * global canonical build ids exactly as a one-GPU table's. Probes of a multi table run on
 * `stream` and the keys' device and return after the device work (the host reads the
 * pieces' sizes). hj_table_chain_links is not defined for multi tables. */
hj_status hj_build_begin_multi(int ngpu, const int* devices, int parallelism, hj_key_type key_type,
                               int64_t expected_rows, int plan, hj_table** out);

/* Append one build batch of partition `partition` (one RecordBatch's key column).
 * keys: int32/int64 values; validity: Arrow LSB bitmap (NULL = all valid) starting at
 * bit `validity_offset`; ids: optional explicit build ids (NULL = canonical numbering).
 * stream: the stream on which device input is produced (NULL = the null stream); the
 * build waits for the work enqueued on it up to this call.
 * Thread-safe: one caller per partition, partitions concurrently
 * (JoinStateInstance::add, version10/parallel_join_execution_state.rs:91-133). */
hj_status hj_build_append(hj_table* t, int partition, const void* keys,
                          const uint8_t* validity, int64_t validity_offset,
                          const uint64_t* ids, int64_t n, uint32_t flags, void* stream);

/* Barrier: every one of the `parallelism` partitions calls this once. The last
 * arriver runs the device build (InitializeLast::initialize_or_wait,
 * src/utils/initialize_last.rs:26-43); the others block until it is done. After it
 * returns the table is read-only and may be probed concurrently. A direct-addressed
 * build runs on asynchronously when no input was borrowed without HJ_BORROW_KEEP: every
 * later call on the table (probe, lookup, stats) waits for it on the device, and
 * hj_table_stream_wait orders any other stream after it. With the key range left on the
 * device (the default speculative build; DFP_HJ_SPEC_BUILD=0 turns it off) the layout is
 * settled by the first call that uses the table: a build side whose key range takes the
 * hashed layout is built then, so an error of that build (HJ_ERR_OOM, ...) is returned by
 * that call and by every later one. */
hj_status hj_build_finish(hj_table* t, int partition);

/* Optional, before the barrier: every valid build key lies in [key_lo, key_hi] (the caller
 * knows the range, e.g. from an exchange plan's global min/max). The build then skips its
 * key-range reduction and the host's wait for it, and takes its layout from this range
 * (direct-addressed when it spans at most 8x the build rows). The caller's guarantee is the
 * contract and is not checked on the device: a valid build key outside [key_lo, key_hi]
 * is UNDEFINED BEHAVIOUR (the direct-addressed build indexes its histograms and the table
 * by key - key_lo, so such a key can write out of bounds). Pass a range derived from the
 * keys themselves (hj_key_minmax, or an exchange plan's global min/max). New (the
 * reference sizes its table from the row count, new_map_3.rs:162). */
hj_status hj_build_key_range(hj_table* t, int64_t key_lo, int64_t key_hi);

/* Optional, after hj_build_key_range and before the barrier: the table takes the
 * direct-addressed layout over that key range whatever its density (a sparse piece of the
 * sharded-build plan still exports refs, hj_table_dense_export). The range must fit the
 * direct-addressed layout (< 2^28 values). */
hj_status hj_build_dense(hj_table* t);

/* The build keys (an HJ_INT32 table) are int32 offsets v from key_base: the table is keyed
 * by key_base + v in the int64 domain, and once built it takes int64 keys in every probe
 * and lookup. Only a direct-addressed table can be re-keyed this way (it stores no keys,
 * only refs indexed by key - min): a build whose key range exceeds 8 x its rows fails with
 * HJ_ERR_INVALID. The broadcast-build plan gathers 4-byte offsets instead of 8-byte keys
 * with it (half the exchange bytes, half the build's key reads) and probes the original
 * int64 keys. Before the barrier; not for multi-GPU tables. */
hj_status hj_build_key_base(hj_table* t, int64_t key_base);

/* Sharded-build broadcast plan (multi-GPU, a direct-addressed build domain): every rank
 * builds the table of its own contiguous key range from the build rows the radix exchange
 * brought it, the ranks all-gather those pieces into one table, and each probes its own
 * probe rows against it (no probe-side exchange, no replicated build). Replaces, for the
 * multi-GPU case, the one shared table every partition probes
 * (version10/parallel_join_execution_state.rs:405-407, lookup_implementation_3.rs:6-21).
 *
 * hj_table_dense_piece: a finished direct-addressed table's arrays, for the gather: refs
 * (one u32 per key value from *key_min, *nvalues of them: a build row id, kMiss =
 * 0xFFFFFFFF, or bit 31 + the offset of a duplicated key's segment [count, rows
 * descending] in *dup_rows), a device pointer to the number of u32 words of *dup_rows in
 * use (u64, final when the build is), and *packed (refs carry counts <= 15 in bits 27-30,
 * offsets in bits 0-26; else offsets in bits 0-30). HJ_ERR_INVALID for a hashed table. */
hj_status hj_table_dense_piece(const hj_table* t, uint32_t** refs, uint64_t* nvalues, int64_t* key_min,
                               uint32_t** dup_rows, const uint64_t** dup_used, int* packed);

/* Copies of a direct-addressed table's arrays on `stream` (any null destination is
 * skipped): refs [v0, v0 + n) to refs_dst, the first dup_n words of its segment array to
 * dup_dst, and the number of segment words in use (u64) to dup_used_dst — device
 * pointers, the gather's send buffers. */
hj_status hj_table_dense_export(const hj_table* t, uint32_t* refs_dst, uint64_t v0, uint64_t n, uint32_t* dup_dst,
                                uint64_t dup_n, uint64_t* dup_used_dst, void* stream);

/* A finished, probe-only direct-addressed table over caller-owned device arrays (borrowed
 * until hj_table_free; the library frees nothing of them): refs[v] for key key_min + v,
 * v < nvalues, in the layout hj_table_dense_piece describes, and the segments they point
 * into. The arrays are ready in `stream` order; probes on other streams wait for that
 * point. Probes take keys of probe_key_type. */
hj_status hj_table_wrap_dense(int device, hj_key_type probe_key_type, int64_t key_min, uint64_t nvalues,
                              const uint32_t* refs, const uint32_t* dup_rows, int packed, void* stream,
                              hj_table** out);

/* refs[v] += base in the offset field of every duplicated-key ref (bit 31 set, not kMiss),
 * v < n, on `stream`: a gathered piece's refs re-pointed at its segments' place in the
 * concatenated segment array. The caller keeps every offset + base below 2^27 (packed) or
 * 2^31. */
hj_status hj_dense_rebase_dups(uint32_t* refs, uint64_t n, uint32_t base, int packed, void* stream);

/* Canonical id of partition `partition`'s first row (valid after the barrier). */
hj_status hj_build_partition_offset(const hj_table* t, int partition, int64_t* out);

hj_status hj_table_stats_get(const hj_table* t, hj_table_stats* out);

/* Device time of the build (HIP events around clear + insert + duplicate passes), ns;
 * -1 if the table is not built. Cheap: no device work. */
int64_t hj_table_build_ns(const hj_table* t);

/* IndexLookup::get_iter (src/utils/index_lookup.rs:1-6,
 * src/operator/version10/lookup_implementation_3.rs:46-59): build rows of `key` in
 * chain order (newest first = descending). Writes up to `cap` rows, *count = total. */
hj_status hj_table_lookup(const hj_table* t, int64_t key, uint64_t* rows, int64_t cap,
                          int64_t* count);

/* Chain links in canonical form: prev[i] = next older build row with the same key as
 * row i, or -1 (the reference's overflow buffer at parallelism 1, minus 1;
 * src/operator/version10/parallel_join_execution_state.rs:91-133). Host array of
 * build_rows entries. */
hj_status hj_table_chain_links(const hj_table* t, int64_t* prev, int64_t n);

/* Waits for the table's build and its latest probe launch, then releases its memory
 * (probes still running on other streams must be finished by the caller first). */
void hj_table_free(hj_table* t);

/* ---- probe: replaces get_matching_indices + equal_rows_arr inside
 *      lookup_inner_join_probe_batch (src/operator/probe_lookup_implementation/
 *      inner.rs:79-129, src/shared/shared.rs:29-47,
 *      src/shared/datafusion_private.rs:40-80). -------------------------------- */

/* Synchronous, reentrant probe of a finished table, run on `stream` (NULL = the null
 * stream; device input must be ready in that stream's order). Pairs are library-owned. */
hj_status hj_probe(const hj_table* t, const void* keys, const uint8_t* validity,
                   int64_t validity_offset, int64_t n, uint32_t flags, void* stream,
                   hj_pairs* out);

void hj_pairs_free(hj_pairs* p);

/* Asynchronous probe into caller buffers (device memory), on `stream`.
 * Writes min(total, capacity) pairs and the total to *d_total (device int64).
 * `workspace` (device, 8-byte aligned, hj_probe_workspace_bytes(n) bytes) must not be
 * shared by concurrent calls; its bytes 8..15 (uint64) are non-zero after the call if
 * the fused probe's bounded look-back spin gave up (results invalid; never observed).
 * No host synchronisation, no allocation. A table built on another stream needs no
 * wait from the caller: the probe orders itself after the build at its first table read
 * (the sliced probe partitions its rows first, overlapping the build). */
int64_t hj_probe_workspace_bytes(int64_t n);
hj_status hj_probe_async(const hj_table* t, const void* keys, const uint8_t* validity,
                         int64_t validity_offset, int64_t n, uint64_t* out_build,
                         uint32_t* out_probe, int64_t capacity, int64_t* d_total,
                         void* workspace, void* stream);

/* As hj_probe_async, but probe_idx of a match is probe_ids[row] instead of row
 * (rows received through the multi-GPU exchange carry their global ids). */
hj_status hj_probe_async_ids(const hj_table* t, const void* keys, const uint8_t* validity,
                             int64_t validity_offset, const uint32_t* probe_ids, int64_t n,
                             uint64_t* out_build, uint32_t* out_probe, int64_t capacity,
                             int64_t* d_total, void* workspace, void* stream);

/* As hj_probe_async, but probe_idx of a match is probe_base + row: the batch's rows are
 * rows probe_base .. probe_base + n - 1 of a longer probe stream (replaces the caller-side
 * offset of the batch-relative indices of ProbeBuildIndices, src/shared/shared.rs:29-47,
 * when a partition's batches or a rank's share of one batch are numbered globally - the
 * broadcast-build plan's contiguous probe ranges need no id array). probe_base + n must
 * not exceed 2^32. */
hj_status hj_probe_async_base(const hj_table* t, const void* keys, const uint8_t* validity,
                              int64_t validity_offset, int64_t n, uint32_t probe_base,
                              uint64_t* out_build, uint32_t* out_probe, int64_t capacity,
                              int64_t* d_total, void* workspace, void* stream);

/* Probe strategy for later probes of this process: 0 auto (sliced for tables past the L2s
 * - more than 2^20 key values or 2^16 buckets, at most 4 passes of 2047 slices - with a
 * probe side at least as large as the key range / bucket count, else fused),
 * 3 fused (lookup + emission in one launch, tile offsets by decoupled look-back),
 * 4 sliced (probe rows partitioned by slice - 32768 key values of a direct-addressed table
 * or 2048 buckets of a hashed one - lookups out of LDS, then ordered emission; a table of
 * more than 2047 slices is probed in passes over slice ranges, each pass partitioning the
 * probe rows of its range and looking them up, one emission at the end). Results are
 * identical;
 * returns the previous mode, -1 for a bad value (1 and 2 named strategies measured slower
 * and removed). Also settable with DFP_HJ_PROBE_MODE=fused|sliced. */
int hj_set_probe_mode(int mode);

/* Probe tiles of the sliced probe for later probes of this process: 0 auto (2^14 rows for
 * a direct-addressed table, 2^15 for a hashed one), 14 or 15 (rows per tile = 2^tile_log).
 * A longer tile halves the (tile, slice) fragments the lookups walk; results are identical.
 * Returns the previous setting, -1 for a bad value. Also settable with
 * DFP_HJ_SL_TILE_LOG=14|15. The tiles are the probe's own work units (no reference
 * counterpart: the reference probes each RecordBatch row by row, lookup_implementation_3.rs). */
int hj_set_probe_tile_log(int tile_log);

/* Table layout for later builds of this process: 0 auto (a direct-addressed table - one
 * u32 ref per key value - when the build keys' range is at most 8x the build rows, the
 * "perfect hash" of dense integer keys; else 5-slot hashed buckets), 1 hashed buckets
 * always, 2 as 0 but the build partitions its rows by histogram + scan + scatter (both
 * layouts) instead of the tile-local partition and per-slice LDS build from its
 * fragments. Results are identical; returns the previous mode, -1 for a bad value. Also
 * settable with DFP_HJ_DENSE=0 (hashed) and DFP_HJ_FRAG_BUILD=0 (mode 2). */
int hj_set_build_mode(int mode);

/* Per-table device budget for later builds of this process, in bytes (0 = none; also
 * DFP_HJ_DEVICE_BUDGET_BYTES). A one-device table whose build would hold more device
 * memory than this - staged input copies, the table, duplicate segments and the build's
 * scratch - fails its hj_build_append / hj_build_finish with HJ_ERR_OOM ("device budget"),
 * so that a planner can shard the build over several GPUs instead (hj_build_begin_multi,
 * HJ_MULTI_RADIX: every shard is a one-device table of about 1/G of the build, each under
 * the budget). It stands in for one GPU's HBM capacity when a build side larger than one
 * GPU (BASELINE configs[4], the reference's SF300 Q9 on 8 GPUs) is rehearsed at a smaller
 * scale. Returns the previous budget. New (the reference's CPU build grows its tables
 * without bound, new_map_3.rs:325-411). */
int64_t hj_set_device_budget(int64_t bytes);

/* Peak device bytes a built table held during its build (the budget's measure); for a
 * multi-GPU table, the largest shard's. */
hj_status hj_table_device_bytes(const hj_table* t, int64_t* peak_per_device);

/* Makes `stream` wait for the build of `t` (for probes on other streams). */
hj_status hj_table_stream_wait(const hj_table* t, void* stream);

/* ---- radix partitioning for the multi-GPU exchange (new; the reference's nearest
 *      relative is the shard function of
 *      src/utils/partitioned_concurrent_self_hash_join_map.rs:13-16). ------------ */

/* Partition n rows into `nparts` (power of two) by hash bits of the key:
 * out_keys/out_ids are grouped by destination (stable); counts[nparts] (device int64)
 * receives the rows per destination. ids may be NULL (then id = id_base + i); out_ids
 * holds uint64 (id_bytes 8, build rows) or uint32 (id_bytes 4, probe rows: the
 * reference's UInt32 probe indices) ids. out_key_bytes 4 with int64 keys writes
 * int32(key - key_offset) (the caller guarantees the range; a bijection, so the join is
 * unchanged and the exchange moves 4 bytes per key). Null rows are dropped. Device
 * pointers, asynchronous on `stream`; `workspace` of hj_partition_workspace_bytes(n,
 * nparts) bytes. */
int64_t hj_partition_workspace_bytes(int64_t n, int nparts);
hj_status hj_radix_partition(hj_key_type key_type, const void* keys,
                             const uint8_t* validity, int64_t validity_offset,
                             const uint64_t* ids, uint64_t id_base, int64_t n, int nparts,
                             void* out_keys, int out_key_bytes, int64_t key_offset,
                             void* out_ids, int id_bytes, int64_t* counts,
                             void* workspace, void* stream);

/* Destination map and runtime filter of hj_partition_rows. Rows whose key lies outside
 * [key_lo, key_hi] are dropped like null rows: an inner join's probe row outside the
 * global build key range cannot match (a min/max runtime filter ahead of the exchange).
 * by_range 1: destination = (key - key_lo) * nparts / (key_hi - key_lo + 1) (fixed point,
 * floor(2^64 * nparts / range) multiply-high), i.e. contiguous key ranges, so a dense
 * global key domain gives every rank a dense local one; by_range 0: the hash map of
 * hj_radix_partition. Both sides of one join must use the same spec. */
typedef struct hj_part_spec {
    int by_range;
    int64_t key_lo;
    int64_t key_hi;
} hj_part_spec;

/* hj_radix_partition with a spec (NULL: hash map, no filter). */
hj_status hj_partition_rows(hj_key_type key_type, const void* keys,
                            const uint8_t* validity, int64_t validity_offset,
                            const uint64_t* ids, uint64_t id_base, int64_t n, int nparts,
                            const hj_part_spec* spec, void* out_keys, int out_key_bytes,
                            int64_t key_offset, void* out_ids, int id_bytes, int64_t* counts,
                            void* workspace, void* stream);

/* One-pass partition into per-destination regions (the exchange's send buffers): the
 * rows of destination d go to out_keys / out_ids elements [d * region_rows, d *
 * region_rows + counts[d]) in source row order (stable), with hj_partition_rows' map,
 * filter, key narrowing and ids. Every row is read once (a decoupled look-back over the
 * tiles gives each tile's offset in each region), and a region is a contiguous send
 * buffer for one peer, so no grouped copy precedes the exchange. counts[d] is exact even
 * when it exceeds region_rows (rows past the region are not written): region_rows >= n
 * always suffices. workspace: hj_partition_regions_workspace_bytes(n, nparts).
 * Failure on the device: a tile whose look-back wait exceeds its spin limit (never
 * expected) sets the error word (workspace bytes 8..15) and makes every affected count
 * >= 2^60, so a caller that reads the counts for its exchange must treat any count above
 * n as an error (the Python plans raise HJ_ERR_HIP); the output is then invalid. */
int64_t hj_partition_regions_workspace_bytes(int64_t n, int nparts);
hj_status hj_partition_regions(hj_key_type key_type, const void* keys,
                               const uint8_t* validity, int64_t validity_offset,
                               const uint64_t* ids, uint64_t id_base, int64_t n, int nparts,
                               const hj_part_spec* spec, void* out_keys, int out_key_bytes,
                               int64_t key_offset, void* out_ids, int id_bytes, int64_t region_rows,
                               int64_t* counts, void* workspace, void* stream);

/* Key range of one column, one kernel launch, asynchronous on `stream`: out_minmax[0] =
 * min, out_minmax[1] = max of the valid keys (INT64_MAX, INT64_MIN when there are none;
 * out_minmax is device memory). The radix plan's prepare step (DistributedHashJoin.prepare:
 * runtime filter bounds, range map and key narrowing from the global build key range,
 * the range the reference's partitioned map spreads keys over,
 * src/utils/partitioned_concurrent_self_hash_join_map.rs:13-16) and the build's key-range
 * reduction share this kernel. workspace: hj_key_minmax_workspace_bytes() bytes, 8-byte
 * aligned (the call re-arms it: no caller initialisation). */
int64_t hj_key_minmax_workspace_bytes(void);
hj_status hj_key_minmax(hj_key_type key_type, const void* keys, const uint8_t* validity,
                        int64_t validity_offset, int64_t n, int64_t* out_minmax, void* workspace,
                        void* stream);

/* ---- join types and output materialisation. Device pointers,
 *      asynchronous on `stream`. Index arrays are uint32 (idx_bytes 4) or uint64 (8);
 *      an all-ones index is a null index (the outer joins' missing side). ---------- */

/* flags[idx[i]] = 1 for every idx[i] < nflags: ConcurrentBitSet::set_ones on matched
 * build indices (src/utils/concurrent_bit_set.rs:28-60, used by
 * src/operator/probe_lookup_implementation/{left_semi,left_anti,left_outer,full}.rs) and
 * the matched-probe bitmap of get_semi_indices / get_anti_indices
 * (src/shared/datafusion_private.rs:85-135). */
hj_status hj_mark_rows(const void* idx, int idx_bytes, int64_t n, uint8_t* flags, int64_t nflags,
                       void* stream);

/* Ascending positions i < n with flags[i] == want into out (capacity n), count to
 * *d_count (device int64): get_set_indices_array / get_unset_indices_array and
 * get_semi_indices / get_anti_indices. workspace: hj_select_workspace_bytes(n). */
int64_t hj_select_workspace_bytes(int64_t n);
hj_status hj_select_rows(const uint8_t* flags, int64_t n, int want, uint64_t* out,
                         int64_t* d_count, void* workspace, void* stream);

/* Arrow take of a fixed-width column (elem_bytes 1/2/4/8/16) by indices:
 * dst[i] = src[idx[i]]; dst_valid (optional, 8-byte aligned, ceil(n/64)*8 bytes) gets
 * bit i = index not null and source row valid. take_multiple_record_batch
 * (src/shared/shared.rs:83-92). */
hj_status hj_gather_fixed(const void* src, const uint8_t* src_valid, int64_t src_voff,
                          int elem_bytes, const void* idx, int idx_bytes, int64_t n, void* dst,
                          uint8_t* dst_valid, void* stream);

/* Arrow take of a Utf8/Binary (offset_bytes 4) or LargeUtf8/LargeBinary (8) column:
 * out_offsets[n + 1], out_values (capacity values_cap bytes), dst_valid as above;
 * *d_values_len (device int64) = bytes needed (values beyond values_cap are not
 * written: retry with a larger buffer). workspace: hj_gather_var_workspace_bytes(n). */
int64_t hj_gather_var_workspace_bytes(int64_t n);
hj_status hj_gather_var(const void* offsets, int offset_bytes, const uint8_t* values,
                        const uint8_t* src_valid, int64_t src_voff, const void* idx, int idx_bytes,
                        int64_t n, void* out_offsets, uint8_t* out_values, int64_t values_cap,
                        uint8_t* dst_valid, int64_t* d_values_len, void* workspace, void* stream);

/* ---- join keys of several columns, or of non-integer types (SURVEY.md §8a a2/a12:
 *      calculate_hash over every key column, src/shared/shared.rs:11-16, and the
 *      equality re-check equal_rows_arr, src/shared/datafusion_private.rs:52-73). ------
 * Flow: hj_composite_keys on each build batch -> hj_build_append(HJ_INT64 keys, the
 * composite validity); hj_composite_keys on a probe batch -> hj_probe* -> candidate
 * pairs -> hj_filter_equal_pairs -> the join's pairs (canonical order kept). A single
 * Int32/Int64 key column needs none of this (the table compares exact keys). */

/* One key column in device memory. Fixed width: width 1, 2, 4, 8 or 16 bytes, values
 * row-major. Variable width (Utf8 / Binary / LargeUtf8 / LargeBinary): width 0, offsets
 * (offset_bytes 4 or 8, n + 1 entries) into the value bytes. validity: Arrow LSB bitmap
 * (NULL = all valid) from bit validity_offset. Values compare byte-exactly (arrow's eq;
 * for floats its total order, i.e. equal bits). */
typedef struct hj_key_column {
    const void* values;
    const void* offsets;
    const uint8_t* validity;
    int64_t validity_offset;
    int width;
    int offset_bytes;
} hj_key_column;

/* out_keys[i] (device int64) = a 64-bit hash of row i's key tuple over the `ncols`
 * (<= 16) columns; out_valid (device, 8-byte aligned, ceil(n / 64) * 8 bytes) bit i = no
 * key column is null at row i (a null key never matches). Asynchronous on `stream`. */
hj_status hj_composite_keys(int ncols, const hj_key_column* cols, int64_t n, int64_t* out_keys,
                            uint8_t* out_valid, void* stream);

/* Keep the candidate pairs (build_idx[i], probe_idx[i]) whose key tuples are equal in
 * every column, in order: out_build / out_probe (capacity n, distinct from the inputs)
 * receive them and *d_count (device int64) their number. build_cols index the build
 * side's concatenated rows, probe_cols the probe batch's rows. workspace:
 * hj_equal_pairs_workspace_bytes(n). Asynchronous on `stream`. */
int64_t hj_equal_pairs_workspace_bytes(int64_t n);
hj_status hj_filter_equal_pairs(int ncols, const hj_key_column* build_cols,
                                const hj_key_column* probe_cols, const uint64_t* build_idx,
                                const uint32_t* probe_idx, int64_t n, uint64_t* out_build,
                                uint32_t* out_probe, int64_t* d_count, void* workspace,
                                void* stream);

/* ---- multi-process, one GPU per process: RCCL behind the ABI --------------------
 * The reference runs one process; a node of GPUs driven as one process per GPU (the
 * Rust host launching a rank per device) needs the exchange steps of the multi-GPU plans
 * here, not in the host language. A communicator is RCCL's (ncclCommInitRank over xGMI);
 * its 128-byte unique id is made by one rank (hj_comm_unique_id) and handed to every rank
 * by the caller (any out-of-band channel: the launcher's store, a socket, an MPI bcast).
 * The radix precedent is the shard function of
 * src/utils/partitioned_concurrent_self_hash_join_map.rs:13-16; the operator seam that a
 * per-rank plan sits behind is BuildImplementation::build_side
 * (src/operator/build_implementation.rs:50-112). */
typedef struct hj_comm hj_comm;
#define HJ_COMM_ID_BYTES 128
hj_status hj_comm_unique_id(uint8_t id[HJ_COMM_ID_BYTES]);
/* Collective: every rank of `world` calls it with the same id; binds the communicator to
 * `device`. */
hj_status hj_comm_create(int rank, int world, const uint8_t id[HJ_COMM_ID_BYTES], int device,
                         hj_comm** out);
void hj_comm_free(hj_comm* c);

/* The multi-GPU plans run as JOBS on the communicator's worker thread: an entry point
 * below enqueues the job and returns; the job's host steps (its small reads of the plan,
 * the count matrices and segment sizes, each waiting for its own stream only) run on the
 * worker, in submission order, so the caller's thread never waits for them until it asks
 * for the job's result. Every rank submits the same sequence of jobs (the collectives
 * inside must match). Failures are collective: each host read carries every rank's status
 * word and the buffers later collectives need are sized before it, so a rank that fails
 * locally still completes the collectives and every rank's job returns an error (a peer's
 * failure as HJ_ERR_RCCL "a peer rank failed during ..."). The one exception is an
 * allocation failure of the radix plan's received probe rows (sized after the last status
 * exchange): that rank aborts the communicator (unusable afterwards; its peers' jobs then
 * fail in RCCL). Inputs must stay valid until the job's device work has finished (the
 * table's or the pairs' consumers wait for it). Call a communicator's entry points from one
 * thread at a time. A job's device work runs on the communicator's own streams, after the
 * work enqueued on the caller's `stream` before the call (its inputs must be complete
 * there); consumers wait for its results by themselves (a table's completion event, the
 * pairs' read). Two communicators of the same ranks may run jobs concurrently (a caller
 * that alternates steps between them overlaps one step's host reads with the next's): they
 * share no stream. New (the reference has no multi-process path; its partitions' builds
 * are concurrent futures, src/operator/parallel_hash_join_executor.rs:86-122). */
typedef struct hj_dist_job hj_dist_job;

typedef struct hj_dist_info {
    int64_t build_rows;  /* global build rows (the ranks' build_base + n, max) */
    int64_t recv_rows;   /* build rows this rank received and built */
    int sharded;         /* 1: sharded build / radix shard; 0: every rank built the whole build side */
} hj_dist_info;

/* The sharded-build plan's build side, one job per step on every rank.
 * Rank r holds build rows [build_base, build_base + n) of the global build column (the
 * ranks' ranges tile [0, B) in rank order); the job's table holds the WHOLE build side
 * and is probed by this rank's own probe rows with hj_probe_async_base(t, ..., probe_base,
 * ...): build_idx = global build row, probe_idx = probe_base + row, and the ranks' outputs
 * in rank order are the single-GPU canonical output. The table is keyed in
 * `probe_key_type` (the probe keys' width; int32 and int64 build keys may be probed by
 * either on a dense domain). Steps:
 *   1 global key range, build rows and statuses (hj_key_minmax, one grouped all-reduce);
 *   2 when the build key domain is dense (range <= 8 x rows, within the direct-addressed
 *     layout), with < 2^31 rows and a power-of-two world: every valid row to the rank that
 *     owns its contiguous key range (hj_partition_regions by range, keys as int32 offsets
 *     when the range spans < 2^32 values, global ids), the count matrix all-gathered, a
 *     point-to-point exchange (ncclSend/ncclRecv in one group);
 *   3 a direct-addressed build of the rank's own key range (global ids in place of rows),
 *     its refs all-gathered into one array over the whole domain, the duplicate segments
 *     all-gathered end to end and re-pointed (hj_dense_rebase_dups), wrapped as one
 *     probe-only table (hj_table_wrap_dense);
 *   otherwise (sparse domain, >= 2^31 rows, other worlds) every rank all-gathers the valid
 *   build rows with their global ids and builds the whole table (probe keys of the build
 *   key type then).
 * Probes on any stream wait for the table by themselves (hj_table_build_ns spans the whole
 * build side). Per-job scratch is released by a later job once its work has finished (or
 * at hj_comm_free). */
hj_status hj_dist_build_sharded_async(hj_comm* c, hj_key_type key_type, const void* keys,
                                      const uint8_t* validity, int64_t validity_offset, int64_t n,
                                      int64_t build_base, hj_key_type probe_key_type, void* stream,
                                      hj_dist_job** job);
/* The same, waiting for the job: -> the table (free it with hj_table_free). */
hj_status hj_dist_build_sharded(hj_comm* c, hj_key_type key_type, const void* keys,
                                const uint8_t* validity, int64_t validity_offset, int64_t n,
                                int64_t build_base, hj_key_type probe_key_type, void* stream,
                                hj_table** out, hj_dist_info* info);

/* The radix plan, one job per step on every rank (north_star's split: "the build side
 * radix-partitions ... RCCL all-to-all"; the shard function's precedent is
 * src/utils/partitioned_concurrent_self_hash_join_map.rs:13-16, its per-shard inserts
 * 263-281). Rank r holds build rows [build_base, build_base + nb) and probe rows
 * [probe_base, probe_base + np) of the global columns. Steps: the global build key range
 * (one all-reduce, one read) -> runtime filter (probe rows outside it do not travel),
 * contiguous key ranges per rank for a dense build domain (else mix64 hash bits), keys as
 * int32 offsets when the range spans < 2^32 values; both sides partitioned into
 * per-destination regions in one pass each; the build side's count matrix (one read), its
 * point-to-point exchange and the local build (the rank's key range given, global ids in
 * place of rows) on the communicator's streams; the probe side's count matrix (one read),
 * its exchange, and the probe of the received rows with their global u32 ids
 * (probe_base + np <= 2^32). The job's pairs (hj_dist_job_pairs) are this
 * rank's share of the join: probe rows in ascending global id, each probe row's build rows
 * in the canonical (descending) order; the ranks' shares together are the whole join
 * (a merge by probe id restores the single-GPU order). */
hj_status hj_dist_join_radix(hj_comm* c, hj_key_type build_key_type, const void* build_keys,
                             const uint8_t* build_validity, int64_t build_validity_offset,
                             int64_t nb, int64_t build_base, hj_key_type probe_key_type,
                             const void* probe_keys, const uint8_t* probe_validity,
                             int64_t probe_validity_offset, int64_t np, int64_t probe_base,
                             void* stream, hj_dist_job** job);

/* Relational exchanges for multi-GPU query plans (C4/C5: TPC-H Q3 / Q9 over 8 ranks; the
 * reference's TPC-H runner drives whole queries, tpc/src/main.rs:290-384, and its output
 * step is take_multiple_record_batch, src/shared/shared.rs:83-92). Jobs like the plans
 * above (same ordering, failure and lifetime rules); every rank submits the same sequence.
 *
 * hj_dist_shuffle: hash repartition (DataFusion's RepartitionExec Hash over the links) of a
 * key column with `ncols` fixed-width payload columns (col_bytes 1/2/4/8/16): row i goes to
 * rank (mix64 hash bits of keys[i], the hj_partition_rows map; a power-of-two world) with
 * its payload - two sides shuffled on the same key meet on one rank. Steps: the keys grouped
 * by destination (stable), each payload column gathered by that permutation, the count
 * matrix all-gathered with every rank's status (one host read), then keys and columns per
 * peer (ncclSend / ncclRecv in one group, messages above 256 MiB in pieces). The received
 * rows are ordered by (source rank, source row). One rank: the rows as they are.
 * hj_dist_gather: broadcast exchange - every rank receives the concatenation, in rank
 * order, of all ranks' rows of `ncols` columns (n rows on this rank): the small filtered
 * dimension sides of a plan and per-rank partial results (a sum over ranks = a gather of
 * one row per rank). The received buffers are allocated after the last status exchange: a
 * failed allocation aborts the communicator (as the radix plan's received probe rows). */
hj_status hj_dist_shuffle(hj_comm* c, hj_key_type key_type, const void* keys, int64_t n, int ncols,
                          const void* const* cols, const int* col_bytes, void* stream, hj_dist_job** job);
hj_status hj_dist_gather(hj_comm* c, int64_t n, int ncols, const void* const* cols, const int* col_bytes,
                         void* stream, hj_dist_job** job);
/* An exchange job's received rows: waits for the job's host steps and makes `stream` wait
 * for its device work; device pointers owned by the job (valid until hj_dist_job_free):
 * *keys (shuffle; NULL for a gather), cols[0 .. ncols) in the submitted order, *rows. */
hj_status hj_dist_job_columns(hj_dist_job* job, void* stream, const void** keys, const void** cols, int ncols,
                              int64_t* rows);

/* Wait for the job's host steps (not for its device work); its status and info. */
hj_status hj_dist_job_wait(hj_dist_job* job, hj_dist_info* info);
/* Wait and take the job's table (the sharded build side; the radix plan's local shard,
 * which a radix job's hj_dist_job_pairs re-probe then cannot use): the caller frees it. */
hj_status hj_dist_job_table(hj_dist_job* job, hj_table** out, hj_dist_info* info);
/* A radix job's pairs: waits for the probe, re-probes once with the exact size when the
 * matches exceeded the received probe rows; device pointers owned by the job (valid until
 * hj_dist_job_free). */
hj_status hj_dist_job_pairs(hj_dist_job* job, const uint64_t** build_idx, const uint32_t** probe_idx,
                            int64_t* count);
/* Device times of a finished job's stages (waits for them), ms: a radix job's build side
 * (plan to local build), exchange (the build side's exchange to the probe's start) and
 * probe; a sharded job's build side in build_ms (0 for the others). NULL outputs skipped. */
hj_status hj_dist_job_times(hj_dist_job* job, double* build_ms, double* exchange_ms, double* probe_ms);
/* Waits for the job (host steps and device work) and releases it and what it owns. */
void hj_dist_job_free(hj_dist_job* job);

/* ---- synthetic generators of SURVEY.md §8(d) on the device (bench inputs) ----- */
/* out[i] = (i * mul) mod range  (unique build keys when gcd(mul, range) = 1);
 * requires n * mul < 2^64 */
hj_status hj_gen_perm_keys(int64_t* out, int64_t n, int64_t mul, int64_t range,
                           void* stream);
/* out[i] = splitmix64(seed + i) mod range */
hj_status hj_gen_uniform_keys(int64_t* out, int64_t n, uint64_t seed, int64_t range,
                              void* stream);
/* HOST buffer out[0 .. hi - lo): make_exponential_int_array(lo, hi) of
 * src/api_utils.rs:15-23 (f32, libm powf as f32::powf); needs no GPU */
hj_status hj_gen_exponential_keys(int32_t* out, int32_t lo, int32_t hi);

#ifdef __cplusplus
}
#endif
#endif /* DFP_HJ_H */
