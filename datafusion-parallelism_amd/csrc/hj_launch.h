// hj_launch.h — host-callable launchers of the gfx950 kernels (implemented in
// hj_kernels.hip). Every launcher is asynchronous on `stream` and returns the
// hipError_t of its launches.
#pragma once
#include <hip/hip_runtime.h>
#include "hj_device.h"

namespace dfp {

// ---- build ---------------------------------------------------------------
constexpr int kMinBuildTile = 4096;  // build rows per histogram/scatter block, at least
constexpr int kMaxChunks = 131071;   // (chunks + 1) x tiles histogram; 2^28 buckets max

int64_t build_tiles(int64_t total, int cus);
int64_t build_tile_rows(int64_t total, int64_t ntiles);
// bytes of the scan scratch for a histogram of `len` u32
int64_t scan_scratch_bytes(int64_t len);

constexpr int kCoarseBins = 128;     // level-1 partition groups (per-wave LDS copies)
constexpr int kMaxLevel1Bins = 2048; // level-1 bins of the one-level dense partition
// Dense tables whose key range spans <= 2048 blocks of 2^kDenseBlockShift chunks (2048
// values each, i.e. <= 16.7 M values) are partitioned in one level, by block.
constexpr uint32_t kDenseBlockShift = 2;
uint32_t dense_blocks(uint32_t nchunks);
bool dense_one_level(uint32_t nchunks);

// scratch: hist u32[(nchunks + 1) * ntiles], hist1 u32[kCoarseBins * ntiles],
// chunk_starts u32[nchunks + 2],
// scan_scratch scan_scratch_bytes((nchunks + 1) * ntiles), tkeys/skeys u64[total],
// trows/srows u32[total]
hipError_t launch_build(int key_bytes, const Segment* d_segs, int nseg, int64_t total,
                        const ChunkGeom& g, uint32_t* hist, uint32_t* hist1, uint32_t* chunk_starts,
                        int64_t ntiles, int64_t tile_rows, void* scan_scratch,
                        unsigned long long* tkeys, uint32_t* trows, unsigned long long* skeys,
                        uint32_t* srows, uint64_t* row_ids, bool ids_as_rows, Bucket* tbl,
                        uint32_t* dense, uint32_t* dup_rows, BigSeg* big, BuildCounters* ctr,
                        int big_grid, hipStream_t s);
// Dense builds of <= 2047 blocks and <= 2048 tiles of 16384 rows (one tile range per
// segment): the sliced probe's tile-local partition, then one workgroup per block gathers
// its rows from the tiles' fragments (no histogram, scan or global scatter).
// scratch: frag_build_scratch_bytes; tile_base: u32[ftiles], the first row of each tile
// (written by the partition); ids32: the
// explicit ids in row order (ids_as_rows) or NULL
constexpr int64_t kFragTileRows = 16384;  // = the sliced probe's tile
int64_t frag_build_tiles(const int64_t* seg_n, int nseg, int tile_log = 14);
// tile log of the hashed frag build's tiles (15 by default, DFP_HJ_HB_TILE_LOG=14)
int hashed_build_tile_log();
bool frag_build_ok(const ChunkGeom& g, int64_t ftiles);
int64_t frag_build_scratch_bytes(const ChunkGeom& g, int64_t ftiles, int64_t total);
hipError_t launch_build_frag(int key_bytes, const Segment* h_segs, int nseg, const ChunkGeom& g, int64_t ftiles,
                             void* scratch, uint32_t* tile_base, const uint64_t* ids32, uint32_t* dense,
                             uint32_t* dup_rows, BigSeg* big, BuildCounters* ctr, const Segment* d_segs, int64_t total,
                             bool ids_as_rows, int big_grid, const SpecGeo& spec, hipStream_t s);
// Hashed builds of chunks <= 1024 buckets and <= kFragMaxTiles tiles: the probe's hashed
// partition on the build keys (1024-bucket slices, passes of <= 2047 slices), then one
// workgroup per slice gathers its rows from the tiles' fragments and builds the slice's
// chunks in LDS. scratch: hashed_frag_scratch_bytes; tile_base u32[ftiles]. Sets ctr->err
// like launch_build when a chunk overflows (the caller rebuilds at half load).
bool hashed_frag_ok(const ChunkGeom& g, int64_t ftiles);
int64_t hashed_frag_scratch_bytes(const ChunkGeom& g, int64_t ftiles, int64_t total);
hipError_t launch_build_hashed_frag(int key_bytes, const Segment* h_segs, int nseg, const ChunkGeom& g, int64_t ftiles,
                                    void* scratch, uint32_t* tile_base, const uint64_t* ids32, Bucket* tbl,
                                    uint32_t* dup_rows, BigSeg* big, BuildCounters* ctr, const Segment* d_segs,
                                    int64_t total, bool ids_as_rows, int cus, hipStream_t s);
// min and max of the valid keys of the build segments -> out[0], out[1] (int64);
// out holds 2 + 2 * kMinmaxMaxBlocks int64 (per-block partials behind the result);
// mbox (optional, fine-grained host memory): min, max, then seq stored with system-scope
// release once both are visible
// Up to kArgSegs segments travel as a kernel argument: the kernel's first block then
// stores them to d_segs and zeroes *ctr (no H2D copy or memset launches before the build);
// with more, the caller copies d_segs and zeroes ctr itself and passes ctr = nullptr.
constexpr int kMinmaxMaxBlocks = 4096;
constexpr int kArgSegs = 16;
struct SegArgs {
    Segment s[kArgSegs];
};
hipError_t launch_key_minmax(int key_bytes, const Segment* h_segs, Segment* d_segs, int nseg, BuildCounters* ctr,
                             int64_t total, int64_t* out, int64_t* mbox, int64_t seq, hipStream_t s);
// the same reduction in one launch (hj_key_minmax): blocks fold into accumulator words
// with atomics and the last ticket writes the result to out[0..1] and res[0..1]; done:
// three words, zero before the launch and left zero after it
hipError_t launch_key_minmax_one(int key_bytes, const Segment* h_segs, Segment* d_segs, int nseg, BuildCounters* ctr,
                                 int64_t total, int64_t* out, unsigned long long* done, int64_t* mbox, int64_t seq,
                                 hipStream_t s, int64_t* res = nullptr);

// ---- probe ---------------------------------------------------------------
// 0 auto, 3 fused, 4 sliced
void set_probe_mode(int mode);
int get_probe_mode();
// probe tile log of the sliced probe: 0 auto (14 dense, 15 hashed), 14 or 15; returns the previous setting
int set_probe_tile_log(int tl);
int64_t probe_tiles(int64_t n);
int64_t probe_workspace(int64_t n);
// workspace: [0,8) unused, [8,16) error word, then tile counts/offsets, then per-row refs
// built (nullable): the table's build-complete event, waited on by `s` before the first
// kernel that reads the table — the sliced probe partitions and regroups its rows first,
// so a build still running on another stream overlaps them
hipError_t launch_probe(int key_bytes, const TableView& tv, const void* keys, const uint8_t* valid,
                        int64_t voff, const uint32_t* probe_ids, uint32_t probe_base, int64_t n, uint64_t* out_b,
                        uint32_t* out_p, int64_t cap, int64_t* d_total, void* workspace,
                        hipEvent_t built, hipStream_t s);

// ---- table queries -------------------------------------------------------
// refs[v] of a duplicated key (bit 31, not kMiss): offset field (mask) + base, v < n
hipError_t launch_dense_rebase(uint32_t* refs, uint64_t n, uint32_t base, uint32_t mask, hipStream_t s);
hipError_t launch_table_stats(const TableView& tv,
                              unsigned long long* out /* [4]: distinct, dupkeys, duprows, maxrows */,
                              hipStream_t s);
hipError_t launch_chain_links(const TableView& tv, int64_t* prev, int64_t nrows, hipStream_t s);

// ---- multi-GPU radix partition -------------------------------------------
// Destination map of a row: keys outside [lo, hi] are dropped (runtime min/max filter);
// by_range: part = umulhi(key - lo, mul) with mul = floor(2^64 * nparts / (hi - lo + 1))
// (contiguous key ranges), else the low bits of mix64(key).
struct PartSpec {
    int64_t lo, hi;
    uint64_t mul;
    int by_range;
};
hipError_t launch_radix_partition(int key_bytes, const void* keys, const uint8_t* valid,
                                  int64_t voff, const uint64_t* ids, uint64_t id_base,
                                  int64_t n, int nparts, const PartSpec& spec, void* out_keys,
                                  int out_key_bytes, int64_t key_offset, void* out_ids, int id_bytes,
                                  int64_t* counts, void* workspace, hipStream_t s);
int64_t radix_partition_workspace(int64_t n, int nparts);
// One-pass stable partition into per-destination regions: region d holds its rows at
// out[d * cap + i]; counts[d] = the destination's rows (all of them, even past cap: rows
// beyond cap are not written). Workspace: radix_regions_workspace (zeroed here); its
// word at byte 8 is the look-back's error flag.
int64_t radix_regions_workspace(int64_t n, int nparts);
hipError_t launch_radix_regions(int key_bytes, const void* keys, const uint8_t* valid, int64_t voff,
                                const uint64_t* ids, uint64_t id_base, int64_t n, int nparts, const PartSpec& spec,
                                void* out_keys, int out_key_bytes, int64_t key_offset, void* out_ids, int id_bytes,
                                int64_t cap, int64_t* counts, void* workspace, hipStream_t s);

// in-place exclusive scan of u64 (scratch: scan_scratch_bytes(len)); *total = sum
hipError_t launch_scan_u64(unsigned long long* a, int64_t len, void* scratch, unsigned long long* total,
                           hipStream_t s);

// ---- join-type and output primitives (hj_columns.hip) ----------------------
hipError_t launch_mark_rows(const void* idx, int idx_bytes, int64_t n, uint8_t* flags, int64_t nflags,
                            hipStream_t s);
int64_t select_workspace(int64_t n);
hipError_t launch_select_rows(const uint8_t* flags, int64_t n, uint8_t want, uint64_t* out, int64_t* d_count,
                              void* workspace, hipStream_t s);
hipError_t launch_gather_fixed(const void* src, const uint8_t* src_valid, int64_t src_voff, int elem_bytes,
                               const void* idx, int idx_bytes, int64_t n, void* dst, uint8_t* dst_valid,
                               hipStream_t s);
int64_t gather_var_workspace(int64_t n);
hipError_t launch_gather_var(const void* offsets, int offset_bytes, const uint8_t* values, const uint8_t* src_valid,
                             int64_t src_voff, const void* idx, int idx_bytes, int64_t n, void* out_offsets,
                             uint8_t* out_values, int64_t values_cap, uint8_t* dst_valid, int64_t* d_values_len,
                             void* workspace, hipStream_t s);

// ---- multi-GPU table helpers (hj_columns.hip) -------------------------------
hipError_t launch_iota_u32(uint32_t* out, int64_t n, uint32_t base, hipStream_t s);
hipError_t launch_add_u32(uint32_t* a, int64_t n, uint32_t base, hipStream_t s);
hipError_t launch_widen_u32(const uint32_t* in, int64_t n, uint64_t* out, hipStream_t s);
// canonical order of shard pair streams whose probe rows are < nrows (see hj_columns.hip)
int64_t merge_pairs_workspace(int64_t nrows);
hipError_t launch_merge_pairs(const uint64_t* b, const uint32_t* p, int64_t m, int64_t nrows, uint64_t* out_b,
                              uint32_t* out_p, int64_t cap, void* ws, hipStream_t s);

// ---- composite keys (hj_keys.hip) -------------------------------------------
// A key column in device memory: fixed width (width 1/2/4/8/16) or variable width (width
// 0: int32 / int64 offsets + value bytes), optional LSB validity bitmap from bit voff.
struct KeyCol {
    const void* values;
    const void* offsets;
    const uint8_t* valid;
    int64_t voff;
    int width;
    int offset_bytes;
};
constexpr int kMaxKeyCols = 16;
struct KeyCols {
    KeyCol c[kMaxKeyCols];
    int n;
};
// out_keys[i] = hash of row i's key tuple; out_valid: ceil(n / 64) u64 words, bit i = no
// key column null at row i
hipError_t launch_composite_keys(const KeyCols& cols, int64_t n, int64_t* out_keys, uint64_t* out_valid,
                                 hipStream_t s);
int64_t equal_pairs_workspace(int64_t n);
hipError_t launch_equal_pairs(const KeyCols& bc, const KeyCols& pc, const uint64_t* bidx, const uint32_t* pidx,
                              int64_t n, uint64_t* out_b, uint32_t* out_p, int64_t* d_count, void* ws,
                              hipStream_t s);

// ---- generators ----------------------------------------------------------
hipError_t launch_gen_perm(int64_t* out, int64_t n, int64_t mul, int64_t range, hipStream_t s);
hipError_t launch_gen_uniform(int64_t* out, int64_t n, uint64_t seed, int64_t range,
                              hipStream_t s);

}  // namespace dfp
