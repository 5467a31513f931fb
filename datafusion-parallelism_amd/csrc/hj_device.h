// hj_device.h — data layout shared by the gfx950 kernels (hj_kernels.hip) and the
// C-ABI host layer (hj_api.cpp).
//
// Slot table in HBM:
//   Bucket[nb + 1], one 64-byte line each, nb = nchunks << clog2:
//     uint64 key[5]   stored key = mix64(key) (a bijection of the 64-bit keys, so equal
//                     stored keys are equal keys, and the home bucket follows from the
//                     stored key without rehashing), 0 = empty slot
//     uint32 ref[5]   bit 31 clear: the key's only build row
//                     bit 31 set:   offset of its duplicate segment in dup_rows
//     uint32 meta     bit 0: an insert passed this bucket full (a lookup that misses
//                     here continues to the next bucket only if set);
//                     bits 1+6j..6+6j: row count of slot j's duplicated key if <= 63
//                     (0: read it from dup_rows);
//                     side bucket: rows of the key 0
//   A key's probe sequence stays inside its chunk of 2^clog2 buckets (linear probing
//   modulo the chunk), so one workgroup can build a whole chunk in LDS.
//   Bucket[nb] is the side bucket for key 0, whose stored form mix64(0) = 0 collides with
//   "empty": ref[0] + meta = row count.
//   dup_rows[]: per duplicated key a segment [count, row_0 > row_1 > ... ] — rows sorted
//   descending = the reference's newest-first chain order at parallelism 1.
//   row_ids[]: optional u64 explicit build ids (multi-GPU exchange).
//
// The reference's v10 table (src/operator/version10/new_map_3/fixed_table.rs:114-140)
// stores (hash|bit63, row+1) slots, a separate u8 tag array and an overflow chain array;
// this layout keeps the exact key in the slot (the equality re-check of equal_rows_arr,
// src/shared/datafusion_private.rs:40-80, needs no second gather) and replaces pointer
// chasing with one contiguous sorted segment per duplicated key.
#pragma once
#include <stdint.h>

namespace dfp {

constexpr uint64_t kSign = 0x8000000000000000ull;
constexpr int kSlots = 5;
constexpr unsigned kDupFlag = 0x80000000u;
constexpr unsigned kMiss = 0xFFFFFFFFu;
constexpr int kSmallSeg = 16;  // dup segments up to this size are sorted by one thread
constexpr unsigned kInlineCount = 63;           // dup row counts kept in the bucket's meta
constexpr unsigned kCountUnknown = 0xFFFFFFFFu;  // count not inline: read dup_rows[off]

struct alignas(64) Bucket {
    unsigned long long key[kSlots];
    unsigned int ref[kSlots];
    unsigned int meta;
};
static_assert(sizeof(Bucket) == 64, "bucket must be one 64-byte line");

// One appended build batch (after the barrier; row_base = canonical id of row 0).
struct Segment {
    const void* keys;
    const uint8_t* valid;
    int64_t voff;
    const uint64_t* ids;
    int64_t n;
    int64_t row_base;
};

// Device-side build counters (zeroed before every build).
struct BuildCounters {
    unsigned long long n_valid;      // non-null rows (scan total)
    unsigned long long dup_used;     // dup_rows entries allocated
    unsigned long long n_big;        // segments > kSmallSeg
    unsigned long long err;          // bit 0: chunk full; bit 1: chunk dup-directory full
    unsigned long long spill_used;   // fragment build: rows gathered for blocks past the registers
};

// a duplicate segment too large for one thread to sort
struct BigSeg {
    unsigned long long key;
    unsigned int off;
    unsigned int pad;
};

__host__ __device__ inline uint64_t mix64(uint64_t k) {
    // murmur3 fmix64: the GPU's own hash. Emitted pairs are independent of it because
    // candidates are re-filtered by exact key equality.
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// inverse of mix64 (xorshift by 33 is its own inverse on 64 bits; the multipliers' inverses
// mod 2^64 by Newton iteration)
__host__ __device__ constexpr uint64_t inv_odd(uint64_t a) {
    uint64_t x = a;  // correct to 3 bits for odd a
    for (int i = 0; i < 5; ++i) x *= 2 - a * x;
    return x;
}
__host__ __device__ inline uint64_t unmix64(uint64_t k) {
    k ^= k >> 33;
    k *= inv_odd(0xc4ceb9fe1a85ec53ull);
    k ^= k >> 33;
    k *= inv_odd(0xff51afd7ed558ccdull);
    k ^= k >> 33;
    return k;
}
static_assert(inv_odd(0xff51afd7ed558ccdull) * 0xff51afd7ed558ccdull == 1, "inverse multiplier");

// stored form of a key in a hashed table: mix64(key); 0 only for key 0 (the side bucket)
__host__ __device__ inline unsigned long long stored_key(int64_t key) { return mix64((uint64_t)key); }

// home bucket from the high 32 hash bits (multiply-shift range reduction); radix
// partitioning for the multi-GPU exchange uses the LOW bits, so a shard's keys still
// spread over its whole table.
__host__ __device__ inline uint32_t bucket_of(uint64_t h, uint32_t nbuckets) {
    return (uint32_t)(((h >> 32) * (uint64_t)nbuckets) >> 32);
}

// Table geometry handed to the kernels.
struct TableView {
    const struct Bucket* tbl;
    const uint32_t* dup_rows;
    const uint64_t* row_ids;
    uint32_t nb;      // buckets (excl. side bucket) = nchunks << clog2
    uint32_t clog2;   // log2 buckets per chunk
    // dense layout (dense != nullptr): ref of key k = dense[k - dmin] for k - dmin < drange
    const uint32_t* dense;
    int64_t dmin;
    uint64_t drange;
    // offset bits of a duplicated key's ref: 31 (kDupFlag | offset), or kPackedMask for
    // dense tables whose refs also carry counts <= 15 in bits 27-30 (dup_rows < 2^27)
    uint32_t off_mask;
};
constexpr uint32_t kFullMask = 0x7FFFFFFFu;
constexpr uint32_t kPackedMask = 0x07FFFFFFu;

// Run refs (packed dense tables, r06). A duplicated key whose rows, in the canonical
// descending order, are consecutive integers top, top - 1, ..., top - c + 1 - a build side
// clustered by key (sorted input, a fact table stored in foreign-key order; C3's exponential
// keys) - keeps them in the ref itself: kDupFlag | 1 << 27 | (c - 2) << 24 | top, for
// 2 <= c <= kRunMaxRows and top < 2^24. A packed count of 1 occurs in no other ref (a
// duplicated key has >= 2 rows), so bits 27-31 = 0x11 mark a run. Readers then need no
// dup_rows segment read (the emission's random segment reads were its cost at C3: 683 ->
// 453 us without them, profiles/r06_emit_ablations.txt). The key's dup_rows segment is
// still written (the build allocates it before it knows), but no reader uses it.
constexpr uint32_t kRunMaxRows = 9;
__host__ __device__ inline bool run_ref(uint32_t r, uint32_t off_mask) {
    return off_mask == kPackedMask && (r >> 27) == 0x11u;
}
__host__ __device__ inline uint32_t run_ref_count(uint32_t r) { return ((r >> 24) & 7u) + 2u; }
__host__ __device__ inline uint32_t make_run_ref(uint32_t top, uint32_t c) {
    return kDupFlag | (1u << 27) | ((c - 2u) << 24) | top;
}
// the count of a ref when it is in the ref (0 kMiss, 1 a single row, a packed or run count),
// else kCountUnknown (in the segment header)
// (selects without early returns: the kernels' per-row decode stays free of branches —
// r06, C3 86.5-86.9K -> 87.5-87.9K Mrows/s once the scans were fused)
__host__ __device__ inline uint32_t ref_count_inline(uint32_t r, uint32_t off_mask) {
    const uint32_t c4 = off_mask == kPackedMask ? ((r >> 27) & 15u) : 0u;
    const uint32_t run = 0u - (uint32_t)(c4 == 1u);  // all ones for a run ref
    const uint32_t dup = (run_ref_count(r) & run) | ((c4 != 0u ? c4 : kCountUnknown) & ~run);
    const uint32_t c = (r & kDupFlag) ? dup : 1u;
    return r == kMiss ? 0u : c;
}
// row j (0-based, descending) of a duplicated key's ref
__host__ __device__ inline uint32_t dup_ref_row(const uint32_t* dup_rows, uint32_t r, uint32_t off_mask, uint32_t j) {
    return run_ref(r, off_mask) ? (r & 0xFFFFFFu) - j : dup_rows[(r & off_mask) + 1 + j];
}

// Build partition geometry: hashed chunks of 2^clog2 buckets (chunk nchunks = the side
// bucket of INT64_MIN) or, dense, chunks of 2^kDenseShift consecutive key values from dmin.
constexpr uint32_t kDenseShift = 11;
struct ChunkGeom {
    uint32_t nb, clog2, nchunks, dshift;
    int64_t dmin;
    int dense;
    int packed;  // dense refs carry small counts (kPackedMask)
};

// A key range of at most kDenseFactor x rows takes the direct-addressed layout.
constexpr uint64_t kDenseFactor = 8;
constexpr uint64_t kDenseBlockValues = 8192;  // a frag-build block: 4 chunks of 2^kDenseShift values

// Build with the key range left on the device (hj_api.cpp build_attempt): the dense frag
// build is launched before the host knows the range, its kernels read the range the
// reduction left in device memory (mm = {min, max}) and resolve the geometry themselves.
// spec_dense_blocks = the 8192-value blocks a direct-addressed table over [mn, mx] spans,
// or 0 when that range takes another layout (no valid key, wider than kDenseFactor x rows
// or than `cap` blocks): the kernels then do nothing and the host builds once it has read
// the range. Host and device evaluate this one function, so they agree on the outcome.
struct SpecGeo {
    const long long* mm;  // null: the geometry came from the host
    uint64_t rows;
    uint32_t cap;
};
__host__ __device__ inline uint32_t spec_dense_blocks(int64_t mn, int64_t mx, uint64_t rows, uint32_t cap) {
    if (mn > mx) return 0u;
    const uint64_t range = (uint64_t)mx - (uint64_t)mn + 1;  // 0: the whole int64 domain
    if (range == 0 || range > kDenseFactor * rows) return 0u;
    const uint64_t nblk = (range + kDenseBlockValues - 1) / kDenseBlockValues;
    return nblk <= cap ? (uint32_t)nblk : 0u;
}

}  // namespace dfp
