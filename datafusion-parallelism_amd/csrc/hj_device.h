// hj_device.h — data layout shared by the gfx950 kernels (hj_kernels.hip) and the
// C-ABI host layer (hj_api.cpp).
//
// Slot table in HBM:
//   Bucket[nbuckets + 1], 64-byte aligned, one 64-byte line per bucket:
//     uint64 key[4]   stored key = key ^ 2^63, 0 = empty slot
//     uint2  pay[4]   .x = rows with this key, .y = row (x == 1) or dup_rows start (x > 1)
//   Bucket[nbuckets] is the side bucket: slot 0 holds the key INT64_MIN, whose stored
//   form collides with "empty".
//   dup_rows[]      u32 build rows of every key with > 1 row, one segment per key,
//                   sorted descending (= the reference's newest-first chain order).
//   row_ids[]       optional u64 explicit build ids (multi-GPU exchange).
//
// The reference's v10 table (src/operator/version10/new_map_3/fixed_table.rs:114-140)
// stores (hash|bit63, row+1) slots with a separate u8 tag array and an overflow chain
// array; this layout instead keeps the exact key in the slot (so the probe needs no
// second gather for equal_rows_arr, src/shared/datafusion_private.rs:40-80) and
// replaces pointer-chasing chains with one contiguous sorted segment per key.
#pragma once
#include <stdint.h>

namespace dfp {

constexpr uint64_t kSign = 0x8000000000000000ull;
constexpr int kSlots = 4;
constexpr int kProbeThreads = 256;
constexpr int kRowsPerThread = 4;
constexpr int kProbeTile = kProbeThreads * kRowsPerThread;  // 1024 probe rows per tile
constexpr int kSmallSeg = 16;  // dup segments up to this size are sorted by one thread

struct alignas(64) Bucket {
    unsigned long long key[kSlots];
    unsigned int pay[kSlots][2];
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
    unsigned long long n_dupslots;   // keys with > 1 row
    unsigned long long n_duprows;    // 2nd..nth rows of such keys
    unsigned long long dup_used;     // dup_rows entries allocated
    unsigned long long n_big;        // segments > kSmallSeg
    unsigned long long inserted;     // non-null rows inserted
    unsigned long long distinct;     // occupied slots
    unsigned long long max_key_rows; // longest segment
    unsigned long long err;          // != 0: bounded spin gave up / overflow
};

struct DupDir {
    unsigned int start, n, fill, slot;
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

// bucket index from the high 32 hash bits (multiply-shift range reduction);
// radix partitioning for the multi-GPU exchange uses the LOW bits, so a shard's keys
// still spread over its whole table.
__host__ __device__ inline uint32_t bucket_of(uint64_t h, uint32_t nbuckets) {
    return (uint32_t)(((h >> 32) * (uint64_t)nbuckets) >> 32);
}

}  // namespace dfp
