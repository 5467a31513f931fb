// hj_kernels.hip — hand-written gfx950 (CDNA4) kernels of the parallel hash join.
//
// Hot path:
//   build   (replaces Inner::insert_atomically, src/operator/version10/new_map_3/
//            fixed_table.rs:560-672, driven by JoinStateInstance::add,
//            src/operator/version10/parallel_join_execution_state.rs:91-133, and the
//            overflow-chain compaction of the same file, 135-315)
//     coarse_hist/scatter   level 1: rows -> groups of 2^gshift chunks (<= 128 groups)
//     fine_hist/scatter     level 2: group-ordered rows -> chunk order
//     scan_*_kernel         exclusive scans of the histograms (reduce-then-scan)
//     chunk_build_kernel    one workgroup per 2^clog2-bucket chunk: insert with LDS
//                           64-bit CAS + LDS counts, lay out duplicate segments, write
//                           the finished chunk out with coalesced 16-byte stores
//     dup_sort_big_kernel   order large duplicate segments (LDS bitonic / ordered rescan)
//   probe   (replaces get_matching_indices, src/shared/shared.rs:29-47, the chain walk,
//            src/operator/version10/lookup_implementation_3.rs:22-59, and
//            equal_rows_arr, src/shared/datafusion_private.rs:40-80)
//     sl_* (sliced probe)   large probes: rows partitioned by table slice, lookups out
//                           of LDS, ordered emission per tile (see the section below)
//     probe_fused_kernel    small probes: per probe row one table read (exact key
//                           compare, so no separate equality gather); the tile's output
//                           offset by decoupled look-back; ordered (probe asc, build
//                           desc) pair emission
//
// No same-address global atomics on the hot loops (a single word sustains ~88
// atomics/us, MI355X_MICROARCH.md "dequeue"). The one inter-workgroup hand-off is the
// fused probe's look-back (per-tile flags, each written by its own tile).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <type_traits>

#include "hj_device.h"
#include "hj_launch.h"
#include "hj_util.h"

namespace dfp {

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
template <typename K>
__device__ __forceinline__ int64_t ld_key(const void* keys, int64_t i) {
    return (int64_t)(reinterpret_cast<const K*>(keys)[i]);
}

__device__ __forceinline__ int64_t seg_key(const Segment& sg, int64_t i, int key_bytes) {
    return key_bytes == 8 ? ld_key<int64_t>(sg.keys, i) : ld_key<int32_t>(sg.keys, i);
}

__device__ __forceinline__ int find_seg(const Segment* segs, int nseg, int64_t r) {
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (segs[mid].row_base <= r) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// home bucket of a key (its probe sequence never leaves the bucket's chunk), and of its
// stored form (no rehash)
__device__ __forceinline__ uint32_t home_bucket(int64_t key, uint32_t nb) {
    return bucket_of(mix64((uint64_t)key), nb);
}
__device__ __forceinline__ uint32_t stored_bucket(unsigned long long sk, uint32_t nb) { return bucket_of(sk, nb); }

// ---------------------------------------------------------------------------
// build 1: rows -> chunk order in two partition levels. A 32 K-row tile spread over all
// ~5600 chunks of a C2 table leaves ~6 rows per chunk, i.e. partial-line stores (the
// one-level scatter wrote 4.9x its algorithmic bytes). Level 1 splits rows into <= 128
// groups of 2^gshift consecutive chunks (~250-500 rows per group per tile); level 2 then
// sorts the group-ordered rows by chunk, where each tile spans only a group or two, so
// both levels write long runs.
// ---------------------------------------------------------------------------
constexpr int kHistThreads = 1024;
constexpr int kFineLdsBins = 8192;  // fine histogram in LDS (32 KB) up to this many chunks per tile

__device__ __forceinline__ uint32_t chunk_of(int64_t key, const ChunkGeom& g) {
    if (g.dense) return (uint32_t)(((uint64_t)key - (uint64_t)g.dmin) >> g.dshift);
    return key == 0 ? g.nchunks : (home_bucket(key, g.nb) >> g.clog2);  // key 0: the side bucket
}

// The segment descriptors of one tile's rows in LDS (per-row lookups in global memory
// form a dependent load chain). Returns the descriptor array to use (LDS, or the
// global one for a tile made of more than kTileSegs appends) and its count.
constexpr int kTileSegs = 64;
__device__ __forceinline__ const Segment* tile_segments(const Segment* __restrict__ segs, int nseg, int64_t r0,
                                                        int64_t r1, Segment* s_seg, int* s_info, int* ns) {
    if (threadIdx.x == 0) {
        const int a = find_seg(segs, nseg, r0);
        const int b = r1 > r0 ? find_seg(segs, nseg, r1 - 1) : a;
        s_info[0] = a;
        s_info[1] = b - a + 1;
    }
    __syncthreads();
    const int a = s_info[0], cnt = s_info[1];
    if (cnt > kTileSegs) {
        *ns = nseg;
        return segs;
    }
    for (int k = threadIdx.x; k < cnt; k += blockDim.x) s_seg[k] = segs[a + k];
    __syncthreads();
    *ns = cnt;
    return s_seg;
}

// Rows base + u * kHistThreads + threadIdx.x (u < kRowBatch) of the appended build input,
// all loads issued before any use (the tile loops are latency-bound otherwise). ok[u]:
// row exists and is valid. With ids/row_ids, copies the explicit ids to row_ids[r].
constexpr int kRowBatch = 8;
template <typename K>
__device__ __forceinline__ void load_rows(const Segment* __restrict__ segs, int nseg, int64_t base, int64_t r1,
                                          int64_t (&key)[kRowBatch], bool (&ok)[kRowBatch],
                                          uint64_t* __restrict__ row_ids, int64_t* rows, bool ids_as_rows) {
    if (nseg == 1) {  // the whole tile inside one append: uniform pointers, loads batch up
        const Segment sg = segs[0];
#pragma unroll
        for (int u = 0; u < kRowBatch; ++u) {
            const int64_t r = base + (int64_t)u * kHistThreads + threadIdx.x;
            if (rows) rows[u] = r;
            ok[u] = r < r1;
            key[u] = 0;
            if (ok[u]) {
                const int64_t i = r - sg.row_base;
                if (row_ids != nullptr && sg.ids != nullptr) row_ids[r] = sg.ids[i];
                if (ids_as_rows && rows) rows[u] = (int64_t)sg.ids[i];
                ok[u] = bit_valid(sg.valid, sg.voff, i);
                key[u] = ld_key<K>(sg.keys, i);
            }
        }
        return;
    }
#pragma unroll
    for (int u = 0; u < kRowBatch; ++u) {
        const int64_t r = base + (int64_t)u * kHistThreads + threadIdx.x;
        if (rows) rows[u] = r;
        ok[u] = false;
        key[u] = 0;
        if (r < r1) {
            const Segment& sg = segs[find_seg(segs, nseg, r)];  // independent per row
            const int64_t i = r - sg.row_base;
            if (row_ids != nullptr && sg.ids != nullptr) row_ids[r] = sg.ids[i];
            if (ids_as_rows && rows) rows[u] = (int64_t)sg.ids[i];
            ok[u] = bit_valid(sg.valid, sg.voff, i);
            key[u] = ld_key<K>(sg.keys, i);
        }
    }
}

// level 1: rows per (group, tile); hist1[g * ntiles + tile]. NB bins in COPIES LDS
// copies (per-wave copies for the 128-group level; 4 copies of 2048 bins for the
// one-level dense partition): fewer LDS atomic collisions.
template <typename K, int NB, int COPIES>
__global__ void __launch_bounds__(kHistThreads)
coarse_hist_kernel(const Segment* __restrict__ segs, int nseg, int64_t total, ChunkGeom g, uint32_t gshift, uint32_t ngroups, uint32_t* __restrict__ hist1,
                   int64_t ntiles, int64_t tile_rows) {
    __shared__ uint32_t s_h[COPIES][NB];
    const int wave = (threadIdx.x >> 6) % COPIES;
    for (uint32_t k = threadIdx.x; k < (uint32_t)(COPIES * NB); k += kHistThreads) (&s_h[0][0])[k] = 0;
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * tile_rows;
    const int64_t r1 = min<int64_t>(total, r0 + tile_rows);
    __shared__ Segment s_seg[kTileSegs];
    __shared__ int s_info[2];
    int tns;
    const Segment* tsegs = tile_segments(segs, nseg, r0, r1, s_seg, s_info, &tns);
    for (int64_t base = r0; base < r1; base += kHistThreads * kRowBatch) {
        int64_t key[kRowBatch];
        bool ok[kRowBatch];
        load_rows<K>(tsegs, tns, base, r1, key, ok, nullptr, nullptr, false);
#pragma unroll
        for (int u = 0; u < kRowBatch; ++u)
            if (ok[u]) atomicAdd(&s_h[wave][chunk_of(key[u], g) >> gshift], 1u);
    }
    __syncthreads();
    for (uint32_t g = threadIdx.x; g < ngroups; g += kHistThreads) {
        uint32_t v = 0;
        for (int w = 0; w < COPIES; ++w) v += s_h[w][g];
        hist1[(int64_t)g * ntiles + blockIdx.x] = v;
    }
}

// level 2: rows per (chunk, tile) over the group-ordered rows tkeys[0, n_valid); a tile
// touches only the chunks of the groups it spans: hist2 must be zeroed beforehand
__device__ __forceinline__ void fine_range(const unsigned long long* tkeys, int64_t r0, int64_t r1, ChunkGeom g, uint32_t gshift, uint32_t* lo,
                                           uint32_t* hi) {
    const uint32_t g0 = chunk_of((int64_t)tkeys[r0], g) >> gshift;
    const uint32_t g1 = chunk_of((int64_t)tkeys[r1 - 1], g) >> gshift;
    *lo = g0 << gshift;
    *hi = min(g.nchunks, ((g1 + 1) << gshift) - 1);  // inclusive
}

__global__ void __launch_bounds__(kHistThreads)
fine_hist_kernel(const unsigned long long* __restrict__ tkeys, const BuildCounters* __restrict__ ctr, ChunkGeom g, uint32_t gshift, uint32_t* __restrict__ hist, int64_t ntiles,
                 int64_t tile_rows) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_h[];
    const int64_t nvalid = (int64_t)ctr->n_valid;
    const int64_t r0 = (int64_t)blockIdx.x * tile_rows;
    const int64_t r1 = min<int64_t>(nvalid, r0 + tile_rows);
    if (r0 >= r1) return;
    uint32_t lo, hi;
    fine_range(tkeys, r0, r1, g, gshift, &lo, &hi);
    // a tile spanning more than kFineLdsBins chunks (skewed groups) counts in global memory
    const bool in_lds = hi - lo + 1 <= (uint32_t)kFineLdsBins;
    if (in_lds)
        for (uint32_t c = lo + threadIdx.x; c <= hi; c += kHistThreads) s_h[c - lo] = 0;
    __syncthreads();
    for (int64_t base = r0; base < r1; base += kHistThreads * kRowBatch) {
        unsigned long long key[kRowBatch];
#pragma unroll
        for (int u = 0; u < kRowBatch; ++u) {
            const int64_t r = base + (int64_t)u * kHistThreads + threadIdx.x;
            key[u] = r < r1 ? tkeys[r] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < kRowBatch; ++u) {
            if (base + (int64_t)u * kHistThreads + threadIdx.x >= r1) continue;
            const uint32_t c = chunk_of((int64_t)key[u], g);
            if (in_lds) atomicAdd(&s_h[c - lo], 1u);
            else atomicAdd(&hist[(int64_t)c * ntiles + blockIdx.x], 1u);
        }
    }
    __syncthreads();
    if (!in_lds) return;
    for (uint32_t c = lo + threadIdx.x; c <= hi; c += kHistThreads) hist[(int64_t)c * ntiles + blockIdx.x] = s_h[c - lo];
}

// ---------------------------------------------------------------------------
// exclusive scan of u32 / u64 (reduce-then-scan, three launches, no inter-block hand-off)
// ---------------------------------------------------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanPerThread = 16;
constexpr int kScanSeg = kScanThreads * kScanPerThread;

template <typename T>
__global__ void __launch_bounds__(kScanThreads)
scan_reduce_kernel(const T* __restrict__ a, int64_t len, unsigned long long* __restrict__ bsum) {
    __shared__ unsigned long long s_w[kScanThreads / 64];
    const int64_t base = (int64_t)blockIdx.x * kScanSeg + (int64_t)threadIdx.x * kScanPerThread;
    unsigned long long s = 0;
#pragma unroll
    for (int k = 0; k < kScanPerThread; ++k)
        if (base + k < len) s += a[base + k];
    unsigned long long tot;
    block_excl_scan<unsigned long long>(s, s_w, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// single block: exclusive scan of nblk block sums; bsum[nblk] = grand total
__global__ void __launch_bounds__(1024)
scan_top_kernel(unsigned long long* bsum, int64_t nblk, unsigned long long* total_out) {
    __shared__ unsigned long long s_w[16];
    const int64_t per = (nblk + 1023) / 1024;
    const int64_t b0 = (int64_t)threadIdx.x * per;
    unsigned long long s = 0;
    for (int64_t k = 0; k < per; ++k)
        if (b0 + k < nblk) s += bsum[b0 + k];
    unsigned long long tot;
    unsigned long long off = block_excl_scan<unsigned long long>(s, s_w, &tot);
    for (int64_t k = 0; k < per; ++k) {
        if (b0 + k < nblk) {
            const unsigned long long x = bsum[b0 + k];
            bsum[b0 + k] = off;
            off += x;
        }
    }
    if (threadIdx.x == 0) {
        bsum[nblk] = tot;
        if (total_out) *total_out = tot;
    }
}

template <typename T>
__global__ void __launch_bounds__(kScanThreads)
scan_down_kernel(T* __restrict__ a, int64_t len, const unsigned long long* __restrict__ bsum) {
    __shared__ unsigned long long s_w[kScanThreads / 64];
    const int64_t base = (int64_t)blockIdx.x * kScanSeg + (int64_t)threadIdx.x * kScanPerThread;
    T v[kScanPerThread];
    unsigned long long s = 0;
#pragma unroll
    for (int k = 0; k < kScanPerThread; ++k) {
        v[k] = (base + k < len) ? a[base + k] : (T)0;
        s += v[k];
    }
    unsigned long long tot;
    unsigned long long off = bsum[blockIdx.x] + block_excl_scan<unsigned long long>(s, s_w, &tot);
#pragma unroll
    for (int k = 0; k < kScanPerThread; ++k) {
        if (base + k < len) a[base + k] = (T)off;
        off += v[k];
    }
}

// ---------------------------------------------------------------------------
// build 2: the two scatters (positions from the scanned histograms; order inside a
// group / chunk is canonicalised by the chunk build)
// ---------------------------------------------------------------------------
// LDS-staged scatter of one sub-batch (<= kHistThreads * kRowBatch rows) whose rows sit in
// registers (key, row, bin in [0, R)): counting sort by bin in LDS, then stores in bin
// order, so that consecutive lanes write consecutive addresses (whole lines instead of
// one line per lane). s_cur[b] = next global position of bin b (advanced here).
constexpr int kStageRows = kHistThreads * kRowBatch;  // 8192 rows: 64 KB keys + 32 KB rows
constexpr int kStageMaxBins = 2048;
static_assert(kStageMaxBins == kMaxLevel1Bins, "one-level dense partition bins");
constexpr size_t kStageLds = (size_t)kStageRows * 14 + (size_t)kStageMaxBins * 12;  // + u16 bin per row

__device__ __forceinline__ void staged_scatter_batch(const unsigned long long (&key)[kRowBatch],
                                                     const uint32_t (&row)[kRowBatch], const int (&bin)[kRowBatch],
                                                     uint32_t R, unsigned long long* s_k, uint32_t* s_r,
                                                     uint16_t* s_b, uint32_t* s_cur, uint32_t* s_cnt, uint32_t* s_st,
                                                     uint32_t* s_w,
                                                     unsigned long long* __restrict__ out_k,
                                                     uint32_t* __restrict__ out_r) {
    for (uint32_t b = threadIdx.x; b < R; b += kHistThreads) s_cnt[b] = 0;
    __syncthreads();
    uint32_t lrank[kRowBatch];
#pragma unroll
    for (int u = 0; u < kRowBatch; ++u) lrank[u] = bin[u] >= 0 ? atomicAdd(&s_cnt[bin[u]], 1u) : 0u;
    __syncthreads();
    // exclusive scan of the bin counts (R <= 2048: two bins per thread)
    const uint32_t b0 = 2 * threadIdx.x;
    const uint32_t c0 = b0 < R ? s_cnt[b0] : 0u, c1 = b0 + 1 < R ? s_cnt[b0 + 1] : 0u;
    uint32_t nsub;
    const uint32_t ex = block_excl_scan<uint32_t>(c0 + c1, s_w, &nsub);
    if (b0 < R) s_st[b0] = ex;
    if (b0 + 1 < R) s_st[b0 + 1] = ex + c0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kRowBatch; ++u) {
        if (bin[u] < 0) continue;
        const uint32_t pos = s_st[bin[u]] + lrank[u];
        s_k[pos] = key[u];
        s_r[pos] = row[u];
        s_b[pos] = (uint16_t)bin[u];
    }
    __syncthreads();
    // stores in bin order (consecutive lanes, consecutive addresses within a bin)
    for (uint32_t i = threadIdx.x; i < nsub; i += kHistThreads) {
        const uint32_t b = s_b[i];
        const uint32_t g = s_cur[b] + (i - s_st[b]);
        out_k[g] = s_k[i];
        out_r[g] = s_r[i];
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < R; b += kHistThreads) s_cur[b] += s_cnt[b];
    __syncthreads();
}

template <typename K>
__global__ void __launch_bounds__(kHistThreads)
coarse_scatter_staged_kernel(const Segment* __restrict__ segs, int nseg, int64_t total, ChunkGeom g, uint32_t gshift, uint32_t ngroups, const uint32_t* __restrict__ hist1,
                             int64_t ntiles, unsigned long long* __restrict__ tkeys, uint32_t* __restrict__ trows,
                             uint64_t* __restrict__ row_ids, bool ids_as_rows, int64_t tile_rows) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long* s_k = reinterpret_cast<unsigned long long*>(smem);
    uint32_t* s_r = reinterpret_cast<uint32_t*>(s_k + kStageRows);
    uint32_t* s_cur = s_r + kStageRows;
    uint32_t* s_cnt = s_cur + kStageMaxBins;
    uint32_t* s_st = s_cnt + kStageMaxBins;
    uint16_t* s_b = reinterpret_cast<uint16_t*>(s_st + kStageMaxBins);
    __shared__ uint32_t s_w[kHistThreads / 64];
    __shared__ Segment s_seg[kTileSegs];
    __shared__ int s_info[2];
    for (uint32_t g = threadIdx.x; g < ngroups; g += kHistThreads) s_cur[g] = hist1[(int64_t)g * ntiles + blockIdx.x];
    const int64_t r0 = (int64_t)blockIdx.x * tile_rows;
    const int64_t r1 = min<int64_t>(total, r0 + tile_rows);
    int tns;
    const Segment* tsegs = tile_segments(segs, nseg, r0, r1, s_seg, s_info, &tns);  // syncs
    for (int64_t base = r0; base < r1; base += kStageRows) {
        int64_t k64[kRowBatch], rr[kRowBatch];
        bool ok[kRowBatch];
        load_rows<K>(tsegs, tns, base, r1, k64, ok, row_ids, rr, ids_as_rows);
        unsigned long long key[kRowBatch];
        uint32_t row[kRowBatch];
        int bin[kRowBatch];
#pragma unroll
        for (int u = 0; u < kRowBatch; ++u) {
            key[u] = (unsigned long long)k64[u];
            row[u] = (uint32_t)rr[u];
            bin[u] = ok[u] ? (int)(chunk_of(k64[u], g) >> gshift) : -1;
        }
        staged_scatter_batch(key, row, bin, ngroups, s_k, s_r, s_b, s_cur, s_cnt, s_st, s_w, tkeys, trows);
    }
}

__global__ void __launch_bounds__(kHistThreads)
fine_scatter_staged_kernel(const unsigned long long* __restrict__ tkeys, const uint32_t* __restrict__ trows,
                           const BuildCounters* __restrict__ ctr, ChunkGeom g,
                           uint32_t gshift, uint32_t* __restrict__ hist, int64_t ntiles,
                           unsigned long long* __restrict__ skeys, uint32_t* __restrict__ srows, int64_t tile_rows) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long* s_k = reinterpret_cast<unsigned long long*>(smem);
    uint32_t* s_r = reinterpret_cast<uint32_t*>(s_k + kStageRows);
    uint32_t* s_cur = s_r + kStageRows;
    uint32_t* s_cnt = s_cur + kStageMaxBins;
    uint32_t* s_st = s_cnt + kStageMaxBins;
    uint16_t* s_b = reinterpret_cast<uint16_t*>(s_st + kStageMaxBins);
    __shared__ uint32_t s_w[kHistThreads / 64];
    const int64_t nvalid = (int64_t)ctr->n_valid;
    const int64_t r0 = (int64_t)blockIdx.x * tile_rows;
    const int64_t r1 = min<int64_t>(nvalid, r0 + tile_rows);
    if (r0 >= r1) return;
    uint32_t lo, hi;
    fine_range(tkeys, r0, r1, g, gshift, &lo, &hi);
    const uint32_t R = hi - lo + 1;
    if (R > (uint32_t)kStageMaxBins) {
        // a tile spanning many chunks (skewed groups): direct stores, the tile's scanned
        // histogram column is the cursor array (consumed; the chunk build reads chunk_starts)
        for (int64_t r = r0 + threadIdx.x; r < r1; r += kHistThreads) {
            const unsigned long long key = tkeys[r];
            const uint32_t c = chunk_of((int64_t)key, g);
            const uint32_t pos = atomicAdd(&hist[(int64_t)c * ntiles + blockIdx.x], 1u);
            skeys[pos] = key;
            srows[pos] = trows[r];
        }
        return;
    }
    for (uint32_t b = threadIdx.x; b < R; b += kHistThreads) s_cur[b] = hist[(int64_t)(lo + b) * ntiles + blockIdx.x];
    __syncthreads();
    for (int64_t base = r0; base < r1; base += kStageRows) {
        unsigned long long key[kRowBatch];
        uint32_t row[kRowBatch];
        int bin[kRowBatch];
#pragma unroll
        for (int u = 0; u < kRowBatch; ++u) {
            const int64_t r = base + (int64_t)u * kHistThreads + threadIdx.x;
            key[u] = r < r1 ? tkeys[r] : 0ull;
            row[u] = r < r1 ? trows[r] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kRowBatch; ++u) {
            const int64_t r = base + (int64_t)u * kHistThreads + threadIdx.x;
            bin[u] = r < r1 ? (int)(chunk_of((int64_t)key[u], g) - lo) : -1;
        }
        staged_scatter_batch(key, row, bin, R, s_k, s_r, s_b, s_cur, s_cnt, s_st, s_w, skeys, srows);
    }
}

// chunk c's rows are [starts[c], starts[c + 1]) of skeys / srows (chunk nchunks = side)
__global__ void chunk_starts_kernel(const uint32_t* __restrict__ hist, int64_t ntiles, uint32_t nchunks,
                                    const BuildCounters* __restrict__ ctr, uint32_t* __restrict__ starts) {
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c <= nchunks + 1; c += gridDim.x * blockDim.x)
        starts[c] = c <= nchunks ? hist[(int64_t)c * ntiles] : (uint32_t)ctr->n_valid;
}

// ---------------------------------------------------------------------------
// build 3: one workgroup per chunk builds the chunk's buckets in LDS
// ---------------------------------------------------------------------------
constexpr int kChunkRegRows = 4;  // rows per thread kept in registers across passes A-C

__device__ __forceinline__ void sort16_desc(uint32_t (&v)[16]) {
#pragma unroll
    for (int k = 2; k <= 16; k <<= 1) {
#pragma unroll
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int l = i ^ jj;
                if (l > i) {
                    const bool desc = ((i & k) == 0);
                    const uint32_t a = v[i], b = v[l];
                    const bool sw = desc ? (a < b) : (a > b);
                    v[i] = sw ? b : a;
                    v[l] = sw ? a : b;
                }
            }
        }
    }
}

// LDS slot of `key` inside the chunk image (insert = claim an empty slot with CAS; the
// claiming insert gets kSlotNew or-ed into the slot index)
constexpr int kSlotNew = 1 << 30;
template <bool INSERT>
__device__ __forceinline__ int chunk_slot(Bucket* img, uint32_t cmask, uint32_t i0, unsigned long long sk) {
    uint32_t i = i0;
    for (uint32_t probes = 0; probes <= cmask; ++probes) {
        Bucket& B = img[i];
#pragma unroll
        for (int j = 0; j < kSlots; ++j) {
            unsigned long long kk = B.key[j];
            if (INSERT && kk == 0) kk = atomicCAS(&B.key[j], 0ull, sk);
            if (INSERT && kk == 0) return (int)(i * kSlots + j) | kSlotNew;  // claimed here
            if (kk == sk) return (int)(i * kSlots + j);
            if (!INSERT && kk == 0) return -1;
        }
        // passing a full bucket: mark it, so that a lookup missing in a full bucket
        // without the mark can stop there (meta bit 0 = "a probe sequence continues")
        if (INSERT) atomicOr(&B.meta, 1u);
        i = (i + 1) & cmask;
    }
    return -1;
}

template <int kChunkThreads>
__global__ void __launch_bounds__(kChunkThreads)
chunk_build_kernel(uint32_t nb, uint32_t clog2, uint32_t nchunks, const uint32_t* __restrict__ starts,
                   const unsigned long long* __restrict__ skeys,
                   const uint32_t* __restrict__ srows, Bucket* __restrict__ tbl, uint32_t* __restrict__ dup_rows,
                   BigSeg* __restrict__ big, BuildCounters* ctr, uint32_t dupcap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t CB = 1u << clog2, cmask = CB - 1;
    Bucket* img = reinterpret_cast<Bucket*>(smem);
    uint32_t* d_off = reinterpret_cast<uint32_t*>(smem + (size_t)CB * sizeof(Bucket));
    uint32_t* d_cur = d_off + dupcap;
    uint32_t* d_cnt = d_cur + dupcap;
    __shared__ unsigned s_ndup, s_dup;
    __shared__ unsigned long long s_w[kChunkThreads / 64];
    __shared__ unsigned long long s_base;

    const uint32_t c = blockIdx.x;
    const bool side = (c == nchunks);
    const uint32_t start = starts[c];
    const uint32_t end = starts[c + 1];
    const uint32_t nimg = side ? 1u : CB;

    // zero the chunk image
    {
        uint4* p = reinterpret_cast<uint4*>(img);
        for (uint32_t k = threadIdx.x; k < nimg * 4; k += kChunkThreads) p[k] = make_uint4(0, 0, 0, 0);
        if (threadIdx.x == 0) {
            s_ndup = 0;
            s_dup = side ? 1u : 0u;
        }
    }
    __syncthreads();

    // rows of a chunk with <= kChunkThreads * kChunkRegRows rows stay in registers from
    // pass A to pass C (key, row and claimed slot); larger chunks (duplicate-heavy
    // keys) stream their rows twice
    const bool in_regs = end - start <= (uint32_t)(kChunkThreads * kChunkRegRows);
    uint32_t rrow[kChunkRegRows];
    int rslot[kChunkRegRows];
    if (in_regs) {
        unsigned long long rk[kChunkRegRows];
#pragma unroll
        for (int u = 0; u < kChunkRegRows; ++u) {
            const uint32_t r = start + u * kChunkThreads + threadIdx.x;
            rk[u] = r < end ? skeys[r] : 0ull;
            rrow[u] = r < end ? srows[r] : 0u;
        }
        // pass A: claim slots (LDS CAS); the claiming insert stores its row in the ref
        // (final if the key stays single); finding the key already present flags the
        // chunk as holding duplicates
#pragma unroll
        for (int u = 0; u < kChunkRegRows; ++u) {
            rslot[u] = -1;
            if (start + u * kChunkThreads + threadIdx.x >= end) continue;
            const unsigned long long sk = stored_key((int64_t)rk[u]);
            int slot = 0;
            bool claimed = false;
            if (!side) {
                const int v = chunk_slot<true>(img, cmask, stored_bucket(sk, nb) & cmask, sk);
                if (v < 0) { atomicOr(&ctr->err, 1ull); continue; }  // chunk full
                slot = v & ~kSlotNew;
                claimed = (v & kSlotNew) != 0;
            }
            rslot[u] = slot;
            if (claimed) img[slot / kSlots].ref[slot % kSlots] = rrow[u];
            else s_dup = 1u;
        }
        __syncthreads();
        if (s_dup) {  // duplicates: turn refs into row counts
            for (uint32_t sl = threadIdx.x; sl < nimg * kSlots; sl += kChunkThreads) img[sl / kSlots].ref[sl % kSlots] = 0;
            __syncthreads();
#pragma unroll
            for (int u = 0; u < kChunkRegRows; ++u)
                if (rslot[u] >= 0) atomicAdd(&img[rslot[u] / kSlots].ref[rslot[u] % kSlots], 1u);
        }
    } else {
        if (threadIdx.x == 0) s_dup = 1u;
        // pass A (streamed)
        for (uint32_t r = start + threadIdx.x; r < end; r += kChunkThreads) {
            const unsigned long long sk = stored_key((int64_t)skeys[r]);
            int slot;
            if (side) {
                slot = 0;
            } else {
                const uint32_t i0 = stored_bucket(sk, nb) & cmask;
                slot = chunk_slot<true>(img, cmask, i0, sk);
                if (slot < 0) { atomicOr(&ctr->err, 1ull); continue; }  // chunk full
                slot &= ~kSlotNew;
            }
            atomicAdd(&img[slot / kSlots].ref[slot % kSlots], 1u);
        }
    }
    __syncthreads();

    // passes B-D only for chunks holding duplicated keys (block-uniform branch)
    if (s_dup) {
        // pass B: directory of duplicated keys (count > 1)
        for (uint32_t sl = threadIdx.x; sl < nimg * kSlots; sl += kChunkThreads) {
            unsigned& ref = img[sl / kSlots].ref[sl % kSlots];
            const unsigned cnt = ref;
            if (cnt > 1) {
                const unsigned li = atomicAdd(&s_ndup, 1u);
                if (li < dupcap) {
                    d_cnt[li] = cnt;
                    d_cur[li] = 0;
                    ref = kDupFlag | li;
                } else {
                    atomicOr(&ctr->err, 2ull);  // dup directory full: the host retries at half load
                }
            }
        }
        __syncthreads();
        const unsigned ndup = min(s_ndup, dupcap);
        // segment offsets: exclusive scan of (count + 1) over the directory, one global
        // reservation per chunk
        {
            unsigned long long carry = 0;
            for (unsigned b = 0; b < ndup; b += kChunkThreads) {
                const unsigned li = b + threadIdx.x;
                const unsigned long long v = li < ndup ? (unsigned long long)d_cnt[li] + 1 : 0;
                unsigned long long tot;
                const unsigned long long ex = block_excl_scan<unsigned long long>(v, s_w, &tot);
                if (li < ndup) d_off[li] = (uint32_t)(carry + ex);
                carry += tot;
            }
            if (threadIdx.x == 0) s_base = carry ? atomicAdd(&ctr->dup_used, carry) : 0;
            __syncthreads();
            for (unsigned li = threadIdx.x; li < ndup; li += kChunkThreads) {
                d_off[li] += (uint32_t)s_base;
                dup_rows[d_off[li]] = d_cnt[li];  // segment header = row count
            }
        }
        __syncthreads();

        // pass C: place rows: single-row keys keep their row in ref, duplicated keys append
        // to their segment (unordered here, sorted in pass D)
        auto place = [&](int slot, uint32_t row) {
            unsigned& ref = img[slot / kSlots].ref[slot % kSlots];
            const unsigned rv = ref;
            if (rv & kDupFlag) {
                const unsigned li = rv & ~kDupFlag;
                const unsigned k = atomicAdd(&d_cur[li], 1u);
                dup_rows[d_off[li] + 1 + k] = row;
            } else if (rv == 1) {
                ref = row;  // the key's only row (rv == count == 1)
            }
        };
        if (in_regs) {
#pragma unroll
            for (int u = 0; u < kChunkRegRows; ++u)
                if (rslot[u] >= 0) place(rslot[u], rrow[u]);
        } else {
            for (uint32_t r = start + threadIdx.x; r < end; r += kChunkThreads) {
                const unsigned long long sk = stored_key((int64_t)skeys[r]);
                int slot = 0;
                if (!side) {
                    const uint32_t i0 = stored_bucket(sk, nb) & cmask;
                    slot = chunk_slot<false>(img, cmask, i0, sk);
                    if (slot < 0) continue;
                }
                place(slot, srows[r]);
            }
        }
        __syncthreads();

        // pass D: canonical order inside segments (descending rows), final refs
        for (unsigned li = threadIdx.x; li < ndup; li += kChunkThreads) {
            const unsigned n = d_cnt[li], off = d_off[li];
            if (n <= (unsigned)kSmallSeg) {
                uint32_t v[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = (i < (int)n) ? dup_rows[off + 1 + i] : 0u;
                sort16_desc(v);
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (i < (int)n) dup_rows[off + 1 + i] = v[i];
            }
        }
        for (uint32_t sl = threadIdx.x; sl < nimg * kSlots; sl += kChunkThreads) {
            Bucket& B = img[sl / kSlots];
            unsigned& ref = B.ref[sl % kSlots];
            if (ref & kDupFlag) {
                const unsigned li = ref & ~kDupFlag;
                if (d_cnt[li] > (unsigned)kSmallSeg) {
                    const unsigned bi = (unsigned)atomicAdd(&ctr->n_big, 1ull);  // rare: > 16 rows
                    big[bi] = BigSeg{side ? 0ull : unmix64(B.key[sl % kSlots]), d_off[li], 0u};
                }
                ref = kDupFlag | d_off[li];
                // small row counts inline in meta (6 bits per slot): the probe's count pass
                // then needs no dup_rows access
                if (!side && d_cnt[li] <= kInlineCount) atomicOr(&B.meta, d_cnt[li] << (1 + 6 * (sl % kSlots)));
            }
        }
        __syncthreads();

    }
    __syncthreads();

    // pass E: write the finished chunk (coalesced 16-byte stores)
    if (side) {
        if (threadIdx.x == 0) {
            Bucket& S = tbl[nb];
            for (int j = 0; j < kSlots; ++j) { S.key[j] = 0; S.ref[j] = 0; }
            S.ref[0] = img[0].ref[0];
            S.meta = end - start;
        }
    } else {
        const uint4* src = reinterpret_cast<const uint4*>(img);
        uint4* dst = reinterpret_cast<uint4*>(tbl + ((size_t)c << clog2));
        for (uint32_t k = threadIdx.x; k < CB * 4; k += kChunkThreads) dst[k] = src[k];
    }
}

// ---------------------------------------------------------------------------
// build 3 (dense): key ranges of at most 8 x the build rows get a direct-addressed table
// of one u32 ref per key value (dense[key - dmin]; kMiss = absent), same ref / dup_rows
// encoding as the buckets. One workgroup builds GV consecutive key values (one block of
// the partition: 2048 values, or 8192 for the one-level partition): refs in LDS, the
// first insert of a key stores its row (atomicExch); a key seen twice switches its
// 2048-value sub-range to the duplicate passes (counts, directory, canonical descending
// segments), whose directory cannot overflow (a sub-range has at most 2048 keys).
// ---------------------------------------------------------------------------
constexpr uint32_t kDenseSub = 1u << kDenseShift;  // values per duplicate-pass sub-range

template <uint32_t GV, int T, int RR>
__global__ void __launch_bounds__(T)
dense_chunk_build_kernel(ChunkGeom g, const uint32_t* __restrict__ starts, const unsigned long long* __restrict__ skeys,
                         const uint32_t* __restrict__ srows, uint32_t* __restrict__ dense,
                         uint32_t* __restrict__ dup_rows, BigSeg* __restrict__ big, BuildCounters* ctr) {
    constexpr uint32_t NSUB = GV / kDenseSub;
    static_assert(GV % kDenseSub == 0, "block of whole sub-ranges");
    __shared__ uint32_t refs[GV];
    __shared__ uint32_t d_off[kDenseSub], d_cur[kDenseSub], d_cnt[kDenseSub];
    __shared__ unsigned s_ndup, s_dup[NSUB];
    __shared__ unsigned long long s_w[T / 64];
    __shared__ unsigned long long s_base;
    const uint32_t c = blockIdx.x;
    const uint32_t start = starts[c], end = starts[c + 1];
    const uint64_t cbase = (uint64_t)c * GV;  // key index of refs[0]
    for (uint32_t i = threadIdx.x; i < GV; i += T) refs[i] = kMiss;
    const bool in_regs = end - start <= (uint32_t)(T * RR);
    if (threadIdx.x < NSUB) s_dup[threadIdx.x] = in_regs ? 0u : 1u;  // more rows than the registers hold
    __syncthreads();
    uint32_t rrow[RR];
    int ridx[RR];
    auto index_of = [&](unsigned long long key) {
        return (int)(((uint64_t)key - (uint64_t)g.dmin) - cbase);
    };
    if (in_regs) {
#pragma unroll
        for (int u = 0; u < RR; ++u) {
            const uint32_t r = start + u * T + threadIdx.x;
            ridx[u] = r < end ? index_of(skeys[r]) : -1;
            rrow[u] = r < end ? srows[r] : 0u;
        }
#pragma unroll
        for (int u = 0; u < RR; ++u)
            if (ridx[u] >= 0 && atomicExch(&refs[ridx[u]], rrow[u]) != kMiss) s_dup[ridx[u] / kDenseSub] = 1u;
    }
    __syncthreads();
    for (uint32_t q = 0; q < NSUB; ++q) {
        if (!s_dup[q]) continue;  // uniform: every thread reads the same LDS word
        const int lo = (int)(q * kDenseSub), hi = lo + (int)kDenseSub;
        uint32_t* img = refs + lo;
        if (threadIdx.x == 0) s_ndup = 0;
        // counts
        for (uint32_t i = threadIdx.x; i < kDenseSub; i += T) img[i] = 0;
        __syncthreads();
        if (in_regs) {
#pragma unroll
            for (int u = 0; u < RR; ++u)
                if (ridx[u] >= lo && ridx[u] < hi) atomicAdd(&refs[ridx[u]], 1u);
        } else {
            for (uint32_t r = start + threadIdx.x; r < end; r += T) {
                const int i = index_of(skeys[r]);
                if (i >= lo && i < hi) atomicAdd(&refs[i], 1u);
            }
        }
        __syncthreads();
        // directory of duplicated keys; absent keys become kMiss before rows are placed
        for (uint32_t i = threadIdx.x; i < kDenseSub; i += T) {
            const uint32_t cnt = img[i];
            if (cnt == 0) {
                img[i] = kMiss;
            } else if (cnt > 1) {
                const unsigned li = atomicAdd(&s_ndup, 1u);
                d_cnt[li] = cnt;
                d_cur[li] = 0;
                img[i] = kDupFlag | li;
            }
        }
        __syncthreads();
        const unsigned ndup = s_ndup;
        unsigned long long carry = 0;
        for (unsigned b0 = 0; b0 < ndup; b0 += T) {
            const unsigned li = b0 + threadIdx.x;
            const unsigned long long v = li < ndup ? (unsigned long long)d_cnt[li] + 1 : 0;
            unsigned long long tot;
            const unsigned long long ex = block_excl_scan<unsigned long long>(v, s_w, &tot);
            if (li < ndup) d_off[li] = (uint32_t)(carry + ex);
            carry += tot;
        }
        if (threadIdx.x == 0) s_base = carry ? atomicAdd(&ctr->dup_used, carry) : 0;
        __syncthreads();
        for (unsigned li = threadIdx.x; li < ndup; li += T) {
            d_off[li] += (uint32_t)s_base;
            dup_rows[d_off[li]] = d_cnt[li];
        }
        __syncthreads();
        auto place = [&](int i, uint32_t row) {
            const uint32_t rv = refs[i];
            if (rv & kDupFlag) {
                const unsigned li = rv & ~kDupFlag;
                dup_rows[d_off[li] + 1 + atomicAdd(&d_cur[li], 1u)] = row;
            } else {
                refs[i] = row;  // count was 1
            }
        };
        if (in_regs) {
#pragma unroll
            for (int u = 0; u < RR; ++u)
                if (ridx[u] >= lo && ridx[u] < hi) place(ridx[u], rrow[u]);
        } else {
            for (uint32_t r = start + threadIdx.x; r < end; r += T) {
                const int i = index_of(skeys[r]);
                if (i >= lo && i < hi) place(i, srows[r]);
            }
        }
        __syncthreads();
        for (unsigned li = threadIdx.x; li < ndup; li += T) {
            const unsigned n = d_cnt[li], off = d_off[li];
            d_cur[li] = 0;  // (the placement cursor is done): a run ref, or 0
            if (n <= (unsigned)kSmallSeg) {
                uint32_t v[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = (i < (int)n) ? dup_rows[off + 1 + i] : 0u;
                sort16_desc(v);
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (i < (int)n) dup_rows[off + 1 + i] = v[i];
                // consecutive rows: the ref holds them (run ref, hj_device.h)
                bool run = g.packed && n <= kRunMaxRows && v[0] < (1u << 24);
#pragma unroll
                for (int i = 1; i < (int)kRunMaxRows; ++i) run &= i >= (int)n || v[i] == v[0] - (uint32_t)i;
                if (run) d_cur[li] = make_run_ref(v[0], n);
            }
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < kDenseSub; i += T) {
            const uint32_t rv = img[i];
            if (rv != kMiss && (rv & kDupFlag)) {
                const unsigned li = rv & ~kDupFlag;
                if (d_cnt[li] > (unsigned)kSmallSeg) {
                    const unsigned bi = (unsigned)atomicAdd(&ctr->n_big, 1ull);
                    big[bi] = BigSeg{(unsigned long long)((uint64_t)g.dmin + cbase + lo + i), d_off[li], 0u};
                }
                const uint32_t c4 = (g.packed && d_cnt[li] <= 15u) ? d_cnt[li] : 0u;
                img[i] = d_cur[li] ? d_cur[li] : kDupFlag | (c4 << 27) | d_off[li];
            }
        }
        __syncthreads();
    }
    // write out (coalesced)
    uint4* dst = reinterpret_cast<uint4*>(dense + cbase);
    const uint4* src = reinterpret_cast<const uint4*>(refs);
    for (uint32_t i = threadIdx.x; i < GV / 4; i += T) dst[i] = src[i];
}

// ---------------------------------------------------------------------------
// build 4: large duplicate segments (> 16 rows; rare). <= 4096 rows: bitonic sort in
// LDS. Larger: rebuild the segment by an ordered scan of the build input (stream
// compaction of the rows equal to the key; deterministic, no scratch).
// ---------------------------------------------------------------------------
constexpr int kBigThreads = 256;
constexpr int kBigLds = 4096;

__global__ void __launch_bounds__(kBigThreads)
dup_sort_big_kernel(uint32_t* dup_rows, const BigSeg* __restrict__ big, const BuildCounters* ctr,
                    const Segment* __restrict__ segs, int nseg, int64_t total, int key_bytes, bool ids_as_rows) {
    __shared__ uint32_t s_v[kBigLds];
    __shared__ unsigned s_wave[kBigThreads / 64];
    const unsigned long long nbig = ctr->n_big;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (unsigned long long bi = blockIdx.x; bi < nbig; bi += gridDim.x) {
        const BigSeg e = big[bi];
        const uint32_t n = dup_rows[e.off];
        uint32_t* rows = dup_rows + e.off + 1;
        if (n <= (unsigned)kBigLds) {
            unsigned N = 1;
            while (N < n) N <<= 1;
            for (unsigned i = threadIdx.x; i < N; i += kBigThreads) s_v[i] = (i < n) ? rows[i] : 0u;
            __syncthreads();
            for (unsigned k = 2; k <= N; k <<= 1) {
                for (unsigned jj = k >> 1; jj > 0; jj >>= 1) {
                    for (unsigned i = threadIdx.x; i < N; i += kBigThreads) {
                        const unsigned l = i ^ jj;
                        if (l > i) {
                            const bool desc = ((i & k) == 0);
                            const uint32_t a = s_v[i], b = s_v[l];
                            if (desc ? (a < b) : (a > b)) { s_v[i] = b; s_v[l] = a; }
                        }
                    }
                    __syncthreads();
                }
            }
            for (unsigned i = threadIdx.x; i < n; i += kBigThreads) rows[i] = s_v[i];
        } else {
            const int64_t key = (int64_t)e.key;
            unsigned long long done = 0;  // rows placed so far (ascending row order)
            int si = 0;
            for (int64_t base = 0; base < total; base += kBigThreads) {
                const int64_t r = base + threadIdx.x;
                bool hit = false;
                uint32_t rv = (uint32_t)r;
                if (r < total) {
                    while (si + 1 < nseg && segs[si + 1].row_base <= r) ++si;
                    const Segment& sg = segs[si];
                    const int64_t i = r - sg.row_base;
                    if (bit_valid(sg.valid, sg.voff, i)) hit = (seg_key(sg, i, key_bytes) == key);
                    if (ids_as_rows) rv = (uint32_t)sg.ids[i];
                }
                const unsigned long long m = __ballot(hit);
                const unsigned below = __popcll(m & ((1ull << lane) - 1));
                if (lane == 0) s_wave[wave] = __popcll(m);
                __syncthreads();
                unsigned woff = 0, tot = 0;
                for (int w = 0; w < kBigThreads / 64; ++w) {
                    if (w < wave) woff += s_wave[w];
                    tot += s_wave[w];
                }
                if (hit) {
                    const unsigned long long rank = done + woff + below;  // ascending rank
                    rows[n - 1 - rank] = rv;                             // descending layout
                }
                done += tot;
                __syncthreads();
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// probe
// ---------------------------------------------------------------------------
constexpr int kProbeThreads = 256;
constexpr int kGroups = 4;                                 // 4 groups x 1024 rows
constexpr int kProbeTile = kProbeThreads * 4 * kGroups;   // 4096 probe rows per tile

typedef long long v2i64 __attribute__((ext_vector_type(2)));

template <typename K, bool NT = false>
__device__ __forceinline__ void load4(const void* keys, int64_t row0, int64_t n, bool vec, int64_t (&k)[4]) {
    const K* kp = reinterpret_cast<const K*>(keys);
    if (vec && row0 + 4 <= n) {
        if constexpr (sizeof(K) == 8) {
            const v2i64* p = reinterpret_cast<const v2i64*>(kp + row0);
            v2i64 a, b;
            if constexpr (NT) {
                a = __builtin_nontemporal_load(p);
                b = __builtin_nontemporal_load(p + 1);
            } else {
                a = p[0];
                b = p[1];
            }
            k[0] = a.x; k[1] = a.y; k[2] = b.x; k[3] = b.y;
        } else {
            const int4 a = *reinterpret_cast<const int4*>(kp + row0);
            k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) k[q] = (row0 + q < n) ? (int64_t)kp[row0 + q] : 0;
    }
}

// count of build rows behind a match ref
__device__ __forceinline__ uint32_t ref_count(const uint32_t* dup_rows, uint32_t ref, uint32_t off_mask) {
    const uint32_t c = ref_count_inline(ref, off_mask);
    return c == kCountUnknown ? dup_rows[ref & off_mask] : c;
}

// One bucket line: ref of `sk` if present, else kMiss; *more = the line is full, does
// not hold the key, and some insert passed it (meta bit 0): look at the next bucket of
// the chunk. Slots fill in order and are never freed, so an empty slot ends a key's probe
// sequence, and so does a full bucket that no insert ever passed. Branch-free.
__device__ __forceinline__ uint32_t scan_line(const uint4& a0, const uint4& a1, const uint4& a2, const uint4& a3,
                                              unsigned long long sk, bool* more, uint32_t* cnt) {
    const unsigned long long k0 = ((unsigned long long)a0.y << 32) | a0.x;
    const unsigned long long k1 = ((unsigned long long)a0.w << 32) | a0.z;
    const unsigned long long k2 = ((unsigned long long)a1.y << 32) | a1.x;
    const unsigned long long k3 = ((unsigned long long)a1.w << 32) | a1.z;
    const unsigned long long k4 = ((unsigned long long)a2.y << 32) | a2.x;
    const bool e0 = k0 == sk, e1 = k1 == sk, e2 = k2 == sk, e3 = k3 == sk, e4 = k4 == sk;
    const bool z = (k0 == 0) | (k1 == 0) | (k2 == 0) | (k3 == 0) | (k4 == 0);
    uint32_t ref = e4 ? a3.z : kMiss;
    ref = e3 ? a3.y : ref;
    ref = e2 ? a3.x : ref;
    ref = e1 ? a2.w : ref;
    ref = e0 ? a2.z : ref;
    *more = (ref == kMiss) & !z & ((a3.w & 1u) != 0);
    // row count: 0 miss, 1 single row, the inline meta count of a duplicated key, or
    // kCountUnknown (read dup_rows[off])
    const uint32_t m = a3.w;
    uint32_t c = e4 ? (m >> 25) : 0u;
    c = e3 ? (m >> 19) : c;
    c = e2 ? (m >> 13) : c;
    c = e1 ? (m >> 7) : c;
    c = e0 ? (m >> 1) : c;
    c &= 63u;
    *cnt = ref == kMiss ? 0u : (!(ref & kDupFlag) ? 1u : (c ? c : kCountUnknown));
    return ref;
}

// Refs of the four probe rows row0..row0+3 (kMiss: no match, null, or past n).
template <typename K, bool HAS_VALID, bool NT = false>
__device__ __forceinline__ void lookup4(const TableView& tv, const void* __restrict__ keys,
                                        const uint8_t* __restrict__ valid, int64_t voff, int64_t n, bool vec,
                                        int64_t row0, uint32_t (&ref)[4], uint32_t (&cnt)[4]) {
    if (tv.dense != nullptr) {  // direct-addressed table: range check + one 4-byte read per row
        int64_t k[4];
        load4<K, NT>(keys, row0, n, vec, k);
        uint32_t r[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool in = (row0 + q < n) && (!HAS_VALID || bit_valid(valid, voff, row0 + q));
            const uint64_t idx = (uint64_t)k[q] - (uint64_t)tv.dmin;
            r[q] = (in && idx < tv.drange) ? tv.dense[idx] : kMiss;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ref[q] = r[q];
            // packed dense refs carry counts <= 15 (or a run) in bits 24-30 (kPackedMask tables)
            cnt[q] = ref_count_inline(r[q], tv.off_mask);
        }
        return;
    }
    const Bucket* __restrict__ tbl = tv.tbl;
    const uint32_t cmask = (1u << tv.clog2) - 1;
    int64_t k[4];
    load4<K, NT>(keys, row0, n, vec, k);
    bool in[4];
    unsigned long long sk[4];
    uint32_t b[4];
    uint4 L0[4], L1[4], L2[4], L3[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        in[q] = (row0 + q < n) && (!HAS_VALID || bit_valid(valid, voff, row0 + q));
        sk[q] = stored_key(k[q]);
        b[q] = (in[q] && sk[q] != 0) ? stored_bucket(sk[q], tv.nb) : tv.nb;
    }
    // issue the 64-byte bucket line of all four rows before any compare (MLP)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint4* p = reinterpret_cast<const uint4*>(tbl + b[q]);
        L0[q] = p[0]; L1[q] = p[1]; L2[q] = p[2]; L3[q] = p[3];
    }
    bool more[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        ref[q] = scan_line(L0[q], L1[q], L2[q], L3[q], sk[q], &more[q], &cnt[q]);
        if (sk[q] == 0) {  // key 0: the side bucket (ref[0] = word 10, meta = word 15 = rows)
            ref[q] = L3[q].w ? L2[q].z : kMiss;
            cnt[q] = L3[q].w;
            more[q] = false;
        }
        if (!in[q]) { ref[q] = kMiss; cnt[q] = 0; more[q] = false; }
    }
    // rare: the home line is full and does not hold the key
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t bb = b[q];
        for (uint32_t probes = 0; more[q] && probes < cmask; ++probes) {
            bb = (bb & ~cmask) | ((bb + 1) & cmask);
            const uint4* p = reinterpret_cast<const uint4*>(tbl + bb);
            ref[q] = scan_line(p[0], p[1], p[2], p[3], sk[q], &more[q], &cnt[q]);
        }
    }
}

__device__ __forceinline__ uint32_t resolve_count(const uint32_t* dup_rows, uint32_t ref, uint32_t cnt,
                                                  uint32_t off_mask) {
    return cnt == kCountUnknown ? dup_rows[ref & off_mask] : cnt;
}

// Writes the pairs of four probe rows starting at output position `pos` (canonical:
// rows ascending, each row's build rows descending = the order of its dup segment).
template <bool HAS_ROW_IDS, bool HAS_PROBE_IDS>
__device__ __forceinline__ void emit4(const TableView& tv, const uint32_t* __restrict__ probe_ids, uint32_t pbase,
                                      int64_t row0,
                                      const uint32_t (&ref)[4], const uint32_t (&cnt)[4], unsigned long long pos,
                                      uint64_t* __restrict__ out_b, uint32_t* __restrict__ out_p, int64_t cap) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t c = cnt[q];
        if (c == 0) continue;
        const int64_t prow = row0 + q;
        const uint32_t pidx = HAS_PROBE_IDS ? probe_ids[prow] : (uint32_t)prow + pbase;
        const uint32_t r = ref[q];
        if (c == 1) {
            if (pos < (unsigned long long)cap) {
                const uint32_t br = (r & kDupFlag) ? dup_ref_row(tv.dup_rows, r, tv.off_mask, 0) : r;
                out_b[pos] = HAS_ROW_IDS ? tv.row_ids[br] : (uint64_t)br;
                out_p[pos] = pidx;
            }
        } else {
            for (uint32_t t = 0; t < c; ++t) {
                if (pos + t < (unsigned long long)cap) {
                    const uint32_t br = dup_ref_row(tv.dup_rows, r, tv.off_mask, t);
                    out_b[pos + t] = HAS_ROW_IDS ? tv.row_ids[br] : (uint64_t)br;
                    out_p[pos + t] = pidx;
                }
            }
        }
        pos += c;
    }
}

// ---------------------------------------------------------------------------
// fused probe (default): lookup + ordered emission in one launch. A tile's output
// offset comes from a decoupled look-back over the per-tile flags in blockIdx order:
// flag = status (2 bits: 1 aggregate, 2 inclusive prefix) | 62-bit value. Workgroups
// are dispatched in blockIdx order on every XCD, so the lowest unfinished tile is
// always resident and the look-back makes progress; the spin is still bounded and a
// give-up raises the workspace error word instead of hanging. No ticket atomics: the
// flags are written once each, by their own tile.
// ---------------------------------------------------------------------------
constexpr unsigned long long kFlagAgg = 1ull << 62;
constexpr unsigned long long kFlagIncl = 2ull << 62;
constexpr unsigned long long kFlagVal = (1ull << 62) - 1;
constexpr unsigned kLookbackSpinLimit = 1u << 22;
constexpr int kStage = 2048;          // pairs per LDS emission window (16 KB + the 16 KB s_ref)
constexpr int kStageMaxWindows = 8;   // beyond this a group's pairs are stored directly

__device__ __forceinline__ unsigned long long flag_load(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void flag_store(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 of tile t: exclusive prefix of the tile counts before t (t > 0)
__device__ unsigned long long lookback(unsigned long long* flags, int64_t t, unsigned long long* err) {
    const int lane = threadIdx.x & 63;
    unsigned long long excl = 0;
    int64_t j = t - 1;
    unsigned spins = 0;
    while (true) {
        const int64_t idx = j - lane;
        const unsigned long long f = idx >= 0 ? flag_load(flags + idx) : kFlagIncl;
        const unsigned long long st = f >> 62;
        const unsigned long long incl_mask = __ballot(st == 2);
        const unsigned long long zero_mask = __ballot(st == 0);
        const int first = incl_mask ? __ffsll((long long)incl_mask) - 1 : 63;
        const unsigned long long need = (2ull << first) - 1;  // lanes 0..first (first = 63: all)
        if (zero_mask & need) {
            if (++spins > kLookbackSpinLimit) {  // never expected: report, do not hang
                if (lane == 0) atomicOr(err, 1ull);
                return excl;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += wave_sum<unsigned long long>(lane <= first ? (f & kFlagVal) : 0ull);
        if (incl_mask) return excl;
        j -= 64;
    }
}

template <typename K, bool HAS_VALID, bool HAS_ROW_IDS, bool HAS_PROBE_IDS>
__global__ void __launch_bounds__(kProbeThreads)
probe_fused_kernel(TableView tv, const void* __restrict__ keys, const uint8_t* __restrict__ valid, int64_t voff,
                   const uint32_t* __restrict__ probe_ids, uint32_t pbase, int64_t n, bool vec,
                   unsigned long long* flags, unsigned long long* err, uint64_t* __restrict__ out_b,
                   uint32_t* __restrict__ out_p, int64_t cap, int64_t* __restrict__ d_total, int nt) {
    // the tile's refs wait in LDS across the look-back (registers stay free for the
    // lookups' line loads: occupancy is what keeps enough random reads in flight)
    __shared__ __attribute__((aligned(16))) uint32_t s_ref[kProbeTile];
    __shared__ uint64_t s_b[kStage];
    __shared__ unsigned long long s_w[kGroups][kProbeThreads / 64];
    __shared__ unsigned long long s_excl;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t tile0 = (int64_t)blockIdx.x * kProbeTile;
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
        const int64_t row0 = tile0 + (int64_t)g * (kProbeThreads * 4) + (int64_t)threadIdx.x * 4;
        uint32_t ref[4] = {kMiss, kMiss, kMiss, kMiss}, cnt[4] = {0, 0, 0, 0};
        if (row0 < n) {
            if (nt & 1) lookup4<K, HAS_VALID, true>(tv, keys, valid, voff, n, vec, row0, ref, cnt);
            else lookup4<K, HAS_VALID, false>(tv, keys, valid, voff, n, vec, row0, ref, cnt);
        }
        *reinterpret_cast<uint4*>(s_ref + g * (kProbeThreads * 4) + threadIdx.x * 4) =
            make_uint4(ref[0], ref[1], ref[2], ref[3]);
        unsigned long long s = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) s += resolve_count(tv.dup_rows, ref[q], cnt[q], tv.off_mask);
        const unsigned long long ws = wave_sum<unsigned long long>(s);
        if (lane == 0) s_w[g][wave] = ws;
    }
    __syncthreads();
    if (wave == 0) {
        unsigned long long tile_total = 0;
#pragma unroll
        for (int g = 0; g < kGroups; ++g)
            for (int w = 0; w < kProbeThreads / 64; ++w) tile_total += s_w[g][w];
        unsigned long long excl = 0;
        if (blockIdx.x == 0) {
            if (lane == 0) flag_store(flags, kFlagIncl | tile_total);
        } else {
            if (lane == 0) flag_store(flags + blockIdx.x, kFlagAgg | tile_total);
            excl = lookback(flags, blockIdx.x, err);
            if (lane == 0) flag_store(flags + blockIdx.x, kFlagIncl | (excl + tile_total));
        }
        if (lane == 0) {
            s_excl = excl;
            if (blockIdx.x == gridDim.x - 1) *d_total = (int64_t)(excl + tile_total);
        }
    }
    __syncthreads();
    // emission, staged through LDS per group of 1024 rows: each thread drops its pairs
    // into the window [w0, w0 + kStage) of the group's output, then the block copies the
    // window out contiguously (whole lines, no partial-line stores left to merge in an
    // L2 that the random bucket reads keep evicting). Groups with more than
    // kStageMaxWindows windows of output (heavy duplicates) store directly.
    uint32_t ref[kGroups][4];
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
        const uint4 r4 = *reinterpret_cast<const uint4*>(s_ref + g * (kProbeThreads * 4) + threadIdx.x * 4);
        ref[g][0] = r4.x; ref[g][1] = r4.y; ref[g][2] = r4.z; ref[g][3] = r4.w;
    }
    __syncthreads();  // s_ref is reused as the probe-index half of the staging window
    uint32_t* s_p = s_ref;
    unsigned long long gbase = s_excl;
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
        const int64_t row0 = tile0 + (int64_t)g * (kProbeThreads * 4) + (int64_t)threadIdx.x * 4;
        uint32_t cnt[4];
        unsigned long long c_sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            cnt[q] = ref_count(tv.dup_rows, ref[g][q], tv.off_mask);
            c_sum += cnt[q];
        }
        unsigned long long lpos = wave_incl_scan<unsigned long long>(c_sum) - c_sum;  // inside the group
        unsigned long long gt = 0;
        for (int w = 0; w < kProbeThreads / 64; ++w) {
            if (w < wave) lpos += s_w[g][w];
            gt += s_w[g][w];
        }
        if (gt > (unsigned long long)kStage * kStageMaxWindows) {
            if (row0 < n)
                emit4<HAS_ROW_IDS, HAS_PROBE_IDS>(tv, probe_ids, pbase, row0, ref[g], cnt, gbase + lpos, out_b, out_p, cap);
        } else {
            for (unsigned long long w0 = 0; w0 < gt; w0 += kStage) {
                const unsigned long long w1 = w0 + kStage;
                unsigned long long p = lpos;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t c = cnt[q];
                    const unsigned long long a = p > w0 ? p : w0;
                    const unsigned long long b = (p + c) < w1 ? (p + c) : w1;
                    if (a < b) {
                        const uint32_t r = ref[g][q];
                        const uint32_t pidx = HAS_PROBE_IDS ? probe_ids[row0 + q] : (uint32_t)(row0 + q) + pbase;
                        const bool dup = (r & kDupFlag) != 0;
                        for (unsigned long long t = a; t < b; ++t) {
                            const uint32_t br = dup ? dup_ref_row(tv.dup_rows, r, tv.off_mask, (uint32_t)(t - p)) : r;
                            s_b[t - w0] = HAS_ROW_IDS ? tv.row_ids[br] : (uint64_t)br;
                            s_p[t - w0] = pidx;
                        }
                    }
                    p += c;
                }
                __syncthreads();
                const unsigned long long len = (gt - w0) < (unsigned long long)kStage ? (gt - w0) : kStage;
                const unsigned long long o = gbase + w0;
                for (unsigned i = threadIdx.x; i < len; i += kProbeThreads) {
                    if (o + i < (unsigned long long)cap) {
                        if (nt & 2) {
                            __builtin_nontemporal_store(s_b[i], out_b + o + i);
                            __builtin_nontemporal_store(s_p[i], out_p + o + i);
                        } else {
                            out_b[o + i] = s_b[i];
                            out_p[o + i] = s_p[i];
                        }
                    }
                }
                __syncthreads();
            }
        }
        gbase += gt;
    }
}

// ---------------------------------------------------------------------------
// sliced probe (direct-addressed tables of <= kSlMaxSlices x 2^wlog key values): the
// lookups run out of LDS instead of as random device reads. The fused probe does one
// random 4-byte read per in-range probe row and is bound by the memory system's random
// request rate (~57 G/s for an Infinity-Cache-resident table); LDS serves
// random reads at >10x that. The launches:
//   S1  sl_partition_kernel   per 16384-row tile: counting sort of the in-range rows by
//                             slice (2^wlog consecutive key values) in LDS; writes, in
//                             slice order into the tile's region, each row's key offset
//                             in its slice (u16) and row in the tile (u16), and the tile's
//                             slice bounds (u16, tile-major)
//   S2  sl_lookup_kernel      per (slice, tile range), XCD-contiguous item order: the
//                             slice's refs in LDS, then every tile's fragment of that
//                             slice; each entry's ref goes to the refs array (u32) at the
//                             entry's position. The probe waits for a build on another
//                             stream only here (S1/S1b read no table memory).
//   (counts)                  S1 writes a tile's entries as its pair count; S2 adds
//                             count - 1 for every entry whose key is missing or
//                             duplicated (LDS atomics per owner tile, then one atomic per
//                             tile and run), so no pass re-reads the refs to count them.
//                             S3 sums the counts below its tiles itself (no scan launch;
//                             a decoupled look-back inside S3 measured slower: 350 vs 212
//                             us at C2, a tile's offset then waits for the slowest
//                             workgroup holding an earlier tile).
//   S3b sl_emit_kernel        per tile (persistent, prefetching): its (row, ref) pairs
//                             scattered into an LDS image of the tile's refs, then ordered
//                             emission, 64 rows per wave step, one contiguous store run
//                             per step (duplicates expanded over the lanes)
// Pairs are identical to the fused probe's (canonical order); only where the table
// lookups happen changes. The dense build reuses S1/S1b on the build keys (8192-value
// slices), and dense_frag_build_kernel gathers each block's rows from the fragments.
// ---------------------------------------------------------------------------
constexpr int kSlThreads = 1024;
constexpr int kSlTileLog = 14;
constexpr int kSlTile = 1 << kSlTileLog;                // probe rows per tile
constexpr int kSlGroups = kSlTile / (kSlThreads * 4);  // 4 groups of 4096 rows
constexpr int kSlWidthLogMax = 15;                      // key values per slice: 2^wlog <= 32768 (128 KB of refs)
constexpr int kSlHistBins = 4096;                       // per-tile slice histogram in LDS (16 KB)
constexpr int kSlMaxSlices = kSlHistBins - 1;           // slices per pass: key ranges up to ~2^27 values
constexpr int kSlOwnWin = 2048;        // flattened segment positions per owner window (32 per lane)
constexpr int kSlOwnWinHashed = 1024;  // hashed slices: 16 per lane (u64 entries)
// hashed slices with 2^15-row tiles: a 64-tile block holds ~1075 positions at C2h (16.8 per
// fragment), so 1152-position windows take most blocks in one window (r05: C2h lookup 597 ->
// 566 us, bench 65.5-66.1K -> 66.1-66.5K Mrows/s against 1024, profiles/r05_hs_window_ab.txt)
constexpr int kSlOwnWinHashed15 = 1152;
template <int TL> constexpr int hs_own_win() { return TL == 15 ? kSlOwnWinHashed15 : kSlOwnWinHashed; }
// the emission's waves own 2048-row ranges of a tile: the partition counts each range's
// entries (wcnt) so that a tile whose entries all hit one unique row each (no correction
// flag from the lookup) needs no count pass in the emission
constexpr int kSlRanges = 8;
constexpr int kSlRangeRows = kSlTile / kSlRanges;  // 2048
// The probe's tiles: 2^14 rows (kSlTile, also the builds') or 2^15 (DFP_HJ_SL_TILE_LOG=15:
// half the (tile, slice) fragments for the lookup to walk, each twice as long; the
// partition and the emission then run one 1024-thread workgroup per CU with a 128 KB
// image). Per tile log TL: rows, 4096-row partition groups, 2048-row emission ranges.
template <int TL> struct SlT {
    static_assert(TL == 14 || TL == 15, "probe tiles of 2^14 or 2^15 rows");
    static constexpr int kRows = 1 << TL;
    static constexpr int kGroups = kRows / (kSlThreads * 4);
    static constexpr int kRanges = kRows / kSlRangeRows;
    static constexpr int kEmitThreads = kRanges * 64;  // one emission wave per range
};
static_assert(kSlWidthLogMax + kSlTileLog <= 32, "entry = offset << tile bits | row");
static_assert(kSlWidthLogMax <= 16 && kSlTileLog <= 16, "key offsets and rows leave as u16");

// in-place exclusive scan of a tile's kSlHistBins slice counts (kSlThreads threads, four
// bins each); *tot = the tile's rows. Ends with a barrier.
static_assert(kSlHistBins == 4 * kSlThreads, "four bins per thread");
__device__ __forceinline__ void hist_excl_scan(uint32_t* s_hist, uint32_t* s_w, uint32_t* tot) {
    const uint32_t b0 = threadIdx.x * 4;
    const uint4 h = *reinterpret_cast<const uint4*>(s_hist + b0);
    const uint32_t ex = block_excl_scan<uint32_t>(h.x + h.y + h.z + h.w, s_w, tot);
    *reinterpret_cast<uint4*>(s_hist + b0) = make_uint4(ex, ex + h.x, ex + h.x + h.y, ex + h.x + h.y + h.z);
    __syncthreads();
}

constexpr int kSlPrefetch15 = 3;  // 2^15-row partition tiles: groups of keys in flight ahead of the ranked one
// hist_excl_scan without the per-wave loop over the wave totals (lane w < 16 holds wave w's
// total; a DPP scan and two readlanes): the persistent 2^15-row partition, whose unrolled
// loop there spilled
__device__ __forceinline__ void hist_excl_scan_lanes(uint32_t* s_hist, uint32_t* s_w, uint32_t* tot) {
    static_assert(kSlThreads / 64 <= 64, "wave totals in one wave's lanes");
    const uint32_t b0 = threadIdx.x * 4;
    const uint4 h = *reinterpret_cast<const uint4*>(s_hist + b0);
    const uint32_t v = h.x + h.y + h.z + h.w;
    const uint32_t incl = wave_incl_scan_dpp(v);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    const uint32_t wt = wave_incl_scan_dpp(lane < kSlThreads / 64 ? s_w[lane] : 0u);
    const uint32_t off = wave > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)wt, wave - 1) : 0u;
    *tot = (uint32_t)__builtin_amdgcn_readlane((int)wt, kSlThreads / 64 - 1);
    const uint32_t ex = off + incl - v;
    *reinterpret_cast<uint4*>(s_hist + b0) = make_uint4(ex, ex + h.x, ex + h.x + h.y, ex + h.x + h.y + h.z);
    __syncthreads();
}

template <typename K, bool HAS_VALID, int TL = kSlTileLog>
// 2^14-row tiles: 8 waves per SIMD = two workgroups per CU, <= 64 VGPRs; 2^15: one (128 KB of LDS)
__global__ void __launch_bounds__(kSlThreads, TL == 14 ? 8 : 4)
sl_partition_kernel(int64_t dmin, uint64_t drange, uint32_t wlog, uint32_t nslices, const void* __restrict__ keys,
                    const uint8_t* __restrict__ valid, int64_t voff, int64_t n, bool vec,
                    uint16_t* __restrict__ ko, uint16_t* __restrict__ rl, uint16_t* __restrict__ toff, int nt,
                    int64_t tile_off, int64_t row_base, uint32_t* __restrict__ tile_base,
                    unsigned long long* __restrict__ hdr,  // probe: workspace header (error word at [1]); build: null
                    unsigned long long* __restrict__ tcnt,      // probe: the tile's entry count; build: null
                    uint32_t* __restrict__ tent,  // probe: entries of the tile so far (earlier passes: append after them)
                    uint16_t* __restrict__ wcnt,  // probe: entries per 2048-row range of the tile (T::kRanges u16)
                    SpecGeo sg) {  // build with the key range on the device (mm null: dmin, drange, nslices given)
    using T = SlT<TL>;
    __shared__ __attribute__((aligned(16))) uint32_t s_ent[T::kRows];
    if (sg.mm != nullptr) {  // (uniform) the geometry from the reduction's result; none: another layout
        const long long mn = sg.mm[0], mx = sg.mm[1];
        const uint32_t nb = spec_dense_blocks(mn, mx, sg.rows, sg.cap);
        if (nb == 0) return;
        dmin = mn;
        nslices = nb;
        drange = (uint64_t)nb << wlog;
    }
    __shared__ __attribute__((aligned(16))) uint32_t s_hist[kSlHistBins];  // bins 0..nslices (<= kSlMaxSlices + 1)
    // the scan's wave totals and the per-range entry counts alias the entry staging area
    // (free until the scatter), so the workgroup stays within 80 KB: two per CU
    uint32_t* s_w = s_ent;
    uint32_t* s_wc = s_ent + kSlThreads / 64;
    const int64_t tile = blockIdx.x;          // tile of this key array
    const int64_t gtile = tile + tile_off;    // its output region (the build partitions several arrays)
    const int64_t tile0 = tile * T::kRows;
    const uint32_t nbins = nslices + 1;  // bin nslices stays empty: its prefix is the total
    // multi-pass probe (tables beyond kSlMaxSlices slices): this pass's entries follow the
    // tile's entries of the earlier passes (hdr == null marks a later pass)
    const uint32_t ebase = (tent != nullptr && hdr == nullptr) ? tent[gtile] : 0u;
    for (uint32_t b = threadIdx.x; b < kSlHistBins; b += kSlThreads) s_hist[b] = 0;
    if (threadIdx.x < T::kRanges) s_wc[threadIdx.x] = 0;
    // probe: zero the workspace header incl. the error word (no memset launch)
    // (and the emission's tile counter after the tile counts: one tile per workgroup here)
    if (hdr != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
        hdr[0] = hdr[1] = 0;
        tcnt[gridDim.x] = 0;
    }
    __syncthreads();
    // per row: entry (offset << 14 | row) and (slice << 14 | rank in slice), ~0 = no entry
    uint32_t e[T::kGroups][4], sr[T::kGroups][4];
    // the next group's keys load while this group's rows are ranked (one load round trip
    // per tile instead of one per group; two groups of keys fit the 64-register budget).
    // A whole aligned tile takes straight 16-byte loads with no branch between the groups
    // (a branch would make the next group's loads wait at its join).
    auto groups = [&](auto full_tag) {
        constexpr bool FULL = decltype(full_tag)::value;
        auto load_group = [&](int g, int64_t (&dst)[4]) {
            const int loc0 = g * (kSlThreads * 4) + threadIdx.x * 4;
            if constexpr (FULL && sizeof(K) == 8) {
                const v2i64* p = reinterpret_cast<const v2i64*>(reinterpret_cast<const K*>(keys) + tile0 + loc0);
                const v2i64 a = p[0], b = p[1];
                dst[0] = a.x; dst[1] = a.y; dst[2] = b.x; dst[3] = b.y;
            } else if constexpr (FULL) {
                const int4 a = *reinterpret_cast<const int4*>(reinterpret_cast<const K*>(keys) + tile0 + loc0);
                dst[0] = a.x; dst[1] = a.y; dst[2] = a.z; dst[3] = a.w;
            } else if (nt & 1) {
                load4<K, true>(keys, tile0 + loc0, n, vec, dst);
            } else {
                load4<K>(keys, tile0 + loc0, n, vec, dst);
            }
        };
        // groups in flight ahead of the one being ranked: 1 at 2^14-row tiles (32 waves per
        // CU), kSlPrefetch15 at 2^15 (16 waves per CU hold fewer loads in flight per CU)
        constexpr int D = TL == 14 ? 1 : kSlPrefetch15;
        int64_t kr[D + 1][4];  // ring of groups: group g in slot g % (D + 1)
#pragma unroll
        for (int g = 0; g < D && g < T::kGroups; ++g) load_group(g, kr[g]);
#pragma unroll
        for (int g = 0; g < T::kGroups; ++g) {
            const int loc0 = g * (kSlThreads * 4) + threadIdx.x * 4;
            int64_t k[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) k[q] = kr[g % (D + 1)][q];
            if (g + D < T::kGroups) load_group(g + D, kr[(g + D) % (D + 1)]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t row = tile0 + loc0 + q;
                const uint64_t idx = (uint64_t)k[q] - (uint64_t)dmin;
                const bool ok = row < n && (!HAS_VALID || bit_valid(valid, voff, row)) && idx < drange;
                const uint32_t sl = (uint32_t)(idx >> wlog);
                e[g][q] = ((uint32_t)(idx & ((1u << wlog) - 1)) << TL) | (uint32_t)(loc0 + q);
                sr[g][q] = ok ? (sl << TL) | atomicAdd(&s_hist[sl], 1u) : 0xFFFFFFFFu;
            }
            if (wcnt != nullptr) {  // probe: entries per emission range (a wave's rows of one group share a range)
                uint32_t ws = 0;    // the wave's entries in group g: scalar popcounts of the entry ballots
#pragma unroll
                for (int q = 0; q < 4; ++q) ws += (uint32_t)__popcll(__ballot(sr[g][q] != 0xFFFFFFFFu));
                if ((threadIdx.x & 63) == 0 && ws) atomicAdd(&s_wc[(g * (kSlThreads * 4) + threadIdx.x * 4) / kSlRangeRows], ws);
            }
        }
    };
    if (vec && tile0 + T::kRows <= n && !(nt & 1)) groups(std::true_type{});
    else groups(std::false_type{});
    __syncthreads();
    // the range counts leave s_ent before the scan's barriers (its wave totals use s_ent[0, 16))
    const uint32_t my_wc = (wcnt != nullptr && threadIdx.x < T::kRanges) ? s_wc[threadIdx.x] : 0u;
    // exclusive scan of the bins, four per thread
    uint32_t tot;
    hist_excl_scan(s_hist, s_w, &tot);
    if (wcnt != nullptr && threadIdx.x < T::kRanges) {
        uint16_t* wc = wcnt + gtile * T::kRanges + threadIdx.x;
        *wc = (uint16_t)((ebase ? *wc : 0u) + my_wc);
    }
    uint16_t* to = toff + gtile * (int64_t)nbins;
    for (uint32_t b = threadIdx.x; b < nbins; b += kSlThreads) to[b] = (uint16_t)(ebase + s_hist[b]);
    if (tile_base != nullptr && threadIdx.x == 0) tile_base[gtile] = (uint32_t)(row_base + tile0);  // build only
    // probe: the tile's pair count starts as its entries (in-range rows); S2 adds count - 1
    // for every entry whose key is missing (-1) or duplicated (+count - 1). A later pass
    // adds its entries to the count the earlier passes (and their lookups) left.
    if (tcnt != nullptr && threadIdx.x == 0) tcnt[gtile] = (ebase ? tcnt[gtile] : 0ull) + tot;
    if (tent != nullptr && threadIdx.x == 0) tent[gtile] = ebase + tot;
#pragma unroll
    for (int g = 0; g < T::kGroups; ++g)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (sr[g][q] != 0xFFFFFFFFu)
                s_ent[s_hist[sr[g][q] >> TL] + (sr[g][q] & (T::kRows - 1))] = e[g][q];
    __syncthreads();
    // entries leave split: the key offset in the slice (u16, read by S2) and the row in
    // the tile (u16, read by S3)
    uint16_t* dst = ko + gtile * T::kRows;
    uint16_t* dsr = rl + gtile * T::kRows;
    if (ebase != 0) {  // a later pass: unaligned base, one entry per thread (2-byte stores)
        for (uint32_t i = threadIdx.x; i < tot; i += kSlThreads) {
            const uint32_t v = s_ent[i];
            dst[ebase + i] = (uint16_t)(v >> TL);
            dsr[ebase + i] = (uint16_t)(v & (T::kRows - 1));
        }
        return;
    }
    const uint32_t n4 = tot & ~3u;
    for (uint32_t i = threadIdx.x * 4; i < n4; i += kSlThreads * 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(s_ent + i);
        constexpr uint32_t m = T::kRows - 1;
        *reinterpret_cast<uint2*>(dst + i) = make_uint2((v.x >> TL) | ((v.y >> TL) << 16),
                                                        (v.z >> TL) | ((v.w >> TL) << 16));
        *reinterpret_cast<uint2*>(dsr + i) = make_uint2((v.x & m) | ((v.y & m) << 16), (v.z & m) | ((v.w & m) << 16));
    }
    if (threadIdx.x < (tot & 3u)) {
        const uint32_t v = s_ent[n4 + threadIdx.x];
        dst[n4 + threadIdx.x] = (uint16_t)(v >> TL);
        dsr[n4 + threadIdx.x] = (uint16_t)(v & (T::kRows - 1));
    }
}

// Build (S1b): the tiles' segment bounds transposed into blocks of 64 tiles, toffT[b][slice][64],
// so that a lookup wave reads the bounds of its 64 tiles with one coalesced 128-byte load
// (tile-major, every lane's bound is its own memory request). Tiles past ntiles read as
// empty.
constexpr int kSlTrChunk = 64;  // slices per block: grid = tile blocks x slice chunks
__global__ void __launch_bounds__(256)
sl_toff_transpose_kernel(const uint16_t* __restrict__ toff, uint32_t nbins, int64_t ntiles,
                         uint16_t* __restrict__ toffT, SpecGeo sg) {
    __shared__ uint16_t s_t[64][kSlTrChunk + 2];
    if (sg.mm != nullptr) {  // (uniform) bins from the reduction's result; the grid covers the widest
        const uint32_t nb = spec_dense_blocks(sg.mm[0], sg.mm[1], sg.rows, sg.cap);
        if (nb == 0) return;
        nbins = nb + 1;
    }
    const uint32_t nch = (nbins + kSlTrChunk - 1) / kSlTrChunk;
    const int64_t b = blockIdx.x / nch;
    if (b * 64 >= ntiles) return;  // (uniform) past the tiles: a grid sized for more bins
    const uint32_t c0 = (blockIdx.x % nch) * kSlTrChunk;
    const uint32_t cw = min<uint32_t>(kSlTrChunk, nbins - c0);
    for (uint32_t i = threadIdx.x; i < 64 * kSlTrChunk; i += 256) {
        const uint32_t j = i / kSlTrChunk, c = i % kSlTrChunk;
        const int64_t t = b * 64 + j;
        if (c < cw) s_t[j][c] = t < ntiles ? toff[t * nbins + c0 + c] : (uint16_t)0;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 64 * kSlTrChunk; i += 256) {
        const uint32_t c = i / 64, j = i % 64;
        if (c < cw) toffT[(b * nbins + c0 + c) * 64 + j] = s_t[j][c];
    }
}

// ---------------------------------------------------------------------------
// build (dense, <= 2047 blocks of 8192 key values, <= kFragMaxTiles tiles): the probe's
// tile-local partition (sl_partition_kernel, 8192-value slices) replaces the histogram,
// scan and staged scatter; each block then gathers its rows from every tile's fragment
// (bounds in the transposed layout, one block-wide scan over the tiles, owner tile of a
// position by binary search in LDS) and builds exactly as dense_chunk_build_kernel.
// ---------------------------------------------------------------------------
// Blocks are dispatched round-robin over the 8 XCDs (block b on XCD b % 8). Work item of
// block b: the XCD's own contiguous range of items, so that the blocks resident on one
// XCD at a time take consecutive slices — whose fragments of a tile are adjacent in
// memory and share lines in that XCD's L2.
__device__ __forceinline__ uint32_t xcd_item(uint32_t b, uint32_t grid) {
    const uint32_t x = b & 7, local = b >> 3, q = grid >> 3, r = grid & 7;
    return x < r ? x * (q + 1) + local : r * (q + 1) + (x - r) * q + local;
}

constexpr int kFragMaxTiles = 2048;
static_assert(kSlTile == kFragTileRows, "build tiles are the probe's tiles");

template <int T, int RR>
__global__ void __launch_bounds__(T)
dense_frag_build_kernel(ChunkGeom g, uint32_t nblk, int64_t ntiles, const uint16_t* __restrict__ toffT,
                        const uint16_t* __restrict__ ko, const uint16_t* __restrict__ rl,
                        const uint32_t* __restrict__ tile_base, const uint64_t* __restrict__ ids32,
                        uint32_t* __restrict__ dense, uint32_t* __restrict__ dup_rows, BigSeg* __restrict__ big,
                        BuildCounters* ctr, unsigned long long* __restrict__ spill, uint32_t run, SpecGeo sg) {
    constexpr uint32_t GV = kDenseSub << kDenseBlockShift;  // 8192 values per block
    static_assert(GV == kDenseBlockValues, "frag-build blocks");
    constexpr uint32_t NSUB = GV / kDenseSub;
    __shared__ uint32_t refs[GV];
    if (sg.mm != nullptr) {  // (uniform) blocks from the reduction's result; the grid covers `cap`
        const uint32_t nb = spec_dense_blocks(sg.mm[0], sg.mm[1], sg.rows, sg.cap);
        if (blockIdx.x >= nb) return;
        g.dmin = sg.mm[0];
        nblk = nb;
    }
    __shared__ uint32_t d_off[kDenseSub], d_cur[kDenseSub], d_cnt[kDenseSub];
    __shared__ uint32_t s_to[kFragMaxTiles + 1];  // exclusive position of each tile's fragment
    __shared__ uint32_t s_pb[kFragMaxTiles];      // fragment position - s_to (region offset)
    __shared__ unsigned s_ndup, s_dup[NSUB];
    __shared__ unsigned long long s_w[T / 64];
    __shared__ unsigned long long s_base, s_sp;
    __shared__ uint32_t s_carry;
    __shared__ uint32_t s_qo[NSUB + 1], s_qc[NSUB];  // spilled rows: each duplicate sub-range's start, fill
    // key block (slice): runs of `run` consecutive blocks per XCD (blocks are dispatched
    // round-robin over the 8 XCDs), so that the blocks resident on one XCD at once read
    // adjacent fragments of each tile (shared lines in that XCD's L2) while the runs still
    // interleave over the XCDs. A whole XCD-contiguous order puts the skewed distributions'
    // heavy low blocks on one XCD (C3 build 0.35 -> 0.76 ms). The last partial group of
    // 8 * run blocks keeps the plain order.
    const uint32_t c = [&] {
        const uint32_t b = blockIdx.x, grp = 8u * run;
        if (run <= 1 || b >= nblk / grp * grp) return b;
        const uint32_t l = b >> 3;
        return (l / run) * grp + (b & 7u) * run + l % run;
    }();
    const uint64_t cbase = (uint64_t)c * GV;  // key index of refs[0]
    const uint32_t nbins = nblk + 1;
    for (uint32_t i = threadIdx.x; i < GV; i += T) refs[i] = kMiss;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    // fragment bounds of this block in every tile -> exclusive positions (block scan)
    for (int64_t t0 = 0; t0 < ntiles; t0 += T) {
        const int64_t t = t0 + threadIdx.x;
        uint32_t st = 0, len = 0;
        if (t < ntiles) {
            const uint16_t* to = toffT + ((t >> 6) * nbins + c) * 64 + (t & 63);
            st = to[0];
            len = (uint32_t)to[64] - st;
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<uint32_t>(len, reinterpret_cast<uint32_t*>(s_w), &tot) + s_carry;
        if (t < ntiles) {
            s_to[t] = ex;
            s_pb[t] = (uint32_t)t * kSlTile + st - ex;  // >= 0: ex <= t * kSlTile
        }
        __syncthreads();
        if (threadIdx.x == 0) s_carry += tot;
        __syncthreads();
    }
    const uint32_t R = s_carry;
    if (threadIdx.x == 0) {
        s_to[ntiles] = R;
        if (R) atomicAdd(&ctr->n_valid, (unsigned long long)R);
    }
    __syncthreads();
    // positions r0 + u * T + thread (u < RR) -> (key index in the block or -1 past R, row
    // value): the owner tiles by binary searches in lock step (power-of-two steps over s_to,
    // one LDS read per position per step, the RR reads of a step independent: one LDS round
    // trip per step instead of one per step and position), then the entries, branch-free
    // (a branch around a read serializes the positions' reads; positions past R read entry
    // 0 of tile 0 and drop it)
    auto gather = [&](uint32_t r0, int (&gi)[RR], uint32_t (&gr)[RR]) {
        int own[RR];
#pragma unroll
        for (int u = 0; u < RR; ++u) own[u] = 0;
        int top = 1;
        while (top < (int)ntiles) top <<= 1;
        for (int step = top >> 1; step > 0; step >>= 1) {
#pragma unroll
            for (int u = 0; u < RR; ++u) {
                const uint32_t r = r0 + u * T + threadIdx.x;
                // s_to[ntiles] = R stops every position below R at the last tile
                const int cand = own[u] + step;
                const uint32_t v = s_to[min(cand, (int)ntiles)];
                own[u] = v <= r ? cand : own[u];
            }
        }
        uint32_t pos[RR], tb[RR];
#pragma unroll
        for (int u = 0; u < RR; ++u) {
            const uint32_t r = r0 + u * T + threadIdx.x;
            const uint32_t in = 0u - (uint32_t)(r < R);  // masks, not selects: no branch around a read
            const int o = (int)((uint32_t)own[u] & in);
            pos[u] = (s_pb[o] + r) & in;
            tb[u] = tile_base[o];
        }
#pragma unroll
        for (int u = 0; u < RR; ++u) {
            const uint32_t r = r0 + u * T + threadIdx.x;
            const int i = (int)ko[pos[u]];
            const uint32_t rw = tb[u] + rl[pos[u]];
            gi[u] = r < R ? i : -1;
            gr[u] = rw;
        }
        if (ids32 != nullptr) {  // uniform
#pragma unroll
            for (int u = 0; u < RR; ++u) gr[u] = gi[u] >= 0 ? (uint32_t)ids32[gr[u]] : 0u;
        }
    };
    const bool in_regs = R <= (uint32_t)(T * RR);
    if (threadIdx.x < NSUB) s_dup[threadIdx.x] = in_regs ? 0u : 1u;  // more rows than the registers hold
    if (threadIdx.x == 0 && !in_regs) s_sp = atomicAdd(&ctr->spill_used, 2ull * R);
    if (threadIdx.x <= NSUB) s_qo[threadIdx.x] = 0;
    __syncthreads();
    // a block with more rows than the registers hold gathers them once into the spill
    // pool (key index << 32 | row), then files them by duplicate sub-range (a second copy
    // in the pool): each sub-range's duplicate passes stream its own rows only (they
    // streamed every row of the block once per sub-range: C3's build 310 -> 268 us)
    unsigned long long* sp = spill + (in_regs ? 0ull : s_sp);
    if (!in_regs) {
        const int lane = threadIdx.x & 63;
        uint32_t qn[NSUB];
#pragma unroll
        for (uint32_t q = 0; q < NSUB; ++q) qn[q] = 0;
        for (uint32_t r0 = 0; r0 < R; r0 += T * RR) {
            int gi[RR];
            uint32_t gr[RR];
            gather(r0, gi, gr);
#pragma unroll
            for (int u = 0; u < RR; ++u) {
                if (gi[u] >= 0) sp[r0 + u * T + threadIdx.x] = ((unsigned long long)(uint32_t)gi[u] << 32) | gr[u];
#pragma unroll
                for (uint32_t q = 0; q < NSUB; ++q) qn[q] += (uint32_t)(gi[u] >= 0 && (uint32_t)gi[u] / kDenseSub == q);
            }
        }
#pragma unroll
        for (uint32_t q = 0; q < NSUB; ++q)
            if (qn[q]) atomicAdd(&s_qo[q + 1], qn[q]);
        __syncthreads();
        if (threadIdx.x == 0) {
            for (uint32_t q = 0; q < NSUB; ++q) {
                s_qo[q + 1] += s_qo[q];
                s_qc[q] = s_qo[q];
            }
        }
        __syncthreads();
        unsigned long long* sp2 = sp + R;
        for (uint32_t r0 = 0; r0 < R; r0 += T) {
            const uint32_t r = r0 + threadIdx.x;
            const unsigned long long v = r < R ? sp[r] : 0ull;
            const uint32_t q = (uint32_t)(v >> 32) / kDenseSub;
#pragma unroll
            for (uint32_t qq = 0; qq < NSUB; ++qq) {
                const unsigned long long m = __ballot(r < R && q == qq);
                if (m == 0) continue;  // uniform
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&s_qc[qq], (uint32_t)__popcll(m));
                base = (uint32_t)__shfl((int)base, 0, 64);
                if (r < R && q == qq)
                    sp2[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = v;
            }
        }
        __syncthreads();
        sp = sp2;  // by sub-range: sub-range q's rows at [s_qo[q], s_qo[q + 1])
    }
    uint32_t rrow[RR];
    int ridx[RR];
    if (in_regs) {
        gather(0, ridx, rrow);
#pragma unroll
        for (int u = 0; u < RR; ++u)
            if (ridx[u] >= 0 && atomicExch(&refs[ridx[u]], rrow[u]) != kMiss) s_dup[ridx[u] / kDenseSub] = 1u;
    }
    __syncthreads();
    for (uint32_t q = 0; q < NSUB; ++q) {
        if (!s_dup[q]) continue;  // uniform: every thread reads the same LDS word
        const int lo = (int)(q * kDenseSub), hi = lo + (int)kDenseSub;
        uint32_t* img = refs + lo;
        if (threadIdx.x == 0) s_ndup = 0;
        for (uint32_t i = threadIdx.x; i < kDenseSub; i += T) img[i] = 0;
        __syncthreads();
        if (in_regs) {
#pragma unroll
            for (int u = 0; u < RR; ++u)
                if (ridx[u] >= lo && ridx[u] < hi) atomicAdd(&refs[ridx[u]], 1u);
        } else {
            for (uint32_t r = s_qo[q] + threadIdx.x; r < s_qo[q + 1]; r += T) atomicAdd(&refs[(int)(sp[r] >> 32)], 1u);
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < kDenseSub; i += T) {
            const uint32_t cnt = img[i];
            if (cnt == 0) {
                img[i] = kMiss;
            } else if (cnt > 1) {
                const unsigned li = atomicAdd(&s_ndup, 1u);
                d_cnt[li] = cnt;
                d_cur[li] = 0;
                img[i] = kDupFlag | li;
            }
        }
        __syncthreads();
        const unsigned ndup = s_ndup;
        unsigned long long carry = 0;
        for (unsigned b0 = 0; b0 < ndup; b0 += T) {
            const unsigned li = b0 + threadIdx.x;
            const unsigned long long v = li < ndup ? (unsigned long long)d_cnt[li] + 1 : 0;
            unsigned long long tot;
            const unsigned long long ex = block_excl_scan<unsigned long long>(v, s_w, &tot);
            if (li < ndup) d_off[li] = (uint32_t)(carry + ex);
            carry += tot;
        }
        if (threadIdx.x == 0) s_base = carry ? atomicAdd(&ctr->dup_used, carry) : 0;
        __syncthreads();
        for (unsigned li = threadIdx.x; li < ndup; li += T) {
            d_off[li] += (uint32_t)s_base;
            dup_rows[d_off[li]] = d_cnt[li];
        }
        __syncthreads();
        auto place = [&](int i, uint32_t row) {
            const uint32_t rv = refs[i];
            if (rv & kDupFlag) {
                const unsigned li = rv & ~kDupFlag;
                dup_rows[d_off[li] + 1 + atomicAdd(&d_cur[li], 1u)] = row;
            } else {
                refs[i] = row;  // count was 1
            }
        };
        if (in_regs) {
#pragma unroll
            for (int u = 0; u < RR; ++u)
                if (ridx[u] >= lo && ridx[u] < hi) place(ridx[u], rrow[u]);
        } else {
            for (uint32_t r = s_qo[q] + threadIdx.x; r < s_qo[q + 1]; r += T) {
                const unsigned long long v = sp[r];
                place((int)(v >> 32), (uint32_t)v);
            }
        }
        __syncthreads();
        for (unsigned li = threadIdx.x; li < ndup; li += T) {
            const unsigned n = d_cnt[li], off = d_off[li];
            d_cur[li] = 0;  // (the placement cursor is done): a run ref, or 0
            if (n <= (unsigned)kSmallSeg) {
                uint32_t v[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = (i < (int)n) ? dup_rows[off + 1 + i] : 0u;
                sort16_desc(v);
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (i < (int)n) dup_rows[off + 1 + i] = v[i];
                // consecutive rows: the ref holds them (run ref, hj_device.h)
                bool run = g.packed && n <= kRunMaxRows && v[0] < (1u << 24);
#pragma unroll
                for (int i = 1; i < (int)kRunMaxRows; ++i) run &= i >= (int)n || v[i] == v[0] - (uint32_t)i;
                if (run) d_cur[li] = make_run_ref(v[0], n);
            }
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < kDenseSub; i += T) {
            const uint32_t rv = img[i];
            if (rv != kMiss && (rv & kDupFlag)) {
                const unsigned li = rv & ~kDupFlag;
                if (d_cnt[li] > (unsigned)kSmallSeg) {
                    const unsigned bi = (unsigned)atomicAdd(&ctr->n_big, 1ull);
                    big[bi] = BigSeg{(unsigned long long)((uint64_t)g.dmin + cbase + lo + i), d_off[li], 0u};
                }
                const uint32_t c4 = (g.packed && d_cnt[li] <= 15u) ? d_cnt[li] : 0u;
                img[i] = d_cur[li] ? d_cur[li] : kDupFlag | (c4 << 27) | d_off[li];
            }
        }
        __syncthreads();
    }
    uint4* dst = reinterpret_cast<uint4*>(dense + cbase);
    const uint4* src = reinterpret_cast<const uint4*>(refs);
    for (uint32_t i = threadIdx.x; i < GV / 4; i += T) dst[i] = src[i];
}

// ---------------------------------------------------------------------------
// build (hashed, <= kFragMaxTiles tiles): the probe's hashed partition (hs_partition_kernel
// on the build keys, slices of kHbSliceLog buckets) replaces the two-level histogram /
// scan / staged-scatter chain; each workgroup then gathers one slice's rows (stored key +
// row) from every tile's fragment, as the dense frag build does, and builds the slice's
// chunks in LDS exactly as chunk_build_kernel does (CAS inserts inside each key's chunk,
// duplicate counts, directory, canonical descending segments, inline meta counts). Key 0
// (stored 0, home bucket 0: slice 0) goes to the side bucket, written by slice 0's
// workgroup. Tables past 2047 build slices are built in passes over slice ranges.
// ---------------------------------------------------------------------------
constexpr int kHbSliceLog = 10;  // buckets per build slice: 1024 x 64 B = 64 KB of LDS
constexpr uint32_t kHbSideSlot = (1u << kHbSliceLog) * kSlots;  // the side bucket's slot in the image

template <int T, int RR, int TL = kSlTileLog>
__global__ void __launch_bounds__(T)
hashed_frag_build_kernel(uint32_t nb, uint32_t clog2, uint32_t s0, uint32_t nsl, int64_t ntiles,
                         const uint16_t* __restrict__ toffT, const unsigned long long* __restrict__ ko,
                         const uint16_t* __restrict__ rl, const uint32_t* __restrict__ tile_base,
                         const uint64_t* __restrict__ ids32, Bucket* __restrict__ tbl, uint32_t* __restrict__ dup_rows,
                         BigSeg* __restrict__ big, BuildCounters* ctr, unsigned long long* __restrict__ spill,
                         uint32_t dupcap, uint64_t dup_cap, uint64_t spill_cap) {
    constexpr uint32_t SB = 1u << kHbSliceLog;
    // dynamic LDS: the image (SB buckets + the side bucket at img[SB]) | s_to u32[ntiles + 1]
    // (exclusive position of each tile's fragment) | s_pb u32[ntiles] | the duplicate
    // directory (3 x dupcap u32; a slice with more duplicated keys keeps its directory in
    // the spill pool instead)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Bucket* img = reinterpret_cast<Bucket*>(smem);
    uint32_t* s_to = reinterpret_cast<uint32_t*>(smem + (size_t)(SB + 1) * sizeof(Bucket));
    uint32_t* s_pb = s_to + ntiles + 1;
    uint32_t* s_dir = s_pb + ntiles;
    __shared__ unsigned s_ndup, s_dup;
    __shared__ uint32_t* s_dirp;
    __shared__ unsigned long long s_w[T / 64];
    __shared__ unsigned long long s_base, s_sp;
    __shared__ uint32_t s_carry;
    const uint32_t c = blockIdx.x;  // slice of this pass
    const uint32_t b0 = (s0 + c) << kHbSliceLog;
    const uint32_t nimg = min(SB, nb - b0);
    const uint32_t cmask = (1u << clog2) - 1;
    const uint32_t nbins = nsl + 1;
    const bool has_side = (s0 + c) == 0;
    {
        uint4* p = reinterpret_cast<uint4*>(img);
        for (uint32_t k = threadIdx.x; k < (SB + 1) * 4; k += T) p[k] = make_uint4(0, 0, 0, 0);
        if (threadIdx.x == 0) {
            s_ndup = 0;
            s_dup = 0;
            s_carry = 0;
        }
    }
    __syncthreads();
    // fragment bounds of this slice in every tile -> exclusive positions (block scan)
    for (int64_t t0 = 0; t0 < ntiles; t0 += T) {
        const int64_t t = t0 + threadIdx.x;
        uint32_t st = 0, len = 0;
        if (t < ntiles) {
            const uint16_t* to = toffT + ((t >> 6) * nbins + c) * 64 + (t & 63);
            st = to[0];
            len = (uint32_t)to[64] - st;
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<uint32_t>(len, reinterpret_cast<uint32_t*>(s_w), &tot) + s_carry;
        if (t < ntiles) {
            s_to[t] = ex;
            s_pb[t] = (uint32_t)t * SlT<TL>::kRows + st - ex;
        }
        __syncthreads();
        if (threadIdx.x == 0) s_carry += tot;
        __syncthreads();
    }
    const uint32_t R = s_carry;
    if (threadIdx.x == 0) {
        s_to[ntiles] = R;
        if (R) atomicAdd(&ctr->n_valid, (unsigned long long)R);
    }
    __syncthreads();
    auto fetch = [&](uint32_t r, unsigned long long* sk, uint32_t* row) {
        int lo = 0, hi = (int)ntiles - 1;  // largest tile with s_to[tile] <= r
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_to[mid] <= r) lo = mid; else hi = mid - 1;
        }
        const uint32_t pos = s_pb[lo] + r;
        if (pos >= (uint64_t)ntiles * SlT<TL>::kRows) {  // internal check (never expected)
            atomicOr(&ctr->err, 8ull);
            *sk = 0;
            *row = 0;
            return;
        }
        *sk = ko[pos];
        const uint32_t rw = tile_base[lo] + rl[pos];
        *row = ids32 ? (uint32_t)ids32[rw] : rw;
    };
    // slot of a stored key in the image (claiming insert: | kSlotNew); key 0: the side slot,
    // claimed by the first row that flips its LDS marker
    auto slot_of = [&](unsigned long long sk, bool insert) -> int {
        if (sk == 0) {
            if (!insert) return (int)kHbSideSlot;
            const unsigned long long was = atomicCAS(&img[SB].key[0], 0ull, 1ull);
            return (int)kHbSideSlot | (was == 0 ? kSlotNew : 0);
        }
        const uint32_t b = stored_bucket(sk, nb) - b0;  // < nimg: the partition put the row in this slice
        if (b >= nimg) {  // internal check (never expected)
            atomicOr(&ctr->err, 16ull);
            return -1;
        }
        Bucket* ch = img + (b & ~cmask);
        const int v = insert ? chunk_slot<true>(ch, cmask, b & cmask, sk) : chunk_slot<false>(ch, cmask, b & cmask, sk);
        if (v < 0) return -1;
        return (int)(((b & ~cmask) * kSlots + (uint32_t)(v & ~kSlotNew)) | (uint32_t)(v & kSlotNew));
    };
    auto ref_at = [&](uint32_t sl) -> unsigned& { return img[sl / kSlots].ref[sl % kSlots]; };
    const bool in_regs = R <= (uint32_t)(T * RR);
    if (threadIdx.x == 0 && !in_regs) {
        s_sp = atomicAdd(&ctr->spill_used, 2ull * R);
        if (s_sp + 2ull * R > spill_cap) atomicOr(&ctr->err, 64ull);  // internal check
    }
    __syncthreads();
    if (!in_regs && s_sp + 2ull * R > spill_cap) return;
    // more rows than the registers hold: gathered once into the spill pool (key, row)
    unsigned long long* sp = spill + (in_regs ? 0ull : s_sp);
    if (!in_regs) {
        for (uint32_t r = threadIdx.x; r < R; r += T) {
            unsigned long long k;
            uint32_t rw;
            fetch(r, &k, &rw);
            sp[2 * r] = k;
            sp[2 * r + 1] = rw;
        }
        __syncthreads();
    }
    uint32_t rrow[RR];
    int rslot[RR];
    // pass A: claim slots; the claiming insert stores its row (final for a single-row key)
    if (in_regs) {
        unsigned long long rk[RR];
        // owner tiles by lock-step binary searches and branch-free gathers, as the dense
        // frag build does (one LDS round trip per search step for all RR positions)
        int own[RR];
#pragma unroll
        for (int u = 0; u < RR; ++u) own[u] = 0;
        int top = 1;
        while (top < (int)ntiles) top <<= 1;
        for (int step = top >> 1; step > 0; step >>= 1) {
#pragma unroll
            for (int u = 0; u < RR; ++u) {
                const uint32_t r = u * T + threadIdx.x;
                const int cand = own[u] + step;
                const uint32_t v = s_to[min(cand, (int)ntiles)];  // s_to[ntiles] = R
                own[u] = v <= r ? cand : own[u];
            }
        }
        uint32_t pos[RR], tb[RR];
#pragma unroll
        for (int u = 0; u < RR; ++u) {
            const uint32_t r = u * T + threadIdx.x;
            const uint32_t in = 0u - (uint32_t)(r < R);  // positions past R read entry 0 and drop it
            const int o = (int)((uint32_t)own[u] & in);
            pos[u] = (s_pb[o] + r) & in;
            tb[u] = tile_base[o];
        }
#pragma unroll
        for (int u = 0; u < RR; ++u) {
            rk[u] = ko[pos[u]];
            rrow[u] = tb[u] + rl[pos[u]];
        }
        if (ids32 != nullptr) {  // uniform
#pragma unroll
            for (int u = 0; u < RR; ++u) rrow[u] = u * T + threadIdx.x < R ? (uint32_t)ids32[rrow[u]] : 0u;
        }
#pragma unroll
        for (int u = 0; u < RR; ++u) {
            rslot[u] = -1;
            if (u * T + threadIdx.x >= R) continue;
            const int v = slot_of(rk[u], true);
            if (v < 0) { atomicOr(&ctr->err, 1ull); continue; }  // chunk full: the host rebuilds at half load
            rslot[u] = v & ~kSlotNew;
            if (v & kSlotNew) ref_at(rslot[u]) = rrow[u];
            else s_dup = 1u;
        }
    } else {
        if (threadIdx.x == 0) s_dup = 1u;
        for (uint32_t r = threadIdx.x; r < R; r += T) {
            if (slot_of(sp[2 * r], true) < 0) atomicOr(&ctr->err, 1ull);
        }
    }
    __syncthreads();
    const uint32_t nslot = SB * kSlots + kSlots;  // the image's slots and the side bucket's
    if (s_dup) {  // uniform
        // row counts per slot
        for (uint32_t sl = threadIdx.x; sl < nslot; sl += T) ref_at(sl) = 0;
        __syncthreads();
        if (in_regs) {
#pragma unroll
            for (int u = 0; u < RR; ++u)
                if (rslot[u] >= 0) atomicAdd(&ref_at(rslot[u]), 1u);
        } else {
            for (uint32_t r = threadIdx.x; r < R; r += T) {
                const int v = slot_of(sp[2 * r], false);
                if (v >= 0) atomicAdd(&ref_at(v), 1u);
            }
        }
        __syncthreads();
        // the directory of duplicated keys (count > 1): in LDS when it fits, else in the
        // spill pool (generic pointers: the same code serves both)
        for (uint32_t sl = threadIdx.x; sl < nslot; sl += T)
            if (ref_at(sl) > 1) atomicAdd(&s_ndup, 1u);
        __syncthreads();
        const unsigned ndup = s_ndup;
        __syncthreads();  // every wave holds ndup before thread 0 resets the counter for the assignment
        if (threadIdx.x == 0) {
            if (ndup <= dupcap) {
                s_dirp = s_dir;
            } else {
                const unsigned long long at = atomicAdd(&ctr->spill_used, (3ull * ndup + 1) / 2);
                s_dirp = at + (3ull * ndup + 1) / 2 <= spill_cap ? reinterpret_cast<uint32_t*>(spill + at) : nullptr;
                if (s_dirp == nullptr) atomicOr(&ctr->err, 64ull);  // internal check
            }
            s_ndup = 0;
        }
        __syncthreads();
        if (s_dirp == nullptr) return;
        uint32_t* d_off = s_dirp;
        uint32_t* d_cur = d_off + ndup;
        uint32_t* d_cnt = d_cur + ndup;
        for (uint32_t sl = threadIdx.x; sl < nslot; sl += T) {
            unsigned& ref = ref_at(sl);
            const unsigned cnt = ref;
            if (cnt > 1) {
                const unsigned li = atomicAdd(&s_ndup, 1u);
                d_cnt[li] = cnt;
                d_cur[li] = 0;
                ref = kDupFlag | li;
            }
        }
        __syncthreads();
        unsigned long long carry = 0;
        for (unsigned bb = 0; bb < ndup; bb += T) {
            const unsigned li = bb + threadIdx.x;
            const unsigned long long v = li < ndup ? (unsigned long long)d_cnt[li] + 1 : 0;
            unsigned long long tot;
            const unsigned long long ex = block_excl_scan<unsigned long long>(v, s_w, &tot);
            if (li < ndup) d_off[li] = (uint32_t)(carry + ex);
            carry += tot;
        }
        if (threadIdx.x == 0) {
            s_base = carry ? atomicAdd(&ctr->dup_used, carry) : 0;
            if (s_base + carry > dup_cap) atomicOr(&ctr->err, 32ull);  // internal check
        }
        __syncthreads();
        if (s_base + carry > dup_cap) return;
        for (unsigned li = threadIdx.x; li < ndup; li += T) {
            d_off[li] += (uint32_t)s_base;
            dup_rows[d_off[li]] = d_cnt[li];
        }
        __syncthreads();
        auto place = [&](int sl, uint32_t row) {
            unsigned& ref = ref_at(sl);
            const unsigned rv = ref;
            if (rv & kDupFlag) {
                const unsigned li = rv & ~kDupFlag;
                const uint64_t at = (uint64_t)d_off[li] + 1 + atomicAdd(&d_cur[li], 1u);
                if (at < dup_cap) dup_rows[at] = row;
                else atomicOr(&ctr->err, 32ull);  // internal check
            } else if (rv == 1) {
                ref = row;  // the key's only row
            }
        };
        if (in_regs) {
#pragma unroll
            for (int u = 0; u < RR; ++u)
                if (rslot[u] >= 0) place(rslot[u], rrow[u]);
        } else {
            for (uint32_t r = threadIdx.x; r < R; r += T) {
                const int v = slot_of(sp[2 * r], false);
                if (v >= 0) place(v, (uint32_t)sp[2 * r + 1]);
            }
        }
        __syncthreads();
        // canonical order inside segments (descending rows), final refs and inline counts
        for (unsigned li = threadIdx.x; li < ndup; li += T) {
            const unsigned n = d_cnt[li], off = d_off[li];
            if (n <= (unsigned)kSmallSeg) {
                uint32_t v[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = (i < (int)n) ? dup_rows[off + 1 + i] : 0u;
                sort16_desc(v);
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (i < (int)n) dup_rows[off + 1 + i] = v[i];
            }
        }
        for (uint32_t sl = threadIdx.x; sl < nslot; sl += T) {
            Bucket& B = img[sl / kSlots];
            unsigned& ref = B.ref[sl % kSlots];
            if (ref & kDupFlag) {
                const unsigned li = ref & ~kDupFlag;
                const bool side = sl == kHbSideSlot;
                if (d_cnt[li] > (unsigned)kSmallSeg) {
                    const unsigned bi = (unsigned)atomicAdd(&ctr->n_big, 1ull);
                    big[bi] = BigSeg{side ? 0ull : unmix64(B.key[sl % kSlots]), d_off[li], 0u};
                }
                ref = kDupFlag | d_off[li];
                if (!side && d_cnt[li] <= kInlineCount) atomicOr(&B.meta, d_cnt[li] << (1 + 6 * (sl % kSlots)));
            }
        }
        __syncthreads();
    }
    // write the finished buckets (coalesced 16-byte stores); slice 0 also writes the side
    // bucket (keys 0, ref[0], meta = the key-0 rows)
    {
        const uint4* src = reinterpret_cast<const uint4*>(img);
        uint4* dst = reinterpret_cast<uint4*>(tbl + b0);
        for (uint32_t k = threadIdx.x; k < nimg * 4; k += T) dst[k] = src[k];
    }
    if (has_side && threadIdx.x == 0) {
        Bucket& S = tbl[nb];
        const bool used = img[SB].key[0] != 0;
        uint32_t rows0 = 0;
        if (used) rows0 = (img[SB].ref[0] & kDupFlag) ? dup_rows[img[SB].ref[0] & ~kDupFlag] : 1u;
        for (int j = 0; j < kSlots; ++j) {
            S.key[j] = 0;
            S.ref[j] = 0;
        }
        S.ref[0] = used ? img[SB].ref[0] : 0u;
        S.meta = rows0;
    }
}

// grid = nslices x parts; item i: slice i % nslices, tiles [part range) with
// part = i / nslices. Each wave walks runs of 64 tiles: lane l reads tile l's segment
// bounds (prefetched one run ahead), a wave scan flattens the segments over the lanes,
// and the non-empty segments' bases are listed by rank. A 64-bit mask per 64 flattened
// positions marks the segment starts (LDS atomicOr); a position's owner rank is the
// number of starts at or before it (mbcnt) — no per-position search, no scan per row.
// Entries and refs go through buffer descriptors: 32-bit offsets, and positions past
// the run's total take an out-of-range offset (load 0, store dropped) instead of a
// branch. W / 64 entries per lane in flight.
//   dense  (HASHED false): the slice is 2^wlog consecutive key values of the direct-
//          addressed table (u32 refs); an entry is the key's offset in the slice (u16),
//          its ref one LDS read.
//   hashed (HASHED true): the slice is 2048 consecutive buckets (128 KB, kHsSliceLog);
//          an entry is the stored key (mix64(key), u64); its ref comes from the home
//          bucket's line in LDS (exact compare of stored keys, linear probing inside the
//          chunk, as lookup4); key 0 reads the side bucket.
constexpr int kHsSliceLog = 11;  // buckets per hashed slice: 2^11 x 64 B = 128 KB of LDS

// The LDS image of a hashed slice, bank-spread: quad q of the slice's bucket bl lies at
// quad (q ^ ((bl >> 2) & 3)) of its 64-byte line. A ds_read_b128 serves 16 lanes per LDS
// cycle; their bank slot is (4 * (bl % 4) + physical quad) of the 256-byte bank row, so
// with every line in plain order, 16 lanes reading the same quad of random buckets meet on
// 4 slots (about 6-way); the XOR by the next two bucket bits spreads them over all 16.
// (r03 rotated by the bucket's low bits, which leaves the 4 slots as they were.)
__device__ __forceinline__ uint32_t hs_quad_rot(uint32_t bl) { return (bl >> 2) & 3u; }
__device__ __forceinline__ void lds_line(const uint4* __restrict__ img, uint32_t bl, uint4& a0, uint4& a1, uint4& a2,
                                         uint4& a3) {
    const uint4* p = img + (size_t)bl * 4;
    const uint32_t r = hs_quad_rot(bl);
    a0 = p[0 ^ r];
    a1 = p[1 ^ r];
    a2 = p[2 ^ r];
    a3 = p[3 ^ r];
}

// ref of stored key sk (!= 0) in the LDS image of a hashed slice whose first bucket is
// sbase; linear probing wraps inside the key's chunk (cmask), as the table was built
__device__ __forceinline__ uint32_t lds_bucket_ref(const uint4* __restrict__ img, uint32_t nb, uint32_t sbase,
                                                   uint32_t cmask, unsigned long long sk, uint32_t* cnt) {
    uint32_t b = stored_bucket(sk, nb);
    uint4 a0, a1, a2, a3;
    lds_line(img, b - sbase, a0, a1, a2, a3);
    bool more;
    uint32_t ref = scan_line(a0, a1, a2, a3, sk, &more, cnt);
    for (uint32_t probes = 0; more && probes < cmask; ++probes) {
        b = (b & ~cmask) | ((b + 1) & cmask);
        lds_line(img, b - sbase, a0, a1, a2, a3);
        ref = scan_line(a0, a1, a2, a3, sk, &more, cnt);
    }
    return ref;
}

// Measured (r04) and not kept: a count in its segment header deferred to a pass after the
// window (no per-row ballot): C2h lookup 771 -> 771 us.
// Measured (r04) and not kept: every hashed row branch-free (selects, stores dropped by an
// out-of-range offset, the rare rows deferred to a pass after the window, two rows per
// scheduling region; 108 VGPRs): C2h lookup 771 -> 1107 us.
// Measured (r04) and not kept: the home bucket's compares alone, with a duplicated key's
// inline count and the probe past a bucket an insert passed full in wave-uniform branches
// (fewer instructions per row): C2h lookup 771 -> 917 us — the per-row ballots split the
// unrolled rows into separate blocks, so no row's LDS reads overlap another's work.
// Measured (r04) and not kept: the hashed slice image re-laid as quad arrays (low key
// halves, high halves, key 4 + meta, refs: one quad read per lane on 16 of a bank row's
// 256 B instead of 4 of them) with three quad reads and a dependent ref read per entry
// — C2h lookup 770 -> 830 us: the lookup is bound by its per-row dependency chains, not
// by LDS bank conflicts, and the extra dependent read lengthens every chain.

constexpr uint32_t kBigCorr = 1u << 16;  // counts - 1 from here on correct the tile count directly
constexpr int kLkGroup = 4;  // dense lookup: rows per branch-free group (divides the window's rows)
// hashed lookup: rows per group of owner searches and entry loads, of bucket-line reads
// (r05: groups of 2-4 rows were slower in every form, 784-1,303 us against 751)
constexpr int kHsGroup1 = 1;
constexpr int kHsGroup2 = 1;
// a tile's pair count (tcnt) is < 2^45 (16384 rows x < 2^31 build rows); the dense lookup
// adds kOddFlag once per fragment with an entry of a missing or duplicated key, the hashed
// lookup once per fragment with a duplicated key (at most 4095 slices per pass and < 64
// passes: the 18 flag bits never wrap to 0)
constexpr int kOddShift = 46;
constexpr unsigned long long kOddFlag = 1ull << kOddShift;
constexpr unsigned long long kCountMask = kOddFlag - 1;

// Timing ablations (wrong pairs by design) exist only in a diagnostic build of the
// library (tools/build_ablation.py defines DFP_HJ_ABLATIONS); the product library folds
// kAbl to 0 and reads no environment for them.
#ifdef DFP_HJ_ABLATIONS
__constant__ int kAblDev;
#define DFP_ABL(bit) (kAblDev & (bit))
// per-workgroup timeline of the last sliced lookup / emission (diagnostic build only):
// [4 * blockIdx + 0..3] = start, after its first phase (lookup: slice image loaded),
// end (wall clock, 100 MHz), hardware id (xcc << 16 | se << 8 | cu)
__device__ unsigned long long g_dbg_lk_ts[4 * 65536];
__device__ unsigned long long g_dbg_em_ts[4 * 65536];
__device__ __forceinline__ unsigned long long dbg_hwid() {
    const unsigned cu = __builtin_amdgcn_s_getreg(GETREG_IMMED(HW_ID_CU_ID_SIZE - 1, HW_ID_CU_ID_OFFSET, HW_ID));
    const unsigned se = __builtin_amdgcn_s_getreg(GETREG_IMMED(HW_ID_SE_ID_SIZE - 1, HW_ID_SE_ID_OFFSET, HW_ID));
    const unsigned xcc = __builtin_amdgcn_s_getreg(GETREG_IMMED(3, 0, 20));
    return ((unsigned long long)xcc << 16) | (se << 8) | cu;
}
#define DFP_DBG_TS(arr, slot, v) \
    do { if (threadIdx.x == 0 && blockIdx.x < 65536) arr[4 * blockIdx.x + (slot)] = (v); } while (0)
// the sliced lookup's per-phase shader cycles summed over every wave of the last launches
// (DFP_HJ_ABLATE bit 256 turns it on: it adds an s_waitcnt vmcnt(0) before the row work):
// [0] block setup, [1] entry loads issued, [2] wait for them, [3] rows, [4] block end,
// [5] blocks, [6] windows
__device__ unsigned long long g_dbg_lk_ph[8];
#define DFP_PH_DECL unsigned long long ph_t = 0, ph_acc[7] = {0, 0, 0, 0, 0, 0, 0}; \
    const bool ph_on = DFP_ABL(256) != 0; if (ph_on) ph_t = clock64()
#define DFP_PH(i) do { if (ph_on) { const unsigned long long t_ = clock64(); ph_acc[i] += t_ - ph_t; ph_t = t_; } } while (0)
#define DFP_PH_WAIT() do { if (ph_on) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); } while (0)
#define DFP_PH_CNT(i) do { if (ph_on) ph_acc[i] += 1; } while (0)
#define DFP_PH_FLUSH() do { if (ph_on && (threadIdx.x & 63) == 0) \
    for (int i_ = 0; i_ < 7; ++i_) atomicAdd(&g_dbg_lk_ph[i_], ph_acc[i_]); } while (0)
#else
#define DFP_ABL(bit) 0
#define DFP_DBG_TS(arr, slot, v) do { } while (0)
#define DFP_PH_DECL do { } while (0)
#define DFP_PH(i) do { } while (0)
#define DFP_PH_WAIT() do { } while (0)
#define DFP_PH_CNT(i) do { } while (0)
#define DFP_PH_FLUSH() do { } while (0)
#endif

template <bool HASHED, int W, int TL = kSlTileLog>
__global__ void __launch_bounds__(kSlThreads)
sl_lookup_kernel(TableView tv, uint32_t wlog, uint32_t nslices, int64_t ntiles, uint32_t parts, uint32_t s1,
                 uint32_t parts2,  // slices [0, s1): `parts` items each; [s1, nslices): `parts2` smaller ones, last
                 int early,        // 1: each wave sets up its first block and issues its entry loads before the image barrier
                 const void* __restrict__ ko, uint32_t* __restrict__ res, const uint16_t* __restrict__ toff,
                 unsigned long long* __restrict__ tcnt, uint32_t soff) {  // soff: first slice of this pass (hashed)
    extern __shared__ __attribute__((aligned(16))) uint32_t s_tab[];  // dense: 2^wlog refs; hashed: 2048 buckets
    // per wave by rank: the fragment holds an entry of count != 1 (dense: a missing or
    // duplicated key; hashed: a duplicated key, misses being the common case there)
    __shared__ uint8_t s_odd[kSlThreads];
    __shared__ uint32_t s_base[kSlThreads];
    __shared__ uint32_t s_lane[kSlThreads];  // per wave: tile lane of each non-empty segment, by rank
    // per wave, by rank: dense, the correction running sum at each fragment's start;
    // hashed, at each fragment's end
    __shared__ uint32_t s_cst[kSlThreads];
    __shared__ uint32_t s_end[HASHED ? kSlThreads : 1];  // hashed, per wave: end position of each fragment, by rank
    __shared__ unsigned long long s_mask[kSlThreads / 64][W / 64];
    // hashed: per wave, the window's entries that must probe past a full home
    // bucket, queued (stored key, entry index | owner rank << 26) and looked up 64 at a time
    __shared__ unsigned long long s_dqk[HASHED ? kSlThreads : 1];
    __shared__ uint32_t s_dqo[HASHED ? kSlThreads : 1];
    DFP_DBG_TS(g_dbg_lk_ts, 0, wall_clock64());
    // Items: the first s1 slices in `parts` parts each, then the rest in `parts2` smaller
    // ones; every XCD runs its share of the first stage before its share of the second
    // (block b on XCD b % 8 as b / 8-th), so the last round is of small items (the even
    // split left 0.59 of a round: CUs 13 % idle, r04 timelines)
    const uint32_t n1 = s1 * parts;
    uint32_t s, part, np;  // slice, part, parts of this slice
    if (blockIdx.x < n1) {
        const uint32_t item = DFP_ABL(128) ? blockIdx.x : xcd_item(blockIdx.x, n1);
        s = item % s1;
        part = item / s1;
        np = parts;
    } else {
        const uint32_t item = DFP_ABL(128) ? blockIdx.x - n1 : xcd_item(blockIdx.x - n1, gridDim.x - n1);
        s = s1 + item % (nslices - s1);
        part = item / (nslices - s1);
        np = parts2;
    }
    uint32_t sbase = 0;  // hashed: first bucket of the slice
    // the slice's image: whole 1 KB pieces by LDS DMA (global_load_lds_dwordx4, one wave
    // instruction per piece, every piece of a wave in flight at once, no VGPR round trip),
    // the rest (a table's last partial piece) by ordinary loads
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // (hashed: LDS quad i holds source quad i ^ hs_quad_rot(i / 4), the bank-spread lines)
    auto dma = [&](const uint4* src, uint32_t nq) {  // nq uint4 of src -> s_tab
        const uint32_t npieces = nq >> 6;
        for (uint32_t c = (uint32_t)wave; c < npieces; c += kSlThreads / 64) {
            const uint32_t i = c * 64 + lane;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(src + (HASHED ? i ^ hs_quad_rot(i >> 2) : i)),
                (__attribute__((address_space(3))) void*)(reinterpret_cast<uint4*>(s_tab) + c * 64), 16, 0, 0);
        }
        return npieces << 6;
    };
    if constexpr (HASHED) {
        sbase = (soff + s) << kHsSliceLog;
        const uint32_t nbk = min<uint32_t>(1u << kHsSliceLog, tv.nb - sbase);
        const uint4* src = reinterpret_cast<const uint4*>(tv.tbl + sbase);
        uint4* dst = reinterpret_cast<uint4*>(s_tab);
        for (uint32_t i = dma(src, nbk * 4) + threadIdx.x; i < nbk * 4; i += kSlThreads) dst[i] = src[i ^ hs_quad_rot(i >> 2)];
    } else {
        const uint64_t base = (uint64_t)s << wlog;
        const uint32_t len = (uint32_t)min<uint64_t>(1u << wlog, tv.drange - base);
        const uint32_t* __restrict__ dense = tv.dense;
        // dense is 256-byte aligned and slices start at multiples of 64 KB
        const uint32_t done = dma(reinterpret_cast<const uint4*>(dense + base), len >> 2) * 4;
        for (uint32_t i = done + threadIdx.x; i < len; i += kSlThreads) s_tab[i] = dense[base + i];
    }
    // The image is needed only from the first row lookup on: with `early`, each wave sets
    // up its first block and issues that window's entry loads while the image loads, and
    // meets the barrier there (every wave exactly once: a wave without blocks at the end).
    bool img_ready = early == 0;
    if (img_ready) __syncthreads();
    auto wait_image = [&]() {
        if (!img_ready) {
            __syncthreads();
            img_ready = true;
        }
    };
    DFP_DBG_TS(g_dbg_lk_ts, 1, wall_clock64());
    // part boundaries on 64-tile blocks (the transposed bounds' granule)
    const int64_t nblk = (ntiles + 63) / 64;
    const int64_t ta = nblk * part / np * 64, tb = min<int64_t>(nblk * (part + 1) / np * 64, ntiles);
    const int64_t nbins = nslices + 1;
    // per wave: the non-empty segments' bases (tile-relative position - excl) by rank, and
    // one 64-bit start mask per 64-position row of the window
    uint32_t* sbs = s_base + wave * 64;
    uint32_t* slane = s_lane + wave * 64;
    uint32_t* scst = s_cst + wave * 64;
    uint32_t* send = s_end + (HASHED ? wave * 64 : 0);
    unsigned long long* smask = s_mask[wave];
    constexpr int64_t kStep = (kSlThreads / 64) * 64;  // tiles between a wave's blocks
    constexpr uint32_t kOob = 0x3FFFFF0u;               // entry index past every range: load 0, no store
    constexpr uint32_t kOobMask = (1u << 26) - 1;       // off[] = index | owner rank << 26
    constexpr int KB = HASHED ? 8 : 2;                  // entry bytes
    const uint32_t cmask = (1u << tv.clog2) - 1;
    uint32_t side_meta = 0, side_ref = kMiss;  // hashed: the side bucket (key 0), read once
    if constexpr (HASHED) {
        side_meta = tv.tbl[tv.nb].meta;
        side_ref = tv.tbl[tv.nb].ref[0];
    }
    // segment bounds of the lane's tile in block tc (tile-major toff), loaded one block ahead
    auto bounds = [&](int64_t tc, uint32_t* st, uint32_t* len) {
        *st = 0;
        *len = 0;
        if (tc + lane < tb) {  // tile-major bounds: consecutive slices (one XCD's items) share lines in its L2
            const uint16_t* to = toff + (tc + lane) * nbins + s;
            *st = to[0];
            *len = (uint32_t)to[1] - *st;
        }
    };
    uint32_t nst, nlen;
    bounds(ta + (int64_t)wave * 64, &nst, &nlen);
    DFP_PH_DECL;
    for (int64_t tc = ta + (int64_t)wave * 64; tc < tb; tc += kStep) {
        DFP_PH_CNT(5);
        const uint32_t st = nst, len = nlen;
        bounds(tc + kStep, &nst, &nlen);
        const uint32_t incl = wave_incl_scan_dpp(len);
        const uint32_t excl = incl - len;
        const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        // rank of the lane among the non-empty segments (their starts, in position order)
        const unsigned long long ne = __ballot(len != 0);
        const uint32_t rank =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(ne >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ne, 0u));
        const uint32_t nranks = (uint32_t)__builtin_popcountll(ne);
        if (len != 0) {
            sbs[rank] = (uint32_t)lane * SlT<TL>::kRows + st - excl;  // >= 0: excl <= lane * SlT<TL>::kRows
            slane[rank] = (uint32_t)lane;
            if constexpr (HASHED) send[rank] = excl + len;
        }
        // the run's corrections (count - 1 of a missing or duplicated key) as a running sum
        // over the flattened positions, recorded at each fragment's first position: a
        // fragment's correction is its successor's record minus its own (the last one's:
        // the final sum). A segmented sum without LDS atomics, and a row of unique hits
        // costs one ballot. Sums are mod 2^32: a fragment's true correction lies in
        // (-2^14, 2^30) since counts of kBigCorr or more go to the tile count directly.
        // Hashed (half the entries of a uniform probe side miss): the running sum of every
        // row, recorded at each fragment's last position instead.
        scst[lane] = 0;
        uint8_t* sodd = s_odd + wave * 64;
        sodd[lane] = 0;
        uint32_t corr_run = 0;
        // the 64 tiles' regions as buffers (wave-uniform bases): 32-bit offsets, and an
        // out-of-range offset turns a position past R into a dropped access
        const int64_t tcu = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)tc) |
                            ((int64_t)__builtin_amdgcn_readfirstlane((int)(tc >> 32)) << 32);
        const __amdgpu_buffer_rsrc_t rko = __builtin_amdgcn_make_buffer_rsrc(
            (void*)((const char*)ko + tcu * SlT<TL>::kRows * KB), 0, 64 * SlT<TL>::kRows * KB, 0x00020000);
        const __amdgpu_buffer_rsrc_t rres =
            __builtin_amdgcn_make_buffer_rsrc((void*)(res + tcu * SlT<TL>::kRows), 0, 64 * SlT<TL>::kRows * 4, 0x00020000);
        uint32_t kb = 0;  // segments started before the current row
        DFP_PH(0);
        for (uint32_t w0 = 0; w0 < R; w0 += W) {
            DFP_PH_CNT(6);
            if (lane < W / 64) smask[lane] = 0;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");  // LDS only: no wait for the ref stores
            __builtin_amdgcn_wave_barrier();
            if (len != 0 && excl >= w0 && excl < w0 + W) atomicOr(&smask[(excl - w0) >> 6], 1ull << ((excl - w0) & 63));
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");  // LDS only: no wait for the ref stores
            __builtin_amdgcn_wave_barrier();
            // Measured (r04) and not kept, C2 serialized (tools/lookup_ablate.py, lookup with
            // its stores / entry loads / table reads removed: 138 / 122 / 129 / 113 us with
            // none of the three): every row's start mask from one LDS read, the owners' bases
            // and the entry loads in branch-free groups of 8 rows, and the refs stored one
            // window late (after the next window's loads): 146 us (104 without stores) —
            // a shorter skeleton, but the stores then cost 41 us; the 2048-position form of it
            // spills. The hashed analogue (first bucket lines of two rows read together, the
            // correction scans interleaved): C2h 56.8K -> 55.5K Mrows/s.
            constexpr int NU = W / 64;  // rows of 64 positions per window
            uint32_t off[NU];      // the entry's index (or kOob) | owner rank << 26
            uint32_t off_end = 0;  // hashed: bit u = this lane's position u ends its fragment
            using EV = typename std::conditional<HASHED, unsigned long long, uint32_t>::type;
            EV ev[NU];
            // Measured (r04): reading every row's start mask at once (one LDS read, then
            // v_readlane per row) and the owners' bases in batches of 8 rows took the C2
            // lookup 133 -> 150 us (128 VGPRs, spills); the per-row LDS round trips below
            // overlap across the 16 waves of the CU.
            if constexpr (!HASHED) {
                // dense: rows in branch-free groups of kLkGroup (rows past the run read a zero
                // mask and take the out-of-range offset), so that a group's mask reads, then its
                // owners' base reads, then its entry loads issue together: two LDS round trips
                // per group instead of per row (r05)
#pragma unroll
                for (int g0 = 0; g0 < NU; g0 += kLkGroup) {
#pragma unroll
                    for (int u = g0; u < g0 + kLkGroup; ++u) off[u] = kOob;
                    if (w0 + g0 * 64 >= R) continue;  // uniform: past the run
                    unsigned long long mu[kLkGroup];
#pragma unroll
                    for (int j = 0; j < kLkGroup; ++j) {
                        const unsigned long long m = smask[g0 + j];  // the same word for every lane
                        const uint32_t mlo = __builtin_amdgcn_readfirstlane((uint32_t)m);
                        const uint32_t mhi = __builtin_amdgcn_readfirstlane((uint32_t)(m >> 32));
                        mu[j] = ((unsigned long long)mhi << 32) | mlo;
                    }
                    uint32_t kk[kLkGroup], bs[kLkGroup];
#pragma unroll
                    for (int j = 0; j < kLkGroup; ++j) {
                        const unsigned long long m1 = mu[j] >> 1;
                        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
                        kk[j] = kb + (uint32_t)(mu[j] & 1) + below - 1;
                        kb += (uint32_t)__builtin_popcountll(mu[j]);
                    }
#pragma unroll
                    for (int j = 0; j < kLkGroup; ++j) bs[j] = sbs[kk[j] & 63];
#pragma unroll
                    for (int j = 0; j < kLkGroup; ++j) {
                        const uint32_t r = w0 + (g0 + j) * 64 + lane;
                        const uint32_t o = r < R ? bs[j] + r : kOob;
                        // ablation 1024: no entry loads (wrong pairs)
                        ev[g0 + j] = DFP_ABL(1024) ? (r & 0x7FFF) : __builtin_amdgcn_raw_buffer_load_b16(rko, (int)(o * 2), 0, 0);
                        off[g0 + j] = o | ((kk[j] & 63) << 26);
                    }
                }
            }
            if constexpr (HASHED) {
                // hashed: the dense path's row groups (mask reads, then owner bases and
                // fragment ends, then the entry loads of kHsGroup1 rows issue together)
#pragma unroll
                for (int g0 = 0; g0 < NU; g0 += kHsGroup1) {
#pragma unroll
                    for (int u = g0; u < g0 + kHsGroup1; ++u) {
                        off[u] = kOob;
                        ev[u] = 0;
                    }
                    if (w0 + g0 * 64 >= R) continue;  // uniform: past the run
                    unsigned long long mu[kHsGroup1];
#pragma unroll
                    for (int j = 0; j < kHsGroup1; ++j) {
                        const unsigned long long m = smask[g0 + j];  // the same word for every lane
                        const uint32_t mlo = __builtin_amdgcn_readfirstlane((uint32_t)m);
                        const uint32_t mhi = __builtin_amdgcn_readfirstlane((uint32_t)(m >> 32));
                        mu[j] = ((unsigned long long)mhi << 32) | mlo;
                    }
                    uint32_t kk[kHsGroup1], bs[kHsGroup1], en[kHsGroup1];
#pragma unroll
                    for (int j = 0; j < kHsGroup1; ++j) {
                        const unsigned long long m1 = mu[j] >> 1;
                        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
                        kk[j] = kb + (uint32_t)(mu[j] & 1) + below - 1;
                        kb += (uint32_t)__builtin_popcountll(mu[j]);
                    }
#pragma unroll
                    for (int j = 0; j < kHsGroup1; ++j) {
                        bs[j] = sbs[kk[j] & 63];
                        en[j] = send[kk[j] & 63];
                    }
#pragma unroll
                    for (int j = 0; j < kHsGroup1; ++j) {
                        const uint32_t r = w0 + (g0 + j) * 64 + lane;
                        const uint32_t o = r < R ? bs[j] + r : kOob;
                        if (r + 1 == en[j]) off_end |= 1u << (g0 + j);  // last position of its fragment
                        const uint2 v = __builtin_bit_cast(
                            uint2, __builtin_amdgcn_raw_buffer_load_b64(rko, (int)(o * 8), 0, 0));
                        ev[g0 + j] = ((unsigned long long)v.y << 32) | v.x;
                        off[g0 + j] = o | ((kk[j] & 63) << 26);
                    }
                }
            }
            wait_image();
            DFP_PH(1);
            DFP_PH_WAIT();
            DFP_PH(2);
            // one hashed row the general way (any count, key 0, probes past full buckets)
            auto hashed_row = [&](const int u) __attribute__((always_inline)) {
                if (w0 + u * 64 >= R) return;  // uniform: past the run
                const uint32_t o = off[u] & kOobMask;
                uint32_t v, c;  // ref and its row count (kCountUnknown: in its segment header)
                const unsigned long long sk = ev[u];
                if (o == kOob) {
                    v = kMiss;  // no store, no correction
                    c = 1;
                } else if (DFP_ABL(4)) {  // timing ablation: no bucket lookup (wrong pairs)
                    v = (uint32_t)sk & 0xFFFFFFu;
                    c = 1;
                } else if (sk == 0) {  // key 0: the side bucket (rare; loaded at the start)
                    v = side_meta ? side_ref : kMiss;
                    c = side_meta;
                } else {
                    v = lds_bucket_ref(reinterpret_cast<const uint4*>(s_tab), tv.nb, sbase, cmask, sk, &c);
                }
                // counts not inline: read from the segment header in a wave-uniform branch
                // that waits there. Merged into the common path, that load's wait was an
                // s_waitcnt vmcnt(0) on every row — for the previous rows' ref stores (loads
                // and stores share vmcnt): one store round trip per 64 entries.
                if (__ballot(c == kCountUnknown) != 0) {
                    if (c == kCountUnknown) c = tv.dup_rows[v & tv.off_mask];
                    asm volatile("" : "+v"(c));
                }
                __builtin_amdgcn_raw_buffer_store_b32(v, rres, (int)(o * 4), 0, 0);
                if (c > 1u) sodd[off[u] >> 26] = 1;  // kOob: c = 1 (the emission's 0/1 path is off for its tile)
                uint32_t d = c - 1u;  // kOob: c = 1
                if (d != 0xFFFFFFFFu && d >= kBigCorr) {
                    atomicAdd(&tcnt[tc + slane[off[u] >> 26]], (unsigned long long)d);
                    d = 0;
                }
                corr_run += wave_incl_scan_dpp(d);
                if (off_end & (1u << u)) scst[off[u] >> 26] = corr_run;
                corr_run = (uint32_t)__builtin_amdgcn_readlane((int)corr_run, 63);
            };
            // the queued entries, one per lane: probe on from the bucket after
            // the home one; a hit stores its ref over the kMiss stored for it and adds its
            // row count to its tile (the -1 of a miss was already in the running sum)
            uint32_t dq_n = 0;  // uniform: queued entries of this wave
            auto dq_flush = [&]() __attribute__((always_inline)) {
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");
                __builtin_amdgcn_wave_barrier();
                if ((uint32_t)lane < dq_n) {
                    const unsigned long long sk = s_dqk[wave * 64 + lane];
                    const uint32_t ofs = s_dqo[wave * 64 + lane];
                    uint32_t b = stored_bucket(sk, tv.nb), c = 0;
                    uint32_t ref = kMiss;
                    bool more = true;
                    for (uint32_t probes = 0; more && probes < cmask; ++probes) {
                        b = (b & ~cmask) | ((b + 1) & cmask);
                        uint4 q0, q1, q2, q3;
                        lds_line(reinterpret_cast<const uint4*>(s_tab), b - sbase, q0, q1, q2, q3);
                        ref = scan_line(q0, q1, q2, q3, sk, &more, &c);
                    }
                    if (ref != kMiss) {
                        if (c == kCountUnknown) c = tv.dup_rows[ref & tv.off_mask];
                        if (c > 1u) sodd[ofs >> 26] = 1;
                        __builtin_amdgcn_raw_buffer_store_b32(ref, rres, (int)((ofs & kOobMask) * 4), 0, 0);
                        atomicAdd(&tcnt[tc + slane[ofs >> 26]], (unsigned long long)c);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");
                __builtin_amdgcn_wave_barrier();
                dq_n = 0;
            };
            if constexpr (HASHED) {
                // Rows in groups of kHsGroup2: the group's bucket lines are read together and
                // each row costs five key compares and a select chain. Only a group with a
                // lane on the rare path — key 0 (the side bucket), a probe past a bucket an
                // insert passed full, or a duplicated key (its count) — takes the per-row
                // path below. In the common group every valid entry is a single hit or a miss,
                // so the correction running sum (count - 1 = -1 per miss) is the misses'
                // ballot prefix (mbcnt) instead of a DPP scan. A bucket whose meta bit 0 is
                // set is full (an insert sets it only after finding no free slot), so the
                // empty-slot test of scan_line is not needed for `more`.
#pragma unroll
                for (int g0 = 0; g0 < NU; g0 += kHsGroup2) {
                    if (w0 + g0 * 64 >= R) continue;  // uniform: past the run
                    uint4 ln[kHsGroup2][4];
                    uint32_t hb[kHsGroup2];  // home bucket (absolute; 0 for an unused lane)
#pragma unroll
                    for (int j = 0; j < kHsGroup2; ++j) {
                        const uint32_t o = off[g0 + j] & kOobMask;
                        const unsigned long long sk = ev[g0 + j];
                        const bool use = o != kOob && sk != 0;
                        hb[j] = use ? stored_bucket(sk, tv.nb) : sbase;
                        lds_line(reinterpret_cast<const uint4*>(s_tab), hb[j] - sbase, ln[j][0], ln[j][1], ln[j][2],
                                 ln[j][3]);
                    }
                    uint32_t vv[kHsGroup2];
                    bool mo_[kHsGroup2];
                    bool rare = false;
#pragma unroll
                    for (int j = 0; j < kHsGroup2; ++j) {
                        const uint32_t o = off[g0 + j] & kOobMask;
                        const unsigned long long sk = ev[g0 + j];
                        const uint4 a0 = ln[j][0], a1 = ln[j][1], a2 = ln[j][2], a3 = ln[j][3];
                        const unsigned long long k0 = ((unsigned long long)a0.y << 32) | a0.x;
                        const unsigned long long k1 = ((unsigned long long)a0.w << 32) | a0.z;
                        const unsigned long long k2 = ((unsigned long long)a1.y << 32) | a1.x;
                        const unsigned long long k3 = ((unsigned long long)a1.w << 32) | a1.z;
                        const unsigned long long k4 = ((unsigned long long)a2.y << 32) | a2.x;
                        uint32_t ref = k4 == sk ? a3.z : kMiss;
                        ref = k3 == sk ? a3.y : ref;
                        ref = k2 == sk ? a3.x : ref;
                        ref = k1 == sk ? a2.w : ref;
                        ref = k0 == sk ? a2.z : ref;
                        const bool valid = o != kOob;
                        // a miss in a bucket some insert passed full (meta bit 0, so no free
                        // slot): probe on inside the chunk, the lanes that need it only
                        const bool mo = valid & (sk != 0) & (ref == kMiss) & ((a3.w & 1u) != 0);
                        mo_[j] = mo;  // queued in the common branch below
                        vv[j] = valid ? ref : kMiss;
                        // rare: key 0 (the side bucket) or a duplicated key (its count)
                        rare |= valid & ((sk == 0) | ((ref >= kDupFlag) & (ref != kMiss)));
                    }
                    if (__ballot(rare) == 0) {
#pragma unroll
                        for (int j = 0; j < kHsGroup2; ++j) {
                            const int u = g0 + j;
                            const uint32_t o = off[u] & kOobMask;
                            {  // queued; counted as a miss here, the flush corrects a hit
                                const unsigned long long mm = __ballot(mo_[j]);
                                if (mm != 0) {  // uniform: most rows (one miss in twenty)
                                    const uint32_t nq = (uint32_t)__builtin_popcountll(mm);
                                    if (dq_n + nq > 64) dq_flush();
                                    if (mo_[j]) {
                                        const uint32_t at = wave * 64 + dq_n +
                                            __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
                                        s_dqk[at] = ev[u];
                                        s_dqo[at] = off[u];
                                    }
                                    dq_n += nq;
                                }
                            }
                            __builtin_amdgcn_raw_buffer_store_b32(vv[j], rres, (int)(o * 4), 0, 0);
                            const bool miss = o != kOob && vv[j] == kMiss;
                            const unsigned long long mm = __ballot(miss);
                            const uint32_t ex = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
                            if (off_end & (1u << u)) scst[off[u] >> 26] = corr_run - ex - (miss ? 1u : 0u);
                            corr_run -= (uint32_t)__builtin_popcountll(mm);
                        }
                        continue;
                    }
#pragma unroll
                    for (int j = 0; j < kHsGroup2; ++j) hashed_row(g0 + j);
                }
                if (dq_n != 0) dq_flush();
            } else {
#pragma unroll
                for (int g0 = 0; g0 < NU; g0 += kLkGroup) {
                  if (w0 + g0 * 64 >= R) continue;  // uniform: past the run
                  uint32_t vv[kLkGroup];
                  bool any = false;
#pragma unroll
                  for (int j = 0; j < kLkGroup; ++j) {
                      const int u = g0 + j;
                      const uint32_t o = off[u] & kOobMask;
                      // ablation 2048: no table read (wrong pairs)
                      vv[j] = DFP_ABL(2048) ? ev[u] : s_tab[ev[u] & ((1u << wlog) - 1)];
                      if (!DFP_ABL(512)) __builtin_amdgcn_raw_buffer_store_b32(vv[j], rres, (int)(o * 4), 0, 0);  // 512: no stores
                      any |= o != kOob && vv[j] >= kDupFlag;
                  }
                  // a missing or duplicated key (kMiss and kDupFlag refs have bit 31 set): its
                  // count, the correction and the odd flag in a wave-uniform branch, so that a
                  // group of single hits (every row of a unique-key build) pays compares and one
                  // ballot (r05: the count chain ran on every row)
                  if (__ballot(any) == 0) {
                      if (corr_run != 0) {  // uniform
#pragma unroll
                          for (int j = 0; j < kLkGroup; ++j)
                              if ((smask[g0 + j] >> lane) & 1ull) scst[off[g0 + j] >> 26] = corr_run;
                      }
                      continue;
                  }
                  {
                      // the group's counts, then its rows' correction scans issued together
                      // (independent until the carry) and its start masks in one LDS round
                      // trip: a build with many missing or duplicated keys (C3) has a special
                      // row in nearly every group (r06)
                      uint32_t dd[kLkGroup];
                      unsigned long long sm[kLkGroup];
                      bool unk = false;
#pragma unroll
                      for (int j = 0; j < kLkGroup; ++j) {
                          sm[j] = smask[g0 + j];
                          const bool special = (off[g0 + j] & kOobMask) != kOob && vv[j] >= kDupFlag;
                          dd[j] = special ? ref_count_inline(vv[j], tv.off_mask) : 1u;
                          unk |= dd[j] == kCountUnknown;
                      }
                      if (__ballot(unk) != 0) {
#pragma unroll
                          for (int j = 0; j < kLkGroup; ++j)
                              if (dd[j] == kCountUnknown) dd[j] = tv.dup_rows[vv[j] & tv.off_mask];
#pragma unroll
                          for (int j = 0; j < kLkGroup; ++j) asm volatile("" : "+v"(dd[j]));
                      }
#pragma unroll
                      for (int j = 0; j < kLkGroup; ++j) {
                          const bool odd = dd[j] != 1u;  // non-special rows hold 1
                          if (odd) sodd[off[g0 + j] >> 26] = 1;
                          uint32_t d = dd[j] - 1u;
                          if (odd && d != 0xFFFFFFFFu && d >= kBigCorr) {
                              atomicAdd(&tcnt[tc + slane[off[g0 + j] >> 26]], (unsigned long long)d);
                              d = 0;
                          }
                          dd[j] = d;
                      }
                      uint32_t sc[kLkGroup];
#pragma unroll
                      for (int j = 0; j < kLkGroup; ++j) sc[j] = wave_incl_scan_dpp(dd[j]);
#pragma unroll
                      for (int j = 0; j < kLkGroup; ++j) {
                          if ((sm[j] >> lane) & 1ull) scst[off[g0 + j] >> 26] = sc[j] + corr_run - dd[j];
                          corr_run += (uint32_t)__builtin_amdgcn_readlane((int)sc[j], 63);
                      }
                  }
                }
            }
            DFP_PH(3);
        }
        // one atomic per tile that has a correction (64 contiguous counters)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");  // LDS only: no wait for the ref stores
        __builtin_amdgcn_wave_barrier();
        int cr = 0;
        bool fodd = false;
        if (len != 0) {
            if constexpr (HASHED) {  // end records: a fragment's minus its predecessor's
                cr = (int)(scst[rank] - (rank > 0 ? scst[rank - 1] : 0u));
            } else {  // start records: the successor's minus its own
                const uint32_t nxt = rank + 1 < nranks ? scst[rank + 1] : corr_run;
                cr = (int)(nxt - scst[rank]);
            }
            // a fragment with an entry of count != 1 (dense: missing or duplicated; hashed:
            // duplicated) also turns off its tile's count-free (dense) or 0/1 (hashed)
            // emission (kOddFlag above the count bits, one atomic for both)
            fodd = sodd[rank] != 0;
        }
        // Measured (r05) and not kept: this atomic held back until the next block's first entry
        // loads had issued (an atomic stays in vmcnt until the memory side has done it, and a
        // wait for loads issued after it waits for it too): C2h lookup 542.6 -> 542.3 us, C3
        // 261.5 -> 261.9, with 2 VGPRs spilled (profiles/r05_lookup_tail_ab.txt)
        const unsigned long long add = (unsigned long long)(long long)cr + (fodd ? kOddFlag : 0ull);
        if (add != 0) atomicAdd(&tcnt[tc + lane], add);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");  // LDS only: no wait for the ref stores
        __builtin_amdgcn_wave_barrier();
        DFP_PH(4);
    }
    wait_image();  // a wave without blocks still meets the image barrier
    DFP_PH_FLUSH();
#ifdef DFP_HJ_ABLATIONS
    __syncthreads();
    DFP_DBG_TS(g_dbg_lk_ts, 2, wall_clock64());
    DFP_DBG_TS(g_dbg_lk_ts, 3, dbg_hwid());
#endif
}

// Measured (r05) and not kept: the dense lookup with L lanes per fragment (a lane group
// owns a fragment whole: its entries walked L at a time, the correction in registers; no
// flattening, masks or owner search) — C2 196 / 210 / 265 / 541 us at L = 4 / 8 / 16 / 64
// against 127 us, C3 362-8185 against 268 (profiles/r05_lookup_lanes.txt): L-lane-wide
// accesses touch 64 / L lines per instruction where the flattened rows touch one or two.
// The lookup's time against fragment length (profiles/r05_lookup_fraglen.txt): about 45-50
// us fixed plus 1.6-1.7 ns per entry at C2's geometry.

// S1 of the hashed sliced probe: per 16384-row tile, the valid rows sorted by slice
// (home bucket >> kHsSliceLog) in LDS; the tile's stored keys (u64) and rows in the
// tile (u16) leave in slice order, with the tile's slice bounds (u16). Persistent, one
// workgroup per CU (128 KB of staged keys): the next tile's keys load into registers
// once this tile's keys are staged, while they and the rows are written out.
template <typename K, bool HAS_VALID>
__global__ void __launch_bounds__(kSlThreads, 4)  // 16 waves per CU: <= 128 VGPRs
hs_partition_kernel(uint32_t nb, uint32_t slog, uint32_t s0, uint32_t nslices, const void* __restrict__ keys,
                    const uint8_t* __restrict__ valid, int64_t voff, int64_t n, int64_t ntiles, bool vec,
                    unsigned long long* __restrict__ ko, uint16_t* __restrict__ rl, uint16_t* __restrict__ toff,
                    unsigned long long* __restrict__ hdr, unsigned long long* __restrict__ tcnt,
                    uint32_t* __restrict__ tent,  // probe pass: slices [s0, s0 + nslices); hdr null = a later pass
                    int64_t tile_off, int64_t row_base, uint32_t* __restrict__ tile_base) {  // build: tcnt null
    __shared__ __attribute__((aligned(16))) unsigned long long s_key[kSlTile];  // also the rows (u16) pass
    __shared__ __attribute__((aligned(16))) uint32_t s_hist[kSlHistBins];
    __shared__ uint32_t s_w[kSlThreads / 64];
    const uint32_t nbins = nslices + 1;
    const bool probe = tcnt != nullptr;  // else the hashed frag build's partition of one build segment
    const bool later = probe && hdr == nullptr;
    if (probe && !later && blockIdx.x == 0 && threadIdx.x == 0) {
        hdr[0] = hdr[1] = 0;  // workspace header (error word)
        tcnt[ntiles] = 0;     // the emission's tile counter
    }
    int64_t k[kSlGroups][4], nk[kSlGroups][4];
    auto load = [&](int64_t t, int64_t (&dst)[kSlGroups][4], uint32_t tx) {
#pragma unroll
        for (int g = 0; g < kSlGroups; ++g)
            load4<K>(keys, t * kSlTile + g * (kSlThreads * 4) + tx * 4, n, vec, dst[g]);
    };
    int64_t tile = blockIdx.x;
    if (tile < ntiles) load(tile, nk, threadIdx.x);
    for (; tile < ntiles; tile += gridDim.x) {
        // the thread index made opaque per tile: otherwise the compiler hoists the rows'
        // offsets and addresses out of the tile loop and spills them
        uint32_t tx = threadIdx.x;
        asm volatile("" : "+v"(tx));
        const int64_t tile0 = tile * kSlTile;
        const int64_t gtile = tile + tile_off;  // its output region (the build partitions several segments)
#pragma unroll
        for (int g = 0; g < kSlGroups; ++g)
#pragma unroll
            for (int q = 0; q < 4; ++q) k[g][q] = nk[g][q];
        for (uint32_t b = tx; b < kSlHistBins; b += kSlThreads) s_hist[b] = 0;
        const uint32_t ebase = later ? tent[tile] : 0u;
        __syncthreads();
        uint32_t sr[kSlGroups][4];  // slice << 14 | rank in slice, ~0 = no entry
#pragma unroll
        for (int g = 0; g < kSlGroups; ++g) {
            const int loc0 = g * (kSlThreads * 4) + tx * 4;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t row = tile0 + loc0 + q;
                const unsigned long long sk = stored_key(k[g][q]);
                const uint32_t sl = (stored_bucket(sk, nb) >> slog) - s0;  // wraps past the pass: no entry
                const bool ok = row < n && (!HAS_VALID || bit_valid(valid, voff, row)) && sl < nslices;
                sr[g][q] = ok ? (sl << kSlTileLog) | atomicAdd(&s_hist[sl], 1u) : 0xFFFFFFFFu;
            }
        }
        __syncthreads();
        uint32_t tot;
        hist_excl_scan(s_hist, s_w, &tot);
        uint16_t* to = toff + gtile * (int64_t)nbins;
        for (uint32_t b = tx; b < nbins; b += kSlThreads) to[b] = (uint16_t)(ebase + s_hist[b]);
        if (tx == 0 && probe) {
            tcnt[tile] = (later ? tcnt[tile] : 0ull) + tot;  // S2 corrects it to the tile's pair count
            tent[tile] = ebase + tot;
        }
        if (tx == 0 && tile_base != nullptr) tile_base[gtile] = (uint32_t)(row_base + tile0);
        // pass 1: stored keys in slice order
#pragma unroll
        for (int g = 0; g < kSlGroups; ++g)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (sr[g][q] != 0xFFFFFFFFu)
                    s_key[s_hist[sr[g][q] >> kSlTileLog] + (sr[g][q] & (kSlTile - 1))] = stored_key(k[g][q]);
        __syncthreads();
        if (tile + (int64_t)gridDim.x < ntiles) load(tile + gridDim.x, nk, tx);  // in flight during the write-out
        unsigned long long* dk = ko + gtile * kSlTile + ebase;
        if (ebase & 1) {  // a later pass at an odd base: 8-byte stores
            for (uint32_t i = tx; i < tot; i += kSlThreads) dk[i] = s_key[i];
        } else {
            for (uint32_t i = tx * 2; i < tot; i += kSlThreads * 2) {
                if (i + 2 <= tot) *reinterpret_cast<ulonglong2*>(dk + i) = *reinterpret_cast<const ulonglong2*>(s_key + i);
                else dk[i] = s_key[i];
            }
        }
        __syncthreads();
        // pass 2: rows in the tile (u16), same order
        uint16_t* s_row = reinterpret_cast<uint16_t*>(s_key);
#pragma unroll
        for (int g = 0; g < kSlGroups; ++g)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (sr[g][q] != 0xFFFFFFFFu)
                    s_row[s_hist[sr[g][q] >> kSlTileLog] + (sr[g][q] & (kSlTile - 1))] =
                        (uint16_t)(g * (kSlThreads * 4) + tx * 4 + q);
        __syncthreads();
        uint16_t* dr = rl + gtile * kSlTile + ebase;
        if (ebase & 7) {  // a later pass at an unaligned base: 2-byte stores
            for (uint32_t i = tx; i < tot; i += kSlThreads) dr[i] = s_row[i];
        } else {
            for (uint32_t i = tx * 8; i < tot; i += kSlThreads * 8) {
                if (i + 8 <= tot) *reinterpret_cast<uint4*>(dr + i) = *reinterpret_cast<const uint4*>(s_row + i);
                else for (uint32_t j = i; j < tot; ++j) dr[j] = s_row[j];
            }
        }
        __syncthreads();  // s_key / s_hist are rewritten for the next tile
    }
}

// The same for 2^15-row tiles (a hashed table's probe, and the hashed frag build). The tile's 32 stored
// keys per thread stay in registers; the ranks, then the sorted positions, live in LDS
// (u16 per row: holding them in registers beside the keys spills), and the sorted keys
// leave through a 64 KB staging area in four quarters of 2^13 positions. Once the last
// quarter is staged the key registers are free: the next tile's keys load into them
// while that quarter and the rows are written out.
template <typename K, bool HAS_VALID>
__global__ void __launch_bounds__(kSlThreads, 4)  // 16 waves per CU: <= 128 VGPRs
hs_partition32_kernel(uint32_t nb, uint32_t slog, uint32_t s0, uint32_t nslices, const void* __restrict__ keys,
                      const uint8_t* __restrict__ valid, int64_t voff, int64_t n, int64_t ntiles, bool vec,
                      unsigned long long* __restrict__ ko, uint16_t* __restrict__ rl, uint16_t* __restrict__ toff,
                      unsigned long long* __restrict__ hdr, unsigned long long* __restrict__ tcnt,
                      uint32_t* __restrict__ tent,  // probe pass: slices [s0, s0 + nslices); hdr null = a later pass
                      int64_t tile_off, int64_t row_base, uint32_t* __restrict__ tile_base) {  // build: tcnt null
    using T = SlT<15>;
    constexpr int kQ = T::kRows / 4;      // positions per staging quarter
    constexpr uint16_t kNone = 0xFFFFu;   // no entry (positions and ranks are < 2^15)
    __shared__ __attribute__((aligned(16))) unsigned long long s_key[kQ];  // also the rows (u16) pass
    __shared__ __attribute__((aligned(16))) uint16_t s_pos[T::kRows];      // per row: rank, then position
    __shared__ __attribute__((aligned(16))) uint32_t s_hist[kSlHistBins];
    __shared__ uint32_t s_w[kSlThreads / 64];
    const uint32_t nbins = nslices + 1;
    const bool probe = tcnt != nullptr;  // else the hashed frag build's partition of one build segment
    const bool later = probe && hdr == nullptr;
    if (probe && !later && blockIdx.x == 0 && threadIdx.x == 0) {
        hdr[0] = hdr[1] = 0;  // workspace header (error word)
        tcnt[ntiles] = 0;     // the emission's tile counter
    }
    int64_t k[T::kGroups][4];  // the keys, then their stored keys
    auto load = [&](int64_t t, uint32_t tx) {
#pragma unroll
        for (int g = 0; g < T::kGroups; ++g)
            load4<K>(keys, t * T::kRows + g * (kSlThreads * 4) + tx * 4, n, vec, k[g]);
    };
    auto slice_of = [&](unsigned long long sk) { return (stored_bucket(sk, nb) >> slog) - s0; };  // wraps past the pass
    int64_t tile = blockIdx.x;
    if (tile < ntiles) load(tile, threadIdx.x);
    for (; tile < ntiles; tile += gridDim.x) {
        // the thread index made opaque per tile: otherwise the compiler hoists every per-row
        // offset and address of the 32 rows out of the tile loop and spills them
        uint32_t tx = threadIdx.x;
        asm volatile("" : "+v"(tx));
        const int64_t tile0 = tile * T::kRows;
        const int64_t gtile = tile + tile_off;  // its output region (the build partitions several segments)
        for (uint32_t b = tx; b < kSlHistBins; b += kSlThreads) s_hist[b] = 0;
        const uint32_t ebase = later ? tent[tile] : 0u;
        __syncthreads();
        // ranks in slice: rows loc0 .. loc0 + 3 of group g are four adjacent u16 (one 8-byte LDS
        // access). One group at a time (a scheduling barrier after each): interleaving the 32
        // rows' key hashes for ILP spills
#pragma unroll
        for (int g = 0; g < T::kGroups; ++g) {
            const int loc0 = g * (kSlThreads * 4) + tx * 4;
            uint32_t r[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t row = tile0 + loc0 + q;
                const unsigned long long sk = stored_key(k[g][q]);
                k[g][q] = (int64_t)sk;
                const uint32_t sl = slice_of(sk);
                const bool ok = row < n && (!HAS_VALID || bit_valid(valid, voff, row)) && sl < nslices;
                r[q] = ok ? atomicAdd(&s_hist[sl], 1u) : kNone;
            }
            *reinterpret_cast<uint2*>(s_pos + loc0) = make_uint2(r[0] | (r[1] << 16), r[2] | (r[3] << 16));
            // Measured (r05) and not kept: 2 or 8 groups per scheduling region (the rank
            // atomics of several groups in flight; no spills either way): partition equal
            // within noise, C2h 70.2-70.4K vs 70.3-70.6K Mrows/s (profiles/r05_hs32_rank_groups.txt)
            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
        asm volatile("" : "+v"(tx));  // (again: the offsets of the phases below are recomputed, not kept live)
        uint32_t tot;
        hist_excl_scan_lanes(s_hist, s_w, &tot);
        asm volatile("" : "+v"(tx));
        uint16_t* to = toff + gtile * (int64_t)nbins;
        for (uint32_t b = tx; b < nbins; b += kSlThreads) to[b] = (uint16_t)(ebase + s_hist[b]);
        if (tx == 0 && probe) {
            tcnt[tile] = (later ? tcnt[tile] : 0ull) + tot;  // S2 corrects it to the tile's pair count
            tent[tile] = ebase + tot;
        }
        if (tx == 0 && tile_base != nullptr) tile_base[gtile] = (uint32_t)(row_base + tile0);
        // ranks -> sorted positions (each thread rewrites only its own rows)
#pragma unroll
        for (int g = 0; g < T::kGroups; ++g) {
            const int loc0 = g * (kSlThreads * 4) + tx * 4;
            const uint2 v = *reinterpret_cast<const uint2*>(s_pos + loc0);
            uint32_t r[4] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16};
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (r[q] != kNone) r[q] += s_hist[slice_of((unsigned long long)k[g][q])];
            *reinterpret_cast<uint2*>(s_pos + loc0) = make_uint2(r[0] | (r[1] << 16), r[2] | (r[3] << 16));
        }
        unsigned long long* dk = ko + gtile * T::kRows + ebase;
        // stored keys in slice order, a quarter of the positions at a time (every quarter is
        // staged, so that the next tile's loads follow every use of k)
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            asm volatile("" : "+v"(tx));
            const uint32_t p0 = h * kQ;
            const uint32_t p1 = min<uint32_t>(tot, p0 + kQ);
#pragma unroll
            for (int g = 0; g < T::kGroups; ++g) {
                const int loc0 = g * (kSlThreads * 4) + tx * 4;
                const uint2 v = *reinterpret_cast<const uint2*>(s_pos + loc0);
                const uint32_t r[4] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16};
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (r[q] - p0 < (uint32_t)kQ) s_key[r[q] - p0] = (unsigned long long)k[g][q];  // kNone: never
            }
            __syncthreads();
            // the last quarter staged: the key registers are free, the next tile loads into them
            if (h == 3 && tile + (int64_t)gridDim.x < ntiles) load(tile + gridDim.x, tx);
            if (ebase & 1) {  // a later pass at an odd base: 8-byte stores
                for (uint32_t i = p0 + tx; i < p1; i += kSlThreads) dk[i] = s_key[i - p0];
            } else {
                for (uint32_t i = p0 + tx * 2; i < p1; i += kSlThreads * 2) {
                    if (i + 2 <= p1) *reinterpret_cast<ulonglong2*>(dk + i) = *reinterpret_cast<const ulonglong2*>(s_key + (i - p0));
                    else dk[i] = s_key[i - p0];
                }
            }
            __syncthreads();
        }
        // rows in the tile (u16), same order: 2^15 u16 in the staging area
        uint16_t* s_row = reinterpret_cast<uint16_t*>(s_key);
#pragma unroll
        for (int g = 0; g < T::kGroups; ++g) {
            const int loc0 = g * (kSlThreads * 4) + tx * 4;
            const uint2 v = *reinterpret_cast<const uint2*>(s_pos + loc0);
            const uint32_t r[4] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16};
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (r[q] != kNone) s_row[r[q]] = (uint16_t)(loc0 + q);
        }
        __syncthreads();
        uint16_t* dr = rl + gtile * T::kRows + ebase;
        if (ebase & 7) {  // a later pass at an unaligned base: 2-byte stores
            for (uint32_t i = tx; i < tot; i += kSlThreads) dr[i] = s_row[i];
        } else {
            for (uint32_t i = tx * 8; i < tot; i += kSlThreads * 8) {
                if (i + 8 <= tot) *reinterpret_cast<uint4*>(dr + i) = *reinterpret_cast<const uint4*>(s_row + i);
                else for (uint32_t j = i; j < tot; ++j) dr[j] = s_row[j];
            }
        }
        __syncthreads();  // s_key / s_pos / s_hist are rewritten for the next tile
    }
}

// Measured (r05) and not kept: the 2^15-row form with the sorted positions packed two per
// register (u16 halves) instead of in LDS and the keys staged in two halves of 2^14
// positions (so that the next tile's loads overlap more of the write-out): 62-72 VGPRs
// spilled at the 128-register budget.
// Measured (r05) and not kept: this partition in two workgroups per CU (one tile each, the
// sorted keys staged in two 64 KB halves): its 16 (1024 threads) or 32 (512 threads) stored
// keys per thread plus their ranks need more than the 64 / 128 VGPRs that two workgroups per
// CU allow (50-130 spilled), so it was not timed.

// row count behind a ref; packed dense refs carry counts <= 15 in bits 27-30. Other
// duplicated keys read the count from their segment header, in a wave-uniform branch
// that also waits for it there: merged into the common path, that load's wait would be
// an s_waitcnt vmcnt(0) on every step for every ref (loads and stores share vmcnt) —
// waiting for the next tile's prefetch in the emission's count pass and for the
// previous step's stores in its write pass (C2 emit 222 -> ? us).
__device__ __forceinline__ uint32_t sl_count(const TableView& tv, uint32_t r) {
    uint32_t c = ref_count_inline(r, tv.off_mask);
    if (__ballot(c == kCountUnknown) != 0) {
        if (c == kCountUnknown) c = tv.dup_rows[r & tv.off_mask];
        asm volatile("" : "+v"(c));  // the wait stays in this branch
    }
    return c;
}

// S3b: 512 threads per tile, two workgroups per CU (64 KB of LDS and <= 128 VGPRs each).
// Wave w owns the tile's rows [w * 2048, (w + 1) * 2048) and walks them 64 at a time,
// lane l on row +l: pass 1 counts the wave's pairs, pass 2 writes them. Within a wave
// step the pairs of consecutive rows are consecutive, so the stores of one instruction
// cover one contiguous run (no LDS staging, no barriers in the emission).
constexpr int kSlEmitThreads = 512;
constexpr int kSlWaveRows = kSlTile / (kSlEmitThreads / 64);  // 2048
// the count-free emission reads a wave's entry count as wcnt[tile * kSlRanges + wave]: one
// partition range per emission wave
static_assert(kSlEmitThreads / 64 == kSlRanges && kSlWaveRows == kSlRangeRows,
              "emission waves and the partition's entry-count ranges must coincide");

template <bool HAS_ROW_IDS, bool HAS_PROBE_IDS, int TL = kSlTileLog>
// 16 waves per CU (two 512-thread workgroups, or one of 1024 for 2^15-row tiles): <= 128 VGPRs
__global__ void __launch_bounds__(SlT<TL>::kEmitThreads, 4)
sl_emit_kernel(TableView tv, const uint32_t* __restrict__ tent, const uint16_t* __restrict__ rl,
               const uint32_t* __restrict__ res, const uint32_t* __restrict__ probe_ids, uint32_t pbase,
               const unsigned long long* __restrict__ tcnt, int64_t ntiles, uint64_t* __restrict__ out_b,
               uint32_t* __restrict__ out_p, int64_t cap, int64_t* __restrict__ d_total,
               const uint16_t* __restrict__ wcnt,  // entries per 2048-row range (null: always count)
               unsigned long long* __restrict__ dyn,  // tile counter (zeroed by S1), null: static tiles
               bool flag01) {  // hashed: a tile without the lookup's flag has row counts 0 or 1
    // (wcnt non-null: the dense count-free path; flag01: the hashed 0/1 path; at most one)
    __shared__ __attribute__((aligned(16))) uint32_t s_ref[SlT<TL>::kRows];  // the tile's refs, kMiss = none
    __shared__ unsigned long long s_w[SlT<TL>::kEmitThreads / 64];
    __shared__ unsigned long long s_pre[SlT<TL>::kEmitThreads / 64];
    __shared__ uint32_t s_own[SlT<TL>::kEmitThreads / 64][64];  // per wave: owner markers of one output window
    __shared__ int64_t s_nxt;                              // dyn: the tile after the next one
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // Measured (r04) and not kept: nontemporal pair stores (C2 162.4K -> 140.8K Mrows/s) and
    // nontemporal probe-key loads in the partition (-3.5 %), profiles/r04_nontemporal_ab.txt
    auto put = [&](unsigned long long o, uint64_t b, uint32_t p) {
        out_b[o] = b;
        out_p[o] = p;
    };
    constexpr int U = SlT<TL>::kRows / (SlT<TL>::kEmitThreads * 4);  // 8 x (4 rows + 4 refs) per thread
    uint2 e4[U];
    uint4 r4[U];
    uint32_t cnt = 0;
    // count-free tiles: every entry's key had exactly one row (no correction flag), so a
    // wave's pair count is its range's entry count and a row's count is 0 (kMiss) or 1
    uint32_t nflag = 1, nwc = 0;
    // Persistent: workgroup b takes tile b, then tiles b + grid, b + 2 grid, ... (static)
    // or, with dyn, the grid + i-th tile for the i-th draw of the tile counter (every
    // workgroup's tiles still ascend, and a slow CU takes fewer tiles: the static grid's
    // workgroups ended 110-153 us into a 154 us C2 emission); the next tile's entries are
    // loaded while this tile's pairs are counted and written. All loads of a tile are
    // issued at once, after its entry count. A tile's output offset is the sum of the
    // pair counts (tcnt, final once S2 is done) of the tiles below it: the first tile's
    // from scratch, each next one's as this one's plus the grid's counts in between (one
    // load per thread), so no scan launch runs between S2 and S3.
    auto count_sum = [&](int64_t lo, int64_t hi) -> unsigned long long {  // this thread's share
        unsigned long long v = 0;
        for (int64_t j = lo + threadIdx.x; j < hi; j += SlT<TL>::kEmitThreads) v += tcnt[j] & kCountMask;
        return v;
    };
    auto fetch = [&](int64_t t) {
        cnt = DFP_ABL(2) ? 0u : tent[t];  // the tile's entries over every pass
        if (wcnt != nullptr || flag01) nflag = (uint32_t)(tcnt[t] >> kOddShift);  // the lookup's flag: some count != 1
        if (wcnt != nullptr) nwc = wcnt[t * SlT<TL>::kRanges + wave];
        const uint16_t* te = rl + t * SlT<TL>::kRows;
        const uint32_t* tr = res + t * SlT<TL>::kRows;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = (u * SlT<TL>::kEmitThreads + threadIdx.x) * 4;
            if (i < cnt) {  // whole uint4s: the region holds SlT<TL>::kRows entries, lanes past cnt are ignored
                e4[u] = *reinterpret_cast<const uint2*>(te + i);
                r4[u] = *reinterpret_cast<const uint4*>(tr + i);
            }
        }
    };
    DFP_DBG_TS(g_dbg_em_ts, 0, wall_clock64());
    int64_t tile = blockIdx.x;
    if (tile < ntiles) fetch(tile);
    unsigned long long base = 0;  // the current tile's output offset
    int64_t next;                 // this workgroup's next tile
    {
        const unsigned long long v = wave_sum<unsigned long long>(count_sum(0, min<int64_t>(tile, ntiles)));
        if (lane == 0) s_pre[wave] = v;
        if (dyn != nullptr && threadIdx.x == 0) s_nxt = (int64_t)gridDim.x + (int64_t)atomicAdd(dyn, 1ull);
        __syncthreads();
        for (int w = 0; w < SlT<TL>::kEmitThreads / 64; ++w) base += s_pre[w];
        next = dyn != nullptr ? s_nxt : tile + gridDim.x;
        __syncthreads();
    }
    DFP_DBG_TS(g_dbg_em_ts, 1, wall_clock64());
    // The image is cleared once; the write pass puts kMiss back into every row it reads, so
    // no clear and no barrier for it stand between a tile and the next one's scatter
    // (the diagnostic ablation without a write pass clears it before every tile)
    const bool reset_rows = !DFP_ABL(1);
    auto clear_image = [&]() {
        for (int i = threadIdx.x * 4; i < SlT<TL>::kRows; i += SlT<TL>::kEmitThreads * 4)
            *reinterpret_cast<uint4*>(s_ref + i) = make_uint4(kMiss, kMiss, kMiss, kMiss);
        __syncthreads();
    };
    if (reset_rows) clear_image();
    while (tile < ntiles) {
        // dyn: draw the tile after the next one now; its value is needed only at the end
        // of this tile, so the atomic's round trip hides behind the tile's work
        unsigned long long draw = 0;
        if (dyn != nullptr && threadIdx.x == 0 && next < ntiles) draw = atomicAdd(dyn, 1ull);
        const int64_t tile0 = tile * SlT<TL>::kRows;
        if (!reset_rows) clear_image();
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = (u * SlT<TL>::kEmitThreads + threadIdx.x) * 4;
            if (i < cnt) s_ref[e4[u].x & 0xFFFF] = r4[u].x;
            if (i + 1 < cnt) s_ref[e4[u].x >> 16] = r4[u].y;
            if (i + 2 < cnt) s_ref[e4[u].y & 0xFFFF] = r4[u].z;
            if (i + 3 < cnt) s_ref[e4[u].y >> 16] = r4[u].w;
        }
        __syncthreads();
        const bool fast = wcnt != nullptr && nflag == 0;  // this tile's (read before the prefetch)
        // hashed, no duplicated key in the tile: every row has 0 or 1 pairs (misses are the
        // common case, so a wave's pairs are still counted, by its hits)
        const bool b01 = flag01 && nflag == 0;
        const uint32_t fast_wc = nwc;
        if (next < ntiles) fetch(next);
        // pass 1: this wave's pair count (a count-free tile: its entries in the wave's range)
        const int row_w = wave * kSlWaveRows;
        if (fast) {
            if (lane == 0) s_w[wave] = fast_wc;
        } else if (b01) {
            uint32_t lsum = 0;  // <= 32
#pragma unroll 8
            for (int k = 0; k < kSlWaveRows; k += 64) lsum += s_ref[row_w + k + lane] != kMiss ? 1u : 0u;
            const uint32_t wsum = wave_sum_dpp(lsum);
            if (lane == 0) s_w[wave] = wsum;
        } else {
            uint32_t lsum = 0;  // < 32 rows x < 2^26 rows each
#pragma unroll 8
            for (int k = 0; k < kSlWaveRows; k += 64) lsum += sl_count(tv, s_ref[row_w + k + lane]);
            // wave total in u64: two 32-bit halves of the per-lane sums
            const unsigned long long wsum = (unsigned long long)wave_sum_dpp(lsum & 0xFFFFu) +
                                            ((unsigned long long)wave_sum_dpp(lsum >> 16) << 16);
            if (lane == 0) s_w[wave] = wsum;
        }
        __syncthreads();
        unsigned long long pos = base, tile_total = 0;
        for (int w = 0; w < SlT<TL>::kEmitThreads / 64; ++w) {
            if (w < wave) pos += s_w[w];
            tile_total += s_w[w];
        }
        if (tile == ntiles - 1 && threadIdx.x == 0) *d_total = (int64_t)(base + tile_total);
        if (!DFP_ABL(1)) {
            // pass 2: write the wave's pairs, 64 rows per step. Steps whose rows all have
            // at most one pair store them directly; a step with a duplicated key expands
            // its pairs over the lanes, 64 output positions at a time (owner row by a
            // max-scan of start markers), so every store instruction writes one
            // contiguous run and the duplicate segments are read in parallel.
            uint32_t* own = s_own[wave];
            if (fast || b01) {
                // count-free tile: one pair per hit row, the prefix a popcount of the hit mask
#pragma unroll 4
                for (int k = 0; k < kSlWaveRows; k += 64) {
                    const int loc = row_w + k + lane;
                    const uint32_t r = s_ref[loc];
                    if (reset_rows) s_ref[loc] = kMiss;
                    const unsigned long long hit = __ballot(r != kMiss);
                    if (r != kMiss) {
                        const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(hit >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hit, 0u));
                        const unsigned long long o = pos + below;
                        const int64_t row = tile0 + loc;
                        if (o < (unsigned long long)cap) {
                            put(o, HAS_ROW_IDS ? tv.row_ids[r] : (uint64_t)r,
                                HAS_PROBE_IDS ? probe_ids[row] : (uint32_t)row + pbase);
                        }
                    }
                    pos += (uint32_t)__builtin_popcountll(hit);
                }
            }
            // Measured (r04) and not kept: counted tiles in batches of 4 steps whose duplicate
            // segment reads (up to 8 output windows) were all issued before any of their
            // stores — C3 emission 666 -> 670 us: the segment reads are bound by the rate of
            // random line reads into dup_rows (30 MB, Infinity-Cache resident), not by one
            // round trip per window.
#pragma unroll 2
            for (int k = 0; !fast && !b01 && k < kSlWaveRows; k += 64) {
                const int loc = row_w + k + lane;
                const uint32_t r = s_ref[loc];
                if (reset_rows) s_ref[loc] = kMiss;
                const uint32_t c = sl_count(tv, r);
                const int64_t row = tile0 + loc;
                uint32_t total;
                if (__ballot(c > 1) == 0) {
                    // at most one pair per row: the prefix is a popcount of the hit mask
                    const unsigned long long hit = __ballot(c != 0);
                    total = (uint32_t)__builtin_popcountll(hit);
                    if (c) {
                        const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(hit >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hit, 0u));
                        const unsigned long long o = pos + below;
                        if (o < (unsigned long long)cap) {
                            put(o, HAS_ROW_IDS ? tv.row_ids[r] : (uint64_t)r,
                                HAS_PROBE_IDS ? probe_ids[row] : (uint32_t)row + pbase);
                        }
                    }
                } else {
                    const uint32_t incl = wave_incl_scan_dpp(c);  // < 2^32: 64 rows of < 2^26 rows each
                    total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                    const uint32_t excl = incl - c;
                    // a step whose duplicated keys are all run refs (or single rows): the build row
                    // of output position p is (top + excl) - p of its owner row - one cross-lane
                    // read per window instead of two, no segment read (r06)
                    const bool runs_only = __ballot(c > 1u && !run_ref(r, tv.off_mask)) == 0;
                    const uint32_t vsum = ((r & kDupFlag) ? (r & 0xFFFFFFu) : r) + excl;
                    uint32_t carry = 0;
                    // Measured (r04) and not kept: each window's pairs stored one window later
                    // (the next window's segment read issued first, two register sets): C3
                    // emission 666 -> 676 us — the compiler's in-order vmcnt waits still put a
                    // store round trip in every iteration.
                    for (uint32_t w0 = 0; w0 < total; w0 += 64) {
                        own[lane] = 0;
                        __builtin_amdgcn_wave_barrier();
                        if (c && excl >= w0 && excl < w0 + 64) own[excl - w0] = (uint32_t)lane + 1;
                        __builtin_amdgcn_wave_barrier();
                        const uint32_t ol = max(wave_incl_max_dpp(own[lane]), carry);
                        carry = (uint32_t)__builtin_amdgcn_readlane((int)ol, 63);
                        const int j = (int)((ol - 1) & 63);
                        const uint32_t p = w0 + lane;
                        uint32_t br;
                        if (runs_only) {
                            br = (uint32_t)__shfl((int)vsum, j, 64) - p;
                        } else {
                            const uint32_t xj = (uint32_t)__shfl((int)excl, j, 64);
                            const uint32_t rj = (uint32_t)__shfl((int)r, j, 64);
                            br = !(rj & kDupFlag) ? rj
                                 : DFP_ABL(8) ? (rj & tv.off_mask) + (p - xj)  // ablation: no segment reads
                                              : (p < total ? dup_ref_row(tv.dup_rows, rj, tv.off_mask, p - xj) : 0u);
                        }
                        const unsigned long long o = pos + p;
                        if (p < total && o < (unsigned long long)cap) {
                            const int64_t rowj = tile0 + row_w + k + j;
                            put(o, HAS_ROW_IDS ? tv.row_ids[br] : (uint64_t)br,
                                HAS_PROBE_IDS ? probe_ids[rowj] : (uint32_t)rowj + pbase);
                        }
                        __builtin_amdgcn_wave_barrier();
                    }
                }
                pos += total;
            }
        }
        // the next tile's offset: this one's plus the counts of the tiles in between (loaded
        // only now: a wait on them would also wait for the next tile's entries in flight)
        const unsigned long long pre = wave_sum<unsigned long long>(next < ntiles ? count_sum(tile, next) : 0ull);
        if (lane == 0) s_pre[wave] = pre;
        if (dyn != nullptr && threadIdx.x == 0) s_nxt = next < ntiles ? (int64_t)gridDim.x + (int64_t)draw : ntiles;
        __syncthreads();  // s_ref, s_w, s_pre and s_nxt are rewritten for the next tile
        for (int w = 0; w < SlT<TL>::kEmitThreads / 64; ++w) base += s_pre[w];
        tile = next;
        next = dyn != nullptr ? s_nxt : next + gridDim.x;
    }
    DFP_DBG_TS(g_dbg_em_ts, 2, wall_clock64());
    DFP_DBG_TS(g_dbg_em_ts, 3, dbg_hwid());
}

#ifdef DFP_HJ_ABLATIONS
// diagnostic build only: copy the last sliced lookup's (which = 0) or emission's (1)
// per-workgroup timeline (4 u64 per workgroup, see g_dbg_lk_ts) to host memory
extern "C" __attribute__((visibility("default"))) int hj_debug_timeline(int which, unsigned long long* host, int nblocks) {
    const size_t bytes = sizeof(unsigned long long) * 4 * (size_t)std::min(nblocks, 65536);
    return which == 0 ? (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dbg_lk_ts), bytes)
                      : (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dbg_em_ts), bytes);
}
// diagnostic build only: the lookup's phase cycle sums (g_dbg_lk_ph, 8 u64); reset = 1
// zeroes them after the copy
extern "C" __attribute__((visibility("default"))) int hj_debug_lookup_phases(unsigned long long* host, int reset) {
    int e = (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dbg_lk_ph), 8 * sizeof(unsigned long long));
    if (e == 0 && reset) {
        static const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        e = (int)hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_lk_ph), z, sizeof(z));
    }
    return e;
}
#endif

// ---------------------------------------------------------------------------
// table queries (not on the hot path)
// ---------------------------------------------------------------------------
__global__ void table_stats_kernel(TableView tv, unsigned long long* out) {
    unsigned long long distinct = 0, dupk = 0, dupr = 0, mx = 0;
    const uint64_t nslots = tv.dense ? tv.drange - 1 : (uint64_t)tv.nb * kSlots;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= nslots; s += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t c = 0;
        if (tv.dense) {
            c = ref_count(tv.dup_rows, tv.dense[s], tv.off_mask);
        } else if (s == nslots) {  // side bucket
            c = tv.tbl[tv.nb].meta;
        } else if (tv.tbl[s / kSlots].key[s % kSlots] != 0) {
            c = ref_count(tv.dup_rows, tv.tbl[s / kSlots].ref[s % kSlots], tv.off_mask);
        }
        if (c) {
            distinct++;
            if (c > 1) { dupk++; dupr += c; }
            if (c > mx) mx = c;
        }
    }
    distinct = wave_sum(distinct);
    dupk = wave_sum(dupk);
    dupr = wave_sum(dupr);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long o = __shfl_xor(mx, d, 64);
        mx = o > mx ? o : mx;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&out[0], distinct);
        atomicAdd(&out[1], dupk);
        atomicAdd(&out[2], dupr);
        atomicMax(&out[3], mx);
    }
}

__global__ void chain_fill_kernel(int64_t* prev, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        prev[i] = -1;
}

__global__ void chain_links_kernel(TableView tv, int64_t* prev) {
    const uint64_t nslots = tv.dense ? tv.drange - 1 : (uint64_t)tv.nb * kSlots;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= nslots; s += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t ref;
        if (tv.dense) {
            ref = tv.dense[s];
            if (ref == kMiss) continue;
        } else if (s == nslots) {
            if (tv.tbl[tv.nb].meta < 2) continue;
            ref = tv.tbl[tv.nb].ref[0];
        } else {
            if (tv.tbl[s / kSlots].key[s % kSlots] == 0) continue;
            ref = tv.tbl[s / kSlots].ref[s % kSlots];
        }
        if (!(ref & kDupFlag)) continue;
        const uint32_t c = ref_count(tv.dup_rows, ref, tv.off_mask);
        for (uint32_t t = 0; t + 1 < c; ++t)
            prev[dup_ref_row(tv.dup_rows, ref, tv.off_mask, t)] = dup_ref_row(tv.dup_rows, ref, tv.off_mask, t + 1);
    }
}

// ---------------------------------------------------------------------------
// radix partition (multi-GPU exchange): stable multi-split by the low hash bits
// ---------------------------------------------------------------------------
constexpr int kPartThreads = 256;
constexpr int kPartChunk = 4096;  // rows per block
constexpr int kMaxParts = 64;

template <typename K>
__device__ __forceinline__ int part_of(const void* keys, const uint8_t* valid, int64_t voff, int64_t i, int64_t n,
                                       int mask, const PartSpec& sp) {
    if (i >= n || !bit_valid(valid, voff, i)) return -1;
    const int64_t k = ld_key<K>(keys, i);
    if (k < sp.lo || k > sp.hi) return -1;  // cannot match: dropped before the exchange
    if (sp.by_range) return (int)__umul64hi((uint64_t)k - (uint64_t)sp.lo, sp.mul);
    return (int)(mix64((uint64_t)k) & (uint64_t)mask);
}

template <typename K>
__global__ void __launch_bounds__(kPartThreads)
part_hist_kernel(const void* keys, const uint8_t* valid, int64_t voff, int64_t n, int nparts, PartSpec sp,
                 uint32_t* hist, int64_t nblocks) {
    __shared__ unsigned s_h[kMaxParts];
    for (int p = threadIdx.x; p < nparts; p += kPartThreads) s_h[p] = 0;
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * kPartChunk;
    for (int k = threadIdx.x; k < kPartChunk; k += kPartThreads) {
        const int p = part_of<K>(keys, valid, voff, r0 + k, n, nparts - 1, sp);
        if (p >= 0) atomicAdd(&s_h[p], 1u);
    }
    __syncthreads();
    for (int p = threadIdx.x; p < nparts; p += kPartThreads) hist[(int64_t)p * nblocks + blockIdx.x] = s_h[p];
}

__global__ void part_counts_kernel(const uint32_t* hist, int64_t nblocks, int nparts, const unsigned long long* total,
                                   int64_t* counts) {
    const int p = threadIdx.x;
    if (p < nparts) {
        const unsigned long long st = hist[(int64_t)p * nblocks];
        const unsigned long long en = (p + 1 < nparts) ? hist[(int64_t)(p + 1) * nblocks] : *total;
        counts[p] = (int64_t)(en - st);
    }
}

template <typename K, typename OK, typename ID>
__global__ void __launch_bounds__(kPartThreads)
part_scatter_kernel(const void* keys, const uint8_t* valid, int64_t voff, const uint64_t* ids, uint64_t id_base,
                    int64_t n, int nparts, PartSpec sp, const uint32_t* hist, int64_t nblocks, OK* out_keys,
                    int64_t key_offset, ID* out_ids) {
    __shared__ unsigned long long s_off[kMaxParts];
    __shared__ unsigned s_wc[kPartThreads / 64][kMaxParts];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int p = threadIdx.x; p < nparts; p += kPartThreads) s_off[p] = hist[(int64_t)p * nblocks + blockIdx.x];
    int bits = 0;
    while ((1 << bits) < nparts) ++bits;
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * kPartChunk;
    for (int k0 = 0; k0 < kPartChunk; k0 += kPartThreads) {
        const int64_t i = r0 + k0 + threadIdx.x;
        const int p = part_of<K>(keys, valid, voff, i, n, nparts - 1, sp);
        // lanes with the same partition: AND of per-bit ballots (multi-split)
        unsigned long long same = __ballot(p >= 0);
        for (int bt = 0; bt < bits; ++bt) {
            const unsigned long long m = __ballot(p >= 0 && ((p >> bt) & 1));
            same &= ((p >> bt) & 1) ? m : ~m;
        }
        const unsigned rank = __popcll(same & ((1ull << lane) - 1));
        for (int q = lane; q < nparts; q += 64) s_wc[wave][q] = 0;
        __syncthreads();
        if (p >= 0 && rank == 0) s_wc[wave][p] = __popcll(same);
        __syncthreads();
        if (p >= 0) {
            unsigned long long pos = s_off[p] + rank;
            for (int w = 0; w < wave; ++w) pos += s_wc[w][p];
            out_keys[pos] = (OK)(ld_key<K>(keys, i) - key_offset);  // OK narrower: caller checked the range
            out_ids[pos] = (ID)(ids ? ids[i] : id_base + (uint64_t)i);
        }
        __syncthreads();
        for (int q = threadIdx.x; q < nparts; q += kPartThreads) {
            unsigned t = 0;
            for (int w = 0; w < kPartThreads / 64; ++w) t += s_wc[w][q];
            s_off[q] += t;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// radix partition into per-destination regions, one pass (the multi-GPU exchange's send
// buffers). part_hist + scan + part_scatter read the keys twice and run five launches; here
// every 16384-row tile reads its rows once: a stable wave multi-split (per-bit ballots)
// ranks each row among its wave's rows of the same destination, a per-destination scan
// over the tile's (iteration, wave) counts places it inside the tile, and a decoupled
// look-back over the tiles' per-destination flags gives the tile's offset in each
// destination region. Region d of the outputs starts at element d * cap: the regions are
// the per-peer send buffers (no grouped copy), each in source row order (stable: received
// build ids ascend, and a rank's received probe rows stay in global row order).
// ---------------------------------------------------------------------------
// 512-thread tiles of 8192 rows, several workgroups per CU (so that one tile's look-back
// wait overlaps the others' loads). 10^8 rows into one region with the runtime filter
// (tools/part_bench.py, tools/lib_variants.py): 512 x 16 355 us, 256 x 16 380, 256 x 32 397,
// 1024 x 8 428; the first 1024 x 16 form (loads interleaved with the ballots) 472-520
#ifndef DFP_RP_THREADS
#define DFP_RP_THREADS 512
#endif
#ifndef DFP_RP_ITERS
#define DFP_RP_ITERS 16
#endif
constexpr int kRpThreads = DFP_RP_THREADS;
constexpr int kRpIters = DFP_RP_ITERS;
constexpr int kRpTile = kRpThreads * kRpIters;  // rows per tile
constexpr int kRpSlots = kRpIters * (kRpThreads / 64);  // (iteration, wave) counts per destination
static_assert(kRpSlots % 64 == 0, "the per-destination scan gives each lane whole slots");
constexpr unsigned kRpSpinLimit = 1u << 22;
constexpr unsigned long long kRpPoison = 1ull << 60;  // offset published by a tile whose look-back gave up
// diagnostic builds only (tools/lib_variants.py with DFP_HJ_ABLATIONS, DFP_RP_ABL; wrong output): 1 no look-back wait, 2 no
// stores, 4 no ids. The wait costs about half the kernel (355 -> 180 us for 10^8 rows
// with the filter); batching 2-16 look-back windows per flag round trip, longer spin
// sleeps and a persistent ticketed form that loads the next tile during the wait were all
// slower (tools/lib_variants.py).
#if defined(DFP_HJ_ABLATIONS) && defined(DFP_RP_ABL)
constexpr int kRpAbl = DFP_RP_ABL;
#else
constexpr int kRpAbl = 0;
#endif

template <typename K, typename OK, typename ID, bool HAS_VALID, bool HAS_IDS>
__global__ void __launch_bounds__(kRpThreads)
part_regions_kernel(const void* __restrict__ keys, const uint8_t* __restrict__ valid, int64_t voff,
                    const uint64_t* __restrict__ ids, uint64_t id_base, int64_t n, int nparts, int bits, PartSpec sp,
                    int64_t key_offset, OK* __restrict__ out_keys, ID* __restrict__ out_ids, int64_t cap,
                    unsigned long long* flags, int64_t* __restrict__ counts, unsigned long long* err) {
    extern __shared__ uint32_t s_cnt[];  // [nparts][kRpSlots]: rows per (iteration, wave), then their prefix
    __shared__ unsigned long long s_off[kMaxParts];  // the tile's offset in each region
    __shared__ uint32_t s_tot[kMaxParts];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t tile0 = (int64_t)blockIdx.x * kRpTile;
    for (int i = threadIdx.x; i < nparts * kRpSlots; i += kRpThreads) s_cnt[i] = 0;
    __syncthreads();
    int64_t key[kRpIters];
    uint32_t dr[kRpIters];  // destination << 8 | rank among the wave's rows of it; ~0 = dropped
    const unsigned long long lt = (1ull << lane) - 1;
    // every load of the tile issued before any use: the ballots below are convergence
    // points, and loads interleaved with them wait one round trip per iteration (16 per
    // tile: 520 us for 10^8 rows, against one round trip)
    bool vb[kRpIters];
#pragma unroll
    for (int it = 0; it < kRpIters; ++it) {
        const int64_t row = tile0 + (int64_t)it * kRpThreads + threadIdx.x;
        key[it] = row < n ? (int64_t)reinterpret_cast<const K*>(keys)[row] : 0;
        vb[it] = row < n && (!HAS_VALID || bit_valid(valid, voff, row));
    }
#pragma unroll
    for (int it = 0; it < kRpIters; ++it) {
        int p = -1;
        if (vb[it] && key[it] >= sp.lo && key[it] <= sp.hi)
            p = sp.by_range ? (int)__umul64hi((uint64_t)key[it] - (uint64_t)sp.lo, sp.mul)
                            : (int)(mix64((uint64_t)key[it]) & (uint64_t)(nparts - 1));
        unsigned long long same = __ballot(p >= 0);
        for (int bt = 0; bt < bits; ++bt) {
            const unsigned long long m = __ballot(p >= 0 && ((p >> bt) & 1));
            same &= ((p >> bt) & 1) ? m : ~m;
        }
        const uint32_t rank = (uint32_t)__popcll(same & lt);
        if (p >= 0 && rank == 0) s_cnt[p * kRpSlots + it * (kRpThreads / 64) + wave] = (uint32_t)__popcll(same);
        dr[it] = p >= 0 ? ((uint32_t)p << 8) | rank : 0xFFFFFFFFu;
    }
    __syncthreads();
    // per destination: exclusive prefix over the (iteration, wave) slots in row order
    for (int d = wave; d < nparts; d += kRpThreads / 64) {
        uint32_t* c = s_cnt + d * kRpSlots;
        constexpr int PER = kRpSlots / 64;
        uint32_t v[PER], sum = 0;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            v[q] = c[lane * PER + q];
            sum += v[q];
        }
        const uint32_t incl = wave_incl_scan_dpp(sum);
        uint32_t ex = incl - sum;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            c[lane * PER + q] = ex;
            ex += v[q];
        }
        if (lane == 63) s_tot[d] = incl;
    }
    __syncthreads();
    // look-back (wave 0): lane l looks at destination l % nparts of tile t - 1 - l / nparts
    // (a window of 64 / nparts tiles per round); per destination, the nearest inclusive
    // flag ends its walk. Flags: status (1 aggregate, 2 inclusive) << 62 | value.
    if ((kRpAbl & 1) && threadIdx.x < nparts) s_off[threadIdx.x] = 0;
    if (wave == 0 && !(kRpAbl & 1)) {
        const int d = lane & (nparts - 1), k = lane >> bits;  // nparts <= 64: every lane maps
        const int per = 64 >> bits;                           // tiles per window
        const int64_t t = blockIdx.x;
        const unsigned long long tot = s_tot[d];
        if (k == 0) flag_store(flags + t * nparts + d, (t == 0 ? kFlagIncl : kFlagAgg) | tot);
        unsigned long long excl = 0;
        // lanes of one destination: bits d, d + nparts, ... of a mask
        unsigned long long dmask = 0;
        for (int q = 0; q < per; ++q) dmask |= 1ull << (q * nparts + d);
        bool done = t == 0;
        int64_t j0 = t - 1;  // window: tiles j0 - k
        unsigned spins = 0;
        bool failed = false;
        while (__ballot(!done) != 0) {
            const int64_t j = j0 - k;
            unsigned long long f = kFlagIncl;  // before tile 0: an inclusive zero
            if (!done && j >= 0) f = flag_load(flags + j * nparts + d);
            const unsigned long long st = f >> 62;
            const unsigned long long incl_m = __ballot(st == 2) & dmask;
            const unsigned long long zero_m = __ballot(st == 0) & dmask;
            // this destination's lanes up to its nearest inclusive flag (all if none)
            const int first = incl_m ? __ffsll((long long)incl_m) - 1 : 63;
            const unsigned long long need = dmask & ((2ull << first) - 1);
            const bool wait = !done && (zero_m & need) != 0;
            if (__ballot(wait) != 0) {
                if (++spins > kRpSpinLimit) {  // never expected: report, do not hang
                    if (lane == 0) atomicOr(err, 1ull);
                    failed = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            unsigned long long v = (!done && ((need >> lane) & 1)) ? (f & kFlagVal) : 0ull;
            for (int o = nparts; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);  // sum over the destination's lanes
            if (!done) excl += v;
            if (incl_m) done = true;
            j0 -= per;
        }
        // a tile that gave up publishes a poisoned offset (>= 2^60 rows): its own rows are
        // not stored (pos >= cap), every later tile's offset and the region counts come out
        // above any region size, and hj_partition_regions' contract makes a count above
        // region_rows the caller's error signal (the error word says the same)
        if (failed) excl = kRpPoison;
        if (k == 0) {
            if (t > 0) flag_store(flags + t * nparts + d, kFlagIncl | (excl + tot));
            s_off[d] = excl;
            if (t == (int64_t)gridDim.x - 1) counts[d] = (int64_t)(excl + tot);
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kRpIters; ++it) {
        if (dr[it] == 0xFFFFFFFFu || (kRpAbl & 2)) continue;
        const int d = (int)(dr[it] >> 8);
        const int64_t row = tile0 + (int64_t)it * kRpThreads + threadIdx.x;
        const unsigned long long pos =
            s_off[d] + s_cnt[d * kRpSlots + it * (kRpThreads / 64) + wave] + (dr[it] & 0xFF);
        if (pos >= (unsigned long long)cap) continue;  // region overflow: counts say so
        const int64_t o = (int64_t)d * cap + (int64_t)pos;
        out_keys[o] = (OK)(key[it] - key_offset);  // OK narrower: the caller checked the range
        if (!(kRpAbl & 4)) out_ids[o] = (ID)(HAS_IDS ? ids[row] : id_base + (uint64_t)row);
    }
}

// ---------------------------------------------------------------------------
// generators
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void gen_perm_kernel(int64_t* out, int64_t n, int64_t mul, int64_t range) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (int64_t)(((uint64_t)i * (uint64_t)mul) % (uint64_t)range);  // caller keeps n*mul < 2^64
}

__global__ void gen_uniform_kernel(int64_t* out, int64_t n, uint64_t seed, int64_t range) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (int64_t)(splitmix64(seed + (uint64_t)i) % (uint64_t)range);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
int64_t build_tiles(int64_t total, int cus) {
    // one tile per CU (the staged scatters hold one 123 KB workgroup per CU; a second
    // partial round of tiles would double their time), at least kMinBuildTile rows each
    const int64_t by_rows = (total + kMinBuildTile - 1) / kMinBuildTile;
    return std::max<int64_t>(std::min<int64_t>(by_rows, std::max(cus, 1)), total > 0 ? 1 : 0);
}
int64_t build_tile_rows(int64_t total, int64_t ntiles) { return ntiles ? (total + ntiles - 1) / ntiles : 0; }

int64_t scan_scratch_bytes(int64_t len) { return 8 * ((len + kScanSeg - 1) / kScanSeg + 2); }

// in-place exclusive scan of a[0, len); bsum needs scan_scratch_bytes(len); the grand
// total goes to a[len] only through *total (if non-null)
template <typename T>
static hipError_t launch_scan(T* a, int64_t len, unsigned long long* bsum, unsigned long long* total,
                              hipStream_t s) {
    const int64_t nblk = (len + kScanSeg - 1) / kScanSeg;
    if (nblk == 0) return hipSuccess;
    scan_reduce_kernel<T><<<(unsigned)nblk, kScanThreads, 0, s>>>(a, len, bsum);
    scan_top_kernel<<<1, 1024, 0, s>>>(bsum, nblk, total);
    scan_down_kernel<T><<<(unsigned)nblk, kScanThreads, 0, s>>>(a, len, bsum);
    return hipGetLastError();
}

static hipError_t set_stage_lds() {
    static const bool lds_ok = [] {
        return hipFuncSetAttribute((const void*)coarse_scatter_staged_kernel<int64_t>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStageLds) == hipSuccess &&
               hipFuncSetAttribute((const void*)coarse_scatter_staged_kernel<int32_t>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStageLds) == hipSuccess &&
               hipFuncSetAttribute((const void*)fine_scatter_staged_kernel,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStageLds) == hipSuccess;
    }();
    return lds_ok ? hipSuccess : hipErrorInvalidConfiguration;
}

uint32_t dense_blocks(uint32_t nchunks) { return (nchunks + (1u << kDenseBlockShift) - 1) >> kDenseBlockShift; }
bool dense_one_level(uint32_t nchunks) { return dense_blocks(nchunks) <= (uint32_t)kMaxLevel1Bins; }

uint32_t coarse_shift(uint32_t nchunks) {
    // smallest shift with (nchunks >> shift) + 1 <= kCoarseBins groups (side chunk included)
    uint32_t sh = 0;
    while ((nchunks >> sh) + 1 > (uint32_t)kCoarseBins) ++sh;
    return sh;
}

hipError_t launch_scan_u64(unsigned long long* a, int64_t len, void* scratch, unsigned long long* total,
                           hipStream_t s) {
    if (len <= 0) return total ? hipMemsetAsync(total, 0, 8, s) : hipSuccess;
    return launch_scan<unsigned long long>(a, len, (unsigned long long*)scratch, total, s);
}

// One launch: every block reduces its share and folds it into two accumulator words with
// 64-bit atomic max (the min as the max of the complemented order-preserving unsigned
// form, so all-zero words are the identity), then takes a ticket; the block with the last
// ticket reads and clears the accumulators and the ticket and writes out[0], out[1] (and
// the host mailbox). acc[0..2] must be zero before the first launch and are left zero. A
// block's accumulator atomics return before its ticket is taken (their results are
// consumed first), so the last ticket sees every block's fold; no fences and no partials
// (a per-block __threadfence + partials took 137 us for 10^7 keys at 2442 blocks).
#ifndef DFP_MM_THREADS
#define DFP_MM_THREADS 1024
#endif
#ifndef DFP_MM_BLOCKS
#define DFP_MM_BLOCKS 256
#endif
constexpr int kMinmaxThreads = DFP_MM_THREADS;
constexpr unsigned kMinmaxBlocks = DFP_MM_BLOCKS;  // one per CU: 256 folds per accumulator word
__device__ __forceinline__ unsigned long long mm_ord(long long v) { return (unsigned long long)v ^ (1ull << 63); }
__device__ __forceinline__ long long mm_val(unsigned long long u) { return (long long)(u ^ (1ull << 63)); }
template <typename K>
__global__ void __launch_bounds__(kMinmaxThreads)
key_minmax_kernel(const Segment* __restrict__ segs, SegArgs sa, int nseg, int64_t total, long long* out,
                  BuildCounters* __restrict__ ctr, unsigned long long* acc, long long* mbox, long long seq,
                  long long* res) {
    __shared__ long long s_mn[kMinmaxThreads / 64], s_mx[kMinmaxThreads / 64];
    long long mn = LLONG_MAX, mx = LLONG_MIN;
    const bool by_arg = ctr != nullptr;  // segments in the argument; block 0 publishes them
    if (by_arg && blockIdx.x == 0) {
        if (threadIdx.x < (unsigned)nseg) const_cast<Segment*>(segs)[threadIdx.x] = sa.s[threadIdx.x];
        if (threadIdx.x == 0) *ctr = BuildCounters{};
    }
    for (int si = 0; si < nseg; ++si) {
        const Segment sg = by_arg ? sa.s[si] : segs[si];
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        if (sizeof(K) == 8 && sg.valid == nullptr && (reinterpret_cast<uintptr_t>(sg.keys) & 15) == 0) {
            // no nulls, 16-byte aligned int64 keys: 16-byte loads, sixteen in flight per lane
            const v2i64* kp = reinterpret_cast<const v2i64*>(sg.keys);
            const int64_t n2 = sg.n >> 1;
            for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j0 < n2; j0 += 16 * stride) {
                v2i64 v[16];
                bool in[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int64_t j = j0 + u * stride;
                    in[u] = j < n2;
                    v[u] = in[u] ? kp[j] : v2i64{0, 0};
                }
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    if (!in[u]) continue;
                    const long long a = v[u].x, b = v[u].y;
                    mn = min(mn, min(a, b));
                    mx = max(mx, max(a, b));
                }
            }
            if ((sg.n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
                const long long k = (long long)ld_key<K>(sg.keys, sg.n - 1);
                mn = min(mn, k);
                mx = max(mx, k);
            }
            continue;
        }
        for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < sg.n; i0 += 4 * stride) {
            long long k[4];
            bool ok[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {  // four independent loads in flight
                const int64_t i = i0 + u * stride;
                ok[u] = i < sg.n && bit_valid(sg.valid, sg.voff, i);
                k[u] = i < sg.n ? (long long)ld_key<K>(sg.keys, i) : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (!ok[u]) continue;
                mn = k[u] < mn ? k[u] : mn;
                mx = k[u] > mx ? k[u] : mx;
            }
        }
    }
    auto block_reduce = [&]() {
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const long long x = __shfl_xor(mn, d, 64), y = __shfl_xor(mx, d, 64);
            mn = x < mn ? x : mn;
            mx = y > mx ? y : mx;
        }
        if ((threadIdx.x & 63) == 0) {
            s_mn[threadIdx.x >> 6] = mn;
            s_mx[threadIdx.x >> 6] = mx;
        }
        __syncthreads();
        for (int w = 0; w < kMinmaxThreads / 64; ++w) {
            mn = s_mn[w] < mn ? s_mn[w] : mn;
            mx = s_mx[w] > mx ? s_mx[w] : mx;
        }
    };
    block_reduce();
    if (threadIdx.x != 0) return;
    const unsigned long long r0 = atomicMax(&acc[0], ~mm_ord(mn));
    const unsigned long long r1 = atomicMax(&acc[1], mm_ord(mx));
    asm volatile("" ::"v"(r0), "v"(r1));  // both folds have returned before the ticket
    if (atomicAdd(&acc[2], 1ull) != (unsigned long long)gridDim.x - 1) return;
    const long long rmn = mm_val(~atomicExch(&acc[0], 0ull));
    const long long rmx = mm_val(atomicExch(&acc[1], 0ull));
    atomicExch(&acc[2], 0ull);  // re-armed for the next launch
    out[0] = rmn;
    out[1] = rmx;
    if (res != nullptr) {
        res[0] = rmn;
        res[1] = rmx;
    }
    if (mbox != nullptr) {  // host mailbox (fine-grained): result, then the sequence number
        mbox[0] = rmn;
        mbox[1] = rmx;
        __hip_atomic_store(&mbox[2], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t launch_key_minmax_one(int key_bytes, const Segment* h_segs, Segment* d_segs, int nseg, BuildCounters* ctr,
                                 int64_t total, int64_t* out, unsigned long long* done, int64_t* mbox, int64_t seq,
                                 hipStream_t s, int64_t* res) {
    // blocks fold into the accumulators one at a time (~27 ns per atomic on one word:
    // 2048 blocks took 87 us for 10^7 keys, 128 blocks 27 us; tools/minmax_bench.py)
    const int64_t cap = total <= (int64_t)1 << 24 ? kMinmaxBlocks / 2 : kMinmaxBlocks;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((total + 4095) / 4096, cap));
    SegArgs sa{};
    if (ctr != nullptr) {
        if (nseg > kArgSegs) return hipErrorInvalidValue;
        for (int i = 0; i < nseg; ++i) sa.s[i] = h_segs[i];
    }
    if (key_bytes == 8)
        key_minmax_kernel<int64_t><<<grid, kMinmaxThreads, 0, s>>>(d_segs, sa, nseg, total, (long long*)out, ctr, done,
                                                                   (long long*)mbox, (long long)seq, (long long*)res);
    else
        key_minmax_kernel<int32_t><<<grid, kMinmaxThreads, 0, s>>>(d_segs, sa, nseg, total, (long long*)out, ctr, done,
                                                                   (long long*)mbox, (long long)seq, (long long*)res);
    return hipGetLastError();
}

template <typename K>
__global__ void __launch_bounds__(256)
key_minmax_part_kernel(const Segment* __restrict__ segs, SegArgs sa, int nseg, int64_t total, long long* out,
                  BuildCounters* __restrict__ ctr) {
    __shared__ long long s_mn[4], s_mx[4];
    long long mn = LLONG_MAX, mx = LLONG_MIN;
    const bool by_arg = ctr != nullptr;  // segments in the argument; block 0 publishes them
    if (by_arg && blockIdx.x == 0) {
        if (threadIdx.x < (unsigned)nseg) const_cast<Segment*>(segs)[threadIdx.x] = sa.s[threadIdx.x];
        if (threadIdx.x == 0) *ctr = BuildCounters{};
    }
    for (int si = 0; si < nseg; ++si) {
        const Segment sg = by_arg ? sa.s[si] : segs[si];
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        if (sizeof(K) == 8 && sg.valid == nullptr && (reinterpret_cast<uintptr_t>(sg.keys) & 15) == 0) {
            // no nulls, 16-byte aligned int64 keys: 16-byte loads, eight in flight per lane
            const v2i64* kp = reinterpret_cast<const v2i64*>(sg.keys);
            const int64_t n2 = sg.n >> 1;
            for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j0 < n2; j0 += 8 * stride) {
                v2i64 v[8];
                bool in[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int64_t j = j0 + u * stride;
                    in[u] = j < n2;
                    v[u] = in[u] ? kp[j] : v2i64{0, 0};
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    if (!in[u]) continue;
                    const long long a = v[u].x, b = v[u].y;
                    mn = min(mn, min(a, b));
                    mx = max(mx, max(a, b));
                }
            }
            if ((sg.n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
                const long long k = (long long)ld_key<K>(sg.keys, sg.n - 1);
                mn = min(mn, k);
                mx = max(mx, k);
            }
            continue;
        }
        for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < sg.n; i0 += 4 * stride) {
            long long k[4];
            bool ok[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {  // four independent loads in flight
                const int64_t i = i0 + u * stride;
                ok[u] = i < sg.n && bit_valid(sg.valid, sg.voff, i);
                k[u] = i < sg.n ? (long long)ld_key<K>(sg.keys, i) : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (!ok[u]) continue;
                mn = k[u] < mn ? k[u] : mn;
                mx = k[u] > mx ? k[u] : mx;
            }
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const long long a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    if ((threadIdx.x & 63) == 0) {
        s_mn[threadIdx.x >> 6] = mn;
        s_mx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) {
            mn = s_mn[w] < mn ? s_mn[w] : mn;
            mx = s_mx[w] > mx ? s_mx[w] : mx;
        }
        // per-block partials (out[2 + 2b], out[3 + 2b]), reduced by minmax_final_kernel: a
        // single word sustains ~88 atomics/us, so 1024 blocks' atomics would cost ~12 us
        out[2 + 2 * blockIdx.x] = mn;
        out[3 + 2 * blockIdx.x] = mx;
    }
}

__global__ void __launch_bounds__(1024) minmax_final_kernel(long long* out, unsigned nblk, long long* mbox,
                                                            long long seq) {
    __shared__ long long s_mn[16], s_mx[16];
    long long mn = LLONG_MAX, mx = LLONG_MIN;
    for (unsigned b = threadIdx.x; b < nblk; b += blockDim.x) {
        mn = min(mn, out[2 + 2 * b]);
        mx = max(mx, out[3 + 2 * b]);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        mn = min(mn, (long long)__shfl_xor(mn, d, 64));
        mx = max(mx, (long long)__shfl_xor(mx, d, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        s_mn[threadIdx.x >> 6] = mn;
        s_mx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            mn = min(mn, s_mn[w]);
            mx = max(mx, s_mx[w]);
        }
        out[0] = mn;
        out[1] = mx;
        if (mbox != nullptr) {  // host mailbox (fine-grained): result, then the sequence number
            mbox[0] = mn;
            mbox[1] = mx;
            __hip_atomic_store(&mbox[2], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// The build's key-range reduction: per-block partials, then minmax_final_kernel (result
// and host mailbox). Two launches, but 256-thread blocks that fit beside the previous
// step's probe kernels in the pipelined bench: the one-launch form (1024-thread blocks)
// waited for free CUs there and stretched the pipelined C2 build span 0.26 -> 0.60 ms.
hipError_t launch_key_minmax(int key_bytes, const Segment* h_segs, Segment* d_segs, int nseg, BuildCounters* ctr,
                             int64_t total, int64_t* out, int64_t* mbox, int64_t seq, hipStream_t s) {
    const unsigned grid =
        (unsigned)std::max<int64_t>(1, std::min<int64_t>((total + 4095) / 4096, kMinmaxMaxBlocks));
    SegArgs sa{};
    if (ctr != nullptr) {
        if (nseg > kArgSegs) return hipErrorInvalidValue;
        for (int i = 0; i < nseg; ++i) sa.s[i] = h_segs[i];
    }
    if (key_bytes == 8)
        key_minmax_part_kernel<int64_t><<<grid, 256, 0, s>>>(d_segs, sa, nseg, total, (long long*)out, ctr);
    else
        key_minmax_part_kernel<int32_t><<<grid, 256, 0, s>>>(d_segs, sa, nseg, total, (long long*)out, ctr);
    minmax_final_kernel<<<1, 1024, 0, s>>>((long long*)out, grid, (long long*)mbox, (long long)seq);
    return hipGetLastError();
}

int64_t frag_build_tiles(const int64_t* seg_n, int nseg, int tl) {
    const int64_t tile = (int64_t)1 << tl;
    int64_t t = 0;
    for (int i = 0; i < nseg; ++i) t += (seg_n[i] + tile - 1) / tile;
    return t;
}
// the hashed frag build's tiles: 2^15 rows (half the (tile, slice) fragments each slice's
// workgroup gathers), DFP_HJ_HB_TILE_LOG=14 for the probe's 2^14
int hashed_build_tile_log() {
    static const int v = [] {
        const char* e = getenv("DFP_HJ_HB_TILE_LOG");
        return e && atoi(e) == 14 ? 14 : 15;
    }();
    return v;
}
bool frag_build_ok(const ChunkGeom& g, int64_t ftiles) {
    return g.dense && dense_one_level(g.nchunks) && dense_blocks(g.nchunks) <= (uint32_t)kSlMaxSlices &&
           ftiles <= kFragMaxTiles;
}
int64_t frag_build_scratch_bytes(const ChunkGeom& g, int64_t ftiles, int64_t total) {
    const int64_t nbins = dense_blocks(g.nchunks) + 1;
    return 2 * ftiles * kSlTile + 2 * ftiles * kSlTile + 2 * ftiles * nbins + 2 * ((ftiles + 63) & ~(int64_t)63) * nbins +
           16 * total + 6 * 256;  // spill pool: the spilled rows twice (gathered, then by sub-range)
}

// dense frag build: consecutive key blocks per XCD run (DFP_HJ_FRAG_RUN; 1 = plain order)
uint32_t frag_run() {
    static const uint32_t v = [] {
        const char* e = getenv("DFP_HJ_FRAG_RUN");
        return e ? (uint32_t)std::max(1, atoi(e)) : 4u;
    }();
    return v;
}
// dense frag build workgroup size (DFP_HJ_FRAG_T): 512 threads x 16 rows (default) or
// 1024 x 8. Alone the 1024-thread form is faster (C2 70 vs 74 us, C3 234 vs 309 us); beside
// a probe on another stream the 8-wave workgroups (110 VGPRs, 74 KB LDS) fit on CUs that a
// probe kernel's workgroup half fills, where a 16-wave one does not: the pipelined bench's
// build span 0.36 -> 0.26 ms, C2 142.0K -> 146.2K Mrows/s, C3 66.2K -> 67.5K
// (profiles/r02_frag_threads.txt)
uint32_t frag_threads() {  // read per build, so that tests can run both forms in one process
    const char* e = getenv("DFP_HJ_FRAG_T");
    return e && atoi(e) == 1024 ? 1024u : 512u;
}
hipError_t launch_build_frag(int key_bytes, const Segment* h_segs, int nseg, const ChunkGeom& g, int64_t ftiles,
                             void* scratch, uint32_t* tile_base, const uint64_t* ids32, uint32_t* dense,
                             uint32_t* dup_rows, BigSeg* big, BuildCounters* ctr, const Segment* d_segs, int64_t total,
                             bool ids_as_rows, int big_grid, const SpecGeo& spec, hipStream_t s) {
    // spec.mm: the grid and the scratch cover g's `cap` blocks; the kernels take theirs from
    // the key range in device memory (SpecGeo)
    const uint32_t nblk = dense_blocks(g.nchunks), nbins = nblk + 1;
    constexpr uint32_t GV = kDenseSub << kDenseBlockShift;
    const uint32_t wlog = 31 - __builtin_clz(GV);
    auto a256 = [](uintptr_t x) { return (x + 255) & ~(uintptr_t)255; };
    uintptr_t p = a256((uintptr_t)scratch);
    uint16_t* ko = (uint16_t*)p;   p = a256(p + 2 * ftiles * kSlTile);
    uint16_t* rl = (uint16_t*)p;   p = a256(p + 2 * ftiles * kSlTile);
    uint16_t* toff = (uint16_t*)p; p = a256(p + 2 * ftiles * nbins);
    uint16_t* toffT = (uint16_t*)p; p = a256(p + 2 * ((ftiles + 63) & ~(int64_t)63) * nbins);
    // Measured (r04) and not kept: the partition writing the bounds in the 64-tile layout
    // itself (no transpose launch): its scattered 2-byte stores cost the partition what the
    // launch costs (C2 build partition 38 -> 48 us against an 8 us transpose); the key-range
    // partials folded by every partition block instead of minmax_final_kernel: the build
    // partition 38 -> 44 us against a 5.5 us launch, and the probe's partition (the same
    // kernel) 218 -> 224 us.
    unsigned long long* spill = (unsigned long long*)p;  // 2 x total rows at most
    int64_t t0 = 0;
    for (int i = 0; i < nseg; ++i) {
        const Segment& sg = h_segs[i];
        const int64_t nt = (sg.n + kSlTile - 1) / kSlTile;
        if (nt == 0) continue;
        const bool vec = (reinterpret_cast<uintptr_t>(sg.keys) & 15) == 0;
        const uint64_t drange = (uint64_t)nblk * GV;
#define DFP_BLP(KT, HV)                                                                                          \
    sl_partition_kernel<KT, HV><<<(unsigned)nt, kSlThreads, 0, s>>>(g.dmin, drange, wlog, nblk, sg.keys, sg.valid, \
                                                                   sg.voff, sg.n, vec, ko, rl, toff, 0, t0,          \
                                                                   sg.row_base, tile_base, nullptr, nullptr, nullptr, \
                                                                   nullptr, spec)
        if (key_bytes == 8) {
            if (sg.valid) DFP_BLP(int64_t, true); else DFP_BLP(int64_t, false);
        } else {
            if (sg.valid) DFP_BLP(int32_t, true); else DFP_BLP(int32_t, false);
        }
#undef DFP_BLP
        t0 += nt;
    }
    sl_toff_transpose_kernel<<<(unsigned)((ftiles + 63) / 64 * ((nblk + kSlTrChunk) / kSlTrChunk)), 256, 0, s>>>(
        toff, nbins, ftiles, toffT, spec);
    if (frag_threads() != 1024)
        dense_frag_build_kernel<512, 16><<<nblk, 512, 0, s>>>(g, nblk, ftiles, toffT, ko, rl, tile_base,
                                                             ids_as_rows ? ids32 : nullptr, dense, dup_rows, big, ctr,
                                                             spill, frag_run(), spec);
    else
        dense_frag_build_kernel<1024, 8><<<nblk, 1024, 0, s>>>(g, nblk, ftiles, toffT, ko, rl, tile_base,
                                                               ids_as_rows ? ids32 : nullptr, dense, dup_rows, big, ctr,
                                                               spill, frag_run(), spec);
    dup_sort_big_kernel<<<big_grid, kBigThreads, 0, s>>>(dup_rows, big, ctr, d_segs, nseg, total, key_bytes,
                                                         ids_as_rows);
    return hipGetLastError();
}

// hashed frag build: chunks of <= 2^kHbSliceLog buckets, <= kFragMaxTiles tiles
bool hashed_frag_ok(const ChunkGeom& g, int64_t ftiles) {
    return !g.dense && g.clog2 <= (uint32_t)kHbSliceLog && ftiles <= kFragMaxTiles && ftiles > 0;
}
uint32_t hashed_frag_slices(const ChunkGeom& g) { return (g.nb + (1u << kHbSliceLog) - 1) >> kHbSliceLog; }
int64_t hashed_frag_scratch_bytes(const ChunkGeom& g, int64_t ftiles, int64_t total) {
    const int64_t nbins = std::min<uint32_t>(hashed_frag_slices(g), (uint32_t)kSlMaxSlices) + 1;
    const int64_t kSlTile = (int64_t)1 << hashed_build_tile_log();  // ftiles: of this size
    return 8 * ftiles * kSlTile + 2 * ftiles * kSlTile + 2 * ftiles * nbins + 2 * ((ftiles + 63) & ~(int64_t)63) * nbins +
           32 * total + 6 * 256;  // spill pool: 16 B per row (rows) + up to 16 B per row (directories)
}
template <int TL>
hipError_t launch_build_hashed_frag_tl(int key_bytes, const Segment* h_segs, int nseg, const ChunkGeom& g, int64_t ftiles,
                                    void* scratch, uint32_t* tile_base, const uint64_t* ids32, Bucket* tbl,
                                    uint32_t* dup_rows, BigSeg* big, BuildCounters* ctr, const Segment* d_segs,
                                    int64_t total, bool ids_as_rows, int cus, hipStream_t s) {
    constexpr int T = 512, RR = 8;
    constexpr int64_t kSlTile = SlT<TL>::kRows;  // this build's tiles (ftiles of them)
    const uint32_t nsl_all = hashed_frag_slices(g);
    const int64_t nbins_max = std::min<uint32_t>(nsl_all, (uint32_t)kSlMaxSlices) + 1;
    auto a256 = [](uintptr_t x) { return (x + 255) & ~(uintptr_t)255; };
    uintptr_t p = a256((uintptr_t)scratch);
    unsigned long long* ko = (unsigned long long*)p; p = a256(p + 8 * ftiles * kSlTile);
    uint16_t* rl = (uint16_t*)p;   p = a256(p + 2 * ftiles * kSlTile);
    uint16_t* toff = (uint16_t*)p; p = a256(p + 2 * ftiles * nbins_max);
    uint16_t* toffT = (uint16_t*)p; p = a256(p + 2 * ((ftiles + 63) & ~(int64_t)63) * nbins_max);
    unsigned long long* spill = (unsigned long long*)p;  // rows past the registers + directories past the LDS
    // LDS: the slice image + side bucket, the tiles' fragment positions, then a duplicate
    // directory of what is left of 80 KB (two workgroups per CU); slices with more
    // duplicated keys keep their directory in the spill pool
    const size_t img = (size_t)((1u << kHbSliceLog) + 1) * sizeof(Bucket) + 8 * (size_t)ftiles + 4;
    const size_t budget = 80 * 1024 - 256;
    const uint32_t dupcap = img < budget ? (uint32_t)((budget - img) / 12) : 0u;
    const size_t lds = img + (size_t)dupcap * 12;
    const void* kfn = (const void*)hashed_frag_build_kernel<T, RR, TL>;
    hipError_t e = hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    // DFP_HJ_DEBUG_SYNC=1: synchronise after every launch and report the failing one (stderr)
    static const bool dbg_sync = getenv("DFP_HJ_DEBUG_SYNC") != nullptr;
    auto chk = [&](const char* what) -> hipError_t {
        if (!dbg_sync) return hipSuccess;
        const hipError_t q = hipStreamSynchronize(s);
        if (q != hipSuccess) fprintf(stderr, "dfp-hj: %s failed: %s\n", what, hipGetErrorString(q));
        return q;
    };
    for (uint32_t s0 = 0; s0 < nsl_all; s0 += (uint32_t)kSlMaxSlices) {
        const uint32_t nsl = std::min<uint32_t>(nsl_all - s0, (uint32_t)kSlMaxSlices), nbins = nsl + 1;
        int64_t t0 = 0;
        for (int i = 0; i < nseg; ++i) {
            const Segment& sg = h_segs[i];
            const int64_t nt = (sg.n + kSlTile - 1) / kSlTile;
            if (nt == 0) continue;
            const bool vec = (reinterpret_cast<uintptr_t>(sg.keys) & 15) == 0;
            const unsigned pgrid = (unsigned)std::min<int64_t>(nt, cus);
#define DFP_HBP(KT, HV)                                                                                             \
    if (TL == 15)                                                                                                   \
        hs_partition32_kernel<KT, HV><<<pgrid, kSlThreads, 0, s>>>(g.nb, kHbSliceLog, s0, nsl, sg.keys, sg.valid,     \
                                                                  sg.voff, sg.n, nt, vec, ko, rl, toff, nullptr,     \
                                                                  nullptr, nullptr, t0, sg.row_base, tile_base);     \
    else                                                                                                            \
        hs_partition_kernel<KT, HV><<<pgrid, kSlThreads, 0, s>>>(g.nb, kHbSliceLog, s0, nsl, sg.keys, sg.valid,       \
                                                                sg.voff, sg.n, nt, vec, ko, rl, toff, nullptr, nullptr, \
                                                                nullptr, t0, sg.row_base, tile_base)
            if (key_bytes == 8) {
                if (sg.valid) DFP_HBP(int64_t, true); else DFP_HBP(int64_t, false);
            } else {
                if (sg.valid) DFP_HBP(int32_t, true); else DFP_HBP(int32_t, false);
            }
#undef DFP_HBP
            if ((e = chk("hs_partition (build)")) != hipSuccess) return e;
            t0 += nt;
        }
        sl_toff_transpose_kernel<<<(unsigned)((ftiles + 63) / 64 * ((nbins + kSlTrChunk - 1) / kSlTrChunk)), 256, 0,
                                   s>>>(toff, nbins, ftiles, toffT, SpecGeo{});
        if ((e = chk("toff transpose")) != hipSuccess) return e;
        hashed_frag_build_kernel<T, RR, TL><<<nsl, T, lds, s>>>(g.nb, g.clog2, s0, nsl, ftiles, toffT, ko, rl, tile_base,
                                                           ids_as_rows ? ids32 : nullptr, tbl, dup_rows, big, ctr,
                                                           spill, dupcap, (uint64_t)(2 * total + 2),
                                                           (uint64_t)(4 * total));
        if ((e = chk("hashed_frag_build")) != hipSuccess) return e;
    }
    dup_sort_big_kernel<<<cus, kBigThreads, 0, s>>>(dup_rows, big, ctr, d_segs, nseg, total, key_bytes, ids_as_rows);
    return hipGetLastError();
}

hipError_t launch_build_hashed_frag(int key_bytes, const Segment* h_segs, int nseg, const ChunkGeom& g, int64_t ftiles,
                                    void* scratch, uint32_t* tile_base, const uint64_t* ids32, Bucket* tbl,
                                    uint32_t* dup_rows, BigSeg* big, BuildCounters* ctr, const Segment* d_segs,
                                    int64_t total, bool ids_as_rows, int cus, hipStream_t s) {
    return hashed_build_tile_log() == 15
               ? launch_build_hashed_frag_tl<15>(key_bytes, h_segs, nseg, g, ftiles, scratch, tile_base, ids32, tbl,
                                                 dup_rows, big, ctr, d_segs, total, ids_as_rows, cus, s)
               : launch_build_hashed_frag_tl<14>(key_bytes, h_segs, nseg, g, ftiles, scratch, tile_base, ids32, tbl,
                                                 dup_rows, big, ctr, d_segs, total, ids_as_rows, cus, s);
}

hipError_t launch_build(int key_bytes, const Segment* d_segs, int nseg, int64_t total, const ChunkGeom& g,
                        uint32_t* hist, uint32_t* hist1, uint32_t* chunk_starts, int64_t ntiles,
                        int64_t tile_rows, void* scan_scratch,
                        unsigned long long* tkeys, uint32_t* trows, unsigned long long* skeys, uint32_t* srows,
                        uint64_t* row_ids, bool ids_as_rows, Bucket* tbl, uint32_t* dense, uint32_t* dup_rows,
                        BigSeg* big, BuildCounters* ctr, int big_grid, hipStream_t s) {
    const uint32_t nb = g.nb, clog2 = g.clog2, nchunks = g.nchunks;
    const int64_t hlen = (int64_t)(nchunks + 1) * ntiles;
    if (g.dense && dense_one_level(nchunks)) {
        // one partition level: rows -> blocks of kDenseBlockChunks chunks (<= 2048 blocks,
        // LDS-staged scatter), each block built by one workgroup straight from tkeys/trows
        const uint32_t gshift = kDenseBlockShift;
        const uint32_t nblk = dense_blocks(nchunks);
        if (ntiles > 0) {
            unsigned long long* scr = (unsigned long long*)scan_scratch;
            if (key_bytes == 8)
                coarse_hist_kernel<int64_t, kStageMaxBins, 4><<<(unsigned)ntiles, kHistThreads, 0, s>>>(
                    d_segs, nseg, total, g, gshift, nblk, hist1, ntiles, tile_rows);
            else
                coarse_hist_kernel<int32_t, kStageMaxBins, 4><<<(unsigned)ntiles, kHistThreads, 0, s>>>(
                    d_segs, nseg, total, g, gshift, nblk, hist1, ntiles, tile_rows);
            hipError_t e = launch_scan(hist1, (int64_t)nblk * ntiles, scr, &ctr->n_valid, s);
            if (e != hipSuccess) return e;
            if ((e = set_stage_lds()) != hipSuccess) return e;
            // block starts from the scanned level-1 histogram, before the scatter consumes it
            chunk_starts_kernel<<<(unsigned)std::min<uint32_t>((nblk + 1 + 255) / 256, 4096), 256, 0, s>>>(
                hist1, ntiles, nblk - 1, ctr, chunk_starts);
            if (key_bytes == 8)
                coarse_scatter_staged_kernel<int64_t><<<(unsigned)ntiles, kHistThreads, kStageLds, s>>>(
                    d_segs, nseg, total, g, gshift, nblk, hist1, ntiles, tkeys, trows, row_ids, ids_as_rows,
                    tile_rows);
            else
                coarse_scatter_staged_kernel<int32_t><<<(unsigned)ntiles, kHistThreads, kStageLds, s>>>(
                    d_segs, nseg, total, g, gshift, nblk, hist1, ntiles, tkeys, trows, row_ids, ids_as_rows,
                    tile_rows);
            dense_chunk_build_kernel<kDenseSub << kDenseBlockShift, 1024, 8><<<nblk, 1024, 0, s>>>(
                g, chunk_starts, tkeys, trows, dense, dup_rows, big, ctr);
            dup_sort_big_kernel<<<big_grid, kBigThreads, 0, s>>>(dup_rows, big, ctr, d_segs, nseg, total, key_bytes,
                                                                 ids_as_rows);
        }
        return hipGetLastError();
    }
    const uint32_t gshift = coarse_shift(nchunks);
    const uint32_t ngroups = (nchunks >> gshift) + 1;
    if (ntiles > 0) {
        unsigned long long* scr = (unsigned long long*)scan_scratch;
        // level 1: group order
        if (key_bytes == 8)
            coarse_hist_kernel<int64_t, kCoarseBins, kHistThreads / 64><<<(unsigned)ntiles, kHistThreads, 0, s>>>(
                d_segs, nseg, total, g, gshift, ngroups, hist1, ntiles, tile_rows);
        else
            coarse_hist_kernel<int32_t, kCoarseBins, kHistThreads / 64><<<(unsigned)ntiles, kHistThreads, 0, s>>>(
                d_segs, nseg, total, g, gshift, ngroups, hist1, ntiles, tile_rows);
        hipError_t e = launch_scan(hist1, (int64_t)ngroups * ntiles, scr, &ctr->n_valid, s);
        if (e != hipSuccess) return e;
        if ((e = set_stage_lds()) != hipSuccess) return e;
        if (key_bytes == 8)
            coarse_scatter_staged_kernel<int64_t><<<(unsigned)ntiles, kHistThreads, kStageLds, s>>>(
                d_segs, nseg, total, g, gshift, ngroups, hist1, ntiles, tkeys, trows, row_ids,
                ids_as_rows, tile_rows);
        else
            coarse_scatter_staged_kernel<int32_t><<<(unsigned)ntiles, kHistThreads, kStageLds, s>>>(
                d_segs, nseg, total, g, gshift, ngroups, hist1, ntiles, tkeys, trows, row_ids,
                ids_as_rows, tile_rows);
        // level 2: chunk order (tiles over the n_valid group-ordered rows)
        if ((e = hipMemsetAsync(hist, 0, sizeof(uint32_t) * (size_t)hlen, s)) != hipSuccess) return e;
        fine_hist_kernel<<<(unsigned)ntiles, kHistThreads, sizeof(uint32_t) * kFineLdsBins, s>>>(tkeys, ctr, g, gshift,
                                                                                         hist, ntiles, tile_rows);
        if ((e = launch_scan(hist, hlen, scr, &ctr->n_valid, s)) != hipSuccess) return e;
        chunk_starts_kernel<<<(unsigned)std::min<uint32_t>((nchunks + 2 + 255) / 256, 4096), 256, 0, s>>>(
            hist, ntiles, nchunks, ctr, chunk_starts);
        fine_scatter_staged_kernel<<<(unsigned)ntiles, kHistThreads, kStageLds, s>>>(
            tkeys, trows, ctr, g, gshift, hist, ntiles, skeys, srows, tile_rows);
    }
    if (g.dense) {
        if (ntiles > 0) {
            dense_chunk_build_kernel<kDenseSub, 512, 4><<<nchunks, 512, 0, s>>>(g, chunk_starts, skeys, srows, dense,
                                                                                dup_rows, big, ctr);
            dup_sort_big_kernel<<<big_grid, kBigThreads, 0, s>>>(dup_rows, big, ctr, d_segs, nseg, total, key_bytes,
                                                                 ids_as_rows);
        }
        return hipGetLastError();
    }
    // chunk build: LDS = bucket image + dup directory (3 u32 per entry). 512-bucket
    // chunks run 512-thread workgroups, four per CU (32 KB image + directory in 38 KB);
    // 1024-bucket chunks two per CU; 2048-bucket chunks one. A chunk with more
    // duplicated keys than its directory holds makes the host rebuild at half load.
    const uint32_t CB = 1u << clog2;
    const size_t img = (size_t)CB * sizeof(Bucket);
    const size_t lds_cap = (CB <= 512 ? 40 * 1024 : CB <= 1024 ? 80 * 1024 : 160 * 1024) - 2048;
    uint32_t dupcap = (uint32_t)std::min<size_t>((size_t)CB * kSlots, (lds_cap - img) / 12);
    const size_t lds = img + (size_t)dupcap * 12;
    const void* kfn = CB <= 512 ? (const void*)chunk_build_kernel<512> : (const void*)chunk_build_kernel<1024>;
    hipError_t e = hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (ntiles > 0) {
        if (CB <= 512)
            chunk_build_kernel<512><<<nchunks + 1, 512, lds, s>>>(nb, clog2, nchunks, chunk_starts, skeys, srows,
                                                                 tbl, dup_rows, big, ctr, dupcap);
        else
            chunk_build_kernel<1024><<<nchunks + 1, 1024, lds, s>>>(nb, clog2, nchunks, chunk_starts, skeys, srows,
                                                                   tbl, dup_rows, big, ctr, dupcap);
        dup_sort_big_kernel<<<big_grid, kBigThreads, 0, s>>>(dup_rows, big, ctr, d_segs, nseg, total, key_bytes,
                                                             ids_as_rows);
    }
    return hipGetLastError();
}

int64_t probe_tiles(int64_t n) { return (n + kProbeTile - 1) / kProbeTile; }

// fused probe workspace (all regions 256-byte aligned): [0,16) header (bytes 8..15:
// error word) | tcnt u64[nt + 2] (the look-back's per-tile flags)
namespace {
struct ProbeWs {
    unsigned long long* tcnt;
    int64_t bytes;
};
inline uintptr_t al256(uintptr_t x) { return (x + 255) & ~(uintptr_t)255; }
ProbeWs probe_ws_layout(void* base, int64_t n) {
    const int64_t nt = probe_tiles(n > 0 ? n : 0);
    ProbeWs w;
    uintptr_t p = (uintptr_t)base + 256;
    w.tcnt = (unsigned long long*)p; p = al256(p + 8 * (nt + 2));
    w.bytes = (int64_t)(p - (uintptr_t)base) + 256;  // + slack for an unaligned base
    return w;
}

// sliced probe workspace (2^tl-row tiles), after the 16-byte header (error word at
// bytes 8..15): tcnt u64[nt + 2] (pair counts) | tent u32[nt + 2] (entries per tile over
// the passes) | toff u16[nt][kSlMaxSlices + 1] (one pass's bounds) |
// ko (entries: u16 key offsets in a dense slice, u64 stored keys in a hashed one; 8 B per
// row reserved) | rl u16[nt * kSlTile] (rows in tile) | res u32[nt * kSlTile] (refs)
struct SlicedWs {
    unsigned long long* tcnt;
    uint32_t* tent;
    uint16_t* toff;
    void* ko;
    uint16_t* rl;
    uint32_t* res;
    uint16_t* wcnt;   // entries per 2048-row range of a tile (kSlRanges per tile)
    int64_t bytes;
};
SlicedWs sliced_ws_layout(void* base, int64_t n, int tl) {
    const int64_t tile = (int64_t)1 << tl;  // this probe's tiles
    const int64_t nt = (n + tile - 1) / tile;
    SlicedWs w;
    uintptr_t p = (uintptr_t)base + 256;
    w.tcnt = (unsigned long long*)p;  p = al256(p + 8 * (nt + 2));
    w.tent = (uint32_t*)p;            p = al256(p + 4 * (nt + 2));
    w.toff = (uint16_t*)p;            p = al256(p + 2 * nt * (kSlMaxSlices + 1));  // one pass's bounds
    w.ko = (void*)p;                  p = al256(p + 8 * nt * tile);
    w.rl = (uint16_t*)p;              p = al256(p + 2 * nt * tile);
    w.res = (uint32_t*)p;             p = al256(p + 4 * nt * tile);
    w.wcnt = (uint16_t*)p;            p = al256(p + 2 * (tile / kSlRangeRows) * (nt + 2));
    w.bytes = (int64_t)(p - (uintptr_t)base) + 256;
    return w;
}

int env_probe_mode() {  // 0 auto, 3 fused, 4 sliced (1 and 2 were retired strategies)
    const char* e = getenv("DFP_HJ_PROBE_MODE");
    if (!e) return 0;
    if (e[0] == 'f') return 3;
    if (e[0] == 's') return 4;
    return 0;
}
std::atomic<int> g_probe_mode{-1};
int probe_mode() {
    int m = g_probe_mode.load(std::memory_order_relaxed);
    if (m < 0) {
        m = env_probe_mode();
        g_probe_mode.store(m, std::memory_order_relaxed);
    }
    return m;
}
}  // namespace

void set_probe_mode(int mode) {
    g_probe_mode.store(mode == 3 || mode == 4 ? mode : 0, std::memory_order_relaxed);
}
int get_probe_mode() { return probe_mode(); }

int64_t probe_workspace(int64_t n) {
    return std::max(probe_ws_layout(nullptr, n).bytes,
                    std::max(sliced_ws_layout(nullptr, n, 14).bytes, sliced_ws_layout(nullptr, n, 15).bytes));
}

namespace {
// slice width: 2^15 key values (128 KB of refs, one lookup workgroup per CU): half the
// (tile, slice) fragments of 2^14 (64 KB, two workgroups per CU); C2 lookups 221 vs
// 243 us (DFP_HJ_SLICE_LOG=14 for the narrower slices)
uint32_t sl_wlog() {
    static const uint32_t w = [] {
        const char* e = getenv("DFP_HJ_SLICE_LOG");
        const int v = e ? atoi(e) : 15;
        return (uint32_t)std::min(std::max(v, 10), kSlWidthLogMax);
    }();
    return w;
}
int sl_num_cus() {
    static const int c = [] {
        int d = 0, v = 0;
        if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) !=
                                                  hipSuccess || v < 1)
            v = 256;
        return v;
    }();
    return c;
}
// persistent emission grid: workgroups per CU (DFP_HJ_SL_EMIT_WGS; a large value gives
// one workgroup per tile)
int sl_env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? std::max(1, atoi(e)) : dflt;
}
int sl_emit_wgs_per_cu() {
    static const int v = sl_env_int("DFP_HJ_SL_EMIT_WGS", 2);
    return v;
}
uint32_t sl_slices(const TableView& tv) {
    if (tv.dense == nullptr) return (tv.nb + (1u << kHsSliceLog) - 1) >> kHsSliceLog;  // 128 KB bucket slices
    const uint32_t w = sl_wlog();
    return (uint32_t)std::min<uint64_t>((tv.drange + (1u << w) - 1) >> w, 1u << 30);
}
// auto choice: the sliced probe pays for its two extra passes once the table is past
// the L2s (direct-addressed: > 1 M key values = 4 MB of refs; hashed: > 2^16 buckets =
// 4 MB) and the probe side outweighs the slice loads (every slice is read once or a few
// times per probe)
// A table of more than kSlMaxSlices slices is probed in passes over consecutive slice
// ranges (each pass partitions the probe rows of its range, appending to the tiles'
// entries, and looks them up; one emission at the end). Every pass re-reads the probe
// keys: auto takes up to kSlAutoPasses passes, a forced sliced probe any number.
constexpr uint32_t kSlAutoPasses = 4;
constexpr int64_t kSlMinTilesPerPart = 1536;  // lookup items: tiles per (slice, part) at least
uint32_t sl_passes(uint32_t nsl) { return (nsl + kSlMaxSlices - 1) / kSlMaxSlices; }

bool sl_auto(const TableView& tv, int64_t n) {
    static const int64_t min_range = [] {
        const char* e = getenv("DFP_HJ_SLICED_MIN_RANGE");
        return e ? atoll(e) : (int64_t)1 << 20;
    }();
    if (n < 4 * (int64_t)kSlTile) return false;
    const uint32_t passes = sl_passes(sl_slices(tv));
    if (passes > kSlAutoPasses) return false;
    // hashed: one pass only. A second pass re-reads the probe keys and halves the
    // fragments (slice x tile) the lookups walk: a 4*10^7-key table probed by 10^8 rows
    // took 2.77 ms sliced (two passes) and 2.53 ms fused (tools/large_tables.py, r03)
    if (tv.dense == nullptr) return passes == 1 && (int64_t)tv.nb * 16 >= min_range && n >= (int64_t)tv.nb;
    // direct-addressed: the slice loads (4 bytes per key value) pay off well before the
    // probe side outnumbers the key range: 1.2*10^8 values probed by 10^8 rows took 1.00 ms
    // sliced and 1.21 ms fused
    return (int64_t)tv.drange >= min_range && 4 * n >= (int64_t)tv.drange;
}

template <int TL>
hipError_t launch_probe_sliced_tl(int key_bytes, const TableView& tv, const void* keys, const uint8_t* valid,
                               int64_t voff, const uint32_t* probe_ids, uint32_t pbase, int64_t n, uint64_t* out_b,
                               uint32_t* out_p, int64_t cap, int64_t* d_total, void* workspace, hipEvent_t built,
                               hipStream_t s) {
    const bool hashed = tv.dense == nullptr;
    constexpr int64_t kTile = SlT<TL>::kRows;
    const int64_t nt = (n + kTile - 1) / kTile;
    const uint32_t nsl_all = sl_slices(tv), wlog = sl_wlog();
    const uint32_t npass = sl_passes(nsl_all);
    SlicedWs w = sliced_ws_layout((void*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255), n, TL);
    const bool vec = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
    hipError_t e = hipSuccess;
    // workspace [0, 16): header with the caller's error word, zeroed by S1 (the layout
    // starts >= 256 bytes in)
    unsigned long long* hdr = reinterpret_cast<unsigned long long*>(workspace);
    static const int sl_nt = [] {  // 1: nontemporal probe-key loads in S1 (partial tiles' path)
        const char* ev = getenv("DFP_HJ_SL_NT");
        return ev ? atoi(ev) : 0;
    }();
#ifdef DFP_HJ_ABLATIONS
    // diagnostic build only (wrong pairs): emit 1 no stores, 2 no entries, 8 no duplicate
    // segment reads; lookup 4 no bucket lookup (hashed), 128 plain item order
    {  // re-read per call, so that a tool can switch ablations between probes
        static int abl_last = -1;
        const char* ev = getenv("DFP_HJ_ABLATE");
        const int v = ev ? atoi(ev) : 0;
        if (v != abl_last && hipMemcpyToSymbol(HIP_SYMBOL(kAblDev), &v, sizeof(v)) == hipSuccess) abl_last = v;
    }
#endif
    const size_t tab_lds = hashed ? (sizeof(Bucket) << kHsSliceLog) : (sizeof(uint32_t) << wlog);
    // dense lookup window: 2048 positions (32 per lane) or DFP_HJ_SL_DENSE_WIN=1024
    // (measured equal on C2 and C3, r04)
    static const bool dense_w1024 = sl_env_int("DFP_HJ_SL_DENSE_WIN", kSlOwnWin) == 1024;
    const void* lk = hashed        ? (const void*)sl_lookup_kernel<true, hs_own_win<TL>(), TL>
                     : dense_w1024 ? (const void*)sl_lookup_kernel<false, 1024, TL>
                                   : (const void*)sl_lookup_kernel<false, kSlOwnWin, TL>;
    e = hipFuncSetAttribute(lk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tab_lds);
    if (e != hipSuccess) return e;
    // (slice, tile range) work items: about 512 of them (768 before r05), so that the resident workgroups
    // (one per CU at 128 KB slices) run several rounds and the tail stays short; more items
    // load each slice image more often (profiles/r03_lookup_items.txt: C2 768 vs 1024 items
    // +0.5 % in three alternating pairs, C3 +0.7 %, C2h the same one part per slice)
    static const uint32_t target = [] {
        const char* ev = getenv("DFP_HJ_SLICED_ITEMS");
        // r05: 512 (C2 / C3: 2 parts per slice, the 50 slices past the whole rounds in fifths)
        // against 768 (3 parts) and 1224 (4): lookup C2 116.5 -> 115.1 us, C3 262 -> 258, C3
        // bench probe 1.153-1.159 -> 1.140-1.146 ms (profiles/r05_lookup_items2.txt)
        return ev ? (uint32_t)std::max(1, atoi(ev)) : 512u;
    }();
    for (uint32_t pass = 0; pass < npass; ++pass) {
        const uint32_t s0 = pass * (uint32_t)kSlMaxSlices;
        const uint32_t nsl = std::min<uint32_t>(nsl_all - s0, (uint32_t)kSlMaxSlices);
        unsigned long long* h = pass == 0 ? hdr : nullptr;  // a later pass appends to the tiles' entries
        if (hashed && TL == 15) {
            const unsigned pgrid = (unsigned)std::min<int64_t>(nt, sl_num_cus());
#define DFP_HSP(KT, HV)                                                                                             \
    hs_partition32_kernel<KT, HV><<<pgrid, kSlThreads, 0, s>>>(tv.nb, kHsSliceLog, s0, nsl, keys, valid, voff, n, nt, \
                                                              vec, (unsigned long long*)w.ko, w.rl, w.toff, h, w.tcnt,   \
                                                              w.tent, 0, 0, nullptr)
            if (key_bytes == 8) {
                if (valid) DFP_HSP(int64_t, true); else DFP_HSP(int64_t, false);
            } else {
                if (valid) DFP_HSP(int32_t, true); else DFP_HSP(int32_t, false);
            }
#undef DFP_HSP
        } else if (hashed) {
            const unsigned pgrid = (unsigned)std::min<int64_t>(nt, sl_num_cus());
#define DFP_HSP(KT, HV)                                                                                           \
    hs_partition_kernel<KT, HV><<<pgrid, kSlThreads, 0, s>>>(tv.nb, kHsSliceLog, s0, nsl, keys, valid, voff, n, nt, \
                                                            vec, (unsigned long long*)w.ko, w.rl, w.toff, h, w.tcnt,   \
                                                            w.tent, 0, 0, nullptr)
            if (key_bytes == 8) {
                if (valid) DFP_HSP(int64_t, true); else DFP_HSP(int64_t, false);
            } else {
                if (valid) DFP_HSP(int32_t, true); else DFP_HSP(int32_t, false);
            }
#undef DFP_HSP
        } else {
            // this pass's key range: slices [s0, s0 + nsl) of 2^wlog values from dmin
            const uint64_t lo = (uint64_t)s0 << wlog;
            const int64_t dmin_p = (int64_t)((uint64_t)tv.dmin + lo);
            const uint64_t drange_p = std::min<uint64_t>(tv.drange - lo, (uint64_t)nsl << wlog);
#define DFP_SLP(KT, HV)                                                                                      \
    sl_partition_kernel<KT, HV, TL><<<(unsigned)nt, kSlThreads, 0, s>>>(dmin_p, drange_p, wlog, nsl, keys, valid, voff, n, \
                                                                   vec, (uint16_t*)w.ko, w.rl, w.toff, sl_nt, 0, 0,   \
                                                                   nullptr, h, w.tcnt, w.tent, w.wcnt, SpecGeo{})
            if (key_bytes == 8) {
                if (valid) DFP_SLP(int64_t, true); else DFP_SLP(int64_t, false);
            } else {
                if (valid) DFP_SLP(int32_t, true); else DFP_SLP(int32_t, false);
            }
#undef DFP_SLP
        }
        uint32_t parts = std::max<uint32_t>(1, (target + nsl - 1) / nsl);
        parts = (uint32_t)std::min<int64_t>(parts, (nt + 63) / 64);
        // at least ~1536 tiles per part: a smaller probe (a rank's share on N GPUs) loads each
        // slice image fewer times (profiles/r05_lookup_items_small.txt: 1.25*10^7 rows over C2's
        // table, one part per slice 24.4 us against 37.1 us at C2's three; C2 keeps three)
        parts = std::max<uint32_t>(1, std::min<uint32_t>(parts, (uint32_t)(nt / ((kSlMinTilesPerPart << kSlTileLog) >> TL))));
        // the last round of small items: the slices beyond whole rounds of `parts` items
        // over the CUs split so that they fill about one round (DFP_HJ_SL_TAIL=0: even split)
        uint32_t s1 = nsl, parts2 = parts;
        {
            static const bool tail_on = [] {
                const char* ev = getenv("DFP_HJ_SL_TAIL");
                return !(ev != nullptr && ev[0] == '0');
            }();
            const uint32_t cus = (uint32_t)sl_num_cus();
            const uint32_t rounds = nsl * parts / cus;
            const uint32_t a = rounds * cus / parts;  // slices in the whole rounds
            if (tail_on && rounds >= 1 && a < nsl && a > 0) {
                // the split whose tail rounds take the least time (in items of `parts` parts):
                // ceil(r p / cus) rounds of 1/p items. C2: 50 slices over 256 CUs, p = 5 (one
                // round of fifths); C2h (one part per slice): 162 slices, p = 3 (two rounds of
                // thirds, 0.67 of an item instead of a whole round with 94 CUs idle)
                const uint32_t r = nsl - a;
                const uint32_t pmax = (uint32_t)std::min<int64_t>(8 * parts, (nt + 63) / 64);
                auto tail = [&](uint32_t p) { return (double)((r * p + cus - 1) / cus) / p; };
                uint32_t p2 = parts;
                for (uint32_t p = parts + 1; p <= pmax; ++p)
                    if (tail(p) < tail(p2) - 1e-9) p2 = p;
                if (p2 > parts && tail(p2) <= tail(parts) - 0.15 / parts) {  // by >= 0.15 of an item
                    s1 = a;
                    parts2 = p2;
                }
            }
        }
        const unsigned lgrid = s1 * parts + (nsl - s1) * parts2;
        // DFP_HJ_SL_EARLY=0: the image barrier right after the image load (A/B)
        static const int early = [] {
            const char* ev = getenv("DFP_HJ_SL_EARLY");
            return (ev != nullptr && ev[0] == '0') ? 0 : 1;
        }();
        if (pass == 0 && built != nullptr) {  // S1 reads no table memory: the build may still be running
            e = hipStreamWaitEvent(s, built, 0);
            if (e != hipSuccess) return e;
        }
        TableView tp = tv;  // this pass's table slices
        if (!hashed) {
            const uint64_t lo = (uint64_t)s0 << wlog;
            tp.dense = tv.dense + lo;
            tp.drange = std::min<uint64_t>(tv.drange - lo, (uint64_t)nsl << wlog);
        }
        if (hashed)
            sl_lookup_kernel<true, hs_own_win<TL>(), TL><<<lgrid, kSlThreads, tab_lds, s>>>(
                tp, wlog, nsl, nt, parts, s1, parts2, early, w.ko, w.res, w.toff, w.tcnt, s0);
        else if (dense_w1024)
            sl_lookup_kernel<false, 1024, TL><<<lgrid, kSlThreads, tab_lds, s>>>(tp, wlog, nsl, nt, parts, s1, parts2, early,
                                                                           w.ko, w.res, w.toff, w.tcnt, 0u);
        else
            sl_lookup_kernel<false, kSlOwnWin, TL><<<lgrid, kSlThreads, tab_lds, s>>>(tp, wlog, nsl, nt, parts, s1, parts2,
                                                                                early, w.ko, w.res, w.toff, w.tcnt, 0u);
    }
    const bool ri = tv.row_ids != nullptr, pi = probe_ids != nullptr;
    // DFP_HJ_COUNT_FREE=0: every tile takes the emission's general count and write passes
    // (A/B of the dense count-free path and of the hashed 0/1 path)
    // DFP_HJ_EMIT_DYN=0: the emission's static tile schedule (A/B of the tile counter)
    static const bool emit_dyn = [] {
        const char* e = getenv("DFP_HJ_EMIT_DYN");
        return !(e != nullptr && e[0] == '0');
    }();
    static const bool count_free = [] {
        const char* e = getenv("DFP_HJ_COUNT_FREE");
        return !(e != nullptr && e[0] == '0');
    }();
    // (2^15-row tiles: one 1024-thread workgroup per CU holds the 128 KB image; half the grid)
    const int ewgs = TL == kSlTileLog ? sl_emit_wgs_per_cu() : std::max(1, sl_emit_wgs_per_cu() >> (TL - kSlTileLog));
    const unsigned egrid = (unsigned)std::min<int64_t>(nt, (int64_t)ewgs * sl_num_cus());
#define DFP_SLE(RI, PI)                                                                                           \
    sl_emit_kernel<RI, PI, TL><<<egrid, SlT<TL>::kEmitThreads, 0, s>>>(tv, w.tent, w.rl, w.res, probe_ids, pbase, w.tcnt, nt,   \
                                                           out_b, out_p, cap, d_total,                      \
                                                           hashed || !count_free ? nullptr : w.wcnt,          \
                                                           emit_dyn ? w.tcnt + nt : nullptr, hashed && count_free)
    if (ri && pi) DFP_SLE(true, true);
    else if (ri) DFP_SLE(true, false);
    else if (pi) DFP_SLE(false, true);
    else DFP_SLE(false, false);
#undef DFP_SLE
    return hipGetLastError();
}
// probe tiles (hj_set_probe_tile_log / DFP_HJ_SL_TILE_LOG): 0 auto = 2^14 rows for a
// direct-addressed table, 2^15 for a hashed one (r05, profiles/r05_tile_log_ab.txt: C2h's
// lookup walks half the (tile, slice) fragments, 687 -> 588 us, bench 61.4-62.2K ->
// 65.7-65.8K Mrows/s; C2's partition in one 1024-thread workgroup per CU instead of two
// loses more than its lookup gains, 214 -> 250 us against 117 -> 102 us)
std::atomic<int> g_tile_log{-1};
int sl_tile_log_setting() {
    int v = g_tile_log.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* e = getenv("DFP_HJ_SL_TILE_LOG");
        const int x = e ? atoi(e) : 0;
        v = x == 14 || x == 15 ? x : 0;
        g_tile_log.store(v, std::memory_order_relaxed);
    }
    return v;
}
int sl_tile_log(bool hashed) {
    const int v = sl_tile_log_setting();
    return v ? v : hashed ? 15 : 14;
}
hipError_t launch_probe_sliced(int key_bytes, const TableView& tv, const void* keys, const uint8_t* valid,
                               int64_t voff, const uint32_t* probe_ids, uint32_t pbase, int64_t n, uint64_t* out_b,
                               uint32_t* out_p, int64_t cap, int64_t* d_total, void* workspace, hipEvent_t built,
                               hipStream_t s) {
    if (sl_tile_log(tv.dense == nullptr) == 15)
        return launch_probe_sliced_tl<15>(key_bytes, tv, keys, valid, voff, probe_ids, pbase, n, out_b, out_p, cap,
                                          d_total, workspace, built, s);
    return launch_probe_sliced_tl<14>(key_bytes, tv, keys, valid, voff, probe_ids, pbase, n, out_b, out_p, cap, d_total,
                                      workspace, built, s);
}
}  // namespace

int set_probe_tile_log(int tl) {
    const int old = sl_tile_log_setting();
    g_tile_log.store(tl, std::memory_order_relaxed);
    return old;
}

hipError_t launch_probe(int key_bytes, const TableView& tv, const void* keys, const uint8_t* valid, int64_t voff,
                        const uint32_t* probe_ids, uint32_t pbase, int64_t n, uint64_t* out_b, uint32_t* out_p, int64_t cap,
                        int64_t* d_total, void* workspace, hipEvent_t built, hipStream_t s) {
    const int64_t nt = probe_tiles(n);
    const int mode = probe_mode();
    const uint32_t nsl = sl_slices(tv);
    // a hashed key's probe sequence stays inside its chunk: chunks must not span slices
    const bool sl_ok = tv.dense != nullptr || tv.clog2 <= (uint32_t)kHsSliceLog;
    if (nt > 0 && nsl >= 1 && sl_ok && (mode == 4 || (mode == 0 && sl_auto(tv, n))))
        return launch_probe_sliced(key_bytes, tv, keys, valid, voff, probe_ids, pbase, n, out_b, out_p, cap, d_total,
                                   workspace, built, s);  // S1 zeroes the error word
    if (built != nullptr) {
        const hipError_t ew = hipStreamWaitEvent(s, built, 0);
        if (ew != hipSuccess) return ew;
    }
    hipError_t e0 = hipMemsetAsync((char*)workspace + 8, 0, 8, s);  // error word (fused look-back)
    if (e0 != hipSuccess) return e0;
    if (nt == 0) return hipMemsetAsync(d_total, 0, sizeof(int64_t), s);
    // align the layout on the workspace base
    ProbeWs w = probe_ws_layout((void*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255), n);
    const bool vec = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
    static const int fused_nt = [] {  // 1: keys nontemporal, 2: pair stores nontemporal
        const char* e = getenv("DFP_HJ_NT");
        return e ? atoi(e) : 0;
    }();
    // fused lookup + emission; tile flags live in the tile-count region
    hipError_t e = hipMemsetAsync(w.tcnt, 0, sizeof(unsigned long long) * nt, s);
    if (e != hipSuccess) return e;
    unsigned long long* err = reinterpret_cast<unsigned long long*>((char*)workspace + 8);
    const bool ri = tv.row_ids != nullptr, pi = probe_ids != nullptr;
#define DFP_FUSED(KT, HV, RI, PI)                                                                             \
    probe_fused_kernel<KT, HV, RI, PI><<<(unsigned)nt, kProbeThreads, 0, s>>>(tv, keys, valid, voff, probe_ids, pbase, n, \
                                                                             vec, w.tcnt, err, out_b, out_p, cap, \
                                                                             d_total, fused_nt)
#define DFP_FUSED_K(KT, HV)                              \
    do {                                                 \
        if (ri && pi) DFP_FUSED(KT, HV, true, true);     \
        else if (ri) DFP_FUSED(KT, HV, true, false);     \
        else if (pi) DFP_FUSED(KT, HV, false, true);     \
        else DFP_FUSED(KT, HV, false, false);            \
    } while (0)
    if (key_bytes == 8) {
        if (valid) DFP_FUSED_K(int64_t, true); else DFP_FUSED_K(int64_t, false);
    } else {
        if (valid) DFP_FUSED_K(int32_t, true); else DFP_FUSED_K(int32_t, false);
    }
#undef DFP_FUSED_K
#undef DFP_FUSED
    return hipGetLastError();
}

// A gathered direct-addressed table (the sharded-build broadcast plan): each piece's
// duplicated-key refs point into its own segment array; once the pieces' segment arrays
// sit one after another, the refs of one piece move by that piece's base. Streams the
// piece's refs once (a piece starts at any element: 4-byte accesses, coalesced).
__global__ void __launch_bounds__(256) dense_rebase_kernel(uint32_t* __restrict__ refs, uint64_t n, uint32_t base,
                                                           uint32_t mask) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = refs[i];
        // (a run ref holds its rows, not a segment offset: unchanged)
        if (r != kMiss && (r & kDupFlag) && !run_ref(r, mask)) refs[i] = (r & ~mask) | ((r & mask) + base);
    }
}

hipError_t launch_dense_rebase(uint32_t* refs, uint64_t n, uint32_t base, uint32_t mask, hipStream_t s) {
    if (n == 0 || base == 0) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
    dense_rebase_kernel<<<(unsigned)blocks, 256, 0, s>>>(refs, n, base, mask);
    return hipGetLastError();
}

hipError_t launch_table_stats(const TableView& tv, unsigned long long* out, hipStream_t s) {
    table_stats_kernel<<<1024, 256, 0, s>>>(tv, out);
    return hipGetLastError();
}

hipError_t launch_chain_links(const TableView& tv, int64_t* prev, int64_t nrows, hipStream_t s) {
    chain_fill_kernel<<<1024, 256, 0, s>>>(prev, nrows);
    chain_links_kernel<<<1024, 256, 0, s>>>(tv, prev);
    return hipGetLastError();
}

int64_t radix_partition_workspace(int64_t n, int nparts) {
    const int64_t nblocks = (n + kPartChunk - 1) / kPartChunk;
    const int64_t hlen = nblocks * nparts;
    return 4 * (hlen + 4) + scan_scratch_bytes(hlen) + 16;
}

hipError_t launch_radix_partition(int key_bytes, const void* keys, const uint8_t* valid, int64_t voff,
                                  const uint64_t* ids, uint64_t id_base, int64_t n, int nparts, const PartSpec& spec,
                                  void* out_keys, int out_key_bytes, int64_t key_offset, void* out_ids, int id_bytes,
                                  int64_t* counts, void* workspace, hipStream_t s) {
    if (nparts < 1 || nparts > kMaxParts || (nparts & (nparts - 1))) return hipErrorInvalidValue;
    const int64_t nblocks = (n + kPartChunk - 1) / kPartChunk;
    if (nblocks == 0) return hipMemsetAsync(counts, 0, sizeof(int64_t) * nparts, s);
    const int64_t hlen = nblocks * nparts;
    uint32_t* hist = reinterpret_cast<uint32_t*>(workspace);
    unsigned long long* scratch =
        reinterpret_cast<unsigned long long*>(((uintptr_t)(hist + hlen + 4) + 15) & ~(uintptr_t)15);
    const int64_t nsb = (hlen + kScanSeg - 1) / kScanSeg;
    unsigned long long* total = scratch + nsb;  // scan_top writes bsum[nblk] = grand total
    if (key_bytes == 8)
        part_hist_kernel<int64_t><<<(unsigned)nblocks, kPartThreads, 0, s>>>(keys, valid, voff, n, nparts, spec, hist,
                                                                            nblocks);
    else
        part_hist_kernel<int32_t><<<(unsigned)nblocks, kPartThreads, 0, s>>>(keys, valid, voff, n, nparts, spec, hist,
                                                                            nblocks);
    hipError_t e = launch_scan(hist, hlen, scratch, nullptr, s);
    if (e != hipSuccess) return e;
    part_counts_kernel<<<1, 64, 0, s>>>(hist, nblocks, nparts, total, counts);
#define DFP_PS(K, OK, ID)                                                                                 \
    part_scatter_kernel<K, OK, ID><<<(unsigned)nblocks, kPartThreads, 0, s>>>(                                  \
        keys, valid, voff, ids, id_base, n, nparts, spec, hist, nblocks, (OK*)out_keys, key_offset, (ID*)out_ids)
    if (key_bytes == 8 && out_key_bytes == 8) {
        if (id_bytes == 8) DFP_PS(int64_t, int64_t, uint64_t); else DFP_PS(int64_t, int64_t, uint32_t);
    } else if (key_bytes == 8) {
        if (id_bytes == 8) DFP_PS(int64_t, int32_t, uint64_t); else DFP_PS(int64_t, int32_t, uint32_t);
    } else {
        if (id_bytes == 8) DFP_PS(int32_t, int32_t, uint64_t); else DFP_PS(int32_t, int32_t, uint32_t);
    }
#undef DFP_PS
    return hipGetLastError();
}

int64_t radix_regions_workspace(int64_t n, int nparts) {
    const int64_t nt = (n + kRpTile - 1) / kRpTile;
    return 256 + 8 * std::max<int64_t>(nt, 1) * nparts;
}

hipError_t launch_radix_regions(int key_bytes, const void* keys, const uint8_t* valid, int64_t voff,
                                const uint64_t* ids, uint64_t id_base, int64_t n, int nparts, const PartSpec& spec,
                                void* out_keys, int out_key_bytes, int64_t key_offset, void* out_ids, int id_bytes,
                                int64_t cap, int64_t* counts, void* workspace, hipStream_t s) {
    if (nparts < 1 || nparts > kMaxParts || (nparts & (nparts - 1))) return hipErrorInvalidValue;
    const int64_t nt = (n + kRpTile - 1) / kRpTile;
    unsigned long long* err = reinterpret_cast<unsigned long long*>((char*)workspace + 8);
    unsigned long long* flags = reinterpret_cast<unsigned long long*>((char*)workspace + 256);
    hipError_t e = hipMemsetAsync(workspace, 0, (size_t)radix_regions_workspace(n, nparts), s);
    if (e != hipSuccess) return e;
    if (nt == 0) return hipMemsetAsync(counts, 0, sizeof(int64_t) * nparts, s);
    int bits = 0;
    while ((1 << bits) < nparts) ++bits;
    const size_t lds = sizeof(uint32_t) * (size_t)nparts * kRpSlots;
#define DFP_RP(K, OK, ID, HV, HI)                                                                                  \
    do {                                                                                                           \
        auto kfn = part_regions_kernel<K, OK, ID, HV, HI>;                                                         \
        if (lds > 64 * 1024) {                                                                                     \
            const hipError_t ea = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                                      (int)lds);                                                   \
            if (ea != hipSuccess) return ea;                                                                       \
        }                                                                                                          \
        kfn<<<(unsigned)nt, kRpThreads, lds, s>>>(keys, valid, voff, ids, id_base, n, nparts, bits, spec,           \
                                                  key_offset, (OK*)out_keys, (ID*)out_ids, cap, flags, counts, err); \
    } while (0)
#define DFP_RP_V(K, OK, ID)                                                      \
    do {                                                                         \
        if (valid) {                                                             \
            if (ids) DFP_RP(K, OK, ID, true, true); else DFP_RP(K, OK, ID, true, false);   \
        } else {                                                                 \
            if (ids) DFP_RP(K, OK, ID, false, true); else DFP_RP(K, OK, ID, false, false); \
        }                                                                        \
    } while (0)
    if (key_bytes == 8 && out_key_bytes == 8) {
        if (id_bytes == 8) DFP_RP_V(int64_t, int64_t, uint64_t); else DFP_RP_V(int64_t, int64_t, uint32_t);
    } else if (key_bytes == 8) {
        if (id_bytes == 8) DFP_RP_V(int64_t, int32_t, uint64_t); else DFP_RP_V(int64_t, int32_t, uint32_t);
    } else {
        if (id_bytes == 8) DFP_RP_V(int32_t, int32_t, uint64_t); else DFP_RP_V(int32_t, int32_t, uint32_t);
    }
#undef DFP_RP_V
#undef DFP_RP
    return hipGetLastError();
}

hipError_t launch_gen_perm(int64_t* out, int64_t n, int64_t mul, int64_t range, hipStream_t s) {
    gen_perm_kernel<<<2048, 256, 0, s>>>(out, n, mul, range);
    return hipGetLastError();
}

hipError_t launch_gen_uniform(int64_t* out, int64_t n, uint64_t seed, int64_t range, hipStream_t s) {
    gen_uniform_kernel<<<2048, 256, 0, s>>>(out, n, seed, range);
    return hipGetLastError();
}

}  // namespace dfp
