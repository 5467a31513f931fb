// hj_kernels.hip — hand-written gfx950 (CDNA4) kernels of the parallel hash join.
//
// Hot path:
//   insert_kernel   build: concurrent open-addressing insert with 64-bit atomicCAS on
//                   the key word and a 32-bit atomicAdd row count per slot. Replaces
//                   Inner::insert_atomically (src/operator/version10/new_map_3/
//                   fixed_table.rs:560-672) driven by JoinStateInstance::add
//                   (src/operator/version10/parallel_join_execution_state.rs:91-133).
//   dup_* kernels   build: turn the rows of duplicated keys into one contiguous segment
//                   per key, sorted descending (the reference's chain order newest ->
//                   oldest at parallelism 1, src/utils/concurrent_self_hash_join_map.rs:
//                   83-124,223-249), replacing the overflow chain array.
//   probe_kernel    probe: hash lookup + exact key compare + ordered pair emission in one
//                   pass (single-pass decoupled look-back over 4096-row tiles). Replaces
//                   get_matching_indices (src/shared/shared.rs:29-47), the chain walk
//                   (src/operator/version10/lookup_implementation_3.rs:22-59) and
//                   equal_rows_arr (src/shared/datafusion_private.rs:40-80).
//
// Design rules followed (cdna_hip_programming.md): wave64 ballots/shuffles, 16-byte
// vector loads for streamed keys, no same-address atomics in the hot loops (the
// single-word atomic rate is ~88/us, MI355X_MICROARCH.md "dequeue"), inter-workgroup
// hand-off only through 8-byte agent-scope {flag,value} granules (Guideline 16, R2),
// bounded spins.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "hj_device.h"
#include "hj_launch.h"

namespace dfp {

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool bit_valid(const uint8_t* v, int64_t off, int64_t i) {
    if (v == nullptr) return true;
    const int64_t b = off + i;
    return (v[b >> 3] >> (b & 7)) & 1;
}

template <typename K>
__device__ __forceinline__ int64_t ld_key(const void* keys, int64_t i) {
    return (int64_t)(reinterpret_cast<const K*>(keys)[i]);
}

__device__ __forceinline__ unsigned long long wave_incl_scan(unsigned long long v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        unsigned long long t = __shfl_up(v, (unsigned)d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// build: insert
// ---------------------------------------------------------------------------
constexpr int kInsThreads = 256;
constexpr int kDupBuf = 2048;  // LDS staging of dup entries per block (16 KB + 8 KB)

template <typename K>
__global__ void __launch_bounds__(kInsThreads)
insert_kernel(const Segment* __restrict__ segs, int nseg, int64_t total, Bucket* tbl,
              uint32_t nb, uint64_t* __restrict__ row_ids, uint2* __restrict__ duprows,
              uint32_t* __restrict__ dupslots, BuildCounters* ctr) {
    __shared__ uint2 s_rows[kDupBuf];
    __shared__ uint32_t s_slots[kDupBuf];
    __shared__ unsigned s_nrows, s_nslots;
    __shared__ unsigned long long s_base_r, s_base_s;
    if (threadIdx.x == 0) { s_nrows = 0; s_nslots = 0; }
    __syncthreads();

    auto flush = [&]() {
        // one global reservation per block and flush, never per row
        if (threadIdx.x == 0) {
            if (s_nrows) s_base_r = atomicAdd(&ctr->n_duprows, (unsigned long long)s_nrows);
            if (s_nslots) s_base_s = atomicAdd(&ctr->n_dupslots, (unsigned long long)s_nslots);
        }
        __syncthreads();
        for (unsigned k = threadIdx.x; k < s_nrows; k += kInsThreads) duprows[s_base_r + k] = s_rows[k];
        for (unsigned k = threadIdx.x; k < s_nslots; k += kInsThreads) dupslots[s_base_s + k] = s_slots[k];
        __syncthreads();
        if (threadIdx.x == 0) { s_nrows = 0; s_nslots = 0; }
        __syncthreads();
    };

    const int64_t stride = (int64_t)gridDim.x * kInsThreads;
    for (int64_t base = (int64_t)blockIdx.x * kInsThreads; base < total; base += stride) {
        const int64_t r = base + threadIdx.x;
        if (r < total) {
            int lo = 0, hi = nseg - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (segs[mid].row_base <= r) lo = mid; else hi = mid - 1;
            }
            const Segment sg = segs[lo];
            const int64_t i = r - sg.row_base;
            if (sg.ids != nullptr) row_ids[r] = sg.ids[i];
            if (bit_valid(sg.valid, sg.voff, i)) {
                const int64_t key = ld_key<K>(sg.keys, i);
                const unsigned long long skey = (unsigned long long)key ^ kSign;
                Bucket* B;
                int j = 0;
                bool ok = true;
                if (skey == 0) {
                    B = tbl + nb;  // side bucket for INT64_MIN
                } else {
                    uint32_t b = bucket_of(mix64((uint64_t)key), nb);
                    for (uint32_t probes = 0;; ++probes) {
                        B = tbl + b;
                        const ulonglong2* kp = reinterpret_cast<const ulonglong2*>(B->key);
                        const ulonglong2 k01 = kp[0], k23 = kp[1];
                        unsigned long long k[4] = {k01.x, k01.y, k23.x, k23.y};
                        bool done = false;
#pragma unroll
                        for (int jj = 0; jj < kSlots; ++jj) {
                            if (done) continue;
                            unsigned long long kk = k[jj];
                            if (kk == 0) kk = atomicCAS(&B->key[jj], 0ull, skey);  // claim
                            if (kk == 0 || kk == skey) { done = true; j = jj; }
                        }
                        if (done) break;
                        b = (b + 1 == nb) ? 0 : b + 1;  // linear probing over buckets
                        if (probes > nb) { ok = false; atomicOr(&ctr->err, 1ull); break; }
                    }
                }
                if (ok) {
                    const uint32_t slot = (uint32_t)((B - tbl) * kSlots + j);
                    const unsigned c = atomicAdd(&B->pay[j][0], 1u);
                    if (c == 0) {
                        B->pay[j][1] = (uint32_t)r;
                    } else {
                        const unsigned e = atomicAdd(&s_nrows, 1u);
                        s_rows[e] = make_uint2(slot, (uint32_t)r);
                        if (c == 1) s_slots[atomicAdd(&s_nslots, 1u)] = slot;
                    }
                }
            }
        }
        __syncthreads();
        if (s_nrows > kDupBuf - kInsThreads || s_nslots > kDupBuf - kInsThreads) flush();
    }
    __syncthreads();
    if (s_nrows || s_nslots) flush();
}

// ---------------------------------------------------------------------------
// build: duplicate-key segments
// ---------------------------------------------------------------------------
constexpr int kDupThreads = 256;
constexpr int kDupPerThread = 16;
constexpr int kDupChunk = kDupThreads * kDupPerThread;  // dupslots per block reservation

__device__ __forceinline__ Bucket* slot_bucket(Bucket* tbl, uint32_t slot, int& j) {
    j = (int)(slot & (kSlots - 1));
    return tbl + (slot / kSlots);
}

// pass A: per duplicated key, reserve its dup_rows segment (one atomic per 4096 keys),
// seed it with the first-arrived row, and park the dir index in the slot.
__global__ void __launch_bounds__(kDupThreads)
dup_alloc_kernel(Bucket* tbl, const uint32_t* __restrict__ dupslots, DupDir* dir,
                 uint32_t* dup_rows, BuildCounters* ctr) {
    __shared__ unsigned long long s_wave[kDupThreads / 64];
    __shared__ unsigned long long s_base;
    const unsigned long long nds = ctr->n_dupslots;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (unsigned long long c0 = (unsigned long long)blockIdx.x * kDupChunk; c0 < nds;
         c0 += (unsigned long long)gridDim.x * kDupChunk) {
        unsigned n[kDupPerThread];
        unsigned long long mine = 0;
#pragma unroll
        for (int q = 0; q < kDupPerThread; ++q) {
            const unsigned long long d = c0 + (unsigned long long)threadIdx.x * kDupPerThread + q;
            n[q] = 0;
            if (d < nds) {
                int j;
                Bucket* B = slot_bucket(tbl, dupslots[d], j);
                n[q] = B->pay[j][0];
            }
            mine += n[q];
        }
        const unsigned long long incl = wave_incl_scan(mine);
        if (lane == 63) s_wave[wave] = incl;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long tot = 0;
            for (int w = 0; w < kDupThreads / 64; ++w) tot += s_wave[w];
            s_base = tot ? atomicAdd(&ctr->dup_used, tot) : 0;
        }
        __syncthreads();
        unsigned long long off = s_base + incl - mine;
        for (int w = 0; w < wave; ++w) off += s_wave[w];
#pragma unroll
        for (int q = 0; q < kDupPerThread; ++q) {
            const unsigned long long d = c0 + (unsigned long long)threadIdx.x * kDupPerThread + q;
            if (d < nds) {
                const uint32_t slot = dupslots[d];
                int j;
                Bucket* B = slot_bucket(tbl, slot, j);
                const uint32_t first = B->pay[j][1];
                dir[d] = DupDir{(unsigned)off, n[q], 1u, slot};
                dup_rows[off] = first;
                B->pay[j][1] = (uint32_t)d;
                off += n[q];
            }
        }
        __syncthreads();
    }
}

// pass B: scatter the 2nd..nth rows of every duplicated key into its segment.
__global__ void __launch_bounds__(kDupThreads)
dup_scatter_kernel(const Bucket* tbl, const uint2* __restrict__ duprows, DupDir* dir,
                   uint32_t* dup_rows, const BuildCounters* ctr) {
    const unsigned long long ndr = ctr->n_duprows;
    for (unsigned long long e = (unsigned long long)blockIdx.x * kDupThreads + threadIdx.x; e < ndr;
         e += (unsigned long long)gridDim.x * kDupThreads) {
        const uint2 sr = duprows[e];
        const uint32_t d = tbl[sr.x / kSlots].pay[sr.x & (kSlots - 1)][1];
        const unsigned pos = atomicAdd(&dir[d].fill, 1u);
        dup_rows[dir[d].start + pos] = sr.y;
    }
}

// in-register bitonic sort of 16 u32, descending (compile-time indices: no scratch)
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

// pass C: sort small segments (<= 16 rows) in registers, queue larger ones.
__global__ void __launch_bounds__(kDupThreads)
dup_sort_small_kernel(Bucket* tbl, const DupDir* __restrict__ dir, uint32_t* dup_rows,
                      uint32_t* big, BuildCounters* ctr) {
    const unsigned long long nds = ctr->n_dupslots;
    for (unsigned long long d = (unsigned long long)blockIdx.x * kDupThreads + threadIdx.x; d < nds;
         d += (unsigned long long)gridDim.x * kDupThreads) {
        const DupDir e = dir[d];
        if (e.n <= (unsigned)kSmallSeg) {
            uint32_t v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = (i < (int)e.n) ? dup_rows[e.start + i] : 0u;
            sort16_desc(v);
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (i < (int)e.n) dup_rows[e.start + i] = v[i];
            int j;
            Bucket* B = slot_bucket(tbl, e.slot, j);
            B->pay[j][1] = e.start;
        } else {
            big[atomicAdd(&ctr->n_big, 1ull)] = (uint32_t)d;  // rare: keys with > 16 rows
        }
    }
}

constexpr int kBigThreads = 256;
constexpr int kBigLds = 4096;

// pass D: one workgroup per large segment. <= 4096 rows: bitonic sort in LDS.
// Larger: rebuild the segment by an ordered scan of the whole build input (stream
// compaction of rows equal to the key; deterministic, no scratch).
__global__ void __launch_bounds__(kBigThreads)
dup_sort_big_kernel(Bucket* tbl, uint32_t nb, const DupDir* __restrict__ dir,
                    uint32_t* dup_rows, const uint32_t* __restrict__ big,
                    const BuildCounters* ctr, const Segment* __restrict__ segs, int nseg,
                    int64_t total, int key_bytes) {
    __shared__ uint32_t s_v[kBigLds];
    __shared__ unsigned s_wave[kBigThreads / 64];
    const unsigned long long nbig = ctr->n_big;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (unsigned long long bi = blockIdx.x; bi < nbig; bi += gridDim.x) {
        const DupDir e = dir[big[bi]];
        if (e.n <= (unsigned)kBigLds) {
            unsigned N = 1;
            while (N < e.n) N <<= 1;
            for (unsigned i = threadIdx.x; i < N; i += kBigThreads)
                s_v[i] = (i < e.n) ? dup_rows[e.start + i] : 0u;
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
            for (unsigned i = threadIdx.x; i < e.n; i += kBigThreads) dup_rows[e.start + i] = s_v[i];
        } else {
            int j;
            Bucket* B = slot_bucket(tbl, e.slot, j);
            const bool side = (B == tbl + nb);
            const unsigned long long skey = side ? 0ull : B->key[j];
            const int64_t key = (int64_t)(skey ^ kSign);
            unsigned long long done = 0;  // rows placed so far (ascending row order)
            for (int64_t base = 0; base < total; base += kBigThreads) {
                const int64_t r = base + threadIdx.x;
                bool hit = false;
                if (r < total) {
                    int lo = 0, hi = nseg - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (segs[mid].row_base <= r) lo = mid; else hi = mid - 1;
                    }
                    const Segment sg = segs[lo];
                    const int64_t i = r - sg.row_base;
                    if (bit_valid(sg.valid, sg.voff, i)) {
                        const int64_t k = key_bytes == 8 ? ld_key<int64_t>(sg.keys, i)
                                                         : ld_key<int32_t>(sg.keys, i);
                        hit = (k == key);
                    }
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
                    dup_rows[e.start + (e.n - 1 - rank)] = (uint32_t)r;  // descending layout
                }
                done += tot;
                __syncthreads();
            }
        }
        if (threadIdx.x == 0) {
            int j;
            Bucket* B = slot_bucket(tbl, e.slot, j);
            B->pay[j][1] = e.start;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// probe
// ---------------------------------------------------------------------------
constexpr int kGroups = 4;                    // 4 groups x 1024 rows = 4096-row tile
constexpr int kTile = kProbeTile * kGroups;
constexpr unsigned long long kFlagA = 1ull << 62, kFlagP = 2ull << 62, kValMask = (1ull << 62) - 1;

template <typename K>
__device__ __forceinline__ void load4(const void* keys, int64_t row0, int64_t n, bool vec,
                                      int64_t (&k)[4]) {
    const K* kp = reinterpret_cast<const K*>(keys);
    if (vec && row0 + 4 <= n) {
        if constexpr (sizeof(K) == 8) {
            const longlong2* p = reinterpret_cast<const longlong2*>(kp + row0);
            const longlong2 a = p[0], b = p[1];
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

template <typename K>
__global__ void __launch_bounds__(kProbeThreads)
probe_kernel(const Bucket* __restrict__ tbl, uint32_t nb, const uint32_t* __restrict__ dup_rows,
             const uint64_t* __restrict__ row_ids, const void* __restrict__ keys,
             const uint8_t* __restrict__ valid, int64_t voff,
             const uint32_t* __restrict__ probe_ids, int64_t n, uint64_t* __restrict__ out_b,
             uint32_t* __restrict__ out_p, int64_t cap, int64_t* d_total,
             unsigned long long* status, unsigned int* ticket, int64_t ntiles, bool vec) {
    __shared__ unsigned s_tile;
    __shared__ unsigned long long s_wtot[kGroups][kProbeThreads / 64];
    __shared__ unsigned long long s_excl;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

    // dynamic tile id in dispatch order: every predecessor tile is already running,
    // so the look-back below cannot wait on a workgroup that is not resident.
    if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const int64_t tile = s_tile;
    const int64_t tile_row0 = tile * kTile;

    uint32_t cnt[kGroups][4];
    uint32_t rv[kGroups][4];
    unsigned long long gsum[kGroups];

#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
        const int64_t row0 = tile_row0 + (int64_t)g * kProbeTile + (int64_t)threadIdx.x * 4;
        int64_t k[4];
        load4<K>(keys, row0, n, vec, k);
        bool in[4];
        uint32_t b[4];
        unsigned long long sk[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            in[q] = (row0 + q < n) && bit_valid(valid, voff, row0 + q);
            sk[q] = (unsigned long long)k[q] ^ kSign;
            b[q] = bucket_of(mix64((uint64_t)k[q]), nb);
            cnt[g][q] = 0;
            rv[g][q] = 0;
        }
        // issue the first bucket load of all four rows before any compare (MLP)
        ulonglong2 k01[4], k23[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const ulonglong2* kp = reinterpret_cast<const ulonglong2*>(tbl[b[q]].key);
            if (in[q] && sk[q] != 0) { k01[q] = kp[0]; k23[q] = kp[1]; }
            else { k01[q] = make_ulonglong2(0, 0); k23[q] = make_ulonglong2(0, 0); }
        }
        unsigned long long tsum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (!in[q]) continue;
            if (sk[q] == 0) {  // INT64_MIN lives in the side bucket
                const uint2 p = *reinterpret_cast<const uint2*>(tbl[nb].pay[0]);
                cnt[g][q] = p.x; rv[g][q] = p.y;
            } else {
                uint32_t bb = b[q];
                unsigned long long kk[4] = {k01[q].x, k01[q].y, k23[q].x, k23[q].y};
                for (uint32_t probes = 0; probes <= nb; ++probes) {
                    int hitj = -1;
                    bool empty = false;
#pragma unroll
                    for (int jj = 0; jj < kSlots; ++jj) {
                        if (hitj < 0 && !empty) {
                            if (kk[jj] == sk[q]) hitj = jj;
                            else if (kk[jj] == 0) empty = true;
                        }
                    }
                    if (hitj >= 0) {
                        const uint2 p = *reinterpret_cast<const uint2*>(tbl[bb].pay[hitj]);
                        cnt[g][q] = p.x; rv[g][q] = p.y;
                        break;
                    }
                    if (empty) break;
                    bb = (bb + 1 == nb) ? 0 : bb + 1;  // bucket overflow (rare)
                    const ulonglong2* kp = reinterpret_cast<const ulonglong2*>(tbl[bb].key);
                    const ulonglong2 a = kp[0], c = kp[1];
                    kk[0] = a.x; kk[1] = a.y; kk[2] = c.x; kk[3] = c.y;
                }
            }
            tsum += cnt[g][q];
        }
        gsum[g] = tsum;
    }

    // block scan of the per-thread match counts, ordered (group, thread)
    unsigned long long gincl[kGroups];
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
        gincl[g] = wave_incl_scan(gsum[g]);
        if (lane == 63) s_wtot[g][wave] = gincl[g];
    }
    __syncthreads();
    unsigned long long agg = 0;
#pragma unroll
    for (int g = 0; g < kGroups; ++g)
        for (int w = 0; w < kProbeThreads / 64; ++w) agg += s_wtot[g][w];

    // decoupled look-back (one wave); status words are single 8-byte agent-scope
    // granules {flag:2, value:62}
    if (wave == 0) {
        unsigned long long excl = 0;
        if (tile == 0) {
            if (lane == 0) st_agent(&status[0], kFlagP | agg);
        } else {
            if (lane == 0) st_agent(&status[tile], kFlagA | agg);
            int64_t pred = tile - 1;
            unsigned spins = 0;
            while (true) {
                const int64_t idx = pred - lane;
                const unsigned long long v = idx >= 0 ? ld_agent(&status[idx]) : kFlagP;
                const unsigned long long f = v >> 62;
                const unsigned long long pm = __ballot(f == 2);
                const unsigned long long xm = __ballot(f == 0);
                const int firstP = pm ? (__ffsll((long long)pm) - 1) : 64;
                const unsigned long long need = firstP >= 63 ? ~0ull : ((2ull << firstP) - 1);
                if (xm & need) {
                    if (++spins > (1u << 26)) {  // bounded: never hang the GPU
                        if (lane == 0) st_agent(reinterpret_cast<unsigned long long*>(ticket) + 1, 1ull);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += wave_sum(lane <= firstP ? (v & kValMask) : 0ull);
                if (firstP < 64) break;
                pred -= 64;
            }
            if (lane == 0) st_agent(&status[tile], kFlagP | (excl + agg));
        }
        if (lane == 0) {
            s_excl = excl;
            if (tile == ntiles - 1) *d_total = (int64_t)(excl + agg);
        }
    }
    __syncthreads();

    // ordered emission: probe ascending, build descending within a probe row
    unsigned long long gbase = s_excl;
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
        unsigned long long pos = gbase + gincl[g] - gsum[g];
        for (int w = 0; w < wave; ++w) pos += s_wtot[g][w];
        for (int w = 0; w < kProbeThreads / 64; ++w) gbase += s_wtot[g][w];
        const int64_t row0 = (int64_t)g * kProbeTile + (int64_t)threadIdx.x * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t c = cnt[g][q];
            if (c == 0) continue;
            const int64_t prow = tile_row0 + row0 + q;
            const uint32_t pidx = probe_ids ? probe_ids[prow] : (uint32_t)prow;
            if (c == 1) {
                if (pos < (unsigned long long)cap) {
                    const uint32_t br = rv[g][q];
                    out_b[pos] = row_ids ? row_ids[br] : (uint64_t)br;
                    out_p[pos] = pidx;
                }
            } else {
                for (uint32_t t = 0; t < c; ++t) {
                    if (pos + t < (unsigned long long)cap) {
                        const uint32_t br = dup_rows[rv[g][q] + t];
                        out_b[pos + t] = row_ids ? row_ids[br] : (uint64_t)br;
                        out_p[pos + t] = pidx;
                    }
                }
            }
            pos += c;
        }
    }
}

// ---------------------------------------------------------------------------
// table queries (not on the hot path)
// ---------------------------------------------------------------------------
__global__ void table_stats_kernel(const Bucket* tbl, uint32_t nb, unsigned long long* out) {
    unsigned long long distinct = 0, dupk = 0, dupr = 0, mx = 0;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < (uint64_t)(nb + 1) * kSlots;
         s += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned c = tbl[s / kSlots].pay[s % kSlots][0];
        if (c) { distinct++; if (c > 1) { dupk++; dupr += c; } if (c > mx) mx = c; }
    }
    distinct = wave_sum(distinct); dupk = wave_sum(dupk); dupr = wave_sum(dupr);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) { unsigned long long o = __shfl_xor(mx, d, 64); mx = o > mx ? o : mx; }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&out[0], distinct); atomicAdd(&out[1], dupk); atomicAdd(&out[2], dupr);
        atomicMax(&out[3], mx);
    }
}

__global__ void chain_fill_kernel(int64_t* prev, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        prev[i] = -1;
}

__global__ void chain_links_kernel(const Bucket* tbl, uint32_t nb, const uint32_t* dup_rows,
                                   int64_t* prev) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < (uint64_t)(nb + 1) * kSlots;
         s += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned c = tbl[s / kSlots].pay[s % kSlots][0];
        if (c > 1) {
            const unsigned st = tbl[s / kSlots].pay[s % kSlots][1];
            for (unsigned t = 0; t + 1 < c; ++t) prev[dup_rows[st + t]] = dup_rows[st + t + 1];
        }
    }
}

// ---------------------------------------------------------------------------
// radix partition (multi-GPU exchange): stable multi-split by the low hash bits
// ---------------------------------------------------------------------------
constexpr int kPartThreads = 256;
constexpr int kPartChunk = 4096;  // rows per block
constexpr int kMaxParts = 64;

template <typename K>
__device__ __forceinline__ int part_of(const void* keys, const uint8_t* valid, int64_t voff,
                                       int64_t i, int64_t n, int mask) {
    if (i >= n || !bit_valid(valid, voff, i)) return -1;
    return (int)(mix64((uint64_t)ld_key<K>(keys, i)) & (uint64_t)mask);
}

template <typename K>
__global__ void __launch_bounds__(kPartThreads)
part_hist_kernel(const void* keys, const uint8_t* valid, int64_t voff, int64_t n, int nparts,
                 unsigned long long* hist, int64_t nblocks) {
    __shared__ unsigned s_h[kMaxParts];
    for (int p = threadIdx.x; p < nparts; p += kPartThreads) s_h[p] = 0;
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * kPartChunk;
    for (int k = threadIdx.x; k < kPartChunk; k += kPartThreads) {
        const int p = part_of<K>(keys, valid, voff, r0 + k, n, nparts - 1);
        if (p >= 0) atomicAdd(&s_h[p], 1u);
    }
    __syncthreads();
    for (int p = threadIdx.x; p < nparts; p += kPartThreads) hist[(int64_t)p * nblocks + blockIdx.x] = s_h[p];
}

// single-block exclusive scan over hist (partition-major), totals to counts[]
__global__ void __launch_bounds__(1024)
part_scan_kernel(unsigned long long* hist, int64_t len, int64_t nblocks, int nparts, int64_t* counts) {
    __shared__ unsigned long long s_w[16];
    __shared__ unsigned long long s_carry;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int64_t base = 0; base < len; base += 1024) {
        const int64_t i = base + threadIdx.x;
        const unsigned long long v = i < len ? hist[i] : 0;
        const unsigned long long incl = wave_incl_scan(v);
        if (lane == 63) s_w[wave] = incl;
        __syncthreads();
        unsigned long long off = s_carry;
        for (int w = 0; w < wave; ++w) off += s_w[w];
        if (i < len) hist[i] = off + incl - v;
        __syncthreads();
        if (threadIdx.x == 0) for (int w = 0; w < 16; ++w) s_carry += s_w[w];
        __syncthreads();
    }
    // counts[p] = start(p+1) - start(p)
    for (int p = threadIdx.x; p < nparts; p += 1024) {
        const unsigned long long st = hist[(int64_t)p * nblocks];
        const unsigned long long en = (p + 1 < nparts) ? hist[(int64_t)(p + 1) * nblocks] : s_carry;
        counts[p] = (int64_t)(en - st);
    }
}

template <typename K>
__global__ void __launch_bounds__(kPartThreads)
part_scatter_kernel(const void* keys, const uint8_t* valid, int64_t voff, const uint64_t* ids,
                    uint64_t id_base, int64_t n, int nparts, const unsigned long long* hist,
                    int64_t nblocks, K* out_keys, uint64_t* out_ids) {
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
        const int p = part_of<K>(keys, valid, voff, i, n, nparts - 1);
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
            out_keys[pos] = (K)ld_key<K>(keys, i);
            out_ids[pos] = ids ? ids[i] : id_base + (uint64_t)i;
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
hipError_t launch_insert(int key_bytes, const Segment* d_segs, int nseg, int64_t total,
                         Bucket* tbl, uint32_t nbuckets, uint64_t* row_ids, uint2* duprows,
                         uint32_t* dupslots, BuildCounters* ctr, int grid, hipStream_t s) {
    if (total <= 0) return hipSuccess;
    int64_t need = (total + kInsThreads - 1) / kInsThreads;
    const int g = (int)(need < grid ? need : grid);
    if (key_bytes == 8)
        insert_kernel<int64_t><<<g, kInsThreads, 0, s>>>(d_segs, nseg, total, tbl, nbuckets, row_ids,
                                                         duprows, dupslots, ctr);
    else
        insert_kernel<int32_t><<<g, kInsThreads, 0, s>>>(d_segs, nseg, total, tbl, nbuckets, row_ids,
                                                         duprows, dupslots, ctr);
    return hipGetLastError();
}

hipError_t launch_dup_passes(Bucket* tbl, uint32_t nbuckets, const uint2* duprows,
                             const uint32_t* dupslots, DupDir* dir, uint32_t* dup_rows,
                             uint32_t* big, BuildCounters* ctr, int grid, hipStream_t s) {
    // fixed grids that read their trip counts from device counters: no host sync
    dup_alloc_kernel<<<grid, kDupThreads, 0, s>>>(tbl, dupslots, dir, dup_rows, ctr);
    dup_scatter_kernel<<<grid, kDupThreads, 0, s>>>(tbl, duprows, dir, dup_rows, ctr);
    dup_sort_small_kernel<<<grid, kDupThreads, 0, s>>>(tbl, dir, dup_rows, big, ctr);
    return hipGetLastError();
}

hipError_t launch_dup_big(Bucket* tbl, uint32_t nbuckets, const DupDir* dir, uint32_t* dup_rows,
                          const uint32_t* big, const BuildCounters* ctr, const Segment* segs,
                          int nseg, int64_t total, int key_bytes, int grid, hipStream_t s) {
    dup_sort_big_kernel<<<grid, kBigThreads, 0, s>>>(tbl, nbuckets, dir, dup_rows, big, ctr, segs, nseg,
                                                     total, key_bytes);
    return hipGetLastError();
}

int64_t probe_tiles(int64_t n) { return (n + kTile - 1) / kTile; }

hipError_t launch_probe(int key_bytes, const Bucket* tbl, uint32_t nbuckets,
                        const uint32_t* dup_rows, const uint64_t* row_ids, const void* keys,
                        const uint8_t* valid, int64_t voff, const uint32_t* probe_ids, int64_t n,
                        uint64_t* out_b, uint32_t* out_p, int64_t cap, int64_t* d_total,
                        unsigned long long* status, unsigned int* ticket, hipStream_t s) {
    const int64_t nt = probe_tiles(n);
    if (nt == 0) return hipSuccess;
    const bool vec = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
    if (key_bytes == 8)
        probe_kernel<int64_t><<<(unsigned)nt, kProbeThreads, 0, s>>>(tbl, nbuckets, dup_rows, row_ids, keys,
                                                                    valid, voff, probe_ids, n, out_b, out_p,
                                                                    cap, d_total, status, ticket, nt, vec);
    else
        probe_kernel<int32_t><<<(unsigned)nt, kProbeThreads, 0, s>>>(tbl, nbuckets, dup_rows, row_ids, keys,
                                                                    valid, voff, probe_ids, n, out_b, out_p,
                                                                    cap, d_total, status, ticket, nt, vec);
    return hipGetLastError();
}

hipError_t launch_table_stats(const Bucket* tbl, uint32_t nbuckets, unsigned long long* out,
                              hipStream_t s) {
    table_stats_kernel<<<1024, 256, 0, s>>>(tbl, nbuckets, out);
    return hipGetLastError();
}

hipError_t launch_chain_links(const Bucket* tbl, uint32_t nbuckets, const uint32_t* dup_rows,
                              int64_t* prev, int64_t nrows, hipStream_t s) {
    chain_fill_kernel<<<1024, 256, 0, s>>>(prev, nrows);
    chain_links_kernel<<<1024, 256, 0, s>>>(tbl, nbuckets, dup_rows, prev);
    return hipGetLastError();
}

int64_t radix_partition_workspace(int64_t n, int nparts) {
    const int64_t nblocks = (n + kPartChunk - 1) / kPartChunk;
    return (nblocks * nparts + 1) * 8;
}

hipError_t launch_radix_partition(int key_bytes, const void* keys, const uint8_t* valid,
                                  int64_t voff, const uint64_t* ids, uint64_t id_base, int64_t n,
                                  int nparts, void* out_keys, uint64_t* out_ids, int64_t* counts,
                                  void* workspace, hipStream_t s) {
    if (nparts < 1 || nparts > kMaxParts || (nparts & (nparts - 1))) return hipErrorInvalidValue;
    const int64_t nblocks = (n + kPartChunk - 1) / kPartChunk;
    if (nblocks == 0) return hipMemsetAsync(counts, 0, sizeof(int64_t) * nparts, s);
    unsigned long long* hist = reinterpret_cast<unsigned long long*>(workspace);
    if (key_bytes == 8) {
        part_hist_kernel<int64_t><<<(unsigned)nblocks, kPartThreads, 0, s>>>(keys, valid, voff, n, nparts, hist, nblocks);
        part_scan_kernel<<<1, 1024, 0, s>>>(hist, nblocks * nparts, nblocks, nparts, counts);
        part_scatter_kernel<int64_t><<<(unsigned)nblocks, kPartThreads, 0, s>>>(
            keys, valid, voff, ids, id_base, n, nparts, hist, nblocks, (int64_t*)out_keys, out_ids);
    } else {
        part_hist_kernel<int32_t><<<(unsigned)nblocks, kPartThreads, 0, s>>>(keys, valid, voff, n, nparts, hist, nblocks);
        part_scan_kernel<<<1, 1024, 0, s>>>(hist, nblocks * nparts, nblocks, nparts, counts);
        part_scatter_kernel<int32_t><<<(unsigned)nblocks, kPartThreads, 0, s>>>(
            keys, valid, voff, ids, id_base, n, nparts, hist, nblocks, (int32_t*)out_keys, out_ids);
    }
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
