// hj_columns.hip — gfx950 kernels around the join's index pairs:
//
//   mark_rows_kernel       flags[idx[i]] = 1: the reference's ConcurrentBitSet::set_ones
//                          on matched build indices (src/utils/concurrent_bit_set.rs:28-60,
//                          e.g. src/operator/probe_lookup_implementation/full.rs:160-163)
//                          and the matched-probe bitmap of get_semi_indices /
//                          get_anti_indices (src/shared/datafusion_private.rs:85-135)
//   select_*_kernel        ascending indices i with flags[i] == want: get_set_indices /
//                          get_unset_indices, get_semi_indices / get_anti_indices
//   gather_fixed_kernel    Arrow `take` of a fixed-width column by (u32 | u64) indices with
//                          null propagation: take_multiple_record_batch
//                          (src/shared/shared.rs:83-92) for primitive columns
//   gather_var_*_kernel    the same for Utf8 / Binary (i32 offsets) and LargeUtf8 /
//                          LargeBinary (i64 offsets): lengths, scan, byte copy
//
// All HBM-bound streaming / gather work: no LDS tiling beyond block scans.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "hj_launch.h"
#include "hj_util.h"

namespace dfp {

// ---------------------------------------------------------------------------
// index -> flag marking
// ---------------------------------------------------------------------------
template <typename I>
__global__ void mark_rows_kernel(const I* __restrict__ idx, int64_t n, uint8_t* __restrict__ flags, int64_t nflags) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t v = (uint64_t)idx[i];
        if (v < (uint64_t)nflags) flags[v] = 1;  // idempotent byte stores: no atomics needed
    }
}

hipError_t launch_mark_rows(const void* idx, int idx_bytes, int64_t n, uint8_t* flags, int64_t nflags,
                            hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
    if (idx_bytes == 8)
        mark_rows_kernel<uint64_t><<<grid, 256, 0, s>>>((const uint64_t*)idx, n, flags, nflags);
    else
        mark_rows_kernel<uint32_t><<<grid, 256, 0, s>>>((const uint32_t*)idx, n, flags, nflags);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// stream compaction of flag positions (ascending)
// ---------------------------------------------------------------------------
constexpr int kSelThreads = 256;
constexpr int kSelPer = 16;  // flags per thread (one 16-byte load)
constexpr int kSelTile = kSelThreads * kSelPer;

__device__ __forceinline__ void load_flags16(const uint8_t* flags, int64_t n, int64_t i0, uint8_t (&f)[kSelPer]) {
    if (i0 + kSelPer <= n && ((reinterpret_cast<uintptr_t>(flags + i0) & 15) == 0)) {
        const uint4 v = *reinterpret_cast<const uint4*>(flags + i0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < kSelPer; ++k) f[k] = (uint8_t)(w[k >> 2] >> ((k & 3) * 8));
    } else {
#pragma unroll
        for (int k = 0; k < kSelPer; ++k) f[k] = (i0 + k < n) ? flags[i0 + k] : 0xFF;
    }
}

__global__ void __launch_bounds__(kSelThreads)
select_count_kernel(const uint8_t* __restrict__ flags, int64_t n, uint8_t want, unsigned long long* __restrict__ tcnt) {
    __shared__ unsigned long long s_w[kSelThreads / 64];
    const int64_t i0 = (int64_t)blockIdx.x * kSelTile + (int64_t)threadIdx.x * kSelPer;
    uint8_t f[kSelPer];
    load_flags16(flags, n, i0, f);
    unsigned long long c = 0;
#pragma unroll
    for (int k = 0; k < kSelPer; ++k) c += (i0 + k < n) && (f[k] == want);
    unsigned long long tot;
    block_excl_scan<unsigned long long>(c, s_w, &tot);
    if (threadIdx.x == 0) tcnt[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(kSelThreads)
select_write_kernel(const uint8_t* __restrict__ flags, int64_t n, uint8_t want,
                    const unsigned long long* __restrict__ toff, uint64_t* __restrict__ out) {
    __shared__ unsigned long long s_w[kSelThreads / 64];
    const int64_t i0 = (int64_t)blockIdx.x * kSelTile + (int64_t)threadIdx.x * kSelPer;
    uint8_t f[kSelPer];
    load_flags16(flags, n, i0, f);
    unsigned long long c = 0;
#pragma unroll
    for (int k = 0; k < kSelPer; ++k) c += (i0 + k < n) && (f[k] == want);
    unsigned long long tot;
    unsigned long long pos = toff[blockIdx.x] + block_excl_scan<unsigned long long>(c, s_w, &tot);
#pragma unroll
    for (int k = 0; k < kSelPer; ++k)
        if ((i0 + k < n) && (f[k] == want)) out[pos++] = (uint64_t)(i0 + k);
}

int64_t select_workspace(int64_t n) {
    const int64_t nt = (n + kSelTile - 1) / kSelTile;
    return 8 * (nt + 2) + scan_scratch_bytes(nt) + 256;
}

hipError_t launch_select_rows(const uint8_t* flags, int64_t n, uint8_t want, uint64_t* out, int64_t* d_count,
                              void* workspace, hipStream_t s) {
    const int64_t nt = (n + kSelTile - 1) / kSelTile;
    if (nt == 0) return hipMemsetAsync(d_count, 0, 8, s);
    unsigned long long* tcnt = (unsigned long long*)(((uintptr_t)workspace + 7) & ~(uintptr_t)7);
    void* scratch = tcnt + (nt + 2);
    select_count_kernel<<<(unsigned)nt, kSelThreads, 0, s>>>(flags, n, want, tcnt);
    hipError_t e = launch_scan_u64(tcnt, nt, scratch, (unsigned long long*)d_count, s);
    if (e != hipSuccess) return e;
    select_write_kernel<<<(unsigned)nt, kSelThreads, 0, s>>>(flags, n, want, tcnt, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// gather (Arrow take). Index all-ones (UINT32_MAX / UINT64_MAX) = null index (the
// outer joins' null build / probe side). Output validity: one wave writes the 64 bits
// of its 64 consecutive rows with one 8-byte store (dst_valid 8-byte aligned, bit 0 =
// row 0).
// ---------------------------------------------------------------------------
template <typename I>
__device__ __forceinline__ bool load_index(const I* idx, int64_t i, uint64_t* v) {
    const I x = idx[i];
    *v = (uint64_t)x;
    return x != (I)~(I)0;
}

// dst_valid holds ceil(n / 64) * 8 bytes, 8-byte aligned
__device__ __forceinline__ void write_valid_bits(uint8_t* dst_valid, int64_t wave_row0, int64_t n, bool valid) {
    const unsigned long long m = __ballot(valid);
    if ((threadIdx.x & 63) == 0 && dst_valid != nullptr && wave_row0 < n)
        *reinterpret_cast<unsigned long long*>(dst_valid + (wave_row0 >> 3)) = m;
}

template <typename I, int EB>
__global__ void __launch_bounds__(256)
gather_fixed_kernel(const uint8_t* __restrict__ src, const uint8_t* __restrict__ src_valid, int64_t src_voff,
                    const I* __restrict__ idx, int64_t n, uint8_t* __restrict__ dst, uint8_t* __restrict__ dst_valid) {
    using W = typename std::conditional<EB == 1, uint8_t,
              typename std::conditional<EB == 2, uint16_t,
              typename std::conditional<EB == 4, uint32_t,
              typename std::conditional<EB == 8, uint64_t, uint4>::type>::type>::type>::type;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        bool valid = false;
        if (i < n) {
            uint64_t v;
            const bool has = load_index<I>(idx, i, &v);
            W x{};
            if (has) {
                x = reinterpret_cast<const W*>(src)[v];
                valid = bit_valid(src_valid, src_voff, (int64_t)v);
            }
            reinterpret_cast<W*>(dst)[i] = x;  // null slots hold zeros (Arrow: unspecified)
        }
        write_valid_bits(dst_valid, base + (threadIdx.x & ~63), n, valid);
    }
}

hipError_t launch_gather_fixed(const void* src, const uint8_t* src_valid, int64_t src_voff, int elem_bytes,
                               const void* idx, int idx_bytes, int64_t n, void* dst, uint8_t* dst_valid,
                               hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 16384);
#define DFP_G(I, EB)                                                                                    \
    gather_fixed_kernel<I, EB><<<grid, 256, 0, s>>>((const uint8_t*)src, src_valid, src_voff, (const I*)idx, n, \
                                                    (uint8_t*)dst, dst_valid)
#define DFP_GI(I)                          \
    switch (elem_bytes) {                  \
        case 1: DFP_G(I, 1); break;        \
        case 2: DFP_G(I, 2); break;        \
        case 4: DFP_G(I, 4); break;        \
        case 8: DFP_G(I, 8); break;        \
        case 16: DFP_G(I, 16); break;      \
        default: return hipErrorInvalidValue; \
    }
    if (idx_bytes == 8) {
        DFP_GI(uint64_t)
    } else {
        DFP_GI(uint32_t)
    }
#undef DFP_GI
#undef DFP_G
    return hipGetLastError();
}

// variable-width: pass 1 lengths (u64, in the workspace), scan, pass 2 offsets + bytes
template <typename I, typename O>
__global__ void __launch_bounds__(256)
gather_var_len_kernel(const O* __restrict__ offsets, const uint8_t* __restrict__ src_valid, int64_t src_voff,
                      const I* __restrict__ idx, int64_t n, unsigned long long* __restrict__ lens,
                      uint8_t* __restrict__ dst_valid) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        bool valid = false;
        if (i < n) {
            uint64_t v;
            unsigned long long len = 0;
            if (load_index<I>(idx, i, &v) && bit_valid(src_valid, src_voff, (int64_t)v)) {
                valid = true;
                len = (unsigned long long)(offsets[v + 1] - offsets[v]);
            }
            lens[i] = len;
        }
        write_valid_bits(dst_valid, base + (threadIdx.x & ~63), n, valid);
    }
}

// one wave per 64 rows: each row's bytes are copied by the whole wave (coalesced for
// long strings; short strings cost one pass each)
template <typename I, typename O>
__global__ void __launch_bounds__(256)
gather_var_copy_kernel(const O* __restrict__ offsets, const uint8_t* __restrict__ values,
                       const uint8_t* __restrict__ src_valid, int64_t src_voff, const I* __restrict__ idx, int64_t n,
                       const unsigned long long* __restrict__ starts, O* __restrict__ out_offsets,
                       uint8_t* __restrict__ out_values, int64_t values_cap) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t w0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; w0 < n; w0 += waves * 64) {
        const int64_t i = w0 + lane;
        uint64_t src0 = 0;
        unsigned long long len = 0, dst0 = 0;
        if (i < n) {
            uint64_t v;
            dst0 = starts[i];
            out_offsets[i] = (O)dst0;
            if (load_index<I>(idx, i, &v) && bit_valid(src_valid, src_voff, (int64_t)v)) {
                src0 = (uint64_t)offsets[v];
                len = (unsigned long long)(offsets[v + 1] - offsets[v]);
            }
        }
        const int rows = (int)min<int64_t>(64, n - w0);
        for (int r = 0; r < rows; ++r) {
            const unsigned long long L = __shfl(len, r, 64);
            if (L == 0) continue;
            const uint64_t s0 = __shfl(src0, r, 64);
            const unsigned long long d0 = __shfl(dst0, r, 64);
            if (d0 + L > (unsigned long long)values_cap) continue;  // host re-sizes and retries
            for (unsigned long long b = lane; b < L; b += 64) out_values[d0 + b] = values[s0 + b];
        }
    }
}

__global__ void write_last_offset_kernel(const unsigned long long* total, void* out_offsets, int64_t n, int ob) {
    if (ob == 8) reinterpret_cast<int64_t*>(out_offsets)[n] = (int64_t)*total;
    else reinterpret_cast<int32_t*>(out_offsets)[n] = (int32_t)*total;
}

int64_t gather_var_workspace(int64_t n) { return 8 * (n + 2) + scan_scratch_bytes(n) + 256; }

hipError_t launch_gather_var(const void* offsets, int offset_bytes, const uint8_t* values, const uint8_t* src_valid,
                             int64_t src_voff, const void* idx, int idx_bytes, int64_t n, void* out_offsets,
                             uint8_t* out_values, int64_t values_cap, uint8_t* dst_valid, int64_t* d_values_len,
                             void* workspace, hipStream_t s) {
    if (n <= 0) {
        hipError_t e = hipMemsetAsync(d_values_len, 0, 8, s);
        if (e != hipSuccess) return e;
        return hipMemsetAsync(out_offsets, 0, offset_bytes, s);
    }
    unsigned long long* lens = (unsigned long long*)(((uintptr_t)workspace + 7) & ~(uintptr_t)7);
    void* scratch = lens + (n + 2);
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 16384);
    const unsigned cgrid = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
#define DFP_V(I, O)                                                                                                   \
    do {                                                                                                              \
        gather_var_len_kernel<I, O><<<grid, 256, 0, s>>>((const O*)offsets, src_valid, src_voff, (const I*)idx, n,     \
                                                         lens, dst_valid);                                            \
        hipError_t e = launch_scan_u64(lens, n, scratch, (unsigned long long*)d_values_len, s);                       \
        if (e != hipSuccess) return e;                                                                                \
        gather_var_copy_kernel<I, O><<<cgrid, 256, 0, s>>>((const O*)offsets, values, src_valid, src_voff,             \
                                                           (const I*)idx, n, lens, (O*)out_offsets, out_values,       \
                                                           values_cap);                                               \
    } while (0)
    if (idx_bytes == 8) {
        if (offset_bytes == 8) DFP_V(uint64_t, int64_t); else DFP_V(uint64_t, int32_t);
    } else {
        if (offset_bytes == 8) DFP_V(uint32_t, int64_t); else DFP_V(uint32_t, int32_t);
    }
#undef DFP_V
    write_last_offset_kernel<<<1, 1, 0, s>>>((const unsigned long long*)d_values_len, out_offsets, n, offset_bytes);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// multi-GPU table helpers (hj_build_begin_multi, hj_api.cpp)
// ---------------------------------------------------------------------------
// out[i] = base + i (u32 probe ids of a contiguous row range)
__global__ void iota_u32_kernel(uint32_t* __restrict__ out, int64_t n, uint32_t base) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = base + (uint32_t)i;
}
// a[i] += base (merged probe rows -> the caller's probe row base)
__global__ void add_u32_kernel(uint32_t* __restrict__ a, int64_t n, uint32_t base) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        a[i] += base;
}
// out[i] = in[i] (u32 -> u64 ids for the partition kernel)
__global__ void widen_u32_kernel(const uint32_t* __restrict__ in, int64_t n, uint64_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}
// Canonical merge of the shards' pair streams: every probe row's pairs come from one shard
// (its key's owner), contiguous and in build-descending order, and each stream ascends in
// probe row. cnt[r] = pairs of row r, first[r] = index of its first pair; after an
// exclusive scan of cnt, pair i goes to start[r] + (i - first[r]).
__global__ void pairs_rank_kernel(const uint32_t* __restrict__ p, int64_t m, unsigned long long* __restrict__ cnt,
                                  unsigned long long* __restrict__ first) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t r = p[i];
        atomicAdd(&cnt[r], 1ull);
        atomicMin(&first[r], (unsigned long long)i);
    }
}
__global__ void pairs_place_kernel(const uint64_t* __restrict__ b, const uint32_t* __restrict__ p, int64_t m,
                                   const unsigned long long* __restrict__ start,
                                   const unsigned long long* __restrict__ first, uint64_t* __restrict__ out_b,
                                   uint32_t* __restrict__ out_p, int64_t cap) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t r = p[i];
        const unsigned long long pos = start[r] + ((unsigned long long)i - first[r]);
        if (pos < (unsigned long long)cap) {
            out_b[pos] = b[i];
            out_p[pos] = r;
        }
    }
}

static unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192)); }

hipError_t launch_iota_u32(uint32_t* out, int64_t n, uint32_t base, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    iota_u32_kernel<<<grid_for(n), 256, 0, s>>>(out, n, base);
    return hipGetLastError();
}

hipError_t launch_add_u32(uint32_t* a, int64_t n, uint32_t base, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    add_u32_kernel<<<grid_for(n), 256, 0, s>>>(a, n, base);
    return hipGetLastError();
}

hipError_t launch_widen_u32(const uint32_t* in, int64_t n, uint64_t* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    widen_u32_kernel<<<grid_for(n), 256, 0, s>>>(in, n, out);
    return hipGetLastError();
}

int64_t merge_pairs_workspace(int64_t nrows) { return 16 * (nrows + 2) + scan_scratch_bytes(nrows + 1) + 512; }

hipError_t launch_merge_pairs(const uint64_t* b, const uint32_t* p, int64_t m, int64_t nrows, uint64_t* out_b,
                              uint32_t* out_p, int64_t cap, void* ws, hipStream_t s) {
    if (m <= 0 || nrows <= 0) return hipSuccess;
    uintptr_t q = ((uintptr_t)ws + 255) & ~(uintptr_t)255;
    unsigned long long* cnt = (unsigned long long*)q;
    q = (q + 8 * (nrows + 1) + 255) & ~(uintptr_t)255;
    unsigned long long* first = (unsigned long long*)q;
    q = (q + 8 * (nrows + 1) + 255) & ~(uintptr_t)255;
    void* scr = (void*)q;
    hipError_t e = hipMemsetAsync(cnt, 0, 8 * (size_t)nrows, s);
    if (e == hipSuccess) e = hipMemsetAsync(first, 0xFF, 8 * (size_t)nrows, s);
    if (e != hipSuccess) return e;
    pairs_rank_kernel<<<grid_for(m), 256, 0, s>>>(p, m, cnt, first);
    if ((e = launch_scan_u64(cnt, nrows, scr, nullptr, s)) != hipSuccess) return e;
    pairs_place_kernel<<<grid_for(m), 256, 0, s>>>(b, p, m, cnt, first, out_b, out_p, cap);
    return hipGetLastError();
}

}  // namespace dfp
