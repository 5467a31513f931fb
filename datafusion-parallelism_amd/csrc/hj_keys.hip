// hj_keys.hip — gfx950 kernels for join keys of several columns or of non-integer types
// (SURVEY.md §8a rows a2 and a12 in full generality):
//
//   composite_keys_kernel   one 64-bit key per row from all key columns: the reference's
//                           calculate_hash over every key column (src/shared/shared.rs:
//                           11-16, create_hashes); a null in any key column makes the row
//                           null (it never matches). The table is then built and probed on
//                           these keys with the single-key kernels, so a probe yields the
//                           rows whose composite keys are equal — the reference's
//                           candidates of equal hash.
//   equal_pairs_kernel      equal_rows_arr (src/shared/datafusion_private.rs:40-80): a
//                           candidate pair survives when its key tuples are equal in every
//                           column (byte-exact; arrow's eq on floats is total-order, i.e.
//                           equal bits), then the survivors are compacted in order
//                           (select + gather), so the pairs stay canonical.
//
// Columns: fixed width 1/2/4/8/16 bytes, or variable width (Utf8 / Binary with i32 or i64
// offsets). HBM-bound streaming work; byte loads for unaligned or variable-width values.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "hj_device.h"
#include "hj_launch.h"
#include "hj_util.h"

namespace dfp {

// 8 bytes of a value starting at p (len <= 8 of them, little-endian, zero padded)
__device__ __forceinline__ uint64_t load_le(const uint8_t* p, uint32_t len) {
    uint64_t v = 0;
    for (uint32_t i = 0; i < len; ++i) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

__device__ __forceinline__ uint64_t fixed_word(const KeyCol& c, int64_t row, int half) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(c.values) + row * c.width + half * 8;
    const uint32_t w = c.width < 8 ? (uint32_t)c.width : 8u;
    if ((reinterpret_cast<uintptr_t>(p) & (w - 1)) == 0) {
        switch (w) {
            case 1: return *p;
            case 2: return *reinterpret_cast<const uint16_t*>(p);
            case 4: return *reinterpret_cast<const uint32_t*>(p);
            default: return *reinterpret_cast<const uint64_t*>(p);
        }
    }
    return load_le(p, w);
}

__device__ __forceinline__ void var_range(const KeyCol& c, int64_t row, int64_t* a, int64_t* b) {
    if (c.offset_bytes == 8) {
        const int64_t* o = reinterpret_cast<const int64_t*>(c.offsets);
        *a = o[row];
        *b = o[row + 1];
    } else {
        const int32_t* o = reinterpret_cast<const int32_t*>(c.offsets);
        *a = o[row];
        *b = o[row + 1];
    }
}

// hash of one column value (equal values, equal hashes: a function of the bytes only)
__device__ __forceinline__ uint64_t value_hash(const KeyCol& c, int64_t row) {
    if (c.width > 0) {
        uint64_t h = mix64(fixed_word(c, row, 0) ^ ((uint64_t)c.width * 0x9E3779B97F4A7C15ull));
        if (c.width == 16) h = mix64(h ^ fixed_word(c, row, 1));
        return h;
    }
    int64_t a, b;
    var_range(c, row, &a, &b);
    const uint8_t* p = reinterpret_cast<const uint8_t*>(c.values) + a;
    const uint64_t len = (uint64_t)(b - a);
    uint64_t h = mix64(len ^ 0xC2B2AE3D27D4EB4Full);
    for (uint64_t i = 0; i < len; i += 8) h = mix64(h ^ load_le(p + i, (uint32_t)min<uint64_t>(8, len - i)));
    return h;
}

__global__ void __launch_bounds__(256)
composite_keys_kernel(KeyCols cols, int64_t n, int64_t* __restrict__ out_keys, uint64_t* __restrict__ out_valid) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // whole waves step together: lane l of the wave holding rows [r0, r0 + 64) writes
    // bit l of the validity word r0 / 64 (one ballot per word, no atomics)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i - (threadIdx.x & 63) < n; i += stride) {
        bool valid = i < n;
        uint64_t h = 0x243F6A8885A308D3ull;
        if (valid) {
            for (int j = 0; j < cols.n; ++j) {
                const KeyCol& c = cols.c[j];
                if (!bit_valid(c.valid, c.voff, i)) valid = false;
                h = mix64(h ^ value_hash(c, i)) + (uint64_t)(j + 1) * 0x9E3779B97F4A7C15ull;
            }
            out_keys[i] = (int64_t)h;
        }
        const unsigned long long word = __ballot(valid);
        if ((threadIdx.x & 63) == 0) out_valid[i >> 6] = word;
    }
}

// byte-exact equality of the key tuples of build row b and probe row p
__device__ __forceinline__ bool tuples_equal(const KeyCols& bc, const KeyCols& pc, uint64_t b, uint64_t p) {
    for (int j = 0; j < bc.n; ++j) {
        const KeyCol& x = bc.c[j];
        const KeyCol& y = pc.c[j];
        if (x.width > 0) {
            if (fixed_word(x, (int64_t)b, 0) != fixed_word(y, (int64_t)p, 0)) return false;
            if (x.width == 16 && fixed_word(x, (int64_t)b, 1) != fixed_word(y, (int64_t)p, 1)) return false;
            continue;
        }
        int64_t xa, xb, ya, yb;
        var_range(x, (int64_t)b, &xa, &xb);
        var_range(y, (int64_t)p, &ya, &yb);
        if (xb - xa != yb - ya) return false;
        const uint8_t* xp = reinterpret_cast<const uint8_t*>(x.values) + xa;
        const uint8_t* yp = reinterpret_cast<const uint8_t*>(y.values) + ya;
        for (int64_t i = 0; i < xb - xa; ++i)
            if (xp[i] != yp[i]) return false;
    }
    return true;
}

__global__ void __launch_bounds__(256)
equal_pairs_kernel(KeyCols bc, KeyCols pc, const uint64_t* __restrict__ bidx, const uint32_t* __restrict__ pidx,
                   int64_t n, uint8_t* __restrict__ flags) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        flags[i] = tuples_equal(bc, pc, bidx[i], pidx[i]) ? 1 : 0;
}

__global__ void __launch_bounds__(256)
gather_pairs_kernel(const uint64_t* __restrict__ pos, const int64_t* __restrict__ d_count,
                    const uint64_t* __restrict__ bidx, const uint32_t* __restrict__ pidx, int64_t n,
                    uint64_t* __restrict__ out_b, uint32_t* __restrict__ out_p) {
    const int64_t m = *d_count;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n && i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t j = pos[i];
        out_b[i] = bidx[j];
        out_p[i] = pidx[j];
    }
}

hipError_t launch_composite_keys(const KeyCols& cols, int64_t n, int64_t* out_keys, uint64_t* out_valid,
                                 hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
    composite_keys_kernel<<<grid, 256, 0, s>>>(cols, n, out_keys, out_valid);
    return hipGetLastError();
}

int64_t equal_pairs_workspace(int64_t n) {
    const int64_t a = (n + 255) & ~(int64_t)255;
    return a + 8 * a + select_workspace(n) + 512;
}

hipError_t launch_equal_pairs(const KeyCols& bc, const KeyCols& pc, const uint64_t* bidx, const uint32_t* pidx,
                              int64_t n, uint64_t* out_b, uint32_t* out_p, int64_t* d_count, void* ws,
                              hipStream_t s) {
    if (n <= 0) return hipMemsetAsync(d_count, 0, sizeof(int64_t), s);
    const int64_t a = (n + 255) & ~(int64_t)255;
    uint8_t* base = reinterpret_cast<uint8_t*>(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    uint8_t* flags = base;
    uint64_t* pos = reinterpret_cast<uint64_t*>(base + a);
    void* sws = base + 9 * a;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
    equal_pairs_kernel<<<grid, 256, 0, s>>>(bc, pc, bidx, pidx, n, flags);
    hipError_t e = launch_select_rows(flags, n, 1, pos, d_count, sws, s);
    if (e != hipSuccess) return e;
    gather_pairs_kernel<<<grid, 256, 0, s>>>(pos, d_count, bidx, pidx, n, out_b, out_p);
    return hipGetLastError();
}

}  // namespace dfp
