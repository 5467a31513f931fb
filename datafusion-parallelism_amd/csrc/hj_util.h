// hj_util.h — small device helpers shared by the gfx950 kernel files (wave64 scans,
// Arrow validity bits).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfp {

// Arrow LSB validity bitmap (NULL = all valid)
__device__ __forceinline__ bool bit_valid(const uint8_t* v, int64_t off, int64_t i) {
    if (v == nullptr) return true;
    const int64_t b = off + i;
    return (v[b >> 3] >> (b & 7)) & 1;
}

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T t = __shfl_up(v, (unsigned)d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// Inclusive wave64 scan of u32 in DPP moves (no LDS round trips; __shfl_up is a
// ds_bpermute per step): row_shr 1/2/4/8 scans each 16-lane row, then row_bcast:15 and
// row_bcast:31 carry the row totals into the rows above (GFX9 DPP, gfx950 included).
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    // opaque result: otherwise the compiler rewrites a caller's `incl - v` as the sum of the
    // six shifted partials, which keeps every DPP move apart from its add (18 VALU + 3
    // instead of 6 fused v_add_u32_dpp + 1 per scan; r06: C3 emission 494.5 -> 475.7 us)
    asm volatile("" : "+v"(x));
    return (uint32_t)x;
}

// Inclusive wave64 max-scan of u32, same DPP pattern (0 is the identity)
__device__ __forceinline__ uint32_t wave_incl_max_dpp(uint32_t v) {
    uint32_t x = v;
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
    return x;
}

// wave64 total of u32 (scan, then lane 63 read as a scalar)
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_dpp(v), 63);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// exclusive block scan of one value per thread (blockDim.x <= 1024), returns the
// exclusive prefix, *total = block total. Uses s_w[blockDim.x / 64].
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* s_w, T* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const T incl = wave_incl_scan(v);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    T off = 0, tot = 0;
    for (int w = 0; w < nw; ++w) {
        const T x = s_w[w];
        if (w < wave) off += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return off + incl - v;
}

}  // namespace dfp
