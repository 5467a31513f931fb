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
