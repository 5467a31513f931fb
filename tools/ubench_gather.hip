// Microbenchmark (diagnostic, not product): what bounds a hash-probe lookup on gfx950?
// P = 1e8 rows of int64 keys; per row: hash -> random 64-byte line of a table, write a
// 4-byte result. Variants differ in how the line is fetched:
//   A  no table access (stream keys in, result out)
//   B  one 16-byte load per row (lane = row)
//   C  four 16-byte loads per row (lane = row; today's probe_lookup)
//   D  four lanes per row, one 16-byte load each (one line per row per wave-instruction)
//   E  two lanes per row, two 16-byte loads each
// build: hipcc --offload-arch=gfx950 -O3 -o ubench_gather tools/ubench_gather.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33; return k;
}
__device__ __forceinline__ uint32_t line_of(uint64_t key, uint32_t nl) {
    return (uint32_t)(((mix64(key) >> 32) * (uint64_t)nl) >> 32);
}

template <int V>
__global__ void __launch_bounds__(256) kern(const int64_t* __restrict__ keys, int64_t n, const uint4* __restrict__ tbl,
                                            uint32_t nl, uint32_t* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    if constexpr (V == 0 || V == 1 || V == 2) {
        // lane = 4 consecutive rows
        for (int64_t r0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; r0 < n; r0 += stride * 4) {
            const longlong2 a = *reinterpret_cast<const longlong2*>(keys + r0);
            const longlong2 b = *reinterpret_cast<const longlong2*>(keys + r0 + 2);
            const int64_t k[4] = {a.x, a.y, b.x, b.y};
            uint32_t res[4];
            uint4 L[4][4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t l = line_of(k[q], nl);
                if (V >= 1) L[q][0] = tbl[(size_t)l * 4];
                if (V == 2) { L[q][1] = tbl[(size_t)l * 4 + 1]; L[q][2] = tbl[(size_t)l * 4 + 2]; L[q][3] = tbl[(size_t)l * 4 + 3]; }
                res[q] = l;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (V >= 1) res[q] ^= L[q][0].x ^ L[q][0].w;
                if (V == 2) res[q] ^= L[q][1].y ^ L[q][2].z ^ L[q][3].w;
            }
            *reinterpret_cast<uint4*>(out + r0) = make_uint4(res[0], res[1], res[2], res[3]);
        }
    } else if constexpr (V == 3) {
        // 4 lanes per row: lane piece p loads 16 B of the row's line; 4 rows per group-iteration
        const int lane = threadIdx.x & 63, p = lane & 3;
        for (int64_t base = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63); base < n; base += stride) {
            // a wave covers 16 rows per step, 4 steps = 64 rows
            uint4 L[4];
            uint32_t l[4];
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const int64_t r = base + st * 16 + (lane >> 2);
                const int64_t key = keys[r];
                l[st] = line_of(key, nl);
                L[st] = tbl[(size_t)l[st] * 4 + p];
            }
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                uint32_t v = L[st].x ^ L[st].w;
                v ^= __shfl_xor(v, 1, 64);
                v ^= __shfl_xor(v, 2, 64);
                if (p == 0) out[base + st * 16 + (lane >> 2)] = v ^ l[st];
            }
        }
    } else {
        // 2 lanes per row, 2 x 16 B each; 8 rows... a wave covers 32 rows per step
        const int lane = threadIdx.x & 63, p = lane & 1;
        for (int64_t base = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63); base < n; base += stride) {
            uint4 L[2][2];
            uint32_t l[2];
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                const int64_t r = base + st * 32 + (lane >> 1);
                const int64_t key = keys[r];
                l[st] = line_of(key, nl);
                L[st][0] = tbl[(size_t)l[st] * 4 + 2 * p];
                L[st][1] = tbl[(size_t)l[st] * 4 + 2 * p + 1];
            }
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                uint32_t v = L[st][0].x ^ L[st][1].w;
                v ^= __shfl_xor(v, 1, 64);
                if (p == 0) out[base + st * 32 + (lane >> 1)] = v ^ l[st];
            }
        }
    }
}

template <int V>
float run(const int64_t* keys, int64_t n, const uint4* tbl, uint32_t nl, uint32_t* out, int grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int it = 0; it < 5; ++it) {
        CK(hipEventRecord(a));
        kern<V><<<grid, 256>>>(keys, n, tbl, nl, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best;
}

__global__ void fill(int64_t* k, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        k[i] = (int64_t)mix64((uint64_t)i + 12345);
}

int main() {
    const int64_t n = 100000000;
    int64_t* keys; uint32_t* out; uint4* tbl;
    CK(hipMalloc(&keys, n * 8)); CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&tbl, (size_t)1 << 30));
    CK(hipMemset(tbl, 1, (size_t)1 << 30));
    fill<<<4096, 256>>>(keys, n);
    CK(hipDeviceSynchronize());
    const char* names[] = {"A stream only", "B 1x16B/row", "C 4x16B/row (lane=row)", "D 4 lanes/row x16B",
                           "E 2 lanes/row x32B"};
    for (uint32_t mb : {2u, 32u, 256u, 1024u}) {
        const uint32_t nl = (uint32_t)(((uint64_t)mb << 20) / 64);
        for (int grid : {2048, 8192}) {
            float t[5] = {run<0>(keys, n, tbl, nl, out, grid), run<1>(keys, n, tbl, nl, out, grid),
                          run<2>(keys, n, tbl, nl, out, grid), run<3>(keys, n, tbl, nl, out, grid),
                          run<4>(keys, n, tbl, nl, out, grid)};
            for (int v = 0; v < 5; ++v)
                printf("table %5u MB grid %5d  %-26s %7.3f ms  %6.1f Grows/s\n", mb, grid, names[v], t[v], n / t[v] / 1e6);
        }
    }
    return 0;
}
