// Microbenchmark: the HBM rate of pure streaming kernels with the sliced probe's traffic
// mixes, to price each probe kernel against what the memory system gives
// for its read:write ratio, not against the 8 TB/s spec alone.
//   copy-mix R:W   every thread reads 16-B words of a source and writes 16-B words of a
//                  destination, R bytes read per W bytes written, coalesced, grid-stride
// Ratios: 4:1 (sl_partition: 8 B keys in, 2 B entries out per row at 50 % in range),
// 1:2 (sl_emit: 6 B entries in, 12 B pairs out), 1:0 (read only), 0:1 (write only), 1:1.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_stream tools/ubench_stream.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

// words_r 16-B words read, words_w written; thread i handles word i of the larger stream and
// the matching word of the smaller one (i * small / large), all coalesced runs
__global__ void __launch_bounds__(256) mix_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                  int64_t words_r, int64_t words_w, uint32_t* sink) {
    const int64_t big = words_r > words_w ? words_r : words_w;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < big; i += (int64_t)gridDim.x * blockDim.x) {
        if (words_r >= words_w) {
            const uint4 v = src[i];
            acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
            if (words_w && (i % (words_r / words_w)) == 0) dst[i / (words_r / words_w)] = acc;
        } else {
            const int64_t ratio = words_w / (words_r ? words_r : 1);
            if (words_r && (i % ratio) == 0) {
                const uint4 v = src[i / ratio];
                acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
            }
            dst[i] = make_uint4(acc.x + (uint32_t)i, acc.y, acc.z, acc.w);
        }
    }
    if (acc.x == 0x12345678u) *sink = acc.y;  // keeps the loads alive
}

int main(int argc, char** argv) {
    const int64_t total = (argc > 1 ? atoll(argv[1]) : 1000) << 20;  // bytes moved per launch (r + w)
    const int ratios[][2] = {{1, 0}, {0, 1}, {1, 1}, {4, 1}, {1, 2}};
    uint4 *src, *dst;
    uint32_t* sink;
    CHECK(hipMalloc(&src, total));
    CHECK(hipMalloc(&dst, total));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(src, 1, total));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (auto& r : ratios) {
        const int64_t words = total / 16;
        const int64_t wr = words * r[0] / (r[0] + r[1]), ww = words * r[1] / (r[0] + r[1]);
        for (int grid : {2048, 8192, 32768}) {
            float best = 1e9f;
            for (int it = 0; it < 6; ++it) {
                CHECK(hipEventRecord(a));
                mix_kernel<<<grid, 256>>>(src, dst, wr, ww, sink);
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                float ms;
                CHECK(hipEventElapsedTime(&ms, a, b));
                if (it > 0 && ms < best) best = ms;
            }
            const double bytes = 16.0 * (wr + ww);
            printf("R:W %d:%d grid %5d  %.1f MB in %7.1f us = %.2f TB/s\n", r[0], r[1], grid, bytes / 1e6, best * 1e3,
                   bytes / (best * 1e-3) / 1e12);
        }
    }
    return 0;
}
