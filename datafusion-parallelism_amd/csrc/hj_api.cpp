// hj_api.cpp — C-ABI host layer (include/hj.h) over the gfx950 kernels.
//
// Mirrors the reference's build/probe choreography:
//   * hj_build_begin      ~ BuildImplementation::new / JoinStateInstances::new
//                           (src/operator/build_implementation.rs:34-48,
//                            src/operator/version10/parallel_join_execution_state.rs:377-403)
//   * hj_build_append     ~ process_input_batch -> JoinStateInstance::add
//                           (src/operator/version10/build_implementation.rs:60-71,
//                            parallel_join_execution_state.rs:91-133)
//   * hj_build_finish     ~ compact_join_map: every partition arrives, the last arriver
//                           finalises, the others wait (InitializeLast,
//                           src/utils/initialize_last.rs:26-43; BarrierOnce,
//                           src/utils/barrier_once.rs:4-35)
//   * hj_probe            ~ lookup_inner_join_probe_batch minus the Arrow take
//                           (src/operator/probe_lookup_implementation/inner.rs:79-129)
// Errors: HJ_ERR_INVALID carries the reference's DataFusionError::Internal texts where
// one exists (e.g. "State already consumed for partition N",
// src/operator/version10/build_implementation.rs:32-33).
//
// There is no CPU code path: without a GPU every entry point fails with
// HJ_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "../../include/hj.h"
#include "hj_device.h"
#include "hj_host.h"
#include "hj_launch.h"

using namespace dfp;

struct MultiTable;  // hj_build_begin_multi facade (below)

namespace {

thread_local std::string g_err;

hj_status fail(hj_status st, const std::string& msg) {
    g_err = msg;
    return st;
}

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return fail(HJ_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_));    \
    } while (0)

struct ThreadStreams {
    std::unordered_map<int, hipStream_t> m;
    ~ThreadStreams() {
        for (auto& kv : m) (void)hipStreamDestroy(kv.second);
    }
};
thread_local ThreadStreams g_streams;

hipStream_t thread_stream(int dev) {
    auto it = g_streams.m.find(dev);
    if (it != g_streams.m.end()) return it->second;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    g_streams.m[dev] = s;
    return s;
}

// Tables reuse build streams and events (creating them costs ~0.1 ms per table).
struct BuildResources {
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t evp = nullptr;  // end of the table's latest probe launch (no timing)
    // key-range mailbox, fine-grained host memory written by the minmax kernel: min, max,
    // sequence number (the host spins on it instead of a copy + stream synchronize)
    int64_t* h_minmax = nullptr;
    int64_t* d_mbox = nullptr;  // its device address
    int64_t mb_seq = 0;
};
std::mutex g_pool_mu;
std::unordered_map<int, std::vector<BuildResources>> g_pool;

// Release scope of the events that only order this device's own streams (the probe-end
// events; DFP_HJ_EV_SCOPE=1 also the build events): a default event's system-scope release
// writes the L2 back after every probe (measured: DESIGN.md §4.7)
int ev_scope() {
    static const int v = [] {
        const char* e = getenv("DFP_HJ_EV_SCOPE");
        return e ? atoi(e) : 0;
    }();
    return v;
}
// (measured: probe-end events without any system-scope fence changed nothing either,
// profiles/r04_nontemporal_ab.txt)
unsigned probe_ev_flags() { return hipEventDisableTiming | (ev_scope() >= 1 ? hipEventReleaseToDevice : 0u); }
unsigned build_ev_flags() { return ev_scope() >= 2 ? hipEventReleaseToDevice : hipEventDefault; }

bool acquire_resources(int dev, BuildResources* r) {
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        auto& v = g_pool[dev];
        if (!v.empty()) {
            *r = v.back();
            v.pop_back();
            return true;
        }
    }
    return hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev0, build_ev_flags()) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev1, build_ev_flags()) == hipSuccess &&
           hipEventCreateWithFlags(&r->evp, probe_ev_flags()) == hipSuccess &&
           hipHostMalloc((void**)&r->h_minmax, 4 * sizeof(int64_t), hipHostMallocCoherent | hipHostMallocMapped) ==
               hipSuccess &&
           hipHostGetDevicePointer((void**)&r->d_mbox, r->h_minmax, 0) == hipSuccess;
}

void release_resources(int dev, const BuildResources& r) {
    std::lock_guard<std::mutex> g(g_pool_mu);
    g_pool[dev].push_back(r);
}

// Caching device allocator: tables come and go per query, and hipMallocAsync/
// hipFreeAsync cost ~0.1 ms per call on ROCm; blocks are kept per (device, size class)
// and handed out again. A block is only reused after its table was freed, and the
// caller frees a table only after every stream that probed it has been synchronised
// (hj_table_free contract).
struct DevCache {
    std::mutex mu;
    std::map<uint64_t, std::vector<void*>> bins;  // key = device << 48 | size class (ordered: best fit)
    std::unordered_map<void*, size_t> cls;        // size class of every block handed out
    size_t cached_bytes = 0;
};
DevCache g_cache;

size_t size_class(size_t bytes) {
    if (bytes <= 4096) return 4096;
    if (bytes <= (1u << 20)) {  // powers of two below 1 MiB
        size_t c = 4096;
        while (c < bytes) c <<= 1;
        return c;
    }
    const size_t step = bytes <= (256u << 20) ? (2u << 20) : (32u << 20);
    return (bytes + step - 1) / step * step;
}

// Blocks of 64 MiB and more may also come from a cached block up to 1/4 larger (best fit):
// multi-GB scratch of slightly different sizes (each join of a query, each probe batch)
// reuses the same blocks instead of piling up until an allocation fails and the whole
// cache is released (the 8-shard SF300 Q9 on one GPU spent seconds there).
constexpr size_t kBestFitMin = size_t(64) << 20;

void* cache_alloc(int dev, size_t bytes, hipError_t* err) {
    const size_t c = size_class(bytes);
    const uint64_t key = ((uint64_t)dev << 48) | c;
    {
        std::lock_guard<std::mutex> g(g_cache.mu);
        auto it = g_cache.bins.find(key);
        if ((it == g_cache.bins.end() || it->second.empty()) && c >= kBestFitMin) {
            for (it = g_cache.bins.lower_bound(key);
                 it != g_cache.bins.end() && (it->first >> 48) == (uint64_t)dev &&
                 (it->first & ((1ull << 48) - 1)) <= c + c / 4;
                 ++it)
                if (!it->second.empty()) break;
            if (it != g_cache.bins.end() && ((it->first >> 48) != (uint64_t)dev ||
                                             (it->first & ((1ull << 48) - 1)) > c + c / 4))
                it = g_cache.bins.end();
        }
        if (it != g_cache.bins.end() && !it->second.empty()) {
            void* p = it->second.back();
            it->second.pop_back();
            const size_t bc = (size_t)(it->first & ((1ull << 48) - 1));
            g_cache.cached_bytes -= bc;
            g_cache.cls[p] = bc;
            *err = hipSuccess;
            return p;
        }
    }
    void* p = nullptr;
    // DFP_HJ_ALLOC_LOG=1: every cache miss (a hipMalloc) and every release of the cache to stderr
    static const bool alog = [] {
        const char* e = getenv("DFP_HJ_ALLOC_LOG");
        return e != nullptr && e[0] == '1';
    }();
    if (alog) fprintf(stderr, "[dfp alloc] miss dev %d bytes %zu class %zu cached %zu\n", dev, bytes, c, g_cache.cached_bytes);
    *err = hipMalloc(&p, c);
    if (*err != hipSuccess) {
        (void)hipGetLastError();
        // Cached blocks of this device are released until the allocation fits - not the whole
        // cache: the 8-shard SF300 Q9 on one GPU (torch holding 156 GB beside this cache's up to
        // 129 GB) released everything on such a miss and re-allocated it in the next join, 1.5-3.9
        // s per query against 0.29 s (profiles/r06_q9_sf300_alloc.txt)
        std::lock_guard<std::mutex> g(g_cache.mu);
        if (alog) fprintf(stderr, "[dfp alloc] hipMalloc %zu failed with %zu cached bytes\n", c, g_cache.cached_bytes);
        // first the smallest cached block of at least this size is released (one hipFree of about
        // the request: the big blocks other joins reuse stay cached), then, if that is not enough,
        // blocks from the largest down. (Handing a larger cached block out instead, with no free,
        // left the HSA runtime no device memory for its own resources: the process aborted with
        // HSA_STATUS_ERROR_OUT_OF_RESOURCES, gpurun_out/r06m.)
        for (auto it = g_cache.bins.lower_bound(key); it != g_cache.bins.end() && (it->first >> 48) == (uint64_t)dev;
             ++it) {
            if (it->second.empty()) continue;
            void* q = it->second.back();
            it->second.pop_back();
            (void)hipFree(q);
            g_cache.cached_bytes -= (size_t)(it->first & ((1ull << 48) - 1));
            *err = hipMalloc(&p, c);
            if (*err == hipSuccess) {
                if (alog) fprintf(stderr, "[dfp alloc] released one cached block of %zu bytes: ok\n",
                                  (size_t)(it->first & ((1ull << 48) - 1)));
                g_cache.cls[p] = c;
                return p;
            }
            (void)hipGetLastError();
            break;
        }
        size_t freed = 0;
        for (;;) {
            auto lo = g_cache.bins.lower_bound((uint64_t)dev << 48);
            auto hi = g_cache.bins.lower_bound((uint64_t)(dev + 1) << 48);
            auto big = g_cache.bins.end();
            for (auto it = hi; it != lo;) {  // the largest class with a cached block
                --it;
                if (!it->second.empty()) {
                    big = it;
                    break;
                }
            }
            if (big == g_cache.bins.end()) break;
            void* q = big->second.back();
            big->second.pop_back();
            (void)hipFree(q);
            const size_t qc = (size_t)(big->first & ((1ull << 48) - 1));
            g_cache.cached_bytes -= qc;
            freed += qc;
            if (freed >= c) {
                *err = hipMalloc(&p, c);
                if (*err == hipSuccess) break;
                (void)hipGetLastError();
            }
        }
        if (*err != hipSuccess) *err = hipMalloc(&p, c);
        if (alog) fprintf(stderr, "[dfp alloc] released %zu bytes: %s\n", freed, *err == hipSuccess ? "ok" : "failed");
        if (*err == hipSuccess) {
            g_cache.cls[p] = c;
            return p;
        }
    }
    if (*err != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(g_cache.mu);
    g_cache.cls[p] = c;
    return p;
}

void cache_free(int dev, void* p, size_t bytes) {
    if (p == nullptr) return;
    std::lock_guard<std::mutex> g(g_cache.mu);
    size_t c = size_class(bytes);
    auto it = g_cache.cls.find(p);  // a best-fit block goes back to its own class
    if (it != g_cache.cls.end()) {
        c = it->second;
        g_cache.cls.erase(it);
    }
    g_cache.bins[((uint64_t)dev << 48) | c].push_back(p);
    g_cache.cached_bytes += c;
}

int device_count() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// true when p is device (or managed) memory visible to the current device
bool is_device_ptr(const void* p) {
    if (p == nullptr) return true;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// Keys per slot of a hashed table. 0.5 keeps a 10^7-key table within the sliced probe's
// 2047 slices of 2048 buckets (128 KB of LDS each; C2h), where the slices are read once
// per probe; the fused probe measured 2048 us at 0.35 and 2150 us at 0.5 on C2
// (profiles/r01_load_factor.txt). Override with DFP_HJ_LOAD_FACTOR.
constexpr double kDefaultLoadFactor = 0.5;

// Table layout: 0 auto (direct-addressed when the key range is at most kDenseFactor x the
// build rows, else hashed buckets), 1 hashed always. DFP_HJ_DENSE=0 selects 1.
std::atomic<int> g_build_mode{-1};
int build_mode_raw() {
    int m = g_build_mode.load(std::memory_order_relaxed);
    if (m < 0) {
        const char* e = getenv("DFP_HJ_DENSE");
        m = (e && e[0] == '0') ? 1 : 0;
        const char* f = getenv("DFP_HJ_FRAG_BUILD");
        if (m == 0 && f && f[0] == '0') m = 2;
        g_build_mode.store(m, std::memory_order_relaxed);
    }
    return m;
}
// 0 and 2 both choose the direct-addressed layout for dense key ranges; 2 keeps the
// histogram + scan + staged-scatter partition for it (the tile-local one is the default)
int build_mode() { return build_mode_raw() == 1 ? 1 : 0; }
bool frag_build_mode() { return build_mode_raw() == 0; }
// Per-table device budget in bytes (0 = none): a one-device table whose build would hold
// more than this (staged input, table, duplicate segments, build scratch) refuses with
// HJ_ERR_OOM, the signal for a planner to shard the build over several GPUs. Stands in
// for the capacity of one GPU's HBM (C5: a build side larger than one GPU). Set with
// hj_set_device_budget or DFP_HJ_DEVICE_BUDGET_BYTES.
std::atomic<int64_t> g_budget{-1};
int64_t device_budget() {
    int64_t b = g_budget.load(std::memory_order_relaxed);
    if (b < 0) {
        const char* e = getenv("DFP_HJ_DEVICE_BUDGET_BYTES");
        b = e ? std::max<int64_t>(0, atoll(e)) : 0;
        int64_t unset = -1;
        g_budget.compare_exchange_strong(unset, b, std::memory_order_relaxed);
        b = g_budget.load(std::memory_order_relaxed);
    }
    return b;
}
// DFP_HJ_SPEC_BUILD=0: the host reads the build's key range before it launches the build
// (rounds 1-3; the device idles for the mailbox round trip between the reduction and the
// partition)
bool spec_build_on() {
    static const bool v = [] {
        const char* e = getenv("DFP_HJ_SPEC_BUILD");
        return !(e != nullptr && e[0] == '0');
    }();
    return v;
}
double load_factor() {
    const char* e = getenv("DFP_HJ_LOAD_FACTOR");
    double lf = e ? atof(e) : kDefaultLoadFactor;
    if (!(lf > 0.05 && lf <= 0.95)) lf = kDefaultLoadFactor;
    return lf;
}

struct HostSeg {
    const void* keys = nullptr;
    const uint8_t* valid = nullptr;
    int64_t voff = 0;
    const uint64_t* ids = nullptr;
    int64_t n = 0;
    std::vector<void*> owned;    // device copies owned by the table
    hipEvent_t ready = nullptr;  // borrowed device input: produced when this fires
};

}  // namespace

struct hj_table {
    int device = 0;
    int parallelism = 1;
    hj_key_type kt = HJ_INT64;
    int key_bytes = 8;

    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::vector<HostSeg>> parts;
    std::vector<char> finished;
    int arrived = 0;
    bool built = false;
    bool sync_finish = false;  // some input was borrowed without HJ_BORROW_KEEP
    // end of the latest probe launch on each stream that probed the table: hj_table_free
    // waits for all of them (res.evp serves the first stream; others get their own event)
    mutable std::mutex probe_mu;
    mutable std::vector<std::pair<hipStream_t, hipEvent_t>> probe_evs;
    hj_status build_st = HJ_OK;
    std::string build_err;
    bool has_ids = false, has_no_ids = false;
    bool ids_u31 = true;  // every id batch carries HJ_IDS_U31: ids replace row numbers

    std::vector<int64_t> part_off;
    int64_t total_rows = 0;

    // device state
    Bucket* tbl = nullptr;
    uint32_t nb = 0, clog2 = 10, nchunks = 0;
    uint32_t* dup_rows = nullptr;
    BuildCounters* ctr = nullptr;  // the build's counters (dup_rows words in use), table-owned
    bool wrapped = false;          // hj_table_wrap_dense: arrays borrowed from the caller
    uint64_t* row_ids = nullptr;
    uint32_t* dense = nullptr;  // direct-addressed layout (dense key range), else buckets
    bool packed = false;        // dense refs with inline counts (dup_rows offsets < 2^27)
    int64_t dmin = 0;
    uint64_t drange = 0;
    bool has_range = false;     // hj_build_key_range: the caller's key range replaces the reduction
    bool force_dense = false;   // hj_build_dense: direct-addressed over that range whatever the density
    int64_t range_lo = 0, range_hi = 0;
    bool has_base = false;      // hj_build_key_base: int32 build keys are offsets from key_base;
    int64_t key_base = 0;       // the built (direct-addressed) table is keyed in the int64 domain
    BuildResources res;
    // the stream the build runs on: the producers' stream when every append came on the
    // same one (a probe there needs no cross-stream wait), else res.stream
    hipStream_t bstream = nullptr;
    hipStream_t app_stream = nullptr;
    int app_streams = 0;  // 0 none yet, 1 one stream, 2 several
    int64_t build_ns = 0;
    std::vector<std::pair<void*, size_t>> allocs;   // live for the table's lifetime
    std::vector<std::pair<void*, size_t>> scratch;  // build-only, released after the build
    // multi-GPU facade: shards on several devices behind this handle (hj_build_begin_multi)
    MultiTable* multi = nullptr;
    std::vector<std::tuple<int, void*, size_t>> multi_bufs;  // (device, block, bytes) the shards borrow
    // device bytes the table holds (allocs + scratch) and their peak: the device budget's
    // measure (hj_set_device_budget)
    int64_t live_bytes = 0, peak_bytes = 0;
    std::vector<hj_table*> owned_tables;  // freed with this table (hj_dist.cpp's local pieces)
    hipEvent_t ext_ev0 = nullptr;         // table_set_start_event: the build time's start (owned)
    // build with the key range left on the device (SpecGeo, build_attempt): the host has not
    // read the range yet; ensure_geometry reads it before any use of the table's geometry
    std::atomic<bool> spec_pending{false};
    std::mutex spec_mu;
    int64_t spec_seq = 0;
    uint32_t spec_cap = 0;
    const int64_t* spec_mm = nullptr;  // the reduction's result in device memory (scratch)
    std::vector<Segment> spec_segs;    // the build's segments, for a build in another layout
    bool mm_known = false;             // the key range read after a speculative build
    int64_t mm_lo = 0, mm_hi = 0;
};

namespace dfp {
namespace host {
hj_status set_error(hj_status st, const std::string& msg) { return fail(st, msg); }
void* dev_block(int dev, size_t bytes) {
    hipError_t e;
    return cache_alloc(dev, bytes ? bytes : 64, &e);
}
void free_block(int dev, void* p, size_t bytes) { cache_free(dev, p, bytes ? bytes : 64); }
void table_adopt_block(hj_table* t, int dev, void* p, size_t bytes) {
    t->multi_bufs.emplace_back(dev, p, bytes ? bytes : 64);
}
void table_adopt_table(hj_table* t, hj_table* other) { t->owned_tables.push_back(other); }
void table_set_start_event(hj_table* t, hipEvent_t ev) {
    if (t->ext_ev0) (void)hipEventDestroy(t->ext_ev0);
    t->ext_ev0 = ev;
    t->build_ns = -1;
}
}  // namespace host
}  // namespace dfp

namespace {

// Spin until the minmax kernel's mailbox shows `seq` (a few us after the kernel ends,
// against ~20 us for copy + stream synchronize). Every 4096 polls the stream is queried:
// an error returns; a finished stream whose mailbox never updated falls back to a copy.
hipError_t wait_mailbox(int64_t* mm, int64_t seq, const int64_t* d_minmax, hipStream_t s) {
    for (uint32_t i = 1;; ++i) {
        if (__atomic_load_n(&mm[2], __ATOMIC_ACQUIRE) == seq) return hipSuccess;
        if ((i & 4095) == 0) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipErrorNotReady) continue;
            if (q != hipSuccess) return q;
            if (__atomic_load_n(&mm[2], __ATOMIC_ACQUIRE) == seq) return hipSuccess;
            return hipMemcpy(mm, d_minmax, 2 * sizeof(int64_t), hipMemcpyDeviceToHost);
        }
        __builtin_ia32_pause();
    }
}

hj_status dev_alloc(hj_table* t, std::vector<std::pair<void*, size_t>>& list, void** p, size_t bytes) {
    if (bytes == 0) bytes = 64;
    const int64_t budget = device_budget();
    if (budget > 0 && t->live_bytes + (int64_t)bytes > budget)
        return fail(HJ_ERR_OOM, "device budget: this build needs more than " + std::to_string(budget) +
                                    " bytes of one device (DFP_HJ_DEVICE_BUDGET_BYTES / hj_set_device_budget); "
                                    "shard it over several GPUs (hj_build_begin_multi, radix plan)");
    hipError_t e;
    *p = cache_alloc(t->device, bytes, &e);
    if (*p == nullptr) return fail(HJ_ERR_OOM, std::string("device allocation: ") + hipGetErrorString(e));
    list.emplace_back(*p, bytes);
    t->live_bytes += (int64_t)bytes;
    t->peak_bytes = std::max(t->peak_bytes, t->live_bytes);
    return HJ_OK;
}

// only once no queued work uses the blocks any more
void free_list(hj_table* t, std::vector<std::pair<void*, size_t>>& list) {
    for (auto& pb : list) {
        cache_free(t->device, pb.first, pb.second);
        t->live_bytes -= (int64_t)pb.second;
    }
    list.clear();
}

hipDeviceProp_t* device_props(int dev) {
    static std::mutex mu;
    static std::unordered_map<int, hipDeviceProp_t> cache;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(dev);
    if (it == cache.end()) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, dev) != hipSuccess) return nullptr;
        it = cache.emplace(dev, p).first;
    }
    return &it->second;
}

// One device build attempt at load factor lf; sets *retry when a chunk overflowed.
hj_status build_attempt(hj_table* t, const std::vector<Segment>& segs, double lf, bool* retry) {
    *retry = false;
    const int64_t total = t->total_rows;
    hj_status st;
    void* p;
    hipStream_t s = t->bstream;
    Segment* d_segs;
    BuildCounters* ctr;
    int64_t* d_minmax;
    if ((st = dev_alloc(t, t->scratch, &p, sizeof(Segment) * std::max<size_t>(segs.size(), 1))) != HJ_OK) return st;
    d_segs = (Segment*)p;
    // the counters live with the table: hj_table_dense_piece hands out dup_used
    if ((st = dev_alloc(t, t->allocs, &p, sizeof(BuildCounters))) != HJ_OK) return st;
    ctr = (BuildCounters*)p;
    t->ctr = ctr;
    if ((st = dev_alloc(t, t->scratch, &p, (2 + 2 * kMinmaxMaxBlocks) * sizeof(int64_t))) != HJ_OK) return st;
    d_minmax = (int64_t*)p;
    // few segments: the key-range kernel publishes them and zeroes the counters (no
    // reduction when the caller gave the range)
    const bool need_range = total > 0 && build_mode() == 0 && !t->has_range;
    const bool minmax = need_range && !t->mm_known;  // the reduction runs (not read back yet)
    const bool by_arg = minmax && segs.size() <= (size_t)kArgSegs;
    if (!by_arg) {
        if (!segs.empty())
            HIP_TRY(hipMemcpyAsync(d_segs, segs.data(), sizeof(Segment) * segs.size(), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemsetAsync(ctr, 0, sizeof(BuildCounters), s));
    }

    std::vector<int64_t> seg_n(segs.size());
    for (size_t i = 0; i < segs.size(); ++i) seg_n[i] = segs[i].n;
    const int64_t ftiles = frag_build_tiles(seg_n.data(), (int)segs.size());
    // Speculative dense frag build: the kernels take the range from the reduction's result
    // in device memory (SpecGeo), so the build runs on with no host round trip between the
    // reduction and the partition; the grid and the blocks cover the widest range the frag
    // build takes (kDenseFactor x rows, <= kMaxLevel1Bins blocks). The host reads the range
    // when the table is first used (ensure_geometry); a range that takes another layout
    // (the kernels then wrote nothing) is built there.
    const bool packed_ok = (uint64_t)(2 * total + 2) < (1ull << 27);  // every dup_rows offset fits
    const uint32_t spec_cap =
        (uint32_t)std::min<uint64_t>(kMaxLevel1Bins, (kDenseFactor * (uint64_t)total + kDenseBlockValues - 1) /
                                                         kDenseBlockValues);
    const ChunkGeom spec_g{0, 0, spec_cap << kDenseBlockShift, kDenseShift, 0, 1, packed_ok ? 1 : 0};
    const bool spec = minmax && spec_build_on() && !t->has_base && !t->force_dense && t->multi == nullptr &&
                      device_budget() <= 0 && frag_build_mode() && spec_cap > 0 && frag_build_ok(spec_g, ftiles);
    // layout: a dense key range gets the direct-addressed table (one u32 ref per key value)
    ChunkGeom g{};
    bool dense = false;
    if (need_range || (t->has_range && total > 0 && (build_mode() == 0 || t->force_dense))) {
        int64_t mm[2] = {t->range_lo, t->range_hi};
        if (t->mm_known) {
            mm[0] = t->mm_lo;
            mm[1] = t->mm_hi;
        }
        if (minmax) {
            int64_t* mb = t->res.h_minmax;
            const int64_t seq = ++t->res.mb_seq;
            HIP_TRY(launch_key_minmax(t->key_bytes, segs.data(), d_segs, (int)segs.size(), by_arg ? ctr : nullptr,
                                      total, d_minmax, t->res.d_mbox, seq, s));
            if (spec) {
                t->spec_seq = seq;
                t->spec_cap = spec_cap;
                t->spec_mm = d_minmax;
                t->spec_segs = segs;
                mm[0] = 1;  // not read: the geometry below is spec_g's
                mm[1] = 0;
            } else {
                HIP_TRY(wait_mailbox(mb, seq, d_minmax, s));
                mm[0] = mb[0];
                mm[1] = mb[1];
            }
        }
        if (spec) {
            dense = true;
            g = spec_g;
            t->dmin = 0;
            t->drange = 0;
        } else if (mm[0] <= mm[1]) {
            const uint64_t range = (uint64_t)mm[1] - (uint64_t)mm[0] + 1;
            const uint64_t nch = (range + (1u << kDenseShift) - 1) >> kDenseShift;
            if (range != 0 && (range <= kDenseFactor * (uint64_t)total || t->force_dense) &&
                nch <= (uint64_t)kMaxChunks) {
                dense = true;
                g = ChunkGeom{0, 0, (uint32_t)nch, kDenseShift, mm[0], 1, packed_ok ? 1 : 0};
                t->dmin = mm[0];
                t->drange = range;
            }
        }
    }
    if (!dense && t->has_base && total > 0)
        return fail(HJ_ERR_INVALID, "hj_build_key_base: the build keys do not make a direct-addressed table "
                                    "(key range > 8 x rows); build from int64 keys instead");
    if (!dense) {
        // geometry: 5-slot buckets, chunks of 2^clog2 buckets (one workgroup builds one)
        const double want = (double)total / (kSlots * lf);
        // smallest chunks that fit the chunk count limit (512 buckets build four per CU)
        uint32_t clog2 = 9;
        uint64_t nchunks = (uint64_t)(want / (1u << clog2)) + 1;
        while (nchunks > (uint64_t)kMaxChunks && clog2 < 11) {
            ++clog2;
            nchunks = (uint64_t)(want / (1u << clog2)) + 1;
        }
        if (nchunks > (uint64_t)kMaxChunks) {
            // very large builds: fill the largest table geometry fuller (up to 0.8 slots/key)
            const double full = (double)kMaxChunks * (1u << clog2) * kSlots;
            if ((double)total / full > 0.8)
                return fail(HJ_ERR_INVALID, "build side too large for one device table; shard it (hj_radix_partition)");
            nchunks = kMaxChunks;
        }
        g = ChunkGeom{(uint32_t)(nchunks << clog2), clog2, (uint32_t)nchunks, 0, 0, 0, 0};
        t->dmin = 0;
        t->drange = 0;
    }
    t->clog2 = g.clog2;
    t->nchunks = g.nchunks;
    t->packed = g.packed != 0;
    t->nb = g.nb;
    const uint64_t nchunks = g.nchunks;
    // dense builds that fit the tile-local partition skip the histogram/scan/scatter path
    const bool frag = dense && total > 0 && frag_build_mode() && frag_build_ok(g, ftiles);
    // hashed tables: the frag build unless mode 2 keeps the histogram path (DFP_HJ_FRAG_BUILD=0)
    // (the hashed frag build's tiles are 2^hashed_build_tile_log() rows, the dense one's 2^14)
    const int64_t hftiles = frag_build_tiles(seg_n.data(), (int)segs.size(), hashed_build_tile_log());
    const bool hfrag = !dense && total > 0 && build_mode_raw() != 2 && hashed_frag_ok(g, hftiles);
    hipDeviceProp_t* prop0 = device_props(t->device);
    const int64_t ntiles = build_tiles(total, prop0 ? prop0->multiProcessorCount : 256);
    const int64_t tile_rows = build_tile_rows(total, ntiles);
    const int64_t hlen = (int64_t)(nchunks + 1) * ntiles;

    t->tbl = nullptr;
    t->dense = nullptr;
    if (dense) {
        // the one-level build writes whole blocks of 2^kDenseBlockShift chunks
        const uint64_t dchunks = dense_one_level((uint32_t)nchunks)
                                     ? (uint64_t)dense_blocks((uint32_t)nchunks) << kDenseBlockShift
                                     : nchunks;
        if ((st = dev_alloc(t, t->allocs, &p, sizeof(uint32_t) * (size_t)(dchunks << kDenseShift))) != HJ_OK)
            return st;
        t->dense = (uint32_t*)p;
    } else {
        if ((st = dev_alloc(t, t->allocs, &p, (size_t)(t->nb + 1) * sizeof(Bucket))) != HJ_OK) return st;
        t->tbl = (Bucket*)p;
    }
    if ((st = dev_alloc(t, t->allocs, &p, sizeof(uint32_t) * (size_t)(2 * total + 2))) != HJ_OK) return st;
    t->dup_rows = (uint32_t*)p;
    const bool ids_as_rows = t->has_ids && t->ids_u31;  // no id indirection at probe time
    if (t->has_ids && !ids_as_rows) {
        if ((st = dev_alloc(t, t->allocs, &p, sizeof(uint64_t) * (size_t)std::max<int64_t>(total, 1))) != HJ_OK)
            return st;
        t->row_ids = (uint64_t*)p;
    }
    if (frag || hfrag) {
        void* fscr;
        uint32_t* d_tb;
        uint64_t* ids32 = nullptr;
        BigSeg* fbig;
        const int64_t fbytes =
            frag ? frag_build_scratch_bytes(g, ftiles, total) : hashed_frag_scratch_bytes(g, hftiles, total);
        if ((st = dev_alloc(t, t->scratch, &fscr, (size_t)fbytes)) != HJ_OK) return st;
        if ((st = dev_alloc(t, t->scratch, &p, sizeof(uint32_t) * (size_t)(frag ? ftiles : hftiles))) != HJ_OK)
            return st;
        d_tb = (uint32_t*)p;
        if ((st = dev_alloc(t, t->scratch, &p, sizeof(BigSeg) * (size_t)(total / (kSmallSeg + 1) + 2))) != HJ_OK)
            return st;
        fbig = (BigSeg*)p;
        if (t->has_ids) {  // explicit ids in row order: the table's row_ids, or scratch when held in place of rows
            uint64_t* dst = t->row_ids;
            if (ids_as_rows && segs.size() == 1) {
                ids32 = const_cast<uint64_t*>(segs[0].ids);  // one device segment: read in place (borrowed)
                dst = nullptr;
            } else if (ids_as_rows) {
                if ((st = dev_alloc(t, t->scratch, &p, sizeof(uint64_t) * (size_t)total)) != HJ_OK) return st;
                dst = ids32 = (uint64_t*)p;
            }
            if (dst != nullptr)
                for (const Segment& sg : segs)
                    HIP_TRY(hipMemcpyAsync(dst + sg.row_base, sg.ids, sizeof(uint64_t) * (size_t)sg.n,
                                           hipMemcpyDefault, s));
        }
        hipDeviceProp_t* prop = device_props(t->device);
        const int cus = prop ? prop->multiProcessorCount : 256;
        if (frag) {
            HIP_TRY(launch_build_frag(t->key_bytes, segs.data(), (int)segs.size(), g, ftiles, fscr, d_tb, ids32,
                                      t->dense, t->dup_rows, fbig, ctr, d_segs, total, ids_as_rows, cus,
                                      spec ? SpecGeo{(const long long*)d_minmax, (uint64_t)total, spec_cap}
                                           : SpecGeo{nullptr, 0, 0},
                                      s));
            // a direct-addressed build cannot overflow (no retry): nothing to read back, the
            // build stays asynchronous; consumers wait on its completion event
            if (spec) t->spec_pending.store(true, std::memory_order_release);
            return HJ_OK;
        }
        HIP_TRY(launch_build_hashed_frag(t->key_bytes, segs.data(), (int)segs.size(), g, hftiles, fscr, d_tb, ids32,
                                         t->tbl, t->dup_rows, fbig, ctr, d_segs, total, ids_as_rows, cus, s));
        // a chunk can overflow (adversarial keys): read the error word back, rebuild at half load
        BuildCounters hc;
        HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(hc), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        free_list(t, t->scratch);
        if (hc.err & ~3ull)
            return fail(HJ_ERR_HIP, "hashed build: internal check failed (error bits " + std::to_string(hc.err) + ")");
        if (hc.err) {
            *retry = true;
            free_list(t, t->allocs);
            t->row_ids = nullptr;
        }
        return HJ_OK;
    }
    uint32_t *hist, *hist1, *srows, *trows;
    unsigned long long *skeys, *tkeys;
    BigSeg* big;
    void* scan;
    if ((st = dev_alloc(t, t->scratch, &p, sizeof(uint32_t) * (size_t)std::max<int64_t>(hlen, 1))) != HJ_OK) return st;
    hist = (uint32_t*)p;
    if ((st = dev_alloc(t, t->scratch, &p, sizeof(uint32_t) * (size_t)std::max<int64_t>(kMaxLevel1Bins * ntiles, 1))) !=
        HJ_OK)
        return st;
    hist1 = (uint32_t*)p;
    uint32_t* chunk_starts;
    if ((st = dev_alloc(t, t->scratch, &p, sizeof(uint32_t) * (size_t)(nchunks + 2))) != HJ_OK) return st;
    chunk_starts = (uint32_t*)p;
    if ((st = dev_alloc(t, t->scratch, &p, (size_t)scan_scratch_bytes(std::max<int64_t>(hlen, kMaxLevel1Bins * ntiles)))) !=
        HJ_OK)
        return st;
    scan = p;
    if ((st = dev_alloc(t, t->scratch, &p, 8 * (size_t)std::max<int64_t>(total, 1))) != HJ_OK) return st;
    skeys = (unsigned long long*)p;
    if ((st = dev_alloc(t, t->scratch, &p, 4 * (size_t)std::max<int64_t>(total, 1))) != HJ_OK) return st;
    srows = (uint32_t*)p;
    if ((st = dev_alloc(t, t->scratch, &p, 8 * (size_t)std::max<int64_t>(total, 1))) != HJ_OK) return st;
    tkeys = (unsigned long long*)p;
    if ((st = dev_alloc(t, t->scratch, &p, 4 * (size_t)std::max<int64_t>(total, 1))) != HJ_OK) return st;
    trows = (uint32_t*)p;
    if ((st = dev_alloc(t, t->scratch, &p, sizeof(BigSeg) * (size_t)(total / (kSmallSeg + 1) + 2))) != HJ_OK)
        return st;
    big = (BigSeg*)p;

    if (total == 0) HIP_TRY(hipMemsetAsync(t->tbl, 0, (size_t)(t->nb + 1) * sizeof(Bucket), s));
    hipDeviceProp_t* prop = device_props(t->device);
    const int cus = prop ? prop->multiProcessorCount : 256;
    HIP_TRY(launch_build(t->key_bytes, d_segs, (int)segs.size(), total, g, hist, hist1, chunk_starts, ntiles, tile_rows,
                         scan, tkeys, trows, skeys, srows, t->row_ids, ids_as_rows, t->tbl, t->dense, t->dup_rows, big,
                         ctr, cus, s));
    if (dense) return HJ_OK;  // cannot overflow: asynchronous, as above
    BuildCounters hc;
    HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(hc), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    free_list(t, t->scratch);  // the build has completed: scratch blocks are idle
    if (hc.err) {
        *retry = true;
        free_list(t, t->allocs);
        t->row_ids = nullptr;
    }
    return HJ_OK;
}

hj_status run_multi_build_entry(hj_table* t, const std::vector<Segment>& segs, const std::vector<HostSeg*>& hsegs);

// build attempts until no chunk overflows (halving the load factor each time)
hj_status build_attempts(hj_table* t, const std::vector<Segment>& segs) {
    double lf = load_factor();
    for (int attempt = 0;; ++attempt) {
        bool retry = false;
        hj_status st = build_attempt(t, segs, lf, &retry);
        if (st != HJ_OK) return st;
        if (!retry) return HJ_OK;
        // a chunk overflowed (adversarial key distribution): halve the load and rebuild
        if (attempt >= 4) return fail(HJ_ERR_INVALID, "build: a table chunk overflowed at every load factor");
        lf *= 0.5;
        HIP_TRY(hipEventRecord(t->res.ev0, t->bstream));
    }
}

// The geometry of a speculative build (build_attempt): the key range from the mailbox.
// When it takes the dense frag layout the kernels have built the table; otherwise they
// wrote nothing, and the table is built here in its layout (the range now known), on the
// build stream, with ev1 recorded again after it.
hj_status ensure_geometry(const hj_table* ct) {
    hj_table* t = const_cast<hj_table*>(ct);
    // settled: by the build, or by another caller (whose build may have failed)
    auto settled = [t]() { return t->build_st == HJ_OK ? HJ_OK : fail(t->build_st, t->build_err); };
    if (!t->spec_pending.load(std::memory_order_acquire)) return settled();
    std::lock_guard<std::mutex> g(t->spec_mu);
    if (!t->spec_pending.load(std::memory_order_relaxed)) return settled();
    HIP_TRY(hipSetDevice(t->device));
    int64_t* mb = t->res.h_minmax;
    HIP_TRY(wait_mailbox(mb, t->spec_seq, t->spec_mm, t->bstream));
    const int64_t mn = mb[0], mx = mb[1];
    if (spec_dense_blocks(mn, mx, (uint64_t)t->total_rows, t->spec_cap) != 0) {
        const uint64_t range = (uint64_t)mx - (uint64_t)mn + 1;
        t->dmin = mn;
        t->drange = range;
        t->nchunks = (uint32_t)((range + (1u << kDenseShift) - 1) >> kDenseShift);
        t->spec_pending.store(false, std::memory_order_release);
        return HJ_OK;
    }
    // another layout: drain the (idle) speculative kernels, release their blocks, build
    // (the build time then runs from here: ev0 again)
    HIP_TRY(hipStreamSynchronize(t->bstream));
    HIP_TRY(hipEventRecord(t->res.ev0, t->bstream));
    free_list(t, t->allocs);
    free_list(t, t->scratch);
    t->dense = nullptr;
    t->tbl = nullptr;
    t->dup_rows = nullptr;
    t->row_ids = nullptr;
    t->ctr = nullptr;
    t->mm_known = true;
    t->mm_lo = mn;
    t->mm_hi = mx;
    hj_status st = build_attempts(t, t->spec_segs);
    if (st == HJ_OK && hipEventRecord(t->res.ev1, t->bstream) != hipSuccess)
        st = fail(HJ_ERR_HIP, "hipEventRecord failed");
    t->build_ns = -1;
    if (st != HJ_OK) {  // the table is unusable from here on
        (void)hipStreamSynchronize(t->bstream);
        t->build_st = st;
        t->build_err = g_err;
    }
    // only now: a concurrent caller that saw the flag waits on spec_mu until the table
    // (and ev1) are complete; one that sees it clear reads the finished geometry
    t->spec_pending.store(false, std::memory_order_release);
    return st;
}

// The settler: a process-wide thread that settles speculative builds (ensure_geometry) as
// soon as their key range lands, instead of at the table's first use. A range that takes
// another layout (a hashed table: wide or sparse keys) is then rebuilt while the caller's
// previous probe still runs, not on the first probe's critical path.
// DFP_HJ_SETTLE=0 leaves the settle to the first use.
struct Settler {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<hj_table*> q;
    hj_table* busy = nullptr;
};
Settler& settler() {
    static Settler* s = [] {
        Settler* st = new Settler();  // never destroyed: its detached thread may outlive main
        std::thread([st] {
            for (;;) {
                hj_table* t;
                {
                    std::unique_lock<std::mutex> g(st->mu);
                    st->cv.wait(g, [st] { return !st->q.empty(); });
                    t = st->q.front();
                    st->q.pop_front();
                    st->busy = t;
                }
                (void)ensure_geometry(t);  // a failure is recorded on the table (build_st)
                {
                    std::lock_guard<std::mutex> g(st->mu);
                    st->busy = nullptr;
                }
                st->cv.notify_all();
            }
        }).detach();
        return st;
    }();
    return *s;
}
bool settler_on() {
    static const bool v = [] {
        const char* e = getenv("DFP_HJ_SETTLE");
        return !(e && e[0] == '0');
    }();
    return v;
}
void settler_enqueue(hj_table* t) {
    Settler& st = settler();
    {
        std::lock_guard<std::mutex> g(st.mu);
        st.q.push_back(t);
    }
    st.cv.notify_all();
}
// before a table is freed: out of the queue, and not being settled
void settler_forget(hj_table* t) {
    if (!settler_on()) return;
    Settler& st = settler();
    std::unique_lock<std::mutex> g(st.mu);
    for (auto it = st.q.begin(); it != st.q.end();)
        it = *it == t ? st.q.erase(it) : it + 1;
    st.cv.wait(g, [&st, t] { return st.busy != t; });
}

// The device build, run once by the last partition to arrive at the barrier.
hj_status run_build(hj_table* t) {
    HIP_TRY(hipSetDevice(t->device));
    // canonical numbering: partition 0's appends in order, then partition 1, ...
    std::vector<Segment> segs;
    std::vector<HostSeg*> hsegs;
    t->part_off.assign(t->parallelism, 0);
    int64_t row = 0;
    for (int p = 0; p < t->parallelism; ++p) {
        t->part_off[p] = row;
        for (auto& hs : t->parts[p]) {
            if (hs.n == 0) continue;
            segs.push_back(Segment{hs.keys, hs.valid, hs.voff, hs.ids, hs.n, row});
            hsegs.push_back(&hs);
            row += hs.n;
        }
    }
    t->total_rows = row;
    if (t->multi) return run_multi_build_entry(t, segs, hsegs);
    if (row > 0x7FFFFFF0ll) return fail(HJ_ERR_INVALID, "build side exceeds 2^31-16 rows on one device; shard it");
    if (t->has_ids && t->has_no_ids)
        return fail(HJ_ERR_INVALID, "explicit build ids must be given for every batch or none");
    t->bstream = t->app_streams == 1 ? t->app_stream : t->res.stream;
    hipStream_t s = t->bstream;
    // wait for the producers of borrowed device input
    for (int p = 0; p < t->parallelism; ++p)
        for (auto& hs : t->parts[p])
            if (hs.ready) HIP_TRY(hipStreamWaitEvent(s, hs.ready, 0));
    HIP_TRY(hipEventRecord(t->res.ev0, s));
    hj_status bst = build_attempts(t, segs);
    if (bst != HJ_OK) return bst;
    // ev1 marks the table complete: probes and queries on other streams wait on it
    // (hipStreamWaitEvent, no host synchronisation); build_ns is read when first asked
    HIP_TRY(hipEventRecord(t->res.ev1, s));
    t->build_ns = -1;
    if (t->has_base) {  // offsets from key_base -> the int64 keys they stand for
        if (t->dense != nullptr) t->dmin += t->key_base;
        t->kt = HJ_INT64;
        t->key_bytes = 8;
    }
    return HJ_OK;
}

// device build time, waiting for the build if it is still running
int64_t build_time_ns(hj_table* t) {
    if (t->build_ns < 0) {
        float ms = 0;
        if (hipEventSynchronize(t->res.ev1) != hipSuccess ||
            hipEventElapsedTime(&ms, t->ext_ev0 ? t->ext_ev0 : t->res.ev0, t->res.ev1) != hipSuccess)
            return -1;
        t->build_ns = (int64_t)(ms * 1e6);
    }
    return t->build_ns;
}

// make stream s wait for the table's build
hj_status wait_built(const hj_table* t, hipStream_t s) {
    if (s != t->bstream) HIP_TRY(hipStreamWaitEvent(s, t->res.ev1, 0));
    return HJ_OK;
}

hj_status check_table(const hj_table* t) {
    if (t == nullptr) return fail(HJ_ERR_INVALID, "null table");
    if (!t->built) return fail(HJ_ERR_INVALID, "table is not built: every partition must call hj_build_finish");
    if (t->build_st != HJ_OK) return fail(t->build_st, t->build_err);
    return ensure_geometry(t);
}

TableView view_of(const hj_table* t) {
    return TableView{t->tbl, t->dup_rows, t->row_ids, t->nb, t->clog2, t->dense, t->dmin, t->drange,
                     t->packed ? kPackedMask : kFullMask};
}

// device copy of host input (keys + validity bitmap slice)
struct TmpInput {
    void* keys = nullptr;
    uint8_t* valid = nullptr;
    hipStream_t s = nullptr;
    ~TmpInput() {
        if (keys) (void)hipFreeAsync(keys, s);
        if (valid) (void)hipFreeAsync(valid, s);
    }
};

hj_status stage_input(int key_bytes, const void* keys, const uint8_t* valid, int64_t voff, int64_t n, uint32_t flags,
                      hipStream_t s, TmpInput& tmp, const void** dkeys, const uint8_t** dvalid, int64_t* dvoff) {
    if (flags & HJ_INPUT_DEVICE) {
        if (!is_device_ptr(keys) || !is_device_ptr(valid))
            return fail(HJ_ERR_INVALID, "HJ_INPUT_DEVICE given but a pointer is not device memory");
        *dkeys = keys;
        *dvalid = valid;
        *dvoff = voff;
        return HJ_OK;
    }
    tmp.s = s;
    if (n > 0) {
        HIP_TRY(hipMallocAsync(&tmp.keys, (size_t)n * key_bytes, s));
        HIP_TRY(hipMemcpyAsync(tmp.keys, keys, (size_t)n * key_bytes, hipMemcpyDefault, s));
    }
    *dkeys = tmp.keys;
    *dvalid = nullptr;
    *dvoff = 0;
    if (valid && n > 0) {
        const int64_t b0 = voff >> 3;
        const int64_t nbytes = ((voff & 7) + n + 7) >> 3;
        HIP_TRY(hipMallocAsync((void**)&tmp.valid, (size_t)nbytes, s));
        HIP_TRY(hipMemcpyAsync(tmp.valid, valid + b0, (size_t)nbytes, hipMemcpyDefault, s));
        *dvalid = tmp.valid;
        *dvoff = voff & 7;
    }
    return HJ_OK;
}

// record the end of a probe on stream s (one event per probing stream, under the
// table's probe lock: probes of one table may run concurrently from several threads)
hj_status note_probe(const hj_table* t, hipStream_t s) {
    std::lock_guard<std::mutex> g(t->probe_mu);
    for (auto& se : t->probe_evs)
        if (se.first == s) {
            HIP_TRY(hipEventRecord(se.second, s));
            return HJ_OK;
        }
    hipEvent_t ev = t->res.evp;
    if (!t->probe_evs.empty()) HIP_TRY(hipEventCreateWithFlags(&ev, probe_ev_flags()));
    t->probe_evs.emplace_back(s, ev);
    HIP_TRY(hipEventRecord(ev, s));
    return HJ_OK;
}

// argument checks shared by the single- and multi-GPU probes (probe rows are numbered
// in u32: base + row, or the row inside a radix piece)
hj_status check_probe_args(int64_t n, uint32_t pbase, int64_t cap, const void* ws) {
    if (n < 0 || n > 0xFFFFFFFFll) return fail(HJ_ERR_INVALID, "probe batch must have < 2^32 rows");
    if ((int64_t)pbase + n > 0x100000000ll) return fail(HJ_ERR_INVALID, "probe_base + rows exceeds 2^32");
    if (cap < 0) return fail(HJ_ERR_INVALID, "negative capacity");
    if (reinterpret_cast<uintptr_t>(ws) & 7) return fail(HJ_ERR_INVALID, "workspace must be 8-byte aligned");
    return HJ_OK;
}

hj_status probe_impl(const hj_table* t, const void* keys, const uint8_t* valid, int64_t voff,
                     const uint32_t* probe_ids, uint32_t pbase, int64_t n, uint64_t* out_b, uint32_t* out_p,
                     int64_t cap, int64_t* d_total, void* ws, hipStream_t s) {
    hj_status st = check_probe_args(n, pbase, cap, ws);
    if (st == HJ_OK) st = ensure_geometry(t);
    if (st != HJ_OK) return st;
    // the probe orders itself after the build (on another stream) at its first table read
    HIP_TRY(launch_probe(t->key_bytes, view_of(t), keys, valid, voff, probe_ids, pbase, n, out_b, out_p, cap, d_total, ws,
                         s != t->bstream ? t->res.ev1 : nullptr, s));
    // hj_table_free waits for it before the table's blocks return to the cache
    return note_probe(t, s);
}

}  // namespace

// ---- multi-GPU table (hj_build_begin_multi): one process drives several GPUs --------
//
// The reference runs its join in one process over `parallelism` partitions; the drop-in
// for a node of GPUs is a table whose shards live on several devices behind the same
// build / probe / pairs ABI (SURVEY.md §8b "hj_build_begin_multi"). Two plans (§8e):
//   broadcast  every GPU builds the whole build side (its rows copied over xGMI); a
//              probe batch is split into contiguous row ranges, one per GPU, and their
//              pairs are concatenated: canonical order with no merge. Cheaper whenever
//              B·G < B + P (C2: 8·10^7 < 1.1·10^8).
//   radix      the build side is sharded by key hash (the low bits of mix64, the
//              multi-GPU partition kernel's map; the reference's precedent is the shard
//              function of src/utils/partitioned_concurrent_self_hash_join_map.rs:13-16):
//              shard g builds only its keys, with the rows' global canonical ids; a probe
//              batch is partitioned the same way, each piece probed by its owner, and the
//              pieces' pairs merged back into canonical order (every probe row's pairs
//              come from one shard). Needed once the build side outgrows one GPU.
// Shard tables are ordinary single-device tables; the exchange is device-to-device copies
// (peer access over xGMI), no collective. A multi table's probes are synchronous (the
// host reads the pieces' sizes).
struct MultiTable {
    int plan = HJ_MULTI_AUTO;
    std::vector<int> devices;
    std::vector<hj_table*> shards;
    std::vector<hipStream_t> streams;          // one per shard, on its device
    std::mutex probe_mu;                       // a multi probe uses the shard streams
    int64_t total_rows = 0;
    ~MultiTable() {
        for (size_t g = 0; g < shards.size(); ++g) hj_table_free(shards[g]);
        for (size_t g = 0; g < streams.size(); ++g) {
            (void)hipSetDevice(devices[g]);
            (void)hipStreamDestroy(streams[g]);
        }
    }
};

namespace {

int ptr_device(const void* p, int dflt) {
    hipPointerAttribute_t a;
    if (p == nullptr || hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return dflt;
    }
    return (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) ? a.device : dflt;
}

// device buffers of one multi operation, returned to the cache at scope exit. Before
// that, every stream that may still use them is drained — on the success path they are
// idle already; on an error return, earlier shards' copies, partitions, builds or probes
// may still be queued, and a block handed back to the cache could be reused under them.
void drain_multi(const MultiTable* m);
struct TmpBufs {
    std::vector<std::tuple<int, void*, size_t>> v;
    const MultiTable* m = nullptr;                      // its shard streams and builds
    std::vector<std::pair<int, hipStream_t>> streams;  // other streams that used the blocks
    ~TmpBufs() {
        if (m != nullptr) drain_multi(m);
        for (auto& ds : streams) {
            (void)hipSetDevice(ds.first);
            (void)hipStreamSynchronize(ds.second);
        }
        for (auto& b : v) cache_free(std::get<0>(b), std::get<1>(b), std::get<2>(b));
    }
    void* get(int dev, size_t bytes) {
        hipError_t e;
        (void)hipSetDevice(dev);
        void* p = cache_alloc(dev, bytes ? bytes : 64, &e);
        if (p) v.emplace_back(dev, p, bytes ? bytes : 64);
        return p;
    }
};

#define MT_ALLOC(var, type, dev, bytes)                                                   \
    type var = (type)tmp.get((dev), (bytes));                                             \
    if (var == nullptr) return fail(HJ_ERR_OOM, "multi-GPU table: device allocation failed")

hj_status sync_streams(const MultiTable* m) {
    for (size_t g = 0; g < m->streams.size(); ++g) {
        HIP_TRY(hipSetDevice(m->devices[g]));
        HIP_TRY(hipStreamSynchronize(m->streams[g]));
    }
    return HJ_OK;
}

// error-path drain (TmpBufs): the shard streams, and every shard build that was enqueued
// (an empty shard builds on its own resource stream)
void drain_multi(const MultiTable* m) {
    for (size_t g = 0; g < m->streams.size(); ++g) {
        (void)hipSetDevice(m->devices[g]);
        (void)hipStreamSynchronize(m->streams[g]);
    }
    for (const hj_table* sh : m->shards)
        if (sh != nullptr && sh->built && sh->build_st == HJ_OK) {
            (void)hipSetDevice(sh->device);
            (void)hipEventSynchronize(sh->res.ev1);
        }
}

// DFP_HJ_MULTI_STAGE=1: treat every shard's device as foreign, so that the staging
// copies (keys, validity re-based at voff & 7, ids) run even when all shards share one
// GPU (tests of the cross-device branches on a one-GPU box)
bool force_stage() {
    const char* e = getenv("DFP_HJ_MULTI_STAGE");
    return e != nullptr && e[0] == '1';
}

// owner shard of a key under the radix plan (hj_partition_rows' hash map, G a power of two)
int owner_of(int64_t key, int G) { return (int)(mix64((uint64_t)key) & (uint64_t)(G - 1)); }

// copy `bytes` from src (on any device) to dst on device `dev`, ordered on stream s
hipError_t copy_to(void* dst, const void* src, size_t bytes, hipStream_t s) {
    return bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s) : hipSuccess;
}

hj_status run_multi_build(hj_table* t, const std::vector<Segment>& segs, const std::vector<HostSeg*>& hsegs) {
    MultiTable* m = t->multi;
    const int G = (int)m->devices.size();
    const int kb = t->key_bytes;
    const int64_t total = t->total_rows;
    if (m->plan == HJ_MULTI_AUTO)  // replicate build sides that fit comfortably on every GPU
        m->plan = (total <= ((int64_t)1 << 27) || (G & (G - 1)) != 0) ? HJ_MULTI_BROADCAST : HJ_MULTI_RADIX;
    m->total_rows = total;
    if (t->has_ids && t->has_no_ids) return fail(HJ_ERR_INVALID, "explicit build ids must be given for every batch or none");
    hj_status st;
    m->shards.assign(G, nullptr);
    for (int g = 0; g < G; ++g) {
        if ((st = hj_build_begin(m->devices[g], 1, t->kt, 0, &m->shards[g])) != HJ_OK) return st;
        if (t->has_range && (st = hj_build_key_range(m->shards[g], t->range_lo, t->range_hi)) != HJ_OK) return st;
    }
    TmpBufs tmp;
    tmp.m = m;
    const uint32_t keep = HJ_INPUT_DEVICE | HJ_BORROW | HJ_BORROW_KEEP;
    // fault injection for the error-path tests: fail before shard `inject` builds, after
    // the earlier shards' builds were enqueued
    const char* inj = getenv("DFP_HJ_INJECT_SHARD_FAIL");
    const int inject = inj ? atoi(inj) : -1;
    if (m->plan == HJ_MULTI_BROADCAST) {
        // every shard appends every segment in canonical order (its rows keep their
        // canonical numbers, or the caller's ids)
        for (int g = 0; g < G; ++g) {
            const int dev = m->devices[g];
            hipStream_t s = m->streams[g];
            HIP_TRY(hipSetDevice(dev));
            for (size_t i = 0; i < segs.size(); ++i) {
                const Segment& sg = segs[i];
                if (hsegs[i]->ready) HIP_TRY(hipStreamWaitEvent(s, hsegs[i]->ready, 0));
                const void* k = sg.keys;
                const uint8_t* v = sg.valid;
                const uint64_t* ids = sg.ids;
                if (force_stage() || ptr_device(sg.keys, t->device) != dev) {  // over xGMI into this GPU's HBM
                    MT_ALLOC(kd, void*, dev, (size_t)sg.n * kb);
                    HIP_TRY(copy_to(kd, sg.keys, (size_t)sg.n * kb, s));
                    k = kd;
                    if (sg.valid) {
                        const size_t nbytes = (size_t)(((sg.voff & 7) + sg.n + 7) >> 3);
                        MT_ALLOC(vd, uint8_t*, dev, nbytes);
                        HIP_TRY(copy_to(vd, sg.valid + (sg.voff >> 3), nbytes, s));
                        v = vd;
                    }
                    if (sg.ids) {
                        MT_ALLOC(id, uint64_t*, dev, (size_t)sg.n * 8);
                        HIP_TRY(copy_to(id, sg.ids, (size_t)sg.n * 8, s));
                        ids = id;
                    }
                }
                const int64_t voff = (v == sg.valid) ? sg.voff : (sg.voff & 7);
                if ((st = hj_build_append(m->shards[g], 0, k, v, voff, ids, sg.n,
                                          keep | (ids && t->ids_u31 ? HJ_IDS_U31 : 0), s)) != HJ_OK)
                    return st;
            }
            if (g == inject) return fail(HJ_ERR_HIP, "injected shard failure (DFP_HJ_INJECT_SHARD_FAIL)");
            if ((st = hj_build_finish(m->shards[g], 0)) != HJ_OK) return st;
        }
        // the shards hold borrowed copies: keep them with the table
        st = sync_streams(m);
        if (st != HJ_OK) return st;
        for (auto& b : tmp.v) t->multi_bufs.push_back(b);
        tmp.v.clear();
        return HJ_OK;
    }
    // radix: partition every segment on its device by owner shard (stable; global ids)
    struct Piece {
        int dev;
        void* keys;
        uint64_t* ids;
        std::vector<void*> scratch;  // counts and partition workspace
        std::vector<int64_t> cnt;
    };
    std::vector<Piece> pcs(segs.size());
    for (size_t i = 0; i < segs.size(); ++i) {
        const Segment& sg = segs[i];
        Piece& pc = pcs[i];
        pc.dev = ptr_device(sg.keys, t->device);
        HIP_TRY(hipSetDevice(pc.dev));
        hipStream_t s = thread_stream(pc.dev);
        tmp.streams.emplace_back(pc.dev, s);
        if (hsegs[i]->ready) HIP_TRY(hipStreamWaitEvent(s, hsegs[i]->ready, 0));
        MT_ALLOC(ok, void*, pc.dev, (size_t)sg.n * kb);
        MT_ALLOC(oi, uint64_t*, pc.dev, (size_t)sg.n * 8);
        MT_ALLOC(cn, int64_t*, pc.dev, 8 * (size_t)G);
        MT_ALLOC(ws, void*, pc.dev, (size_t)hj_partition_workspace_bytes(sg.n, G));
        if ((st = hj_partition_rows(t->kt, sg.keys, sg.valid, sg.voff, sg.ids, (uint64_t)sg.row_base, sg.n, G, nullptr,
                                    ok, kb, 0, oi, 8, cn, ws, s)) != HJ_OK)
            return st;
        pc.keys = ok;
        pc.ids = oi;
        pc.scratch = {cn, ws};
        pc.cnt.assign(G, 0);
        HIP_TRY(hipMemcpyAsync(pc.cnt.data(), cn, 8 * (size_t)G, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    const bool u31 = t->has_ids ? t->ids_u31 : total < ((int64_t)1 << 31);
    for (int g = 0; g < G; ++g) {
        const int dev = m->devices[g];
        hipStream_t s = m->streams[g];
        HIP_TRY(hipSetDevice(dev));
        int64_t tot = 0;
        for (auto& pc : pcs) tot += pc.cnt[g];
        void* rk = nullptr;
        uint64_t* ri = nullptr;
        if (tot > 0) {
            rk = tmp.get(dev, (size_t)tot * kb);
            ri = (uint64_t*)tmp.get(dev, (size_t)tot * 8);
            if (!rk || !ri) return fail(HJ_ERR_OOM, "multi-GPU table: device allocation failed");
        }
        int64_t at = 0;
        for (auto& pc : pcs) {  // segment order: the ids ascend (stable partition)
            int64_t off = 0;
            for (int q = 0; q < g; ++q) off += pc.cnt[q];
            const int64_t c = pc.cnt[g];
            HIP_TRY(copy_to((char*)rk + at * kb, (const char*)pc.keys + off * kb, (size_t)c * kb, s));
            HIP_TRY(copy_to(ri + at, pc.ids + off, (size_t)c * 8, s));
            at += c;
        }
        if (tot > 0 && (st = hj_build_append(m->shards[g], 0, rk, nullptr, 0, ri, tot, keep | (u31 ? HJ_IDS_U31 : 0),
                                             s)) != HJ_OK)
            return st;
        if (g == inject) return fail(HJ_ERR_HIP, "injected shard failure (DFP_HJ_INJECT_SHARD_FAIL)");
        if ((st = hj_build_finish(m->shards[g], 0)) != HJ_OK) return st;
    }
    if ((st = sync_streams(m)) != HJ_OK) return st;
    // keep the shards' borrowed receive buffers; the partition outputs, counts and
    // workspaces go back to the cache at scope exit
    std::vector<std::tuple<int, void*, size_t>> keep_bufs, drop;
    for (auto& b : tmp.v) {
        bool is_piece = false;
        for (auto& pc : pcs) {
            is_piece |= std::get<1>(b) == pc.keys || std::get<1>(b) == (void*)pc.ids;
            for (void* q : pc.scratch) is_piece |= std::get<1>(b) == q;
        }
        (is_piece ? drop : keep_bufs).push_back(b);
    }
    tmp.v = drop;
    for (auto& b : keep_bufs) t->multi_bufs.push_back(b);
    return HJ_OK;
}

// Probe of a multi table into caller buffers on the keys' device; synchronous.
hj_status multi_probe(const hj_table* t, const void* keys, const uint8_t* valid, int64_t voff,
                      const uint32_t* probe_ids, uint32_t pbase, int64_t n, uint64_t* out_b, uint32_t* out_p,
                      int64_t cap, int64_t* d_total, void* workspace, hipStream_t s) {
    {
        const hj_status cs = check_probe_args(n, pbase, cap, workspace);
        if (cs != HJ_OK) return cs;
    }
    MultiTable* m = t->multi;
    std::lock_guard<std::mutex> lk(m->probe_mu);
    const int G = (int)m->devices.size();
    const int kb = t->key_bytes;
    const int d = ptr_device(keys ? (const void*)keys : (const void*)out_b, t->device);
    TmpBufs tmp;
    tmp.m = m;
    tmp.streams.emplace_back(d, s);
    hj_status st;
    HIP_TRY(hipSetDevice(d));
    hipEvent_t ready;  // the caller's inputs are produced in stream s's order
    HIP_TRY(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    struct EvGuard {
        hipEvent_t e;
        ~EvGuard() { (void)hipEventDestroy(e); }
    } evg{ready};
    HIP_TRY(hipEventRecord(ready, s));
    struct Part {
        int64_t n = 0;
        uint64_t* ob = nullptr;
        uint32_t* op = nullptr;
        int64_t cap = 0;
        int64_t* dt = nullptr;
        int64_t total = 0;
        const void* k = nullptr;
        const uint8_t* v = nullptr;
        int64_t voff = 0;
        const uint32_t* ids = nullptr;
        uint32_t base = 0;  // probe_idx = base + row when ids is null
        void* ws = nullptr;
    };
    std::vector<Part> parts(G);
    // per shard: its rows on its device
    if (m->plan == HJ_MULTI_BROADCAST) {
        for (int g = 0; g < G; ++g) {
            const int dev = m->devices[g];
            hipStream_t sg = m->streams[g];
            Part& P = parts[g];
            const int64_t a = n * g / G, b = n * (g + 1) / G;
            P.n = b - a;
            HIP_TRY(hipSetDevice(dev));
            HIP_TRY(hipStreamWaitEvent(sg, ready, 0));
            if (dev == d && !force_stage()) {
                P.k = (const char*)keys + a * kb;
                P.v = valid;
                P.voff = voff + a;
            } else {
                MT_ALLOC(kd, void*, dev, (size_t)P.n * kb);
                HIP_TRY(copy_to(kd, (const char*)keys + a * kb, (size_t)P.n * kb, sg));
                P.k = kd;
                if (valid) {
                    const int64_t b0 = (voff + a) >> 3, b1 = (voff + b + 7) >> 3;
                    MT_ALLOC(vd, uint8_t*, dev, (size_t)(b1 - b0));
                    HIP_TRY(copy_to(vd, valid + b0, (size_t)(b1 - b0), sg));
                    P.v = vd;
                    P.voff = (voff + a) & 7;
                }
            }
            if (probe_ids) {
                MT_ALLOC(ids, uint32_t*, dev, 4 * (size_t)P.n);
                HIP_TRY(copy_to(ids, probe_ids + a, 4 * (size_t)P.n, sg));
                P.ids = ids;
            } else {
                P.base = pbase + (uint32_t)a;  // contiguous rows: no id array
            }
        }
    } else {
        // radix: partition the batch by owner on its device; the rows travel with their
        // row numbers (u32), the caller's ids are applied after the merge
        HIP_TRY(hipSetDevice(d));
        MT_ALLOC(ok, void*, d, (size_t)n * kb);
        MT_ALLOC(oi, uint32_t*, d, (size_t)n * 4);
        MT_ALLOC(cn, int64_t*, d, 8 * (size_t)G);
        MT_ALLOC(ws, void*, d, (size_t)hj_partition_workspace_bytes(n, G));
        if ((st = hj_partition_rows(t->kt, keys, valid, voff, nullptr, 0, n, G, nullptr, ok, kb, 0, oi, 4, cn, ws, s)) !=
            HJ_OK)
            return st;
        std::vector<int64_t> cnt(G);
        HIP_TRY(hipMemcpyAsync(cnt.data(), cn, 8 * (size_t)G, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        int64_t off = 0;
        for (int g = 0; g < G; ++g) {
            const int dev = m->devices[g];
            hipStream_t sg = m->streams[g];
            Part& P = parts[g];
            P.n = cnt[g];
            if (dev == d && !force_stage()) {  // a shard on the batch's device probes its region in place
                P.k = (const char*)ok + off * kb;
                P.ids = oi + off;
                off += P.n;
                continue;
            }
            HIP_TRY(hipSetDevice(dev));
            MT_ALLOC(kd, void*, dev, (size_t)P.n * kb);
            MT_ALLOC(id, uint32_t*, dev, (size_t)P.n * 4);
            HIP_TRY(copy_to(kd, (const char*)ok + off * kb, (size_t)P.n * kb, sg));
            HIP_TRY(copy_to(id, oi + off, (size_t)P.n * 4, sg));
            P.k = kd;
            P.ids = id;
            off += P.n;
        }
    }
    // probe every shard (capacity: its rows; once more at the exact size if exceeded)
    for (int pass = 0; pass < 2; ++pass) {
        bool again = false;
        for (int g = 0; g < G; ++g) {
            Part& P = parts[g];
            if (pass == 1 && P.total <= P.cap) continue;
            const int dev = m->devices[g];
            HIP_TRY(hipSetDevice(dev));
            P.cap = pass == 0 ? std::max<int64_t>(P.n, 1) : P.total;
            P.ob = (uint64_t*)tmp.get(dev, 8 * (size_t)P.cap);
            P.op = (uint32_t*)tmp.get(dev, 4 * (size_t)P.cap);
            if (!P.dt) P.dt = (int64_t*)tmp.get(dev, 8);
            if (!P.ws) P.ws = tmp.get(dev, (size_t)hj_probe_workspace_bytes(P.n));
            if (!P.ob || !P.op || !P.dt || !P.ws) return fail(HJ_ERR_OOM, "multi-GPU probe: device allocation failed");
            st = P.ids ? hj_probe_async_ids(m->shards[g], P.k, P.v, P.voff, P.ids, P.n, P.ob, P.op, P.cap, P.dt, P.ws,
                                            m->streams[g])
                       : hj_probe_async_base(m->shards[g], P.k, P.v, P.voff, P.n, P.base, P.ob, P.op, P.cap, P.dt,
                                             P.ws, m->streams[g]);
            if (st != HJ_OK) return st;
            HIP_TRY(hipMemcpyAsync(&P.total, P.dt, 8, hipMemcpyDeviceToHost, m->streams[g]));
            again = true;
        }
        if (!again) break;
        if ((st = sync_streams(m)) != HJ_OK) return st;
    }
    int64_t total = 0;
    unsigned long long err = 0;  // the shards' look-back error words, ORed into the caller's
    for (auto& P : parts) {
        total += P.total;
        unsigned long long e = 0;
        HIP_TRY(hipMemcpy(&e, (char*)P.ws + 8, 8, hipMemcpyDeviceToHost));
        err |= e;
    }
    HIP_TRY(hipSetDevice(d));
    if (workspace) HIP_TRY(hipMemcpyAsync((char*)workspace + 8, &err, 8, hipMemcpyHostToDevice, s));
    if (m->plan == HJ_MULTI_BROADCAST) {  // contiguous row ranges: concatenation is canonical
        int64_t at = 0;
        for (auto& P : parts) {
            const int64_t c = std::min<int64_t>(P.total, std::max<int64_t>(cap - at, 0));
            HIP_TRY(copy_to(out_b + at, P.ob, 8 * (size_t)c, s));
            HIP_TRY(copy_to(out_p + at, P.op, 4 * (size_t)c, s));
            at += P.total;
        }
    } else if (total > 0) {  // gather the pieces' pairs, then the canonical merge by probe row
        MT_ALLOC(cb, uint64_t*, d, 8 * (size_t)total);
        MT_ALLOC(cp, uint32_t*, d, 4 * (size_t)total);
        int64_t at = 0;
        for (auto& P : parts) {
            HIP_TRY(copy_to(cb + at, P.ob, 8 * (size_t)P.total, s));
            HIP_TRY(copy_to(cp + at, P.op, 4 * (size_t)P.total, s));
            at += P.total;
        }
        MT_ALLOC(mw, void*, d, (size_t)merge_pairs_workspace(n));
        HIP_TRY(launch_merge_pairs(cb, cp, total, n, out_b, out_p, cap, mw, s));
        if (probe_ids)  // row -> the caller's probe id, in place (each thread its own element)
            HIP_TRY(launch_gather_fixed(probe_ids, nullptr, 0, 4, out_p, 4, std::min(total, cap), out_p, nullptr, s));
        else if (pbase)  // row -> base + row
            HIP_TRY(launch_add_u32(out_p, std::min(total, cap), pbase, s));
    }
    HIP_TRY(hipMemcpyAsync(d_total, &total, 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));  // total lives on this frame; the scratch goes back to the cache
    return HJ_OK;
}

}  // namespace

namespace {
hj_status run_multi_build_entry(hj_table* t, const std::vector<Segment>& segs, const std::vector<HostSeg*>& hsegs) {
    return run_multi_build(t, segs, hsegs);
}
}  // namespace

extern "C" {

const char* hj_last_error(void) { return g_err.c_str(); }

const char* hj_version(void) { return "dfp-hj 0.2 (gfx950)"; }

int hj_device_count(void) { return device_count(); }

hj_status hj_build_begin(int device, int parallelism, hj_key_type key_type, int64_t expected_rows, hj_table** out) {
    (void)expected_rows;
    if (out == nullptr) return fail(HJ_ERR_INVALID, "null out");
    *out = nullptr;
    if (parallelism < 1) return fail(HJ_ERR_INVALID, "parallelism must be >= 1");
    if (key_type != HJ_INT32 && key_type != HJ_INT64) return fail(HJ_ERR_INVALID, "unsupported key type");
    const int nd = device_count();
    if (nd == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible: the HIP path cannot run (no CPU fallback)");
    if (device < 0 || device >= nd) return fail(HJ_ERR_INVALID, "bad device ordinal");
    HIP_TRY(hipSetDevice(device));
    hj_table* t = new hj_table();
    t->device = device;
    t->parallelism = parallelism;
    t->kt = key_type;
    t->key_bytes = key_type == HJ_INT64 ? 8 : 4;
    t->parts.resize(parallelism);
    t->finished.assign(parallelism, 0);
    if (!acquire_resources(device, &t->res)) {
        delete t;
        return fail(HJ_ERR_HIP, "stream/event creation failed");
    }
    // keep freed blocks in the pool: repeated builds re-use device memory
    static std::once_flag pool_once[64];
    if (device < 64)
        std::call_once(pool_once[device], [device] {
            hipMemPool_t pool;
            if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
                uint64_t thr = UINT64_MAX;
                (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
            }
        });
    *out = t;
    return HJ_OK;
}

hj_status hj_build_begin_multi(int ngpu, const int* devices, int parallelism, hj_key_type key_type,
                               int64_t expected_rows, int plan, hj_table** out) {
    if (out == nullptr) return fail(HJ_ERR_INVALID, "null out");
    *out = nullptr;
    if (ngpu < 1 || ngpu > 64 || devices == nullptr) return fail(HJ_ERR_INVALID, "ngpu must be 1..64 with a device list");
    if (plan != HJ_MULTI_AUTO && plan != HJ_MULTI_BROADCAST && plan != HJ_MULTI_RADIX)
        return fail(HJ_ERR_INVALID, "unknown multi-GPU plan");
    if (plan == HJ_MULTI_RADIX && (ngpu & (ngpu - 1)))
        return fail(HJ_ERR_INVALID, "the radix plan shards over a power-of-two number of GPUs");
    const int nd = device_count();
    if (nd == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible: the HIP path cannot run (no CPU fallback)");
    for (int g = 0; g < ngpu; ++g)
        if (devices[g] < 0 || devices[g] >= nd) return fail(HJ_ERR_INVALID, "bad device ordinal");
    hj_status st = hj_build_begin(devices[0], parallelism, key_type, expected_rows, out);
    if (st != HJ_OK) return st;
    hj_table* t = *out;
    MultiTable* m = new MultiTable();
    m->plan = plan;
    m->devices.assign(devices, devices + ngpu);
    for (int g = 0; g < ngpu; ++g) {
        hipStream_t s = nullptr;
        if (hipSetDevice(devices[g]) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
            delete m;
            hj_table_free(t);
            *out = nullptr;
            return fail(HJ_ERR_HIP, "multi-GPU table: stream creation failed");
        }
        m->streams.push_back(s);
        for (int q = 0; q < ngpu; ++q)  // xGMI peer access for the shards' copies (already on: fine)
            if (devices[q] != devices[g]) {
                (void)hipDeviceEnablePeerAccess(devices[q], 0);
                (void)hipGetLastError();
            }
    }
    (void)hipSetDevice(devices[0]);
    t->multi = m;
    return HJ_OK;
}

hj_status hj_build_append(hj_table* t, int partition, const void* keys, const uint8_t* validity,
                          int64_t validity_offset, const uint64_t* ids, int64_t n, uint32_t flags, void* stream) {
    if (t == nullptr) return fail(HJ_ERR_INVALID, "null table");
    if (partition < 0 || partition >= t->parallelism) return fail(HJ_ERR_INVALID, "bad partition");
    if (n < 0 || validity_offset < 0) return fail(HJ_ERR_INVALID, "negative length/offset");
    if (n > 0 && keys == nullptr) return fail(HJ_ERR_INVALID, "null keys");
    {
        std::lock_guard<std::mutex> g(t->mu);
        if (t->finished[partition])
            return fail(HJ_ERR_INVALID, "State already consumed for partition " + std::to_string(partition));
        if (n > 0) {
            if (ids) {
                t->has_ids = true;
                if (!(flags & HJ_IDS_U31)) t->ids_u31 = false;
            } else {
                t->has_no_ids = true;
            }
        }
    }
    HIP_TRY(hipSetDevice(t->device));
    HostSeg hs;
    hs.n = n;
    if (n == 0) return HJ_OK;
    {
        std::lock_guard<std::mutex> g(t->mu);
        if (t->app_streams == 0) {
            t->app_stream = (hipStream_t)stream;
            t->app_streams = 1;
        } else if (t->app_stream != (hipStream_t)stream) {
            t->app_streams = 2;
        }
    }
    // the producer's stream: the build waits for its work (borrow) or copies in its order
    hipStream_t s = (hipStream_t)stream;
    const bool dev_in = (flags & HJ_INPUT_DEVICE) != 0;
    if (dev_in && (!is_device_ptr(keys) || !is_device_ptr(validity) || !is_device_ptr(ids)))
        return fail(HJ_ERR_INVALID, "HJ_INPUT_DEVICE given but a pointer is not device memory");
    if (dev_in && (flags & HJ_BORROW)) {
        if (!(flags & HJ_BORROW_KEEP)) {
            std::lock_guard<std::mutex> g(t->mu);
            t->sync_finish = true;  // the caller may drop the buffer once hj_build_finish returns
        }
        HIP_TRY(hipEventCreateWithFlags(&hs.ready, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(hs.ready, s));
        hs.keys = keys;
        hs.valid = validity;
        hs.voff = validity_offset;
        hs.ids = ids;
    } else {
        // staged copies count toward the device budget
        const int64_t staged = n * t->key_bytes + (validity ? (((validity_offset & 7) + n + 7) >> 3) : 0) +
                               (ids ? n * 8 : 0);
        {
            std::lock_guard<std::mutex> g(t->mu);
            const int64_t budget = device_budget();
            if (budget > 0 && t->live_bytes + staged > budget)
                return fail(HJ_ERR_OOM, "device budget: staging this build input exceeds " + std::to_string(budget) +
                                            " bytes of one device (DFP_HJ_DEVICE_BUDGET_BYTES); shard the build");
            t->live_bytes += staged;
            t->peak_bytes = std::max(t->peak_bytes, t->live_bytes);
        }
        void* dk = nullptr;
        HIP_TRY(hipMalloc(&dk, (size_t)n * t->key_bytes));
        hs.owned.push_back(dk);
        HIP_TRY(hipMemcpyAsync(dk, keys, (size_t)n * t->key_bytes, hipMemcpyDefault, s));
        hs.keys = dk;
        if (validity) {
            const int64_t b0 = validity_offset >> 3;
            const int64_t nbytes = ((validity_offset & 7) + n + 7) >> 3;
            void* dv = nullptr;
            HIP_TRY(hipMalloc(&dv, (size_t)nbytes));
            hs.owned.push_back(dv);
            HIP_TRY(hipMemcpyAsync(dv, validity + b0, (size_t)nbytes, hipMemcpyDefault, s));
            hs.valid = (const uint8_t*)dv;
            hs.voff = validity_offset & 7;
        }
        if (ids) {
            void* di = nullptr;
            HIP_TRY(hipMalloc(&di, (size_t)n * 8));
            hs.owned.push_back(di);
            HIP_TRY(hipMemcpyAsync(di, ids, (size_t)n * 8, hipMemcpyDefault, s));
            hs.ids = (const uint64_t*)di;
        }
        HIP_TRY(hipStreamSynchronize(s));
    }
    std::lock_guard<std::mutex> g(t->mu);
    t->parts[partition].push_back(std::move(hs));
    return HJ_OK;
}

hj_status hj_build_finish(hj_table* t, int partition) {
    if (t == nullptr) return fail(HJ_ERR_INVALID, "null table");
    if (partition < 0 || partition >= t->parallelism) return fail(HJ_ERR_INVALID, "bad partition");
    std::unique_lock<std::mutex> g(t->mu);
    if (t->finished[partition])
        return fail(HJ_ERR_INVALID, "State already consumed for partition " + std::to_string(partition));
    t->finished[partition] = 1;
    t->arrived++;
    if (t->arrived == t->parallelism) {
        // last arriver finalises (InitializeLast::initialize_or_wait)
        hj_status st = run_build(t);
        // borrowed input (no HJ_BORROW_KEEP) must be read before this returns: a
        // speculative build's geometry is settled now (a build in another layout reads it)
        if (st == HJ_OK && t->sync_finish) st = ensure_geometry(t);
        // a failed build may have queued work on its stream before the error (ev1 is not
        // recorded then): drain it, so that hj_table_free returns idle blocks to the cache
        if (st != HJ_OK) (void)hipStreamSynchronize(t->bstream);
        if (st == HJ_OK && t->sync_finish && hipEventSynchronize(t->res.ev1) != hipSuccess)
            st = fail(HJ_ERR_HIP, "build failed on the device");
        t->build_st = st;
        t->build_err = st == HJ_OK ? "" : g_err;
        t->built = true;
        t->cv.notify_all();
        if (st == HJ_OK && t->spec_pending.load(std::memory_order_acquire) && settler_on()) settler_enqueue(t);
    } else {
        // a partition that never arrives would block the rest forever; like the
        // reference's "Possible deadlock" timeouts (src/utils/parallel_compaction_batch_list.rs:56-58)
        const char* e = getenv("DFP_HJ_BARRIER_TIMEOUT_S");
        const double secs = e ? atof(e) : 300.0;
        if (!t->cv.wait_for(g, std::chrono::duration<double>(secs), [t] { return t->built; }))
            return fail(HJ_ERR_INVALID, "Possible deadlock: partition " + std::to_string(partition) +
                                            " waited for the build barrier; every partition must call "
                                            "hj_build_finish concurrently");
    }
    if (t->build_st != HJ_OK) return fail(t->build_st, t->build_err);
    return HJ_OK;
}

hj_status hj_build_key_range(hj_table* t, int64_t key_lo, int64_t key_hi) {
    if (t == nullptr) return fail(HJ_ERR_INVALID, "null table");
    if (key_lo > key_hi) return fail(HJ_ERR_INVALID, "hj_build_key_range: key_lo > key_hi");
    if (t->key_bytes == 4 && (key_lo < INT32_MIN || key_hi > INT32_MAX))
        return fail(HJ_ERR_INVALID, "hj_build_key_range: outside the int32 key domain");
    std::lock_guard<std::mutex> g(t->mu);
    if (t->built || t->arrived > 0) return fail(HJ_ERR_INVALID, "hj_build_key_range: after the barrier started");
    t->has_range = true;
    t->range_lo = key_lo;
    t->range_hi = key_hi;
    return HJ_OK;
}

hj_status hj_build_dense(hj_table* t) {
    if (t == nullptr) return fail(HJ_ERR_INVALID, "null table");
    if (t->multi != nullptr) return fail(HJ_ERR_INVALID, "hj_build_dense: not for a multi-GPU table");
    std::lock_guard<std::mutex> g(t->mu);
    if (t->built || t->arrived > 0) return fail(HJ_ERR_INVALID, "hj_build_dense: after the barrier started");
    if (!t->has_range) return fail(HJ_ERR_INVALID, "hj_build_dense: needs hj_build_key_range first");
    if ((uint64_t)t->range_hi - (uint64_t)t->range_lo >= ((uint64_t)kMaxChunks << kDenseShift))
        return fail(HJ_ERR_INVALID, "hj_build_dense: key range beyond the direct-addressed layout");
    t->force_dense = true;
    return HJ_OK;
}

hj_status hj_build_key_base(hj_table* t, int64_t key_base) {
    if (t == nullptr) return fail(HJ_ERR_INVALID, "null table");
    if (t->multi != nullptr) return fail(HJ_ERR_INVALID, "hj_build_key_base: not for a multi-GPU table");
    if (t->kt != HJ_INT32) return fail(HJ_ERR_INVALID, "hj_build_key_base: the build keys must be int32 offsets");
    std::lock_guard<std::mutex> g(t->mu);
    if (t->built || t->arrived > 0) return fail(HJ_ERR_INVALID, "hj_build_key_base: after the barrier started");
    t->has_base = true;
    t->key_base = key_base;
    return HJ_OK;
}

hj_status hj_table_dense_piece(const hj_table* t, uint32_t** refs, uint64_t* nvalues, int64_t* key_min,
                               uint32_t** dup_rows, const uint64_t** dup_used, int* packed) {
    hj_status st = check_table(t);
    if (st != HJ_OK) return st;
    if (!refs || !nvalues || !key_min || !dup_rows || !dup_used || !packed) return fail(HJ_ERR_INVALID, "null out");
    if (t->multi != nullptr || t->dense == nullptr || t->ctr == nullptr || t->wrapped)
        return fail(HJ_ERR_INVALID, "hj_table_dense_piece: not a built direct-addressed single-device table");
    *refs = t->dense;
    *nvalues = t->drange;
    *key_min = t->dmin;
    *dup_rows = t->dup_rows;
    *dup_used = reinterpret_cast<const uint64_t*>(&t->ctr->dup_used);
    *packed = t->packed ? 1 : 0;
    return HJ_OK;
}

hj_status hj_table_dense_export(const hj_table* t, uint32_t* refs_dst, uint64_t v0, uint64_t n, uint32_t* dup_dst,
                                uint64_t dup_n, uint64_t* dup_used_dst, void* stream) {
    hj_status st = check_table(t);
    if (st != HJ_OK) return st;
    if (t->multi != nullptr || t->dense == nullptr || t->ctr == nullptr || t->wrapped)
        return fail(HJ_ERR_INVALID, "hj_table_dense_export: not a built direct-addressed single-device table");
    if (refs_dst != nullptr && (v0 > t->drange || n > t->drange - v0))
        return fail(HJ_ERR_INVALID, "hj_table_dense_export: refs range past the table's key range");
    if (dup_dst != nullptr && dup_n > (uint64_t)(2 * t->total_rows + 2))
        return fail(HJ_ERR_INVALID, "hj_table_dense_export: more segment words than the table holds");
    HIP_TRY(hipSetDevice(t->device));
    hipStream_t s = (hipStream_t)stream;
    if (s != t->bstream) HIP_TRY(hipStreamWaitEvent(s, t->res.ev1, 0));  // after the build
    if (refs_dst != nullptr && n > 0)
        HIP_TRY(hipMemcpyAsync(refs_dst, t->dense + v0, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    if (dup_dst != nullptr && dup_n > 0)
        HIP_TRY(hipMemcpyAsync(dup_dst, t->dup_rows, dup_n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    if (dup_used_dst != nullptr)
        HIP_TRY(hipMemcpyAsync(dup_used_dst, &t->ctr->dup_used, sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
    return note_probe(t, s);  // hj_table_free waits for these reads too
}

hj_status hj_table_wrap_dense(int device, hj_key_type probe_key_type, int64_t key_min, uint64_t nvalues,
                              const uint32_t* refs, const uint32_t* dup_rows, int packed, void* stream,
                              hj_table** out) {
    if (out == nullptr) return fail(HJ_ERR_INVALID, "null out");
    *out = nullptr;
    if (probe_key_type != HJ_INT32 && probe_key_type != HJ_INT64) return fail(HJ_ERR_INVALID, "unsupported key type");
    if (refs == nullptr || dup_rows == nullptr || nvalues == 0)
        return fail(HJ_ERR_INVALID, "hj_table_wrap_dense: null arrays or an empty key range");
    if (nvalues > ((uint64_t)kMaxChunks << kDenseShift))
        return fail(HJ_ERR_INVALID, "hj_table_wrap_dense: key range beyond the direct-addressed layout");
    const int nd = device_count();
    if (nd == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible: the HIP path cannot run (no CPU fallback)");
    if (device < 0 || device >= nd) return fail(HJ_ERR_INVALID, "bad device ordinal");
    HIP_TRY(hipSetDevice(device));
    hj_table* t = new hj_table();
    t->device = device;
    t->kt = probe_key_type;
    t->key_bytes = probe_key_type == HJ_INT64 ? 8 : 4;
    t->parts.resize(1);
    t->finished.assign(1, 1);
    t->arrived = 1;
    if (!acquire_resources(device, &t->res)) {
        delete t;
        return fail(HJ_ERR_HIP, "stream/event creation failed");
    }
    t->wrapped = true;
    t->dense = const_cast<uint32_t*>(refs);
    t->dup_rows = const_cast<uint32_t*>(dup_rows);
    t->dmin = key_min;
    t->drange = nvalues;
    t->packed = packed != 0;
    t->bstream = (hipStream_t)stream;
    // the arrays are ready at this point of `stream`: probes elsewhere wait for it
    if (hipEventRecord(t->res.ev0, t->bstream) != hipSuccess || hipEventRecord(t->res.ev1, t->bstream) != hipSuccess) {
        release_resources(device, t->res);
        delete t;
        return fail(HJ_ERR_HIP, "hipEventRecord failed");
    }
    t->built = true;
    *out = t;
    return HJ_OK;
}

hj_status hj_dense_rebase_dups(uint32_t* refs, uint64_t n, uint32_t base, int packed, void* stream) {
    if (n > 0 && refs == nullptr) return fail(HJ_ERR_INVALID, "null refs");
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    const uint32_t mask = packed ? kPackedMask : kFullMask;
    if (base > mask) return fail(HJ_ERR_INVALID, "hj_dense_rebase_dups: base beyond the offset field");
    HIP_TRY(launch_dense_rebase(refs, n, base, mask, (hipStream_t)stream));
    return HJ_OK;
}

hj_status hj_build_partition_offset(const hj_table* t, int partition, int64_t* out) {
    hj_status st = check_table(t);
    if (st != HJ_OK) return st;
    if (partition < 0 || partition >= t->parallelism || out == nullptr) return fail(HJ_ERR_INVALID, "bad args");
    *out = t->part_off[partition];
    return HJ_OK;
}

hj_status hj_table_stats_get(const hj_table* t, hj_table_stats* out) {
    hj_status st = check_table(t);
    if (st != HJ_OK) return st;
    if (out == nullptr) return fail(HJ_ERR_INVALID, "null out");
    if (t->multi) {  // broadcast: every shard holds the table; radix: the shards' sums
        const MultiTable* m = t->multi;
        memset(out, 0, sizeof(*out));
        for (size_t g = 0; g < m->shards.size(); ++g) {
            hj_table_stats s;
            if ((st = hj_table_stats_get(m->shards[g], &s)) != HJ_OK) return st;
            if (m->plan == HJ_MULTI_BROADCAST && g > 0) {
                out->build_ns = std::max(out->build_ns, s.build_ns);
                continue;
            }
            out->inserted_rows += s.inserted_rows;
            out->distinct_keys += s.distinct_keys;
            out->dup_keys += s.dup_keys;
            out->dup_rows += s.dup_rows;
            out->max_key_rows = std::max(out->max_key_rows, s.max_key_rows);
            out->buckets += s.buckets;
            out->table_bytes += s.table_bytes;
            out->build_ns = std::max(out->build_ns, s.build_ns);
        }
        out->build_rows = t->total_rows;
        return HJ_OK;
    }
    HIP_TRY(hipSetDevice(t->device));
    hipStream_t s = thread_stream(t->device);
    unsigned long long* d = nullptr;
    HIP_TRY(hipMallocAsync((void**)&d, 4 * sizeof(unsigned long long), s));
    HIP_TRY(hipMemsetAsync(d, 0, 4 * sizeof(unsigned long long), s));
    if (wait_built(t, s) != HJ_OK) return HJ_ERR_HIP;
    HIP_TRY(launch_table_stats(view_of(t), d, s));
    unsigned long long h[4];
    HIP_TRY(hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipFreeAsync(d, s));
    HIP_TRY(hipStreamSynchronize(s));
    out->build_rows = t->total_rows;
    out->distinct_keys = (int64_t)h[0];
    out->dup_keys = (int64_t)h[1];
    out->dup_rows = (int64_t)h[2];
    out->max_key_rows = (int64_t)h[3];
    out->inserted_rows = (int64_t)h[0] - (int64_t)h[1] + (int64_t)h[2];
    out->buckets = t->dense ? 0 : t->nb;
    out->table_bytes = t->dense ? (int64_t)sizeof(uint32_t) * ((int64_t)t->nchunks << kDenseShift)
                                : (int64_t)(t->nb + 1) * (int64_t)sizeof(Bucket);
    out->build_ns = build_time_ns(const_cast<hj_table*>(t));
    return HJ_OK;
}

int64_t hj_table_build_ns(const hj_table* t) {
    if (t == nullptr || !t->built || t->build_st != HJ_OK) return -1;
    if (t->multi == nullptr && ensure_geometry(t) != HJ_OK) return -1;  // a pending speculative build settles first
    if (t->multi) {
        int64_t ns = 0;
        for (hj_table* sh : t->multi->shards) ns = std::max(ns, hj_table_build_ns(sh));
        return ns;
    }
    return build_time_ns(const_cast<hj_table*>(t));
}

int64_t hj_probe_workspace_bytes(int64_t n) { return probe_workspace(n); }

int hj_set_build_mode(int mode) {
    if (mode < 0 || mode > 2) return -1;
    const int old = build_mode_raw();
    g_build_mode.store(mode, std::memory_order_relaxed);
    return old;
}

int64_t hj_set_device_budget(int64_t bytes) {
    const int64_t old = device_budget();
    g_budget.store(bytes < 0 ? 0 : bytes, std::memory_order_relaxed);
    return old;
}

hj_status hj_table_device_bytes(const hj_table* t, int64_t* peak_per_device) {
    if (t == nullptr || peak_per_device == nullptr) return fail(HJ_ERR_INVALID, "null table/out");
    if (t->multi) {  // the largest shard: each shard is one device's table
        int64_t mx = 0;
        for (const hj_table* sh : t->multi->shards)
            if (sh != nullptr) mx = std::max(mx, sh->peak_bytes);
        *peak_per_device = mx;
        return HJ_OK;
    }
    *peak_per_device = t->peak_bytes;
    return HJ_OK;
}

int hj_set_probe_mode(int mode) {
    if (mode != 0 && mode != 3 && mode != 4) return -1;  // 1 and 2 were retired strategies
    const int old = get_probe_mode();
    set_probe_mode(mode);
    return old;
}

int hj_set_probe_tile_log(int tile_log) {
    if (tile_log != 0 && tile_log != 14 && tile_log != 15) return -1;
    return set_probe_tile_log(tile_log);
}

hj_status hj_probe_async(const hj_table* t, const void* keys, const uint8_t* validity, int64_t validity_offset,
                         int64_t n, uint64_t* out_build, uint32_t* out_probe, int64_t capacity, int64_t* d_total,
                         void* workspace, void* stream) {
    hj_status st = check_table(t);
    if (st != HJ_OK) return st;
    if (d_total == nullptr || workspace == nullptr) return fail(HJ_ERR_INVALID, "null d_total/workspace");
    if (n > 0 && keys == nullptr) return fail(HJ_ERR_INVALID, "null keys");
    HIP_TRY(hipSetDevice(t->device));
    if (t->multi)
        return multi_probe(t, keys, validity, validity_offset, nullptr, 0, n, out_build, out_probe, capacity, d_total,
                           workspace, (hipStream_t)stream);
    return probe_impl(t, keys, validity, validity_offset, nullptr, 0, n, out_build, out_probe, capacity, d_total,
                      workspace, (hipStream_t)stream /* NULL = the null stream */);
}

hj_status hj_probe_async_base(const hj_table* t, const void* keys, const uint8_t* validity, int64_t validity_offset,
                              int64_t n, uint32_t probe_base, uint64_t* out_build, uint32_t* out_probe,
                              int64_t capacity, int64_t* d_total, void* workspace, void* stream) {
    hj_status st = check_table(t);
    if (st != HJ_OK) return st;
    if (d_total == nullptr || workspace == nullptr) return fail(HJ_ERR_INVALID, "null d_total/workspace");
    if (n > 0 && keys == nullptr) return fail(HJ_ERR_INVALID, "null keys");
    HIP_TRY(hipSetDevice(t->device));
    if (t->multi)
        return multi_probe(t, keys, validity, validity_offset, nullptr, probe_base, n, out_build, out_probe, capacity,
                           d_total, workspace, (hipStream_t)stream);
    return probe_impl(t, keys, validity, validity_offset, nullptr, probe_base, n, out_build, out_probe, capacity,
                      d_total, workspace, (hipStream_t)stream);
}

hj_status hj_probe_async_ids(const hj_table* t, const void* keys, const uint8_t* validity, int64_t validity_offset,
                             const uint32_t* probe_ids, int64_t n, uint64_t* out_build, uint32_t* out_probe,
                             int64_t capacity, int64_t* d_total, void* workspace, void* stream) {
    hj_status st = check_table(t);
    if (st != HJ_OK) return st;
    if (d_total == nullptr || workspace == nullptr) return fail(HJ_ERR_INVALID, "null d_total/workspace");
    HIP_TRY(hipSetDevice(t->device));
    if (t->multi)
        return multi_probe(t, keys, validity, validity_offset, probe_ids, 0, n, out_build, out_probe, capacity,
                           d_total, workspace, (hipStream_t)stream);
    return probe_impl(t, keys, validity, validity_offset, probe_ids, 0, n, out_build, out_probe, capacity, d_total,
                      workspace, (hipStream_t)stream /* NULL = the null stream */);
}

hj_status hj_probe(const hj_table* t, const void* keys, const uint8_t* validity, int64_t validity_offset, int64_t n,
                   uint32_t flags, void* stream, hj_pairs* out) {
    hj_status st = check_table(t);
    if (st != HJ_OK) return st;
    if (out == nullptr) return fail(HJ_ERR_INVALID, "null out");
    memset(out, 0, sizeof(*out));
    if (n < 0) return fail(HJ_ERR_INVALID, "negative length");
    if (n > 0 && keys == nullptr) return fail(HJ_ERR_INVALID, "null keys");
    HIP_TRY(hipSetDevice(t->device));
    hipStream_t s = (hipStream_t)stream;  // NULL = null stream
    TmpInput tmp;
    const void* dk;
    const uint8_t* dv;
    int64_t dvo;
    if ((st = stage_input(t->key_bytes, keys, validity, validity_offset, n, flags, s, tmp, &dk, &dv, &dvo)) != HJ_OK)
        return st;
    void* ws = nullptr;
    int64_t* d_total = nullptr;
    HIP_TRY(hipMallocAsync(&ws, (size_t)hj_probe_workspace_bytes(n), s));
    HIP_TRY(hipMallocAsync((void**)&d_total, sizeof(int64_t), s));
    int64_t cap = std::max<int64_t>(n, 1);
    uint64_t* ob = nullptr;
    uint32_t* op = nullptr;
    int64_t total = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        HIP_TRY(hipMalloc((void**)&ob, (size_t)cap * 8));
        HIP_TRY(hipMalloc((void**)&op, (size_t)cap * 4));
        if (t->multi) st = multi_probe(t, dk, dv, dvo, nullptr, 0, n, ob, op, cap, d_total, ws, s);
        else st = probe_impl(t, dk, dv, dvo, nullptr, 0, n, ob, op, cap, d_total, ws, s);
        if (st != HJ_OK) break;
        uint64_t werr = 0;
        HIP_TRY(hipMemcpyAsync(&total, d_total, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(&werr, (char*)ws + 8, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (werr != 0) {
            st = fail(HJ_ERR_HIP, "probe: tile look-back gave up (results invalid)");
            break;
        }
        if (total <= cap) break;
        (void)hipFree(ob);
        (void)hipFree(op);
        ob = nullptr;
        op = nullptr;
        cap = total;
    }
    (void)hipFreeAsync(ws, s);
    (void)hipFreeAsync(d_total, s);
    if (st != HJ_OK) {
        if (ob) (void)hipFree(ob);
        if (op) (void)hipFree(op);
        (void)hipStreamSynchronize(s);
        return st;
    }
    out->count = total;
    if (flags & HJ_OUTPUT_HOST) {
        out->build_idx = (uint64_t*)malloc((size_t)std::max<int64_t>(total, 1) * 8);
        out->probe_idx = (uint32_t*)malloc((size_t)std::max<int64_t>(total, 1) * 4);
        if (!out->build_idx || !out->probe_idx) {
            free(out->build_idx);
            free(out->probe_idx);
            (void)hipFree(ob);
            (void)hipFree(op);
            return fail(HJ_ERR_OOM, "host allocation failed");
        }
        if (total > 0) {
            HIP_TRY(hipMemcpyAsync(out->build_idx, ob, (size_t)total * 8, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(out->probe_idx, op, (size_t)total * 4, hipMemcpyDeviceToHost, s));
        }
        HIP_TRY(hipStreamSynchronize(s));
        (void)hipFree(ob);
        (void)hipFree(op);
        out->device_resident = 0;
    } else {
        HIP_TRY(hipStreamSynchronize(s));
        out->build_idx = ob;
        out->probe_idx = op;
        out->device_resident = 1;
    }
    return HJ_OK;
}

void hj_pairs_free(hj_pairs* p) {
    if (p == nullptr) return;
    if (p->device_resident) {
        if (p->build_idx) (void)hipFree(p->build_idx);
        if (p->probe_idx) (void)hipFree(p->probe_idx);
    } else {
        free(p->build_idx);
        free(p->probe_idx);
    }
    memset(p, 0, sizeof(*p));
}

hj_status hj_table_lookup(const hj_table* t, int64_t key, uint64_t* rows, int64_t cap, int64_t* count) {
    hj_status st = check_table(t);
    if (st != HJ_OK) return st;
    if (count == nullptr || (cap > 0 && rows == nullptr)) return fail(HJ_ERR_INVALID, "bad args");
    hj_pairs pr;
    int32_t k32 = (int32_t)key;
    if (t->kt == HJ_INT32 && (int64_t)k32 != key) {  // cannot be present
        *count = 0;
        return HJ_OK;
    }
    const void* kp = t->kt == HJ_INT64 ? (const void*)&key : (const void*)&k32;
    if ((st = hj_probe(t, kp, nullptr, 0, 1, HJ_OUTPUT_HOST, thread_stream(t->device), &pr)) != HJ_OK) return st;
    *count = pr.count;
    for (int64_t i = 0; i < std::min<int64_t>(cap, pr.count); ++i) rows[i] = pr.build_idx[i];
    hj_pairs_free(&pr);
    return HJ_OK;
}

hj_status hj_table_chain_links(const hj_table* t, int64_t* prev, int64_t n) {
    hj_status st = check_table(t);
    if (st != HJ_OK) return st;
    if (t->has_ids) return fail(HJ_ERR_INVALID, "chain links are defined for canonical row numbering (no explicit ids)");
    if (t->multi) return fail(HJ_ERR_INVALID, "chain links are not defined for a multi-GPU table");
    if (n != t->total_rows || (n > 0 && prev == nullptr))
        return fail(HJ_ERR_INVALID, "prev must hold build_rows entries");
    if (n == 0) return HJ_OK;
    HIP_TRY(hipSetDevice(t->device));
    hipStream_t s = thread_stream(t->device);
    int64_t* d = nullptr;
    HIP_TRY(hipMallocAsync((void**)&d, (size_t)n * 8, s));
    if (wait_built(t, s) != HJ_OK) return HJ_ERR_HIP;
    HIP_TRY(launch_chain_links(view_of(t), d, n, s));
    HIP_TRY(hipMemcpyAsync(prev, d, (size_t)n * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipFreeAsync(d, s));
    HIP_TRY(hipStreamSynchronize(s));
    return HJ_OK;
}

hj_status hj_table_stream_wait(const hj_table* t, void* stream) {
    hj_status st = check_table(t);
    if (st != HJ_OK) return st;
    if (t->multi) {
        for (hj_table* sh : t->multi->shards)
            if ((st = hj_table_stream_wait(sh, stream)) != HJ_OK) return st;
        return HJ_OK;
    }
    HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, t->res.ev1, 0));
    return HJ_OK;
}

void hj_table_free(hj_table* t) {
    if (t == nullptr) return;
    if (t->spec_seq != 0) settler_forget(t);
    (void)hipSetDevice(t->device);
    // the blocks return to the cache (reused by any stream): the build and the latest
    // probe must be done (earlier probes on other streams are the caller's to finish)
    if (t->built && t->build_st == HJ_OK) (void)hipEventSynchronize(t->res.ev1);
    for (auto& se : t->probe_evs) {
        (void)hipEventSynchronize(se.second);
        if (se.second != t->res.evp) (void)hipEventDestroy(se.second);
    }
    free_list(t, t->allocs);
    free_list(t, t->scratch);
    delete t->multi;  // its shards first: they borrow multi_bufs
    for (auto& b : t->multi_bufs) cache_free(std::get<0>(b), std::get<1>(b), std::get<2>(b));
    for (hj_table* o : t->owned_tables) hj_table_free(o);
    if (t->ext_ev0) (void)hipEventDestroy(t->ext_ev0);
    for (auto& part : t->parts)
        for (auto& hs : part) {
            for (void* p : hs.owned) (void)hipFree(p);
            if (hs.ready) (void)hipEventDestroy(hs.ready);
        }
    release_resources(t->device, t->res);
    delete t;
}

int64_t hj_partition_workspace_bytes(int64_t n, int nparts) { return radix_partition_workspace(n, nparts); }

hj_status hj_radix_partition(hj_key_type key_type, const void* keys, const uint8_t* validity, int64_t validity_offset,
                             const uint64_t* ids, uint64_t id_base, int64_t n, int nparts, void* out_keys,
                             int out_key_bytes, int64_t key_offset, void* out_ids, int id_bytes, int64_t* counts,
                             void* workspace, void* stream) {
    return hj_partition_rows(key_type, keys, validity, validity_offset, ids, id_base, n, nparts, nullptr, out_keys,
                             out_key_bytes, key_offset, out_ids, id_bytes, counts, workspace, stream);
}

namespace {
// shared argument checks of hj_partition_rows / hj_partition_regions -> the kernel's map
hj_status part_args(hj_key_type key_type, const void* keys, const uint8_t* validity, const uint64_t* ids,
                    uint64_t id_base, int64_t n, int nparts, const hj_part_spec* spec, const void* out_keys,
                    int out_key_bytes, int64_t key_offset, const void* out_ids, int id_bytes, const int64_t* counts,
                    const void* workspace, PartSpec* ps) {
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (nparts < 1 || nparts > 64 || (nparts & (nparts - 1)))
        return fail(HJ_ERR_INVALID, "nparts must be a power of two <= 64");
    if (n < 0) return fail(HJ_ERR_INVALID, "negative length");
    if (id_bytes != 4 && id_bytes != 8) return fail(HJ_ERR_INVALID, "id_bytes must be 4 or 8");
    if (key_type != HJ_INT32 && key_type != HJ_INT64) return fail(HJ_ERR_INVALID, "unsupported key type");
    const int kb = key_type == HJ_INT64 ? 8 : 4;
    if ((out_key_bytes != 4 && out_key_bytes != 8) || out_key_bytes > kb)
        return fail(HJ_ERR_INVALID, "out_key_bytes must be 4 or the key width");
    if (kb == 4 && key_offset != 0) return fail(HJ_ERR_INVALID, "key_offset applies to int64 keys");
    if (id_bytes == 4 && ids == nullptr && (uint64_t)id_base + (uint64_t)n > 0x100000000ull)
        return fail(HJ_ERR_INVALID, "32-bit ids overflow: id_base + n > 2^32");
    if (!is_device_ptr(keys) || !is_device_ptr(validity) || !is_device_ptr(ids) || !is_device_ptr(out_keys) ||
        !is_device_ptr(out_ids) || !is_device_ptr(counts) || !is_device_ptr(workspace))
        return fail(HJ_ERR_INVALID, "the partition takes device pointers");
    *ps = PartSpec{INT64_MIN, INT64_MAX, 0, 0};
    if (spec != nullptr) {
        if (spec->key_lo > spec->key_hi) return fail(HJ_ERR_INVALID, "hj_part_spec: key_lo > key_hi");
        ps->lo = spec->key_lo;
        ps->hi = spec->key_hi;
        ps->by_range = spec->by_range != 0;
        if (ps->by_range) {
            // mul = floor(2^64 * nparts / range), range = hi - lo + 1 in [1, 2^64]
            const unsigned __int128 range = (unsigned __int128)((uint64_t)ps->hi - (uint64_t)ps->lo) + 1;
            const unsigned __int128 m = ((unsigned __int128)nparts << 64) / range;
            ps->mul = m > (unsigned __int128)UINT64_MAX ? UINT64_MAX : (uint64_t)m;
        }
    }
    return HJ_OK;
}
}  // namespace

// workspace: [0, 24) the accumulators and ticket, [64, 64 + sizeof(Segment)) the segment, then the
// build counters the kernel zeroes (unused here), the partials from byte 256
int64_t hj_key_minmax_workspace_bytes(void) { return 256 + (2 + 2 * (int64_t)kMinmaxMaxBlocks) * 8; }

hj_status hj_key_minmax(hj_key_type key_type, const void* keys, const uint8_t* validity, int64_t validity_offset,
                        int64_t n, int64_t* out_minmax, void* workspace, void* stream) {
    static_assert(64 + sizeof(Segment) <= 128 && sizeof(BuildCounters) <= 128, "hj_key_minmax workspace layout");
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (key_type != HJ_INT32 && key_type != HJ_INT64) return fail(HJ_ERR_INVALID, "unknown key type");
    if (n < 0) return fail(HJ_ERR_INVALID, "negative n");
    if (out_minmax == nullptr || workspace == nullptr || (n > 0 && keys == nullptr))
        return fail(HJ_ERR_INVALID, "null pointer");
    if ((reinterpret_cast<uintptr_t>(workspace) & 7) != 0) return fail(HJ_ERR_INVALID, "workspace not 8-byte aligned");
    char* ws = static_cast<char*>(workspace);
    Segment sg{};
    sg.keys = keys;
    sg.valid = validity;
    sg.voff = validity_offset;
    sg.n = n;
    sg.row_base = 0;
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(ws, 0, 24, s));
    HIP_TRY(launch_key_minmax_one(key_type == HJ_INT64 ? 8 : 4, &sg, reinterpret_cast<Segment*>(ws + 64), 1,
                              reinterpret_cast<BuildCounters*>(ws + 128), n,
                              reinterpret_cast<int64_t*>(ws + 256), reinterpret_cast<unsigned long long*>(ws),
                              nullptr, 0, s, out_minmax));
    return HJ_OK;
}

int64_t hj_partition_regions_workspace_bytes(int64_t n, int nparts) {
    return radix_regions_workspace(n < 0 ? 0 : n, nparts < 1 ? 1 : nparts);
}

hj_status hj_partition_regions(hj_key_type key_type, const void* keys, const uint8_t* validity,
                               int64_t validity_offset, const uint64_t* ids, uint64_t id_base, int64_t n, int nparts,
                               const hj_part_spec* spec, void* out_keys, int out_key_bytes, int64_t key_offset,
                               void* out_ids, int id_bytes, int64_t region_rows, int64_t* counts, void* workspace,
                               void* stream) {
    PartSpec ps;
    hj_status st = part_args(key_type, keys, validity, ids, id_base, n, nparts, spec, out_keys, out_key_bytes,
                             key_offset, out_ids, id_bytes, counts, workspace, &ps);
    if (st != HJ_OK) return st;
    if (region_rows < 0) return fail(HJ_ERR_INVALID, "negative region_rows");
    if (n > 0 && (keys == nullptr || out_keys == nullptr || out_ids == nullptr || counts == nullptr ||
                  workspace == nullptr))
        return fail(HJ_ERR_INVALID, "null pointer");
    HIP_TRY(launch_radix_regions(key_type == HJ_INT64 ? 8 : 4, keys, validity, validity_offset, ids, id_base, n,
                                 nparts, ps, out_keys, out_key_bytes, key_offset, out_ids, id_bytes, region_rows,
                                 counts, workspace, (hipStream_t)stream));
    return HJ_OK;
}

hj_status hj_partition_rows(hj_key_type key_type, const void* keys, const uint8_t* validity, int64_t validity_offset,
                            const uint64_t* ids, uint64_t id_base, int64_t n, int nparts, const hj_part_spec* spec,
                            void* out_keys, int out_key_bytes, int64_t key_offset, void* out_ids, int id_bytes,
                            int64_t* counts, void* workspace, void* stream) {
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (nparts < 1 || nparts > 64 || (nparts & (nparts - 1)))
        return fail(HJ_ERR_INVALID, "nparts must be a power of two <= 64");
    if (n < 0) return fail(HJ_ERR_INVALID, "negative length");
    if (id_bytes != 4 && id_bytes != 8) return fail(HJ_ERR_INVALID, "id_bytes must be 4 or 8");
    const int kb = key_type == HJ_INT64 ? 8 : 4;
    if ((out_key_bytes != 4 && out_key_bytes != 8) || out_key_bytes > kb)
        return fail(HJ_ERR_INVALID, "out_key_bytes must be 4 or the key width");
    if (kb == 4 && key_offset != 0) return fail(HJ_ERR_INVALID, "key_offset applies to int64 keys");
    if (id_bytes == 4 && ids == nullptr && (uint64_t)id_base + (uint64_t)n > 0x100000000ull)
        return fail(HJ_ERR_INVALID, "32-bit ids overflow: id_base + n > 2^32");
    if (!is_device_ptr(keys) || !is_device_ptr(validity) || !is_device_ptr(ids) || !is_device_ptr(out_keys) ||
        !is_device_ptr(out_ids) || !is_device_ptr(counts) || !is_device_ptr(workspace))
        return fail(HJ_ERR_INVALID, "hj_partition_rows takes device pointers");
    PartSpec ps{INT64_MIN, INT64_MAX, 0, 0};
    if (spec != nullptr) {
        if (spec->key_lo > spec->key_hi) return fail(HJ_ERR_INVALID, "hj_part_spec: key_lo > key_hi");
        ps.lo = spec->key_lo;
        ps.hi = spec->key_hi;
        ps.by_range = spec->by_range != 0;
        if (ps.by_range) {
            // mul = floor(2^64 * nparts / range), range = hi - lo + 1 in [1, 2^64]
            const unsigned __int128 range = (unsigned __int128)((uint64_t)ps.hi - (uint64_t)ps.lo) + 1;
            const unsigned __int128 m = ((unsigned __int128)nparts << 64) / range;
            ps.mul = m > (unsigned __int128)UINT64_MAX ? UINT64_MAX : (uint64_t)m;
        }
    }
    HIP_TRY(launch_radix_partition(key_type == HJ_INT64 ? 8 : 4, keys, validity, validity_offset, ids, id_base, n,
                                   nparts, ps, out_keys, out_key_bytes, key_offset, out_ids, id_bytes, counts,
                                   workspace, (hipStream_t)stream));
    return HJ_OK;
}

// ---- composite keys (hj_keys.hip) --------------------------------------------------

namespace {
hj_status key_cols(int ncols, const hj_key_column* cols, KeyCols* out) {
    if (ncols < 1 || ncols > kMaxKeyCols) return fail(HJ_ERR_INVALID, "ncols must be 1..16");
    if (cols == nullptr) return fail(HJ_ERR_INVALID, "null key columns");
    out->n = ncols;
    for (int j = 0; j < ncols; ++j) {
        const hj_key_column& c = cols[j];
        const int w = c.width;
        if (!(w == 0 || w == 1 || w == 2 || w == 4 || w == 8 || w == 16))
            return fail(HJ_ERR_INVALID, "key column width must be 0 (variable), 1, 2, 4, 8 or 16");
        if (w == 0 && c.offset_bytes != 4 && c.offset_bytes != 8)
            return fail(HJ_ERR_INVALID, "variable-width key column: offset_bytes must be 4 or 8");
        if (c.values == nullptr || (w == 0 && c.offsets == nullptr))
            return fail(HJ_ERR_INVALID, "null key column buffer");
        if (c.validity_offset < 0) return fail(HJ_ERR_INVALID, "negative validity offset");
        if (!is_device_ptr(c.values) || !is_device_ptr(c.offsets) || !is_device_ptr(c.validity))
            return fail(HJ_ERR_INVALID, "key columns take device pointers");
        out->c[j] = KeyCol{c.values, c.offsets, c.validity, c.validity_offset, w, c.offset_bytes};
    }
    return HJ_OK;
}
}  // namespace

hj_status hj_composite_keys(int ncols, const hj_key_column* cols, int64_t n, int64_t* out_keys, uint8_t* out_valid,
                            void* stream) {
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (n < 0) return fail(HJ_ERR_INVALID, "negative length");
    KeyCols kc;
    hj_status st = key_cols(ncols, cols, &kc);
    if (st != HJ_OK) return st;
    if (n > 0 && (out_keys == nullptr || out_valid == nullptr)) return fail(HJ_ERR_INVALID, "null output");
    if (reinterpret_cast<uintptr_t>(out_valid) & 7) return fail(HJ_ERR_INVALID, "out_valid must be 8-byte aligned");
    if (!is_device_ptr(out_keys) || !is_device_ptr(out_valid))
        return fail(HJ_ERR_INVALID, "hj_composite_keys takes device pointers");
    HIP_TRY(launch_composite_keys(kc, n, out_keys, reinterpret_cast<uint64_t*>(out_valid), (hipStream_t)stream));
    return HJ_OK;
}

int64_t hj_equal_pairs_workspace_bytes(int64_t n) { return equal_pairs_workspace(n < 0 ? 0 : n); }

hj_status hj_filter_equal_pairs(int ncols, const hj_key_column* build_cols, const hj_key_column* probe_cols,
                                const uint64_t* build_idx, const uint32_t* probe_idx, int64_t n, uint64_t* out_build,
                                uint32_t* out_probe, int64_t* d_count, void* workspace, void* stream) {
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (n < 0) return fail(HJ_ERR_INVALID, "negative length");
    KeyCols bc, pc;
    hj_status st;
    if ((st = key_cols(ncols, build_cols, &bc)) != HJ_OK || (st = key_cols(ncols, probe_cols, &pc)) != HJ_OK) return st;
    for (int j = 0; j < ncols; ++j)
        if (bc.c[j].width != pc.c[j].width)
            return fail(HJ_ERR_INVALID, "build and probe key column " + std::to_string(j) + " differ in width");
    if (d_count == nullptr || workspace == nullptr ||
        (n > 0 && (build_idx == nullptr || probe_idx == nullptr || out_build == nullptr || out_probe == nullptr)))
        return fail(HJ_ERR_INVALID, "null pointer");
    if ((const void*)out_build == (const void*)build_idx || (const void*)out_probe == (const void*)probe_idx)
        return fail(HJ_ERR_INVALID, "outputs must not alias the candidate pairs");
    if (!is_device_ptr(build_idx) || !is_device_ptr(probe_idx) || !is_device_ptr(out_build) ||
        !is_device_ptr(out_probe) || !is_device_ptr(d_count) || !is_device_ptr(workspace))
        return fail(HJ_ERR_INVALID, "hj_filter_equal_pairs takes device pointers");
    HIP_TRY(launch_equal_pairs(bc, pc, build_idx, probe_idx, n, out_build, out_probe, d_count, workspace,
                               (hipStream_t)stream));
    return HJ_OK;
}

hj_status hj_gen_perm_keys(int64_t* out, int64_t n, int64_t mul, int64_t range, void* stream) {
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (range <= 0 || n < 0) return fail(HJ_ERR_INVALID, "bad range");
    HIP_TRY(launch_gen_perm(out, n, mul, range, (hipStream_t)stream));
    return HJ_OK;
}

hj_status hj_gen_uniform_keys(int64_t* out, int64_t n, uint64_t seed, int64_t range, void* stream) {
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (range <= 0 || n < 0) return fail(HJ_ERR_INVALID, "bad range");
    HIP_TRY(launch_gen_uniform(out, n, seed, range, (hipStream_t)stream));
    return HJ_OK;
}

// host buffer: src/api_utils.rs:15-23 in f32; f32::powf is libm powf, called through a
// volatile pointer so that it is neither folded nor vectorized (libmvec differs)
hj_status hj_gen_exponential_keys(int32_t* out, int32_t lo, int32_t hi) {
    if (hi < lo || (hi > lo && out == nullptr)) return fail(HJ_ERR_INVALID, "bad range");
    float (*volatile pw)(float, float) = powf;
    const int32_t diff = hi - lo;
    const float base = 16.0f;
    for (int32_t n = 0; n < diff; ++n) {
        const float x = (float)n / (float)diff;
        const float y = (pw(base, x) - 1.0f) / (base - 1.0f);
        out[n] = lo + (int32_t)(y * (float)diff);
    }
    return HJ_OK;
}


// ---- join types and output materialisation (hj_columns.hip) ---------------------

hj_status hj_mark_rows(const void* idx, int idx_bytes, int64_t n, uint8_t* flags, int64_t nflags, void* stream) {
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (n < 0 || nflags < 0 || (idx_bytes != 4 && idx_bytes != 8)) return fail(HJ_ERR_INVALID, "bad arguments");
    if ((n > 0 && idx == nullptr) || (nflags > 0 && flags == nullptr))
        return fail(HJ_ERR_INVALID, "null pointer");
    if (!is_device_ptr(idx) || !is_device_ptr(flags)) return fail(HJ_ERR_INVALID, "hj_mark_rows takes device pointers");
    HIP_TRY(launch_mark_rows(idx, idx_bytes, n, flags, nflags, (hipStream_t)stream));
    return HJ_OK;
}

int64_t hj_select_workspace_bytes(int64_t n) { return select_workspace(n < 0 ? 0 : n); }

hj_status hj_select_rows(const uint8_t* flags, int64_t n, int want, uint64_t* out, int64_t* d_count, void* workspace,
                         void* stream) {
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (n < 0 || want < 0 || want > 255) return fail(HJ_ERR_INVALID, "bad arguments");
    if (d_count == nullptr || workspace == nullptr || (n > 0 && (flags == nullptr || out == nullptr)))
        return fail(HJ_ERR_INVALID, "null pointer");
    if (!is_device_ptr(flags) || !is_device_ptr(out) || !is_device_ptr(d_count) || !is_device_ptr(workspace))
        return fail(HJ_ERR_INVALID, "hj_select_rows takes device pointers");
    HIP_TRY(launch_select_rows(flags, n, (uint8_t)want, out, d_count, workspace, (hipStream_t)stream));
    return HJ_OK;
}

hj_status hj_gather_fixed(const void* src, const uint8_t* src_valid, int64_t src_voff, int elem_bytes, const void* idx,
                          int idx_bytes, int64_t n, void* dst, uint8_t* dst_valid, void* stream) {
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (n < 0 || (idx_bytes != 4 && idx_bytes != 8) ||
        !(elem_bytes == 1 || elem_bytes == 2 || elem_bytes == 4 || elem_bytes == 8 || elem_bytes == 16))
        return fail(HJ_ERR_INVALID, "bad arguments (elem_bytes 1/2/4/8/16, idx_bytes 4/8)");
    if (n > 0 && (idx == nullptr || dst == nullptr)) return fail(HJ_ERR_INVALID, "null pointer");
    if (reinterpret_cast<uintptr_t>(dst_valid) & 7) return fail(HJ_ERR_INVALID, "dst_valid must be 8-byte aligned");
    if (!is_device_ptr(src) || !is_device_ptr(src_valid) || !is_device_ptr(idx) || !is_device_ptr(dst) ||
        !is_device_ptr(dst_valid))
        return fail(HJ_ERR_INVALID, "hj_gather_fixed takes device pointers");
    HIP_TRY(launch_gather_fixed(src, src_valid, src_voff, elem_bytes, idx, idx_bytes, n, dst, dst_valid,
                                (hipStream_t)stream));
    return HJ_OK;
}

int64_t hj_gather_var_workspace_bytes(int64_t n) { return gather_var_workspace(n < 0 ? 0 : n); }

hj_status hj_gather_var(const void* offsets, int offset_bytes, const uint8_t* values, const uint8_t* src_valid,
                        int64_t src_voff, const void* idx, int idx_bytes, int64_t n, void* out_offsets,
                        uint8_t* out_values, int64_t values_cap, uint8_t* dst_valid, int64_t* d_values_len,
                        void* workspace, void* stream) {
    if (device_count() == 0) return fail(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (n < 0 || values_cap < 0 || (idx_bytes != 4 && idx_bytes != 8) || (offset_bytes != 4 && offset_bytes != 8))
        return fail(HJ_ERR_INVALID, "bad arguments (offset_bytes 4/8, idx_bytes 4/8)");
    if (out_offsets == nullptr || d_values_len == nullptr || workspace == nullptr ||
        (n > 0 && (idx == nullptr || offsets == nullptr)))
        return fail(HJ_ERR_INVALID, "null pointer");
    if (reinterpret_cast<uintptr_t>(dst_valid) & 7) return fail(HJ_ERR_INVALID, "dst_valid must be 8-byte aligned");
    if (!is_device_ptr(offsets) || !is_device_ptr(values) || !is_device_ptr(src_valid) || !is_device_ptr(idx) ||
        !is_device_ptr(out_offsets) || !is_device_ptr(out_values) || !is_device_ptr(dst_valid) ||
        !is_device_ptr(d_values_len) || !is_device_ptr(workspace))
        return fail(HJ_ERR_INVALID, "hj_gather_var takes device pointers");
    HIP_TRY(launch_gather_var(offsets, offset_bytes, values, src_valid, src_voff, idx, idx_bytes, n, out_offsets,
                              out_values, values_cap, dst_valid, d_values_len, workspace, (hipStream_t)stream));
    return HJ_OK;
}

}  // extern "C"
