// hj_dist.cpp — RCCL behind the C ABI (include/hj.h, "multi-process"): the sharded-build
// plan's build side as one call per step, so that a host in any language (the Rust
// drop-in: one process per GPU) drives the multi-GPU join through hj_* calls alone.
//
// The plan is the one distributed.py's DistributedHashJoin.join_sharded runs over
// torch.distributed: a global key range, every build row to the rank that
// owns its contiguous key range (the reference's precedent for a shard function:
// src/utils/partitioned_concurrent_self_hash_join_map.rs:13-16), a direct-addressed
// build of each rank's range, and the pieces all-gathered into one table over the whole
// key domain that every rank probes with its own probe rows
// (src/operator/version10/parallel_join_execution_state.rs:405-407: one table shared by
// every partition). Every device step is enqueued on the caller's stream; RCCL runs its
// collectives there too (xGMI is point to point: the exchange is per-peer
// ncclSend/ncclRecv in one group, not an all-to-all).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <utility>
#include <vector>

#include "../../include/hj.h"
#include "hj_device.h"
#include "hj_host.h"
#include "hj_launch.h"

using namespace dfp;
using dfp::host::set_error;

namespace {

#define HIP_OK(expr)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return set_error(HJ_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)
#define NCCL_OK(expr)                                                                           \
    do {                                                                                        \
        ncclResult_t r_ = (expr);                                                               \
        if (r_ != ncclSuccess) return set_error(HJ_ERR_RCCL, std::string(#expr ": ") + ncclGetErrorString(r_)); \
    } while (0)
#define ST_OK(expr)                       \
    do {                                  \
        hj_status s_ = (expr);            \
        if (s_ != HJ_OK) return s_;       \
    } while (0)

// RCCL messages above this travel in pieces (RCCL 2.26 on ROCm 7 truncated single
// transfers near 763 MiB; the Python plans use the same bound)
constexpr size_t kMaxMsgBytes = size_t(256) << 20;
constexpr uint64_t kDenseMax = (uint64_t)kMaxChunks << kDenseShift;  // widest direct-addressed range
constexpr int64_t kHostWords = 8192;                                   // pinned mailbox (64 KiB)

}  // namespace

struct hj_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1, device = 0;
    int64_t* host = nullptr;   // pinned mailbox for the plan's small reads
    hipEvent_t ev = nullptr;   // marks a read's copy
    // scratch of earlier calls: released once their end event has fired
    struct Deferred {
        hipEvent_t done;
        std::vector<std::pair<void*, size_t>> blocks;
    };
    std::vector<Deferred> deferred;
};

namespace {

// the blocks of one call; on success they go to the communicator's deferred list behind the
// call's end event, on failure they are released after the stream drained
struct Scratch {
    hj_comm* c;
    hipStream_t s;
    std::vector<std::pair<void*, size_t>> blocks;
    bool handed_over = false;
    Scratch(hj_comm* c_, hipStream_t s_) : c(c_), s(s_) {}
    void* get(size_t bytes) {
        bytes = std::max<size_t>(bytes, 64);
        void* p = dfp::host::dev_block(c->device, bytes);
        if (p) blocks.emplace_back(p, bytes);
        return p;
    }
    // the block now belongs to the table (freed with it)
    void give(hj_table* t, void* p) {
        for (size_t i = 0; i < blocks.size(); ++i)
            if (blocks[i].first == p) {
                dfp::host::table_adopt_block(t, c->device, p, blocks[i].second);
                blocks.erase(blocks.begin() + (long)i);
                return;
            }
    }
    hj_status defer() {
        hipEvent_t e;
        HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIP_OK(hipEventRecord(e, s));
        c->deferred.push_back({e, std::move(blocks)});
        blocks.clear();
        handed_over = true;
        return HJ_OK;
    }
    ~Scratch() {
        if (handed_over || blocks.empty()) return;
        (void)hipStreamSynchronize(s);  // error path: the queued work may still use them
        for (auto& b : blocks) dfp::host::free_block(c->device, b.first, b.second);
    }
};

#define GET(var, type, bytes)                                                   \
    type var = (type)scr.get(bytes);                                            \
    if (var == nullptr) return set_error(HJ_ERR_OOM, "hj_dist: device allocation failed")

void release_finished(hj_comm* c, bool wait) {
    std::vector<hj_comm::Deferred> keep;
    for (auto& d : c->deferred) {
        if (wait) (void)hipEventSynchronize(d.done);
        if (wait || hipEventQuery(d.done) == hipSuccess) {
            for (auto& b : d.blocks) dfp::host::free_block(c->device, b.first, b.second);
            (void)hipEventDestroy(d.done);
        } else {
            keep.push_back(std::move(d));
        }
    }
    c->deferred = std::move(keep);
}

// a small device array to the host, waiting for this stream's work up to here only
hj_status read_host(hj_comm* c, const void* d, int64_t words, hipStream_t s) {
    if (words > kHostWords) return set_error(HJ_ERR_INVALID, "hj_dist: host read too large");
    HIP_OK(hipMemcpyAsync(c->host, d, (size_t)words * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipEventRecord(c->ev, s));
    HIP_OK(hipEventSynchronize(c->ev));
    return HJ_OK;
}

// out[offs[d] .. + lens[d]) = rank d's piece (elements of esz bytes), on every rank; `mine`
// (esz * lens[me] bytes, may lie inside out) holds this rank's piece
hj_status allgather_var(hj_comm* c, Scratch& scr, char* out, const std::vector<int64_t>& offs,
                        const std::vector<int64_t>& lens, const char* mine, int esz, hipStream_t s) {
    const int W = c->world, me = c->rank;
    if (W == 1) {
        if (lens[0] && out + offs[0] * esz != mine)
            HIP_OK(hipMemcpyAsync(out + offs[0] * esz, mine, (size_t)lens[0] * esz, hipMemcpyDeviceToDevice, s));
        return HJ_OK;
    }
    const int64_t m = *std::max_element(lens.begin(), lens.end());
    if (m == 0) return HJ_OK;
    bool even = true;
    for (int d = 0; d < W; ++d) even &= lens[d] == m && offs[d] == (int64_t)d * m;
    // in pieces of <= kMaxMsgBytes per rank (every rank derives the same split)
    const int64_t per = std::max<int64_t>(1, (int64_t)(kMaxMsgBytes / (size_t)esz));
    if (even && m <= per) {  // in place: rank d's piece already sits at out + d * m
        NCCL_OK(ncclAllGather(out + (int64_t)me * m * esz, out, (size_t)m * esz, ncclUint8, c->comm, s));
        return HJ_OK;
    }
    const int64_t chunk = std::min(m, per);
    GET(pad, char*, (size_t)chunk * esz);
    GET(tmp, char*, (size_t)chunk * esz * W);
    for (int64_t a = 0; a < m; a += chunk) {
        const int64_t k = std::min(chunk, m - a);
        const int64_t mk = std::max<int64_t>(0, std::min(k, lens[me] - a));
        if (mk > 0) HIP_OK(hipMemcpyAsync(pad, mine + a * esz, (size_t)mk * esz, hipMemcpyDeviceToDevice, s));
        NCCL_OK(ncclAllGather(pad, tmp, (size_t)k * esz, ncclUint8, c->comm, s));
        for (int d = 0; d < W; ++d) {
            const int64_t dk = std::max<int64_t>(0, std::min(k, lens[d] - a));
            if (dk > 0)
                HIP_OK(hipMemcpyAsync(out + (offs[d] + a) * esz, tmp + (int64_t)d * k * esz, (size_t)dk * esz,
                                      hipMemcpyDeviceToDevice, s));
        }
    }
    return HJ_OK;
}

// one element count per rank -> host (rank order)
hj_status allgather_count(hj_comm* c, Scratch& scr, const int64_t* d_val, std::vector<int64_t>* out, hipStream_t s) {
    const int W = c->world;
    GET(all, int64_t*, 8 * (size_t)W);
    if (W == 1)
        HIP_OK(hipMemcpyAsync(all, d_val, 8, hipMemcpyDeviceToDevice, s));
    else
        NCCL_OK(ncclAllGather(d_val, all, 1, ncclInt64, c->comm, s));
    ST_OK(read_host(c, all, W, s));
    out->assign(c->host, c->host + W);
    return HJ_OK;
}

// the rank's contiguous share [lo, hi] of [gmin, gmax] under the partition kernel's range
// map (part = umulhi(key - gmin, mul), mul = floor(2^64 W / range)); false when empty
bool range_share(int64_t gmin, int64_t gmax, int W, int r, int64_t* lo, int64_t* hi) {
    if (W == 1) {
        *lo = gmin;
        *hi = gmax;
        return true;
    }
    const unsigned __int128 rng = (unsigned __int128)((uint64_t)gmax - (uint64_t)gmin) + 1;
    unsigned __int128 mul = ((unsigned __int128)W << 64) / rng;
    if (mul > (unsigned __int128)UINT64_MAX) mul = UINT64_MAX;
    auto first = [&](int q) -> unsigned __int128 {  // smallest offset x with (x * mul) >> 64 >= q
        const unsigned __int128 num = (unsigned __int128)q << 64;
        return (num + mul - 1) / mul;
    };
    const unsigned __int128 a = first(r), b = first(r + 1);  // [a, b)
    if (a >= rng || a >= b) return false;
    const unsigned __int128 last = std::min<unsigned __int128>(b, rng) - 1;
    *lo = (int64_t)((uint64_t)gmin + (uint64_t)a);
    *hi = (int64_t)((uint64_t)gmin + (uint64_t)last);
    return true;
}

}  // namespace

extern "C" {

hj_status hj_comm_unique_id(uint8_t id[HJ_COMM_ID_BYTES]) {
    static_assert(HJ_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");
    if (id == nullptr) return set_error(HJ_ERR_INVALID, "null id");
    ncclUniqueId u;
    NCCL_OK(ncclGetUniqueId(&u));
    memcpy(id, u.internal, HJ_COMM_ID_BYTES);
    return HJ_OK;
}

hj_status hj_comm_create(int rank, int world, const uint8_t id[HJ_COMM_ID_BYTES], int device, hj_comm** out) {
    if (out == nullptr || id == nullptr) return set_error(HJ_ERR_INVALID, "null id/out");
    *out = nullptr;
    if (world < 1 || rank < 0 || rank >= world) return set_error(HJ_ERR_INVALID, "bad rank/world");
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0)
        return set_error(HJ_ERR_NO_DEVICE, "no GPU visible: the HIP path cannot run (no CPU fallback)");
    if (device < 0 || device >= nd) return set_error(HJ_ERR_INVALID, "bad device ordinal");
    HIP_OK(hipSetDevice(device));
    hj_comm* c = new hj_comm();
    c->rank = rank;
    c->world = world;
    c->device = device;
    if (hipHostMalloc((void**)&c->host, kHostWords * 8, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev, hipEventDisableTiming) != hipSuccess) {
        hj_comm_free(c);
        return set_error(HJ_ERR_HIP, "hj_comm_create: pinned mailbox / event");
    }
    if (world > 1) {
        ncclUniqueId u;
        memcpy(u.internal, id, HJ_COMM_ID_BYTES);
        const ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
        if (r != ncclSuccess) {
            c->comm = nullptr;
            hj_comm_free(c);
            return set_error(HJ_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        }
    }
    *out = c;
    return HJ_OK;
}

void hj_comm_free(hj_comm* c) {
    if (c == nullptr) return;
    (void)hipSetDevice(c->device);
    release_finished(c, true);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->ev) (void)hipEventDestroy(c->ev);
    if (c->host) (void)hipHostFree(c->host);
    delete c;
}

hj_status hj_dist_build_sharded(hj_comm* c, hj_key_type key_type, const void* keys, const uint8_t* validity,
                                int64_t voff, int64_t n, int64_t build_base, void* stream, hj_table** out,
                                hj_dist_info* info) {
    if (c == nullptr || out == nullptr) return set_error(HJ_ERR_INVALID, "null communicator/out");
    *out = nullptr;
    if (key_type != HJ_INT32 && key_type != HJ_INT64) return set_error(HJ_ERR_INVALID, "unsupported key type");
    if (n < 0 || build_base < 0 || voff < 0) return set_error(HJ_ERR_INVALID, "negative n/base/offset");
    if (n > 0 && keys == nullptr) return set_error(HJ_ERR_INVALID, "null keys");
    HIP_OK(hipSetDevice(c->device));
    release_finished(c, false);
    const int W = c->world, me = c->rank;
    const int kb = key_type == HJ_INT64 ? 8 : 4;
    hipStream_t s = (hipStream_t)stream;
    Scratch scr(c, s);

    // 1. the global key range and build rows: [min, max, base + n], one grouped all-reduce
    GET(mm, int64_t*, 4 * 8);
    GET(mws, void*, (size_t)hj_key_minmax_workspace_bytes());
    ST_OK(hj_key_minmax(key_type, keys, validity, voff, n, mm, mws, s));
    c->host[0] = build_base + n;
    HIP_OK(hipMemcpyAsync(mm + 2, c->host, 8, hipMemcpyHostToDevice, s));
    if (W > 1) {
        NCCL_OK(ncclGroupStart());
        NCCL_OK(ncclAllReduce(mm, mm, 1, ncclInt64, ncclMin, c->comm, s));
        NCCL_OK(ncclAllReduce(mm + 1, mm + 1, 2, ncclInt64, ncclMax, c->comm, s));
        NCCL_OK(ncclGroupEnd());
    }
    ST_OK(read_host(c, mm, 3, s));
    const int64_t gmin = c->host[0], gmax = c->host[1], rows = c->host[2];
    if (info) {
        info->build_rows = rows;
        info->recv_rows = 0;
        info->sharded = 0;
    }
    hj_table* t = nullptr;
    if (gmin > gmax) {  // no valid build row anywhere: an empty table
        ST_OK(hj_build_begin(c->device, 1, key_type, 0, &t));
        hj_status st = hj_build_finish(t, 0);
        if (st != HJ_OK) {
            hj_table_free(t);
            return st;
        }
        *out = t;
        return scr.defer();
    }
    const uint64_t rng_m1 = (uint64_t)gmax - (uint64_t)gmin;  // range - 1
    const bool dense = rng_m1 < kDenseMax && rng_m1 < (uint64_t)8 * (uint64_t)rows;
    const bool pow2 = (W & (W - 1)) == 0 && W <= 64;
    const bool packed = 2 * rows + 2 * (int64_t)W + 2 < ((int64_t)1 << 27);
    const bool sharded = dense && pow2 && rows < ((int64_t)1 << 31) && packed;

    if (!sharded) {
        // every rank builds the whole build side: valid rows with their global ids
        // compacted (one region), all-gathered in rank order (= canonical order), one build
        const int64_t cap = std::max<int64_t>(n, 1);
        GET(pk, char*, (size_t)cap * kb);
        GET(pi, uint64_t*, (size_t)cap * 8);
        GET(cnt, int64_t*, 8);
        GET(pws, void*, (size_t)hj_partition_regions_workspace_bytes(n, 1));
        ST_OK(hj_partition_regions(key_type, keys, validity, voff, nullptr, (uint64_t)build_base, n, 1, nullptr, pk, kb,
                                   0, pi, 8, cap, cnt, pws, s));
        std::vector<int64_t> lens;
        ST_OK(allgather_count(c, scr, cnt, &lens, s));
        for (int d = 0; d < W; ++d)
            if (lens[d] < 0 || lens[d] >= ((int64_t)1 << 59) || (d == me && lens[d] > cap))
                return set_error(HJ_ERR_HIP, "hj_dist: partition count out of range (device look-back failure)");
        std::vector<int64_t> offs(W, 0);
        for (int d = 1; d < W; ++d) offs[d] = offs[d - 1] + lens[d - 1];
        const int64_t total = offs[W - 1] + lens[W - 1];
        GET(gk, char*, (size_t)std::max<int64_t>(total, 1) * kb);
        GET(gi, uint64_t*, (size_t)std::max<int64_t>(total, 1) * 8);
        ST_OK(allgather_var(c, scr, gk, offs, lens, pk, kb, s));
        ST_OK(allgather_var(c, scr, (char*)gi, offs, lens, (const char*)pi, 8, s));
        ST_OK(hj_build_begin(c->device, 1, key_type, total, &t));
        const uint32_t fl = HJ_INPUT_DEVICE | HJ_BORROW | HJ_BORROW_KEEP | (rows < ((int64_t)1 << 31) ? HJ_IDS_U31 : 0);
        hj_status st = hj_build_append(t, 0, gk, nullptr, 0, gi, total, fl, s);
        if (st == HJ_OK) st = hj_build_finish(t, 0);
        if (st != HJ_OK) {
            hj_table_free(t);
            return st;
        }
        scr.give(t, gk);
        scr.give(t, gi);
        if (info) info->recv_rows = total;
        *out = t;
        return scr.defer();
    }

    // 2. every valid row to the owner of its key range; int32 offsets when the range fits
    const bool narrow = key_type == HJ_INT64 && rng_m1 < ((uint64_t)1 << 32);
    const int64_t koff = narrow ? (int64_t)((uint64_t)gmin + (1ull << 31)) : 0;
    const int okb = narrow ? 4 : kb;
    const hj_key_type lkt = okb == 8 ? HJ_INT64 : HJ_INT32;
    const int64_t cap = std::max<int64_t>(n, 1);
    GET(rk, char*, (size_t)cap * W * okb);
    GET(ri, uint64_t*, (size_t)cap * W * 8);
    GET(cnt, int64_t*, 8 * (size_t)W);
    GET(pws, void*, (size_t)hj_partition_regions_workspace_bytes(n, W));
    hj_part_spec spec{W > 1 ? 1 : 0, gmin, gmax};
    ST_OK(hj_partition_regions(key_type, keys, validity, voff, nullptr, (uint64_t)build_base, n, W, &spec, rk, okb,
                               koff, ri, 8, cap, cnt, pws, s));
    // the count matrix m[s][d] (rows rank s sends to rank d): one all-gather, one read
    GET(allc, int64_t*, 8 * (size_t)W * W);
    if (W == 1)
        HIP_OK(hipMemcpyAsync(allc, cnt, 8, hipMemcpyDeviceToDevice, s));
    else
        NCCL_OK(ncclAllGather(cnt, allc, (size_t)W, ncclInt64, c->comm, s));
    ST_OK(read_host(c, allc, (int64_t)W * W, s));
    std::vector<int64_t> m(c->host, c->host + (size_t)W * W);
    for (int src = 0; src < W; ++src)
        for (int d = 0; d < W; ++d) {
            const int64_t v = m[(size_t)src * W + d];
            if (v < 0 || v >= ((int64_t)1 << 59) || (src == me && v > cap))
                return set_error(HJ_ERR_HIP, "hj_dist: partition count out of range (device look-back failure)");
        }
    std::vector<int64_t> roff(W, 0);
    for (int src = 1; src < W; ++src) roff[src] = roff[src - 1] + m[(size_t)(src - 1) * W + me];
    const int64_t R = roff[W - 1] + m[(size_t)(W - 1) * W + me];
    GET(bk, char*, (size_t)std::max<int64_t>(R, 1) * okb);
    GET(bi, uint64_t*, (size_t)std::max<int64_t>(R, 1) * 8);
    const int64_t self = m[(size_t)me * W + me];
    if (self > 0) {
        HIP_OK(hipMemcpyAsync(bk + roff[me] * okb, rk + (int64_t)me * cap * okb, (size_t)self * okb,
                              hipMemcpyDeviceToDevice, s));
        HIP_OK(hipMemcpyAsync(bi + roff[me], ri + (int64_t)me * cap, (size_t)self * 8, hipMemcpyDeviceToDevice, s));
    }
    if (W > 1) {
        // per peer: keys then ids, in pieces; both sides issue the same sequence
        NCCL_OK(ncclGroupStart());
        for (int p = 0; p < W; ++p) {
            if (p == me) continue;
            const int64_t ns = m[(size_t)me * W + p], nr = m[(size_t)p * W + me];
            for (int col = 0; col < 2; ++col) {
                const int esz = col == 0 ? okb : 8;
                const char* sb = col == 0 ? rk + (int64_t)p * cap * okb : (const char*)(ri + (int64_t)p * cap);
                char* rb = col == 0 ? bk + roff[p] * okb : (char*)(bi + roff[p]);
                const int64_t per = (int64_t)(kMaxMsgBytes / (size_t)esz);
                for (int64_t a = 0; a < ns; a += per)
                    NCCL_OK(ncclSend(sb + a * esz, (size_t)std::min(per, ns - a) * esz, ncclUint8, p, c->comm, s));
                for (int64_t a = 0; a < nr; a += per)
                    NCCL_OK(ncclRecv(rb + a * esz, (size_t)std::min(per, nr - a) * esz, ncclUint8, p, c->comm, s));
            }
        }
        NCCL_OK(ncclGroupEnd());
    }
    if (info) {
        info->recv_rows = R;
        info->sharded = 1;
    }

    // 3. every rank's range (they tile [gmin, gmax] in rank order); this rank's piece
    std::vector<int64_t> lens(W, 0), offs(W, 0), lo(W, 0), hi(W, -1);
    for (int d = 0; d < W; ++d) {
        if (range_share(gmin, gmax, W, d, &lo[d], &hi[d])) lens[d] = hi[d] - lo[d] + 1;
        if (d > 0) offs[d] = offs[d - 1] + lens[d - 1];
    }
    const int64_t nvalues = offs[W - 1] + lens[W - 1];
    if ((uint64_t)nvalues != rng_m1 + 1) return set_error(HJ_ERR_INVALID, "hj_dist: range shares do not tile the domain");
    GET(full, uint32_t*, (size_t)nvalues * 4);
    GET(used, int64_t*, 8);
    HIP_OK(hipMemsetAsync(used, 0, 8, s));
    uint32_t* mine = full + offs[me];
    hj_table* local = nullptr;
    struct LocalGuard {  // freed with the result table, or here on an error
        hj_table** p;
        ~LocalGuard() {
            if (*p) hj_table_free(*p);
        }
    } lg{&local};
    if (lens[me] > 0 && R > 0) {
        ST_OK(hj_build_begin(c->device, 1, lkt, R, &local));
        ST_OK(hj_build_append(local, 0, bk, nullptr, 0, bi, R, HJ_INPUT_DEVICE | HJ_BORROW | HJ_BORROW_KEEP | HJ_IDS_U31,
                              s));
        ST_OK(hj_build_key_range(local, lo[me] - koff, hi[me] - koff));
        ST_OK(hj_build_dense(local));
        ST_OK(hj_build_finish(local, 0));
        ST_OK(hj_table_dense_export(local, mine, 0, (uint64_t)lens[me], nullptr, 0, (uint64_t*)used, s));
    } else if (lens[me] > 0) {
        HIP_OK(hipMemsetAsync(mine, 0xFF, (size_t)lens[me] * 4, s));  // every ref kMiss
    }
    ST_OK(allgather_var(c, scr, (char*)full, offs, lens, (const char*)mine, 4, s));
    std::vector<int64_t> du;
    ST_OK(allgather_count(c, scr, used, &du, s));
    std::vector<int64_t> dbase(W, 0);
    for (int d = 1; d < W; ++d) dbase[d] = dbase[d - 1] + du[d - 1];
    const int64_t dtotal = dbase[W - 1] + du[W - 1];
    if (dtotal >= ((int64_t)1 << 27)) return set_error(HJ_ERR_INVALID, "hj_dist: duplicate segments past packed refs");
    GET(dup, uint32_t*, (size_t)std::max<int64_t>(dtotal, 4) * 4);
    if (dtotal > 0) {
        if (local != nullptr && du[me] > 0)
            ST_OK(hj_table_dense_export(local, nullptr, 0, 0, dup + dbase[me], (uint64_t)du[me], nullptr, s));
        ST_OK(allgather_var(c, scr, (char*)dup, dbase, du, (const char*)(dup + dbase[me]), 4, s));
        for (int d = 0; d < W; ++d)
            if (du[d] > 0 && dbase[d] > 0)
                ST_OK(hj_dense_rebase_dups(full + offs[d], (uint64_t)lens[d], (uint32_t)dbase[d], 1, s));
    } else {
        HIP_OK(hipMemsetAsync(dup, 0, 16, s));
    }
    ST_OK(hj_table_wrap_dense(c->device, key_type, gmin, (uint64_t)nvalues, full, dup, 1, s, &t));
    scr.give(t, full);
    scr.give(t, dup);
    if (local != nullptr) {
        dfp::host::table_adopt_table(t, local);
        local = nullptr;
    }
    *out = t;
    return scr.defer();
}

}  // extern "C"
