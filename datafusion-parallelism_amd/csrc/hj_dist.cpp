// hj_dist.cpp — the multi-GPU plans behind the C ABI (include/hj.h, "multi-process"), one
// process per GPU, so that a host in any language (the Rust drop-in) drives the
// multi-GPU join through hj_* calls alone.
//
// Two plans, each one job per step on the communicator's worker thread:
//   * the sharded-build plan's build side (hj_dist_build_sharded[_async]): a global key
//     range, every build row to the rank that owns its contiguous key range, a
//     direct-addressed build of each rank's range, and the pieces all-gathered into one
//     table over the whole key domain that every rank probes with its own probe rows
//     (src/operator/version10/parallel_join_execution_state.rs:405-407: one table shared
//     by every partition);
//   * the radix plan (hj_dist_join_radix): both sides partitioned by the same map (the
//     reference's shard function, src/utils/partitioned_concurrent_self_hash_join_map.rs:
//     13-16, and its per-shard inserts, 263-281), exchanged point to point, built and
//     probed on their owner, pairs carrying global ids.
//
// Collectives go through the communicator's Transport (hj_comm.h): RCCL here (xGMI is
// point to point: exchanges are per-peer ncclSend/ncclRecv in one group, not an
// all-to-all), an in-process thread transport in the test library. Every rank issues the
// same sequence. Failures are collective: each step's host read carries a status word of
// every rank, and the buffers the later collectives need are sized before that read, so
// that a rank that fails locally still takes part in the collectives and all ranks return
// the error together instead of leaving their peers blocked in a collective.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <stdlib.h>

#include <algorithm>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/hj.h"
#include "hj_comm.h"
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
constexpr int64_t kHostWords = 8192;                                   // pinned mailbox (64 KiB) for reads
constexpr int kEvents = 8;

// ---- RCCL transport -------------------------------------------------------------------

struct RcclTransport final : comm::Transport {
    ncclComm_t comm = nullptr;
    ~RcclTransport() override {
        if (comm) (void)ncclCommDestroy(comm);
    }
    hj_status group_start() override {
        NCCL_OK(ncclGroupStart());
        return HJ_OK;
    }
    hj_status group_end(hipStream_t) override {
        NCCL_OK(ncclGroupEnd());
        return HJ_OK;
    }
    hj_status allreduce_i64(const int64_t* send, int64_t* recv, size_t count, comm::Red op, hipStream_t s) override {
        NCCL_OK(ncclAllReduce(send, recv, count, ncclInt64, op == comm::Red::Min ? ncclMin : ncclMax, comm, s));
        return HJ_OK;
    }
    hj_status allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        NCCL_OK(ncclAllGather(send, recv, bytes, ncclUint8, comm, s));
        return HJ_OK;
    }
    hj_status send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
        NCCL_OK(ncclSend(buf, bytes, ncclUint8, peer, comm, s));
        return HJ_OK;
    }
    hj_status recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
        NCCL_OK(ncclRecv(buf, bytes, ncclUint8, peer, comm, s));
        return HJ_OK;
    }
    void abort() override {
        if (comm) (void)ncclCommAbort(comm);
        comm = nullptr;
    }
};

// ---- per-job scratch --------------------------------------------------------------------

// Device blocks of one job. On success they go to the communicator's deferred list behind
// the job's end event (released by a later job once it fired); on failure they are
// released after the streams drained.
struct Scratch {
    hj_comm* c;
    std::vector<hipStream_t> streams;
    std::vector<std::pair<void*, size_t>> blocks;
    bool handed_over = false;
    Scratch(hj_comm* c_, std::vector<hipStream_t> s_) : c(c_), streams(std::move(s_)) {}
    void* get(size_t bytes) {
        bytes = std::max<size_t>(bytes, 64);
        void* p = dfp::host::dev_block(c->device, bytes);
        if (p) blocks.emplace_back(p, bytes);
        return p;
    }
    // the block now belongs to the table (freed with it) / to the job (freed with it)
    bool take(void* p, size_t* bytes) {
        for (size_t i = 0; i < blocks.size(); ++i)
            if (blocks[i].first == p) {
                *bytes = blocks[i].second;
                blocks.erase(blocks.begin() + (long)i);
                return true;
            }
        return false;
    }
    void give(hj_table* t, void* p) {
        size_t b = 0;
        if (take(p, &b)) dfp::host::table_adopt_block(t, c->device, p, b);
    }
    void give(hj_dist_job* j, void* p) {
        size_t b = 0;
        if (take(p, &b)) j->blocks.emplace_back(p, b);
    }
    // every stream's work so far is what the blocks serve: one event after all of them
    hj_status defer() {
        hipEvent_t e;
        HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (size_t i = 1; i < streams.size(); ++i) {
            HIP_OK(hipEventRecord(e, streams[i]));
            HIP_OK(hipStreamWaitEvent(streams[0], e, 0));
        }
        HIP_OK(hipEventRecord(e, streams[0]));
        c->deferred.push_back({e, std::move(blocks)});
        blocks.clear();
        handed_over = true;
        return HJ_OK;
    }
    ~Scratch() {
        if (handed_over || blocks.empty()) return;
        for (hipStream_t s : streams) (void)hipStreamSynchronize(s);  // error path: queued work may use them
        for (auto& b : blocks) dfp::host::free_block(c->device, b.first, b.second);
    }
};

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

// The worker waits for its reads by polling (it is the plan's critical path and has a core
// to itself; a blocking wait adds the runtime's wake-up latency to every one of the plan's
// host reads).
hj_status spin_wait(hipEvent_t e) {
    for (uint32_t i = 0;; ++i) {
        const hipError_t q = hipEventQuery(e);
        if (q == hipSuccess) return HJ_OK;
        if (q != hipErrorNotReady) return set_error(HJ_ERR_HIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
        if ((i & 63) == 63) std::this_thread::yield();
    }
}

// a small device array to the host mailbox, waiting for this stream's work up to here only
hj_status read_host(hj_comm* c, const void* d, int64_t words, hipStream_t s) {
    if (words > kHostWords) return set_error(HJ_ERR_INVALID, "hj_dist: host read too large");
    HIP_OK(hipMemcpyAsync(c->host, d, (size_t)words * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipEventRecord(c->ev, s));
    return spin_wait(c->ev);
}

// host words -> device (a pinned staging area of their own: the copy is asynchronous)
hj_status write_dev(hj_comm* c, int64_t* d, const int64_t* v, int64_t words, hipStream_t s) {
    int64_t* w = c->host + kHostWords;
    // the previous staged write must have been consumed: every staged write is followed by
    // a read_host on the same stream before the next one
    for (int64_t i = 0; i < words; ++i) w[i] = v[i];
    HIP_OK(hipMemcpyAsync(d, w, (size_t)words * 8, hipMemcpyHostToDevice, s));
    return HJ_OK;
}

// `b` waits for everything enqueued on `a` so far
hj_status join_streams(hj_comm* c, hipStream_t a, hipStream_t b, int slot) {
    if (a == b) return HJ_OK;
    hipEvent_t e = c->evs[(size_t)slot % c->evs.size()];
    HIP_OK(hipEventRecord(e, a));
    HIP_OK(hipStreamWaitEvent(b, e, 0));
    return HJ_OK;
}

// ---- collectives over the transport ----------------------------------------------------

// out[offs[d] .. + lens[d]) = rank d's piece (elements of esz bytes), on every rank; `mine`
// (esz * lens[me] bytes; may lie inside out) holds this rank's piece. Even pieces laid end
// to end: one in-place all-gather; otherwise every rank sends its piece to every peer
// (point to point over the xGMI links, no staging), in pieces of <= kMaxMsgBytes.
hj_status allgather_var(hj_comm* c, char* out, const std::vector<int64_t>& offs, const std::vector<int64_t>& lens,
                        const char* mine, int esz, hipStream_t s) {
    const int W = c->world, me = c->rank;
    if (lens[me] && out + offs[me] * esz != mine)
        HIP_OK(hipMemcpyAsync(out + offs[me] * esz, mine, (size_t)lens[me] * esz, hipMemcpyDeviceToDevice, s));
    if (W == 1) return HJ_OK;
    const int64_t m = *std::max_element(lens.begin(), lens.end());
    if (m == 0) return HJ_OK;
    bool even = true;
    for (int d = 0; d < W; ++d) even &= lens[d] == m && offs[d] == (int64_t)d * m;
    if (even && (size_t)m * esz <= kMaxMsgBytes)
        return c->tr->allgather(out + (int64_t)me * m * esz, out, (size_t)m * esz, s);
    const int64_t per = std::max<int64_t>(1, (int64_t)(kMaxMsgBytes / (size_t)esz));
    ST_OK(c->tr->group_start());
    for (int p = 0; p < W; ++p) {
        if (p == me) continue;
        for (int64_t a = 0; a < lens[me]; a += per)
            ST_OK(c->tr->send(out + (offs[me] + a) * esz, (size_t)std::min(per, lens[me] - a) * esz, p, s));
        for (int64_t a = 0; a < lens[p]; a += per)
            ST_OK(c->tr->recv(out + (offs[p] + a) * esz, (size_t)std::min(per, lens[p] - a) * esz, p, s));
    }
    return c->tr->group_end(s);
}

// every rank's `words` device words (rank order) -> host (c->host[d * words + i]):
// one all-gather into `all` (W * words, device) and one read
hj_status allgather_read(hj_comm* c, const int64_t* mine, int64_t* all, int64_t words, hipStream_t s) {
    if (c->world == 1) {
        if (all != mine) HIP_OK(hipMemcpyAsync(all, mine, (size_t)words * 8, hipMemcpyDeviceToDevice, s));
    } else {
        ST_OK(c->tr->allgather(mine, all, (size_t)words * 8, s));
    }
    return read_host(c, all, words * c->world, s);
}

// region exchange: this rank's region d (rows [d * cap, d * cap + m[me][d])) to rank d,
// rank s's region me into out at the rows of the ranks before s; the own region copied on
// the device (one rank: none, the caller reads the region in place)
hj_status exchange_regions(hj_comm* c, const std::vector<int64_t>& m, const char* regions, int64_t cap, int esz,
                           char* out, hipStream_t s) {
    const int W = c->world, me = c->rank;
    std::vector<int64_t> roff(W, 0);
    for (int src = 1; src < W; ++src) roff[src] = roff[src - 1] + m[(size_t)(src - 1) * W + me];
    const int64_t self = m[(size_t)me * W + me];
    if (self > 0 && out + roff[me] * esz != regions + (int64_t)me * cap * esz)
        HIP_OK(hipMemcpyAsync(out + roff[me] * esz, regions + (int64_t)me * cap * esz, (size_t)self * esz,
                              hipMemcpyDeviceToDevice, s));
    if (W == 1) return HJ_OK;
    const int64_t per = (int64_t)(kMaxMsgBytes / (size_t)esz);
    for (int p = 0; p < W; ++p) {
        if (p == me) continue;
        const int64_t ns = m[(size_t)me * W + p], nr = m[(size_t)p * W + me];
        for (int64_t a = 0; a < ns; a += per)
            ST_OK(c->tr->send(regions + ((int64_t)p * cap + a) * esz, (size_t)std::min(per, ns - a) * esz, p, s));
        for (int64_t a = 0; a < nr; a += per)
            ST_OK(c->tr->recv(out + (roff[p] + a) * esz, (size_t)std::min(per, nr - a) * esz, p, s));
    }
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

// A rank's local failure, held until the next status exchange (every rank then returns
// an error together). The first failure's status and message are kept.
struct LocalFail {
    bool failed = false;
    hj_status st = HJ_OK;
    std::string msg;
    void note(hj_status s) {
        if (s == HJ_OK || failed) return;
        failed = true;
        st = s;
        const char* e = hj_last_error();
        msg = e ? e : "";
    }
    void note_oom(const char* what) {
        if (failed) return;
        failed = true;
        st = HJ_ERR_OOM;
        msg = std::string("hj_dist: device allocation failed (") + what + ")";
    }
    // after a status exchange that showed some rank failed
    hj_status raise(const char* step) const {
        if (failed) return set_error(st, msg);
        return set_error(HJ_ERR_RCCL, std::string("hj_dist: a peer rank failed during ") + step);
    }
};

// one rank: the exchange is the identity (DFP_HJ_DIST_W1_IDENTITY=0 runs the whole plan,
// to price its machinery)
bool w1_identity() {
    static const bool v = [] {
        const char* e = getenv("DFP_HJ_DIST_W1_IDENTITY");
        return !(e && e[0] == '0');
    }();
    return v;
}

// test hook of the thread transport: a rank's plan fails at step `at` of job fail_at
bool injected(hj_comm* c, int64_t job, int at) { return c->fail_at >= 0 && job == c->fail_at / 8 && at == c->fail_at % 8; }

struct Status2 {  // one rank's [value, failed] words
    int64_t v[2];
};

bool counts_ok(const std::vector<int64_t>& m, int W, int me, int64_t cap) {
    for (int src = 0; src < W; ++src)
        for (int d = 0; d < W; ++d) {
            const int64_t v = m[(size_t)src * W + d];
            if (v < 0 || v >= ((int64_t)1 << 59) || (src == me && v > cap)) return false;
        }
    return true;
}

// The communicator's persistent device words (hj_comm::words), carved per plan step:
// [min | max, rows, failed] (8), two count vectors of W + 1 and their all-gathered
// matrices, a [value, failed] status and its all-gather, the key-range workspace.
struct Words {
    int64_t *mm, *cnt, *allc, *cnt2, *allc2, *st, *allst;
    void* mws;
};
size_t words_bytes(int W) {
    const size_t w = 8 + 2 * ((size_t)W + 1) + 2 * (size_t)W * ((size_t)W + 1) + 2 + 2 * (size_t)W;
    return w * 8 + (((size_t)hj_key_minmax_workspace_bytes() + 255) & ~(size_t)255);
}
Words words_of(hj_comm* c) {
    const size_t W = (size_t)c->world;
    Words w;
    int64_t* p = c->words;
    w.mm = p, p += 8;
    w.cnt = p, p += W + 1;
    w.allc = p, p += W * (W + 1);
    w.cnt2 = p, p += W + 1;
    w.allc2 = p, p += W * (W + 1);
    w.st = p, p += 2;
    w.allst = p, p += 2 * W;
    w.mws = p;
    return w;
}

// Receive buffers: sized before the count exchange that carries every rank's status, at a
// bounded slack over the even share (2 x rows / W, never more than the global rows) instead
// of the global rows (W x the expected peak at W ranks). A skewed plan whose received rows
// pass the slack allocates the exact size after that exchange; a failure there is one-sided
// and aborts the communicator (documented in hj.h).
int64_t recv_slack(int64_t rows, int W) {
    if (W == 1) return std::max<int64_t>(rows, 1);
    const int64_t share = (rows + W - 1) / W;
    return std::max<int64_t>(1, std::min<int64_t>(rows, 2 * share + 1024));
}
hj_status grow_recv(hj_comm* c, Scratch& scr, int64_t need, int64_t have, int okb, char** keys, uint64_t** ids,
                    const char* what) {
    if (need <= have) return HJ_OK;
    char* k = (char*)scr.get((size_t)need * okb);
    uint64_t* i = (uint64_t*)scr.get((size_t)need * 8);
    if (!k || !i) {
        c->tr->abort();
        c->aborted = true;
        return set_error(HJ_ERR_OOM, std::string("hj_dist: device allocation failed (") + what +
                                         " past the even-share slack); the communicator was aborted");
    }
    *keys = k;
    *ids = i;
    return HJ_OK;
}

// ---- the sharded-build plan's build side -------------------------------------------------

struct ShardedArgs {
    hj_key_type kt, pkt;
    const void* keys;
    const uint8_t* valid;
    int64_t voff, n, base;
    hipStream_t s;
};

hj_status run_sharded(hj_comm* c, const ShardedArgs& a, hj_dist_job* j, int64_t jobno) {
    const int W = c->world, me = c->rank;
    const int kb = a.kt == HJ_INT64 ? 8 : 4;
    // every step on the communicator's own stream, after the caller's inputs (ev_in: the
    // caller's stream at submission); consumers wait for the table's completion event
    hipStream_t s = c->side;
    HIP_OK(hipStreamWaitEvent(s, j->ev_in, 0));
    Scratch scr(c, {s});
    LocalFail lf;
    hipEvent_t t0 = nullptr;  // the build side's start (the table's build time runs from it)
    HIP_OK(hipEventCreate(&t0));
    HIP_OK(hipEventRecord(t0, s));
    struct EvGuard {
        hipEvent_t* e;
        ~EvGuard() {
            if (*e) (void)hipEventDestroy(*e);
        }
    } t0g{&t0};
    auto get = [&](size_t bytes, const char* what) -> void* {
        void* p = scr.get(bytes);
        if (!p) lf.note_oom(what);
        return p;
    };

    // One rank whose rows start at global row 0: the exchange is the identity and the
    // gathered table is the rank's own build, so the build side is the single-GPU build
    // of the input in place (its key range stays on the device: no partition, no copy, no
    // host read). DFP_HJ_DIST_W1_IDENTITY=0 runs the whole plan at one rank instead (to
    // price its machinery).
    if (W == 1 && a.base == 0 && a.pkt == a.kt && w1_identity() && !injected(c, jobno, 0)) {
        hj_table* t = nullptr;
        ST_OK(hj_build_begin(c->device, 1, a.kt, a.n, &t));
        hj_status st = hj_build_append(t, 0, a.keys, a.valid, a.voff, nullptr, a.n,
                                       HJ_INPUT_DEVICE | HJ_BORROW | HJ_BORROW_KEEP, s);
        if (st == HJ_OK) st = hj_build_finish(t, 0);
        if (st != HJ_OK) {
            hj_table_free(t);
            return st;
        }
        j->info.build_rows = a.n;
        j->info.recv_rows = a.n;
        j->info.sharded = 1;
        dfp::host::table_set_start_event(t, t0);
        t0 = nullptr;
        j->table = t;
        return scr.defer();
    }

    // 1. the global key range, build rows and status: [min | max, rows, failed]
    const Words w = words_of(c);
    int64_t* mm = w.mm;
    void* mws = w.mws;
    if (injected(c, jobno, 0)) lf.note(set_error(HJ_ERR_INVALID, "injected failure (test hook) at the key range"));
    if (!lf.failed) lf.note(hj_key_minmax(a.kt, a.keys, a.valid, a.voff, a.n, mm, mws, s));
    {
        int64_t v[4] = {INT64_MAX, INT64_MIN, a.base + a.n, lf.failed ? 1 : 0};
        ST_OK(write_dev(c, lf.failed ? mm : mm + 2, lf.failed ? v : v + 2, lf.failed ? 4 : 2, s));
    }
    if (W > 1) {
        ST_OK(c->tr->group_start());
        ST_OK(c->tr->allreduce_i64(mm, mm, 1, comm::Red::Min, s));
        ST_OK(c->tr->allreduce_i64(mm + 1, mm + 1, 3, comm::Red::Max, s));
        ST_OK(c->tr->group_end(s));
    }
    ST_OK(read_host(c, mm, 4, s));
    const int64_t gmin = c->host[0], gmax = c->host[1], rows = c->host[2];
    if (c->host[3] != 0) return lf.raise("the key range");
    j->info.build_rows = rows;
    j->info.recv_rows = 0;
    j->info.sharded = 0;
    hj_table* t = nullptr;
    auto finish = [&](hj_table* tt) -> hj_status {
        dfp::host::table_set_start_event(tt, t0);
        t0 = nullptr;
        j->table = tt;
        return scr.defer();
    };
    if (gmin > gmax) {  // no valid build row anywhere: an empty table
        ST_OK(hj_build_begin(c->device, 1, a.pkt, 0, &t));
        hj_status st = hj_build_finish(t, 0);
        if (st != HJ_OK) {
            hj_table_free(t);
            return st;
        }
        return finish(t);
    }
    const uint64_t rng_m1 = (uint64_t)gmax - (uint64_t)gmin;  // range - 1
    const bool dense = rng_m1 < kDenseMax && rng_m1 < (uint64_t)8 * (uint64_t)rows;
    const bool pow2 = (W & (W - 1)) == 0 && W <= 64;
    const bool packed = 2 * rows + 2 * (int64_t)W + 2 < ((int64_t)1 << 27);
    const bool sharded = dense && pow2 && rows < ((int64_t)1 << 31) && packed;

    if (!sharded) {
        // every rank builds the whole build side: valid rows with their global ids
        // compacted (one region), all-gathered in rank order (= canonical order), one build.
        // The table compares the build key type: the probe keys must have it too.
        if (a.pkt != a.kt)
            return set_error(HJ_ERR_INVALID, "hj_dist_build_sharded: a sparse build domain (whole build on every rank) "
                                             "needs probe keys of the build key type");
        const int64_t cap = std::max<int64_t>(a.n, 1);
        char* pk = (char*)get((size_t)cap * kb, "rows");
        uint64_t* pi = (uint64_t*)get((size_t)cap * 8, "ids");
        int64_t* st2 = w.st;
        int64_t* all2 = w.allst;
        void* pws = get((size_t)hj_partition_regions_workspace_bytes(a.n, 1), "workspace");
        // the gathered side: at most the global rows (sized before the status exchange)
        char* gk = (char*)get((size_t)std::max<int64_t>(rows, 1) * kb, "gathered keys");
        uint64_t* gi = (uint64_t*)get((size_t)std::max<int64_t>(rows, 1) * 8, "gathered ids");
        if (injected(c, jobno, 1)) lf.note(set_error(HJ_ERR_INVALID, "injected failure (test hook) at the partition"));
        if (!lf.failed)
            lf.note(hj_partition_regions(a.kt, a.keys, a.valid, a.voff, nullptr, (uint64_t)a.base, a.n, 1, nullptr, pk,
                                         kb, 0, pi, 8, cap, st2, pws, s));
        if (lf.failed) HIP_OK(hipMemsetAsync(st2, 0, 8, s));
        {
            int64_t f = lf.failed ? 1 : 0;
            ST_OK(write_dev(c, st2 + 1, &f, 1, s));
        }
        ST_OK(allgather_read(c, st2, all2, 2, s));
        std::vector<int64_t> lens(W), offs(W, 0);
        bool anyfail = false;
        for (int d = 0; d < W; ++d) {
            lens[d] = c->host[2 * d];
            anyfail |= c->host[2 * d + 1] != 0;
        }
        if (anyfail) return lf.raise("the build-row partition");
        for (int d = 0; d < W; ++d)
            if (lens[d] < 0 || lens[d] >= ((int64_t)1 << 59) || (d == me && lens[d] > cap))
                return set_error(HJ_ERR_HIP, "hj_dist: partition count out of range (device look-back failure)");
        for (int d = 1; d < W; ++d) offs[d] = offs[d - 1] + lens[d - 1];
        const int64_t total = offs[W - 1] + lens[W - 1];
        if (total > std::max<int64_t>(rows, 1)) return set_error(HJ_ERR_HIP, "hj_dist: more valid rows than rows");
        ST_OK(allgather_var(c, gk, offs, lens, pk, kb, s));
        ST_OK(allgather_var(c, (char*)gi, offs, lens, (const char*)pi, 8, s));
        ST_OK(hj_build_begin(c->device, 1, a.kt, total, &t));
        const uint32_t fl = HJ_INPUT_DEVICE | HJ_BORROW | HJ_BORROW_KEEP | (rows < ((int64_t)1 << 31) ? HJ_IDS_U31 : 0);
        hj_status st = hj_build_append(t, 0, gk, nullptr, 0, gi, total, fl, s);
        if (st == HJ_OK) st = hj_build_finish(t, 0);
        if (st != HJ_OK) {
            hj_table_free(t);
            return st;
        }
        scr.give(t, gk);
        scr.give(t, gi);
        j->info.recv_rows = total;
        return finish(t);
    }

    // 2. every valid row to the owner of its key range; int32 offsets when the range fits.
    // Everything the later collectives need is sized here, before the count exchange
    // carries every rank's status: received rows (at most the global rows), the whole
    // domain's refs, the segment words (at most 2 B + 2 G + 2, the packed refs' bound).
    const bool narrow = a.kt == HJ_INT64 && rng_m1 < ((uint64_t)1 << 32);
    const int64_t koff = narrow ? (int64_t)((uint64_t)gmin + (1ull << 31)) : 0;
    const int okb = narrow ? 4 : kb;
    const hj_key_type lkt = okb == 8 ? HJ_INT64 : HJ_INT32;
    const int64_t cap = std::max<int64_t>(a.n, 1);
    std::vector<int64_t> lens(W, 0), offs(W, 0), lo(W, 0), hi(W, -1);
    for (int d = 0; d < W; ++d) {
        if (range_share(gmin, gmax, W, d, &lo[d], &hi[d])) lens[d] = hi[d] - lo[d] + 1;
        if (d > 0) offs[d] = offs[d - 1] + lens[d - 1];
    }
    const int64_t nvalues = offs[W - 1] + lens[W - 1];
    if ((uint64_t)nvalues != rng_m1 + 1) return set_error(HJ_ERR_INVALID, "hj_dist: range shares do not tile the domain");
    const int64_t rcap = W == 1 ? cap : recv_slack(rows, W);
    const int64_t dcap = 2 * rows + 2 * (int64_t)W + 4;
    int64_t* cnt = w.cnt;
    int64_t* allc = w.allc;
    int64_t* used = w.st;
    int64_t* allu = w.allst;
    char* rk = (char*)get((size_t)cap * W * okb, "regions");
    uint64_t* ri = (uint64_t*)get((size_t)cap * W * 8, "regions");
    void* pws = get((size_t)hj_partition_regions_workspace_bytes(a.n, W), "workspace");
    char* bk = W == 1 ? rk : (char*)get((size_t)rcap * okb, "received keys");
    uint64_t* bi = W == 1 ? ri : (uint64_t*)get((size_t)rcap * 8, "received ids");
    uint32_t* full = (uint32_t*)get((size_t)nvalues * 4, "table refs");
    uint32_t* dup = (uint32_t*)get((size_t)dcap * 4, "segments");
    hj_part_spec spec{W > 1 ? 1 : 0, gmin, gmax};
    if (injected(c, jobno, 1)) lf.note(set_error(HJ_ERR_INVALID, "injected failure (test hook) at the partition"));
    if (!lf.failed)
        lf.note(hj_partition_regions(a.kt, a.keys, a.valid, a.voff, nullptr, (uint64_t)a.base, a.n, W, &spec, rk, okb,
                                     koff, ri, 8, cap, cnt, pws, s));
    if (lf.failed) HIP_OK(hipMemsetAsync(cnt, 0, 8 * (size_t)W, s));
    {
        int64_t f = lf.failed ? 1 : 0;
        ST_OK(write_dev(c, cnt + W, &f, 1, s));
    }
    // the count matrix m[s][d] (rows rank s sends to rank d) + statuses: one all-gather, one read
    ST_OK(allgather_read(c, cnt, allc, W + 1, s));
    std::vector<int64_t> m((size_t)W * W);
    bool anyfail = false;
    for (int src = 0; src < W; ++src) {
        for (int d = 0; d < W; ++d) m[(size_t)src * W + d] = c->host[(size_t)src * (W + 1) + d];
        anyfail |= c->host[(size_t)src * (W + 1) + W] != 0;
    }
    if (anyfail) return lf.raise("the build-row partition");
    if (!counts_ok(m, W, me, cap))
        return set_error(HJ_ERR_HIP, "hj_dist: partition count out of range (device look-back failure)");
    int64_t R = 0;
    for (int src = 0; src < W; ++src) R += m[(size_t)src * W + me];
    if (R > std::max<int64_t>(rows, 1)) return set_error(HJ_ERR_HIP, "hj_dist: received rows exceed the global rows");
    if (W > 1) ST_OK(grow_recv(c, scr, R, rcap, okb, &bk, &bi, "received build rows"));
    if (W > 1) {  // per peer: keys then ids, in pieces; both sides issue the same sequence
        ST_OK(c->tr->group_start());
        ST_OK(exchange_regions(c, m, rk, cap, okb, bk, s));
        ST_OK(exchange_regions(c, m, (const char*)ri, cap, 8, (char*)bi, s));
        ST_OK(c->tr->group_end(s));
    }
    j->info.recv_rows = R;
    j->info.sharded = 1;

    // 3. this rank's piece of the whole domain's refs, then the gathers
    uint32_t* mine = full + offs[me];
    hj_table* local = nullptr;
    struct LocalGuard {  // freed with the result table, or here on an error
        hj_table** p;
        ~LocalGuard() {
            if (*p) hj_table_free(*p);
        }
    } lg{&local};
    HIP_OK(hipMemsetAsync(used, 0, 8, s));
    if (injected(c, jobno, 2)) lf.note(set_error(HJ_ERR_INVALID, "injected failure (test hook) at the local build"));
    if (!lf.failed && lens[me] > 0 && R > 0) {
        hj_status st = hj_build_begin(c->device, 1, lkt, R, &local);
        if (st == HJ_OK)
            st = hj_build_append(local, 0, bk, nullptr, 0, bi, R,
                                 HJ_INPUT_DEVICE | HJ_BORROW | HJ_BORROW_KEEP | HJ_IDS_U31, s);
        if (st == HJ_OK) st = hj_build_key_range(local, lo[me] - koff, hi[me] - koff);
        if (st == HJ_OK) st = hj_build_dense(local);
        if (st == HJ_OK) st = hj_build_finish(local, 0);
        if (st == HJ_OK) st = hj_table_dense_export(local, mine, 0, (uint64_t)lens[me], nullptr, 0, (uint64_t*)used, s);
        lf.note(st);
    }
    if (lf.failed || (lens[me] > 0 && R == 0))
        if (lens[me] > 0) HIP_OK(hipMemsetAsync(mine, 0xFF, (size_t)lens[me] * 4, s));  // every ref kMiss
    if (lf.failed) HIP_OK(hipMemsetAsync(used, 0, 8, s));
    {
        int64_t f = lf.failed ? 1 : 0;
        ST_OK(write_dev(c, used + 1, &f, 1, s));
    }
    ST_OK(allgather_var(c, (char*)full, offs, lens, (const char*)mine, 4, s));
    ST_OK(allgather_read(c, used, allu, 2, s));
    std::vector<int64_t> du(W), dbase(W, 0);
    anyfail = false;
    for (int d = 0; d < W; ++d) {
        du[d] = c->host[2 * d];
        anyfail |= c->host[2 * d + 1] != 0;
    }
    if (anyfail) return lf.raise("the local builds");
    for (int d = 1; d < W; ++d) dbase[d] = dbase[d - 1] + du[d - 1];
    const int64_t dtotal = dbase[W - 1] + du[W - 1];
    if (dtotal >= ((int64_t)1 << 27) || dtotal > dcap)
        return set_error(HJ_ERR_INVALID, "hj_dist: duplicate segments past packed refs");
    if (dtotal > 0) {
        if (local != nullptr && du[me] > 0)
            ST_OK(hj_table_dense_export(local, nullptr, 0, 0, dup + dbase[me], (uint64_t)du[me], nullptr, s));
        ST_OK(allgather_var(c, (char*)dup, dbase, du, (const char*)(dup + dbase[me]), 4, s));
        for (int d = 0; d < W; ++d)
            if (du[d] > 0 && dbase[d] > 0)
                ST_OK(hj_dense_rebase_dups(full + offs[d], (uint64_t)lens[d], (uint32_t)dbase[d], 1, s));
    } else {
        HIP_OK(hipMemsetAsync(dup, 0, 16, s));
    }
    // keyed in the probe keys' domain: narrowing shifted only the travelling build keys
    ST_OK(hj_table_wrap_dense(c->device, a.pkt, gmin, (uint64_t)nvalues, full, dup, 1, s, &t));
    scr.give(t, full);
    scr.give(t, dup);
    if (local != nullptr) {
        dfp::host::table_adopt_table(t, local);
        local = nullptr;
    }
    return finish(t);
}

// ---- the radix plan ----------------------------------------------------------------------

struct RadixArgs {
    hj_key_type kt, pkt;
    const void *bkeys, *pkeys;
    const uint8_t *bvalid, *pvalid;
    int64_t bvoff, nb, bbase, pvoff, np, pbase;
    hipStream_t s;
};

// Both sides by the plan of DistributedHashJoin.prepare (distributed.py): the runtime filter
// drops probe rows outside the global build key range before they travel, a dense build
// domain (range <= 8 x rows) is split by contiguous key ranges (else by mix64 hash bits),
// keys travel as int32 offsets when the range spans < 2^32 values, build ids as u64 and
// held in place of rows (< 2^31 rows), probe ids as u32 = probe_base + row. Streams: the
// communicator's probe stream runs the probe side's kernels (its partition, the probe),
// its side stream the build side's partition and every collective (one stream for the
// collectives: each rank's GPU runs them in issue order), its build stream the local build.
hj_status run_radix(hj_comm* c, const RadixArgs& a, hj_dist_job* j, int64_t jobno) {
    const int W = c->world, me = c->rank;
    const int kb = a.kt == HJ_INT64 ? 8 : 4;
    hipStream_t s = c->probe, sd = c->side, sb = c->build;
    Scratch scr(c, {s, sd, sb});
    LocalFail lf;
    auto get = [&](size_t bytes, const char* what) -> void* {
        void* p = scr.get(bytes);
        if (!p) lf.note_oom(what);
        return p;
    };
    // the inputs are complete at the caller's stream's point of submission (ev_in)
    HIP_OK(hipStreamWaitEvent(sd, j->ev_in, 0));
    HIP_OK(hipStreamWaitEvent(s, j->ev_in, 0));
    HIP_OK(hipEventRecord(j->ev_t[0], sd));

    // One rank whose build rows start at global row 0: both exchanges are the identity, so
    // the join is the single-GPU build of the build keys in place (on the build stream) and
    // the probe of the probe keys with ids probe_base + row — no partition, no host read.
    if (W == 1 && a.bbase == 0 && a.pkt == a.kt && w1_identity() && !injected(c, jobno, 0)) {
        HIP_OK(hipStreamWaitEvent(sb, j->ev_in, 0));
        // the build span on the build stream itself: the exchange stream (sd) runs nothing on
        // this path, and its start event could complete after a small build finished on sb
        // (build_ms < 0; test_radix_one_rank_paths, r05)
        HIP_OK(hipEventRecord(j->ev_t[0], sb));
        if (a.pbase < 0 || a.pbase + a.np > ((int64_t)1 << 32))
            return set_error(HJ_ERR_INVALID, "hj_dist_join_radix: probe ids (probe_base + row) must fit 32 bits");
        hj_table* t = nullptr;
        ST_OK(hj_build_begin(c->device, 1, a.kt, a.nb, &t));
        j->table = t;  // freed with the job
        ST_OK(hj_build_append(t, 0, a.bkeys, a.bvalid, a.bvoff, nullptr, a.nb,
                              HJ_INPUT_DEVICE | HJ_BORROW | HJ_BORROW_KEEP, sb));
        ST_OK(hj_build_finish(t, 0));
        HIP_OK(hipEventRecord(j->ev_t[2], sb));
        j->info.build_rows = a.nb;
        j->info.recv_rows = a.nb;
        j->info.sharded = 1;
        HIP_OK(hipEventRecord(j->ev_t[1], s));  // no exchange: an empty span on the probe stream
        HIP_OK(hipEventRecord(j->ev_t[3], s));
        j->out_cap = std::max<int64_t>(a.np, 1);
        void* ws = scr.get((size_t)hj_probe_workspace_bytes(a.np));
        uint64_t* ob = (uint64_t*)scr.get((size_t)j->out_cap * 8);
        uint32_t* op = (uint32_t*)scr.get((size_t)j->out_cap * 4);
        int64_t* dt = (int64_t*)scr.get(8);
        if (!ws || !ob || !op || !dt) return set_error(HJ_ERR_OOM, "hj_dist: device allocation failed (probe output)");
        // (the probe waits for the table's build by itself)
        ST_OK(hj_probe_async_base(t, a.pkeys, a.pvalid, a.pvoff, a.np, (uint32_t)a.pbase, ob, op, j->out_cap, dt, ws, s));
        HIP_OK(hipEventRecord(j->ev_t[4], s));
        HIP_OK(hipMemcpyAsync(j->h_total, dt, 8, hipMemcpyDeviceToHost, s));
        HIP_OK(hipEventRecord(j->ev_total, s));
        j->out_b = ob;
        j->out_p = op;
        j->d_total = dt;
        j->rk = a.pkeys;  // a re-probe reads the caller's probe keys (base mode)
        j->rv = a.pvalid;
        j->rvoff = a.pvoff;
        j->pbase = a.pbase;
        j->base_mode = true;
        j->rn = a.np;
        j->ws = ws;
        j->stream = s;
        for (void* p : {(void*)ob, (void*)op, (void*)dt, ws}) scr.give(j, p);
        return scr.defer();
    }

    // 1. the plan: [min | max, rows, failed] of the build side. A rank's own argument
    // errors are noted before the status word is written, so every rank returns them
    // together (a rank returning alone would leave its peers in the next collective).
    const Words w = words_of(c);
    int64_t* mm = w.mm;
    void* mws = w.mws;
    if (a.pbase < 0 || a.pbase + a.np > ((int64_t)1 << 32))
        lf.note(set_error(HJ_ERR_INVALID, "hj_dist_join_radix: probe ids (probe_base + row) must fit 32 bits"));
    if (a.pkt == HJ_INT32 && a.kt == HJ_INT64)
        lf.note(set_error(HJ_ERR_INVALID, "hj_dist_join_radix: int32 probe keys need int32 build keys"));
    if (injected(c, jobno, 0)) lf.note(set_error(HJ_ERR_INVALID, "injected failure (test hook) at the key range"));
    if (!lf.failed) lf.note(hj_key_minmax(a.kt, a.bkeys, a.bvalid, a.bvoff, a.nb, mm, mws, sd));
    {
        int64_t v[4] = {INT64_MAX, INT64_MIN, a.bbase + a.nb, lf.failed ? 1 : 0};
        ST_OK(write_dev(c, lf.failed ? mm : mm + 2, lf.failed ? v : v + 2, lf.failed ? 4 : 2, sd));
    }
    if (W > 1) {
        ST_OK(c->tr->group_start());
        ST_OK(c->tr->allreduce_i64(mm, mm, 1, comm::Red::Min, sd));
        ST_OK(c->tr->allreduce_i64(mm + 1, mm + 1, 3, comm::Red::Max, sd));
        ST_OK(c->tr->group_end(sd));
    }
    ST_OK(read_host(c, mm, 4, sd));
    const int64_t gmin = c->host[0], gmax = c->host[1], rows = c->host[2];
    if (c->host[3] != 0) return lf.raise("the key range");
    j->info.build_rows = rows;
    j->info.sharded = 1;
    if (gmin > gmax) {  // no valid build row anywhere: nothing can match
        j->total = 0;
        j->info.recv_rows = 0;
        HIP_OK(hipEventRecord(j->ev_t[1], sd));
        HIP_OK(hipEventRecord(j->ev_t[2], sd));
        ST_OK(join_streams(c, sd, s, 3));  // (the stage spans stay ordered)
        HIP_OK(hipEventRecord(j->ev_t[3], s));
        HIP_OK(hipEventRecord(j->ev_t[4], s));
        return scr.defer();
    }
    const uint64_t rng_m1 = (uint64_t)gmax - (uint64_t)gmin;
    const bool dense = rng_m1 < (uint64_t)8 * (uint64_t)rows;
    // int64 build keys spanning < 2^32 values travel as int32(key - gmin - 2^31); int32
    // keys as they are. Probe keys travel at the build keys' width: int64 probe keys are
    // narrowed by the same offset (the runtime filter keeps only keys in the build range,
    // so int32 build keys need none); int32 probe keys cannot take an offset.
    const bool narrow = a.kt == HJ_INT64 && rng_m1 < ((uint64_t)1 << 32);
    const int64_t koff = narrow ? (int64_t)((uint64_t)gmin + (1ull << 31)) : 0;
    const int okb = narrow ? 4 : kb;
    const hj_key_type lkt = okb == 8 ? HJ_INT64 : HJ_INT32;
    const int64_t pkoff = a.pkt == HJ_INT64 && okb == 4 ? koff : 0;
    const bool u31 = rows < ((int64_t)1 << 31);
    hj_part_spec spec{dense && W > 1 ? 1 : 0, gmin, gmax};
    int64_t llo = gmin, lhi = gmax;  // this rank's build key range (the whole range under the hash map)
    bool lempty = false;
    if (spec.by_range) lempty = !range_share(gmin, gmax, W, me, &llo, &lhi);
    const hj_part_spec pspec = spec;

    // 2. both sides into per-destination regions; the build side's receive buffers sized
    // by the global rows before the count exchange carries the statuses
    const int64_t bcap = std::max<int64_t>(a.nb, 1), pcap = std::max<int64_t>(a.np, 1);
    int64_t* bcnt = w.cnt;
    int64_t* ballc = w.allc;
    int64_t* pcnt = w.cnt2;
    int64_t* pallc = w.allc2;
    char* brk = (char*)get((size_t)bcap * W * okb, "build regions");
    uint64_t* bri = (uint64_t*)get((size_t)bcap * W * 8, "build regions");
    void* bws = get((size_t)hj_partition_regions_workspace_bytes(a.nb, W), "workspace");
    char* prk = (char*)get((size_t)pcap * W * okb, "probe regions");
    uint32_t* pri = (uint32_t*)get((size_t)pcap * W * 4, "probe regions");
    void* pws = get((size_t)hj_partition_regions_workspace_bytes(a.np, W), "workspace");
    const int64_t rcap = W == 1 ? bcap : recv_slack(rows, W);
    char* bk = W == 1 ? brk : (char*)get((size_t)rcap * okb, "received build keys");
    uint64_t* bi = W == 1 ? bri : (uint64_t*)get((size_t)rcap * 8, "received build ids");
    if (injected(c, jobno, 1)) lf.note(set_error(HJ_ERR_INVALID, "injected failure (test hook) at the partition"));
    if (!lf.failed)
        lf.note(hj_partition_regions(a.kt, a.bkeys, a.bvalid, a.bvoff, nullptr, (uint64_t)a.bbase, a.nb, W, &spec, brk,
                                     okb, koff, bri, 8, bcap, bcnt, bws, sd));
    if (lf.failed) HIP_OK(hipMemsetAsync(bcnt, 0, 8 * (size_t)W, sd));
    {
        int64_t f = lf.failed ? 1 : 0;
        ST_OK(write_dev(c, bcnt + W, &f, 1, sd));
    }
    // the probe side's partition (on s) needs nothing of the build side's but the plan
    if (!lf.failed)
        lf.note(hj_partition_regions(a.pkt, a.pkeys, a.pvalid, a.pvoff, nullptr, (uint64_t)a.pbase, a.np, W, &pspec,
                                     prk, okb, pkoff, pri, 4, pcap, pcnt, pws, s));
    // the build side's counts (the probe side's partition runs meanwhile)
    ST_OK(allgather_read(c, bcnt, ballc, W + 1, sd));
    std::vector<int64_t> mb((size_t)W * W);
    bool anyfail = false;
    for (int src = 0; src < W; ++src) {
        for (int d = 0; d < W; ++d) mb[(size_t)src * W + d] = c->host[(size_t)src * (W + 1) + d];
        anyfail |= c->host[(size_t)src * (W + 1) + W] != 0;
    }
    if (anyfail) return lf.raise("the build-side partition");
    if (!counts_ok(mb, W, me, bcap))
        return set_error(HJ_ERR_HIP, "hj_dist: partition count out of range (device look-back failure)");
    int64_t Rb = 0;
    for (int src = 0; src < W; ++src) Rb += mb[(size_t)src * W + me];
    if (Rb > std::max<int64_t>(rows, 1)) return set_error(HJ_ERR_HIP, "hj_dist: received rows exceed the global rows");
    if (W > 1) ST_OK(grow_recv(c, scr, Rb, rcap, okb, &bk, &bi, "received build rows"));
    HIP_OK(hipEventRecord(j->ev_t[1], sd));  // exchange start
    if (W > 1) {
        ST_OK(c->tr->group_start());
        ST_OK(exchange_regions(c, mb, brk, bcap, okb, bk, sd));
        ST_OK(exchange_regions(c, mb, (const char*)bri, bcap, 8, (char*)bi, sd));
        ST_OK(c->tr->group_end(sd));
    }
    j->info.recv_rows = Rb;
    // 3. the local build (the rank's key range known: no reduction), on its own stream: the
    // collective stream goes on to the probe side's counts without waiting for it
    hj_table* t = nullptr;
    if (injected(c, jobno, 2)) lf.note(set_error(HJ_ERR_INVALID, "injected failure (test hook) at the local build"));
    ST_OK(join_streams(c, sd, sb, 4));
    if (!lf.failed) {
        hj_status st = hj_build_begin(c->device, 1, lkt, Rb, &t);
        const uint32_t fl = HJ_INPUT_DEVICE | HJ_BORROW | HJ_BORROW_KEEP | (u31 ? HJ_IDS_U31 : 0);
        if (st == HJ_OK) st = hj_build_append(t, 0, bk, nullptr, 0, bi, Rb, fl, sb);
        if (st == HJ_OK && Rb > 0 && !lempty) st = hj_build_key_range(t, llo - koff, lhi - koff);
        if (st == HJ_OK) st = hj_build_finish(t, 0);
        lf.note(st);
    }
    j->table = t;  // freed with the job (or taken by the caller)
    HIP_OK(hipEventRecord(j->ev_t[2], sb));  // the build side's end
    // 4. the probe side's counts (+ every rank's status after its local build)
    {
        int64_t f = lf.failed ? 1 : 0;
        ST_OK(write_dev(c, pcnt + W, &f, 1, s));
    }
    if (lf.failed) HIP_OK(hipMemsetAsync(pcnt, 0, 8 * (size_t)W, s));
    ST_OK(join_streams(c, s, sd, 2));
    ST_OK(allgather_read(c, pcnt, pallc, W + 1, sd));
    std::vector<int64_t> mp((size_t)W * W);
    anyfail = false;
    for (int src = 0; src < W; ++src) {
        for (int d = 0; d < W; ++d) mp[(size_t)src * W + d] = c->host[(size_t)src * (W + 1) + d];
        anyfail |= c->host[(size_t)src * (W + 1) + W] != 0;
    }
    if (anyfail) return lf.raise("the probe-side partition or the local builds");
    if (!counts_ok(mp, W, me, pcap))
        return set_error(HJ_ERR_HIP, "hj_dist: partition count out of range (device look-back failure)");
    int64_t Rp = 0;
    for (int src = 0; src < W; ++src) Rp += mp[(size_t)src * W + me];
    // the probe side's receive buffers: exact size, after the last status exchange. A
    // failure here is one-sided: the communicator is aborted (unusable afterwards).
    char* pk = prk;
    uint32_t* pi = pri;
    if (W > 1) {
        pk = (char*)scr.get((size_t)std::max<int64_t>(Rp, 1) * okb);
        pi = (uint32_t*)scr.get((size_t)std::max<int64_t>(Rp, 1) * 4);
        if (!pk || !pi) {
            c->tr->abort();
            c->aborted = true;
            return set_error(HJ_ERR_OOM, "hj_dist_join_radix: device allocation failed (received probe rows); the "
                                         "communicator was aborted");
        }
        ST_OK(c->tr->group_start());
        ST_OK(exchange_regions(c, mp, prk, pcap, okb, pk, sd));
        ST_OK(exchange_regions(c, mp, (const char*)pri, pcap, 4, (char*)pi, sd));
        ST_OK(c->tr->group_end(sd));
    }
    ST_OK(join_streams(c, sd, s, 3));
    HIP_OK(hipEventRecord(j->ev_t[3], s));  // the probe's start
    // 5. the probe of the received rows with their global ids (on s; it waits for the
    // table's build by itself at its first table read: the sliced probe's partition of the
    // received rows overlaps the local build)
    j->rn = Rp;
    j->out_cap = std::max<int64_t>(Rp, 1);
    void* ws = scr.get((size_t)hj_probe_workspace_bytes(Rp));
    uint64_t* ob = (uint64_t*)scr.get((size_t)j->out_cap * 8);
    uint32_t* op = (uint32_t*)scr.get((size_t)j->out_cap * 4);
    int64_t* dt = (int64_t*)scr.get(8);
    if (!ws || !ob || !op || !dt) return set_error(HJ_ERR_OOM, "hj_dist: device allocation failed (probe output)");
    ST_OK(hj_probe_async_ids(t, pk, nullptr, 0, pi, Rp, ob, op, j->out_cap, dt, ws, s));
    HIP_OK(hipEventRecord(j->ev_t[4], s));
    HIP_OK(hipMemcpyAsync(j->h_total, dt, 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipEventRecord(j->ev_total, s));
    j->out_b = ob;
    j->out_p = op;
    j->d_total = dt;
    j->rk = pk;
    j->ri = pi;
    j->ws = ws;
    j->stream = s;
    // the output and what a re-probe reads belong to the job
    for (void* p : {(void*)ob, (void*)op, (void*)dt, ws, (void*)pk, (void*)pi}) scr.give(j, p);
    if (t) {  // the table borrows the received build rows (one rank: its regions)
        scr.give(t, bk);
        scr.give(t, bi);
    }
    return scr.defer();
}

// ---- relational exchanges (TPC-H plans: tpch.q3_dist / q9_dist) --------

// grouped exchange: this rank's rows grouped by destination (m[me][d] rows for peer d, in
// destination order) to their owners; rank src's rows for this rank land at the rows of the
// ranks before src (stable: source rank, then source row order); the own group by a device copy
hj_status exchange_grouped(hj_comm* c, const std::vector<int64_t>& m, const char* grouped, int esz, char* out,
                           hipStream_t s) {
    const int W = c->world, me = c->rank;
    std::vector<int64_t> soff(W, 0), roff(W, 0);
    for (int d = 1; d < W; ++d) soff[d] = soff[d - 1] + m[(size_t)me * W + d - 1];
    for (int src = 1; src < W; ++src) roff[src] = roff[src - 1] + m[(size_t)(src - 1) * W + me];
    const int64_t self = m[(size_t)me * W + me];
    if (self > 0)
        HIP_OK(hipMemcpyAsync(out + roff[me] * esz, grouped + soff[me] * esz, (size_t)self * esz,
                              hipMemcpyDeviceToDevice, s));
    const int64_t per = std::max<int64_t>(1, (int64_t)(kMaxMsgBytes / (size_t)esz));
    for (int p = 0; p < W; ++p) {
        if (p == me) continue;
        const int64_t ns = m[(size_t)me * W + p], nr = m[(size_t)p * W + me];
        for (int64_t a = 0; a < ns; a += per)
            ST_OK(c->tr->send(grouped + (soff[p] + a) * esz, (size_t)std::min(per, ns - a) * esz, p, s));
        for (int64_t a = 0; a < nr; a += per)
            ST_OK(c->tr->recv(out + (roff[p] + a) * esz, (size_t)std::min(per, nr - a) * esz, p, s));
    }
    return HJ_OK;
}

struct ExchangeArgs {
    hj_key_type kt;  // shuffle: the key column's type
    const void* keys;  // shuffle: the key column; gather: null
    int64_t n;
    std::vector<const void*> cols;
    std::vector<int> widths;
};

bool width_ok(int w) { return w == 1 || w == 2 || w == 4 || w == 8 || w == 16; }

// the received buffers: after the last status exchange, so a failure is one-sided and aborts
// the communicator (its peers' transfers would otherwise wait for it forever)
hj_status recv_buffers(hj_comm* c, Scratch& scr, hj_dist_job* j, int64_t R, int kb, const ExchangeArgs& a,
                       char** rk, std::vector<char*>* rc) {
    bool ok = true;
    if (kb) ok = (*rk = (char*)scr.get((size_t)std::max<int64_t>(R, 1) * kb)) != nullptr;
    rc->assign(a.cols.size(), nullptr);
    for (size_t i = 0; ok && i < a.cols.size(); ++i)
        ok = ((*rc)[i] = (char*)scr.get((size_t)std::max<int64_t>(R, 1) * a.widths[i])) != nullptr;
    if (!ok) {
        if (c->tr) c->tr->abort();
        c->aborted = true;
        return set_error(HJ_ERR_OOM, "hj_dist: device allocation failed (received rows); the communicator was aborted");
    }
    if (kb) scr.give(j, *rk);
    for (char* p : *rc) scr.give(j, p);
    j->out_keys = kb ? *rk : nullptr;
    j->out_cols.assign(rc->begin(), rc->end());
    j->out_rows = R;
    return HJ_OK;
}

// Hash repartition of a key column with fixed-width payload columns (DataFusion's
// RepartitionExec Hash over the links): row i goes to rank (mix64 hash bits of its key, the
// hj_partition_rows map) with its payload; received rows in (source rank, source row)
// order. One rank: the rows as they are (copied into the job's buffers).
hj_status run_shuffle(hj_comm* c, const ExchangeArgs& a, hj_dist_job* j, int64_t jobno) {
    const int W = c->world, me = c->rank;
    const int kb = a.kt == HJ_INT64 ? 8 : 4;
    hipStream_t s = c->side;
    HIP_OK(hipStreamWaitEvent(s, j->ev_in, 0));
    Scratch scr(c, {s});
    LocalFail lf;
    auto get = [&](size_t bytes, const char* what) -> void* {
        void* p = scr.get(bytes);
        if (!p) lf.note_oom(what);
        return p;
    };
    const int64_t n = a.n, cap = std::max<int64_t>(n, 1);
    if (W == 1) {
        char* rk = nullptr;
        std::vector<char*> rc;
        ST_OK(recv_buffers(c, scr, j, n, kb, a, &rk, &rc));
        if (n > 0) {
            HIP_OK(hipMemcpyAsync(rk, a.keys, (size_t)n * kb, hipMemcpyDeviceToDevice, s));
            for (size_t i = 0; i < a.cols.size(); ++i)
                HIP_OK(hipMemcpyAsync(rc[i], a.cols[i], (size_t)n * a.widths[i], hipMemcpyDeviceToDevice, s));
        }
        HIP_OK(hipEventRecord(j->ev_total, s));
        return scr.defer();
    }
    // 1. keys grouped by destination, ids = source rows (the stable permutation), each
    // payload column gathered by it; the counts with this rank's status, all-gathered
    const Words w = words_of(c);
    const int ib = n < ((int64_t)1 << 32) ? 4 : 8;
    char* gk = (char*)get((size_t)cap * kb, "grouped keys");
    void* perm = get((size_t)cap * ib, "permutation");
    void* pws = get((size_t)std::max<int64_t>(hj_partition_workspace_bytes(n, W), 8), "workspace");
    std::vector<char*> gc(a.cols.size(), nullptr);
    for (size_t i = 0; i < a.cols.size(); ++i) gc[i] = (char*)get((size_t)cap * a.widths[i], "grouped payload");
    if (injected(c, jobno, 1)) lf.note(set_error(HJ_ERR_INVALID, "injected failure (test hook) at the partition"));
    if (!lf.failed && n > 0)
        lf.note(hj_partition_rows(a.kt, a.keys, nullptr, 0, nullptr, 0, n, W, nullptr, gk, kb, 0, perm, ib, w.cnt,
                                  pws, s));
    for (size_t i = 0; i < a.cols.size() && !lf.failed; ++i)
        if (n > 0) lf.note(hj_gather_fixed(a.cols[i], nullptr, 0, a.widths[i], perm, ib, n, gc[i], nullptr, s));
    if (lf.failed || n == 0) HIP_OK(hipMemsetAsync(w.cnt, 0, 8 * (size_t)W, s));
    {
        int64_t f = lf.failed ? 1 : 0;
        ST_OK(write_dev(c, w.cnt + W, &f, 1, s));
    }
    ST_OK(allgather_read(c, w.cnt, w.allc, W + 1, s));
    std::vector<int64_t> m((size_t)W * W);
    bool anyfail = false;
    for (int src = 0; src < W; ++src) {
        for (int d = 0; d < W; ++d) m[(size_t)src * W + d] = c->host[(size_t)src * (W + 1) + d];
        anyfail |= c->host[(size_t)src * (W + 1) + W] != 0;
    }
    if (anyfail) return lf.raise("the shuffle's partition");
    if (!counts_ok(m, W, me, n)) return set_error(HJ_ERR_HIP, "hj_dist_shuffle: partition count out of range");
    int64_t R = 0;
    for (int src = 0; src < W; ++src) R += m[(size_t)src * W + me];
    // 2. the received rows: keys, then every payload column, per peer in one group
    char* rk = nullptr;
    std::vector<char*> rc;
    ST_OK(recv_buffers(c, scr, j, R, kb, a, &rk, &rc));
    ST_OK(c->tr->group_start());
    ST_OK(exchange_grouped(c, m, gk, kb, rk, s));
    for (size_t i = 0; i < a.cols.size(); ++i) ST_OK(exchange_grouped(c, m, gc[i], a.widths[i], rc[i], s));
    ST_OK(c->tr->group_end(s));
    HIP_OK(hipEventRecord(j->ev_total, s));
    return scr.defer();
}

// Broadcast exchange: every rank receives the concatenation, in rank order, of all ranks'
// rows of the columns (the small filtered dimension sides of a plan, per-rank partial
// results); one all-gather of the row counts, then the columns (an even split in one
// all-gather, else point to point).
hj_status run_gather(hj_comm* c, const ExchangeArgs& a, hj_dist_job* j, int64_t jobno) {
    const int W = c->world;
    hipStream_t s = c->side;
    HIP_OK(hipStreamWaitEvent(s, j->ev_in, 0));
    Scratch scr(c, {s});
    const Words w = words_of(c);
    {
        int64_t v[2] = {a.n, injected(c, jobno, 0) ? 1 : 0};
        ST_OK(write_dev(c, w.st, v, 2, s));
    }
    ST_OK(allgather_read(c, w.st, w.allst, 2, s));
    std::vector<int64_t> lens(W), offs(W, 0);
    bool anyfail = false;
    for (int d = 0; d < W; ++d) {
        lens[d] = c->host[2 * d];
        anyfail |= c->host[2 * d + 1] != 0 || lens[d] < 0;
    }
    if (anyfail) {
        LocalFail lf;
        if (injected(c, jobno, 0)) lf.note(set_error(HJ_ERR_INVALID, "injected failure (test hook) at the gather"));
        return lf.raise("the gather's row counts");
    }
    for (int d = 1; d < W; ++d) offs[d] = offs[d - 1] + lens[d - 1];
    const int64_t R = offs[W - 1] + lens[W - 1];
    char* rk = nullptr;
    std::vector<char*> rc;
    ST_OK(recv_buffers(c, scr, j, R, 0, a, &rk, &rc));
    for (size_t i = 0; i < a.cols.size(); ++i)
        ST_OK(allgather_var(c, rc[i], offs, lens, (const char*)a.cols[i], a.widths[i], s));
    HIP_OK(hipEventRecord(j->ev_total, s));
    return scr.defer();
}

// ---- the worker ----------------------------------------------------------------------------

void worker_loop(hj_comm* c) {
    (void)hipSetDevice(c->device);
    for (;;) {
        hj_dist_job* j = nullptr;
        {
            std::unique_lock<std::mutex> g(c->qmu);
            c->qcv.wait(g, [c] { return c->stop || !c->q.empty(); });
            if (c->q.empty()) return;  // stop requested and nothing queued
            j = c->q.front();
            c->q.pop_front();
        }
        release_finished(c, false);
        hj_status st = c->aborted ? set_error(HJ_ERR_RCCL, "hj_dist: the communicator was aborted after an earlier "
                                                           "one-sided failure")
                                  : j->fn(j);
        std::string err;
        if (st != HJ_OK) {
            const char* e = hj_last_error();
            err = e ? e : "";
        }
        {
            std::lock_guard<std::mutex> g(j->mu);
            j->st = st;
            j->err = std::move(err);
            j->done = true;
        }
        j->cv.notify_all();
    }
}

hj_status submit(hj_comm* c, hj_dist_job* j) {
    {
        std::lock_guard<std::mutex> g(c->qmu);
        if (c->stop) return set_error(HJ_ERR_INVALID, "hj_dist: communicator is being freed");
        c->q.push_back(j);
    }
    c->qcv.notify_one();
    return HJ_OK;
}

// wait for the job's host steps; -> its status (the message set on this thread)
hj_status wait_job(hj_dist_job* j) {
    std::unique_lock<std::mutex> g(j->mu);
    j->cv.wait(g, [j] { return j->done; });
    if (j->st != HJ_OK) return set_error(j->st, j->err);
    return HJ_OK;
}

hj_status new_job(hj_comm* c, bool join, void* stream, hj_dist_job** out) {
    hj_dist_job* j = new hj_dist_job();
    j->comm = c;
    j->device = c->device;
    // the caller's stream at submission: the job's device work follows it
    bool ok = hipSetDevice(c->device) == hipSuccess &&
              hipEventCreateWithFlags(&j->ev_in, hipEventDisableTiming) == hipSuccess &&
              hipEventRecord(j->ev_in, (hipStream_t)stream) == hipSuccess;
    if (join) {  // the pairs' count word and the stage events
        ok = hipHostMalloc((void**)&j->h_total, 8, hipHostMallocDefault) == hipSuccess &&
             hipEventCreateWithFlags(&j->ev_total, hipEventDisableTiming) == hipSuccess;
        for (auto& e : j->ev_t) ok = ok && hipEventCreate(&e) == hipSuccess;
    }
    if (!ok) {
        hj_dist_job_free(j);
        return set_error(HJ_ERR_HIP, "hj_dist: job events / pinned word");
    }
    *out = j;
    return HJ_OK;
}

hj_status check_comm(hj_comm* c) {
    if (c == nullptr) return set_error(HJ_ERR_INVALID, "null communicator");
    if (c->aborted) return set_error(HJ_ERR_RCCL, "hj_dist: the communicator was aborted");
    return HJ_OK;
}

}  // namespace

namespace dfp {
namespace comm {
bool range_share_of(int64_t gmin, int64_t gmax, int W, int r, int64_t* lo, int64_t* hi) {
    return range_share(gmin, gmax, W, r, lo, hi);
}
hj_status start(hj_comm* c) {
    HIP_OK(hipSetDevice(c->device));
    // DFP_HJ_COMM_PRIORITY=-1: the plan's own streams at high priority (their kernels are
    // the host chain's critical path; measured)
    const char* pe = getenv("DFP_HJ_COMM_PRIORITY");
    const int prio = pe ? atoi(pe) : 0;
    if (hipHostMalloc((void**)&c->host, 2 * kHostWords * 8, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, prio) != hipSuccess ||
        hipStreamCreateWithPriority(&c->build, hipStreamNonBlocking, prio) != hipSuccess ||
        hipStreamCreateWithPriority(&c->probe, hipStreamNonBlocking, prio) != hipSuccess)
        return set_error(HJ_ERR_HIP, "hj_comm: pinned mailbox / event / streams");
    if (hipMalloc((void**)&c->words, words_bytes(c->world)) != hipSuccess) {
        c->words = nullptr;
        return set_error(HJ_ERR_OOM, "hj_comm: the plans' device words");
    }
    c->evs.assign(kEvents, nullptr);
    for (auto& e : c->evs)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
            return set_error(HJ_ERR_HIP, "hj_comm: events");
    c->worker = std::thread(worker_loop, c);
    return HJ_OK;
}
}  // namespace comm
}  // namespace dfp

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
    if (world > 1) {
        auto tr = std::make_unique<RcclTransport>();
        ncclUniqueId u;
        memcpy(u.internal, id, HJ_COMM_ID_BYTES);
        const ncclResult_t r = ncclCommInitRank(&tr->comm, world, u, rank);
        if (r != ncclSuccess) {
            tr->comm = nullptr;
            hj_comm_free(c);
            return set_error(HJ_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        }
        c->tr = std::move(tr);
    }
    hj_status st = dfp::comm::start(c);
    if (st != HJ_OK) {
        const std::string msg = hj_last_error() ? hj_last_error() : "";
        hj_comm_free(c);
        return set_error(st, msg);
    }
    *out = c;
    return HJ_OK;
}

void hj_comm_free(hj_comm* c) {
    if (c == nullptr) return;
    {
        std::lock_guard<std::mutex> g(c->qmu);
        c->stop = true;
    }
    c->qcv.notify_all();
    if (c->worker.joinable()) c->worker.join();
    (void)hipSetDevice(c->device);
    if (c->side) (void)hipStreamSynchronize(c->side);
    if (c->build) (void)hipStreamSynchronize(c->build);
    if (c->probe) (void)hipStreamSynchronize(c->probe);
    release_finished(c, true);
    c->tr.reset();
    for (auto e : c->evs)
        if (e) (void)hipEventDestroy(e);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->build) (void)hipStreamDestroy(c->build);
    if (c->probe) (void)hipStreamDestroy(c->probe);
    if (c->ev) (void)hipEventDestroy(c->ev);
    if (c->host) (void)hipHostFree(c->host);
    if (c->words) (void)hipFree(c->words);
    delete c;
}

hj_status hj_dist_build_sharded_async(hj_comm* c, hj_key_type key_type, const void* keys, const uint8_t* validity,
                                      int64_t voff, int64_t n, int64_t build_base, hj_key_type probe_key_type,
                                      void* stream, hj_dist_job** out) {
    if (out == nullptr) return set_error(HJ_ERR_INVALID, "null out");
    *out = nullptr;
    ST_OK(check_comm(c));
    if (key_type != HJ_INT32 && key_type != HJ_INT64) return set_error(HJ_ERR_INVALID, "unsupported key type");
    if (probe_key_type != HJ_INT32 && probe_key_type != HJ_INT64)
        return set_error(HJ_ERR_INVALID, "unsupported probe key type");
    if (n < 0 || build_base < 0 || voff < 0) return set_error(HJ_ERR_INVALID, "negative n/base/offset");
    if (n > 0 && keys == nullptr) return set_error(HJ_ERR_INVALID, "null keys");
    hj_dist_job* j = nullptr;
    ST_OK(new_job(c, false, stream, &j));
    const ShardedArgs a{key_type, probe_key_type, keys, validity, voff, n, build_base, (hipStream_t)stream};
    const int64_t no = c->jobs++;
    j->fn = [c, a, no](hj_dist_job* jj) { return run_sharded(c, a, jj, no); };
    hj_status st = submit(c, j);
    if (st != HJ_OK) {
        hj_dist_job_free(j);
        return st;
    }
    *out = j;
    return HJ_OK;
}

hj_status hj_dist_build_sharded(hj_comm* c, hj_key_type key_type, const void* keys, const uint8_t* validity,
                                int64_t voff, int64_t n, int64_t build_base, hj_key_type probe_key_type, void* stream,
                                hj_table** out, hj_dist_info* info) {
    if (out == nullptr) return set_error(HJ_ERR_INVALID, "null out");
    *out = nullptr;
    hj_dist_job* j = nullptr;
    ST_OK(hj_dist_build_sharded_async(c, key_type, keys, validity, voff, n, build_base, probe_key_type, stream, &j));
    hj_status st = hj_dist_job_table(j, out, info);
    hj_dist_job_free(j);
    return st;
}

hj_status hj_dist_join_radix(hj_comm* c, hj_key_type build_key_type, const void* build_keys,
                             const uint8_t* build_validity, int64_t build_voff, int64_t nb, int64_t build_base,
                             hj_key_type probe_key_type, const void* probe_keys, const uint8_t* probe_validity,
                             int64_t probe_voff, int64_t np, int64_t probe_base, void* stream, hj_dist_job** out) {
    if (out == nullptr) return set_error(HJ_ERR_INVALID, "null out");
    *out = nullptr;
    ST_OK(check_comm(c));
    for (hj_key_type k : {build_key_type, probe_key_type})
        if (k != HJ_INT32 && k != HJ_INT64) return set_error(HJ_ERR_INVALID, "unsupported key type");
    if (nb < 0 || np < 0 || build_base < 0 || probe_base < 0 || build_voff < 0 || probe_voff < 0)
        return set_error(HJ_ERR_INVALID, "negative rows/base/offset");
    if ((nb > 0 && build_keys == nullptr) || (np > 0 && probe_keys == nullptr))
        return set_error(HJ_ERR_INVALID, "null keys");
    hj_dist_job* j = nullptr;
    ST_OK(new_job(c, true, stream, &j));
    const RadixArgs a{build_key_type, probe_key_type, build_keys, probe_keys, build_validity, probe_validity,
                      build_voff, nb, build_base, probe_voff, np, probe_base, (hipStream_t)stream};
    const int64_t no = c->jobs++;
    j->fn = [c, a, no](hj_dist_job* jj) { return run_radix(c, a, jj, no); };
    hj_status st = submit(c, j);
    if (st != HJ_OK) {
        hj_dist_job_free(j);
        return st;
    }
    *out = j;
    return HJ_OK;
}

hj_status hj_dist_shuffle(hj_comm* c, hj_key_type key_type, const void* keys, int64_t n, int ncols,
                          const void* const* cols, const int* col_bytes, void* stream, hj_dist_job** out) {
    if (out == nullptr) return set_error(HJ_ERR_INVALID, "null out");
    *out = nullptr;
    ST_OK(check_comm(c));
    if (key_type != HJ_INT32 && key_type != HJ_INT64) return set_error(HJ_ERR_INVALID, "unsupported key type");
    if (n < 0 || ncols < 0 || (ncols > 0 && (cols == nullptr || col_bytes == nullptr)))
        return set_error(HJ_ERR_INVALID, "negative n/ncols or null columns");
    if (n > 0 && keys == nullptr) return set_error(HJ_ERR_INVALID, "null keys");
    if ((c->world & (c->world - 1)) != 0 || c->world > 64)
        return set_error(HJ_ERR_INVALID, "hj_dist_shuffle: the hash map needs a power-of-two world <= 64");
    ExchangeArgs a{key_type, keys, n, {}, {}};
    for (int i = 0; i < ncols; ++i) {
        if (!width_ok(col_bytes[i])) return set_error(HJ_ERR_INVALID, "payload column width must be 1/2/4/8/16 bytes");
        if (n > 0 && cols[i] == nullptr) return set_error(HJ_ERR_INVALID, "null payload column");
        a.cols.push_back(cols[i]);
        a.widths.push_back(col_bytes[i]);
    }
    hj_dist_job* j = nullptr;
    ST_OK(new_job(c, true, stream, &j));
    const int64_t no = c->jobs++;
    j->fn = [c, a, no](hj_dist_job* jj) { return run_shuffle(c, a, jj, no); };
    hj_status st = submit(c, j);
    if (st != HJ_OK) {
        hj_dist_job_free(j);
        return st;
    }
    *out = j;
    return HJ_OK;
}

hj_status hj_dist_gather(hj_comm* c, int64_t n, int ncols, const void* const* cols, const int* col_bytes,
                         void* stream, hj_dist_job** out) {
    if (out == nullptr) return set_error(HJ_ERR_INVALID, "null out");
    *out = nullptr;
    ST_OK(check_comm(c));
    if (n < 0 || ncols < 1 || cols == nullptr || col_bytes == nullptr)
        return set_error(HJ_ERR_INVALID, "negative n or no columns");
    ExchangeArgs a{HJ_INT64, nullptr, n, {}, {}};
    for (int i = 0; i < ncols; ++i) {
        if (!width_ok(col_bytes[i])) return set_error(HJ_ERR_INVALID, "column width must be 1/2/4/8/16 bytes");
        if (n > 0 && cols[i] == nullptr) return set_error(HJ_ERR_INVALID, "null column");
        a.cols.push_back(cols[i]);
        a.widths.push_back(col_bytes[i]);
    }
    hj_dist_job* j = nullptr;
    ST_OK(new_job(c, true, stream, &j));
    const int64_t no = c->jobs++;
    j->fn = [c, a, no](hj_dist_job* jj) { return run_gather(c, a, jj, no); };
    hj_status st = submit(c, j);
    if (st != HJ_OK) {
        hj_dist_job_free(j);
        return st;
    }
    *out = j;
    return HJ_OK;
}

hj_status hj_dist_job_columns(hj_dist_job* j, void* stream, const void** keys, const void** cols, int ncols,
                              int64_t* rows) {
    if (j == nullptr || rows == nullptr || (ncols > 0 && cols == nullptr)) return set_error(HJ_ERR_INVALID, "null args");
    ST_OK(wait_job(j));
    if (j->out_rows < 0) return set_error(HJ_ERR_INVALID, "hj_dist_job_columns: not an exchange job");
    if ((size_t)ncols != j->out_cols.size()) return set_error(HJ_ERR_INVALID, "hj_dist_job_columns: column count");
    HIP_OK(hipSetDevice(j->device));
    HIP_OK(hipStreamWaitEvent((hipStream_t)stream, j->ev_total, 0));  // consumers on `stream` follow the exchange
    if (keys) *keys = j->out_keys;
    for (int i = 0; i < ncols; ++i) cols[i] = j->out_cols[(size_t)i];
    *rows = j->out_rows;
    return HJ_OK;
}

hj_status hj_dist_job_wait(hj_dist_job* j, hj_dist_info* info) {
    if (j == nullptr) return set_error(HJ_ERR_INVALID, "null job");
    ST_OK(wait_job(j));
    if (info) *info = j->info;
    return HJ_OK;
}

hj_status hj_dist_job_table(hj_dist_job* j, hj_table** out, hj_dist_info* info) {
    if (j == nullptr || out == nullptr) return set_error(HJ_ERR_INVALID, "null job/out");
    *out = nullptr;
    ST_OK(wait_job(j));
    if (j->table_taken || j->table == nullptr) return set_error(HJ_ERR_INVALID, "hj_dist_job_table: no table to take");
    *out = j->table;
    j->table_taken = true;
    if (info) *info = j->info;
    return HJ_OK;
}

hj_status hj_dist_job_pairs(hj_dist_job* j, const uint64_t** build_idx, const uint32_t** probe_idx, int64_t* count) {
    if (j == nullptr || count == nullptr) return set_error(HJ_ERR_INVALID, "null job/count");
    ST_OK(wait_job(j));
    if (j->total < 0) {
        if (j->d_total == nullptr) return set_error(HJ_ERR_INVALID, "hj_dist_job_pairs: not a join job");
        HIP_OK(hipSetDevice(j->device));
        HIP_OK(hipEventSynchronize(j->ev_total));
        int64_t total = *j->h_total;
        if (total > j->out_cap) {  // duplicate-heavy keys: once more with the exact size
            void* ob = dfp::host::dev_block(j->device, (size_t)total * 8);
            void* op = dfp::host::dev_block(j->device, (size_t)total * 4);
            if (!ob || !op) {
                if (ob) dfp::host::free_block(j->device, ob, (size_t)total * 8);
                if (op) dfp::host::free_block(j->device, op, (size_t)total * 4);
                return set_error(HJ_ERR_OOM, "hj_dist_job_pairs: device allocation failed");
            }
            j->blocks.emplace_back(ob, (size_t)total * 8);
            j->blocks.emplace_back(op, (size_t)total * 4);
            if (j->table_taken) return set_error(HJ_ERR_INVALID, "hj_dist_job_pairs: re-probe needs the job's table");
            if (j->base_mode)
                ST_OK(hj_probe_async_base(j->table, j->rk, j->rv, j->rvoff, j->rn, (uint32_t)j->pbase, (uint64_t*)ob,
                                          (uint32_t*)op, total, j->d_total, j->ws, j->stream));
            else
                ST_OK(hj_probe_async_ids(j->table, j->rk, nullptr, 0, j->ri, j->rn, (uint64_t*)ob, (uint32_t*)op,
                                         total, j->d_total, j->ws, j->stream));
            HIP_OK(hipMemcpyAsync(j->h_total, j->d_total, 8, hipMemcpyDeviceToHost, j->stream));
            HIP_OK(hipEventRecord(j->ev_total, j->stream));
            HIP_OK(hipEventSynchronize(j->ev_total));
            j->out_b = (uint64_t*)ob;
            j->out_p = (uint32_t*)op;
            j->out_cap = total;
            total = *j->h_total;
        }
        j->total = total;
    }
    if (build_idx) *build_idx = j->out_b;
    if (probe_idx) *probe_idx = j->out_p;
    *count = j->total;
    return HJ_OK;
}

hj_status hj_dist_job_times(hj_dist_job* j, double* build_ms, double* exchange_ms, double* probe_ms) {
    if (j == nullptr) return set_error(HJ_ERR_INVALID, "null job");
    ST_OK(wait_job(j));
    HIP_OK(hipSetDevice(j->device));
    auto span = [](hipEvent_t a, hipEvent_t b, double* out) -> hj_status {
        if (out == nullptr) return HJ_OK;
        float ms = 0;
        HIP_OK(hipEventSynchronize(b));
        HIP_OK(hipEventElapsedTime(&ms, a, b));
        *out = ms;
        return HJ_OK;
    };
    if (j->ev_t[0] == nullptr) {  // a sharded build side: its table's build time
        if (build_ms) *build_ms = j->table ? (double)hj_table_build_ns(j->table) / 1e6 : 0.0;
        if (exchange_ms) *exchange_ms = 0;
        if (probe_ms) *probe_ms = 0;
        return HJ_OK;
    }
    ST_OK(span(j->ev_t[0], j->ev_t[2], build_ms));
    ST_OK(span(j->ev_t[1], j->ev_t[3], exchange_ms));
    ST_OK(span(j->ev_t[3], j->ev_t[4], probe_ms));
    return HJ_OK;
}

void hj_dist_job_free(hj_dist_job* j) {
    if (j == nullptr) return;
    if (j->fn) {  // submitted: wait for the worker to finish it
        std::unique_lock<std::mutex> g(j->mu);
        j->cv.wait(g, [j] { return j->done; });
    }
    (void)hipSetDevice(j->device);
    // this job's own device work only (its probe stream is the communicator's: a later job's
    // work may already be queued behind it there)
    if (j->ev_total) (void)hipEventSynchronize(j->ev_total);
    if (j->table && !j->table_taken) hj_table_free(j->table);
    for (auto& b : j->blocks) dfp::host::free_block(j->device, b.first, b.second);
    for (auto e : j->ev_t)
        if (e) (void)hipEventDestroy(e);
    if (j->ev_total) (void)hipEventDestroy(j->ev_total);
    if (j->ev_in) (void)hipEventDestroy(j->ev_in);
    if (j->h_total) (void)hipHostFree(j->h_total);
    delete j;
}

}  // extern "C"
