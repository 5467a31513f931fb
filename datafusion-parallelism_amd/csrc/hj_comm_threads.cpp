// hj_comm_threads.cpp — TEST LIBRARY ONLY (lib/libdfp_hj_commtest.so; never linked into
// the product library lib/libdfp_hj.so). An in-process transport for hj_comm: W ranks are
// threads of one process (on one GPU or several), a host barrier stands for the
// interconnect and device copies move the data. It runs hj_dist.cpp's multi-rank code
// (the plans' count matrices, exchanges, uneven all-gathers, segment rebases, status
// words) at W = 2 / 4 / 8 where only one GPU is available, since RCCL refuses two ranks on
// one device. It also checks what RCCL would only hang on: every rank must issue the same
// collectives with the same sizes, and each receive must meet a send of the same size.
//
// A group runs when its last call is issued: every rank synchronizes its stream, posts its
// calls and meets the others at a barrier; each rank stages what it receives (device to
// host) from its peers' send buffers; a second barrier; each rank writes its received
// data into its own buffers (host to device) and synchronizes its stream. The barrier
// times out (the caller's bound) instead of hanging when a rank stops issuing.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hj.h"
#include "hj_comm.h"
#include "hj_host.h"

using dfp::host::set_error;

namespace {

enum class Kind { AllReduce, AllGather, Send, Recv };

struct Op {
    Kind k;
    const void* sbuf;
    void* rbuf;
    size_t bytes;  // per rank (allgather), of the message (send/recv), count * 8 (allreduce)
    dfp::comm::Red red;
    int peer;
};

}  // namespace

struct hj_test_hub {
    int world = 1;
    double timeout_s = 60;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    int64_t gen = 0;
    bool broken = false;
    std::vector<const std::vector<Op>*> slots;
    // each rank's posted group, owned by the hub (not the posting call's stack): a peer that is
    // still staging from it when the rank's second barrier times out reads valid memory
    std::vector<std::vector<Op>> posted;
};

namespace {

// -> false after the timeout (the hub is then broken: every later barrier fails at once)
bool barrier(hj_test_hub* h) {
    std::unique_lock<std::mutex> g(h->mu);
    if (h->broken) return false;
    const int64_t my = h->gen;
    if (++h->arrived == h->world) {
        h->arrived = 0;
        ++h->gen;
        h->cv.notify_all();
        return true;
    }
    const auto until = std::chrono::steady_clock::now() + std::chrono::duration<double>(h->timeout_s);
    while (h->gen == my && !h->broken)
        if (h->cv.wait_until(g, until) == std::cv_status::timeout && h->gen == my) {
            h->broken = true;
            h->cv.notify_all();
            return false;
        }
    return !h->broken || h->gen != my;
}

struct ThreadTransport final : dfp::comm::Transport {
    hj_test_hub* hub;
    int rank;
    int depth = 0;
    std::vector<Op> pending;
    ThreadTransport(hj_test_hub* h, int r) : hub(h), rank(r) {}

    hj_status group_start() override {
        ++depth;
        return HJ_OK;
    }
    hj_status group_end(hipStream_t s) override {
        if (depth == 0) return set_error(HJ_ERR_RCCL, "thread transport: group_end without group_start");
        if (--depth > 0) return HJ_OK;
        return flush(s);
    }
    hj_status add(const Op& op, hipStream_t s) {
        pending.push_back(op);
        return depth == 0 ? flush(s) : HJ_OK;
    }
    hj_status allreduce_i64(const int64_t* send, int64_t* recv, size_t count, dfp::comm::Red op,
                            hipStream_t s) override {
        return add(Op{Kind::AllReduce, send, recv, count * 8, op, -1}, s);
    }
    hj_status allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        return add(Op{Kind::AllGather, send, recv, bytes, dfp::comm::Red::Min, -1}, s);
    }
    hj_status send(const void* buf, size_t bytes, int peer, hipStream_t s) override {
        if (peer < 0 || peer >= hub->world || peer == rank) return set_error(HJ_ERR_RCCL, "thread transport: bad peer");
        return add(Op{Kind::Send, buf, nullptr, bytes, dfp::comm::Red::Min, peer}, s);
    }
    hj_status recv(void* buf, size_t bytes, int peer, hipStream_t s) override {
        if (peer < 0 || peer >= hub->world || peer == rank) return set_error(HJ_ERR_RCCL, "thread transport: bad peer");
        return add(Op{Kind::Recv, nullptr, buf, bytes, dfp::comm::Red::Min, peer}, s);
    }

    hj_status flush(hipStream_t s) {
        if (hipStreamSynchronize(s) != hipSuccess) return set_error(HJ_ERR_HIP, "thread transport: stream sync");
        const int W = hub->world;
        {
            std::lock_guard<std::mutex> g(hub->mu);
            if (hub->broken) {
                pending.clear();
                return set_error(HJ_ERR_RCCL, "thread transport: the hub broke at an earlier timeout");
            }
            hub->posted[(size_t)rank].swap(pending);
            pending.clear();
            hub->slots[(size_t)rank] = &hub->posted[(size_t)rank];
        }
        const std::vector<Op>& ops = hub->posted[(size_t)rank];
        if (!barrier(hub)) return set_error(HJ_ERR_RCCL, "thread transport: barrier timeout (a rank did not reach the collective)");
        // validate: the same collectives everywhere; every receive meets a send of its size
        std::string bad;
        std::vector<const Op*> mine_coll;
        for (const Op& o : ops)
            if (o.k == Kind::AllReduce || o.k == Kind::AllGather) mine_coll.push_back(&o);
        for (int q = 0; q < W && bad.empty(); ++q) {
            std::vector<const Op*> qc;
            for (const Op& o : *hub->slots[(size_t)q])
                if (o.k == Kind::AllReduce || o.k == Kind::AllGather) qc.push_back(&o);
            if (qc.size() != mine_coll.size()) bad = "ranks issued different numbers of collectives in a group";
            for (size_t i = 0; i < qc.size() && bad.empty(); ++i)
                if (qc[i]->k != mine_coll[i]->k || qc[i]->bytes != mine_coll[i]->bytes ||
                    (qc[i]->k == Kind::AllReduce && qc[i]->red != mine_coll[i]->red))
                    bad = "ranks issued different collectives (kind, size or operation)";
        }
        // each (peer, direction): the k-th receive from p meets p's k-th send to me
        std::vector<std::vector<const Op*>> from(W), to(W);  // my recvs from p / p's sends to me
        for (const Op& o : ops)
            if (o.k == Kind::Recv) from[(size_t)o.peer].push_back(&o);
        for (int p = 0; p < W; ++p)
            for (const Op& o : *hub->slots[(size_t)p])
                if (o.k == Kind::Send && o.peer == rank) to[(size_t)p].push_back(&o);
        for (int p = 0; p < W && bad.empty(); ++p) {
            if (from[(size_t)p].size() != to[(size_t)p].size()) bad = "a receive without its send (or the reverse)";
            for (size_t i = 0; i < from[(size_t)p].size() && bad.empty(); ++i)
                if (from[(size_t)p][i]->bytes != to[(size_t)p][i]->bytes) bad = "a receive and its send differ in size";
        }
        // my sends must be received too (the peer checks the same pairs from its side)
        for (const Op& o : ops)
            if (o.k == Kind::Send && bad.empty()) {
                size_t mine_k = 0, theirs = 0;
                for (const Op& x : ops)
                    if (x.k == Kind::Send && x.peer == o.peer) ++mine_k;
                for (const Op& x : *hub->slots[(size_t)o.peer])
                    if (x.k == Kind::Recv && x.peer == rank) ++theirs;
                if (mine_k != theirs) bad = "a send without its receive";
            }
        // stage what this rank receives
        std::vector<std::vector<char>> staged(ops.size());
        hj_status st = HJ_OK;
        auto d2h = [&](void* dst, const void* src, size_t n) {
            if (n == 0 || st != HJ_OK) return;
            if (hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
                st = set_error(HJ_ERR_HIP, "thread transport: staging copy failed");
        };
        bool broken_now;
        {
            std::lock_guard<std::mutex> g(hub->mu);
            broken_now = hub->broken;  // a broken hub stages nothing more
        }
        if (bad.empty() && !broken_now) {
            size_t ci = 0;
            std::vector<size_t> ri(W, 0);
            for (size_t i = 0; i < ops.size(); ++i) {
                const Op& o = ops[i];
                if (o.k == Kind::AllReduce || o.k == Kind::AllGather) {
                    staged[i].resize(o.bytes * (size_t)W);
                    for (int q = 0; q < W; ++q) {
                        std::vector<const Op*> qc;
                        for (const Op& x : *hub->slots[(size_t)q])
                            if (x.k == Kind::AllReduce || x.k == Kind::AllGather) qc.push_back(&x);
                        d2h(staged[i].data() + (size_t)q * o.bytes, qc[ci]->sbuf, o.bytes);
                    }
                    ++ci;
                } else if (o.k == Kind::Recv) {
                    const Op* snd = to[(size_t)o.peer][ri[(size_t)o.peer]++];
                    staged[i].resize(o.bytes);
                    d2h(staged[i].data(), snd->sbuf, o.bytes);
                }
            }
        }
        if (!barrier(hub)) return set_error(HJ_ERR_RCCL, "thread transport: barrier timeout");
        if (!bad.empty()) return set_error(HJ_ERR_RCCL, "thread transport: " + bad);
        if (st != HJ_OK) return st;
        // write what this rank received into its own buffers
        for (size_t i = 0; i < ops.size(); ++i) {
            const Op& o = ops[i];
            const void* src = staged[i].data();
            std::vector<int64_t> red;
            size_t n = staged[i].size();
            if (o.k == Kind::AllReduce) {
                const size_t cnt = o.bytes / 8;
                red.resize(cnt);
                const int64_t* v = reinterpret_cast<const int64_t*>(staged[i].data());
                for (size_t e = 0; e < cnt; ++e) {
                    int64_t acc = v[e];
                    for (int q = 1; q < W; ++q) {
                        const int64_t x = v[(size_t)q * cnt + e];
                        acc = o.red == dfp::comm::Red::Min ? std::min(acc, x) : std::max(acc, x);
                    }
                    red[e] = acc;
                }
                src = red.data();
                n = o.bytes;
            } else if (o.k == Kind::Send) {
                continue;
            }
            if (n > 0 && (hipMemcpyAsync(o.rbuf, src, n, hipMemcpyHostToDevice, s) != hipSuccess ||
                          hipStreamSynchronize(s) != hipSuccess))
                return set_error(HJ_ERR_HIP, "thread transport: write copy failed");
        }
        return HJ_OK;
    }
};

}  // namespace

extern "C" {

hj_test_hub* hj_test_hub_create(int world, double timeout_s) {
    if (world < 1) return nullptr;
    hj_test_hub* h = new hj_test_hub();
    h->world = world;
    h->timeout_s = timeout_s > 0 ? timeout_s : 60;
    h->slots.assign((size_t)world, nullptr);
    h->posted.assign((size_t)world, {});
    return h;
}

void hj_test_hub_free(hj_test_hub* h) { delete h; }

// one rank's communicator over the hub (world > 1: the thread transport; 1: none, as RCCL)
hj_status hj_test_comm_create(hj_test_hub* h, int rank, int device, hj_comm** out) {
    if (h == nullptr || out == nullptr || rank < 0 || rank >= h->world) return set_error(HJ_ERR_INVALID, "bad args");
    *out = nullptr;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return set_error(HJ_ERR_NO_DEVICE, "no GPU visible");
    if (device < 0 || device >= nd) return set_error(HJ_ERR_INVALID, "bad device ordinal");
    hj_comm* c = new hj_comm();
    c->rank = rank;
    c->world = h->world;
    c->device = device;
    if (h->world > 1) c->tr = std::make_unique<ThreadTransport>(h, rank);
    hj_status st = dfp::comm::start(c);
    if (st != HJ_OK) {
        const std::string msg = hj_last_error() ? hj_last_error() : "";
        hj_comm_free(c);
        return set_error(st, msg);
    }
    *out = c;
    return HJ_OK;
}

// host only (no GPU): the sharded plan's key-range share of rank r (hj_dist.cpp's
// range_share), for the CPU test that checks it against the Python plan's
// ExchangePlan.local_key_range; -> 1 and [*lo, *hi], or 0 when the share is empty
int hj_test_range_share(int64_t gmin, int64_t gmax, int world, int rank, int64_t* lo, int64_t* hi) {
    return dfp::comm::range_share_of(gmin, gmax, world, rank, lo, hi) ? 1 : 0;
}

// the rank's plan fails (locally) at step `step` (0 key range, 1 partition, 2 local build)
// of its job number `job` (0-based, in submission order)
void hj_test_comm_fail_at(hj_comm* c, int job, int step) {
    if (c) c->fail_at = job < 0 ? -1 : job * 8 + step;
}

}  // extern "C"
