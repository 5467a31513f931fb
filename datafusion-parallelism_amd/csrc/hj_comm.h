// hj_comm.h — the communicator behind hj_comm_* / hj_dist_* (internal; not part of the C
// ABI). Its collectives go through a Transport chosen when the communicator is made:
// RCCL (ncclComm_t over xGMI, hj_comm_create) in the product library, or the in-process
// thread transport of the test library (hj_comm_threads.cpp: W ranks as threads of one
// process, host barrier + device copies), so that every multi-rank code path of
// hj_dist.cpp runs at W > 1 in tests on one GPU.
//
// A communicator runs its plan steps on one worker thread (a job queue): the C entry
// points enqueue a job and return, the caller waits for the job's result only when it
// needs the table or the pairs. The plan's small host reads (key range, count matrix,
// segment sizes) therefore wait on the worker, not on the caller's thread.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/hj.h"

namespace dfp {
namespace comm {

enum class Red { Min, Max };

// Stream-ordered collectives of one rank. Calls between group_start and group_end are one
// group (RCCL semantics: a group's point-to-point calls progress together); a call outside
// a group is a group of its own. Every rank issues the same sequence.
struct Transport {
    virtual ~Transport() = default;
    virtual hj_status group_start() = 0;
    virtual hj_status group_end(hipStream_t s) = 0;
    virtual hj_status allreduce_i64(const int64_t* send, int64_t* recv, size_t count, Red op, hipStream_t s) = 0;
    // recv[d * bytes .. (d + 1) * bytes) = rank d's send (send may lie inside recv at slot me)
    virtual hj_status allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
    virtual hj_status send(const void* buf, size_t bytes, int peer, hipStream_t s) = 0;
    virtual hj_status recv(void* buf, size_t bytes, int peer, hipStream_t s) = 0;
    // make the communicator unusable after a one-sided failure (RCCL: ncclCommAbort)
    virtual void abort() {}
};

}  // namespace comm
}  // namespace dfp

// one queued plan step (hj_dist_job in the C ABI)
struct hj_dist_job {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    hj_status st = HJ_OK;
    std::string err;
    std::function<hj_status(hj_dist_job*)> fn;
    // results
    hj_table* table = nullptr;  // sharded: the whole build side's table; radix: the local shard
    bool table_taken = false;
    hj_dist_info info{};
    // radix: the rank's pairs (device, job-owned) and what a re-probe needs
    uint64_t* out_b = nullptr;
    uint32_t* out_p = nullptr;
    int64_t out_cap = 0;
    int64_t* d_total = nullptr;  // device
    int64_t* h_total = nullptr;  // pinned
    hipEvent_t ev_total = nullptr;
    hipEvent_t ev_in = nullptr;  // the caller's stream at submission (the inputs are complete there)
    int64_t total = -1;
    // radix: timing events (build side start, exchange start, build side end, probe start,
    // probe end); null for a sharded build side (its table's build time covers it)
    hipEvent_t ev_t[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    const void* rk = nullptr;  // received probe keys / ids (job-owned blocks)
    const uint32_t* ri = nullptr;
    int64_t rn = 0;
    bool base_mode = false;      // one-rank identity: a re-probe reads the caller's keys, ids pbase + row
    const uint8_t* rv = nullptr;  // (its validity bitmap and offset)
    int64_t rvoff = 0, pbase = 0;
    void* ws = nullptr;
    hipStream_t stream = nullptr;
    // exchange jobs (hj_dist_shuffle / hj_dist_gather): the received rows, job-owned blocks
    const void* out_keys = nullptr;
    std::vector<const void*> out_cols;
    int64_t out_rows = -1;
    std::vector<std::pair<void*, size_t>> blocks;  // job-owned device blocks
    struct hj_comm* comm = nullptr;  // valid until hj_comm_free (the job's free needs only `device`)
    int device = 0;
};

struct hj_comm {
    std::unique_ptr<dfp::comm::Transport> tr;  // null when world == 1 (no collective runs)
    int rank = 0, world = 1, device = 0;
    std::atomic<bool> aborted{false};
    int64_t* host = nullptr;  // pinned mailbox for the plan's small reads
    // the plans' small device words (key range and status, minmax workspace, count and
    // status vectors), allocated once with the communicator so that no plan can fail to get
    // them between two collectives (a one-sided failure there would leave the peers blocked).
    // Jobs run one at a time on the worker and every word is consumed by a host read of the
    // job that wrote it, so consecutive jobs share them.
    int64_t* words = nullptr;
    hipEvent_t ev = nullptr;  // marks a read's copy
    // the jobs' device work runs on the communicator's own streams (after the caller's
    // stream at submission): two communicators' jobs never share a stream, so their
    // collectives cannot be ordered differently on different ranks
    hipStream_t side = nullptr;   // the sharded plan; the radix plan's build-side partition and collectives
    hipStream_t build = nullptr;  // the radix plan's local build
    hipStream_t probe = nullptr;  // the radix plan's probe side
    std::vector<hipEvent_t> evs;  // cross-stream ordering events (reused)
    // scratch of earlier jobs: released once their end event has fired
    struct Deferred {
        hipEvent_t done;
        std::vector<std::pair<void*, size_t>> blocks;
    };
    std::vector<Deferred> deferred;
    // the worker thread and its queue
    std::thread worker;
    std::mutex qmu;
    std::condition_variable qcv;
    std::deque<hj_dist_job*> q;
    bool stop = false;
    int fail_at = -1;  // test hook (thread transport): the job index whose plan fails on this rank
    std::atomic<int64_t> jobs{0};
};

namespace dfp {
namespace comm {
// finish a communicator made by hj_comm_create or the test library: pinned mailbox,
// events, the worker thread. -> HJ_OK or an error (the communicator is then freed)
hj_status start(hj_comm* c);
// the rank's contiguous share [lo, hi] of the key range [gmin, gmax] under the partition
// kernel's range map (hj_dist.cpp); false when empty
bool range_share_of(int64_t gmin, int64_t gmax, int W, int r, int64_t* lo, int64_t* hi);
}  // namespace comm
}  // namespace dfp
