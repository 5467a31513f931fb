#!/usr/bin/env python3
"""Benchmark of the MI355X hash join: build + probe of BASELINE.json's C2 workload.

One step = the whole join on device-resident synthetic input: build a table from
10^7 unique int64 keys (hj_build_begin/append/finish: table clear + insert + duplicate
passes) and probe it with 10^8 uniform int64 keys (probe kernel, canonical pair
emission into preallocated output). With N > 1 ranks (one process per GPU, launched by
torch.distributed.run) every rank holds a C2-sized shard (weak scaling) and a step also
radix-partitions both sides and exchanges them with RCCL all-to-all first.

Prints ONE JSON line (rank 0). `value` = probe rows of all ranks / step wall time
(Mrows/s); `probe_mrows_s` = probe rows / probe-kernel time; `build_ms` = device build
time. `roofline` prices the probe kernel (the dominant kernel) by its algorithmic bytes
8P + 16B + 12M over its HIP-event time; `traffic` is the PMC-measured
HBM bytes per probe launch from profiles/ (null if not measured for this config).
`cpu_baseline` times the oracle's multithreaded Version-10 restatement (oracle/hj_oracle.c)
on host cores over a bounded sample (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import datafusion_parallelism_amd as dfp  # noqa: E402
from datafusion_parallelism_amd.table import HashTable  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# The single-GPU job's timed steps record no timing events: a torch event's system-scope
# release writes the L2 back between two probes (C2 0.620 -> 0.612 ms per step,
# profiles/r04_step_events_ab.txt); probe_ms_in_step comes from an instrumented pass after
# the timed loop. DFP_BENCH_STEP_EVENTS=1: events around every timed probe (rounds 1-3).
STEP_EVENTS = os.environ.get("DFP_BENCH_STEP_EVENTS", "0") == "1"
PERM_MUL = 7368787
MIX_MUL = 0x9E3779B97F4A7C15  # odd: multiplication mod 2^64 is a bijection of int64
MIX_MUL_I64 = MIX_MUL - (1 << 64)

CONFIGS = {
    # BASELINE.json configs[1]: 10^8-probe x 10^7-build int64 uniform keys
    "c2": dict(workload="C2: 10^8-probe x 10^7-build int64 inner equi-join, uniform keys",
               build_rows=10**7, probe_rows=10**8, build_gen="perm", probe_range_mul=2),
    # C2 with both sides' keys mapped by the bijection k -> k * MIX_MUL (mod 2^64): the same
    # pairs, but the keys spread over the whole int64 domain, so the build takes the
    # hashed (open-addressing bucket) table instead of the direct-addressed one
    "c2h": dict(workload="C2h: C2's keys mapped onto the int64 domain by k -> k * 0x9E3779B97F4A7C15 "
                         "(mod 2^64); hashed bucket table",
                build_rows=10**7, probe_rows=10**8, build_gen="perm", probe_range_mul=2, mix=True),
    # BASELINE.json configs[2]: 10^8 rows with exponential/skewed build keys
    "c3": dict(workload="C3: 10^8-probe x 10^7-build int64, exponential build keys",
               build_rows=10**7, probe_rows=10**8, build_gen="exp", probe_range_mul=1),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def gen_inputs(cfg, rank, world, dev, strong=True):
    """Device-resident synthetic input of this rank (generated on the GPU).
    strong: the config's global join (B build x P probe rows) split into `world` contiguous
    shards, rank r holding build rows [rB/W, (r+1)B/W) and probe rows [rP/W, (r+1)P/W);
    weak: every rank holds a whole config-sized join over a global key domain of W x B."""
    L = dfp.load()
    B, P = cfg["build_rows"], cfg["probe_rows"]
    s = torch.cuda.current_stream(dev).cuda_stream
    gB = B if strong else world * B  # global build rows
    b0, b1 = (B * rank // world, B * (rank + 1) // world) if strong else (rank * B, (rank + 1) * B)
    p0, p1 = (P * rank // world, P * (rank + 1) // world) if strong else (rank * P, (rank + 1) * P)
    if cfg["build_gen"] == "perm":
        tmp = torch.empty(gB, dtype=torch.int64, device=dev)  # permutation of [0, gB)
        assert L.hj_gen_perm_keys(tmp.data_ptr(), gB, PERM_MUL, gB, s) == 0
        bk = tmp[b0:b1].clone()
        del tmp
    else:
        from datafusion_parallelism_amd.api_utils import make_exponential_int_array

        e = make_exponential_int_array(0, B).astype(np.int64)
        e = e[b0:b1] if strong else e + rank * B
        bk = torch.from_numpy(np.ascontiguousarray(e)).to(dev)
    pk = torch.empty(p1 - p0, dtype=torch.int64, device=dev)
    prange = cfg["probe_range_mul"] * gB
    assert L.hj_gen_uniform_keys(pk.data_ptr(), p1 - p0, 0xC0FFEE + p0, prange, s) == 0
    if cfg.get("mix"):  # int64 multiplication wraps mod 2^64 on the device
        bk.mul_(MIX_MUL_I64)
        pk.mul_(MIX_MUL_I64)
    torch.cuda.synchronize(dev)
    return bk, pk, b0, p0


def local_reference_count(cfg, rank, world, dev):
    """Pairs of this rank's probe rows against the whole build side, on this GPU with no
    exchange (outside the timed region): summed over the ranks, the count the exchange
    plan must reproduce."""
    bk, pk, _, _ = gen_inputs(cfg, 0, 1, dev, strong=True)  # the whole join
    P = pk.numel()
    p0, p1 = P * rank // world, P * (rank + 1) // world
    with HashTable(1, "int64", dev.index or 0) as t:
        t.append(0, bk)
        t.finish(0)
        b, _ = t.probe(pk[p0:p1], device_output=True)
        n = int(b.numel())
    del bk, pk
    return n


class SingleGpuJoin:
    """One step = build + probe on this GPU (no exchange)."""

    def __init__(self, bk, pk, dev, same_stream=False, priority="none"):
        self.bk, self.pk, self.dev = bk, pk, dev
        # builds run on their own stream: a probe partitions its rows while its table is
        # still being built (the library orders the first table read after the build).
        # priority: "probe-high" runs the probes on a high-priority stream, "build-low" the
        # builds on a low-priority one (HIP stream priorities order the dispatch of
        # workgroups from concurrent kernels)
        bprio = 1 if priority == "build-low" else 0
        self.bstream = None if same_stream else torch.cuda.Stream(dev, priority=bprio)
        self.pstream = torch.cuda.Stream(dev, priority=-1) if priority == "probe-high" else None
        P = pk.numel()
        self.ws = torch.empty(HashTable.workspace_bytes(P), dtype=torch.uint8, device=dev)
        self.d_total = torch.zeros(1, dtype=torch.int64, device=dev)
        self.cap = P
        self._alloc()
        # two event pairs: step k's pair is read while step k + 1 runs
        self.evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(2)]
        self.k = 0
        self.prev = None  # (table, events) of the step not collected yet
        self.probe_ms = []
        self.build_ms = []
        self.matches = 0
        self.step_events = STEP_EVENTS

    def _alloc(self):
        self.ob = torch.empty(self.cap, dtype=torch.int64, device=self.dev)
        self.op = torch.empty(self.cap, dtype=torch.int32, device=self.dev)

    def step(self):
        """One join: build a fresh table (on the build stream), probe it (on the current
        stream). Returns without waiting for the device, then collects the previous step
        (waiting for its probe). Steps thus overlap their host work (table set-up,
        launches) with the previous step's device work, and a probe's partition with its
        build, as a pipeline of joins does. probe_ms runs from the probe's launch to its
        end (with the wait for the rest of the build)."""
        t = HashTable(1, "int64", self.dev.index or 0)
        s = self.pstream or torch.cuda.current_stream(self.dev)
        if self.bstream is not None:
            with torch.cuda.stream(self.bstream):
                t.append(0, self.bk)
                t.finish(0)  # device build (runs on asynchronously for a direct-addressed table)
        else:
            t.append(0, self.bk)
            t.finish(0)
            t.stream_wait(s.cuda_stream)  # probe_ms times the probe alone
        ev = self.evs[self.k & 1]
        self.k += 1
        if self.step_events:
            ev[0].record(s)
        t.probe_async(self.pk.data_ptr(), self.pk.numel(), self.ob.data_ptr(), self.op.data_ptr(), self.cap,
                      self.d_total.data_ptr(), self.ws.data_ptr(), s.cuda_stream)
        if self.step_events:
            ev[1].record(s)
        self.collect()
        self.prev = (t, ev)

    def collect(self):
        """Per-step event timings of the previous step (its events have completed: see
        step()); the pair count (identical every step) is read once after the timed loop
        (finish())."""
        if self.prev is None:
            return
        t, ev = self.prev
        if self.step_events:
            ev[1].synchronize()
            self.probe_ms.append(ev[0].elapsed_time(ev[1]))
        self.build_ms.append(t.build_ns() / 1e6)
        t.close()  # waits for the table's probes (the library's probe-end event)
        self.prev = None

    def finish(self):
        self.collect()
        self.matches = int(self.d_total.item())
        if self.matches > self.cap:
            raise RuntimeError("output capacity too small")
        if not self.step_events:  # probe_ms_in_step: a few pipelined steps with events, untimed
            build_ms, self.probe_ms, self.step_events = self.build_ms, [], True
            for _ in range(6):
                self.step()
            self.collect()
            self.build_ms = build_ms
        # after the timed loop: the probe alone on a finished table (the roofline's
        # launch time; inside the pipeline a probe also waits for the end of its build)
        t = HashTable(1, "int64", self.dev.index or 0)
        t.append(0, self.bk)
        t.finish(0)
        st = t.stats()
        P = self.pk.numel()
        dense = st["buckets"] == 0
        sliced = P >= (st["table_bytes"] // 4 if dense else st["buckets"]) and P >= 65536
        if sliced:
            self.kernel_desc = ("the whole hj_probe_async, sliced probe (DESIGN.md §4): " +
                                ("sl_partition" if dense else "hs_partition") +
                                " + sl_lookup + sl_emit (tile offsets from the lookup's tile counts); " +
                                ("direct-addressed table" if dense else
                                 f"hashed table, {st['buckets']} buckets = {st['table_bytes']} B"))
        else:
            self.kernel_desc = "probe_fused_kernel (" + ("direct-addressed" if dense else "hashed") + " table)"
        s = self.pstream or torch.cuda.current_stream(self.dev)
        t.stream_wait(s.cuda_stream)
        torch.cuda.synchronize(self.dev)
        self.probe_in_step_ms = self.probe_ms
        self.probe_ms = []
        for _ in range(5):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(s)
            t.probe_async(self.pk.data_ptr(), self.pk.numel(), self.ob.data_ptr(), self.op.data_ptr(), self.cap,
                          self.d_total.data_ptr(), self.ws.data_ptr(), s.cuda_stream)
            ev[1].record(s)
            ev[1].synchronize()
            self.probe_ms.append(ev[0].elapsed_time(ev[1]))
        t.close()


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _join_cpu(oracle, bk, pk, nthreads, runs=3):
    """Build + one emitting probe pass of the oracle's Version-10 restatement, `runs` times
    (the GPU box's host is shared: single runs spread by up to 2x); -> the median run's
    timings plus every run's value and their range."""
    res = []
    for _ in range(runs):
        t0 = time.perf_counter()
        tbl = oracle.V10Table(bk, nthreads=nthreads)
        t1 = time.perf_counter()
        b, _ = tbl.probe(pk, nthreads=nthreads, emit=True)
        t2 = time.perf_counter()
        tbl.close()
        res.append({"threads": nthreads, "build_ms": round((t1 - t0) * 1e3, 2), "probe_ms": round((t2 - t1) * 1e3, 2),
                    "probe_mrows_s": round(len(pk) / (t2 - t1) / 1e6, 2),
                    "value": round(len(pk) / (t2 - t0) / 1e6, 3), "pairs": int(len(b))})
        del b
    vals = sorted(r["value"] for r in res)
    med = sorted(res, key=lambda r: r["value"])[len(res) // 2]
    return dict(med, runs=[r["value"] for r in res], range=[vals[0], vals[-1]])


def _cpu_quota():
    """CPUs granted by the cgroup CPU quota (v2 cpu.max or v1 cfs quota), None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            return max(1, -(-int(q) // int(per)))
        return None
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return max(1, -(-q // per)) if q > 0 else None
    except (OSError, ValueError):
        return None


def cpu_baseline(cfg):
    """The reference's CPU join, restated in C (oracle/hj_oracle.c, reference Version 10:
    concurrent open-addressing insert + chain walk + key re-check), timed on this host's
    cores at the reference's PARALLELISM = 8 threads and at every core this process may
    use, with no extrapolation:
      * this config (build B + probe P with pair emission);
      * C1a (benches/lookup_speed.rs:135-154, 240-246): a 4,194,304-row build (8 partitions
        x 64 batches x 8192 Int32 rows, batch i holding keys i*8192..(i+1)*8192), then each
        of the 8 partitions' lookup loops, get_iter of the raw values 0..8,388,607 as
        hashes, single-threaded one after another as the reference's bench runs them; the
        build is build_speed.rs's workload (131-213);
      * C1b (BASELINE.json configs[0]): 2^20 unique build keys x 2^20 probe keys over 2^21,
        full inner join with pair emission."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    B, P = cfg["build_rows"], cfg["probe_rows"]
    if cfg["build_gen"] == "perm":
        bk = oracle.perm_keys(B, PERM_MUL, B)
    else:
        bk = oracle.make_exponential_int_array(0, B).astype(np.int64)
    pk = oracle.uniform_keys(P, 0xC0FFEE, cfg["probe_range_mul"] * B)
    if cfg.get("mix"):
        bk = (bk.astype(np.uint64) * np.uint64(MIX_MUL)).astype(np.int64)
        pk = (pk.astype(np.uint64) * np.uint64(MIX_MUL)).astype(np.int64)
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 8
    quota = _cpu_quota()
    # the cores this process may actually run on: the affinity mask, capped by a cgroup
    # CPU quota (a GPU box shares its host: nproc shows every CPU, the quota its share)
    all_threads = min(affinity, quota) if quota else affinity
    # 16: a one-GPU box's share of its host's CPUs (the pool gives 16 per GPU; the quota
    # is not always visible from inside)
    counts = sorted({8, min(16, all_threads), all_threads})
    main = {f"threads_{n}": _join_cpu(oracle, bk, pk, n) for n in counts}
    del pk
    # C1a: lookup_speed
    c1a_keys = np.tile(np.arange(64 * 8192, dtype=np.int64), 8)
    t0 = time.perf_counter()
    tbl = oracle.V10Table(c1a_keys, nthreads=8)
    t1 = time.perf_counter()
    rows = sum(tbl.lookup_hashes(0, 2 * 512 * 8192) for _ in range(8))
    t2 = time.perf_counter()
    tbl.close()
    c1a = {"build_rows": int(len(c1a_keys)), "build_threads": 8, "build_ms": round((t1 - t0) * 1e3, 2),
           "lookups": 8 * 2 * 512 * 8192, "lookup_threads": 1, "lookup_ms": round((t2 - t1) * 1e3, 2),
           "mlookups_s": round(8 * 2 * 512 * 8192 / (t2 - t1) / 1e6, 2), "rows_yielded": int(rows)}
    # C1b: 2^20 x 2^20
    n1 = 1 << 20
    c1b_b = oracle.perm_keys(n1, PERM_MUL, n1)
    c1b_p = oracle.uniform_keys(n1, 0xC0FFEE, 2 * n1)
    c1b = {f"threads_{n}": _join_cpu(oracle, c1b_b, c1b_p, n) for n in counts}
    m8 = main["threads_8"]
    return {
        "value": m8["value"],
        "unit": "Mrows/s",
        "cores": 8,
        "kind": "port",
        "sample": f"full {B}-row build + {P}-row probe with pair emission (no extrapolation), 3 runs per thread "
                  f"count, value = the median run (runs and range beside it); C restatement of reference "
                  f"Version 10 (oracle/hj_oracle.c) on {_cpu_model()}; value = probe rows / (build + probe) at "
                  f"the reference's PARALLELISM = 8 threads; also at all {all_threads} usable cores (affinity "
                  f"{affinity} of the host's {os.cpu_count()} logical CPUs, cgroup quota "
                  f"{quota if quota else 'none'}); plus C1a (lookup_speed) and C1b (2^20 x 2^20). Bias in the "
                  f"CPU's favour: the restated table is pre-sized from the row count (no generation doubling or "
                  f"migration, new_map_3.rs:325-411) and the build skips the payload column concatenation that "
                  f"build_speed.rs times",
        "runs": m8["runs"],
        "range": m8["range"],
        "build_ms": m8["build_ms"],
        "probe_mrows_s": m8["probe_mrows_s"],
        "this_config": main,
        "c1a_lookup_speed": c1a,
        "c1b_1m_x_1m": c1b,
    }


class _TimedJoin:
    """tpch's join_fn with HIP events on the current stream around every join (build +
    probe): the per-join device spans and sizes of a query run (B, P, M)."""

    def __init__(self):
        from datafusion_parallelism_amd import tpch

        self._join = tpch._join
        self.record = False
        self.joins = []

    def __call__(self, build, probe):
        if not self.record:
            return self._join(build, probe)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b, p = self._join(build, probe)
        e1.record()
        self.joins.append((int(build.numel()), int(probe.numel()), int(b.numel()), e0, e1))
        return b, p


def bench_c4(args, json_out):
    """--config c4: TPC-H Q3 at SF100 (BASELINE.json configs[3], quoted on 8 GPUs; one
    MI355X holds SF100, so this line is the one-GPU plan tpch.q3 with the tables resident in
    HBM). A step = one whole query (filters, both hash joins, the group-by sum, the top 10);
    value = lineitem rows / s. roofline: the two joins (customer ⋈ orders, orders ⋈
    lineitem) with 8P + 16B + 12M algorithmic bytes each over their device spans (HIP events
    around build + probe). cpu_baseline: the same plan on the host at SF1 with the oracle's C
    join (kind "port")."""
    from datafusion_parallelism_amd import tpch

    if int(os.environ.get("WORLD_SIZE", "1")) != 1:
        raise SystemExit("--config c4 is a one-GPU line (tools/bench_tpch.py --dist runs the 8-rank plans)")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sf = float(os.environ.get("DFP_BENCH_C4_SF", "100"))
    t = tpch.generate(sf, dev, seed=1)
    nl = int(t.l_orderkey.numel())
    tj = _TimedJoin()
    for _ in range(args.warmup):
        tpch.q3(t, join_fn=tj)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = tpch.q3(t, join_fn=tj)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    # per-join spans from instrumented runs after the timed loop (median of 3)
    spans = []
    for _ in range(3):
        tj.joins, tj.record = [], True
        tpch.q3(t, join_fn=tj)
        torch.cuda.synchronize(dev)
        tj.record = False
        spans.append([(B, P, M, e0.elapsed_time(e1)) for B, P, M, e0, e1 in tj.joins])
    joins = []
    for i in range(len(spans[0])):
        B, P, M = spans[0][i][:3]
        ms = float(np.median([s[i][3] for s in spans]))
        joins.append({"build_rows": B, "probe_rows": P, "matches": M, "ms": round(ms, 4),
                      "alg_bytes": 8 * P + 16 * B + 12 * M})
    alg = sum(j["alg_bytes"] for j in joins)
    jms = sum(j["ms"] for j in joins)
    achieved = alg / (jms / 1e3) / 1e9
    value = nl / (elapsed / args.steps) / 1e6
    cpu = None if args.no_cpu_baseline else cpu_baseline_c4()
    line = {
        "metric": "probe Mrows/s + build ms, 10^8-row int64 inner join; 1/2/4/8 GPUs",
        "value": round(value, 3), "unit": "Mrows/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "int64",
        "data": "synthetic TPC-H-shaped tables generated on the device (tpch.generate: spec key structure and value "
                "domains, not dbgen's streams)",
        "config": {"workload": f"C4: TPC-H Q3 SF{sf:g} (lineitem ⋈ orders ⋈ customer), one MI355X, tables in HBM",
                   "lineitem_rows": nl, "groups": res.groups, "parallelism": "single-gpu"},
        "value_unit_note": "lineitem rows per second of whole queries",
        "query_ms": round(elapsed / args.steps * 1e3, 4),
        "joins": joins,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "Q3's two hash joins (build + probe each; HIP events around each join)",
                     "alg_bytes_per_launch": alg, "alg_bytes_formula": "sum over the joins of 8*P + 16*B + 12*M"},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), file=json_out, flush=True)


def cpu_baseline_c4():
    """tpch.q3 on the host (torch CPU tensors) at SF1 with the oracle's C inner join
    (oracle/hj_oracle.c, one thread): lineitem rows / s, 3 runs (median, range)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    from datafusion_parallelism_amd import tpch

    def join(build, probe):
        b, p = oracle.inner_join(build.numpy(), probe.numpy())
        return torch.from_numpy(b.astype(np.int64)), torch.from_numpy(p.astype(np.int64))

    t = tpch.generate(1, "cpu", seed=1)
    nl = int(t.l_orderkey.numel())
    vals = []
    for _ in range(3):
        t0 = time.perf_counter()
        tpch.q3(t, join_fn=join)
        vals.append(nl / (time.perf_counter() - t0) / 1e6)
    vals.sort()
    return {"value": round(vals[1], 3), "unit": "Mrows/s", "cores": 1, "kind": "port",
            "sample": f"tpch.q3 at SF1 ({nl} lineitem rows) on the host: torch CPU ops for the filters, group-by and "
                      f"top-k, the oracle's C inner join (oracle/hj_oracle.c, single thread) for both joins; 3 runs, "
                      f"median (range beside it); on {_cpu_model()}",
            "runs": [round(v, 3) for v in vals], "range": [round(vals[0], 3), round(vals[-1], 3)]}


def load_traffic(config_name):
    p = os.path.join(ROOT, "profiles", f"traffic_{config_name}.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def _spawn_ranks(n: int) -> int:
    """`--gpus N` without a launcher: start N fresh rank processes of this script (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, rendezvous on
    127.0.0.1), as torch.distributed.run would. Runs before anything in this process
    touches a GPU, and never replaces this process: the children are new processes, this
    one waits for them and exits with the worst status. Rank 0's JSON line reaches stdout
    (inherited fd 1)."""
    import datetime
    import signal
    import subprocess

    # The rendezvous store lives in this (GPU-free) parent and keeps its listening socket
    # for the children's whole life: the children join it as clients (DFP_BENCH_STORE), so no
    # port is ever found by binding and closing a socket (another process could take it
    # before a child listens: the EADDRINUSE of gpurun_out/r05y).
    store = dist.TCPStore("127.0.0.1", 0, None, True, timeout=datetime.timedelta(seconds=600),
                          wait_for_workers=False)
    port = store.port
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DFP_BENCH_STORE=f"127.0.0.1:{port}")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        for p in procs:
            rc = max(rc, p.wait())
            if rc != 0:  # one rank failed: the others would wait at a collective forever
                for q in procs:
                    if q.poll() is None:
                        q.send_signal(signal.SIGTERM)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
        del store  # the listening socket closes only after every rank has exited
    return rc


def _spawned_store():
    """A rank started by _spawn_ranks joins the parent's store as a client (None under a
    launcher: torch.distributed.run's env:// rendezvous then applies)."""
    spec = os.environ.get("DFP_BENCH_STORE")
    if not spec:
        return None
    import datetime

    host, port = spec.rsplit(":", 1)
    return dist.TCPStore(host, int(port), None, False, timeout=datetime.timedelta(seconds=600))


def init_group(backend: str, rank: int, world: int, **kw) -> str:
    """init_process_group for a multi-rank run: through the spawning parent's store when this
    rank was spawned by _spawn_ranks, else env:// (the launcher's MASTER_*). Returns which."""
    store = _spawned_store()
    if store is not None:
        dist.init_process_group(backend, store=store, rank=rank, world_size=world, **kw)
        return "parent-store"
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return "env"


def _median(xs):
    return round(float(np.median(xs)), 4) if xs else None


def stage_fields(job) -> dict:
    """Per-step stage times of a job's timed steps (medians, ms): build_ms (the device build
    span: the local build, or the multi-GPU build side - plan, exchange, local build,
    gathers - on its stream), probe_ms, exchange_ms, and host_ms_per_step (host time
    inside the join call per step; None for a job that does not record it)."""
    return {"build_ms": _median(job.build_ms), "probe_ms": _median(job.probe_ms),
            "exchange_ms": _median(getattr(job, "exchange_ms", [])),
            "host_ms_per_step": _median(getattr(job, "host_ms", []))}


def _clear_stage_lists(job) -> None:
    for name in ("probe_ms", "build_ms", "exchange_ms", "host_ms", "step_ms"):
        if hasattr(job, name):
            getattr(job, name).clear()


class DryRunJob:
    """--dry-run: the launcher, rendezvous, timing and reporting skeleton on the CPU (gloo),
    with a stand-in step (no GPU, no join): for tests of the multi-rank plumbing on a
    machine without a GPU. Its line says so in `data`; it is not a measurement."""

    kernel_desc = "dry run (no kernel)"
    pipelined = False

    def __init__(self):
        self.probe_ms, self.build_ms, self.exchange_ms, self.host_ms = [], [], [], []
        self.matches = 0
        g = torch.Generator().manual_seed(1)
        self.bk = torch.randint(0, 1 << 20, (1 << 16,), generator=g)
        self.pk = torch.randint(0, 1 << 21, (1 << 17,), generator=g)

    def step(self):
        # stand-ins timed like the real jobs' stages: a "build" (sort of the build keys) and
        # a "probe" (binary search of the probe keys); host time = the whole step call
        h0 = time.perf_counter()
        t0 = time.perf_counter()
        sk, _ = torch.sort(self.bk)
        t1 = time.perf_counter()
        pos = torch.searchsorted(sk, self.pk).clamp_(max=sk.numel() - 1)
        self.matches = int((sk[pos] == self.pk).sum())
        t2 = time.perf_counter()
        self.build_ms.append((t1 - t0) * 1e3)
        self.probe_ms.append((t2 - t1) * 1e3)
        self.exchange_ms.append(0.0)
        self.host_ms.append((time.perf_counter() - h0) * 1e3)

    def collect(self):
        pass

    def finish(self):
        pass


def dry_run(args, json_out):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    rendezvous = None
    if world > 1:
        rendezvous = init_group("gloo", rank, world)
    job = DryRunJob()
    for _ in range(args.warmup):
        job.step()
    _clear_stage_lists(job)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        job.step()
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    ranks = torch.tensor([1], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(ranks)
    if rank == 0:
        print(json.dumps({"metric": "probe Mrows/s + build ms, 10^8-row int64 inner join; 1/2/4/8 GPUs",
                          "value": None, "unit": "Mrows/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(float(el.item()) / args.steps * 1e3, 4),
                          "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int64",
                          "data": "dry-run (CPU, gloo: launcher and timing skeleton only, not a measurement)",
                          "ranks_reporting": int(ranks.item()), "rendezvous": rendezvous,
                          "config": {"workload": "dry run"},
                          **stage_fields(job)}),
              file=json_out, flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS) + ["c4"],
                    help="c2 (the headline), c2h, c3: joins of SURVEY.md §8d; c4: TPC-H Q3 SF100 on one GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stream-priority", default="none", choices=["none", "probe-high", "build-low"],
                    help="single GPU: HIP stream priorities of the probe / build streams")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the radix-exchange path even with one rank (testing)")
    ap.add_argument("--chunks", type=int, default=1,
                    help="multi-GPU radix plan: probe-side chunks whose exchange overlaps the previous chunk's probe "
                         "(each chunk's probe reloads the table's slices; 1 = one probe)")
    ap.add_argument("--same-stream", action="store_true",
                    help="run each build on the probe's stream (no build/probe overlap)")
    ap.add_argument("--sync-steps", action="store_true",
                    help="synchronize the device after every step (no host/device overlap between steps)")
    ap.add_argument("--no-compress-keys", action="store_true",
                    help="multi-GPU: exchange full int64 keys / u64 build ids even when 32 bits suffice")
    ap.add_argument("--plan", default="auto", choices=["auto", "broadcast", "radix", "sharded"],
                    help="multi-GPU plan for the strong-scaling line (auto: broadcast when B*G < B+P)")
    ap.add_argument("--no-weak", action="store_true",
                    help="multi-GPU: skip the weak-scaling extra (a config-sized join per rank, radix exchange)")
    ap.add_argument("--native", default="auto", choices=["auto", "on", "off"],
                    help="multi-GPU sharded plan: its build side through the C entry point hj_dist_build_sharded "
                         "(RCCL inside the library; auto = on RCCL groups) or the torch.distributed steps (off)")
    ap.add_argument("--comms", type=int, default=None,
                    help="multi-GPU native plans: communicators used in turn (consecutive steps' host reads overlap; "
                         "default 2 on one rank, 1 on more: DistributedHashJoin)")
    ap.add_argument("--build-priority", default="normal", choices=["normal", "high"],
                    help="multi-GPU plans: the build side's stream at high HIP priority (its kernels are the critical "
                         "path of the build side's host reads)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo: run the multi-rank launcher and timing skeleton without a GPU (tests)")
    args = ap.parse_args()
    if args.gpus > 1 and "RANK" not in os.environ:
        # no launcher: spawn the ranks (before any GPU call in this process), never run one
        sys.exit(_spawn_ranks(args.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {os.environ['WORLD_SIZE']}: the launcher and the "
                         f"flag disagree")
    # The one JSON line goes to the original stdout; everything else that writes to fd 1
    # (RCCL's version banner, HIP runtime messages) is sent to stderr.
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    if args.dry_run:
        return dry_run(args, json_out)
    if args.config == "c4":
        return bench_c4(args, json_out)
    cfg = CONFIGS[args.config]

    one_rank_store = None
    if args.force_dist and "RANK" not in os.environ:  # one rank without a launcher: an in-memory store
        # (a free TCP port found by binding port 0 can be taken again before the store listens)
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
        one_rank_store = dist.HashStore()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    if one_rank_store is not None:
        dist.init_process_group("nccl", store=one_rank_store, rank=0, world_size=1, device_id=dev)
    elif world > 1 or args.force_dist:
        init_group("nccl", rank, world, device_id=dev)

    use_dist = world > 1 or args.force_dist
    bk, pk, bbase, pbase = gen_inputs(cfg, rank, world, dev, strong=True)
    B, P = bk.numel(), pk.numel()
    gB, gP = cfg["build_rows"], cfg["probe_rows"]  # the whole join (strong scaling)
    plan = None
    if not use_dist:
        job = SingleGpuJoin(bk, pk, dev, same_stream=args.same_stream, priority=args.stream_priority)
    else:
        from datafusion_parallelism_amd.distributed import DistributedHashJoin

        dj = DistributedHashJoin(chunks=args.chunks, compress_keys=not args.no_compress_keys,
                                 native={"auto": None, "on": True, "off": False}[args.native], comms=args.comms)
        plan = args.plan if args.plan != "auto" else DistributedHashJoin.choose_plan(gB, gP, world)
        if args.plan == "auto" and plan == "broadcast":
            # the broadcast side's sharded form: each rank builds 1/G of the table and the
            # pieces are gathered (join_sharded falls back to a whole build per rank for a
            # sparse build domain)
            plan = "sharded"
        job = (BroadcastJob(dj, bk, pk, pbase, dev) if plan == "broadcast" else
               ShardedJob(dj, bk, pk, bbase, pbase, dev, priority=-1 if args.build_priority == "high" else 0)
               if plan == "sharded" else
               DistJob(dj, bk, pk, bbase, pbase, dev, same_stream=args.same_stream))

    def barrier():
        if use_dist:
            dist.barrier()

    def timed(job, steps, warmup):
        """warmup untimed steps, then `steps` timed ones between barriers + device syncs;
        -> max over ranks of the elapsed seconds"""
        # warmup runs as the timed loop does (pipelined steps hold two tables at once: the
        # allocator's cache fills here, not inside the timed region)
        per_step_sync = args.sync_steps or (use_dist and not getattr(job, "pipelined", False))
        for _ in range(warmup):
            job.step()
            if per_step_sync:
                torch.cuda.synchronize(dev)
                job.collect()
        if hasattr(job, "drain"):  # no native job in flight across torch's barrier below
            job.drain()
        torch.cuda.synchronize(dev)
        job.collect()
        _clear_stage_lists(job)
        # the local job's steps overlap one step's host work with the previous step's
        # device work (SingleGpuJoin.step); the exchange jobs synchronize inside a step
        barrier()
        torch.cuda.synchronize(dev)
        t_start = time.perf_counter()
        for _ in range(steps):
            job.step()
            if per_step_sync:
                torch.cuda.synchronize(dev)
                job.collect()
        if hasattr(job, "drain"):  # a prefetched native build side: inside the timed region
            job.drain()
        torch.cuda.synchronize(dev)
        barrier()
        elapsed = time.perf_counter() - t_start
        job.finish()
        if use_dist:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed

    elapsed = timed(job, args.steps, args.warmup)
    ms_per_step = elapsed / args.steps * 1e3
    total_probe_rows = gP  # strong scaling: the one global join, whatever the rank count
    value = total_probe_rows / (elapsed / args.steps) / 1e6
    weak = None
    if use_dist and world > 1 and not args.no_weak:
        # extra: weak scaling, a config-sized join on every rank (radix all-to-all)
        wbk, wpk, wb0, wp0 = gen_inputs(cfg, rank, world, dev, strong=False)
        wjob = DistJob(dj, wbk, wpk, wb0, wp0, dev)
        we = timed(wjob, max(3, args.steps // 2), max(2, args.warmup // 4))
        wsteps = max(3, args.steps // 2)
        weak = {"scaling": "weak", "value": round(gP * world / (we / wsteps) / 1e6, 3), "unit": "Mrows/s",
                "ms_per_step": round(we / wsteps * 1e3, 4), "probe_rows_per_gpu": gP, "build_rows_per_gpu": gB,
                "plan": "radix", "exchange_ms": round(float(np.median(wjob.exchange_ms)), 4)}
        del wbk, wpk, wjob

    probe_ms = float(np.median(job.probe_ms))
    build_ms = float(np.median(job.build_ms))
    M = job.matches
    if use_dist:  # pairs of the whole join (all ranks)
        mt = torch.tensor([M, local_reference_count(cfg, rank, world, dev)], dtype=torch.int64, device=dev)
        dist.all_reduce(mt)
        M_all, M_ref = int(mt[0].item()), int(mt[1].item())
        if M_all != M_ref:  # the exchange plan lost or invented pairs
            raise RuntimeError(f"multi-GPU pair count {M_all} != {M_ref} of the same join without exchange")
    else:
        M_all = M
    alg_bytes = 8 * P + 16 * B + 12 * M
    achieved = alg_bytes / (probe_ms / 1e3) / 1e9
    traffic = load_traffic(args.config) if not use_dist else None
    roofline = {
        "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": (traffic or {}).get("hbm_bytes_per_launch"),
        "traffic_lower": ((traffic or {}).get("probe_phase") or {}).get("hbm_bytes_lower"),
        "kernel": job.kernel_desc,
        "alg_bytes_per_launch": alg_bytes,
        "alg_bytes_formula": "8*P + 16*B + 12*M (SURVEY.md §8d)",
        # the probe rows' lookups run out of LDS (no random device reads per row); the HBM
        # streams of the sliced pipeline (keys, entries, refs, rows, pairs) are in DESIGN.md §4
        "probe_rows_per_s": round(P / (probe_ms / 1e3) / 1e9, 2),
        "probe_rows_unit": "G/s",
    }

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(cfg)
        line = {
            "metric": "probe Mrows/s + build ms, 10^8-row int64 inner join; 1/2/4/8 GPUs",
            "value": round(value, 3),
            "unit": "Mrows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (device-generated seeded keys, SURVEY.md §8d generators)",
            "config": {
                "workload": cfg["workload"],
                "build_rows": gB,
                "probe_rows": gP,
                "matches": M_all,
                "parallelism": "single-gpu" if not use_dist else f"{plan} x{world} (RCCL)",
            },
            "probe_mrows_s": round(P / (probe_ms / 1e3) / 1e6, 1),
            "probe_ms": round(probe_ms, 4),
            "probe_ms_in_step": (round(float(np.median(job.probe_in_step_ms)), 4)
                                 if getattr(job, "probe_in_step_ms", None) else None),
            "build_ms": round(build_ms, 4),
            "pipelined_steps": not (args.sync_steps or (use_dist and not getattr(job, "pipelined", False))),
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if use_dist:
            line["exchange_ms"] = _median(job.exchange_ms)
            line["plan"] = plan
            if plan == "sharded":
                line["native_build_side"] = bool(getattr(dj, "last_native", False))
            line["host_ms_per_step"] = _median(getattr(job, "host_ms", []))
            line["build_ms_source"] = ("HIP events on the build stream around the build side (plan, exchange, "
                                       "local build" + (", table gathers)" if plan == "sharded" else ")"))
            line["probe_ms_source"] = "HIP events on the probe stream, launch to end (with any wait for its table)"
        if weak is not None:
            line["weak"] = weak
        print(json.dumps(line), file=json_out, flush=True)
    if use_dist:
        dist.destroy_process_group()


class DistJob:
    """One step = the radix plan (DistributedHashJoin.join): global key range (one host
    read), both sides partitioned in one pass each into per-destination regions (runtime
    filter, int32 key offsets, u32 ids), each side's counts exchanged and read while the
    device runs the next stage, the build side's regions exchanged (RCCL point to point; a rank's own region stays in
    place) and built with global ids, the probe side's exchanged and probed once with
    global probe ids. exchange_ms = from the end of the partitions to the end of the
    exchanges (events); probe_ms = the whole step on the device."""

    def __init__(self, dj, bk, pk, bbase, pbase, dev, same_stream=False):
        self.dj, self.bk, self.pk, self.dev = dj, bk, pk, dev
        self.bbase = bbase
        self.pbase = pbase
        self.probe_ms, self.build_ms, self.exchange_ms, self.host_ms, self.step_ms = [], [], [], [], []
        self.matches = 0
        self.cap = pk.numel()
        self.kernel_desc = ("one-pass region partition (both sides) + RCCL point-to-point exchange + local build + "
                            "sliced probe with global ids")
        self._pending = None
        # the plan (key range + host read) and the build side (partition, exchange, local
        # build) on their own stream, as SingleGpuJoin's builds: the inputs are resident
        # before the timed steps, so step k + 1's plan is read while step k's probe runs, and
        # the build side runs beside the probe side's partition
        self.bstream = None
        if not same_stream:
            from datafusion_parallelism_amd.distributed import concurrent_stream

            # the plan and the build side on their own stream, beside the probe side's partition
            self.bstream = concurrent_stream(dev)
        # the inputs exist once this event fires: the build stream waits for it, not for
        # the previous step's probe on the current stream
        self.ready = torch.cuda.Event()
        self.ready.record()

    pipelined = True  # step k is collected (its pair count read) after step k + 1 is enqueued

    def step(self):
        ev = {k: torch.cuda.Event(enable_timing=True)
              for k in ("start", "build_start", "build_end", "partitioned", "exchanged", "probe_start", "end")}
        self.dj.events = ev
        ev["start"].record()
        h0 = time.perf_counter()
        table, result = self.dj.join(self.bk, self.bbase, self.pk, self.pbase, self.cap, check=False,
                                     build_stream=self.bstream, inputs_ready=self.ready)
        self.host_ms.append((time.perf_counter() - h0) * 1e3)
        ev["end"].record()
        self.dj.events = None
        native = bool(getattr(self.dj, "last_native", False))
        prev, self._pending = self._pending, (table, result, ev, native)
        if prev is not None:
            self._collect(*prev)

    def collect(self):
        if self._pending is None:
            return
        pending, self._pending = self._pending, None
        self._collect(*pending)

    def drain(self):
        self.collect()

    def _collect(self, table, result, ev, native=False):
        b, _ = result()
        self.matches = int(b.numel())
        del b, _
        if native:  # hj_dist_join_radix: the job's own stage events (build side, exchange, probe)
            bms, xms, pms = result.job.times()
            self.build_ms.append(bms)
            self.exchange_ms.append(xms)
            self.probe_ms.append(pms)
            table.close()
            return
        ev["end"].synchronize()
        # both probe events on the probe's (current) stream; the build span on the build stream
        self.probe_ms.append(ev["probe_start"].elapsed_time(ev["end"]))
        self.step_ms.append(ev["start"].elapsed_time(ev["end"]))
        self.exchange_ms.append(ev["partitioned"].elapsed_time(ev["exchanged"]))
        self.build_ms.append(ev["build_start"].elapsed_time(ev["build_end"]))
        table.close()

    def finish(self):
        self.collect()


class ShardedJob:
    """One step = the sharded-build broadcast plan (DistributedHashJoin.join_sharded): the
    build side range-partitioned and exchanged (RCCL), a local build of the rank's own key
    range, an all_gather of the table pieces, and the probe of the rank's own probe rows
    (no probe-side exchange, no replicated build). The build side runs on its own stream,
    so step k's overlaps step k - 1's probe; step k - 1 is collected after step k is
    enqueued. exchange_ms = the whole build side (plan, exchange, local build, gather) on
    its stream; probe_ms = the probe, from its launch to its end."""

    pipelined = True

    def __init__(self, dj, bk, pk, bbase, pbase, dev, priority=0):
        self.dj, self.bk, self.pk, self.bbase, self.pbase, self.dev = dj, bk, pk, bbase, pbase, dev
        self.probe_ms, self.build_ms, self.exchange_ms, self.host_ms = [], [], [], []
        self.matches = 0
        self.cap = pk.numel()
        from datafusion_parallelism_amd.distributed import concurrent_stream

        self.bstream = concurrent_stream(dev, priority=priority)  # on another hardware queue than the probes'
        self.kernel_desc = ("sharded build: range exchange of the build side (RCCL), local build of the rank's key "
                            "range, all_gather of the table pieces, sliced probe of the local rows")
        self._pending = None
        # the next steps' native build sides (one per communicator), started during this
        # step's probe: their host reads wait on the communicators' workers meanwhile
        self._next = collections.deque()
        self.depth = max(1, getattr(dj, "_ncomms", 1))
        self.ready = torch.cuda.Event()  # the inputs exist: the build stream waits for this only
        self.ready.record()

    def _start(self):
        return self.dj.start_sharded(self.bk, self.bbase, self.bstream, self.ready, self.pk.dtype)

    def step(self):
        ev = {k: torch.cuda.Event(enable_timing=True)
              for k in ("build_start", "partitioned", "exchanged", "build_end", "probe_start", "end")}
        self.dj.events = ev
        cur = torch.cuda.current_stream(self.dev)
        h0 = time.perf_counter()
        pending = self._next.popleft() if self._next else self._start()
        table, result = self.dj.join_sharded(self.bk, self.bbase, self.pk, self.pbase, self.cap,
                                             build_stream=self.bstream, inputs_ready=self.ready, pending=pending)
        if self.dj.last_native:
            # the next steps' build sides, queued now: the workers' host reads wait while the
            # device runs this step's probe (the build keys are resident and unchanged)
            while len(self._next) < self.depth:
                self._next.append(self._start())
        self.host_ms.append((time.perf_counter() - h0) * 1e3)
        self.dj.events = None
        ev["end"].record(cur)
        # the native build side (hj_dist_build_sharded: one C call) records no partition /
        # exchange events: its exchange is inside build_ms
        prev, self._pending = self._pending, (table, result, ev, bool(getattr(self.dj, "last_native", False)))
        if prev is not None:
            self._collect(*prev)

    def collect(self):
        if self._pending is not None:
            pending, self._pending = self._pending, None
            self._collect(*pending)

    def _collect(self, table, result, ev, native):
        b, _ = result()
        self.matches = int(b.numel())
        ev["end"].synchronize()
        # the build side (plan, exchange, local build, gathers) on the build stream; the
        # probe from its launch to its end on the probe stream (with any wait for the table)
        if native:  # the build side ran as a job: its table's build time spans it (plan to gathers)
            self.build_ms.append(table.build_ns() / 1e6)
        else:
            self.exchange_ms.append(ev["partitioned"].elapsed_time(ev["exchanged"]))
            self.build_ms.append(ev["build_start"].elapsed_time(ev["build_end"]))
        self.probe_ms.append(ev["probe_start"].elapsed_time(ev["end"]))
        table.close()

    def drain(self):
        """The prefetched build sides (the steps after the last): finish their jobs."""
        while self._next:
            nxt = self._next.popleft()
            t, _ = nxt.table()
            nxt.close()
            t.close()

    def finish(self):
        self.drain()
        self.collect()


class BroadcastJob:
    """One step = all_gather of the build shards (RCCL), a local build of the whole build
    side (canonical numbering = the global build ids), and the probe of this rank's own
    probe rows: no probe-side exchange (SURVEY.md §8e broadcast build, chosen when
    B·G < B + P). Steps are pipelined like SingleGpuJoin's: the gather runs on its own
    stream (into one of two buffers), the build on another, the probe on the current
    stream, so step k's gather and build overlap step k - 1's probe; step k - 1 is
    collected after step k is enqueued. exchange_ms = the all_gather (events on the
    gather stream); probe_ms = the probe, from its launch to its end (with the wait for
    its build)."""

    pipelined = True

    def __init__(self, dj, bk, pk, pbase, dev):
        self.dj, self.bk, self.pk, self.pbase, self.dev = dj, bk, pk, pbase, dev
        self.probe_ms, self.build_ms, self.exchange_ms, self.host_ms = [], [], [], []
        self.matches = 0
        n = pk.numel()
        self.ws = torch.empty(HashTable.workspace_bytes(n), dtype=torch.uint8, device=dev)
        self.d_total = torch.zeros(1, dtype=torch.int64, device=dev)
        self.cap = n
        self.ob = torch.empty(n, dtype=torch.int64, device=dev)
        self.op = torch.empty(n, dtype=torch.int32, device=dev)
        self.kernel_desc = ("RCCL all_gather of the build shards (int32 key offsets for a direct-addressed build "
                            "domain) + local build + sliced probe of the local rows")
        W = dj.world  # shard sizes of the strong split (rows [rB/W, (r+1)B/W)), exchanged once
        nb = torch.tensor([int(bk.numel())], dtype=torch.int64, device=dev)
        allb = [torch.empty_like(nb) for _ in range(W)]
        dist.all_gather(allb, nb, group=dj.group)
        self.sizes = [int(x) for x in torch.cat(allb).tolist()]  # known before the timed steps
        # two gather buffers per key width: step k + 2 reuses step k's once step k is collected
        self.gbuf = {dt: [torch.empty(sum(self.sizes), dtype=dt, device=dev) for _ in range(2)]
                     for dt in {bk.dtype, torch.int32}}
        from datafusion_parallelism_amd.distributed import concurrent_stream

        # on other hardware queues than the probes' (concurrent_stream)
        self.cstream = concurrent_stream(dev)  # the gathers
        self.bstream = concurrent_stream(dev)  # the builds
        self.evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(2)]
        self.k = 0
        self.prev = None

    def _gather(self, out, src):
        if len(set(self.sizes)) == 1:
            return dist.all_gather_into_tensor(out, src, group=self.dj.group, async_op=True)
        parts = list(torch.split(out, self.sizes))
        return dist.all_gather(parts, src, group=self.dj.group, async_op=True)

    def step(self):
        from datafusion_parallelism_amd.distributed import broadcast_key_plan

        ev = self.evs[self.k & 1]
        slot = self.k & 1
        self.k += 1
        h0 = time.perf_counter()
        with torch.cuda.stream(self.cstream):
            ev[0].record(self.cstream)
            # the global key range (hj_key_minmax + one all-reduce; the host waits for this
            # stream only): a direct-addressed build domain travels as int32 offsets
            plan = broadcast_key_plan(self.bk, sum(self.sizes), self.dj.group) if self.dj.compress_keys else None
            src = self.bk if plan is None else (self.bk - plan[0]).to(torch.int32)
            g = self.gbuf[src.dtype][slot]
            work = self._gather(g, src)
            work.wait()  # the gather stream waits for the collective
            ev[1].record(self.cstream)
        self.bstream.wait_stream(self.cstream)
        t = HashTable(1, "int64" if plan is None else "int32", self.dev.index or 0)
        with torch.cuda.stream(self.bstream):
            t.append(0, g)
            if plan is not None:  # keyed back to the int64 probe keys, no key-range reduction
                t.key_range(0, plan[1] - 1)
                t.key_base(plan[0])
            t.finish(0)
        cur = torch.cuda.current_stream(self.dev)
        ev[2].record(cur)
        t.probe_async(self.pk.data_ptr(), self.pk.numel(), self.ob.data_ptr(), self.op.data_ptr(), self.cap,
                      self.d_total.data_ptr(), self.ws.data_ptr(), cur.cuda_stream, probe_base=self.pbase)
        ev[3].record(cur)
        self.host_ms.append((time.perf_counter() - h0) * 1e3)
        self.collect()
        self.prev = (t, ev)

    def collect(self):
        if self.prev is None:
            return
        t, ev = self.prev
        ev[3].synchronize()
        self.exchange_ms.append(ev[0].elapsed_time(ev[1]))
        self.probe_ms.append(ev[2].elapsed_time(ev[3]))
        self.build_ms.append(t.build_ns() / 1e6)
        t.close()
        self.prev = None

    def finish(self):
        self.collect()
        torch.cuda.synchronize(self.dev)
        self.matches = int(self.d_total.item())
        if self.matches > self.cap:
            raise RuntimeError("output capacity too small")


if __name__ == "__main__":
    main()
