#!/usr/bin/env python3
"""TPC-H-shaped Q3 and Q9: query time with the tables resident in
HBM (generation excluded), for the scale factors given on the command line
(`q3:10 q9:100` ...). Prints one JSON line per run (rank 0).

BASELINE.json configs[3]/[4] (C4/C5) quote SF100 Q3 and SF300 Q9 on 8 GPUs. Without
--dist this measures the one-GPU plans (tpch.q3 / q9). With --dist it runs the
multi-GPU plans (tpch.q3_dist / q9_dist: broadcasts + RCCL shuffles), one process per
GPU, each holding its block of the tables:

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29511 tools/bench_tpch.py --dist q3:100 q9:300

Timed region: barrier + device synchronise on both sides, max over ranks."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from datafusion_parallelism_amd import tpch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("runs", nargs="*", default=["q3:10"])
    ap.add_argument("--dist", action="store_true", help="multi-GPU plans (torch.distributed, RCCL)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shards", type=int, default=0,
                    help="one-GPU plans with every join on a table of this many radix shards on GPU 0 "
                         "(hj_build_begin_multi on [0] * K: C4/C5's sharded builds in one process)")
    ap.add_argument("--budget", type=int, default=0,
                    help="one-GPU plans under a per-table device budget in bytes (hj_set_device_budget): a join "
                         "whose build exceeds it is sharded over --shards (default 8) radix shards on GPU 0 "
                         "(tpch.planned_join); the line lists each join's plan and peak device bytes")
    a = ap.parse_args()
    if a.budget:
        from datafusion_parallelism_amd.table import set_device_budget

        set_device_budget(a.budget)
    rank, world = 0, 1
    if a.dist:
        store = None
        if "RANK" not in os.environ:  # one rank without a launcher: an in-memory store, no port
            os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
            store = dist.HashStore()
        rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        local = int(os.environ.get("LOCAL_RANK", rank))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", store=store, rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))
    dev = f"cuda:{torch.cuda.current_device()}"
    for run in a.runs:
        q, sf = run.split(":")
        sf = float(sf)
        t = tpch.generate(sf, dev, q9=(q == "q9"), rank=rank, world=world)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()  # the generator's temporaries back to the device (the library allocates its own)
        if a.dist:
            fn = tpch.q3_dist if q == "q3" else tpch.q9_dist
        else:
            fn = tpch.q3 if q == "q3" else tpch.q9
            jf = None
            if a.budget:
                jf = tpch.planned_join([0] * (a.shards or 8))
            elif a.shards:
                jf = tpch.multi_join([0] * a.shards)
            if jf is not None:
                base = fn
                fn = lambda tt, base=base, jf=jf: base(tt, join_fn=jf)  # noqa: E731
        r = fn(t)  # warm-up
        if a.budget:
            joins = [{"build_rows": n, "plan": p, "peak_device_bytes": b} for n, p, b in jf.log]
            jf.log.clear()
        times = []
        for _ in range(a.reps):
            if a.dist:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn(t)
            torch.cuda.synchronize()
            if a.dist:
                dist.barrier()
            dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
            if a.dist:
                dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            times.append(float(dt.item()))
            print(f"[rep] {q} sf {sf} {times[-1] * 1e3:.1f} ms torch reserved {torch.cuda.memory_reserved() >> 20} MiB "
                  f"allocated {torch.cuda.memory_allocated() >> 20} MiB", file=sys.stderr, flush=True)
        nl = torch.tensor([t.l_orderkey.numel()], dtype=torch.int64, device=dev)
        if a.dist:
            dist.all_reduce(nl)
        nl = int(nl.item())
        best = min(times)
        line = {
            "what": f"TPC-H-shaped {q.upper()} on {world} GPU(s), tables resident in HBM"
                    + (" (multi-GPU plan: broadcast + RCCL shuffles)" if a.dist else ""),
            "query": q, "sf": sf, "n_gpus": world,
            "plan": "dist" if a.dist else (
                f"device budget {a.budget} B: one GPU per join, {a.shards or 8} radix shards on one GPU above it"
                if a.budget else f"{a.shards} radix shards on one GPU" if a.shards else "single"),
            "lineitem_rows": nl,
            "query_ms_min": round(best * 1e3, 3), "query_ms_median": round(sorted(times)[len(times) // 2] * 1e3, 3),
            "lineitem_mrows_s": round(nl / best / 1e6, 1),
            "times_ms": [round(x * 1e3, 3) for x in times],
        }
        if q == "q3":
            line.update(groups=r.groups, top1=[r.l_orderkey[0], r.revenue[0], r.o_orderdate[0]] if r.l_orderkey else None)
        else:
            line.update(groups=len(r), first=list(r[0]) if r else None)
        if a.budget:
            line["joins"] = joins
        if rank == 0:
            print(json.dumps(line), flush=True)
        del t
        torch.cuda.empty_cache()
    if a.dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
