#!/usr/bin/env python3
"""TPC-H-shaped Q3 and Q9 on one MI355X: query time with the
tables resident in HBM (generation excluded), for the scale factors given on the command
line (`q3:10 q9:100` ...). Prints one JSON line per run. BASELINE.json configs[3]/[4]
quote SF100 Q3 and SF300 Q9 on 8 GPUs; this measures the single-GPU queries."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from datafusion_parallelism_amd import tpch  # noqa: E402


def main():
    runs = sys.argv[1:] or ["q3:10"]
    for run in runs:
        q, sf = run.split(":")
        sf = float(sf)
        t = tpch.generate(sf, "cuda:0", q9=(q == "q9"))
        torch.cuda.synchronize()
        fn = tpch.q3 if q == "q3" else tpch.q9
        r = fn(t)  # warm-up
        times = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn(t)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        nl = t.l_orderkey.numel()
        best = min(times)
        line = {
            "what": f"TPC-H-shaped {q.upper()} on one GPU, tables resident in HBM",
            "query": q, "sf": sf, "lineitem_rows": nl, "orders_rows": t.o_orderkey.numel(),
            "query_ms_min": round(best * 1e3, 3), "query_ms_median": round(sorted(times)[len(times) // 2] * 1e3, 3),
            "lineitem_mrows_s": round(nl / best / 1e6, 1),
        }
        if q == "q3":
            line.update(groups=r.groups, top1=[r.l_orderkey[0], r.revenue[0], r.o_orderdate[0]] if r.l_orderkey else None)
        else:
            line.update(groups=len(r), first=list(r[0]) if r else None)
        print(json.dumps(line), flush=True)
        del t
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
