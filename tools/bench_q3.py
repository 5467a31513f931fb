#!/usr/bin/env python3
"""TPC-H-shaped Q3 on one MI355X: query time with the tables
resident in HBM (generation excluded), for the scale factors given on the command line.
Prints one JSON line per scale factor. BASELINE.json configs[3] quotes SF100 Q3 on 8
GPUs; this measures the single-GPU query (the 8-GPU radix-partitioned plan is a later
row)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from datafusion_parallelism_amd import tpch  # noqa: E402


def main():
    sfs = [float(x) for x in sys.argv[1:]] or [10.0]
    for sf in sfs:
        t = tpch.generate(sf, "cuda:0")
        torch.cuda.synchronize()
        r = tpch.q3(t)  # warm-up
        times = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = tpch.q3(t)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        nl = t.l_orderkey.numel()
        best = min(times)
        print(json.dumps({
            "what": "TPC-H-shaped Q3 (customer x orders x lineitem), one GPU, tables resident in HBM",
            "sf": sf, "lineitem_rows": nl, "orders_rows": t.o_orderkey.numel(),
            "customer_rows": t.c_custkey.numel(), "groups": r.groups,
            "query_ms_min": round(best * 1e3, 3), "query_ms_median": round(sorted(times)[len(times) // 2] * 1e3, 3),
            "lineitem_mrows_s": round(nl / best / 1e6, 1),
            "top1": [r.l_orderkey[0], r.revenue[0], r.o_orderdate[0]] if r.l_orderkey else None,
        }), flush=True)
        del t
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
