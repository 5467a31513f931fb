#!/usr/bin/env python3
"""Print one steady-state step of a rocprofv3 kernel trace: the kernels (start offset,
duration, queue/stream) between two consecutive launches of an anchor kernel.

usage: timeline.py TRACE_DIR ANCHOR_SUBSTRING [step_from_end=3]
"""
import csv
import glob
import sys

d, anchor = sys.argv[1], sys.argv[2]
back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
rows = []
for f in glob.glob(f"{d}/*kernel_trace.csv"):
    rows += list(csv.DictReader(open(f)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", ""),
             r.get("Queue_Id", "")) for r in rows)
idx = [i for i, e in enumerate(ev) if anchor in e[2]]
a, b = idx[-back - 1], idx[-back]
t0 = ev[a][0]
for s, e, n, st, q in ev[a:b + 1]:
    n = n.replace("void ", "").replace("dfp::", "")
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  s{st} q{q}  {n[:70]}")
