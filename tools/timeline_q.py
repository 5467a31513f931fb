#!/usr/bin/env python3
"""Device timeline of one steady-state step from a rocprofv3 kernel trace (+ memory-copy
trace when present): every kernel / copy between two consecutive launches of the anchor
kernel, with its queue, start offset, gap on its queue and duration.
usage: timeline_q.py OUTDIR [anchor substring, default key_minmax] [step from the end, default 3]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "key_minmax"
back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "Q" + r.get("Queue_Id", "?"), r["Kernel_Name"]))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy",
                     f"{r.get('Direction', '')} {int(r.get('Bytes', 0) or 0)}B"))
rows.sort()
idx = [i for i, r in enumerate(rows) if anchor in r[3]]
i0, i1 = idx[-back], idx[-back + 1]
t0 = rows[i0][0]
last = {}
for s, e, q, n in rows[i0:i1]:
    gap = (s - last.get(q, s)) / 1e3
    last[q] = max(last.get(q, 0), e)
    print(f"{(s - t0) / 1e3:8.1f} {q:>6} gap {gap:7.1f} {(e - s) / 1e3:7.1f} us  {n.replace('void ', '').replace('dfp::', '')[:80]}")
print(f"step span {(rows[i1][0] - t0) / 1e3:.1f} us")
