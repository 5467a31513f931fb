#!/usr/bin/env python3
"""Print the device timeline of one bench step from a rocprofv3 kernel-trace CSV: every
kernel/copy of the step (from its key_minmax_kernel to the next one) with the idle gap
before it. usage: step_timeline.py KERNEL_TRACE_CSV [step index from the end, default 2]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
idx = [i for i, r in enumerate(rows) if "key_minmax" in r["Kernel_Name"]]
i0, i1 = idx[-back], idx[-back + 1]
t0 = int(rows[i0]["Start_Timestamp"])
prev = t0
busy = 0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1e3:8.1f}  gap {(s - prev) / 1e3:6.1f}  {(e - s) / 1e3:7.1f} us  {r['Kernel_Name'][:70]}")
    prev = e
end = int(rows[i1]["Start_Timestamp"])
print(f"step span {(end - t0) / 1e3:.1f} us, device busy {busy / 1e3:.1f} us, idle {(end - t0 - busy) / 1e3:.1f} us")
