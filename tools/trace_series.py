"""Print the durations (us) of the dispatches of each kernel whose name contains one of the
given substrings, in dispatch order, from a rocprofv3 kernel_trace.csv (grouped by GROUP
dispatches: mean of each group).

usage: trace_series.py TRACE.csv GROUP[:SKIP] SUBSTR [SUBSTR ...]  (SKIP: leading dispatches
of each group left out of its mean)
"""
import csv
import sys

path = sys.argv[1]
group, skip = (int(x) for x in (sys.argv[2] + ":0").split(":")[:2])
for sub in sys.argv[3:]:
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    groups = [d[i + skip:i + group] for i in range(0, len(d), group)]
    print(sub, " | ".join(f"{sum(g) / len(g):7.1f}" for g in groups))
