#!/usr/bin/env python3
"""Print a rocprofv3 --stats kernel summary (every *kernel_stats.csv under DIR) as
short name, calls, average and total microseconds, sorted by total time.

usage: kstats.py DIR [DIR ...]
"""
import csv
import glob
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*$", "", name)          # drop the argument list
    name = re.sub(r"^void ", "", name)
    return name.replace("dfp::", "")


for d in sys.argv[1:]:
    for path in sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)):
        rows = list(csv.DictReader(open(path)))
        rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
        print(f"# {path}")
        for r in rows:
            print(f"{short(r['Name'])[:70]:70s} {int(r['Calls']):6d} avg {float(r['AverageNs']) / 1e3:9.2f} us"
                  f"  min {float(r['MinNs']) / 1e3:9.2f}  total {float(r['TotalDurationNs']) / 1e3:10.1f} us")
