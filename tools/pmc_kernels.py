#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counters per kernel (every *counter_collection.csv under DIR):
kernel short name, dispatches, and each counter's average per dispatch.

usage: pmc_kernels.py DIR [NAME_REGEX]
"""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "").replace("dfp::", "")
        if pat and not pat.search(name):
            continue
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r["Dispatch_Id"])
for name, ctrs in sorted(acc.items(), key=lambda kv: -len(disp[kv[0]])):
    n = len(disp[name])
    print(f"{name[:60]:60s} n={n:3d} " + " ".join(f"{c}={v / n:.4g}" for c, v in sorted(ctrs.items())))
