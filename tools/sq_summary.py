#!/usr/bin/env python3
"""Per-kernel averages of one rocprofv3 --pmc pass (SQ counters) over a
tools/probe_one.py run: usage sq_summary.py DIR (holds sq_counter_collection.csv).
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import sys

path = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dfp::", "")
    if not any(k in name for k in ("sl_", "hs_", "dense_frag", "hashed_frag", "key_minmax")):
        continue
    acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in acc.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
    parts = " ".join(f"{c.replace('SQ_', '')}={v:.3g}" for c, v in sorted(avg.items()))
    frac = " ".join(f"{c.replace('SQ_', '')}/WAVE={avg[c] / wc:.2f}" for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                             "SQ_ACTIVE_INST_ANY") if c in avg)
    print(f"{name[:40]:40s} {frac}\n    {parts}")
