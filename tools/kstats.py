#!/usr/bin/env python3
"""Print the kernels of rocprofv3 --stats CSVs (one per argument) above a time floor."""
import csv
import sys

floor_us = 3.0
for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        us = float(r["AverageNs"]) / 1e3
        if us >= floor_us:
            print(f"  {r['Name'][:64]:64s} {r['Calls']:>4} {us:9.1f}us")
