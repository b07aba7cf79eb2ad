#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    name = re.sub(r"\(.*", "", r["Name"]).replace("tts::", "")
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):7d} x {float(r['AverageNs'])/1e3:8.2f} us "
          f"{100*float(r['TotalDurationNs'])/tot:5.1f}%  {name[:90]}")
