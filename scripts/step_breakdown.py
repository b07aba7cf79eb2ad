"""Per-kernel breakdown of one graph-replayed decode step from a rocprofv3 kernel trace
(run_kernel_trace.csv): kernels between two consecutive finalize launches, averaged over
the middle steps.   usage: python scripts/step_breakdown.py TRACE.csv"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    m = re.match(r"(?:void )?tts::(?:\(anonymous namespace\)::)?(\w+)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


fin = [i for i, r in enumerate(rows) if "finalize" in r["Kernel_Name"]]
mid = fin[len(fin) // 4: 3 * len(fin) // 4]
agg = collections.OrderedDict()
spans = []
for a, b in zip(mid, mid[1:]):
    seg = rows[a + 1:b + 1]
    spans.append((int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1000)
    for r in seg:
        agg.setdefault(short(r["Kernel_Name"])[:80], []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
n = max(1, len(spans))
print(f"steps {n}  span/step {sum(spans) / n:.1f} us  kernels/step {sum(len(v) for v in agg.values()) / n:.0f}")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:80s} per-step {len(v) / n:5.1f} x {sum(v) / len(v):7.2f} us = {sum(v) / n:8.1f} us")
