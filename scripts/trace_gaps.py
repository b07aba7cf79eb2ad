#!/usr/bin/env python3
"""Busy vs idle time of a rocprofv3 kernel trace: the kernels sorted by start, split into
bursts at idle gaps longer than --burst-gap us (one burst = one decode call of a probe), and per
burst its span, the sum of kernel durations, the idle time between kernels and the largest gaps
(with the kernels on either side).  usage: trace_gaps.py kernel_trace.csv [--burst-gap 2000]"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    burst_gap = float(sys.argv[sys.argv.index("--burst-gap") + 1]) if "--burst-gap" in sys.argv else 2000.0
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), re.sub(r"\(.*", "", r["Kernel_Name"]))
                 for r in rows), key=lambda k: k[0])
    bursts, cur = [], [ks[0]]
    for k in ks[1:]:
        if (k[0] - max(x[1] for x in cur[-4:])) / 1e3 > burst_gap:
            bursts.append(cur)
            cur = []
        cur.append(k)
    bursts.append(cur)
    for i, b in enumerate(bursts):
        span = (max(k[1] for k in b) - b[0][0]) / 1e3
        busy = sum(k[1] - k[0] for k in b) / 1e3
        gaps, end = [], b[0][1]
        for p, k in zip(b, b[1:]):
            g = (k[0] - end) / 1e3
            if g > 0:
                gaps.append((g, p[2][-40:], k[2][-40:]))
            end = max(end, k[1])
        idle = sum(g[0] for g in gaps)
        print(f"burst {i}: {len(b)} kernels, span {span / 1e3:.2f} ms, kernels {busy / 1e3:.2f} ms, idle {idle / 1e3:.2f} ms")
        for g in sorted(gaps, reverse=True)[:5]:
            print(f"    gap {g[0]:8.1f} us  after {g[1]}  before {g[2]}")


if __name__ == "__main__":
    main()
