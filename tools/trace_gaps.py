"""Per-kernel durations and the idle gaps between consecutive dispatches
from a rocprofv3 --kernel-trace CSV (diagnostic for launch-bound loops).
usage: trace_gaps.py <kernel_trace.csv> [name-substring]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
by = {}
prev_end = None
gaps = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"]
    by.setdefault(name[:60], []).append((e - s) / 1e3)
    if prev_end is not None and sub in name:
        gaps.append((s - prev_end) / 1e3)
    prev_end = max(prev_end or 0, e)
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    v2 = sorted(v)
    print(f"{len(v):6d} x {k:60s} mean {sum(v) / len(v):8.2f} med {v2[len(v2) // 2]:8.2f} us  total {sum(v) / 1e3:8.2f} ms")
if gaps:
    g = sorted(gaps)
    n = len(g)
    print(f"gaps before '{sub}': n {n} mean {sum(g) / n:.2f} med {g[n // 2]:.2f} p90 {g[int(n * 0.9)]:.2f} "
          f"p99 {g[int(n * 0.99)]:.2f} max {g[-1]:.2f} us; sum {sum(x for x in g if x > 0) / 1e3:.2f} ms")
    big = [x for x in gaps if x > 5]
    print(f"gaps > 5 us: {len(big)}, summing {sum(big) / 1e3:.2f} ms")
