"""Summarise a rocprofv3 kernel_trace.csv: per (kernel, grid) average duration and
per-step time, plus the idle gaps between consecutive kernels on the GPU."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
agg = defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    name = name[:60]
    agg[(name, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0
out = []
for (name, grid), d in agg.items():
    s = sum(d)
    tot += s
    out.append((s, name, grid, len(d), s / len(d)))
for s, name, grid, n, avg in sorted(out, reverse=True)[:30]:
    print(f"{name:60s} blocks={grid:6d} n={n:5d} avg={avg:8.2f}us per_step={s / steps:8.1f}us")
gaps = 0.0
for a, b in zip(rows, rows[1:]):
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    if 0 < g < 200:
        gaps += g
print(f"kernel time per step {tot / steps:.1f} us; small gaps (<200us) per step {gaps / steps:.1f} us")
