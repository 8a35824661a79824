"""List the kernels of one benchmark step from a rocprofv3 kernel trace: the span
between two consecutive launches of the anchor kernel (default: the Laplacian
backward), with durations; prints totals by kernel family.

    python tools/step_kernels.py gpurun_out/sNN/prof/run_kernel_trace.csv [anchor-substring]
"""
import csv
import sys
from collections import defaultdict


def main(path, anchor="jet_bwd_split<8, 4, true"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    a, b = idx[-3], idx[-2]
    per = rows[a + 1:b + 1]
    fam = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in per:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        busy += d
        name = r["Kernel_Name"].replace("void ", "")
        key = name.split("(")[0] if name.startswith("insr::") else "torch/runtime: " + name.split("<")[0].split("(")[0]
        fam[key][0] += 1
        fam[key][1] += d
    for k, (n, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"{t:8.1f} us  {n:3d}x  {k}")
    print(f"{len(per)} kernels, {busy:.1f} us busy per step")


if __name__ == "__main__":
    main(*sys.argv[1:])
