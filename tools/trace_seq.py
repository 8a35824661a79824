"""The kernel sequence of a rocprofv3 --kernel-trace CSV: the last N dispatches in start order with their
duration, the idle gap before each, and the grid / workgroup sizes (to tell copies and small launches apart).

    python tools/trace_seq.py gpurun_out/<dir>/run_kernel_trace.csv [--tail 60]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--tail", type=int, default=60)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))[-a.tail:]
    prev = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000.0 if prev is not None else 0.0
        grid = r.get("Grid_Size_X") or r.get("Grid_Size", "")
        wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size", "")
        print(f"{gap:8.2f} {(e - s) / 1000.0:8.2f}  grid={grid:>9s} wg={wg:>4s}  {r['Kernel_Name'].split('(')[0][:70]}")
        prev = e


if __name__ == "__main__":
    main()
