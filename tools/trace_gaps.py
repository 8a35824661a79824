"""Idle gaps between consecutive kernels of a rocprofv3 --kernel-trace CSV: per (kernel -> next
kernel) pair the count, median and sum of (next start - this end), the largest sums first.

    python tools/trace_gaps.py gpurun_out/<dir>/run_kernel_trace.csv [--top 12] [--tail N]
"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--tail", type=int, default=0, help="only the last N kernels (steady state)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    if a.tail:
        rows = rows[-a.tail:]
    gaps = {}
    for x, y in zip(rows, rows[1:]):
        k = x["Kernel_Name"].split("(")[0][:48] + " -> " + y["Kernel_Name"].split("(")[0][:48]
        gaps.setdefault(k, []).append((int(y["Start_Timestamp"]) - int(x["End_Timestamp"])) / 1000.0)
    print(f"{len(rows)} kernels")
    for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        print(f"{k:100s} n={len(v):5d} median={statistics.median(v):8.2f} us sum={sum(v):10.1f} us")


if __name__ == "__main__":
    main()
