"""Concurrent kernels in a rocprofv3 --kernel-trace CSV: for every pair of kernel families whose dispatches
ran at the same time (intervals intersecting, e.g. a side-stream frozen-network jet under a reverse jet), the
number of overlapping dispatch pairs and the overlapped time; plus the busy time of the trace (union of the
intervals) against the sum of the kernel durations -- their difference is the time concurrency saved.

    python tools/trace_overlap.py gpurun_out/<dir>/run_kernel_trace.csv [--tail N] [--top 12]
"""
import argparse
import csv


def family(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--tail", type=int, default=0, help="only the last N kernels (steady state)")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    if a.tail:
        rows = rows[-a.tail:]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), family(r["Kernel_Name"])) for r in rows]
    total = sum(e - s for s, e, _ in iv)
    union, cur_s, cur_e = 0, None, None
    for s, e, _ in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        union += cur_e - cur_s
    pairs = {}
    for i, (s, e, f) in enumerate(iv):
        for s2, e2, f2 in iv[i + 1:]:
            if s2 >= e:
                break
            ov = min(e, e2) - s2
            if ov > 0:
                k = tuple(sorted((f, f2)))
                c = pairs.setdefault(k, [0, 0])
                c[0] += 1
                c[1] += ov
    span = iv[-1][1] - iv[0][0] if iv else 0
    print(f"{len(iv)} kernels, span {span / 1e3:.1f} us, sum of durations {total / 1e3:.1f} us, busy (union) "
          f"{union / 1e3:.1f} us, concurrency saved {(total - union) / 1e3:.1f} us")
    for (f1, f2), (n, ov) in sorted(pairs.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {n:6d} overlaps {ov / 1e3:10.1f} us  {f1}  ||  {f2}")


if __name__ == "__main__":
    main()
