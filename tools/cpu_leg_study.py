"""Stability of bench.py's CPU leg on the GPU box (verdict r5 item 8): the oracle's fluid2Dtlgn step timed
in fresh CPU-only child processes under several thread counts, with and without pinning the process to a
fixed CPU set before torch starts its thread pool.  Prints the box's CPU share (cgroup quota / cpuset /
affinity / OMP_NUM_THREADS / load) and one JSON line per configuration (min / median / max ms per
iteration, spread = max / min).  No GPU work.

  python tools/cpu_leg_study.py [seconds per configuration]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def share():
    info = {"affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count(),
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "loadavg": os.getloadavg()}
    for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective", "/sys/fs/cgroup/cpu.weight"):
        try:
            info[os.path.basename(f)] = open(f).read().strip()
        except OSError:
            info[os.path.basename(f)] = None
    return info


CHILD = r'''
import json, os, sys, time
threads, pin, seconds = int(sys.argv[1]), sys.argv[2], float(sys.argv[3])
if len(sys.argv) > 6 and sys.argv[6] == "passive":  # (must precede the OpenMP runtime's start)
    os.environ["OMP_WAIT_POLICY"] = "PASSIVE"
    os.environ["GOMP_SPINCOUNT"] = "0"
cpus = sorted(os.sched_getaffinity(0))
if pin == "first":
    os.sched_setaffinity(0, cpus[:threads])
elif pin == "spread":
    step = max(1, len(cpus) // threads)
    os.sched_setaffinity(0, cpus[::step][:threads])
os.environ["OMP_NUM_THREADS"] = str(threads)  # (OMP_PROC_BIND=close on top of the affinity: 5x slower here)
sys.path.insert(0, sys.argv[4])
import bench
r = bench.cpu_baseline("fluid2Dtlgn", seconds, n_rounds=1, iters=int(sys.argv[5]))
print(json.dumps(r))
'''


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    print(json.dumps({"share": share()}), flush=True)
    omp = int(os.environ.get("OMP_NUM_THREADS", "16"))
    h = max(1, omp // 2)
    configs = [(max(1, omp * 3 // 4), "none", "active"), (max(1, omp * 3 // 4), "none", "passive"),
               (h, "none", "passive"), (h, "first", "passive"), (h, "spread", "passive"),
               (max(1, omp // 4), "none", "passive"), (max(1, omp * 3 // 4), "none", "passive")]
    for threads, pin, wait in configs:
        t0 = time.time()
        out = subprocess.run([sys.executable, "-c", CHILD, str(threads), pin, str(seconds), ROOT, "20", wait],
                             capture_output=True, text=True, timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else None
        rec = {"threads": threads, "pin": pin, "omp_wait": wait, "wall_s": round(time.time() - t0, 1)}
        if line:
            r = json.loads(line)
            rec.update({k: r.get(k) for k in ("value", "value_min_time", "spread_max_over_min", "statistic",
                                               "rounds")})
        else:
            rec["error"] = out.stderr[-500:]
        print(json.dumps(rec), flush=True)
    print(json.dumps({"share_after": share()}), flush=True)


if __name__ == "__main__":
    main()
