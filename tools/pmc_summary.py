"""Per-dispatch HBM traffic of the HIP kernels from rocprofv3 --pmc runs.

    python tools/pmc_summary.py gpurun_out/s13 > profiles/r01/pmc_traffic.json

Reads <dir>/pmc_fetch/*counter_collection.csv (FETCH_SIZE) and <dir>/pmc_write/...
(WRITE_SIZE), which MUST come from separate passes (TCC counter slots), and
<dir>/pmc_sq/... (SQ stall counters) when present.  Corrections as prescribed in
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE counts half the bytes of 16-B/lane streaming reads, so it is
doubled; WRITE_SIZE is exact for 16-B/lane streaming stores.  Keys are
"<kernel name>|grid=<threads>", values are means over the profiled dispatches.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(path):
    agg = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(path, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
            agg[f"{name}|grid={r['Grid_Size']}"][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(d):
    fetch, write, sq = load(os.path.join(d, "pmc_fetch")), load(os.path.join(d, "pmc_write")), \
        load(os.path.join(d, "pmc_sq"))
    out = {"_source": f"rocprofv3 --pmc, separate FETCH_SIZE / WRITE_SIZE / SQ passes of bench.py --no-graph ({d})",
           "_units": "bytes per dispatch; fetch_bytes = 2 x FETCH_SIZE KiB x 1024 (gfx950 correction)"}
    for k in sorted(set(fetch) | set(write)):
        e = {}
        if "FETCH_SIZE" in fetch.get(k, {}):
            v = fetch[k]["FETCH_SIZE"]
            e["fetch_bytes"] = round(2 * 1024 * sum(v) / len(v))
            e["dispatches"] = len(v)
        if "WRITE_SIZE" in write.get(k, {}):
            v = write[k]["WRITE_SIZE"]
            e["write_bytes"] = round(1024 * sum(v) / len(v))
        if k in sq:
            e["sq"] = {c: round(sum(v) / len(v)) for c, v in sq[k].items()}
        out[k] = e
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
