"""One line per bench JSON output file: value (M pts/s), ms per step, median timestep, CPU baseline.

    python tools/summarize_lines.py gpurun_out/<dir>/*.out
"""
import json
import sys

for path in sys.argv[1:]:
    try:
        line = next(ln for ln in open(path) if ln.startswith("{"))
    except (OSError, StopIteration):
        print(f"{path}: no bench line")
        continue
    d = json.loads(line)
    t = d.get("timesteps") or {}
    c = d.get("cpu_baseline") or {}
    r = d.get("roofline") or {}
    print(f"{path}: {d['value'] / 1e6:.2f} M  {d['ms_per_step']} ms/step  median {((t.get('value_median') or 0) / 1e6):.2f} M"
          + (f"  frac {r.get('frac')}" if r else "")
          + (f"  cpu {c.get('value')} (spread {c.get('spread_max_over_min')}, x{d.get('speedup_vs_cpu_baseline')})" if c else ""))
