"""Same-box A/B helper: bench.py with the sampler draw plan switched off (every sampler call its own
insr_sample_boxes launch, base/sampling.py draw_plan -> no-op).  Tools only; the product always plans.

    python tools/ab_noplan.py --api plain --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
"""
import contextlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]
import base._loop as L  # noqa: E402

L.draw_plan = lambda owner: contextlib.nullcontext()
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
