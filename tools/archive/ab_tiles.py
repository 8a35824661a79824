"""A/B helper: run bench.py with a forced tile count (the former INSR_SPLIT_TILES_* env knobs,
now the per-call INSR_JET_TILES mode bits, set as the bench thread's knob scope).  MIN_BLOCKS one of
128 / 256 / 512 / 1024.  Usage:
    python tools/ab_tiles.py FWD BWD MIN_BLOCKS -- <bench.py args>"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]

if __name__ == "__main__":
    fwd, bwd, mb = (int(v) for v in sys.argv[1:4])
    import base
    base._native.load()
    base._native.set_default_knobs(tiles=(fwd, bwd, mb))
    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[5:]
    runpy.run_path(sys.argv[0], run_name="__main__")
