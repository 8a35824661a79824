"""Diagnostic (results NOT valid): bench.py with the Adam launch's weight-plane writes switched off
(shapes = NULL: the planes go stale, so the jets after it compute with old weights) -- to see whether
the ~8.5 us idle gap after every adam_multi_kernel in the kernel trace comes from those scattered
2-byte plane stores.  Run under rocprofv3 --kernel-trace and compare the gaps with a normal run.

    rocprofv3 --kernel-trace -d out -o run --output-format csv -- python tools/diag_adam_gap.py --steps 10
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]

if __name__ == "__main__":
    import base._native as nat
    real = nat.load()

    class _NoPlanes:
        def __getattr__(self, name):
            f = getattr(real, name)
            if name == "insr_adam_step_nets":
                return lambda *a: f(*a[:6], None, *a[7:])
            if name == "insr_adam_plateau_step_nets":
                return lambda *a: f(*a[:6], None, *a[7:])
            return f
    nat._lib = _NoPlanes()
    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:] + ["--no-cpu-baseline", "--no-roofline"]
    runpy.run_path(sys.argv[0], run_name="__main__")
