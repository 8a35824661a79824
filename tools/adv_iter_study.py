"""Timing study of the one-launch advection iteration (csrc/advect_iter.hip): the launch alone over batch
sizes and hidden-layer counts (HIP events, 50 launches each), and with --diag the s_memtime phase stamps of
block 0's first tile (the diagnostic library, make -C insr-pde_amd/csrc diag).

    python tools/adv_iter_study.py [--diag]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]
import torch  # noqa: E402

STAMP_NAMES = {0: "tile start", 1: "draw + layer 0", 2: "layer-0 sincos/LDS", 3: "barrier", 4: "L1 gemm",
               6: "L2 gemm", 8: "L3 gemm", 12: "fwd tail", 13: "out layer + residual", 31: "reverse end"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--diag", action="store_true")
    a = ap.parse_args()
    import base
    from base import _native as nat
    from base import advect_iter
    lib = nat.load(os.path.join(ROOT, "insr-pde_amd", "lib", "libinsr_hip_diag.so") if a.diag else None,
                   check_build=not a.diag)
    for L in (3, 1):
        torch.manual_seed(0)
        net = base.MLP(1, 1, L, 64, nonlinearity="sine").cuda()
        prev = base.MLP(1, 1, L, 64, nonlinearity="sine").cuda()
        for n in (16, 1024, 4096, 16384, 65536):
            h = max(n // 100, 10) // 2
            with torch.no_grad():
                for _ in range(3):
                    advect_iter.advect1d_iteration(net, prev, n, h, 1.5, 1e-4, 0.05, 1.0, n, 2 * h)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    advect_iter.advect1d_iteration(net, prev, n, h, 1.5, 1e-4, 0.05, 1.0, n, 2 * h)
                e1.record()
                torch.cuda.synchronize()
            rows = lib.insr_advect1d_rows(n + 2 * h)
            print(f"L={L} n={n}+{2 * h} blocks={rows}: {e0.elapsed_time(e1) / 50 * 1000:.1f} us per launch", flush=True)
            if a.diag and n == 4096:
                buf = (ctypes.c_ulonglong * 256)()
                lib.insr_diag_stamps_adv.argtypes = [ctypes.c_void_p, ctypes.c_int]
                lib.insr_diag_stamps_adv(buf, 256)
                for w in range(8):
                    st = [buf[w * 32 + k] for k in range(32)]
                    t0 = st[0]
                    marks = [(k, st[k] - t0) for k in range(32) if st[k] >= t0 and st[k] - t0 < 10 ** 8]
                    print(f"  wave {w}: " + " ".join(f"{k}:{v}" for k, v in marks), flush=True)


if __name__ == "__main__":
    main()
