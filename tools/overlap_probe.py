"""Probe: can a phase's no-grad target jets (frozen networks, independent of the training step)
run in the resources a reverse jet leaves idle?  Times, at the fluid2Dtlgn / 8-way-shard sizes,
(A) the velocity value backward alone (jet_bwd_x6 + its row sums), (B) the advection target alone
(u_prev(clamp(x - dt u_prev(x))), one mixed launch), (C) both issued together on two streams, and the
same for the pressure phase's Laplacian backward (jet_fb_x6 + sums) beside the velocity Jacobian jet.
Prints one JSON line per (size, pair): the concurrent time against max / sum of the two alone.

    python tools/overlap_probe.py [--sizes 16384,8192] [--reps 30]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]

import torch  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps  # us per rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="16384,8192")
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    import base
    from base import _jet
    base._native.load()
    torch.manual_seed(0)
    vel = base.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    vel_prev = base.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    pres = base.MLP(2, 1, 4, 128, nonlinearity="sine").cuda()
    for p in vel_prev.parameters():
        p.requires_grad_(False)
    side = torch.cuda.Stream()
    for n in [int(v) for v in args.sizes.split(",")]:
        nb = (n // 100) // 2 * 4
        xa = (torch.rand(n + nb, 2, device="cuda") * 2 - 1).requires_grad_(True)
        x = xa[:n]
        # value phase: a saved value forward of the trainable field, its backward = A
        ya = vel(xa)
        gy = torch.randn_like(ya)

        def bwd_value():
            vel.mark_grad_stale()
            torch.autograd.backward(ya, gy, retain_graph=True)

        def target_advect():
            with torch.no_grad():
                _jet.advect_target(vel_prev, x.detach(), 0.05, -1.0, 1.0)

        # pressure phase: saved Laplacian forward of the pressure field, its backward; the velocity Jacobian
        lap, g = base.laplace(pres(xa), xa, return_grad=True)
        glap = torch.randn_like(lap)

        def bwd_lap():
            pres.mark_grad_stale()
            torch.autograd.backward(lap, glap, retain_graph=True)

        xd = x.detach()

        def target_jac():
            with torch.no_grad():
                _jet.run_jet(vel, xd, base._native.MODE_GRAD)

        for name, a, b in (("value_bwd+advect_target", bwd_value, target_advect),
                           ("lap_bwd+velocity_jacobian", bwd_lap, target_jac)):
            ta = timed(a, args.reps)
            tb = timed(b, args.reps)

            def both():
                side.wait_stream(torch.cuda.current_stream())
                a()
                with torch.cuda.stream(side):
                    b()
                torch.cuda.current_stream().wait_stream(side)
            tc = timed(both, args.reps)
            print(json.dumps({"n": n, "pair": name, "a_us": round(ta, 2), "b_us": round(tb, 2),
                              "concurrent_us": round(tc, 2), "max_us": round(max(ta, tb), 2),
                              "sum_us": round(ta + tb, 2), "hidden_frac": round((ta + tb - tc) / min(ta, tb), 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
