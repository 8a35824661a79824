"""Precision record of the DEFAULT policy (round 5): every op the models use and every parameter
gradient, through the library's default kernels at the BASELINE batch sizes -- f16x3 forwards, the
default backward routing (the resident f16x3 Laplacian backward from 4,096 points, the fused value
backward, the two-kernel gradient backward) -- and one Adam step through the fused sums + Adam
epilogue (base._jet.defer_reductions, as BaseModel._update_network runs it), each against an fp64
evaluation of the reference algorithm (oracle/siren_oracle.py in double).  The reference's own fp32
error (the oracle in fp32) is printed beside it: the headroom to the north_star's 1e-5 is
1e-5 / err_hip.  One JSON line per (net, op, n).

    python tools/prec_defaults.py [--sizes fluid_pres:16708,fluid_pres:65536,...]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]

import torch  # noqa: E402

from oracle import siren_oracle as O  # noqa: E402

NETS = {"fluid_pres": (2, 1, 4, 128), "fluid_vel": (2, 2, 4, 128), "advect": (1, 1, 3, 64),
        "el2d": (2, 2, 5, 128), "el3d": (3, 3, 5, 256)}
OPS = {"fluid_pres": ("laplace", "gradient"), "fluid_vel": ("value", "jacobian"), "advect": ("value", "gradient"),
       "el2d": ("jacobian",), "el3d": ("jacobian",)}
DEFAULT = ("fluid_pres:16708,fluid_pres:65536,fluid_vel:16708,fluid_vel:65536,advect:4136,el2d:20400,"
           "el3d:16384")


def nerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


def oracle_op(op, ref, x):
    y = ref(x)
    return {"value": lambda: y, "gradient": lambda: O.op_gradient(y, x), "jacobian": lambda: O.op_jacobian(y, x)[0],
            "laplace": lambda: O.op_laplace(y, x)}[op]()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default=DEFAULT)
    ap.add_argument("--lr", type=float, default=1e-4)
    args = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    import base
    from base import _jet
    base._native.load()
    for item in args.sizes.split(","):
        name, n = item.split(":")
        n = int(n)
        din, dout, L, W = NETS[name]
        for op in OPS[name]:
            t0 = time.time()
            torch.manual_seed(0)
            ref32 = O.OracleSiren(din, dout, L, W)
            ref64 = O.OracleSiren(din, dout, L, W)
            ref64.load_state_dict(ref32.state_dict())
            ref64 = ref64.double()
            torch.manual_seed(0)
            net = base.MLP(din, dout, L, W, nonlinearity="sine").cuda()
            x = torch.rand(n, din, generator=torch.Generator().manual_seed(1)) * 2 - 1
            x32 = x.clone().requires_grad_(True)
            x64 = x.double().requires_grad_(True)
            v64 = oracle_op(op, ref64, x64)
            v32 = oracle_op(op, ref32, x32)
            R = torch.randn(v64.shape, generator=torch.Generator().manual_seed(2), dtype=torch.float64)
            (v64 * R).sum().backward()
            (v32 * R.float()).sum().backward()
            g64 = [p.grad if p.grad is not None else torch.zeros_like(p) for p in ref64.parameters()]
            g32 = [p.grad if p.grad is not None else torch.zeros_like(p) for p in ref32.parameters()]
            # the product path: default kernels; backward + one Adam step as BaseModel._update_network
            # runs them (batched reverse jets, the sums held back for the fused sums + Adam launch)
            opt = base.FusedAdam([{"params": list(net.parameters()), "lr": args.lr, "module": net}])
            p0 = [p.detach().clone() for p in net.parameters()]
            xg = x.cuda().requires_grad_(True)
            y = net(xg)
            v = {"value": lambda: y, "gradient": lambda: base.gradient(y, xg),
                 "jacobian": lambda: base.jacobian(y, xg)[0], "laplace": lambda: base.laplace(y, xg)}[op]()
            opt.zero_grad()
            with _jet.defer_reductions():
                with _jet.batched_backward():
                    (v * R.float().cuda()).sum().backward()
                fused = "_insr_pending_reduce" in net.__dict__
                gh = [p.grad.detach().clone() if p.grad is not None else None for p in net.parameters()] \
                    if not fused else None
                opt.step()
            torch.cuda.synchronize()
            if gh is None:  # the sums landed in the Adam launch: .grad holds them afterwards
                gh = [p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p) for p in net.parameters()]
            pe_hip = [nerr(a, b) for a, b in zip(gh, g64)]
            pe_ref = [nerr(a, b) for a, b in zip(g32, g64)]
            # Adam step 1 against fp64 Adam on the fp64 gradient (entries whose sign is not at the noise floor)
            ad = 0.0
            for p, q0, g in zip(net.parameters(), p0, g64):
                m = 0.1 * g
                vv = 0.001 * g * g
                step = -(args.lr / 0.1) * m / ((vv / 0.001).sqrt() + 1e-8)
                live = g.abs() > 1e-3 * g.abs().max()
                d = (p.detach().double().cpu() - q0.double().cpu()) - step
                if bool(live.any()):
                    ad = max(ad, float(d[live].abs().max()) / args.lr)
            rec = {"net": name, "op": op, "n": n, "policy": "default", "fused_sums_adam": fused,
                   "field_err_hip_vs_fp64": nerr(v, v64), "field_err_ref_fp32_vs_fp64": nerr(v32, v64),
                   "param_grad_err_hip_vs_fp64_max": max(pe_hip), "param_grad_err_ref_fp32_vs_fp64_max": max(pe_ref),
                   "param_grad_err_hip_vs_fp64": [round(e, 9) for e in pe_hip],
                   "adam_step_err_over_lr": ad, "seconds": round(time.time() - t0, 1)}
            rec["headroom_to_1e-5"] = 1e-5 / max(rec["field_err_hip_vs_fp64"], rec["param_grad_err_hip_vs_fp64_max"])
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
