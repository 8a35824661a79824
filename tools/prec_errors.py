"""Normwise error of the HIP jets against the CPU oracle for each matrix-core
precision (fp32 MFMA, split-bf16 x6 / x3, plain bf16), per network / op: value, derivative and
parameter gradients.  Prints one JSON line per (net, op, precision).

    python tools/prec_errors.py [--n 4000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]

import torch  # noqa: E402

from oracle import siren_oracle as O  # noqa: E402

NETS = {"fluid_pres": (2, 1, 4, 128), "fluid_vel": (2, 2, 4, 128), "advect": (1, 1, 3, 64),
        "el2d": (2, 2, 5, 128), "el3d": (3, 3, 5, 256)}


def nerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4000)
    ap.add_argument("--nets", default=",".join(NETS))
    ap.add_argument("--combos", default="0:0,1:1,2:2,3:3",
                    help="forward:backward precision pairs (0 fp32, 1 bf16x6, 2 bf16x3, 3 bf16), comma separated")
    ap.add_argument("--bwd-f16", type=int, default=-1, help="INSR_JET_BWD_F16 mask (-1: library default)")
    args = ap.parse_args()
    combos = [tuple(int(v) for v in c.split(":")) for c in args.combos.split(",")]
    names = ["f32", "bf16x6", "bf16x3", "bf16", "f16x3"]
    import base
    lib = base._native.load()
    if args.bwd_f16 >= 0:
        base._native.set_default_knobs(bwd_f16=args.bwd_f16)
    mask = base._native.bwd_f16_mask()
    for name in args.nets.split(","):
        din, dout, L, W = NETS[name]
        torch.manual_seed(0)
        ref = O.OracleSiren(din, dout, L, W)
        torch.manual_seed(0)
        net = base.MLP(din, dout, L, W, nonlinearity="sine").cuda()
        x = torch.rand(args.n, din, generator=torch.Generator().manual_seed(1)) * 2 - 1
        ops = ["value", "gradient", "jacobian"] + (["laplace"] if din <= 2 and dout == 1 else [])
        for op in ops:
            xr = x.clone().requires_grad_(True)
            yr = ref(xr)
            vr = {"value": lambda: yr, "gradient": lambda: O.op_gradient(yr, xr),
                  "jacobian": lambda: O.op_jacobian(yr, xr)[0], "laplace": lambda: O.op_laplace(yr, xr)}[op]()
            R = torch.randn(vr.shape, generator=torch.Generator().manual_seed(2))
            for p in ref.parameters():
                p.grad = None
            (vr * R).sum().backward()
            gref = [p.grad if p.grad is not None else torch.zeros_like(p) for p in ref.parameters()]
            for pf, pb in combos:
                base._native.set_default_knobs(prec=(pf, pb))
                net.zero_grad(set_to_none=True)
                xg = x.cuda().requires_grad_(True)
                y = net(xg)
                v = {"value": lambda: y, "gradient": lambda: base.gradient(y, xg),
                     "jacobian": lambda: base.jacobian(y, xg)[0], "laplace": lambda: base.laplace(y, xg)}[op]()
                (v * R.cuda()).sum().backward()
                torch.cuda.synchronize()
                pe = [nerr(p.grad if p.grad is not None else torch.zeros_like(p), g)
                      for p, g in zip(net.parameters(), gref)]
                print(json.dumps({"net": name, "op": op, "prec": names[pf] if pf == pb else f"{names[pf]}/{names[pb]}", "n": args.n,
                                  "bwd_f16": mask,
                                  "field_err": nerr(v, vr), "param_grad_err_max": max(pe),
                                  "param_grad_err": [round(e, 9) for e in pe]}), flush=True)


if __name__ == "__main__":
    main()
