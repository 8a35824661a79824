"""Attribute the torch kernels of the plain reference-API fluid step (pde/fluid_plain.py, the
reference's fluid/model.py:72-151 phase bodies) to their source expressions.

The network calls and the diff-ops are replaced by leaf tensors of the jets' output shapes (what
base hands back: u (n, 2), p (n, 1), J (n, c, 2), lap (n, 1)); everything else is the phase
body's own torch code, run forward and backward (unit seeds, as BaseModel._backward) under
torch.profiler on the CPU.  Ops that launch no kernel on the GPU (views, empty allocations) are
dropped; the rest are listed per phase and per source line.  base-internal ops are marked
[base]; the diff-op assembly (J[..., 0, 0:1] + J[..., 1, 1:2] for divergence) is the only one.

    python tools/plain_glue_count.py
"""
import collections

import torch
from torch.profiler import ProfilerActivity, profile

NO_KERNEL = {"aten::select", "aten::slice", "aten::view", "aten::expand", "aten::as_strided",
             "aten::empty", "aten::empty_like", "aten::empty_strided", "aten::detach", "aten::alias",
             "aten::reshape", "aten::unsqueeze", "aten::squeeze", "aten::t", "aten::transpose",
             "aten::lift_fresh", "aten::resolve_conj", "aten::resolve_neg", "detach", "aten::_unsafe_view",
             "aten::result_type", "aten::to", "aten::_to_copy", "aten::ones_like", "aten::zeros",
             "aten::new_empty_strided", "aten::is_nonzero", "aten::item", "aten::_local_scalar_dense"}
N, NB, DT = 16384, 162, 0.05


def leaf(*shape):
    return torch.randn(*shape, requires_grad=True)


def advect():
    x = torch.rand(N, 2) * 2 - 1
    u_old, u, target = torch.randn(N, 2), leaf(N, 2), torch.randn(N, 2)
    ux, uy = leaf(NB, 2), leaf(NB, 2)
    yield "foot = clamp(x - u_old * dt)   (fluid/model.py:83-84)", lambda: torch.clamp(x - u_old * DT, -1.0, 1.0)
    yield "mean((u - target) ** 2)        (fluid/model.py:89)", lambda: torch.mean((u - target) ** 2)
    yield "bc: (mean(ux[...,0]**2) + mean(uy[...,1]**2)) * 1.0  (fluid/model.py:96-98)", \
        lambda: (torch.mean(ux[..., 0] ** 2) + torch.mean(uy[..., 1] ** 2)) * 1.0


def pressure():
    J = torch.randn(N, 2, 2)
    lap = leaf(N, 1)
    gx, gy = leaf(NB, 2), leaf(NB, 2)  # gradient(p, b): a view of the (NB, 1, 2) jet output
    yield "[base] divergence: J[...,0,0:1] + J[...,1,1:2]  (diff_ops.divergence)", lambda: J[..., 0, 0:1] + J[..., 1, 1:2]
    div = J[..., 0, 0:1] + J[..., 1, 1:2]
    yield "mean((div_u - lap_p) ** 2)     (fluid/model.py:113)", lambda: torch.mean((div - lap) ** 2)
    yield "bc: mean(gx[...,0]**2) + mean(gy[...,1]**2)  (fluid/model.py:119-122)", \
        lambda: torch.mean(gx[..., 0] ** 2) + torch.mean(gy[..., 1] ** 2)


def projection():
    u_old, grad_p, u = torch.randn(N, 2), torch.randn(N, 2), leaf(N, 2)
    ux, uy = leaf(NB, 2), leaf(NB, 2)
    yield "target = u_old - grad_p; mean((u - target) ** 2)  (fluid/model.py:138-140)", \
        lambda: torch.mean((u - (u_old - grad_p)) ** 2)
    yield "bc: (mean(ux[...,0]**2) + mean(uy[...,1]**2)) * 1.0  (fluid/model.py:147-149)", \
        lambda: (torch.mean(ux[..., 0] ** 2) + torch.mean(uy[..., 1] ** 2)) * 1.0


def count(fn):
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        out = fn()
        if out.requires_grad:
            out.backward(torch.ones_like(out))
    ops = collections.Counter()
    for ev in prof.events():
        if ev.name.startswith("aten::") and ev.name not in NO_KERNEL and ev.cpu_parent is not None \
                and not ev.cpu_parent.name.startswith("aten::"):
            ops[ev.name] += 1
        elif ev.name.startswith("aten::") and ev.name not in NO_KERNEL and ev.cpu_parent is None:
            ops[ev.name] += 1
    return ops


def main():
    total = 0
    for phase in (advect, pressure, projection):
        sub = 0
        print(f"== {phase.__name__}")
        for label, fn in phase():
            ops = count(fn)
            n = sum(ops.values())
            sub += n
            print(f"  {n:3d}  {label}\n       {dict(ops)}")
        print(f"  {sub:3d}  total {phase.__name__}")
        total += sub
    print(f"{total} torch ops with a kernel per step (fwd + bwd)")


if __name__ == "__main__":
    main()
