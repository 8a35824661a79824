"""Diagnostic: fused vs unfused fluid advect phase, with/without shared loss-gradient buffers."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "insr-pde_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import base
from base import losses
from tests.test_gpu_fused import _fluid

orig_shared = losses._shared_a


def run(phase, fuse, share):
    losses._shared_a = orig_shared if share else (lambda specs: [None] * len(specs))
    g = torch.Generator().manual_seed(9)
    xs = [(torch.rand(4096, 2, generator=g) * 2 - 1).cuda() for _ in range(4)]
    bx = (torch.rand(40, 2, generator=g) * 2 - 1).cuda()
    by = (torch.rand(40, 2, generator=g) * 2 - 1).cuda()
    model = _fluid(None, fuse, False)
    it = {"k": 0}

    def sample():
        x = xs[it["k"] % len(xs)]
        it["k"] += 1
        return x.clone().requires_grad_(True)
    model._sample_in_training = sample
    model._boundary_pair = lambda n: (bx.clone().requires_grad_(True), by.clone().requires_grad_(True))
    model.timestep = 1
    getattr(model, phase)()
    return model.velocity_field.flat_params().detach().clone(), model.pressure_field.flat_params().detach().clone()


base._native.load()
for phase in ("_advect_velocity", "_projection"):
    r = {(f, s): run(phase, f, s) for f in (False, True) for s in (False, True)}
    ref = r[(False, False)]
    for k, v in r.items():
        d = [float((a - b).abs().max()) for a, b in zip(v, ref)]
        n = [int((a != b).sum()) for a, b in zip(v, ref)]
        print(phase, "fuse=%s share=%s" % k, "maxdiff", d, "ndiff", n, flush=True)
