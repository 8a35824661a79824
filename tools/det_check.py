import sys, os
sys.path[:0] = ['.', 'insr-pde_amd', 'tests']  # run from the repo root
import torch
import base
from base import sampling
base._native.load()
from test_gpu_fullsize import _fluidM

def run(graph, phases=("_advect_velocity", "_solve_pressure", "_projection"), cfgname="fluid2DtlgnM"):
    sampling._SAMPLER.clear()
    m = _fluidM(graph)
    out = []
    for ph in phases:
        getattr(m, ph)()
        torch.cuda.synchronize()
        out.append((ph, m.velocity_field.flat_params().detach().cpu().clone(), m.pressure_field.flat_params().detach().cpu().clone()))
    return out

a = run(False); b = run(False); c = run(True); d = run(True)
for name, r in (("eager-eager", b), ("eager-graph", c), ("graph-graph", d)):
    ref = a if name != "graph-graph" else c
    for (ph, v1, p1), (_, v2, p2) in zip(ref, r):
        print(name, ph, float((v1 - v2).abs().max()), float((p1 - p2).abs().max()))
