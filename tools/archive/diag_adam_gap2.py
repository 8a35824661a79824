"""Diagnostic: where does the ~8.7 us idle gap after every adam_multi_kernel come from?
(r4r kernel traces: 0.00 us between every other pair of kernels of a replayed step, 8.6-9.0 us
after each Adam launch, with or without its weight-plane writes.)  One hipGraph of N launches of
ONE variant, replayed R times; run under rocprofv3 --kernel-trace and read the gaps after each
kernel (tools/trace_gaps.py).

  --variant plateau    FusedAdam.step(plateau=...) (Adam + plateau ticket, planes)   [the loop's]
  --variant noplateau  the Adam launch without the plateau step (no ticket)
  --variant noplanes   Adam + plateau, shapes = NULL (no plane writes)
  --variant add        a torch add_ over the same 66,690 floats (control)
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="plateau", choices=["plateau", "noplateau", "noplanes", "add"])
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--replays", type=int, default=5)
    a = ap.parse_args()
    import torch
    import base
    nat = base._native
    lib = nat.load()
    torch.manual_seed(0)
    net = base.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    net.refresh_wsplit()
    g = net.flat_grad_buffer()
    g.copy_(torch.randn_like(g) * 1e-3)
    opt = base.FusedAdam([{"params": net, "module": net, "lr": 1e-4}])
    sched = base.DevicePlateau(opt, patience=10)
    loss = torch.ones(1, device="cuda")
    st = nat.stream_of(torch.device("cuda"))

    def noplanes():
        arr = lambda t: (ctypes.c_void_p * 1)(t.data_ptr())  # noqa: E731
        mlp, m, v = opt._nets[0]
        sizes = (ctypes.c_long * 1)(mlp.flat_params().numel())
        nat.check(lib.insr_adam_plateau_step_nets(1, arr(mlp.flat_params()), arr(g), arr(m), arr(v), sizes, None,
                                                  nat.ptr(opt.state), 0.9, 0.999, 1e-8, nat.ptr(loss), 10, st),
                  "adam")

    body = {
        "plateau": lambda: opt.step(plateau=(sched, loss)),
        "noplateau": lambda: nat.check(lib.insr_adam_step_nets(
            1, (ctypes.c_void_p * 1)(net.flat_params().data_ptr()), (ctypes.c_void_p * 1)(g.data_ptr()),
            (ctypes.c_void_p * 1)(opt._nets[0][1].data_ptr()), (ctypes.c_void_p * 1)(opt._nets[0][2].data_ptr()),
            (ctypes.c_long * 1)(net.flat_params().numel()), (ctypes.c_int * 4)(2, 2, 4, 128), nat.ptr(opt.state),
            0.9, 0.999, 1e-8, 1, st), "adam"),
        "noplanes": noplanes,
        "add": lambda: g.add_(1e-9),
    }[a.variant]
    for _ in range(3):
        body()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(gr, stream=side):
            for _ in range(a.n):
                body()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    for _ in range(a.replays):
        gr.replay()
    torch.cuda.synchronize()
    print("ok", a.variant, flush=True)


if __name__ == "__main__":
    main()
