"""What a sums + Adam launch (insr_adam_step_partials, capi.hip reduce_adam_kernel) spends its time on:
the partial rows it reads, the plateau ticket, the weight-plane rewrite.  Times graph-replayed launches
(host-free) with HIP events for variants of one shape: the headline value backward's (209 rows of the
2 -> 2 4 x 128 net) and the 8-way shard's (131 rows), with / without the plateau step (loss) and the
weight planes (shape).  Prints one JSON line per variant: us per launch.
Usage: python tools/study/adam_sums_cost.py
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "insr-pde_amd"))
import base  # noqa: E402
from base import _native as nat  # noqa: E402


def main():
    lib = nat.load()
    dev = torch.device("cuda", 0)
    din, dout, L, W = 2, 2, 4, 128
    count = lib.insr_siren_param_count(din, dout, L, W)
    stride = lib.insr_jet_partial_stride(din, dout, L, W)
    net = base.MLP(din, dout, L, W, nonlinearity="sine").cuda()
    net.ensure_packed()
    net.ensure_wsplit()
    prm = net.flat_params()
    m = torch.zeros(count, device=dev)
    v = torch.zeros(count, device=dev)
    grad = torch.zeros(count, device=dev)
    st = torch.zeros(17, device=dev)
    st[0] = 1e-7  # lr (tiny: the parameters stay in the planes' range over many replays)
    st[2] = 1e30  # best
    st[6] = 0.5
    loss = torch.ones(1, device=dev)
    shape = (ctypes.c_int * 4)(din, dout, L, W)
    out = []
    for nb in (209, 131, 64, 16):
        part = torch.randn(nb * stride, device=dev) * 1e-3
        for with_loss in (True, False):
            for with_shape in (True, False):
                s = torch.cuda.Stream(device=dev)

                def launch():
                    rc = lib.insr_adam_step_partials(nat.ptr(part), nb, stride, nat.ptr(grad), 0, nat.ptr(prm),
                                                     nat.ptr(m), nat.ptr(v), count, shape if with_shape else None,
                                                     nat.ptr(st), 0.9, 0.999, 1e-8,
                                                     nat.ptr(loss) if with_loss else None, 10 ** 6,
                                                     ctypes.c_void_p(s.cuda_stream))
                    assert rc == 0, rc

                with torch.cuda.stream(s):
                    for _ in range(3):
                        launch()
                    torch.cuda.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=s):
                        for _ in range(20):
                            launch()
                    for _ in range(3):
                        g.replay()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(25):
                        g.replay()
                    e1.record(s)
                    torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / (25 * 20)
                rec = {"rows": nb, "plateau": with_loss, "planes": with_shape, "us_per_launch": round(us, 2),
                       "row_MB": round(nb * stride * 4 / 1e6, 1)}
                print(json.dumps(rec), flush=True)
                out.append(rec)


if __name__ == "__main__":
    main()
