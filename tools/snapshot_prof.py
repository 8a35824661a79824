"""Host profile of the prev-net snapshot prev.load_state_dict(net.state_dict()) on the GPU (diagnostic)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]

import torch  # noqa: E402

import base  # noqa: E402

base._native.load()
a = base.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
b = base.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
x = torch.rand(64, 2, device="cuda")
a(x), b(x)  # packs the nets and writes their weight planes
torch.cuda.synchronize()
assert b._snapshot_source(a.state_dict()) is a, "fast path not taken"
for name, fn in (("state_dict", lambda: a.state_dict()), ("snapshot", lambda: b.load_state_dict(a.state_dict()))):
    fn()
    t0 = time.perf_counter()
    for _ in range(2000):
        fn()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) / 2000 * 1e6:.1f} us", flush=True)
cProfile.run("for _ in range(2000): b.load_state_dict(a.state_dict())", "/tmp/snap.prof")
pstats.Stats("/tmp/snap.prof").sort_stats("tottime").print_stats(18)
