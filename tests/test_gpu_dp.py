"""Data parallelism on the GPU: 2 ranks (gloo, both on cuda:0 -- a functional rehearsal
of the RCCL path, which needs one GPU per rank) each take HALF of the reference golden
sample set; after the one all-reduce in BaseModel._dp_sync the gradients must equal the
single-process full-batch gradients recorded from the reference (1e-5 normwise)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "ref_phases.npz")


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pde.config import make_config
    from pde.fluid import Fluid2DModel
    ph = dict(np.load(GOLD))
    cfg = make_config("fluid", num_hidden_layers=4, hidden_features=128, sample_resolution=32, dt=0.05,
                      proj_dir="/tmp/insr_dp_test", insr_progress=False)
    model = Fluid2DModel(cfg)
    for k, net in (("vel", model.velocity_field), ("vel_prev", model.velocity_field_prev),
                   ("pres", model.pressure_field)):
        with torch.no_grad():
            net.flat_params().copy_(torch.from_numpy(ph[f"fluid/{k}/params0"]).cuda())

    def half(a):
        a = torch.from_numpy(a).cuda()
        n = a.shape[0] // world
        return a[rank * n:(rank + 1) * n].clone()

    model._sample_in_training = lambda: half(ph["fluid/x0"]).requires_grad_(True)
    model._boundary_pair = lambda n: (half(ph["fluid/bcx0"]).requires_grad_(True),
                                      half(ph["fluid/bcy0"]).requires_grad_(True))
    out = {}
    for phase in ("_advect_velocity", "_solve_pressure", "_projection"):
        model._reset_optimizer()
        ld = getattr(Fluid2DModel, phase)._insr_phase(model)
        model.optimizer.zero_grad()
        sum(ld.values()).backward()
        synced = model._dp_sync(ld)
        out[phase] = ({k: float(v) for k, v in synced.items()},
                      model.velocity_field.flat_grad_buffer().cpu().numpy().copy(),
                      model.pressure_field.flat_grad_buffer().cpu().numpy().copy())
    q.put((rank, out))
    dist.destroy_process_group()


def test_two_rank_gradients_equal_full_batch():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ph = dict(np.load(GOLD))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    nerr = lambda a, b: np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)  # noqa: E731
    for phase, (losses, gv, gp) in res[0].items():
        for k, v in losses.items():
            ref = float(ph[f"fluid/{phase}/loss_{k}"])
            assert abs(v - ref) <= 1e-5 * abs(ref) + 1e-12, (phase, k)
        for g, key in ((gv, "grad_vel"), (gp, "grad_pres")):
            ref = ph[f"fluid/{phase}/{key}"]
            if np.abs(ref).max() > 0:
                assert nerr(g, ref) < 1e-5, (phase, key, nerr(g, ref))
        assert np.array_equal(gv, res[1][phase][1]) and np.array_equal(gp, res[1][phase][2])
