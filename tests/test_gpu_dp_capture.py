"""The data-parallel iteration with the RCCL all-reduce CAPTURED in the iteration's hipGraph
(base/_loop.py PhaseLoop._dp_split: backend 'nccl'), on one GPU: a world-1 RCCL process group with
cfg.insr_dp_always runs the DP code itself -- gradient arena, all-reduce, global-count loss means, unfused sums +
Adam + plateau -- so the captured collective (one graph per iteration, groups of insr_graph_unroll
iterations) can be checked against the two-graph split with the eager all-reduce
(cfg.insr_dp_capture = False) and against the single-process path (no process group): every
fluid phase, parameters bit for bit and the same losses read by the loop.  (A world-1 all-reduce
sums one rank: the three paths compute the same numbers; the multi-rank sums are covered by the
gloo tests, the rank-1 RCCL communicator by test_gpu_comm.py.)"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "ref_phases.npz")


def _worker(port, q, plain=False):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]
    import torch.distributed as dist
    from pde.config import make_config
    if plain:  # the reference bodies as written, lowered by the loop (base/lower.py)
        from pde.fluid_plain import Fluid2DPlainModel as Fluid2DModel
    else:
        from pde.fluid import Fluid2DModel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ph = dict(np.load(GOLD))
    out = {}
    # single / split / captured without in-kernel loss seeds (base/losses.py lazy_losses): the three compute the
    # loss values in the same launches; "seeded" = captured with them (the default), against "captured"
    runs = (("single", dict(insr_dp_always=False, insr_seed_in_bwd=False)),
            ("split", dict(insr_dp_always=True, insr_dp_capture=False, insr_seed_in_bwd=False)),
            ("captured", dict(insr_dp_always=True, insr_dp_capture=True, insr_seed_in_bwd=False)),
            ("seeded", dict(insr_dp_always=True, insr_dp_capture=True)))
    for name, kw in (runs[:3] if plain else runs):
        torch.manual_seed(0)
        cfg = make_config("fluid", num_hidden_layers=4, hidden_features=128, sample_resolution=32, dt=0.05,
                          proj_dir="/tmp/insr_dp_capture_test", insr_progress=False, early_stop=False,
                          max_n_iters=10, insr_graph=True, insr_sync_every=4, insr_graph_unroll=4, lr=1e-4, **kw)
        m = Fluid2DModel(cfg)
        m.timestep = 1
        for k, net in (("vel", m.velocity_field), ("vel_prev", m.velocity_field_prev), ("pres", m.pressure_field)):
            with torch.no_grad():
                net.flat_params().copy_(torch.from_numpy(ph[f"fluid/{k}/params0"]).cuda())
        trace = []
        for phase in ("_advect_velocity", "_solve_pressure", "_projection"):
            m.tb = type("TB", (), {"add_scalars": lambda self, tag, vals, global_step: trace.append(
                (tag, global_step, vals["main"], vals["bc"]))})()
            getattr(m, phase)()
            err = getattr(m, "_insr_capture_error", None)
            assert err is None, err
        torch.cuda.synchronize()
        out[name] = (m.velocity_field.flat_params().cpu().numpy().copy(),
                     m.pressure_field.flat_params().cpu().numpy().copy(), trace, m._dp_active())
    q.put(out)
    dist.destroy_process_group()


def test_captured_allreduce_equals_split_and_single_process():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(port, q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert not res["single"][3] and res["split"][3] and res["captured"][3] and res["seeded"][3]
    for name in ("split", "captured"):
        assert np.array_equal(res[name][0], res["single"][0]), name
        assert np.array_equal(res[name][1], res["single"][1]), name
        assert res[name][2] == res["single"][2], name
    # the seeded DP iteration: the same parameters (the seeds are the group launch's gradients bit for bit),
    # the loss values from another summation order
    assert np.array_equal(res["seeded"][0], res["captured"][0]) and np.array_equal(res["seeded"][1], res["captured"][1])
    assert len(res["seeded"][2]) == len(res["captured"][2])
    for (t1, s1, m1, b1), (t2, s2, m2, b2) in zip(res["seeded"][2], res["captured"][2]):
        assert (t1, s1) == (t2, s2) and abs(m1 - m2) <= 1e-6 * abs(m2) and abs(b1 - b2) <= 1e-6 * abs(b2)


def test_captured_allreduce_plain_bodies():
    """The same three DP paths for the reference's fluid bodies as written (pde/fluid_plain.py: lowered losses,
    deferred jets, multi-job reverse jets): DP code path == single process, parameters bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(port, q, True))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert not res["single"][3] and res["split"][3] and res["captured"][3]
    for name in ("split", "captured"):
        assert np.array_equal(res[name][0], res["single"][0]), name
        assert np.array_equal(res[name][1], res["single"][1]), name
        assert len(res[name][2]) == len(res["single"][2]), name
        for (t1, s1, m1, b1), (t2, s2, m2, b2) in zip(res[name][2], res["single"][2]):
            assert (t1, s1) == (t2, s2) and abs(m1 - m2) <= 1e-6 * abs(m2) and abs(b1 - b2) <= 1e-6 * abs(b2)
