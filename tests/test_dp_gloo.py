"""Data-parallel host logic on the CPU with gloo, world_size 2: BaseModel._dp_sync
all-reduces the concatenated flat gradients of every trainable network plus the loss
scalars in ONE collective, averaging for mean-type losses and summing for the
elasticity energies.  (The HIP jets themselves need a GPU; here the per-rank
gradients are planted directly in the networks' flat .grad buffers.)"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, reduction, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import base

    class Toy(base.BaseModel):
        _dp_loss_reduction = reduction

        def __init__(self):
            self.device = torch.device("cpu")
            torch.manual_seed(0)
            self.a = base.MLP(2, 2, 1, 32, nonlinearity="sine")
            self.b = base.MLP(2, 1, 1, 32, nonlinearity="sine")

        @property
        def _trainable_networks(self):
            return {"a": self.a, "b": self.b}

        def _sample_in_training(self):
            pass

        def initialize(self):
            pass

        def step(self):
            pass

    m = Toy()
    for k, net in enumerate((m.a, m.b)):
        g = net.flat_grad_buffer()
        g.copy_(torch.arange(g.numel(), dtype=torch.float32) * (rank + 1) + k)
    losses = {"main": torch.tensor(1.0 + rank), "bc": torch.tensor(10.0 * (rank + 1))}
    out = m._dp_sync(losses)
    res = (rank, m.a.flat_grad_buffer().clone(), m.b.flat_grad_buffer().clone(),
           {k: float(v) for k, v in out.items()}, m.a.grad_touched())
    # second iteration: b receives no gradient (zero_grad, no backward reaches it) -> it stays out of
    # the reduced span (arena [a | losses | b]: only [a | losses] is all-reduced) and untouched (Adam
    # skips it, as torch skips .grad None)
    m.b.mark_grad_stale(set_to_none=True)
    ga = m.a.flat_grad_buffer()
    ga.fill_(float(rank + 1))
    m._dp_sync({"main": torch.tensor(0.0)})
    red = m._insr_dp_red
    b_in_span = red.data_ptr() <= m.b._flat_grad.data_ptr() < red.data_ptr() + 4 * red.numel()
    res2 = (m.a.flat_grad_buffer().clone(), m.b.grad_touched(), float(b_in_span))
    # plain numpy by value: a queued tensor travels as a shared-memory fd that the parent may
    # try to fetch after this process has exited (ConnectionResetError)
    q.put(tuple(v.numpy().copy() if isinstance(v, torch.Tensor) else v for v in res + res2))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("reduction", ["mean", "sum"])
def test_dp_sync_two_ranks(reduction, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, reduction, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [tuple(torch.from_numpy(v) if hasattr(v, "dtype") and not isinstance(v, float) else v for v in q.get(timeout=120))
           for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    scale = {"mean": 1.0 / world, "sum": 1.0}[reduction]
    rsum = sum(r + 1 for r in range(world))  # sum over ranks of (rank + 1)
    for rank, ga, gb, losses, touched, ga2, b_touched2, b_arena_max in res:
        assert torch.allclose(ga2, torch.full_like(ga2, rsum * scale))
        assert not b_touched2 and b_arena_max == 0.0  # (here: b's slice is outside the reduced span)
        n_a = ga.numel()
        expect_a = torch.arange(n_a, dtype=torch.float32) * rsum * scale
        expect_b = (torch.arange(gb.numel(), dtype=torch.float32) * rsum + world) * scale
        assert torch.allclose(ga, expect_a) and torch.allclose(gb, expect_b)
        assert abs(losses["main"] - sum(1.0 + r for r in range(world)) * scale) < 1e-5
        assert abs(losses["bc"] - 10.0 * rsum * scale) < 1e-4
        assert touched
    assert torch.equal(res[0][1], res[1][1])  # replicas identical -> identical Adam steps


def _worker_dp_always(port, q):
    import sys
    import types
    sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    import base

    class Toy(base.BaseModel):
        def __init__(self, always):
            self.device = torch.device("cpu")
            self.cfg = types.SimpleNamespace(insr_dp_always=always)
            torch.manual_seed(0)
            self.a = base.MLP(2, 2, 1, 32, nonlinearity="sine")

        @property
        def _trainable_networks(self):
            return {"a": self.a}

        def _sample_in_training(self):
            pass

        def initialize(self):
            pass

        def step(self):
            pass

    out = []
    for always in (False, True):
        m = Toy(always)
        g = m.a.flat_grad_buffer()
        g.copy_(torch.arange(g.numel(), dtype=torch.float32))
        res = m._dp_sync({"main": torch.tensor(2.0)})
        out.append((m._dp_active(), "_insr_dp_arena" in m.__dict__, float(res["main"]),
                    bool(torch.equal(m.a.flat_grad_buffer(), torch.arange(g.numel(), dtype=torch.float32)))))
    q.put(out)
    dist.destroy_process_group()


def test_dp_path_at_world_one():
    """cfg.insr_dp_always (bench.py --dp-path): with a world-1 process group the iteration takes the
    data-parallel path itself -- gradient arena bound, the collective run (a no-op sum) -- so one GPU
    can time a rank's DP step; without it a world-1 group changes nothing."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_dp_always, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0
    (act0, arena0, loss0, g0), (act1, arena1, loss1, g1) = res
    assert not act0 and not arena0 and loss0 == 2.0 and g0
    assert act1 and arena1 and loss1 == 2.0 and g1
