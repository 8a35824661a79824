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
    q.put((rank, m.a.flat_grad_buffer().clone(), m.b.flat_grad_buffer().clone(),
           {k: float(v) for k, v in out.items()}, m.a.grad_touched()))
    dist.destroy_process_group()


@pytest.mark.parametrize("reduction", ["mean", "sum"])
def test_dp_sync_two_ranks(reduction):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, reduction, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    scale = {"mean": 1.0 / world, "sum": 1.0}[reduction]
    for rank, ga, gb, losses, touched in res:
        n_a = ga.numel()
        expect_a = torch.arange(n_a, dtype=torch.float32) * (1 + 2) * scale
        expect_b = (torch.arange(gb.numel(), dtype=torch.float32) * 3 + 2) * scale
        assert torch.allclose(ga, expect_a) and torch.allclose(gb, expect_b)
        assert abs(losses["main"] - (1.0 + 2.0) * scale) < 1e-6
        assert abs(losses["bc"] - 30.0 * scale) < 1e-5
        assert touched
    assert torch.equal(res[0][1], res[1][1])  # replicas identical -> identical Adam steps
