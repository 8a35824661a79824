"""Strong-scaling sampling of the elasticity model under data parallelism (gloo, world 2, CPU):
each rank draws ONLY its share of every part of the global batch (elasticity/model.py:198-250 restated
in pde/elasticity.py, sharded) -- the mesh sampler is asked for N / world points, never the
world-sized batch; grid / mesh-vertex rows are the rank's contiguous slice, so the union over ranks
is the global batch; ranks draw independent random rows.  The single-process emulation
(cfg.insr_shard = (r, K), bench.py --shard-of K) takes the same rows."""
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


def _model(config, **over):
    import base.baseModel as bm
    bm._local_device = lambda: torch.device("cpu")  # CPU stand-in: no network is evaluated here
    from pde.config import baseline_config
    from pde.elasticity import ElasticityModel
    cfg = baseline_config(config, proj_dir="/tmp/insr_dp_shard", **over)
    torch.manual_seed(0)
    return ElasticityModel(cfg)


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(1234)  # identical seeds on every rank: the rank must be folded in by the model
    m = _model("elasticity3Dbunny")
    calls = []
    orig = m.mesh_sampler.sample

    def spy(n, generator=None):
        calls.append(n)
        return orig(n, generator=generator)
    m.mesh_sampler.sample = spy
    x = m._sample_in_training(64)
    # box scene with a grid part and fixed faces (elasticity2Dstretch: random + uniform)
    e = _model("elasticity2Dstretch")
    xb = e._sample_in_training(100)
    fl, fr = e._sample_fixed_in_training(100)
    q.put((rank, calls, x.detach().numpy().copy(), xb.detach().numpy().copy(), fl.detach().numpy().copy(),
           fr.detach().numpy().copy()))
    dist.destroy_process_group()


def test_strong_dp_draws_the_rank_share_only():
    import numpy as np
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n3 = 64 ** 3
    for rank, calls, x, xb, fl, fr in res:
        assert calls == [n3 // world], calls  # no world-sized draw on the mesh
        assert x.shape == (n3 // world, 3)
        assert xb.shape == (2 * 100 ** 2 // world, 2)  # random + uniform parts, each halved
        assert fl.shape == fr.shape == (2 * 100 // world, 2)
        assert np.all(fl[:, 0] == -1.0) and np.all(fr[:, 0] == 1.0)
    # the ranks' random rows are independent draws; their grid rows tile the global grid
    assert not np.array_equal(res[0][2], res[1][2])
    h = 100 ** 2 // world
    grid = np.concatenate([r[3][h:] for r in res])
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]
    from base.sampling import sample_uniform
    assert np.array_equal(grid, sample_uniform(100, 2).numpy())


def test_single_process_shard_emulation_takes_the_same_rows():
    """cfg.insr_shard = (r, K) (bench.py --shard-of K) runs the strong-scaling code path: rank r's
    share of each part, in one process."""
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]
    from base.sampling import sample_uniform
    for r in range(4):
        e = _model("elasticity2Dstretch", insr_shard=(r, 4))
        xb = e._sample_in_training(100)
        assert xb.shape == (2 * 2500, 2)
        assert torch.equal(xb[2500:].detach(), sample_uniform(100, 2)[r * 2500:(r + 1) * 2500])
        fl, fr = e._sample_fixed_in_training(100)
        assert fl.shape == (50, 2) and fr.shape == (50, 2)
    m = _model("elasticity3Dbunny", insr_shard=(0, 8))
    calls = []
    orig = m.mesh_sampler.sample
    m.mesh_sampler.sample = lambda n, generator=None: calls.append(n) or orig(n, generator=generator)
    assert m._sample_in_training(64).shape == (64 ** 3 // 8, 3) and calls == [64 ** 3 // 8]
