"""Loss groups evaluated inside the reverse jets (round 5: base/losses.py lazy_losses, include/insr_siren.h
InsrSeed / insr_siren_jet_bwd_seeded / InsrLossFin).

A phase body's unit-seeded loss group (insr_sq_loss_group: the squared residuals of fluid/model.py:96-101,
121-125,147-151 and the wall terms, seeded with 1 by base/baseModel.py:77) holds its launch back; the value
backward (jet_bwd_x6) or the saved-stream Laplacian sweep (jet_fb_x6) evaluates the terms where it reads
its adjoints, and the sums launch that follows finishes the loss values.  Checked here against the same
computation with the group launched:

  * the three fluid phases through the real loop (eager and graph-replayed; 32^2 points: value jets seeded,
    the small Laplacian jet's group launched first; 64^2: the jet_fb Laplacian sweep seeded too) --
    parameters, Adam moments and the flat .grad bit for bit (the seeds are the group kernel's gradient,
    bit for bit), the learning rate and step equal, the loss values (another summation order) and the
    plateau's best within 1e-6 relative;
  * one reverse jet per path directly through the python API: value 2 -> 2 at 16,384 + 2 x 162 points
    (the headline's value backward) and Laplacian 2 -> 1 at 16,708 points (its jet_fb sweep);
  * the fallbacks: a non-unit seed launches the group (bit for bit the eager result), and a group whose
    gradient reaches anything but a reverse jet is an error (settle_lazy raises)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "ref_phases.npz")
PHASES = ("_advect_velocity", "_solve_pressure", "_projection")


@pytest.fixture(scope="module")
def B():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    base._native.load()
    return base


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _loops(B, res, seeds, graph, iters=6):
    from pde.config import make_config
    from pde.fluid import Fluid2DModel
    ph = dict(np.load(GOLD))
    torch.manual_seed(0)
    cfg = make_config("fluid", num_hidden_layers=4, hidden_features=128, sample_resolution=res, dt=0.05,
                      proj_dir="/tmp/insr_seeds_test", insr_progress=False, early_stop=False, max_n_iters=iters,
                      insr_graph=graph, insr_sync_every=3, lr=1e-4, insr_seed_in_bwd=seeds)
    m = Fluid2DModel(cfg)
    m.timestep = 1
    for k, net in (("vel", m.velocity_field), ("vel_prev", m.velocity_field_prev), ("pres", m.pressure_field)):
        with torch.no_grad():
            net.flat_params().copy_(torch.from_numpy(ph[f"fluid/{k}/params0"]).cuda())
    stats0 = dict(B._jet.SEED_STATS)
    trace, out = [], {}
    for phase in PHASES:
        m.tb = type("TB", (), {"add_scalars": lambda self, tag, vals, global_step: trace.append(
            (tag, global_step, vals["main"], vals["bc"]))})()
        getattr(m, phase)()
        assert getattr(m, "_insr_capture_error", None) is None, m._insr_capture_error
        torch.cuda.synchronize()
        opt = m.optimizer
        out[phase] = [opt._nets[k][q].detach().cpu().numpy().copy() for k in (0, 1) for q in (1, 2)]
        out[phase + "/state"] = opt.state.detach().cpu().numpy().copy()
    for name, net in (("vel", m.velocity_field), ("pres", m.pressure_field)):
        out[name] = net.flat_params().detach().cpu().numpy().copy()
        out[name + "/grad"] = net.flat_grad_buffer().detach().cpu().numpy().copy()
    stats = {k: v - stats0.get(k, 0) for k, v in B._jet.SEED_STATS.items()}
    return out, trace, stats


@pytest.mark.parametrize("res,graph", [(32, False), (32, True), (64, True)])
def test_seeded_loops_equal_launched_groups(B, res, graph):
    from base import _native as nat
    on, tr_on, st_on = _loops(B, res, True, graph)
    off, tr_off, st_off = _loops(B, res, False, graph)
    assert st_on["seeded"] > 0 and st_off["seeded"] == 0
    assert st_on.get(nat.MODE_VALUE, 0) > 0
    if res >= 64:  # the pressure phase's Laplacian jet (jet_fb sweep from 4,096 points) took its group too
        assert st_on.get(nat.MODE_LAP, 0) > 0
    for k in off:
        if k.endswith("/state"):
            a, b = on[k], off[k]
            assert a[nat.OPT_LR] == b[nat.OPT_LR] and a[nat.OPT_STEP] == b[nat.OPT_STEP], k
            assert rel(a[nat.OPT_BEST], b[nat.OPT_BEST]) < 1e-6, k
        else:
            for x, y in zip(on[k] if isinstance(on[k], list) else [on[k]], off[k] if isinstance(off[k], list) else [off[k]]):
                assert np.array_equal(x, y), k
    assert len(tr_on) == len(tr_off) > 0
    for (t1, s1, m1, b1), (t2, s2, m2, b2) in zip(tr_on, tr_off):
        assert (t1, s1) == (t2, s2)
        assert abs(m1 - m2) <= 1e-6 * abs(m2) and abs(b1 - b2) <= 1e-6 * abs(b2) + 1e-30


def _one_jet(B, mode, lazy, n, nb, seed=5):
    """One reverse jet of a merged [interior; bands] batch through the python API: the loss group of
    the fluid phase bodies on its outputs, unit-seeded backward, deferred sums landed; returns the flat
    .grad and the loss values."""
    from base import _jet
    from base.losses import lazy_losses, register_unit_seed, settle_lazy
    torch.manual_seed(seed)
    dout = 2 if mode == "value" else 1
    net = B.MLP(2, dout, 4, 128, nonlinearity="sine").cuda()
    g = torch.Generator(device="cuda").manual_seed(seed)
    xa = (torch.rand(n + 2 * nb, 2, device="cuda", generator=g) * 2 - 1).requires_grad_(True)
    t1 = torch.rand(n, 2, device="cuda", generator=g)
    t2 = torch.rand(n, device="cuda", generator=g)
    unit = register_unit_seed(torch.ones((), device="cuda"))
    with lazy_losses(lazy):
        if mode == "value":
            y = net(xa)
            main, bc = B.sq_losses(B.mse_term(y, t1, count=2 * n), B.wall_term(y, nb, row0=n))
        else:
            lap, gp = B.laplace(net(xa), xa, return_grad=True)
            main, bc = B.sq_losses(B.mse_term(lap, t1[:, 0], t2, alpha=1.0, beta=-1.0, gamma=-1.0, count=n),
                                   B.wall_term(gp, nb, row0=n))
    s0 = _jet.SEED_STATS["seeded"]
    with _jet.defer_reductions():
        with _jet.batched_backward():
            torch.autograd.backward([main, bc], grad_tensors=[unit, unit])
        settle_lazy()
        grad = net.flat_grad_buffer().detach().cpu().numpy().copy()  # lands the held-back sums (+ losses)
    torch.cuda.synchronize()
    return grad, float(main), float(bc), _jet.SEED_STATS["seeded"] - s0


@pytest.mark.parametrize("mode,n,nb", [("value", 16384, 162), ("lap", 16384, 162), ("value", 8192, 81)])
def test_seeded_jet_equals_launched_group(B, mode, n, nb):
    g_on, m_on, b_on, k_on = _one_jet(B, mode, True, n, nb)
    g_off, m_off, b_off, k_off = _one_jet(B, mode, False, n, nb)
    assert k_on == 1 and k_off == 0
    assert np.array_equal(g_on, g_off)
    assert abs(m_on - m_off) <= 1e-6 * abs(m_off) and abs(b_on - b_off) <= 1e-6 * abs(b_off)


def test_non_unit_seed_launches_the_group(B):
    from base import _jet
    from base.losses import lazy_losses, settle_lazy
    res = {}
    for lazy in (False, True):
        torch.manual_seed(3)
        net = B.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
        x = (torch.rand(600, 2, device="cuda") * 2 - 1).requires_grad_(True)
        t = torch.rand(600, 2, device="cuda")
        with lazy_losses(lazy):
            (loss,) = B.sq_losses(B.mse_term(net(x), t))
        with _jet.batched_backward():
            (3.0 * loss).backward()
        settle_lazy()
        res[lazy] = (net.flat_grad_buffer().detach().cpu().numpy().copy(), float(loss))
    assert np.array_equal(res[True][0], res[False][0]) and res[True][1] == res[False][1]


def test_group_gradient_read_elsewhere_raises(B):
    from base import _jet
    from base.losses import lazy_losses, register_unit_seed, settle_lazy
    torch.manual_seed(4)
    net = B.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    x = (torch.rand(256, 2, device="cuda") * 2 - 1).requires_grad_(True)
    t = torch.rand(256, 2, device="cuda")
    unit = register_unit_seed(torch.ones((), device="cuda"))
    with lazy_losses():
        y = net(x)
        (loss,) = B.sq_losses(B.mse_term(y, t))
    extra = (2.0 * y).sum()  # y's gradient is the sum of two: the group's buffer is read as data
    with _jet.batched_backward():
        torch.autograd.backward([loss, extra], grad_tensors=[unit, torch.ones((), device="cuda")])
    with pytest.raises(RuntimeError):
        settle_lazy()
