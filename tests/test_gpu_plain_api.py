"""The drop-in case: fluid phase bodies written only against the reference's base API
(pde/fluid_plain.py -- plain torch residuals, separate band samplers, one MLP call per point
set, as fluid/model.py:72-151) run on the HIP path and reproduce the REFERENCE golden vectors
(tests/golden/ref_phases.npz, the same fixtures as test_gpu_phases.py) -- losses and
gradients 1e-5 -- and the graph-replayed loop runs them (captures and replays)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ph():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import os
    return dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_phases.npz")))


def nerr(a, b):
    a = torch.as_tensor(np.asarray(a, np.float64))
    b = torch.as_tensor(np.asarray(b, np.float64))
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _model(**kw):
    from pde.config import make_config
    from pde.fluid_plain import Fluid2DPlainModel
    kw.setdefault("num_hidden_layers", 4)
    kw.setdefault("hidden_features", 128)
    cfg = make_config("fluid", proj_dir="/tmp/insr_test", insr_progress=False, early_stop=False, max_n_iters=2,
                      lr=1e-4, dt=0.05, **kw)
    return Fluid2DPlainModel(cfg)


def test_plain_phases_match_reference(ph, monkeypatch):
    import pde.fluid_plain as fp
    model = _model(sample_resolution=32)
    T = lambda k: torch.from_numpy(ph[k]).cuda()  # noqa: E731
    nets = {"vel": model.velocity_field, "vel_prev": model.velocity_field_prev, "pres": model.pressure_field}
    # the reference's phases draw x-face then y-face bands: serve the recorded ones in that order
    served = []
    monkeypatch.setattr(fp, "sample_boundary2D_separate",
                        lambda n, side, device=None: T("fluid/bcx0" if side == "horizontal" else "fluid/bcy0").clone())
    model._sample_in_training = lambda: T("fluid/x0").clone().requires_grad_(True)
    for phase in ("_advect_velocity", "_solve_pressure", "_projection"):
        body = getattr(type(model), phase)._insr_phase
        for k, n in nets.items():
            with torch.no_grad():
                n.flat_params().copy_(T(f"fluid/{k}/params0"))
        model._reset_optimizer()
        ld = body(model)
        for k, v in ld.items():
            ref = float(ph[f"fluid/{phase}/loss_{k}"])
            assert abs(float(v) - ref) <= 1e-5 * abs(ref) + 1e-12, (phase, k, float(v), ref)
        model.optimizer.zero_grad()
        sum(ld.values()).backward()
        for key, net in (("vel", model.velocity_field), ("pres", model.pressure_field)):
            g_ref = ph[f"fluid/{phase}/grad_{key}"]
            if np.abs(g_ref).max() > 0:
                g = net.flat_grad_buffer().detach().cpu().numpy()
                assert nerr(g, g_ref) < 1e-5, (phase, key)
        served.append(phase)
    assert len(served) == 3


def test_plain_step_graph_replay():
    """Full 128^2 phases through PhaseLoop, eager and hipGraph-replayed: the plain model's
    iteration (torch.rand band draws included) captures, and both runs give finite losses of
    the same size (the replayed torch RNG draws other points than the eager run)."""
    from base._loop import PhaseLoop
    results = []
    for graph in (False, True):
        torch.manual_seed(5)
        model = _model(sample_resolution=128, insr_graph=graph, insr_sync_every=10 ** 9)
        model.timestep = 1
        torch.cuda.manual_seed(11)
        losses = []
        for name in ("_advect_velocity", "_solve_pressure", "_projection"):
            pl = PhaseLoop(model, getattr(type(model), name)._insr_phase, name, (), {})
            pl.start()
            for i in range(4):
                out = pl.step(i)
            losses.append([float(v) for v in out.values()])
            assert graph is False or pl.graph is not None, getattr(pl, "capture_error", None)
        results.append(np.array(losses))
    assert np.all(np.isfinite(results[0])) and np.all(np.isfinite(results[1]))
    assert np.allclose(results[0], results[1], rtol=0.5, atol=1e-6), results


@pytest.mark.parametrize("defer", [False, True])
def test_plain_phases_lowered_match_reference(ph, monkeypatch, defer):
    """The same reference bodies as the loop runs them: inside base.lower.lowering() the network and
    diff-op outputs are Lazy, every loss is lowered to ONE fused loss-group launch per phase (no eager
    residual expression left), and losses and gradients still match the reference's golden vectors.
    defer: the body's jets queued and launched together at the first read (base.lower.deferred_jets)."""
    import pde.fluid_plain as fp
    from base import lower as LW
    model = _model(sample_resolution=32)
    T = lambda k: torch.from_numpy(ph[k]).cuda()  # noqa: E731
    nets = {"vel": model.velocity_field, "vel_prev": model.velocity_field_prev, "pres": model.pressure_field}
    monkeypatch.setattr(fp, "sample_boundary2D_separate",
                        lambda n, side, device=None: T("fluid/bcx0" if side == "horizontal" else "fluid/bcy0").clone())
    model._sample_in_training = lambda: T("fluid/x0").clone().requires_grad_(True)
    for phase in ("_advect_velocity", "_solve_pressure", "_projection"):
        body = getattr(type(model), phase)._insr_phase
        for k, n in nets.items():
            with torch.no_grad():
                n.flat_params().copy_(T(f"fluid/{k}/params0"))
        model._reset_optimizer()
        c0 = dict(LW.LOWERED)
        with LW.lowering(model._lower_on()), LW.deferred_jets(defer):
            ld = body(model)
        assert all(isinstance(v, LW.Lazy) for v in ld.values()), phase
        ld = LW.lower_losses(ld)
        assert LW.LOWERED["groups"] == c0["groups"] + 1 and LW.LOWERED["terms"] == c0["terms"] + 2, phase
        assert LW.LOWERED["eager_losses"] == c0["eager_losses"], phase
        for k, v in ld.items():
            ref = float(ph[f"fluid/{phase}/loss_{k}"])
            assert abs(float(v) - ref) <= 1e-5 * abs(ref) + 1e-12, (phase, k, float(v), ref)
        model.optimizer.zero_grad()
        model._backward(ld)
        for key, net in (("vel", model.velocity_field), ("pres", model.pressure_field)):
            g_ref = ph[f"fluid/{phase}/grad_{key}"]
            if np.abs(g_ref).max() > 0:
                g = net.flat_grad_buffer().detach().cpu().numpy()
                assert nerr(g, g_ref) < 1e-5, (phase, key)


def test_lowered_foot_is_one_launch_and_equal():
    """clamp(x - dt u, -1, 1) recorded under lowering and consumed by a no-grad network call is one
    insr_axpy_clamp launch; the value equals the eager expression (fmaf rounding: <= 1 ulp)."""
    from base import lower as LW
    g = torch.Generator(device="cuda").manual_seed(3)
    x = (torch.rand(4096, 2, device="cuda", generator=g) * 2 - 1).requires_grad_(True)
    u = torch.randn(4096, 2, device="cuda", generator=g)
    with LW.lowering():
        ul = LW.leaf(u)
        foot = torch.clamp(x - ul.detach() * 0.05, min=-1.0, max=1.0)
    assert isinstance(foot, LW.Lazy)
    with torch.no_grad():
        fast = LW.materialize(foot)
    eager = torch.clamp(x - u * 0.05, min=-1.0, max=1.0)
    assert fast.grad_fn is None
    assert torch.allclose(fast, eager.detach(), rtol=0, atol=2e-7)
    slow = LW.materialize(foot)  # with gradients: the recorded ops, autograd history kept
    assert slow.grad_fn is not None and torch.equal(slow, eager)


def test_plain_advection_lowered_matches_reference(ph, monkeypatch):
    """advection/model.py:68-91 as written (pde/advection_plain.py), run as the loop runs it: both losses
    lowered to one fused group (mean(((u - u0)/dt + v (ux + u0x)/2)^2) -> a 4-operand COMBO term), two
    reference iterations (phase + Adam + plateau) against the golden loss trace and update."""
    import pde.advection_plain as ap
    from base import lower as LW
    from pde.config import make_config
    cfg = make_config("advection", proj_dir="/tmp/insr_test", insr_progress=False, early_stop=False, max_n_iters=2,
                      lr=1e-4, num_hidden_layers=3, hidden_features=64, sample_resolution=512, dt=0.05, vel=0.25,
                      length=4.0)
    model = ap.Advection1DPlainModel(cfg)
    T = lambda k: torch.from_numpy(ph[k]).cuda()  # noqa: E731
    with torch.no_grad():
        model.field.flat_params().copy_(T("advect/field/params0"))
        model.field_prev.flat_params().copy_(T("advect/field_prev/params0"))
    body = ap.Advection1DPlainModel._advect._insr_phase
    model._reset_optimizer()
    trace = []
    for it in range(2):
        model._sample_in_training = lambda it=it: T(f"advect/x{it}").clone().requires_grad_(True)
        monkeypatch.setattr(ap, "sample_boundary", lambda n, sdim, device=None, it=it, **k: T(f"advect/bc{it}") / 2.0)
        c0 = dict(LW.LOWERED)
        with LW.lowering(model._lower_on()):
            ld = body(model)
        ld = LW.lower_losses(ld)
        assert LW.LOWERED["terms"] == c0["terms"] + 2 and LW.LOWERED["eager_losses"] == c0["eager_losses"]
        if it == 0:
            for k, v in ld.items():
                ref = float(ph[f"advect/_advect/loss_{k}"])
                assert abs(float(v) - ref) <= 1e-5 * abs(ref) + 1e-12, (k, float(v), ref)
        model._update_network(ld)
        trace.append([float(ld[k]) for k in sorted(ld)])
    assert nerr(np.array(trace), ph["advect/_advect/loss_trace"]) < 1e-5


def test_deferred_jets_share_launches(ph, monkeypatch):
    """Under deferred_jets the reference advection body's five network calls take two launches: the frozen
    field's target chain f(clamp(x - dt f(x))) as ONE advection-target job beside the trainable field's
    interior and band jets (plus nothing else); values equal the immediate calls'."""
    import pde.fluid_plain as fp
    from base import _jet
    from base import lower as LW
    model = _model(sample_resolution=32)
    T = lambda k: torch.from_numpy(ph[k]).cuda()  # noqa: E731
    for k, n in {"vel": model.velocity_field, "vel_prev": model.velocity_field_prev, "pres": model.pressure_field}.items():
        with torch.no_grad():
            n.flat_params().copy_(T(f"fluid/{k}/params0"))
    monkeypatch.setattr(fp, "sample_boundary2D_separate",
                        lambda n, side, device=None: T("fluid/bcx0" if side == "horizontal" else "fluid/bcy0").clone())
    model._sample_in_training = lambda: T("fluid/x0").clone().requires_grad_(True)
    body = type(model)._advect_velocity._insr_phase
    launched = []
    real_launch = _jet._launch_fused
    monkeypatch.setattr(_jet, "_launch_fused", lambda jobs: (launched.append(len(jobs)), real_launch(jobs))[1])
    out = {}
    for defer in (False, True):
        launched.clear()
        model._reset_optimizer()
        with LW.lowering(), LW.deferred_jets(defer):
            ld = body(model)
        ld = LW.lower_losses(ld)
        out[defer] = {k: float(v) for k, v in ld.items()}
        if defer:
            assert launched == [4], launched  # [advect target, u(x), u(bx), u(by)] in one launch
        else:
            assert launched == [], launched
    for k in out[False]:
        assert abs(out[True][k] - out[False][k]) <= 1e-6 * abs(out[False][k]) + 1e-12, (k, out)


@pytest.mark.parametrize("kind", ["mean", "sum", "mse_sum", "weighted_mean", "walls"])
def test_lowered_loss_equals_eager(kind):
    """Each loss form the lowering recognises, on real jet outputs: the fused group's value and the network's
    parameter gradients equal the same expression run eagerly (the materialised Lazy loss) -- values 1e-6,
    gradients 1e-5 normwise (another fp32 summation order)."""
    import torch.nn.functional as F
    import base
    from base import lower as LW
    torch.manual_seed(7)
    net = base.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    g = torch.Generator(device="cuda").manual_seed(8)
    x = (torch.rand(3000, 2, device="cuda", generator=g) * 2 - 1).requires_grad_(True)
    bx = (torch.rand(81, 2, device="cuda", generator=g) * 2 - 1).requires_grad_(True)
    tgt = torch.randn(3000, 2, device="cuda", generator=g)
    forms = {
        "mean": lambda u, ub: torch.mean((u - tgt) ** 2),
        "sum": lambda u, ub: 1e2 * torch.sum((u - tgt) ** 2),
        "mse_sum": lambda u, ub: F.mse_loss(u, tgt, reduction="sum"),
        "weighted_mean": lambda u, ub: 0.25 * torch.mean((2.0 * u - tgt) ** 2),
        "walls": lambda u, ub: (torch.mean(ub[..., 0] ** 2) + torch.mean(u[:81][..., 1] ** 2)) * 1.0,
    }
    out = {}
    for lowered in (False, True):
        net.zero_grad(set_to_none=True)
        with LW.lowering():
            u, ub = net(x), net(bx)
            if kind == "walls":  # two band tensors of the same shape
                ub, u = net(bx), net(bx[:81] * 0.5)
                loss = (torch.mean(ub[..., 0] ** 2) + torch.mean(u[..., 1] ** 2)) * 1.0
            else:
                loss = forms[kind](u, ub)
        assert isinstance(loss, LW.Lazy)
        if lowered:
            c0 = LW.LOWERED["terms"]
            loss = LW.lower_losses({"main": loss})["main"]
            assert LW.LOWERED["terms"] == c0 + 1
        else:
            loss = LW.materialize(loss)
        loss.backward()
        torch.cuda.synchronize()
        out[lowered] = (float(loss), net.flat_grad_buffer().detach().clone())
    assert abs(out[True][0] - out[False][0]) <= 1e-6 * abs(out[False][0]), out
    assert nerr(out[True][1].cpu().numpy(), out[False][1].cpu().numpy()) < 1e-5


def test_in_place_write_under_deferred_jets():
    """An in-place write inside the deferred scope, on a tensor made from a queued jet's output: the queue is
    launched and every expression recorded before the write evaluated first (eager order); the losses and the
    network's parameter gradients equal the same body run without the lowering."""
    import base
    from base import lower as LW
    torch.manual_seed(9)
    net = base.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    g = torch.Generator(device="cuda").manual_seed(10)
    x = (torch.rand(2000, 2, device="cuda", generator=g) * 2 - 1).requires_grad_(True)
    tgt = torch.randn(2000, 2, device="cuda", generator=g)

    def body():
        u = net(x)
        d = u - tgt
        v = u * 1.0
        v.add_(0.25)  # d was recorded before the write, v ** 2 after it
        return {"a": torch.mean(d ** 2), "b": torch.mean(v ** 2)}

    out = {}
    for lowered in (False, True):
        net.zero_grad(set_to_none=True)
        if lowered:
            with LW.lowering(), LW.deferred_jets():
                ld = body()
            ld = LW.lower_losses(ld)
        else:
            ld = body()
        sum(ld.values()).backward()
        torch.cuda.synchronize()
        out[lowered] = ({k: float(v) for k, v in ld.items()}, net.flat_grad_buffer().detach().clone())
    for k in ("a", "b"):
        assert abs(out[True][0][k] - out[False][0][k]) <= 1e-6 * abs(out[False][0][k]), (k, out)
    assert nerr(out[True][1].cpu().numpy(), out[False][1].cpu().numpy()) < 1e-5
