"""Frozen work ahead (round 6: base.sampling.frozen_ahead, pde/fluid.py Fluid2DModel._ahead).

Inside a group of U iterations replayed as one hipGraph (base/_loop.py run_group), a fluid phase evaluates
the networks it does not train -- the advection's semi-Lagrangian target on u_prev (fluid/model.py:76-88),
the pressure phase's detached div u (:108-109), the projection's u_prev and detached grad p (:132-136) --
ONCE for all U iterations' points, and each iteration's forward launch holds only the trained network's
jet.  Checked here:

  * the group's outputs, iteration by iteration, against the same jets run on that iteration's points
    alone (the same kernels; only the tile grouping of the fp16 scales differs: <= 2e-6 normwise) and
    against the CPU oracle (1e-5 normwise, the parity contract);
  * whole phases through the loop (U = 4 groups, hipGraph): losses read at the sync points and the trained
    parameters against the same loop with the work inside each iteration's mixed launch;
  * the group path really runs (one frozen evaluation per group and phase)."""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def B():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    base._native.load()
    return base


def nerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _model(res, **kw):
    from pde.config import make_config
    from pde.fluid import Fluid2DModel
    torch.manual_seed(0)
    cfg = make_config("fluid", num_hidden_layers=4, hidden_features=128, sample_resolution=res, dt=0.05,
                      proj_dir="/tmp/insr_frozen_ahead", insr_progress=False, early_stop=False, lr=1e-4, **kw)
    m = Fluid2DModel(cfg)
    m.timestep = 1
    torch.manual_seed(1)
    with torch.no_grad():  # u_prev != u, so the advection target is not trivially u
        m.velocity_field_prev.flat_params().add_(1e-3 * torch.randn_like(m.velocity_field_prev.flat_params()))
    return m


def _oracle(net, din, dout):
    o = O.OracleSiren(din, dout, 4, 128)
    o.load_state_dict({k: v.detach().cpu() for k, v in net.state_dict().items()})
    for p in o.parameters():
        p.requires_grad_(False)
    return o


@pytest.mark.parametrize("res", [32, 128])
def test_group_outputs_equal_per_iteration_jets_and_oracle(B, res):
    from base.diff_ops import gradient, jacobian_only
    from base.sampling import draw_ahead, frozen_ahead
    m = _model(res)
    U, got, xs = 4, [], []
    with draw_ahead(U):
        for k in range(U):
            x = m._sample_in_training()
            xs.append(x.detach().clone())
            got.append((frozen_ahead("advect", x, m._target_all), frozen_ahead("pressure", x, m._div_all),
                        frozen_ahead("projection", x, m._projection_all)))
    assert len({float(x[0, 0]) for x in xs}) == U  # U different draws
    vp, v, p = _oracle(m.velocity_field_prev, 2, 2), _oracle(m.velocity_field, 2, 2), _oracle(m.pressure_field, 2, 1)
    for k in (0, U - 1):
        x = xs[k].clone().requires_grad_(True)
        (tgt,), (J,), (up, gp) = got[k]
        with torch.no_grad():
            t_alone = m._target_all(x)[0]
            J_alone = jacobian_only(m.velocity_field(x), x)
            up_alone = m.velocity_field_prev(x)
            gp_alone = gradient(m.pressure_field(x), x)
        for a, b in ((tgt, t_alone), (J, J_alone), (up, up_alone), (gp, gp_alone)):
            assert a.shape == b.shape and nerr(a, b) < 2e-6
        # the oracle (fluid/model.py:76-88,108-109,132-136 through the reference's autograd operators)
        xc = x.detach().cpu().requires_grad_(True)
        u0 = vp(xc)
        foot = torch.clamp(xc - 0.05 * u0, -1.0, 1.0)
        assert nerr(tgt, vp(foot)) < 1e-5
        assert nerr(J, O.op_jacobian(v(xc), xc)[0]) < 1e-5
        assert nerr(up, u0) < 1e-5
        assert nerr(gp, O.op_gradient(p(xc), xc)) < 1e-5


def _run(res, ahead, iters=10, **kw):
    m = _model(res, max_n_iters=iters, insr_graph=True, insr_sync_every=5, insr_graph_unroll=4,
               insr_frozen_ahead=ahead, **kw)
    seen = []
    m.tb = type("TB", (), {"add_scalars": lambda self, tag, vals, global_step: seen.append(
        (tag, global_step, vals["main"], vals["bc"]))})()
    calls = {"n": 0}
    import base.sampling as S
    orig = S.frozen_ahead

    def spy(name, x, fn, **kw):
        def fn2(X):
            calls["n"] += 1
            return fn(X)
        return orig(name, x, fn2, **kw)
    import pde.fluid as F
    F.frozen_ahead = spy
    try:
        for phase in ("_advect_velocity", "_solve_pressure", "_projection"):
            getattr(m, phase)()
            assert getattr(m, "_insr_capture_error", None) is None, m._insr_capture_error
    finally:
        F.frozen_ahead = orig
    torch.cuda.synchronize()
    return m, seen, calls["n"]


@pytest.mark.parametrize("mode", ["batch", "stream", "pipe"])
@pytest.mark.parametrize("res", [32, 128])
def test_grouped_phases_match_per_iteration_launches(B, res, mode):
    """10 iterations per phase, sync every 5 (host reads after iterations 0, 4 and 9): iterations 0 (eager),
    1 (captured), 2-4 single replays, 5-8 one U = 4 group graph, 9 a single replay.  Same draws in both runs;
    the frozen outputs differ only in the fp16 scales' tile grouping, so the losses agree to ~1e-6 and the
    trained networks stay within Adam's sign-flip bound of each other.  Modes: batched (one evaluation for
    the group), batched on a side stream, pipelined (per iteration on a side stream, one iteration ahead)."""
    kw = {"insr_frozen_stream": True} if mode == "stream" else {}
    on, seen_on, n_on = _run(res, "pipe" if mode == "pipe" else True, **kw)
    off, seen_off, n_off = _run(res, False)
    # frozen evaluations recorded by the group graph's single capture: one per phase (batched), or one per
    # iteration and phase (pipelined)
    assert n_on == (12 if mode == "pipe" else 3) and n_off == 0
    assert [s[:2] for s in seen_on] == [s[:2] for s in seen_off]
    for a, b in zip(seen_on, seen_off):
        assert abs(a[2] - b[2]) <= 2e-5 * abs(b[2]) + 1e-12, (a, b)
    for net in ("velocity_field", "pressure_field"):
        pa, pb = getattr(on, net).flat_params().detach(), getattr(off, net).flat_params().detach()
        d = (pa - pb).abs()
        assert float(d.max()) <= 2 * 10 * 1e-4  # Adam moves a parameter by <= ~lr per step
        assert float((d <= 1e-6 * float(pb.abs().max())).float().mean()) > 0.9
