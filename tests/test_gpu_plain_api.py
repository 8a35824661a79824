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
