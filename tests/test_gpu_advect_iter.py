"""The one-launch advection iteration (csrc/advect_iter.hip, base/advect_iter.py; round 6).

insr_advect1d_iteration draws the iteration's points, runs the frozen and the trainable field's value +
x-derivative jets, forms the residuals of advection/model.py:68-91 and runs the reverse jet, all in one
launch; the Adam launch sums its partial rows.  Checked here against the CPU oracle (the reference's
algorithm, oracle/siren_oracle.py advect1d_loss) on the points the kernel drew: both losses and every
parameter gradient at the parity tolerance for 1..3 hidden layers and ragged / band-free batches; the draws
bit-identical to insr_sample_boxes' with the same boxes and the device stream advanced alike; a training
loop of several iterations replayed from hipGraphs = eager, bit for bit.
"""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.fixture(scope="module")
def B():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    base._native.load()
    return base


def nerr(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def pair(B, L, seed):
    torch.manual_seed(seed)
    ref = O.OracleSiren(1, 1, L, 64)
    torch.manual_seed(seed + 1)
    ref_prev = O.OracleSiren(1, 1, L, 64)
    net = B.MLP(1, 1, L, 64, nonlinearity="sine").cuda()
    prev = B.MLP(1, 1, L, 64, nonlinearity="sine").cuda()
    with torch.no_grad():
        net.flat_params().copy_(O.flat_params(ref).cuda())
        prev.flat_params().copy_(O.flat_params(ref_prev).cuda())
    for p in prev.parameters():
        p.requires_grad_(False)
    return ref, ref_prev, net, prev


def boxes(n, h, half, eps):
    return [(n, [-half], [half]), (h, [(-1 - eps) * half], [(-1 + eps) * half]),
            (h, [(1 - eps) * half], [(1 + eps) * half])]


def test_points_bit_identical_to_the_sampler_launch(B):
    """The kernel's draw = insr_sample_boxes' draw of the same three boxes from the same stream position,
    bit for bit, and the device stream advances by the same count (the next draw continues identically)."""
    from base import advect_iter
    from base.sampling import _sampler, sample_boxes
    _, _, net, prev = pair(B, 3, 5)
    n, h, half, eps = 4096, 20, 1.5, 1e-4
    dev = torch.device("cuda", torch.cuda.current_device())
    state, _ = _sampler(dev)
    s0 = state.clone()
    ref = sample_boxes(boxes(n, h, half, eps), 1, device="cuda").view(-1).clone()
    s1 = state.clone()
    ref2 = sample_boxes(boxes(n, h, half, eps), 1, device="cuda").view(-1).clone()
    state.copy_(s0)
    pts = torch.empty(n + 2 * h, device="cuda")
    with torch.no_grad():
        advect_iter.advect1d_iteration(net, prev, n, h, half, eps, 0.05, 1.0, n, 2 * h, points=pts)
    torch.cuda.synchronize()
    assert torch.equal(pts, ref)
    assert torch.equal(state[:1], s1[:1]) and int(state[1]) == 0  # stream advanced alike, ticket reset
    pts2 = torch.empty_like(pts)
    with torch.no_grad():
        advect_iter.advect1d_iteration(net, prev, n, h, half, eps, 0.05, 1.0, n, 2 * h, points=pts2)
    assert torch.equal(pts2, ref2)


@pytest.mark.parametrize("L,n,h", [(3, 4096, 20), (1, 1000, 3), (2, 777, 10), (2, 4096, 20), (3, 5, 0),
                                   (3, 16384, 81)])
def test_losses_and_gradients_match_the_oracle(B, L, n, h):
    """Both losses and every parameter gradient of advection/model.py:68-91 at the points the kernel drew
    (parity tolerance, normwise per tensor); vel 1.3, dt 0.05, L / 2 = 1.5."""
    from base import advect_iter
    from base.losses import register_unit_seed
    ref, ref_prev, net, prev = pair(B, L, 100 + L)
    half, eps, dt, vel = 1.5, 1e-4, 0.05, 1.3
    pts = torch.empty(n + 2 * h, device="cuda")
    net.zero_grad(set_to_none=True)
    main, bc = advect_iter.advect1d_iteration(net, prev, n, h, half, eps, dt, vel, n, max(2 * h, 1), points=pts)
    one = register_unit_seed(torch.ones((), device="cuda"))
    torch.autograd.backward([main, bc], [one, one])
    torch.cuda.synchronize()
    x = pts[:n].cpu().view(-1, 1).clone().requires_grad_(True)
    xb = pts[n:].cpu().view(-1, 1).clone().requires_grad_(True)
    want = O.advect1d_loss(ref, ref_prev, x, xb, dt, vel)
    assert abs(float(main) - float(want["main"])) <= TOL * abs(float(want["main"])), (float(main), float(want["main"]))
    total = want["main"]
    if h > 0:
        assert abs(float(bc) - float(want["bc"])) <= TOL * abs(float(want["bc"])), (float(bc), float(want["bc"]))
        total = total + want["bc"]
    else:
        assert float(bc) == 0.0
    total.backward()
    for (k, p), q in zip(ref.named_parameters(), net.parameters()):
        assert nerr(q.grad.detach().cpu().numpy(), p.grad.numpy()) < TOL, (k, L, n, h)


def _model(B, fused, graph, iters):
    import pde.advection as adv
    from pde.config import baseline_config
    cfg = baseline_config("advect1D", proj_dir="/tmp/insr_adv_iter", insr_progress=False, early_stop=False,
                          max_n_iters=iters, insr_graph=graph, insr_graph_unroll=2 if graph else 1,
                          insr_sync_every=1000000, insr_advect_fused=fused)
    m = adv.Advection1DModel(cfg)
    m.timestep = 1
    torch.manual_seed(7)
    ref = O.OracleSiren(1, 1, 3, 64)
    with torch.no_grad():
        m.field.flat_params().copy_(O.flat_params(ref).cuda())
    m.field_prev.load_state_dict(m.field.state_dict())  # (step()'s snapshot, advection/model.py:64)
    return m


def test_training_loop_graph_equals_eager(B):
    """Seven iterations of the advection phase through PhaseLoop: replayed from hipGraphs (single and
    2-iteration groups) = eager, every parameter and both losses bit for bit; the capture succeeds."""
    from base import advect_iter
    out = []
    for graph in (False, True):
        torch.cuda.manual_seed(3)  # (a re-seed restarts the device stream: both runs draw the same points)
        m = _model(B, True, graph, 7)
        it0 = advect_iter.STATS["iterations"]
        m._advect()  # the phase loop (PhaseLoop): 7 iterations
        torch.cuda.synchronize()
        assert getattr(m, "_insr_capture_error", None) is None
        if not graph:
            assert advect_iter.STATS["iterations"] - it0 == 7
        out.append(m.field.flat_params().detach().cpu().clone())
    assert torch.equal(out[0], out[1])


def test_fused_route_tracks_the_generic_one(B):
    """The same seven iterations on the fused route and on the generic one (sampler launch, f16x3 jets, loss
    group, reverse jet): the same draws (one device stream) and the same losses up to the fp32-level jets'
    rounding, so the trained parameters agree to Adam's lr scale."""
    out = []
    for fused in (False, True):
        torch.cuda.manual_seed(3)
        m = _model(B, fused, False, 7)
        p0 = m.field.flat_params().detach().cpu().clone()
        m._advect()
        torch.cuda.synchronize()
        out.append(m.field.flat_params().detach().cpu() - p0)
    lr = 1e-4  # advect1D's cfg.lr (pde/config.py); Adam moves each entry by <= ~lr per iteration
    d = (out[0] - out[1]).abs()
    assert float(d.max()) <= 7 * 2 * lr * 1.01
    assert float(d.mean()) < 0.05 * float(out[0].abs().mean())
