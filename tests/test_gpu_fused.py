"""Horizontal fusion of forward jets (insr_siren_jet_fwd_multi / base.fused_forwards).

A fused launch runs each job's blocks with the single-launch arithmetic, so every
output (value, Jacobian, saved streams) must equal the separate launches BIT FOR BIT,
whatever tile count the combined batch selects; the oracle parity of the single launch
(test_gpu_parity.py) then carries over.  Model level: the fluid phases with
insr_fuse_forwards on and off give identical losses and Adam updates equal up to the
fp32 rounding of the gradients (one merged reverse jet vs two), in eager mode and under
hipGraph replay (the oracle check of the fused default is
test_gpu_phases.py::test_fluid_phases[False]).
"""

import contextlib

import pytest
import torch

pytestmark = pytest.mark.gpu

NETS = {"fluid_vel": (2, 2, 4, 128), "fluid_pres": (2, 1, 4, 128), "advect": (1, 1, 3, 64),
        "el3d": (3, 3, 5, 256), "w32": (2, 3, 2, 32)}  # width 32: separate launches behind the same entry


@pytest.fixture(scope="module")
def B():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    base._native.load()
    return base


def _net(B, name, seed):
    din, dout, L, W = NETS[name]
    torch.manual_seed(seed)
    return B.MLP(din, dout, L, W, nonlinearity="sine").cuda()


def _bufs(B, net, n, mode, save):
    lib = B._native.lib()
    din, dout, L, W = net.in_features, net.out_features, net.num_hidden_layers, net.hidden_features
    y = torch.full((n, dout), float("nan"), device="cuda")
    dy = torch.full((n, dout, din), float("nan"), device="cuda") if mode else None
    act = None
    if save:
        act = torch.full((max(lib.insr_jet_act_bytes(n, din, L, W, mode) // 4, 1),), float("nan"), device="cuda")
    return y, dy, act


def _single(B, net, x, mode, save):
    lib, nat = B._native.lib(), B._native
    net.ensure_packed()
    n = x.shape[0]
    y, dy, act = _bufs(B, net, n, mode, save)
    rc = lib.insr_siren_jet_fwd(nat.ptr(x), n, net.in_features, net.out_features, net.num_hidden_layers,
                                net.hidden_features, mode, nat.ptr(net.flat_params()), nat.ptr(y), nat.ptr(dy), None,
                                nat.ptr(act), nat.stream_of(x.device))
    nat.check(rc, "insr_siren_jet_fwd")
    return y, dy, act


def _multi(B, nets, xs, mode, saves):
    lib, nat = B._native.lib(), B._native
    outs, jobs = [], []
    for net, x, save in zip(nets, xs, saves):
        net.ensure_packed()
        y, dy, act = _bufs(B, net, x.shape[0], mode, save)
        outs.append((y, dy, act))
        jobs.append(nat.JetJob(x.data_ptr(), net.flat_params().data_ptr(), y.data_ptr(),
                               None if dy is None else dy.data_ptr(), None,
                               None if act is None else act.data_ptr(), x.shape[0], net.out_features))
    arr = (nat.JetJob * len(jobs))(*jobs)
    n0 = nets[0]
    rc = lib.insr_siren_jet_fwd_multi(arr, len(jobs), n0.in_features, n0.out_features, n0.num_hidden_layers,
                                      n0.hidden_features, mode, nat.stream_of(xs[0].device))
    nat.check(rc, "insr_siren_jet_fwd_multi")
    return outs


def _eq(a, b, n=None, layers=None, w=None):
    """Bit equality; for saved streams (n points, `layers` = L + 1) only the tiles of real
    points: the 16-point tiles past the last one are padding that a launch writes or skips
    depending on its tiles per block; and of the first layer only its value stream (its
    derivative streams are point-independent, rebuilt from W_0 by every backward: not saved)."""
    if a is None or b is None:
        return a is None and b is None
    if n == 0:
        return True  # an empty job saves nothing (its buffer is never written)
    if n is not None:
        ntiles = ((n + 63) // 64) * 4  # [layer][tile][stream][row tile][lane][4]
        a, b = a.view(layers, ntiles, -1)[:, :(n + 15) // 16], b.view(layers, ntiles, -1)[:, :(n + 15) // 16]
        if layers > 1:  # the first layer's value stream: 16 points x w floats per tile
            return torch.equal(a[1:], b[1:]) and torch.equal(a[0, :, :16 * w], b[0, :, :16 * w])
    return torch.equal(a, b)


@pytest.mark.parametrize("name", list(NETS))
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("sizes", [(16384, 16384), (324, 16384, 16384), (1000, 324, 0), (64, 20000, 5, 333)])
def test_multi_matches_single_launches(B, name, mode, sizes):
    din = NETS[name][0]
    nets = [_net(B, name, seed=10 + k) for k in range(len(sizes))]
    g = torch.Generator().manual_seed(3)
    xs = [(torch.rand(n, din, generator=g) * 2 - 1).cuda() for n in sizes]
    saves = [k % 2 == 0 for k in range(len(sizes))]
    fused = _multi(B, nets, xs, mode, saves)
    for net, x, save, (y, dy, act) in zip(nets, xs, saves, fused):
        ys, dys, acts = _single(B, net, x, mode, save)
        assert _eq(y, ys) and _eq(dy, dys) and _eq(act, acts, x.shape[0], net.num_hidden_layers + 1, net.kernel_width), (name, mode, x.shape[0])


@pytest.mark.parametrize("mode", [0, 1])
def test_multi_mixed_output_widths(B, mode):
    """Jobs of one launch may differ in d_out (the pressure band 2->1 and the velocity 2->2)."""
    nets = [_net(B, "fluid_pres", 3), _net(B, "fluid_vel", 4), _net(B, "fluid_pres", 5)]
    g = torch.Generator().manual_seed(8)
    xs = [(torch.rand(n, 2, generator=g) * 2 - 1).cuda() for n in (324, 16384, 1000)]  # one fused launch
    saves = [True, False, True]
    fused = _multi(B, nets, xs, mode, saves)
    for net, x, save, (y, dy, act) in zip(nets, xs, saves, fused):
        ys, dys, acts = _single(B, net, x, mode, save)
        assert _eq(y, ys) and _eq(dy, dys) and _eq(act, acts, x.shape[0], net.num_hidden_layers + 1, net.kernel_width)


def test_multi_rejects_bad_arguments(B):
    lib, nat = B._native.lib(), B._native
    assert lib.insr_siren_jet_fwd_multi(None, 2, 2, 2, 4, 128, 0, None) == -1
    arr = (nat.JetJob * (nat.MAX_FWD_JOBS + 1))()
    assert lib.insr_siren_jet_fwd_multi(arr, nat.MAX_FWD_JOBS + 1, 2, 2, 4, 128, 0, None) == -1  # > INSR_MAX_FWD_JOBS
    assert lib.insr_siren_jet_fwd_multi(arr, 2, 2, 2, 4, 100, 0, None) == -1  # width
    assert lib.insr_siren_jet_fwd_multi(arr, 2, 2, 2, 4, 128, 0, None) == 0   # all jobs empty
    arr[0].n = 10  # a live job with NULL buffers
    assert lib.insr_siren_jet_fwd_multi(arr, 2, 2, 2, 4, 128, 0, None) == -1


def test_fused_scope_values_and_param_grads(B):
    """Inside `fused_forwards()` the jets only queue; the outputs, autograd nodes and saved
    streams are those of separate calls (values and parameter gradients bit-equal)."""
    x = (torch.rand(4096, 2, generator=torch.Generator().manual_seed(5)) * 2 - 1).cuda().requires_grad_(True)
    R = torch.randn(4096, 2, generator=torch.Generator().manual_seed(6)).cuda()
    res = {}
    for fused in (False, True):
        a, b = _net(B, "fluid_vel", 1), _net(B, "fluid_vel", 2)  # fresh nets: .grad starts empty
        if fused:
            with B.fused_forwards():
                ya, yb = a(x), b(x)
        else:
            ya, yb = a(x), b(x)
        ((ya * R).sum() + (yb * R * 0.5).sum()).backward()
        res[fused] = (ya.detach().clone(), yb.detach().clone(), a.flat_grad_buffer().clone(), b.flat_grad_buffer().clone())
    for u, v in zip(res[False], res[True]):
        assert torch.equal(u, v)


def _fluid(ph_cfg, fuse, graph):
    from pde.config import make_config
    from pde.fluid import Fluid2DModel
    cfg = make_config("fluid", proj_dir="/tmp/insr_test", insr_progress=False, early_stop=False, max_n_iters=4,
                      lr=1e-4, num_hidden_layers=4, hidden_features=128, sample_resolution=64, dt=0.05,
                      insr_fuse_forwards=fuse, insr_graph=graph, insr_sync_every=2)
    torch.manual_seed(0)
    model = Fluid2DModel(cfg)
    torch.manual_seed(1)
    model.velocity_field_prev.load_state_dict(
        {k: v + 1e-3 * torch.randn_like(v) for k, v in model.velocity_field.state_dict().items()})
    return model


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("phase", ["_advect_velocity", "_solve_pressure", "_projection"])
def test_fluid_phase_fused_equals_unfused(B, phase, graph):
    g = torch.Generator().manual_seed(9)
    xs = [(torch.rand(4096, 2, generator=g) * 2 - 1).cuda() for _ in range(4)]
    bx = (torch.rand(40, 2, generator=g) * 2 - 1).cuda()
    by = (torch.rand(40, 2, generator=g) * 2 - 1).cuda()
    out = {}
    for fuse in (False, True):
        model = _fluid(None, fuse, graph)
        it = {"k": 0}
        static_x = xs[0].clone()

        def sample():
            if graph:  # a captured phase replays its sampler: keep one static batch
                return static_x.clone().requires_grad_(True)
            x = xs[it["k"] % len(xs)]
            it["k"] += 1
            return x.clone().requires_grad_(True)
        model._sample_in_training = sample
        model._boundary_pair = lambda n: (bx.clone().requires_grad_(True), by.clone().requires_grad_(True))
        model.timestep = 1
        getattr(model, phase)()
        if graph:
            assert getattr(model, "_insr_capture_error", None) is None
        out[fuse] = (model.velocity_field.flat_params().detach().clone(),
                     model.pressure_field.flat_params().detach().clone(),
                     float(model.optimizer.state[0]), float(model.optimizer.state[1]))
    assert out[True][2:] == out[False][2:]
    # the fused phases run ONE reverse jet over the merged [interior; band] batch (other
    # block partition, other fixed summation order of the parameter gradient) where the
    # unfused ones run two and add: equal up to fp32 rounding of the gradients -- Adam moves
    # an entry by at most 2 lr per step either way, and only entries with noise-floor
    # gradients differ visibly
    for a, b in zip(out[True][:2], out[False][:2]):
        d = (a - b).abs()
        assert float(d.max()) <= 4 * 2 * 1e-4 * 1.01, phase
        assert float((d > 1e-6).float().mean()) < 0.02, phase


@pytest.mark.parametrize("n", [4096, 16708])
def test_mixed_mode_launch_matches_single_launches(B, n):
    """insr_siren_jet_fwd_mixed (jets of different modes in one launch) gives each job its own
    single-launch outputs bit for bit: velocity Jacobian + pressure Laplacian/gradient (the
    pressure phase), and frozen value + pressure gradient + trainable value (projection)."""
    from base import _jet
    from base.diff_ops import jacobian_only
    vel, pres, prev = _net(B, "fluid_vel", 1), _net(B, "fluid_pres", 2), _net(B, "fluid_vel", 3)
    g = torch.Generator().manual_seed(21)
    x = (torch.rand(n, 2, generator=g) * 2 - 1).cuda()
    xa = (torch.rand(n + 324, 2, generator=g) * 2 - 1).cuda()

    def pressure_phase(fused):
        xg, xag = x.clone().requires_grad_(True), xa.clone().requires_grad_(True)
        ctx = B.fused_forwards() if fused else contextlib.nullcontext()
        with ctx:
            with torch.no_grad():
                J = jacobian_only(vel(xg), xg)
            lap, gp = B.laplace(pres(xag), xag, return_grad=True)
        return J, lap, gp

    def projection(fused):
        xg, xag = x.clone().requires_grad_(True), xa.clone().requires_grad_(True)
        ctx = B.fused_forwards() if fused else contextlib.nullcontext()
        with ctx:
            with torch.no_grad():
                up = prev(xg)
                gp = B.gradient(pres(xg), xg)
            ua = vel(xag)
        return up, gp, ua

    assert _jet._MIXED
    for phase in (pressure_phase, projection):
        for u, v in zip(phase(False), phase(True)):
            assert torch.equal(u, v), phase.__name__


@pytest.mark.parametrize("fused", [False, True])
def test_advect_target_matches_the_three_steps(B, fused):
    """base.advect_target (INSR_MIX_ADVECT: two value jets of the frozen field and the foot
    clamp(x - dt f(x), -1, 1) in one job, fluid/model.py:96-97) equals f(x), the axpy foot and
    f(foot) launched separately, bit for bit -- alone and inside a mixed launch beside the
    trainable field's value jet."""
    prev, cur = _net(B, "fluid_vel", 4), _net(B, "fluid_vel", 5)
    g = torch.Generator().manual_seed(23)
    x = (torch.rand(16384, 2, generator=g) * 2 - 1).cuda()
    xa = (torch.rand(16708, 2, generator=g) * 2 - 1).cuda()
    dt = 0.05
    with torch.no_grad():
        up_ref = prev(x)
        foot = B.axpy_clamp(x, up_ref, -dt, -1.0, 1.0)
        tgt_ref = prev(foot)
        ua_ref = cur(xa)
    ctx = B.fused_forwards() if fused else contextlib.nullcontext()
    with torch.no_grad(), ctx:
        tgt, up = B.advect_target(prev, x, dt, -1.0, 1.0)
        ua = cur(xa)
    assert torch.equal(up, up_ref) and torch.equal(tgt, tgt_ref) and torch.equal(ua, ua_ref)
