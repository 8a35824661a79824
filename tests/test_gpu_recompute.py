"""The recompute backward (csrc/jet_fb.hpp, insr_jet_bwd_path == 3): one persistent launch that
reruns each tile's forward jet next to its reverse jet -- no saved streams -- vs the CPU oracle
(pinned to the reference: base/diff_ops.py:33-41 laplace, loss.backward() of
base/baseModel.py:73-78) and vs the saved-stream paths.

Tolerance as everywhere (north_star "1e-5 relative fp32"): normwise per tensor,
max|hip - ref| <= 1e-5 max|ref|, every field value and every parameter-gradient tensor.
"""
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-5
V, G, LAP = 0, 1, 2


@pytest.fixture(scope="module")
def B():
    """The recompute path forced on (policy 4: the per-call INSR_JET_POLICY bits every jet of the
    test thread carries) for the module: its own tests below switch to other paths explicitly where
    they compare against them."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    base._native.load()
    with base._native.knobs(policy=4):
        yield base


def nerr(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def pair(B, din, dout, L, W, seed):
    torch.manual_seed(seed)
    ref = O.OracleSiren(din, dout, L, W)
    torch.manual_seed(seed)
    net = B.MLP(din, dout, L, W, nonlinearity="sine")
    return ref, net.cuda()


def grads(net):
    return [(p.grad if p.grad is not None else torch.zeros_like(p)).detach().clone() for p in net.parameters()]


def ref_grads(ref):
    return [(p.grad if p.grad is not None else torch.zeros_like(p)).detach() for p in ref.parameters()]


def policy(lib, p, **kw):
    from base import _native as nat
    return nat.knobs(policy=p, **kw)


def knob(mode):
    """A jet mode with the test thread's knob bits (what base.MLP.call_mode adds)."""
    from base import _native as nat
    return mode | nat.scope_bits()


@pytest.mark.parametrize("n", [1, 15, 17, 300, 4111, 16708])
def test_laplace_jet_all_adjoints_vs_oracle(B, n):
    """The pressure net's 2-d Laplacian jet (fluid/model.py:111,116-120: lap p in the residual, grad p
    on the walls) with adjoints on the value, both gradient streams and the Laplacian stream: every
    parameter gradient vs the oracle; the forward of a path-3 call saves nothing."""
    lib = B._native.lib()
    assert lib.insr_jet_bwd_path(n, 2, 1, 4, 128, knob(LAP)) == 3
    ref, net = pair(B, 2, 1, 4, 128, seed=41)
    x = torch.rand(n, 2, generator=torch.Generator().manual_seed(n)) * 2 - 1
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    gr = O.op_gradient(yr, xr)
    lr_ = O.op_laplace(yr, xr)
    g = torch.Generator().manual_seed(n + 1)
    Ry, Rg, Rl = torch.randn(yr.shape, generator=g), torch.randn(gr.shape, generator=g), torch.randn(lr_.shape, generator=g)
    ((yr * Ry).sum() + (gr * Rg).sum() + (lr_ * Rl).sum()).backward()
    xg = x.cuda().requires_grad_(True)
    y = net(xg)
    lp, gp = B.laplace(y, xg, return_grad=True)
    assert nerr(lp, lr_) < TOL and nerr(gp, gr) < TOL and nerr(y, yr) < TOL
    ((y * Ry.cuda()).sum() + (gp * Rg.cuda()).sum() + (lp * Rl.cuda()).sum()).backward()
    torch.cuda.synchronize()
    for (k, _), a, b in zip(ref.named_parameters(), ref_grads(ref), grads(net)):
        assert nerr(b, a) < TOL, (n, k, nerr(b, a))


@pytest.mark.parametrize("n", [300, 16708])
def test_recompute_matches_two_kernel_path(B, n):
    """Same network, same adjoints: the recompute backward and the saved-stream two-kernel backward
    (policy 2) agree at the fp32 level (different summation orders only)."""
    lib = B._native.lib()
    out = []
    for pol in (4, 2):
        with policy(lib, pol):
            _, net = pair(B, 2, 1, 4, 128, seed=42)
            x = (torch.rand(n, 2, generator=torch.Generator().manual_seed(5)) * 2 - 1).cuda().requires_grad_(True)
            lp = B.laplace(net(x), x)
            R = torch.randn(lp.shape, generator=torch.Generator().manual_seed(6)).cuda()
            (lp * R).sum().backward()
            torch.cuda.synchronize()
            out.append(grads(net))
    for a, b in zip(*out):
        assert nerr(a, b) < TOL


def test_recompute_is_deterministic(B):
    """Fixed summation order: two identical backwards give bit-identical gradients."""
    out = []
    for _ in range(2):
        _, net = pair(B, 2, 1, 4, 128, seed=43)
        x = (torch.rand(16708, 2, generator=torch.Generator().manual_seed(9)) * 2 - 1).cuda().requires_grad_(True)
        lp = B.laplace(net(x), x)
        (lp * lp).sum().backward()
        torch.cuda.synchronize()
        out.append(grads(net))
    for a, b in zip(*out):
        assert torch.equal(a, b)


@pytest.mark.parametrize("kind", ["value", "jacobian"])
def test_forced_recompute_value_and_gradient_jets(B, kind):
    """Policy 4 forces the recompute kernel onto the velocity net's value and 2-d gradient jets
    (fluid/model.py:80,139 and the projection's grad p): both vs the oracle."""
    lib = B._native.lib()
    with policy(lib, 4):
        ref, net = pair(B, 2, 2, 4, 128, seed=44)
        n = 5000
        mode = V if kind == "value" else G
        assert lib.insr_jet_bwd_path(n, 2, 2, 4, 128, knob(mode)) == 3
        x = torch.rand(n, 2, generator=torch.Generator().manual_seed(3)) * 2 - 1
        xr = x.clone().requires_grad_(True)
        xg = x.cuda().requires_grad_(True)
        if kind == "value":
            vr, v = ref(xr), net(xg)
        else:
            vr, v = O.op_jacobian(ref(xr), xr)[0], B.jacobian(net(xg), xg)[0]
        assert nerr(v, vr) < TOL
        R = torch.randn(vr.shape, generator=torch.Generator().manual_seed(4))
        (vr * R).sum().backward()
        (v * R.cuda()).sum().backward()
        torch.cuda.synchronize()
        for (k, _), a, b in zip(ref.named_parameters(), ref_grads(ref), grads(net)):
            assert nerr(b, a) < TOL, (kind, k, nerr(b, a))


def test_batched_jobs_one_launch(B):
    """Three Laplacian calls of one network (the reference's interior + two wall bands,
    fluid/model.py:111,116-117) in one loss.backward(): one recompute launch over the three
    jobs (insr_siren_jet_bwd_grad_multi), vs the oracle."""
    ref, net = pair(B, 2, 1, 4, 128, seed=45)
    sizes = (4096, 162, 162)
    xs = [torch.rand(m, 2, generator=torch.Generator().manual_seed(20 + i)) * 2 - 1 for i, m in enumerate(sizes)]
    lr_ = 0
    for i, x in enumerate(xs):
        xr = x.clone().requires_grad_(True)
        lr_ = lr_ + (i + 1) * (O.op_laplace(ref(xr), xr) ** 2).mean() + (O.op_gradient(ref(xr), xr) ** 2).mean()
    lr_.backward()
    lg = 0
    with B._jet.batched_backward():
        for i, x in enumerate(xs):
            xg = x.cuda().requires_grad_(True)
            y = net(xg)
            lp, gp = B.laplace(y, xg, return_grad=True)
            lg = lg + (i + 1) * (lp ** 2).mean() + (gp ** 2).mean()
        lg.backward()
    torch.cuda.synchronize()
    for (k, _), a, b in zip(ref.named_parameters(), ref_grads(ref), grads(net)):
        assert nerr(b, a) < TOL, (k, nerr(b, a))


def test_large_tangents_stay_finite(B):
    """First layer x 4000: the hidden tangent streams exceed fp16's 65504 unscaled (|t| > 2183) and
    the layer-0 sine arguments take the libm path.  The recompute kernel scales every stream class
    per tile: finite and equal to the bf16x6 saved-stream path (fp32 range everywhere) at 1e-5."""
    lib = B._native.lib()
    out = []
    for pol, prec in ((4, None), (2, "bf16x6")):
        # the reference run: saved streams, every product bf16x6 (no fp16 operand anywhere)
        with policy(lib, pol, bwd_f16=7 if pol == 4 else 0):
            torch.manual_seed(46)
            net = B.MLP(2, 1, 4, 128, nonlinearity="sine", precision=prec).cuda()
            with torch.no_grad():
                net.net[0].weight.mul_(4000.0)
            assert lib.insr_jet_bwd_path(2000, 2, 1, 4, 128, net.call_mode(LAP)) == (3 if pol == 4 else 1)
            x = (torch.rand(2000, 2, generator=torch.Generator().manual_seed(7)) * 2 - 1).cuda().requires_grad_(True)
            lp, gp = B.laplace(net(x), x, return_grad=True)
            R = torch.randn(lp.shape, generator=torch.Generator().manual_seed(8)).cuda()
            ((lp * R).sum() + (gp ** 2).sum()).backward()
            torch.cuda.synchronize()
            out.append(grads(net))
    for a, b in zip(*out):
        assert torch.isfinite(a).all() and torch.isfinite(b).all()
        assert nerr(a, b) < TOL


@pytest.mark.parametrize("shape", [(2, 2, 5, 128), (3, 3, 5, 256), (1, 1, 3, 64)])
def test_large_tangents_gradient_jets(B, shape):
    """The same range stress on the gradient jets of the elasticity / advection nets
    (elasticity/model.py:137-143 jacobian, advection/model.py:78-86 gradient) through their default
    forward and backward paths: finite, and equal to the all-bf16x6 run (fp32 range) at 1e-5."""
    din, dout, L, W = shape
    lib = B._native.lib()
    out = []
    for prec in (None, "bf16x6"):
        # the default (saved-stream) paths; reference: no fp16 operand anywhere
        with policy(lib, 0, bwd_f16=7 if prec is None else 0):
            torch.manual_seed(47)
            net = B.MLP(din, dout, L, W, nonlinearity="sine", precision=prec).cuda()
            with torch.no_grad():
                net.net[0].weight.mul_(4000.0)
            x = (torch.rand(3000, din, generator=torch.Generator().manual_seed(7)) * 2 - 1).cuda().requires_grad_(True)
            J = B.jacobian(net(x), x)[0]
            assert torch.isfinite(J).all()
            R = torch.randn(J.shape, generator=torch.Generator().manual_seed(8)).cuda()
            (J * R).sum().backward()
            torch.cuda.synchronize()
            out.append([J.detach().clone()] + grads(net))
    for a, b in zip(*out):
        assert torch.isfinite(a).all() and torch.isfinite(b).all()
        assert nerr(a, b) < TOL
