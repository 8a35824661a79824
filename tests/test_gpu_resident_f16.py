"""The resident-dW backward with f16x3 products (policy 5: csrc/jet_fb.hpp with SAVED = true, the
reverse sweep of the recompute kernel run on the forward's saved streams; insr_jet_bwd_path == 2):
one persistent launch per backward, dW of every hidden layer in registers across the tile loop, no
z̄ round trip through HBM -- vs the CPU oracle (pinned to the reference: base/diff_ops.py:33-82,
loss.backward() of base/baseModel.py:73-78) and vs the two-kernel saved-stream path.

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
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    base._native.load()
    with base._native.knobs(policy=5):
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


@pytest.mark.parametrize("n", [1, 17, 300, 4111, 16708])
def test_laplace_jet_all_adjoints_vs_oracle(B, n):
    """The pressure net's 2-d Laplacian jet with adjoints on every stream: each parameter gradient."""
    lib = B._native.lib()
    assert lib.insr_jet_bwd_path(n, 2, 1, 4, 128, LAP | B._native.scope_bits()) == 2
    ref, net = pair(B, 2, 1, 4, 128, seed=71)
    x = torch.rand(n, 2, generator=torch.Generator().manual_seed(n)) * 2 - 1
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    gr, lr_ = O.op_gradient(yr, xr), O.op_laplace(yr, xr)
    g = torch.Generator().manual_seed(n + 1)
    Ry, Rg, Rl = torch.randn(yr.shape, generator=g), torch.randn(gr.shape, generator=g), torch.randn(lr_.shape, generator=g)
    ((yr * Ry).sum() + (gr * Rg).sum() + (lr_ * Rl).sum()).backward()
    xg = x.cuda().requires_grad_(True)
    y = net(xg)
    lp, gp = B.laplace(y, xg, return_grad=True)
    ((y * Ry.cuda()).sum() + (gp * Rg.cuda()).sum() + (lp * Rl.cuda()).sum()).backward()
    torch.cuda.synchronize()
    for (k, _), a, b in zip(ref.named_parameters(), ref_grads(ref), grads(net)):
        assert nerr(b, a) < TOL, (n, k, nerr(b, a))


@pytest.mark.parametrize("kind", ["value", "jacobian"])
@pytest.mark.parametrize("n", [33, 5000])
def test_value_and_gradient_jets_vs_oracle(B, kind, n):
    """The velocity net's value and 2-d gradient jets (fluid/model.py:80,139; the projection's grad p)."""
    lib = B._native.lib()
    ref, net = pair(B, 2, 2, 4, 128, seed=72)
    mode = V if kind == "value" else G
    assert lib.insr_jet_bwd_path(n, 2, 2, 4, 128, mode | B._native.scope_bits()) == 2
    x = torch.rand(n, 2, generator=torch.Generator().manual_seed(3)) * 2 - 1
    xr = x.clone().requires_grad_(True)
    xg = x.cuda().requires_grad_(True)
    if kind == "value":
        vr, v = ref(xr), net(xg)
    else:
        vr, v = O.op_jacobian(ref(xr), xr)[0], B.jacobian(net(xg), xg)[0]
    R = torch.randn(vr.shape, generator=torch.Generator().manual_seed(4))
    (vr * R).sum().backward()
    (v * R.cuda()).sum().backward()
    torch.cuda.synchronize()
    for (k, _), a, b in zip(ref.named_parameters(), ref_grads(ref), grads(net)):
        assert nerr(b, a) < TOL, (kind, n, k, nerr(b, a))


@pytest.mark.parametrize("n", [4096, 8192 + 163])
def test_auto_policy_shard_sizes_vs_oracle(B, n):
    """The default policy takes this kernel from 4,096 points (the fluid2DtlgnM 8-way shard's
    pressure batch, 8,192 interior + 163 band points; fluid/model.py:103-125): the pressure loss's
    Laplacian adjoint, each parameter gradient vs the oracle."""
    lib = B._native.lib()
    with B._native.knobs(policy=0):
        assert lib.insr_jet_bwd_path(n, 2, 1, 4, 128, LAP | B._native.scope_bits()) == 2
        ref, net = pair(B, 2, 1, 4, 128, seed=74)
        x = torch.rand(n, 2, generator=torch.Generator().manual_seed(n)) * 2 - 1
        xr = x.clone().requires_grad_(True)
        lr_ = O.op_laplace(ref(xr), xr)
        R = torch.randn(lr_.shape, generator=torch.Generator().manual_seed(n + 2))
        (lr_ * R).sum().backward()
        xg = x.cuda().requires_grad_(True)
        lp = B.laplace(net(xg), xg)
        (lp * R.cuda()).sum().backward()
        torch.cuda.synchronize()
        assert nerr(lp, lr_) < TOL
        for (k, _), a, b in zip(ref.named_parameters(), ref_grads(ref), grads(net)):
            assert nerr(b, a) < TOL, (n, k, nerr(b, a))


@pytest.mark.parametrize("n", [4113, 20400])
def test_five_layer_gradient_jet_auto_policy(B, n):
    """Round 6: the default policy takes this kernel for the 2-d gradient jet of a 5 x 128 net from 4,096
    points -- elasticity2Dstretch's Jacobian of q = f(x) + x (elasticity/model.py:137,143; 20,000 interior +
    2 x 200 constraint points) -- vs the oracle (every parameter gradient) and vs the two-kernel backward."""
    lib = B._native.lib()
    out = []
    for pol in (0, 2):
        with B._native.knobs(policy=pol):
            assert lib.insr_jet_bwd_path(n, 2, 2, 5, 128, G | B._native.scope_bits()) == (2 if pol == 0 else 1)
            ref, net = pair(B, 2, 2, 5, 128, seed=75)
            x = torch.rand(n, 2, generator=torch.Generator().manual_seed(n)) * 2 - 1
            xg = x.cuda().requires_grad_(True)
            J = B.jacobian(net(xg) + xg, xg)[0]
            R = torch.randn(J.shape, generator=torch.Generator().manual_seed(n + 3))
            (J * R.cuda()).sum().backward()
            torch.cuda.synchronize()
            out.append(grads(net))
    xr = x.clone().requires_grad_(True)
    Jr = O.op_jacobian(ref(xr) + xr, xr)[0]
    (Jr * R).sum().backward()
    for (k, _), a, b in zip(ref.named_parameters(), ref_grads(ref), out[0]):
        assert nerr(b, a) < TOL, (n, k, nerr(b, a))
    for a, b in zip(*out):
        assert nerr(a, b) < TOL


@pytest.mark.parametrize("n", [300, 16708])
def test_matches_two_kernel_path(B, n):
    """Same network and adjoints: this kernel vs the saved-stream two-kernel backward (policy 2)."""
    out = []
    for pol in (5, 2):
        with B._native.knobs(policy=pol):
            torch.manual_seed(73)
            net = B.MLP(2, 1, 4, 128, nonlinearity="sine").cuda()
            x = (torch.rand(n, 2, generator=torch.Generator().manual_seed(5)) * 2 - 1).cuda().requires_grad_(True)
            lp = B.laplace(net(x), x)
            R = torch.randn(lp.shape, generator=torch.Generator().manual_seed(6)).cuda()
            (lp * R).sum().backward()
            torch.cuda.synchronize()
            out.append(grads(net))
    for a, b in zip(*out):
        assert nerr(a, b) < TOL


def test_deterministic(B):
    """Fixed summation order: two identical backwards give bit-identical gradients."""
    out = []
    for _ in range(2):
        _, net = pair(B, 2, 1, 4, 128, seed=74)
        x = (torch.rand(16708, 2, generator=torch.Generator().manual_seed(9)) * 2 - 1).cuda().requires_grad_(True)
        lp = B.laplace(net(x), x)
        (lp * lp).sum().backward()
        torch.cuda.synchronize()
        out.append(grads(net))
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_large_tangents_stay_finite(B):
    """First layer x 4000 (hidden tangents far beyond fp16's range unscaled): the per-tile scales of
    every stream class keep the f16x3 products finite and equal to the all-bf16x6 two-kernel run."""
    out = []
    for pol, prec, f16 in ((5, None, 7), (2, "bf16x6", 0)):
        with B._native.knobs(policy=pol, bwd_f16=f16):
            torch.manual_seed(75)
            net = B.MLP(2, 1, 4, 128, nonlinearity="sine", precision=prec).cuda()
            with torch.no_grad():
                net.net[0].weight.mul_(4000.0)
            x = (torch.rand(2000, 2, generator=torch.Generator().manual_seed(7)) * 2 - 1).cuda().requires_grad_(True)
            lp, gp = B.laplace(net(x), x, return_grad=True)
            R = torch.randn(lp.shape, generator=torch.Generator().manual_seed(8)).cuda()
            ((lp * R).sum() + (gp ** 2).sum()).backward()
            torch.cuda.synchronize()
            out.append(grads(net))
    for a, b in zip(*out):
        assert torch.isfinite(a).all() and torch.isfinite(b).all()
        assert nerr(a, b) < TOL
