"""The x6 backward's products on the fp16 matrix cores (INSR_JET_BWD_F16 mode bits): the two-kernel
path's dW GEMM and propagation, the fused tile-split kernel.

f16x3 (two fp16 terms per operand, three products) keeps 22 significant bits but fp16's narrow
range: each dW K slice / propagated tile / fused block scales its adjoints by the power of two
that maps its largest |z̄| into [2^14, 2^15) and undoes it exactly on its output.  Held to the parity tolerance (1e-5 normwise per parameter tensor vs the CPU oracle) for
the Laplacian, gradient and value jets of the fluid nets through the two-kernel path, the 5x256
elasticity3Dbunny net, and adjoint seeds scaled by 1e-12 and 1e12 (the scale is found per slice,
so fp16's range never binds the adjoints).
"""
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-5


# (INSR_BWD_F16_* mask, backward-path policy): the two-kernel path's dW, its propagation, both;
# the fused tile-split kernel (policy 1: fused wherever it exists -- W = 256 stays two-kernel)
@pytest.fixture(scope="module", params=[(1, 2), (2, 2), (3, 2), (4, 1), (7, 0)])
def B(request):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    base._native.load()
    with base._native.knobs(bwd_f16=request.param[0], policy=request.param[1]):  # per-call mode bits
        yield base


def nerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


OPS = {"laplace": ("laplace", O.op_laplace), "gradient": ("gradient", O.op_gradient),
       "value": (None, None)}


@pytest.mark.parametrize("net,op,n,scale", [
    ((2, 1, 4, 128), "laplace", 16708, 1.0),
    ((2, 1, 4, 128), "laplace", 3000, 1e-12),
    ((2, 1, 4, 128), "laplace", 777, 1e12),
    ((2, 1, 4, 128), "gradient", 5000, 1.0),
    ((2, 2, 4, 128), "value", 9000, 1.0),
    ((2, 2, 5, 128), "gradient", 20400, 1.0),
    ((3, 3, 5, 256), "gradient", 4096, 1.0),
])
def test_dw_f16_matches_oracle(B, net, op, n, scale):
    din, dout, L, W = net
    torch.manual_seed(5)
    ref = O.OracleSiren(din, dout, L, W)
    torch.manual_seed(5)
    hip = B.MLP(din, dout, L, W, nonlinearity="sine").cuda()
    x = torch.rand(n, din, generator=torch.Generator().manual_seed(6)) * 2 - 1
    bop, oop = OPS[op]

    def out(mod, f, xx):
        y = f(xx)
        if op == "value":
            return y
        return getattr(B, bop)(y, xx) if mod is B else oop(y, xx)

    xr = x.clone().requires_grad_(True)
    yr = out(O, ref, xr)
    R = torch.randn(yr.shape, generator=torch.Generator().manual_seed(7)) * scale
    (yr * R).sum().backward()
    xg = x.cuda().requires_grad_(True)
    (out(B, hip, xg) * R.cuda()).sum().backward()
    torch.cuda.synchronize()
    for (k, p), q in zip(ref.named_parameters(), hip.parameters()):
        ga = p.grad if p.grad is not None else torch.zeros_like(p)
        gb = q.grad if q.grad is not None else torch.zeros_like(q)
        assert torch.isfinite(gb).all(), k
        assert nerr(gb, ga) < TOL, (k, nerr(gb, ga))



@pytest.mark.parametrize("w0_scale", [40.0, 200.0])
def test_dw_f16_large_tangents(B, w0_scale):
    """Laplacian-jet backward with the first layer scaled x40 / x200: tangents ~40-200x and h's
    Laplacian stream ~1.6e3-4e4x the init's.  h_lap's fp16 scale is found per dW slice / fused block
    from the propagation's bounds (w |q| + w^2 sum t^2), so the products stay in fp16's range; the
    static 2^-10 of an intermediate version held |t| < ~270 only.

    Pre-activations of ~30 x 40 rad make the problem itself ill-conditioned in fp32 (a phase
    rounding of |w z| 2^-24 ~ 1e-4 relative), so the yardstick is an fp64 oracle and the error of
    the same path with bf16x6 products (mask 0): the fp16 products may not add to it."""
    lib = B._native.load()
    torch.manual_seed(5)
    ref = O.OracleSiren(2, 1, 4, 128).double()
    torch.manual_seed(5)
    hip = B.MLP(2, 1, 4, 128, nonlinearity="sine").cuda()
    with torch.no_grad():
        next(ref.parameters()).mul_(w0_scale)
        next(hip.parameters()).mul_(w0_scale)
    x = torch.rand(6000, 2, generator=torch.Generator().manual_seed(6)) * 2 - 1
    xr = x.double().requires_grad_(True)
    yr = O.op_laplace(ref(xr), xr)
    R = torch.randn(yr.shape, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
    (yr * R).sum().backward()

    def grads():
        hip.zero_grad(set_to_none=True)
        xg = x.cuda().requires_grad_(True)
        (B.laplace(hip(xg), xg) * R.float().cuda()).sum().backward()
        torch.cuda.synchronize()
        return [q.grad.clone() if q.grad is not None else torch.zeros_like(q) for q in hip.parameters()]

    g16 = grads()
    with B._native.knobs(bwd_f16=0):
        g6 = grads()
    for (k, p), a, b in zip(ref.named_parameters(), g16, g6):
        assert torch.isfinite(a).all(), k
        g = p.grad if p.grad is not None else torch.zeros_like(p)  # the output bias: no Laplacian
        if g.abs().max() == 0:
            assert a.abs().max() == 0 and b.abs().max() == 0, k
            continue
        e16, e6 = nerr(a, g), nerr(b, g)
        assert e16 < max(TOL, 2.0 * e6), (k, e16, e6)
