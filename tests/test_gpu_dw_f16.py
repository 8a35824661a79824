"""The x6 backward's products on the fp16 matrix cores (insr_jet_set_bwd_f16): the two-kernel
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
    lib = base._native.load()
    old_dw = lib.insr_jet_set_bwd_f16(request.param[0])
    old_pol = lib.insr_jet_set_bwd_policy(request.param[1])
    yield base
    lib.insr_jet_set_bwd_f16(old_dw)
    lib.insr_jet_set_bwd_policy(old_pol)


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
