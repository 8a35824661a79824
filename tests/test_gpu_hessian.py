"""hessian (base/diff_ops.py:6-30) and laplace(normalize=True) (:33-41) on the HIP jets:
the REFERENCE's own Hessians and the parameter gradients of a random functional of them
(tests/golden/ref_ops.npz, recorded by tests/golden/make_golden.py from /root/reference on
(1, 256, d) inputs), and the normalised Laplacian against fp64 autograd of the oracle.
d_in = 1 reads the Laplacian stream; d_in = 2 polarises Laplacian jets of f(x + s v).
Tolerance: 1e-5 normwise on values; 1e-4 on the parameter gradients (the polarisation
subtracts Laplacians of similar size: tr(H) + v.H v - tr(H))."""
import os

import numpy as np
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_ops.npz")


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return dict(np.load(GOLD))


def nerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("name", ["advect", "fluid_vel", "fluid_pres", "el2d"])
def test_hessian_matches_reference(ops, name):
    import base as B
    din, dout, L, W = (int(v) for v in ops[f"{name}/shape"])
    torch.manual_seed(int(ops[f"{name}/seed"]))
    net = B.MLP(din, dout, L, W, nonlinearity="sine").cuda()  # the reference's init, bit for bit
    x3 = torch.from_numpy(ops[f"{name}/x"])[None].cuda().requires_grad_(True)
    h, st = B.hessian(net(x3), x3)
    assert st == int(ops[f"{name}/hessian_status"])
    assert h.shape == ops[f"{name}/hessian"].shape
    assert nerr(h.detach().cpu(), ops[f"{name}/hessian"]) < 1e-5
    net.zero_grad(set_to_none=True)
    (h * torch.from_numpy(ops[f"{name}/hessian_R"]).cuda()).sum().backward()
    g = net.flat_grad_buffer().detach().cpu().numpy()[:net.param_count]
    stride = int(ops[f"{name}/param_stride"])
    assert nerr(g[::stride], ops[f"{name}/hessian_pgrad"]) < 1e-4


def _norm_lap(net, x, eps):
    g = O.op_gradient(net(x), x)
    return O.op_divergence(g / (g.norm(dim=-1, keepdim=True) + eps), x)


def test_laplace_normalize_matches_oracle():
    """div(g / (|g| + eps)) divides by |g| and |g|^3: where the gradient is small every fp32
    evaluation (the reference's too) loses digits, so the HIP result is judged against fp64 and
    must stay within 5x the error of the oracle's own fp32 autograd graph (or 1e-5).  Measured:
    4.3e-4 vs the oracle's 1.4e-4 -- the split-bf16 products round differently from fp32 FMAs
    and the conditioning multiplies either."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import copy
    import base as B
    torch.manual_seed(3)
    ref = O.OracleSiren(2, 1, 3, 64)
    ref64 = copy.deepcopy(ref).double()
    torch.manual_seed(3)
    net = B.MLP(2, 1, 3, 64, nonlinearity="sine").cuda()
    x = torch.rand(500, 2, generator=torch.Generator().manual_seed(4)) * 2 - 1
    eps = 1e-3
    R = torch.randn(500, 1, generator=torch.Generator().manual_seed(5))
    x64 = x.double().requires_grad_(True)
    d64 = _norm_lap(ref64, x64, eps)
    (d64 * R.double()).sum().backward()
    xr = x.clone().requires_grad_(True)
    d32 = _norm_lap(ref, xr, eps)
    (d32 * R).sum().backward()
    xg = x.cuda().requires_grad_(True)
    dg = B.laplace(net(xg), xg, normalize=True, eps=eps)
    (dg * R.cuda()).sum().backward()
    e_or, e_hip = nerr(d32.detach(), d64.detach()), nerr(dg.detach().cpu(), d64.detach())
    assert e_hip <= max(1e-5, 5 * e_or), (e_hip, e_or)
    flat = lambda m: torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1).cpu().double()  # noqa: E731
                                for p in m.parameters()])  # (the output bias gets no gradient)
    g64, g32, gg = flat(ref64), flat(ref), flat(net)
    e_or, e_hip = nerr(g32, g64), nerr(gg, g64)
    assert e_hip <= max(1e-4, 5 * e_or), (e_hip, e_or)


def test_hessian_3d_input_takes_the_reference_route():
    """d_in = 3 has no polarised Hessian jet: hessian() takes the reference's autograd route (the jet
    nodes differentiate themselves with torch ops) and equals the oracle's Hessian
    (tests/test_gpu_fallback.py covers it with parameter gradients)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base as B
    torch.manual_seed(3)
    ref = O.OracleSiren(3, 1, 2, 32)
    torch.manual_seed(3)
    net = B.MLP(3, 1, 2, 32, nonlinearity="sine").cuda()
    x = torch.rand(10, 3)
    xg = x.cuda().requires_grad_(True)
    H, st = B.hessian(net(xg), xg)
    xr = x.clone().requires_grad_(True)
    Hr, _ = O.op_hessian(ref(xr), xr)
    assert st == 0 and H.shape == (10, 1, 3, 3)
    assert float((H.detach().cpu() - Hr.detach()).abs().max() / Hr.abs().max()) < 1e-5


@pytest.mark.parametrize("scale_x,scale_w0", [(4.0, 1.0), (1.0, 3.0), (8.0, 3.0)])
def test_hessian_polarisation_off_domain_and_high_frequency(scale_x, scale_w0):
    """The d_in = 2 Hessian subtracts Laplacian jets of similar size ((Lap_aug(8v) - tr H) / 64).
    Stress: points up to |x| = 8 (outside the [-1, 1]^2 training box) and a first layer scaled x3
    (3x the spatial frequencies: second derivatives x9); judged against fp64 autograd of the
    oracle, the HIP error must stay within 5x the oracle's own fp32 autograd error (or 1e-5)."""
    import copy
    import base as B
    torch.manual_seed(17)
    net = B.MLP(2, 1, 4, 128, nonlinearity="sine").cuda()
    with torch.no_grad():
        net.net[0].weight.mul_(scale_w0)
    ref32 = O.OracleSiren(2, 1, 4, 128)
    ref32.load_state_dict({k: v.detach().cpu() for k, v in net.state_dict().items()})
    ref64 = copy.deepcopy(ref32).double()
    x = (torch.rand(512, 2, generator=torch.Generator().manual_seed(18)) * 2 - 1) * scale_x
    xg = x.cuda().requires_grad_(True)
    h, st = B.hessian(net(xg), xg)
    x64 = x.double().requires_grad_(True)
    h64, _ = O.op_hessian(ref64(x64), x64)
    x32 = x.clone().requires_grad_(True)
    h32, _ = O.op_hessian(ref32(x32), x32)
    e_hip = nerr(h.detach().cpu(), h64.detach())
    e32 = nerr(h32.detach(), h64.detach())
    assert st == 0 and e_hip <= max(5 * e32, 1e-5), (e_hip, e32)
