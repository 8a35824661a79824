"""Parity at the BASELINE.json sizes (SURVEY.md §8 d): the HIP jets against the CPU oracle
on the full fluid2Dtlgn batch (16384 points, SIREN 4x128: pressure Laplacian jet, velocity
divergence) and on a 32768-point shard of elasticity3Dbunny (SIREN 5x256 Jacobian jet, the
two-kernel W = 256 backward), including the parameter gradients of a loss of each.
Tolerance (north_star): 1e-5 relative, normwise per tensor (max |hip - ref| / max |ref|)."""
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-5


def nerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope="module")
def base():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base as B
    B._native.load()
    return B


def pair(B, din, dout, L, W, seed):
    torch.manual_seed(seed)
    ref = O.OracleSiren(din, dout, L, W)
    torch.manual_seed(seed)
    net = B.MLP(din, dout, L, W, nonlinearity="sine").cuda()
    return ref, net


def grads(net):
    return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1).cpu()
                      for p in net.parameters()])


def test_fluid2dtlgn_pressure_full_batch(base):
    """fluid/model.py:110-125 at 128^2 points: lap p, and d/dtheta mean((g - lap p)^2)."""
    ref, net = pair(base, 2, 1, 4, 128, 11)
    torch.manual_seed(5)
    x = torch.rand(16384, 2) * 2 - 1
    g = torch.randn(16384, 1)
    xr = x.clone().requires_grad_(True)
    lr_ = O.op_laplace(ref(xr), xr)
    ((g - lr_) ** 2).mean().backward()
    xg = x.cuda().requires_grad_(True)
    lg = base.laplace(net(xg), xg)
    ((g.cuda() - lg) ** 2).mean().backward()
    assert nerr(lg, lr_) < TOL
    assert nerr(grads(net), grads(ref)) < TOL


def test_fluid2dtlgn_velocity_divergence_full_batch(base):
    ref, net = pair(base, 2, 2, 4, 128, 12)
    x = torch.rand(16384, 2, generator=torch.Generator().manual_seed(6)) * 2 - 1
    xr = x.clone().requires_grad_(True)
    dr = O.op_divergence(ref(xr), xr)
    xg = x.cuda().requires_grad_(True)
    with torch.no_grad():
        dg = base.divergence(net(xg), xg)
    assert nerr(dg, dr) < TOL


def test_elasticity3d_jacobian_shard(base):
    """elasticity/model.py:137-147 on a 32768-point shard (8-GPU strong scaling of 64^3):
    J of q = f(x) + x and the parameter gradient of sum(J^2) (W = 256 two-kernel backward)."""
    ref, net = pair(base, 3, 3, 5, 256, 13)
    x = torch.rand(32768, 3, generator=torch.Generator().manual_seed(7)) * 2 - 1
    xr = x.clone().requires_grad_(True)
    Jr, _ = O.op_jacobian(ref(xr) + xr, xr)
    (Jr ** 2).sum().backward()
    xg = x.cuda().requires_grad_(True)
    Jg, st = base.jacobian(net(xg) + xg, xg)
    (Jg ** 2).sum().backward()
    assert st == 0
    assert nerr(Jg, Jr) < TOL
    assert nerr(grads(net), grads(ref)) < TOL
