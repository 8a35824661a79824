"""The reference-semantics route of base/diff_ops.py (graphs the jet matcher does not fuse): its jet
restatement base._jet.torch_jet, evaluated on the CPU (plain torch ops, no kernel call), against the
oracle's autograd derivatives of the reference network (oracle/siren_oracle.py, pinned to the
reference's golden vectors) -- values, derivatives and the parameter gradients of a functional of
them, to 1e-5 normwise (the north_star's fp32 tolerance).  The GPU side: tests/test_gpu_fallback.py."""
import pytest
import torch

from oracle import siren_oracle as O


@pytest.fixture(scope="module")
def B():
    import base
    return base


def _nw(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("shape", [(1, 1, 3, 64), (2, 1, 4, 128), (2, 2, 4, 128), (3, 3, 2, 40), (2, 3, 1, 20)])
@pytest.mark.parametrize("mode", ["value", "grad", "lap"])
def test_torch_jet_matches_oracle(B, shape, mode):
    from base import _native as nat
    din, dout, L, W = shape
    torch.manual_seed(11)
    ref = O.OracleSiren(din, dout, L, W)
    torch.manual_seed(11)
    net = B.MLP(din, dout, L, W, nonlinearity="sine")
    x = torch.rand(97, din) * 2 - 1
    xr = x.clone().requires_grad_(True)
    xs = x.clone().requires_grad_(True)
    m = {"value": nat.MODE_VALUE, "grad": nat.MODE_GRAD, "lap": nat.MODE_LAP}[mode]
    y, dy, lap = B._jet.torch_jet(net, xs, m)
    yr = ref(xr)
    assert _nw(y.detach(), yr.detach()) < 1e-5
    w = torch.randn(97, dout)
    loss_r = (w * yr).sum()
    loss_s = (w * y).sum()
    if mode != "value":
        Jr = torch.stack([O.op_gradient(yr[:, c:c + 1], xr) for c in range(dout)], dim=1)
        assert dy.shape == (97, dout, din) and _nw(dy.detach(), Jr.detach()) < 1e-5
        wj = torch.randn(97, dout, din)
        loss_r = loss_r + (wj * Jr).sum()
        loss_s = loss_s + (wj * dy).sum()
    if mode == "lap":
        Lr = torch.cat([O.op_laplace(yr[:, c:c + 1], xr) for c in range(dout)], dim=1)
        assert _nw(lap.detach(), Lr.detach()) < 1e-5
        wl = torch.randn(97, dout)
        loss_r = loss_r + (wl * Lr).sum()
        loss_s = loss_s + (wl * lap).sum()
    loss_r.backward()
    loss_s.backward()
    for (n, p), q in zip(net.named_parameters(), ref.parameters()):
        if q.grad is None:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, n
            continue
        assert _nw(p.grad, q.grad) < 1e-5, n
    assert _nw(xs.grad, xr.grad) < 1e-5  # derivatives reach x through the jet's own graph


def test_reference_route_helpers_match_oracle_ops():
    """_ref_divergence / _ref_jacobian_rows / _ref_hessian restate base/diff_ops.py:6-82: on a plain torch
    function they equal the oracle's operators."""
    from base import diff_ops as D
    x = (torch.rand(33, 3) * 2 - 1).requires_grad_(True)
    A = torch.randn(3, 3)
    y = torch.sin(x @ A) * x.sum(-1, keepdim=True)
    assert torch.allclose(D._ref_divergence(y, x), O.op_divergence(y, x), atol=1e-6)
    J = D._ref_jacobian_rows(y, x)
    Jr, _ = O.op_jacobian(y, x)
    assert torch.allclose(J, Jr, atol=1e-6)
    xm = x.detach().unsqueeze(0).requires_grad_(True)  # (meta, obs, dim), as the reference's hessian takes
    ym = torch.sin(xm @ A) * xm.sum(-1, keepdim=True)
    H = D._ref_hessian(ym, xm)
    Hr, _ = O.op_hessian(ym, xm)
    assert torch.allclose(H, Hr, atol=1e-5)
