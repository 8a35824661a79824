"""The reference-semantics route of base/diff_ops.py on the GPU: derivatives of graphs the jet
matcher does not fuse (a post-processed network output, a weighted gradient, d_in = 3 Hessians)
go through torch.autograd.grad(create_graph=True) as the reference's do (base/diff_ops.py:6-82);
the HIP jet nodes inside such a graph differentiate themselves with torch ops on the device
(base/_jet.py torch_jet).  Checked against the oracle (oracle/siren_oracle.py, pinned to the
reference's golden vectors): every returned field and every parameter gradient of a loss built
from it, 1e-5 normwise (the north_star's fp32 tolerance), and the loss backward still runs the HIP
reverse jets for the fused parts of the same graph."""
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
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def pair(B, shape, seed=0):
    din, dout, L, W = shape
    torch.manual_seed(seed)
    ref = O.OracleSiren(din, dout, L, W)
    torch.manual_seed(seed)
    net = B.MLP(din, dout, L, W, nonlinearity="sine").cuda()
    return ref, net


def check_grads(ref, net):
    for (k, a), b in zip(ref.named_parameters(), net.parameters()):
        ga = a.grad if a.grad is not None else torch.zeros_like(a)
        gb = b.grad if b.grad is not None else torch.zeros_like(b)
        if float(ga.abs().max()) == 0.0:
            assert float(gb.abs().max()) == 0.0, k
            continue
        assert nerr(gb, ga) < TOL, (k, nerr(gb, ga))


def points(n, din, seed=3):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(n, din, generator=g) * 2 - 1


CASES = {
    # name: (network shape, op on (D, y-builder, x) -> field)
    "gradient_of_2net": ((2, 1, 4, 128), lambda D, f, x: D.gradient(2.0 * f(x), x)),
    "laplace_of_2net": ((2, 1, 4, 128), lambda D, f, x: D.laplace(2.0 * f(x), x)),
    "gradient_of_sq_slice": ((2, 2, 4, 128), lambda D, f, x: D.gradient(f(x)[..., :1] ** 2, x)),
    "divergence_of_sq": ((2, 2, 3, 64), lambda D, f, x: D.divergence(f(x) ** 2, x)),
    "jacobian_of_sin": ((2, 2, 3, 64), lambda D, f, x: D.jacobian(torch.sin(f(x)), x)[0]),
    "weighted_gradient_divergence": ((2, 1, 4, 128),
                                     lambda D, f, x: D.divergence((1.0 + x ** 2) * D.gradient(f(x), x), x)),
    "gradient_go_divergence": ((2, 2, 3, 64),
                               lambda D, f, x: D.divergence(D.gradient(f(x), x, grad_outputs=x.detach() + 2.0), x)),
    # eps = 1: the normalised field divides by |grad f| + eps; a small eps makes the op ill-conditioned
    # where |grad f| -> 0 (the fp32 oracle itself then drifts from fp64 by more than 1e-5)
    "laplace_normalized_d3": ((3, 1, 3, 64), lambda D, f, x: D.laplace(f(x), x, normalize=True, eps=1.0)),
    # (meta, obs, dim) input as the reference's hessian takes; the network sees the 3-d batch
    "hessian_d3": ((3, 2, 2, 64), lambda D, f, x: (lambda xm: D.hessian(f(xm), xm)[0])(x.unsqueeze(0))),
}


def _oracle_op(name, f, x):
    """The same expression with the reference's own operators (oracle restatement of base/diff_ops.py)."""
    if name == "gradient_of_2net":
        return O.op_gradient(2.0 * f(x), x)
    if name == "laplace_of_2net":
        return O.op_laplace(2.0 * f(x), x)
    if name == "gradient_of_sq_slice":
        return O.op_gradient(f(x)[..., :1] ** 2, x)
    if name == "divergence_of_sq":
        return O.op_divergence(f(x) ** 2, x)
    if name == "jacobian_of_sin":
        return O.op_jacobian(torch.sin(f(x)), x)[0]
    if name == "weighted_gradient_divergence":
        return O.op_divergence((1.0 + x ** 2) * O.op_gradient(f(x), x), x)
    if name == "gradient_go_divergence":
        return O.op_divergence(O.op_gradient(f(x), x, grad_outputs=x.detach() + 2.0), x)
    if name == "laplace_normalized_d3":
        g = O.op_gradient(f(x), x)
        g = g / (g.norm(dim=-1, keepdim=True) + 1.0)
        return O.op_divergence(g, x)
    if name == "hessian_d3":
        xm = x.unsqueeze(0)
        return O.op_hessian(f(xm), xm)[0]
    raise KeyError(name)


@pytest.mark.parametrize("name", list(CASES))
def test_unfused_graph_matches_oracle(B, name):
    shape, op = CASES[name]
    ref, net = pair(B, shape)
    x = points(300, shape[0])
    xr = x.clone().requires_grad_(True)
    xg = x.cuda().requires_grad_(True)
    before = dict(B.diff_ops.FALLBACKS)
    out = op(B, net, xg)
    out_r = _oracle_op(name, ref, xr)
    assert sum(B.diff_ops.FALLBACKS.values()) > sum(before.values())  # the reference route served it
    assert out.shape == out_r.shape
    assert nerr(out, out_r) < TOL, nerr(out, out_r)
    w = torch.randn(out_r.shape, generator=torch.Generator().manual_seed(5))
    (w * out_r).sum().backward()
    (w.cuda() * out).sum().backward()
    torch.cuda.synchronize()
    check_grads(ref, net)


def test_fused_and_unfused_terms_in_one_loss(B):
    """One loss mixing a fused Laplacian (HIP jets both ways) and an unfused gradient of 2 f: the
    parameter gradient is the sum of both routes' contributions (flat .grad folds torch's)."""
    ref, net = pair(B, (2, 1, 4, 128), seed=4)
    x = points(500, 2, seed=9)
    xr = x.clone().requires_grad_(True)
    xg = x.cuda().requires_grad_(True)
    lr_ = O.op_laplace(ref(xr), xr)
    gr = O.op_gradient(2.0 * ref(xr), xr)
    lg = B.laplace(net(xg), xg)
    gg = B.gradient(2.0 * net(xg), xg)
    assert nerr(lg, lr_) < TOL and nerr(gg, gr) < TOL
    ((lr_ ** 2).mean() + (gr ** 2).mean()).backward()
    ((lg ** 2).mean() + (gg ** 2).mean()).backward()
    torch.cuda.synchronize()
    check_grads(ref, net)


def test_fallback_keeps_the_training_step(B):
    """A model whose phase body differentiates a post-processed output still trains through
    BaseModel._update_network (loss.backward + fused Adam): one step equals the oracle's."""
    ref, net = pair(B, (2, 1, 3, 64), seed=6)
    x = points(256, 2, seed=2)
    xr = x.clone().requires_grad_(True)
    xg = x.cuda().requires_grad_(True)
    opt_r = O.OracleAdam(list(ref.parameters()), lr=1e-4)
    loss_r = (O.op_gradient(ref(xr) * 3.0, xr) ** 2).mean()
    loss_r.backward()
    opt_r.step()
    opt = B.FusedAdam([{"params": list(net.parameters()), "lr": 1e-4, "module": net}])
    opt.zero_grad()
    loss = (B.gradient(net(xg) * 3.0, xg) ** 2).mean()
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    assert abs(float(loss) - float(loss_r)) <= TOL * abs(float(loss_r))
    for a, b in zip(ref.parameters(), net.parameters()):
        assert float((a.detach() - b.detach().cpu()).abs().max()) <= 2.5e-4  # Adam's first step ~ lr sign(g)


@pytest.mark.parametrize("name", ["relu", "elu", "sine_nonlinear_out", "relu_nonlinear_out", "sine_w300"])
def test_other_networks_on_the_gpu(B, name):
    """relu / elu / outermost_linear=False / width-300 networks (no HIP jet serves them: TorchMLP) on the
    GPU against the reference's own outputs (tests/golden/ref_nets.npz)."""
    import os
    import numpy as np
    from tests.test_other_nets import GOLD, check_net
    with np.load(GOLD) as z:
        gold = {k: z[k] for k in z.files}
    check_net(B, gold, name, "cuda")
