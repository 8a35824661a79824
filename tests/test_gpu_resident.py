"""The resident-dW backward (csrc/jet_x6r.hpp, insr_jet_bwd_path == 2): one persistent launch
holding every hidden layer's weight gradient in registers across the batch, then the
fixed-order partial sums.  Forced with the INSR_JET_POLICY(3) mode bits over batch sizes from one
point (one block) to 65,536 (16 tiles per block), ragged tails, value / gradient / Laplacian
jets of the fluid nets (4 hidden layers), against the CPU oracle (base/diff_ops.py:44-82 and
loss.backward(), base/baseModel.py:73-78).  Tolerance 1e-5 normwise per parameter tensor.
Also: bit-for-bit determinism, gradient accumulation (accumulate=1) and that the default
policy routes only the fluid2DtlgnM-sized batches here (slower at the headline's 16K)."""
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


@pytest.fixture
def resident(B):
    with B._native.knobs(policy=3):
        yield B._native.lib()


def nerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def pair(B, din, dout, L, W, seed):
    torch.manual_seed(seed)
    ref = O.OracleSiren(din, dout, L, W)
    torch.manual_seed(seed)
    net = B.MLP(din, dout, L, W, nonlinearity="sine").cuda()
    return ref, net


def check_grads(ref, net, what):
    for (k, a), b in zip(ref.named_parameters(), net.parameters()):
        ga = a.grad if a.grad is not None else torch.zeros_like(a)
        gb = b.grad if b.grad is not None else torch.zeros_like(b)
        if ga.abs().max() > 0:
            assert nerr(gb, ga) < TOL, (what, k, nerr(gb, ga))
        else:
            assert gb.abs().max() == 0, (what, k)


def run(B, ref, net, x, mode, seed):
    """A random functional of the mode's outputs, backward on both sides."""
    g = torch.Generator().manual_seed(seed)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    xg = x.cuda().requires_grad_(True)
    y = net(xg)
    R = torch.randn(yr.shape, generator=g)
    if mode == "value":
        outs_r, outs_g = [yr], [y]
    elif mode == "grad":
        outs_r, outs_g = [yr, O.op_jacobian(yr, xr)[0]], [y, B.jacobian(y, xg)[0]]
    else:
        outs_r, outs_g = [yr, O.op_laplace(yr, xr), O.op_gradient(yr, xr)], \
            [y, *B.laplace(y, xg, return_grad=True)]
    loss_r, loss_g = 0, 0
    for a, b in zip(outs_r, outs_g):
        Rk = torch.randn(a.shape, generator=g)
        loss_r = loss_r + (a * Rk).sum()
        loss_g = loss_g + (b * Rk.cuda()).sum()
    loss_r.backward()
    loss_g.backward()
    for a, b in zip(outs_r, outs_g):
        assert nerr(b, a) < TOL
    del R


CASES = [  # (mode, d_in, d_out, L): the kernel is compiled for the fluid nets' 4 hidden layers
    ("lap", 2, 1, 4), ("value", 2, 2, 4), ("value", 2, 1, 4), ("grad", 2, 2, 4), ("lap", 2, 2, 4),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-{c[1]}to{c[2]}-L{c[3]}")
@pytest.mark.parametrize("n", [1, 17, 300, 4103, 16708])
def test_resident_matches_oracle(B, resident, case, n):
    mode, din, dout, L = case
    m = {"value": B._native.MODE_VALUE, "grad": B._native.MODE_GRAD, "lap": B._native.MODE_LAP}[mode]
    assert resident.insr_jet_bwd_path(n, din, dout, L, 128, m | B._native.scope_bits()) == 2
    ref, net = pair(B, din, dout, L, 128, 100 + n % 97 + L)
    x = torch.rand(n, din, generator=torch.Generator().manual_seed(n)) * 2 - 1
    run(B, ref, net, x, mode, n + 1)
    check_grads(ref, net, (case, n))


@pytest.mark.parametrize("mode", ["value", "lap"])
def test_resident_65536_and_deterministic(B, resident, mode):
    """65,536 points (16 tiles per block): oracle parity, and the same gradients bit for bit
    on a second run (fixed summation order everywhere)."""
    ref, net = pair(B, 2, 1 if mode == "lap" else 2, 4, 128, 7)
    x = torch.rand(65536, 2, generator=torch.Generator().manual_seed(3)) * 2 - 1
    run(B, ref, net, x, mode, 5)
    check_grads(ref, net, mode)
    g1 = torch.cat([p.grad.reshape(-1) for p in net.parameters() if p.grad is not None]).clone()
    net.zero_grad(set_to_none=True)
    xg = x.cuda().requires_grad_(True)
    y = net(xg)
    gen = torch.Generator().manual_seed(5)
    torch.randn(y.shape, generator=gen)
    loss = 0
    outs = [y] if mode == "value" else [y, *B.laplace(y, xg, return_grad=True)]
    for o in outs:
        loss = loss + (o * torch.randn(o.shape, generator=gen).cuda()).sum()
    loss.backward()
    g2 = torch.cat([p.grad.reshape(-1) for p in net.parameters() if p.grad is not None])
    assert torch.equal(g1, g2)


def test_resident_accumulates(B, resident):
    """Two jets of one net before one optimiser step: the second backward adds into .grad
    (accumulate = 1 in the fixed-order sums)."""
    ref, net = pair(B, 2, 2, 4, 128, 11)
    xa = torch.rand(5000, 2, generator=torch.Generator().manual_seed(1)) * 2 - 1
    xb = torch.rand(7000, 2, generator=torch.Generator().manual_seed(2)) * 2 - 1
    Ra, Rb = torch.randn(5000, 2), torch.randn(7000, 2)
    ((ref(xa) * Ra).sum() + (ref(xb) * Rb).sum()).backward()
    (net(xa.cuda()) * Ra.cuda()).sum().backward()
    (net(xb.cuda()) * Rb.cuda()).sum().backward()
    check_grads(ref, net, "accumulate")


def test_default_routing(B):
    """Auto policy: the fluid nets' Laplacian backward at the headline batch (16,384 interior +
    324 band points) runs the two-kernel path, value backwards the fused kernel; at the fluid2DtlgnM
    batch (65,536 + 1,308 band points) the value backward runs resident and the Laplacian one the
    two-kernel path while its products run f16x3 (resident with bf16x6 products); the recompute
    path (3) only when forced (policy 4)."""
    lib = B._native.lib()
    nat = B._native
    assert lib.insr_jet_bwd_path(16708, 2, 1, 4, 128, nat.MODE_LAP) == 2    # the f16x3 saved-stream kernel
    assert lib.insr_jet_bwd_path(16708, 2, 2, 4, 128, nat.MODE_VALUE) == 0
    assert lib.insr_jet_bwd_path(1024, 2, 2, 4, 128, nat.MODE_VALUE) == 0
    assert lib.insr_jet_bwd_path(66844, 2, 1, 4, 128, nat.MODE_LAP) == 2    # fluid2DtlgnM batch
    assert lib.insr_jet_bwd_path(66844, 2, 1, 4, 128, nat.MODE_LAP | nat.jet_bwd_f16(0)) == 2
    assert lib.insr_jet_bwd_path(66844, 2, 2, 4, 128, nat.MODE_VALUE) == 2
    # 5 hidden layers (el2D's Jacobian): the saved-stream resident sweep since round 6 (jet_fb.hpp, kernel 1)
    assert lib.insr_jet_bwd_path(20400, 2, 2, 5, 128, nat.MODE_GRAD) == 2
    assert lib.insr_jet_bwd_kernel(20400, 2, 2, 5, 128, nat.MODE_GRAD) == 1
    assert lib.insr_jet_bwd_path(20400, 2, 2, 5, 128, nat.MODE_VALUE) not in (2, 3)
