"""HIP jet kernels vs the CPU oracle (tests/…/oracle pinned to the reference).

Tolerance (north_star: "within 1e-5 relative fp32"): normwise per tensor,
    max|hip - oracle| <= 1e-5 * max|oracle|,
for every field value and every parameter-gradient tensor.  SURVEY.md §8(c)
measured the reference's own fp32 error at ~1e-6 normwise, so pointwise
relative error near zeros is not a meaningful criterion.
"""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-5

NETS = {  # name: (d_in, d_out, L, W)
    "advect": (1, 1, 3, 64),
    "fluid_vel": (2, 2, 4, 128),
    "fluid_pres": (2, 1, 4, 128),
    "el2d": (2, 2, 5, 128),
    "small32": (2, 3, 2, 32),
    "el3d_w64": (3, 3, 3, 64),
    "el3d": (3, 3, 5, 256),          # elasticity3D bunny: width 256
    "w256_lap": (2, 1, 2, 256),      # width 256 with the 4-stream Laplacian jet
    # paper-script widths, zero-padded to the next compiled width (base/networks.py MLP):
    "advect_w20": (1, 1, 2, 20),     # scripts/advect1D.sh:4-5 (2 x 20)
    "el2d_w68": (2, 2, 3, 68),       # scripts/elasticity2Dstretch.sh:3-4 (3 x 68)
    "el3d_w66": (3, 3, 3, 66),       # scripts/elasticity3Dbunny.sh:3-4 (3 x 66)
}


F32, X6 = 0, 1  # matrix-core precision of the tile-split kernels (INSR_JET_PREC mode bits)
VARIANTS = {  # (fwd, bwd) forced tiles per block, (fwd, bwd) precision[, smallest width of the two-kernel backward]
    "split": ((1, 1), (F32, F32)),           # exact-fp32 MFMA, neurons split over a block's waves, 1 tile/block
    "split_t2": ((2, 2), (F32, F32)),        # 2 tiles per block (ragged last block)
    "split_t4": ((4, 4), (F32, F32)),        # 4 tiles per block (capped by LDS / registers)
    "x6": ((1, 1), (X6, X6)),                # split-bf16 (6-product) matrix cores (the default precision)
    "x6_t2": ((2, 2), (X6, X6)),
    "x6_t4": ((4, 4), (X6, X6)),
    "x6_fwd_f32_bwd": ((4, 2), (X6, F32)),   # precisions mix: same saved layout
    "f32_fwd_x6_bwd": ((2, 4), (F32, X6)),
    "x6_auto": ((0, 0), (X6, X6)),           # the default tile policy
    "x6_wide128": ((0, 0), (X6, X6), 128),   # two-kernel backward (prop + dW GEMM) from W = 128
}


@pytest.fixture(scope="module", params=list(VARIANTS))
def base(request):
    """Every test runs for each kernel-variant combination."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base as B
    B._native.load()
    tiles, prec = VARIANTS[request.param][:2]
    wide = VARIANTS[request.param][2] if len(VARIANTS[request.param]) > 2 else 256
    # the variant's knobs ride in every jet call's mode (INSR_JET_TILES / INSR_JET_PREC / WIDE128)
    with B._native.knobs(tiles=tiles, prec=prec, wide128=wide == 128):
        yield B


def nerr(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def pair(base, name, seed=0):
    din, dout, L, W = NETS[name]
    torch.manual_seed(seed)
    ref = O.OracleSiren(din, dout, L, W)
    torch.manual_seed(seed)
    net = base.MLP(din, dout, L, W, nonlinearity="sine")
    # same seed, same RNG order -> identical weights (init parity)
    for a, b in zip(ref.parameters(), net.parameters()):
        assert torch.equal(a.detach(), b.detach())
    return ref, net.cuda()


def param_errs(ref, net):
    out = []
    for (k, a), b in zip(ref.named_parameters(), net.parameters()):
        ga = a.grad if a.grad is not None else torch.zeros_like(a)
        gb = b.grad if b.grad is not None else torch.zeros_like(b)
        out.append((k, nerr(gb, ga)))
    return out


@pytest.mark.parametrize("name", list(NETS))
@pytest.mark.parametrize("n", [1000, 64])
def test_value_and_value_grad(base, name, n):
    ref, net = pair(base, name, seed=3)
    din = NETS[name][0]
    x = torch.rand(n, din, generator=torch.Generator().manual_seed(7)) * 2 - 1
    y_ref = ref(x)
    xg = x.cuda()
    y = net(xg)
    assert nerr(y, y_ref) < TOL
    R = torch.randn(y_ref.shape, generator=torch.Generator().manual_seed(8))
    (y_ref * R).sum().backward()
    (y * R.cuda()).sum().backward()
    for k, e in param_errs(ref, net):
        assert e < TOL, (k, e)


def _ops(mod, y, x):
    ops = {"gradient": lambda: mod.gradient(y, x), "jacobian": lambda: mod.jacobian(y, x)[0],
           "laplace": lambda: mod.laplace(y, x)}
    if y.shape[-1] <= x.shape[-1]:
        ops["divergence"] = lambda: mod.divergence(y, x)
    return ops


ORACLE_OPS = {"gradient": O.op_gradient, "jacobian": lambda y, x: O.op_jacobian(y, x)[0],
              "laplace": O.op_laplace, "divergence": O.op_divergence}


@pytest.mark.parametrize("name", list(NETS))
@pytest.mark.parametrize("op", ["gradient", "jacobian", "laplace", "divergence"])
def test_diff_op_and_param_grad(base, name, op):
    din, dout, L, W = NETS[name]
    if op == "laplace" and din > 2 and not base._native.lib().insr_siren_supported(din, dout, L, W, 2 | base._native.scope_bits()):
        pytest.skip("5-stream Laplacian jet at width 256: split-bf16 kernels only (fp32 backward exceeds LDS)")
    if op == "divergence" and dout > din:
        pytest.skip("divergence needs d_out <= d_in")
    ref, net = pair(base, name, seed=5)
    n = 777
    x = torch.rand(n, din, generator=torch.Generator().manual_seed(11)) * 2 - 1
    xr = x.clone().requires_grad_(True)
    v_ref = ORACLE_OPS[op](ref(xr), xr)
    xg = x.cuda().requires_grad_(True)
    v = _ops(base, net(xg), xg)[op]()
    assert v.shape == v_ref.shape
    assert nerr(v, v_ref) < TOL, op
    R = torch.randn(v_ref.shape, generator=torch.Generator().manual_seed(12))
    (v_ref * R).sum().backward()
    (v * R.cuda()).sum().backward()
    for k, e in param_errs(ref, net):
        assert e < TOL, (op, k, e)


def test_affine_jacobian_and_accumulation(base):
    """q = f(x) + x (elasticity/model.py:137) and grads accumulated over several jets."""
    ref, net = pair(base, "el2d", seed=9)
    x = torch.rand(500, 2, generator=torch.Generator().manual_seed(1)) * 2 - 1
    xr = x.clone().requires_grad_(True)
    qr = ref(xr) + xr
    Jr, st = O.op_jacobian(qr, xr)
    lr_ = (Jr ** 2).sum() + (qr ** 2).sum() + O.op_divergence(qr, xr).sum()
    lr_.backward()
    xg = x.cuda().requires_grad_(True)
    q = net(xg) + xg
    J, st2 = base.jacobian(q, xg)
    assert st2 == st == 0
    assert nerr(J, Jr) < TOL
    lg = (J ** 2).sum() + (q ** 2).sum() + base.divergence(q, xg).sum()
    assert abs(float(lg) - float(lr_)) <= TOL * abs(float(lr_))
    lg.backward()
    for k, e in param_errs(ref, net):
        assert e < TOL, (k, e)


def test_empty_and_tiny_batches(base):
    """Single points make "normwise" pointwise, where even the reference's own fp32
    Laplacian deviates from fp64 by up to ~1e-2 (cancellation in w^2 s sum t_i^2).
    So here the judge is fp64: the HIP error must stay within the reference-fp32
    error band (3x its error, or 1e-5 of the value, whichever is larger)."""
    ref, net = pair(base, "fluid_pres", seed=2)
    ref64 = O.OracleSiren(2, 1, 4, 128).double()
    ref64.load_state_dict({k: v.double() for k, v in ref.state_dict().items()})
    for n in (1, 15, 17, 65):
        x = torch.rand(n, 2, generator=torch.Generator().manual_seed(n)) * 2 - 1
        xr = x.clone().requires_grad_(True)
        x64 = x.double().requires_grad_(True)
        xg = x.cuda().requires_grad_(True)
        l64 = O.op_laplace(ref64(x64), x64).detach()
        e_ref = (O.op_laplace(ref(xr), xr).detach().double() - l64).abs()
        e_hip = (base.laplace(net(xg), xg).detach().cpu().double() - l64).abs()
        bound = torch.maximum(3 * e_ref, 1e-5 * l64.abs().max().expand_as(l64))
        assert bool((e_hip <= bound).all()), (n, e_hip.max().item(), e_ref.max().item())
    y = net(torch.zeros(0, 2, device="cuda"))
    assert y.shape == (0, 1)


def test_no_grad_jets_skip_saving(base):
    _, net = pair(base, "fluid_vel", seed=4)
    x = (torch.rand(300, 2) * 2 - 1).cuda().requires_grad_(True)
    with torch.no_grad():
        y = net(x)
    assert not y.requires_grad
    d = base.divergence(net(x), x).detach()
    assert torch.isfinite(d).all()


@pytest.mark.parametrize("op", ["value", "laplace", "divergence"])
def test_large_batch_default_policy(base, op):
    """Batches large enough for the automatic multi-tile choice (T = 2 / 4)."""
    with base._native.knobs(tiles=(0, 0)):
        name = "fluid_pres" if op != "divergence" else "fluid_vel"
        din = NETS[name][0]
        ref, net = pair(base, name, seed=6)
        n = 20000
        x = torch.rand(n, din, generator=torch.Generator().manual_seed(13)) * 2 - 1
        xr = x.clone().requires_grad_(True)
        xg = x.cuda().requires_grad_(True)
        if op == "value":
            v_ref, v = ref(xr), net(xg)
        else:
            v_ref, v = ORACLE_OPS[op](ref(xr), xr), _ops(base, net(xg), xg)[op]()
        assert nerr(v, v_ref) < TOL
        R = torch.randn(v_ref.shape, generator=torch.Generator().manual_seed(14))
        (v_ref * R).sum().backward()
        (v * R.cuda()).sum().backward()
        for k, e in param_errs(ref, net):
            assert e < TOL, (op, k, e)


@pytest.mark.parametrize("name", ["advect_w20", "el2d_w68", "el3d_w66"])
def test_padded_width_adam_keeps_padding_zero(base, name):
    """A padded net trains like the reference's: the padding's gradient is exactly 0, so
    Adam (FusedAdam on the flat buffer) leaves it at 0 and the real parameters match the
    oracle's torch Adam after 3 steps."""
    din, dout, L, W = NETS[name]
    ref, net = pair(base, name, seed=21)
    opt_r = O.OracleAdam(list(ref.parameters()), lr=1e-3)
    opt = base.FusedAdam([{"params": list(net.parameters()), "lr": 1e-3, "module": net}])
    for it in range(3):
        x = torch.rand(300, din, generator=torch.Generator().manual_seed(30 + it)) * 2 - 1
        xr = x.clone().requires_grad_(True)
        xg = x.cuda().requires_grad_(True)
        for p in ref.parameters():
            p.grad = None
        (O.op_jacobian(ref(xr), xr)[0] ** 2).sum().backward()
        opt_r.step()
        opt.zero_grad()
        (base.jacobian(net(xg), xg)[0] ** 2).sum().backward()
        g = net.flat_grad_buffer()
        opt.step()
    flat = net.flat_params().detach().cpu()
    mask = torch.zeros_like(flat, dtype=torch.bool)
    for p, e in zip(net.parameters(), net._layout()):
        net._view(mask, e).fill_(True)
    assert bool((flat[~mask] == 0).all())
    assert bool((g.detach().cpu()[~mask] == 0).all())
    for a, b in zip(ref.parameters(), net.parameters()):
        assert float((a.detach() - b.detach().cpu()).abs().max()) <= 1e-6 + 1e-5 * float(a.detach().abs().max())
