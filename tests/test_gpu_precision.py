"""Jet precisions (MLP(precision=...), per-call precision bits of the jet mode) vs the CPU
oracle.  The fp32 parity configs run at the library default -- f16x3 products in every forward and
(through the backward's fp16 product mask, INSR_JET_BWD_F16 = 7, and the resident f16x3 Laplacian
sweep) in the backwards, the bf16x6 contract where a kernel has no fp16 products (test_gpu_parity.py,
1e-5).  Each precision below is held to the normwise tolerance (max |hip - oracle| / max |oracle|, per
tensor) it is documented with in DESIGN.md:

    f16x3   2^k-scaled operands in two fp16 terms, 3 products (the default)   1e-5
            (measured fields <= 4.2e-6, gradients <= 5.1e-6, profiles/r03/prec_f16x3.jsonl; the
            round-5 defaults as the bench runs them: profiles/r05/prec_defaults.jsonl, <= 3.5e-6)
    bf16x6  6 bf16 products per fp32 product (opt-in)     1e-5   (measured <= 5e-6)
    bf16x3  3 products (hi*hi + hi*lo + lo*hi)             5e-5   (measured <= 3.3e-5)
    bf16    1 product, fp32 accumulation                   2.5e-2 (measured <= 1.6e-2)
    mixed   bf16x3 forwards / bf16 backwards              1e-2   (measured: fields <= 2.1e-5,
            parameter gradients <= 5.6e-3; BASELINE configs[4] "mixed fp32/bf16 MFMA",
            SURVEY §8(c) <= 1e-2; profiles/r03/prec_pairs.jsonl)

'measured' = profiles/r02/prec_errors_all_precisions.jsonl (tools/prec_errors.py, 4000
points, every net and op).  The bf16 bound is set by the SIREN's first-layer frequency
(omega = 30 multiplies the bf16 rounding of every pre-activation), so it is a property of the
format, not of a kernel; the fp32 line of bench.py stays the parity config and bf16 is a
separate bench line (bench.py --precision bf16).
"""
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu

TOLS = {"bf16x6": 1e-5, "f16x3": 1e-5, "bf16x3": 5e-5, "bf16": 2.5e-2, "mixed": 1e-2}


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


def pair(B, din, dout, L, W, seed, precision):
    torch.manual_seed(seed)
    ref = O.OracleSiren(din, dout, L, W)
    torch.manual_seed(seed)
    net = B.MLP(din, dout, L, W, nonlinearity="sine", precision=precision).cuda()
    return ref, net


def grads(net):
    return [(p.grad if p.grad is not None else torch.zeros_like(p)).detach() for p in net.parameters()]


def check_grads(ref, net, tol):
    for (k, a), b in zip(ref.named_parameters(), grads(net)):
        ga = a.grad if a.grad is not None else torch.zeros_like(a)
        if ga.abs().max() > 0:
            assert nerr(b, ga) < tol, (k, nerr(b, ga))


NETS = {"fluid_vel": (2, 2, 4, 128), "fluid_pres": (2, 1, 4, 128), "advect": (1, 1, 3, 64), "el3d_w64": (3, 3, 3, 64)}
OPS = {"value": lambda B, y, x: y, "gradient": lambda B, y, x: B.gradient(y, x),
       "laplace": lambda B, y, x: B.laplace(y, x)}
ORACLE = {"value": lambda y, x: y, "gradient": O.op_gradient, "laplace": O.op_laplace}


@pytest.mark.parametrize("precision", list(TOLS))
@pytest.mark.parametrize("name", list(NETS))
@pytest.mark.parametrize("op", list(OPS))
def test_precision_jet_and_param_grads(base, precision, name, op):
    din, dout, L, W = NETS[name]
    if op == "laplace" and din > 2:
        pytest.skip("Laplacian jet compiled for d_in <= 2")
    ref, net = pair(base, din, dout, L, W, 41, precision)
    x = torch.rand(2000, din, generator=torch.Generator().manual_seed(42)) * 2 - 1
    xr = x.clone().requires_grad_(True)
    vr = ORACLE[op](ref(xr), xr)
    xg = x.cuda().requires_grad_(True)
    v = OPS[op](base, net(xg), xg)
    tol = TOLS[precision]
    assert nerr(v, vr) < tol
    R = torch.randn(vr.shape, generator=torch.Generator().manual_seed(43))
    (vr * R).sum().backward()
    (v * R.cuda()).sum().backward()
    check_grads(ref, net, tol)


@pytest.mark.parametrize("precision", ["bf16", "bf16x3", "mixed", "f16x3", "bf16x6"])
def test_fluid2dtlgnM_reduced_precision_65536(base, precision):
    """The fluid2DtlgnM bench line's networks at their precision (bench.py --config
    fluid2DtlgnM --precision ...): the pressure Laplacian jet (two-kernel backward at 65,536
    points) and the velocity divergence, with the parameter gradients of the pressure loss.
    The oracle runs in fp64: at this size the fp32 oracle's own summation error reaches the
    1e-5 bound on the output-layer gradient (measured: bf16x6 and f16x3 both 1.10e-5 against
    the fp32 oracle, gpurun_out r3i), so it would test the oracle, not the kernels."""
    tol = TOLS[precision]
    ref, net = pair(base, 2, 1, 4, 128, 51, precision)
    ref = ref.double()
    torch.manual_seed(52)
    x = torch.rand(65536, 2) * 2 - 1
    g = torch.randn(65536, 1)
    xr = x.clone().double().requires_grad_(True)
    lr_ = O.op_laplace(ref(xr), xr)
    ((g.double() - lr_) ** 2).mean().backward()
    xg = x.cuda().requires_grad_(True)
    lg = base.laplace(net(xg), xg)
    ((g.cuda() - lg) ** 2).mean().backward()
    assert nerr(lg, lr_) < tol
    check_grads(ref, net, tol)
    refv, vel = pair(base, 2, 2, 4, 128, 53, precision)
    refv = refv.double()
    xr = x.clone().double().requires_grad_(True)
    dr = O.op_divergence(refv(xr), xr)
    with torch.no_grad():
        dg = base.divergence(vel(xg), xg)
    assert nerr(dg, dr) < tol


def test_precision_is_per_network(base):
    """Two networks of one process at different precisions: the per-call bits, not the
    process-wide default, select the kernels (the bf16 net's error is bf16-sized, the
    default net's stays fp32-level)."""
    x = torch.rand(3000, 2, generator=torch.Generator().manual_seed(61)) * 2 - 1
    errs = {}
    for prec in ("bf16", None):
        ref, net = pair(base, 2, 1, 4, 128, 62, prec)
        xr = x.clone().requires_grad_(True)
        xg = x.cuda().requires_grad_(True)
        errs[prec] = nerr(base.laplace(net(xg), xg), O.op_laplace(ref(xr), xr))
    assert errs[None] < 1e-5
    assert 1e-4 < errs["bf16"] < TOLS["bf16"]
