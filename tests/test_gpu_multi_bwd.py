"""Batched reverse jets (base._jet.batched_backward, insr_siren_jet_bwd_grad_multi).

BaseModel._backward runs every iteration's loss backward inside a batched_backward scope: the
reverse jets of one network and jet mode -- a phase's interior batch and its wall bands from
separate network calls, as the reference's phase bodies make them (fluid/model.py:80,96-97,
:119-120, :139-148) -- launch together at the scope's exit, the fused-path jobs in ONE launch with
ONE fixed-order reduction.  Checked here: the batched gradients equal the job-by-job ones (only
the fp32 summation order differs) and the CPU oracle at the parity tolerance, for value, gradient
and Laplacian jobs, ragged and empty batches, a Laplacian interior that takes the two-kernel path
beside fused band jobs, more jobs than one launch holds, and a direct C-ABI call.
"""
import ctypes

import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-5       # parity tolerance (normwise per tensor, as tests/test_gpu_parity.py)
ORDER_TOL = 2e-6  # batched vs job by job: the same products, partial rows summed in another order


@pytest.fixture(scope="module")
def B():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    base._native.load()
    return base


def nerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def pair(B, din, dout, L, W, seed=0):
    torch.manual_seed(seed)
    ref = O.OracleSiren(din, dout, L, W)
    torch.manual_seed(seed)
    net = B.MLP(din, dout, L, W, nonlinearity="sine").cuda()
    return ref, net


def pts(n, d, seed):
    return torch.rand(n, d, generator=torch.Generator().manual_seed(seed)) * 2 - 1


def grads(net):
    return [p.grad.detach().clone() for p in net.parameters()]


def run(B, net, loss_fn, batched):
    net.zero_grad(set_to_none=True)
    loss = loss_fn()
    if batched:
        with B._jet.batched_backward():
            loss.backward()
    else:
        loss.backward()
    torch.cuda.synchronize()
    return grads(net)


def value_loss(mod, net, xs):
    """mean(u(x)^2) over the interior + one wall term per band (fluid/model.py:89,96-98 shape)."""
    tot = 0.
    for k, x in enumerate(xs):
        y = net(x)
        tot = tot + ((y if k == 0 else y[..., (k - 1) % y.shape[-1]]) ** 2).sum() / max(x.shape[0], 1)
    return tot


@pytest.mark.parametrize("sizes", [(16384, 162, 162), (4096, 81, 81, 1, 17), (777, 0, 64), (5, 5)])
def test_value_jobs_batched_equal_and_match_oracle(B, sizes):
    ref, net = pair(B, 2, 2, 4, 128, seed=1)
    xs = [pts(n, 2, 10 + k) for k, n in enumerate(sizes)]
    xg = [x.cuda().requires_grad_(True) for x in xs]
    g1 = run(B, net, lambda: value_loss(B, net, xg), batched=False)
    g2 = run(B, net, lambda: value_loss(B, net, xg), batched=True)
    for a, b in zip(g2, g1):
        assert nerr(a, b) < ORDER_TOL
    value_loss(O, ref, [x.requires_grad_(True) for x in xs]).backward()
    for (k, p), g in zip(ref.named_parameters(), g2):
        assert nerr(g, p.grad) < TOL, k


def test_lap_interior_two_kernel_beside_fused_band_gradients(B):
    """The pressure phase as the reference writes it (fluid/model.py:108-122): a Laplacian jet of
    the interior (16,384 points: the two-kernel path, alone) and gradient jets of two 162-point band
    pairs (fused, one launch) -- two jet modes, two groups."""
    ref, net = pair(B, 2, 1, 4, 128, seed=2)
    x, bx, by = pts(16384, 2, 1), pts(162, 2, 2), pts(162, 2, 3)
    div = torch.randn(16384, 1, generator=torch.Generator().manual_seed(4))

    def loss(mod, x, bx, by, dv):
        f, lap_op, grad_op = mod
        lap = lap_op(f(x), x)
        gx = grad_op(f(bx), bx)[..., 0]
        gy = grad_op(f(by), by)[..., 1]
        return torch.mean((dv - lap) ** 2) + torch.mean(gx ** 2) + torch.mean(gy ** 2)

    hip, orc = (net, B.laplace, B.gradient), (ref, O.op_laplace, O.op_gradient)
    xg = [t.cuda().requires_grad_(True) for t in (x, bx, by)]
    g1 = run(B, net, lambda: loss(hip, *xg, div.cuda()), batched=False)
    g2 = run(B, net, lambda: loss(hip, *xg, div.cuda()), batched=True)
    for a, b in zip(g2, g1):
        assert nerr(a, b) < ORDER_TOL
    loss(orc, *[t.requires_grad_(True) for t in (x, bx, by)], div).backward()
    for (k, p), g in zip(ref.named_parameters(), g2):
        ga = p.grad if p.grad is not None else torch.zeros_like(p)
        assert nerr(g, ga) < TOL, k


def test_lap_jobs_in_one_saved_stream_sweep(B):
    """Laplacian jets of one network on three point sets (an interior + two bands whose gradient streams
    the loss reads -- the plain pressure body once its band calls share the interior jet's mode) whose
    total takes the saved-stream resident sweep: ONE insr_siren_jet_bwd_multi_sweep launch + its sums,
    with and without the sums held back for the Adam launch; = job by job and = the oracle."""
    ref, net = pair(B, 2, 1, 4, 128, seed=12)
    x, bx, by = pts(16384, 2, 21), pts(162, 2, 22), pts(162, 2, 23)
    div = torch.randn(16384, 1, generator=torch.Generator().manual_seed(24))
    lib, nat = B._native.lib(), B._native
    mode = net.call_mode(nat.MODE_LAP)
    assert lib.insr_jet_bwd_kernel(16384 + 2 * 176, 2, 1, 4, 128, mode) == 1  # the sweep serves the total

    def loss_hip(x, bx, by, dv):
        lap = B.laplace(net(x), x)
        _, gbx = B.laplace(net(bx), bx, return_grad=True)
        _, gby = B.laplace(net(by), by, return_grad=True)
        return torch.mean((dv - lap) ** 2) + torch.mean(gbx[..., 0] ** 2) + torch.mean(gby[..., 1] ** 2)

    xg = [t.cuda().requires_grad_(True) for t in (x, bx, by)]
    g1 = run(B, net, lambda: loss_hip(*xg, div.cuda()), batched=False)
    g2 = run(B, net, lambda: loss_hip(*xg, div.cuda()), batched=True)
    for a, b in zip(g2, g1):
        assert nerr(a, b) < TOL
    net.zero_grad(set_to_none=True)
    with B._jet.defer_reductions():  # (its exit lands the held-back sums)
        with B._jet.batched_backward():
            loss_hip(*xg, div.cuda()).backward()
    torch.cuda.synchronize()
    g3 = grads(net)
    for a, b in zip(g3, g2):
        assert torch.equal(a, b)  # held back or not: the same sums
    lo = (lambda f, z: O.op_laplace(f(z), z))
    xs = [t.requires_grad_(True) for t in (x, bx, by)]
    l0 = torch.mean((div - lo(ref, xs[0])) ** 2) + torch.mean(O.op_gradient(ref(xs[1]), xs[1])[..., 0] ** 2) + \
        torch.mean(O.op_gradient(ref(xs[2]), xs[2])[..., 1] ** 2)
    l0.backward()
    for (k, p), g in zip(ref.named_parameters(), g2):
        ga = p.grad if p.grad is not None else torch.zeros_like(p)
        assert nerr(g, ga) < TOL, k


@pytest.mark.parametrize("policy", [2, 0])
@pytest.mark.parametrize("sizes", [(20000, 200, 200), (8192, 17, 1, 0)])
def test_grad_jobs_in_one_two_kernel_launch(B, sizes, policy):
    """The elasticity body as the reference writes it (elasticity/model.py:137,143,161-174): the Jacobian of
    q = f(x) + x on the interior and the positional constraints on two fixed bands from separate calls of ONE
    5 x 128 network, all gradient jets (the loop's deferred scope promotes the band calls), whose total takes
    the two-kernel backward: ONE insr_siren_jet_bwd_multi_sweep (one propagation + one dW launch over a job
    table, round 6) + its sums, held back for the Adam launch or not; = job by job and = the oracle.  policy 0
    (the default since round 6): the same jobs through ONE saved-stream resident sweep (jet_fb.hpp, 5 layers)."""
    with B._native.knobs(policy=policy):
        _grad_jobs(B, sizes, policy)


def _grad_jobs(B, sizes, policy):
    ref, net = pair(B, 2, 2, 5, 128, seed=13)
    xs = [pts(n, 2, 40 + k) for k, n in enumerate(sizes)]
    lib, nat = B._native.lib(), B._native
    mode = net.call_mode(nat.MODE_GRAD)
    n_pass = 16 * sum((n + 15) // 16 for n in sizes)
    assert lib.insr_jet_bwd_path(n_pass, 2, 2, 5, 128, mode) == (1 if policy == 2 else 2)  # the path of the total

    def loss_hip(xs):
        y0, J0, _ = B._jet.run_jet(net, xs[0], nat.MODE_GRAD)
        tot = 1e-3 * torch.sum(J0 ** 2) + 1e-3 * torch.sum(y0 ** 2)
        for k, x in enumerate(xs[1:]):
            yk, _, _ = B._jet.run_jet(net, x, nat.MODE_GRAD)  # (a promoted call: its values are read)
            tot = tot + (k + 1) * torch.sum((yk - 0.1 * k) ** 2)
        return tot

    def loss_ref(xs):
        y0 = ref(xs[0])
        tot = 1e-3 * torch.sum(O.op_jacobian(y0, xs[0])[0] ** 2) + 1e-3 * torch.sum(y0 ** 2)
        for k, x in enumerate(xs[1:]):
            tot = tot + (k + 1) * torch.sum((ref(x) - 0.1 * k) ** 2)
        return tot

    xg = [t.cuda().requires_grad_(True) for t in xs]
    g1 = run(B, net, lambda: loss_hip(xg), batched=False)
    g2 = run(B, net, lambda: loss_hip(xg), batched=True)
    for a, b in zip(g2, g1):
        assert nerr(a, b) < TOL
    net.zero_grad(set_to_none=True)
    with B._jet.defer_reductions():
        with B._jet.batched_backward():
            loss_hip(xg).backward()
    torch.cuda.synchronize()
    for a, b in zip(grads(net), g2):
        assert torch.equal(a, b)  # held back or not: the same sums
    loss_ref([t.requires_grad_(True) for t in xs]).backward()
    for (k, p), g in zip(ref.named_parameters(), g2):
        ga = p.grad if p.grad is not None else torch.zeros_like(p)
        assert nerr(g, ga) < TOL, k


def test_more_jobs_than_one_launch(B):
    """11 band calls of one network: chunks of INSR_MAX_BWD_JOBS, gradients accumulated."""
    ref, net = pair(B, 2, 2, 4, 128, seed=5)
    xs = [pts(100 + 7 * k, 2, 30 + k) for k in range(B._native.MAX_BWD_JOBS + 3)]
    xg = [x.cuda().requires_grad_(True) for x in xs]
    g1 = run(B, net, lambda: value_loss(B, net, xg), batched=False)
    g2 = run(B, net, lambda: value_loss(B, net, xg), batched=True)
    for a, b in zip(g2, g1):
        assert nerr(a, b) < ORDER_TOL


def test_two_networks_and_accumulation(B):
    """Jobs of two networks in one scope go to their own .grad; a second backward accumulates."""
    _, u = pair(B, 2, 2, 4, 128, seed=6)
    _, p = pair(B, 2, 1, 4, 128, seed=7)
    xs = [pts(n, 2, 40 + n).cuda().requires_grad_(True) for n in (2048, 162, 162)]

    def loss():
        return value_loss(B, u, xs) + value_loss(B, p, xs)

    for net in (u, p):
        net.zero_grad(set_to_none=True)
    loss().backward()
    ref1 = [grads(u), grads(p)]
    for net in (u, p):
        net.zero_grad(set_to_none=True)
    with B._jet.batched_backward():
        loss().backward()
    with B._jet.batched_backward():
        loss().backward()
    torch.cuda.synchronize()
    for net, r in zip((u, p), ref1):
        for a, b in zip(grads(net), r):
            assert nerr(a, 2 * b) < ORDER_TOL


def test_c_abi_multi_equals_single_calls(B):
    """insr_siren_jet_bwd_grad_multi straight through the C ABI: the sum of per-job
    insr_siren_jet_bwd_grad calls (value jets, fused path)."""
    nat = B._native
    lib = nat.lib()
    _, net = pair(B, 2, 2, 4, 128, seed=8)
    cm = net.call_mode(nat.MODE_VALUE)
    net.ensure_wsplit()
    flat = net.flat_params()
    jobs, keep = [], []
    for k, n in enumerate((3000, 162, 33)):
        x = pts(n, 2, 50 + k).cuda()
        act = torch.empty(lib.insr_jet_act_bytes(n, 2, 4, 128, cm) // 4, device="cuda")
        y = torch.empty(n, 2, device="cuda")
        assert lib.insr_siren_jet_fwd(nat.ptr(x), n, 2, 2, 4, 128, cm, nat.ptr(flat), nat.ptr(y), None, None,
                                      nat.ptr(act), nat.stream_of(x.device)) == 0
        gy = torch.randn(n, 2, generator=torch.Generator().manual_seed(60 + k)).cuda()
        jobs.append(nat.BwdJob(x.data_ptr(), act.data_ptr(), gy.data_ptr(), None, None, n))
        keep += [x, act, gy]
    st = nat.stream_of(torch.device("cuda"))
    P = flat.numel()
    g_single = torch.zeros(P, device="cuda")
    for j in jobs:
        wb = lib.insr_jet_bwd_work_bytes(j.n, 2, 2, 4, 128, cm)
        w = torch.empty(wb // 4, device="cuda")
        assert lib.insr_siren_jet_bwd_grad(j.x, j.n, 2, 2, 4, 128, cm, nat.ptr(flat), j.act, j.gy, None, None,
                                           nat.ptr(w), nat.ptr(g_single), 1, st) == 0
        keep.append(w)
    arr = (nat.BwdJob * len(jobs))(*jobs)
    ns = (ctypes.c_long * len(jobs))(*[j.n for j in jobs])
    w = torch.empty(lib.insr_jet_bwd_multi_work_bytes(ns, len(jobs), 2, 2, 4, 128, cm) // 4, device="cuda")
    g_multi = torch.full((P,), float("nan"), device="cuda")  # accumulate = 0 overwrites
    assert lib.insr_siren_jet_bwd_grad_multi(arr, len(jobs), 2, 2, 4, 128, cm, nat.ptr(flat), nat.ptr(w),
                                             nat.ptr(g_multi), 0, st) == 0
    torch.cuda.synchronize()
    n_params = lib.insr_siren_param_count(2, 2, 4, 128)
    assert nerr(g_multi[:n_params], g_single[:n_params]) < ORDER_TOL


@pytest.mark.parametrize("prec", ["x6", "f32"])
@pytest.mark.parametrize("tiles", [(1, 4), (1, 2), (2, 4)])
def test_backward_never_reads_tiles_the_forward_left_unwritten(B, prec, tiles):
    """A backward whose blocks hold more tiles than the forward's (forced here; the fused
    launch of a band beside an interior does it by design) must not read the saved-stream tiles
    past ceil(n / 16): the forward never writes them.  The activation buffer is allocated from
    memory just filled with NaN (the caching allocator hands the freed block back), so a read of
    an unwritten tile poisons the gradient; n = 4,500 points = 282 tiles (not a multiple of 4)."""
    nat = B._native
    p = {"x6": 1, "f32": 0}[prec]
    with nat.knobs(tiles=tiles, prec=(p, p)):
        ref, net = pair(B, 2, 2, 4, 128, seed=9)
        n = 4500
        x = pts(n, 2, 70)
        gy = torch.randn(n, 2, generator=torch.Generator().manual_seed(71))
        cm = net.call_mode(nat.MODE_VALUE)
        poison = torch.full((nat.lib().insr_jet_act_bytes(n, 2, 4, 128, cm) // 4,), float("nan"), device="cuda")
        del poison  # the forward's act buffer reuses this block
        net.zero_grad(set_to_none=True)
        (net(x.cuda()) * gy.cuda()).sum().backward()
        torch.cuda.synchronize()
        (ref(x) * gy).sum().backward()
        for (k, q), g in zip(ref.named_parameters(), grads(net)):
            assert torch.isfinite(g).all(), k
            assert nerr(g, q.grad) < TOL, k
