"""Fused residual losses (base.losses, residual.hip) vs the plain torch fp32 expressions
the reference writes (fluid/model.py:90-151, advection/model.py:78-91).

Tolerance: the fused forward sums in its own (deterministic) order, so losses are
judged against the fp64 value of the same expression at 1e-5 relative (fp32
summation of up to 6e5 squares); gradients are elementwise formulas of the same
residual and agree with torch fp32 to 1e-6 relative normwise."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def B():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    base._native.load()
    return base


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


CASES = [  # (alpha, beta, gamma, delta, which of b, c, d present)
    (1.0, -1.0, 1.0, 1.0, "b"),        # mean((u - target)^2)
    (1.0, -1.0, 1.0, 1.0, ""),         # mean(u^2)
    (1.0, 0.0, -1.0, -1.0, "cd"),      # u - (u_prev - grad_p)
    (20.0, -1.0, 0.125, 1.0, "bcd"),   # (u - u0)/dt + v (ux + u0x)/2
]


@pytest.mark.parametrize("n", [1, 1000, 40000, 300000])  # x2 columns: 300000 -> 5 blocks
@pytest.mark.parametrize("case", range(len(CASES)))
def test_fused_mse_matches_torch(B, n, case):
    alpha, beta, gamma, delta, which = CASES[case]
    g = torch.Generator(device="cuda").manual_seed(n + case)
    t = {k: torch.randn(n, 2, device="cuda", generator=g).requires_grad_(True) for k in "abcd"}
    a = t["a"]
    b, c, d = (t[k] if k in which else None for k in "bcd")

    def ref():
        p = a + beta * b if b is not None else a
        p = alpha * p
        if c is not None:
            q = c + delta * d if d is not None else c
            p = p + gamma * q
        return torch.mean(p ** 2)

    lr = ref()
    gr = torch.autograd.grad(lr, [x for x in (a, b, c, d) if x is not None])
    a, b, c, d = (None if x is None else x.detach().double().requires_grad_(False) for x in (a, b, c, d))
    l64 = ref()
    a, b, c, d = (t[k] if (k == "a" or k in which) else None for k in "abcd")
    for _ in range(2):  # twice: the multi-block path reuses its partials buffer
        lf = B.fused_mse(a, b, c, d, alpha=alpha, beta=beta, gamma=gamma, delta=delta)
        assert rel(lf.detach(), l64) < 1e-5
    gf = torch.autograd.grad(lf, [x for x in (a, b, c, d) if x is not None])
    for x, y in zip(gf, gr):
        assert rel(x, y) < 1e-6


@pytest.mark.parametrize("nb", [1, 162, 654, 50000])
def test_wall_mse_matches_torch(B, nb):
    y = torch.randn(2 * nb, 3, device="cuda", generator=torch.Generator(device="cuda").manual_seed(nb))
    y.requires_grad_(True)
    lr = torch.mean(y[:nb, 0] ** 2) + torch.mean(y[nb:, 1] ** 2)
    (gr,) = torch.autograd.grad(lr, y)
    lf = B.wall_mse(y, nb)
    y64 = y.detach().double()
    assert rel(lf.detach(), torch.mean(y64[:nb, 0] ** 2) + torch.mean(y64[nb:, 1] ** 2)) < 1e-5
    (gf,) = torch.autograd.grad(lf, y)
    assert rel(gf, gr) < 1e-6 and bool((gf[:nb, 1:] == 0).all()) and bool((gf[nb:, 0] == 0).all())


def test_fused_mse_in_graph_replay(B):
    """The two-launch (multi-block) reduction inside a captured hipGraph, replayed."""
    x = torch.randn(400000, device="cuda")
    y = torch.randn(400000, device="cuda")
    B.fused_mse(x, y)  # workspace allocated outside the capture
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        B.fused_mse(x, y)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            out = B.fused_mse(x, y)
    torch.cuda.current_stream().wait_stream(s)
    for k in range(3):
        x.mul_(1.5)
        gr.replay()
        torch.cuda.synchronize()
        assert rel(out, torch.mean((x.double() - y.double()) ** 2)) < 1e-5, k


def test_losses_reject_cpu(B):
    with pytest.raises(B.NativeUnavailable):
        B.fused_mse(torch.ones(3))


def _svd_case(n, d, seed, kind):
    g = torch.Generator().manual_seed(seed)
    J = torch.eye(d).expand(n, d, d) + 0.3 * torch.randn(n, d, d, generator=g)
    if kind == "reflect":      # det < 0 blocks
        J[::2, 0] = -J[::2, 0]
    elif kind == "degenerate":  # repeated / vanishing singular values
        J[: n // 3] = torch.eye(d)
        J[n // 3: 2 * n // 3, :, -1] = 0.0
    return J.contiguous()


@pytest.mark.parametrize("d", [2, 3])
@pytest.mark.parametrize("kind", ["plain", "reflect", "degenerate"])
@pytest.mark.parametrize("n", [7, 5000])
def test_svd_energy_matches_torch_svd(B, d, kind, n):
    """elasticity/model.py:143-163 (torch.svd singular values; arap + volume) in fp64 as
    the judge: energy within 1e-5 relative; gradient U diag(dE/ds) V^T within 1e-4
    normwise (the gradient of a singular value is ill-conditioned near repeated values)."""
    ra, rv = 1.0, 1e3
    J = _svd_case(n, d, 100 * d + n, kind)
    J64 = J.double().requires_grad_(True)
    S = torch.linalg.svdvals(J64)
    E64 = ra * torch.sum((S - 1) ** 2) + rv * torch.sum((torch.prod(S, dim=1) - 1) ** 2)
    (G64,) = torch.autograd.grad(E64, J64)
    Jg = J.cuda().requires_grad_(True)
    E = B.svd_energy(Jg, ra, rv)
    assert rel(E.detach(), E64.detach()) < 1e-5
    (G,) = torch.autograd.grad(E * 2.0, Jg)  # a non-unit upstream gradient
    if kind == "degenerate":  # exactly repeated values: only the well-defined (non-repeated) blocks
        G, G64 = G[2 * n // 3:], G64[2 * n // 3:]
    assert rel(G / 2.0, G64) < 1e-4


# ---- merged launches: losses over row ranges of one network output (base.merge_samples) ----
@pytest.mark.parametrize("n_in,n_bc", [(1000, 40), (16384, 324), (5000, 0)])
def test_offset_losses_match_slices(B, n_in, n_bc):
    """fused_mse(count, a_row0) / wall_mse(row0) / svd_energy(count) on a merged (interior +
    boundary) tensor == the torch expressions on the slices, and the gradient of the merged
    tensor is the slices' gradients with zeros elsewhere."""
    g = torch.Generator(device="cuda").manual_seed(n_in + n_bc)
    rows = n_in + 2 * n_bc
    u = torch.randn(rows, 2, device="cuda", generator=g).requires_grad_(True)
    t = torch.randn(n_in, 2, device="cuda", generator=g)
    ur = u.detach().clone().requires_grad_(True)
    main = B.fused_mse(u, t, count=t.numel())
    parts = [main]
    main_r = torch.mean((ur[:n_in] - t) ** 2)
    parts_r = [main_r]
    if n_bc:
        bc = B.wall_mse(u, n_bc, row0=n_in)
        tail = B.fused_mse(u, count=2 * n_bc * 2, a_row0=n_in, reduction="sum")
        bc_r = torch.mean(ur[n_in:n_in + n_bc, 0] ** 2) + torch.mean(ur[n_in + n_bc:, 1] ** 2)
        tail_r = torch.sum(ur[n_in:] ** 2)
        parts += [bc, tail]
        parts_r += [bc_r, tail_r]
    for a, b in zip(parts, parts_r):
        assert rel(a, b) < 1e-5
    sum(parts).backward()
    sum(parts_r).backward()
    assert rel(u.grad, ur.grad) < 1e-6


def test_svd_energy_count(B):
    g = torch.Generator(device="cuda").manual_seed(3)
    J = (torch.eye(2, device="cuda") + 0.3 * torch.randn(700, 2, 2, device="cuda", generator=g)).requires_grad_(True)
    n = 500
    e = B.svd_energy(J, 1.0, 10.0, count=n)
    Jr = J.detach().double().clone().requires_grad_(True)
    S = torch.linalg.svdvals(Jr[:n])
    er = torch.sum((S - 1) ** 2) + 10.0 * torch.sum((S.prod(1) - 1) ** 2)
    assert rel(e, er) < 1e-5
    e.backward()
    er.backward()
    assert rel(J.grad, Jr.grad) < 1e-4 and float(J.grad[n:].abs().max()) == 0.0


def test_merge_samples(B):
    x = torch.rand(10, 2, device="cuda").requires_grad_(True)
    b = torch.rand(4, 2, device="cuda")
    m = B.merge_samples(x, b)
    assert m.is_leaf and m.requires_grad and m.shape == (14, 2)
    assert torch.equal(m[:10], x.detach()) and torch.equal(m[10:], b)


def test_loss_group_repeated_unit_backward(B):
    """A unit-seeded backward hands out the gradients the forward launch wrote; a second
    backward through the same graph (retain_graph=True) gets equal copies, not None."""
    a = torch.randn(5000, 2, device="cuda", requires_grad=True)
    b = torch.randn(5000, 2, device="cuda")
    loss = B.fused_mse(a, b)
    seed = B.losses.register_unit_seed(torch.ones((), device="cuda"))
    g1, = torch.autograd.grad(loss, (a,), grad_outputs=seed, retain_graph=True)
    g2, = torch.autograd.grad(loss, (a,), grad_outputs=seed, retain_graph=True)
    want = 2.0 * (a.detach() - b) / a.numel()
    assert rel(g1, want) < 1e-6 and torch.equal(g1, g2) and g1.data_ptr() != g2.data_ptr()
