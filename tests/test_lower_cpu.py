"""base/lower.py on the CPU: the recorder and the loss plans, with CPU tensors standing in for the jets'
outputs (the networks are HIP-only; the fused launch itself is covered by tests/test_gpu_plain_api.py).

* every reference phase body's loss (fluid/model.py:72-151, advection/model.py:68-91) is recognised,
  and its plan -- evaluated here with torch ops -- equals the eager expression, value and gradients;
* anything the recorder does not know runs eagerly with the same values and autograd history;
* Lazy tensors answer shape / dtype / requires_grad without materialising.
"""
import os
import sys

import pytest
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "insr-pde_amd"))
from base import lower as LW  # noqa: E402


def _eval_plan(p):
    if p[0] == "bands2":
        (A, B), w = p[1], p[2]
        return w * ((A[:, 0] ** 2).mean() + (B[:, 1] ** 2).mean())
    (a, b, c, d), (al, be, ga, de), w, red = p[1], p[2], p[3], p[4]
    r = a if b is None else a + be * b
    r = al * r
    if c is not None:
        q = c if d is None else c + de * d
        r = r + ga * q
    return w * ((r ** 2).mean() if red == "mean" else (r ** 2).sum())


def _leaves(*ts):
    return [LW.leaf(t) for t in ts]


def _grads(loss, ts):
    return torch.autograd.grad(loss, ts, allow_unused=True)


def _check(build, ts, kind):
    """build(*inputs) -> a loss: its Lazy plan == the eager loss (value and gradients)."""
    ref = build(*ts)
    g_ref = _grads(ref, [t for t in ts if t.requires_grad])
    with LW.lowering():
        lz = build(*_leaves(*ts))
    assert isinstance(lz, LW.Lazy) and lz.shape == ()
    p = LW.plan(lz._insr_node)
    assert p is not None and p[0] == kind
    v = _eval_plan(p)
    assert torch.allclose(v, ref, rtol=1e-6, atol=0), (float(v), float(ref))
    g = _grads(v, [t for t in ts if t.requires_grad])
    for a, b in zip(g, g_ref):
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.allclose(a, b, rtol=1e-5, atol=1e-9)
    # the materialised Lazy loss (the eager route) is the expression itself
    m = LW.materialize(lz)
    assert torch.equal(m, ref)
    gm = _grads(m, [t for t in ts if t.requires_grad])
    for a, b in zip(gm, g_ref):
        if a is not None:
            assert torch.equal(a, b)


def _t(*shape, grad=True, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g).requires_grad_(grad)


def test_fluid_advect_main():
    u, target = _t(64, 2), _t(64, 2, grad=False, seed=1)
    _check(lambda u, t: torch.mean((u - t) ** 2), [u, target], "combo")


def test_fluid_walls_two_tensors():
    ux, uy = _t(9, 2, seed=2), _t(9, 2, seed=3)
    _check(lambda a, b: (torch.mean(a[..., 0] ** 2) + torch.mean(b[..., 1] ** 2)) * 1.0, [ux, uy], "bands2")
    # the pressure walls (no * 1.0) and the bands written in the other order
    _check(lambda a, b: torch.mean(a[:, 0] ** 2) + torch.mean(b[:, 1] ** 2), [ux, uy], "bands2")
    _check(lambda a, b: torch.mean(b[..., 1] ** 2) + torch.mean(a[..., 0] ** 2), [ux, uy], "bands2")


def test_fluid_pressure_main():
    div_u, lap_p = _t(64, 1, grad=False, seed=4), _t(64, 1, seed=5)
    _check(lambda d, l: torch.mean((d.detach() - l) ** 2), [div_u, lap_p], "combo")


def test_fluid_projection_main():
    u, u_old, gp = _t(64, 2), _t(64, 2, grad=False, seed=6), _t(64, 2, seed=7)
    _check(lambda u, uo, g: torch.mean((u - (uo - g.detach())) ** 2), [u, u_old, gp], "combo")


def test_advection_main_and_bc():
    dt, vel = 0.05, 0.8
    u, u0, gu, gu0 = _t(50, 1), _t(50, 1, grad=False, seed=8), _t(50, 1, seed=9), _t(50, 1, seed=10)
    _check(lambda u, u0, gu, gu0: torch.mean(((u - u0) / dt + vel * (gu + gu0.detach()) / 2.) ** 2),
           [u, u0, gu, gu0], "combo")
    ub = _t(10, 1, seed=11)
    _check(lambda b: torch.mean(b ** 2) * 1., [ub], "combo")


def test_initialize_mse_loss():
    u, ref = _t(64, 2), _t(64, 2, grad=False, seed=12)
    _check(lambda u, r: F.mse_loss(u, r), [u, ref], "combo")


def test_unknown_ops_stay_eager():
    u, v = _t(16, 2), _t(16, 2, seed=13)
    with LW.lowering():
        a, b = _leaves(u, v)
        y = torch.sin(a) * b + 1.0           # sin: not recorded -> real; * b, + 1.0 on reals: eager
        z = (a * b).sum()                     # a * b of two tensors: not linear -> eager
        w = torch.mean(a ** 3)                # ** 3 -> eager
    assert not isinstance(y, LW.Lazy) and not isinstance(z, LW.Lazy) and not isinstance(w, LW.Lazy)
    assert torch.equal(y, torch.sin(u) * v + 1.0)
    assert torch.equal(z, (u * v).sum())
    assert torch.equal(w, torch.mean(u ** 3))
    gz = torch.autograd.grad(z, [u])[0]
    assert torch.equal(gz, v)


def test_metadata_without_materialising():
    u = _t(8, 2)
    with LW.lowering():
        (a,) = _leaves(u)
        d = (a - a.detach() * 2.0)
        before = LW.LOWERED["materialized"]
        assert d.shape == (8, 2) and d.dtype == torch.float32 and d.requires_grad and d.dim() == 2
        assert d.numel() == 16 and d.size(0) == 8 and len(d) == 8
        assert not a.detach().requires_grad
        with torch.no_grad():
            assert not (a * 2.0).requires_grad
        assert LW.LOWERED["materialized"] == before
        assert float(torch.mean(d ** 2)) == pytest.approx(float(torch.mean((u - u.detach() * 2.0) ** 2)))


def test_unrecognised_loss_materialised_by_lower_losses():
    u, v = _t(16, 2), _t(16, 2, seed=14)
    with LW.lowering():
        a, b = _leaves(u, v)
        ld = {"main": torch.mean((a - b) ** 2) + torch.mean(a ** 2),  # two unpaired terms: eager
              "bc": torch.mean(a[..., 0] ** 2) + torch.mean(b[..., 0] ** 2)}  # both column 0: eager
    assert LW.plan(ld["main"]._insr_node) is None and LW.plan(ld["bc"]._insr_node) is None
    out = LW.lower_losses(ld)
    assert not any(isinstance(v_, LW.Lazy) for v_ in out.values())
    assert torch.allclose(out["main"], torch.mean((u - v) ** 2) + torch.mean(u ** 2))
    out["main"].backward()
    assert u.grad is not None


def test_broadcasting_and_offsets_stay_eager():
    u, w = _t(16, 1), _t(16, seed=15)
    with LW.lowering():
        (a,) = _leaves(u)
        r = a - w  # (16, 1) - (16,) broadcasts: eager
        s = a + 1.0  # a constant offset: recorded (the elasticity energies' S - 1), but no residual plan takes it
        loss = torch.mean(s ** 2)
    assert not isinstance(r, LW.Lazy) and r.shape == (16, 16)
    assert isinstance(s, LW.Lazy) and s._insr_node.kind == "off" and LW.plan(loss._insr_node) is None
    assert torch.equal(LW.materialize(s), u + 1.0)
    out = LW.lower_losses({"main": loss})  # eager, as written
    assert torch.equal(out["main"], torch.mean((u + 1.0) ** 2))


def test_lowering_inactive_outside_scope():
    u = _t(4, 2)
    assert LW.leaf(u) is u
    with LW.lowering(False):
        assert LW.leaf(u) is u
    with LW.lowering():
        with LW.suspended():
            assert LW.leaf(u) is u
        assert isinstance(LW.leaf(u), LW.Lazy)


def test_detached_sum_of_views():
    """mean((div_u - lap_p) ** 2) with div_u = (J[..., 0, 0:1] + J[..., 1, 1:2]).detach() recorded as a sum of
    two strided views (the deferred divergence, base/lower.py add_views): a 3-operand COMBO term."""
    J, lap = _t(64, 2, 2, grad=False, seed=16), _t(64, 1, seed=17)
    ref = torch.mean(((J[..., 0, 0:1] + J[..., 1, 1:2]).detach() - lap) ** 2)
    with LW.lowering():
        a, b, l_ = LW.leaf(J[..., 0, 0:1]), LW.leaf(J[..., 1, 1:2]), LW.leaf(lap)
        lz = torch.mean(((a + b).detach() - l_) ** 2)
    p = LW.plan(lz._insr_node)
    assert p is not None and p[0] == "combo" and p[1][0] is lap and sum(t is not None for t in p[1]) == 3
    assert torch.allclose(_eval_plan(p), ref, rtol=1e-6)
    g = torch.autograd.grad(_eval_plan(p), [lap])[0]
    assert torch.allclose(g, torch.autograd.grad(ref, [lap])[0], rtol=1e-5, atol=1e-9)


def test_attributes_of_lazy_tensors():
    """Only shape-like metadata is answered by the wrapper; data / grad_fn / is_leaf / T come from the real
    tensor (materialised), so code that inspects autograd state or reads .data sees what eager code sees."""
    u = _t(4, 2)
    with LW.lowering():
        (a,) = _leaves(u)
        b = a * 2.0
        assert isinstance(b, LW.Lazy)
        assert b.shape == (4, 2) and b.requires_grad and b.layout == torch.strided
        assert type(b.grad_fn).__name__ == "MulBackward0" and not b.is_leaf
        assert torch.equal(b.data, (u * 2.0).data) and torch.equal(b.T, (u * 2.0).T)
        assert a.is_leaf == u.is_leaf and a.grad_fn is u.grad_fn


def test_sum_of_squares_losses():
    """ratio * torch.sum((q - target) ** 2) (elasticity/losses.py:6-8 style) and F.mse_loss(..., reduction='sum'):
    one COMBO term with reduction 'sum'."""
    q, tgt = _t(32, 2, seed=18), _t(32, 2, grad=False, seed=19)
    _check(lambda q, t: 1e4 * torch.sum((q - t) ** 2), [q, tgt], "combo")
    _check(lambda q, t: (q - t).pow(2).sum() * 0.5, [q, tgt], "combo")
    _check(lambda q, t: F.mse_loss(q, t, reduction="sum"), [q, tgt], "combo")
    with LW.lowering():
        a, b = _leaves(q, tgt)
        mixed = torch.sum((a - b) ** 2) + torch.mean(a[..., 0] ** 2)  # two reductions: eager
    assert LW.plan(mixed._insr_node) is None


def test_in_place_write_on_a_lazy_tensor():
    """An in-place op on a Lazy tensor evaluates what was recorded before it (eager order): d = u - t read
    before u.add_(1) keeps the old u, u ** 2 after it reads the new one; value and gradients = eager."""
    base, t = _t(16, 2, seed=20), _t(16, 2, grad=False, seed=21)

    def body(u, t):
        d = u - t
        u.add_(1.0)
        u[:, 1] = 0.5 * u[:, 1].detach()
        return torch.mean(d ** 2), torch.mean(u ** 2)

    ref1, ref2 = body(base * 1.0, t)
    g_ref = torch.autograd.grad(ref1 + ref2, [base])[0]
    with LW.lowering():
        (a,) = _leaves(base * 1.0)
        l1, l2 = body(a, t)
    assert LW.plan(l1._insr_node) is None  # reads the old u: eager (its value was computed before the write)
    p2 = LW.plan(l2._insr_node)
    assert p2 is not None and p2[0] == "combo"
    m1, m2 = LW.materialize(l1), _eval_plan(p2)
    assert torch.equal(m1, ref1) and torch.allclose(m2, ref2, rtol=1e-6)
    g = torch.autograd.grad(m1 + m2, [base])[0]
    assert torch.allclose(g, g_ref, rtol=1e-5, atol=1e-9)


def test_plain_tensor_written_behind_the_recorder():
    """A plain tensor a recorded expression reads, written in place before the expression is evaluated: the
    replay raises instead of reading the new values, and the loss is not lowered."""
    u, t = _t(8, 2, seed=22), _t(8, 2, grad=False, seed=23)
    with LW.lowering():
        (a,) = _leaves(u)
        d = a - t
        loss = torch.mean(d ** 2)
        t.zero_()
    assert LW.plan(loss._insr_node) is None
    with pytest.raises(RuntimeError, match="written in place"):
        LW.materialize(loss)


def test_requires_grad_is_not_a_write():
    """requires_grad_ changes no values: nothing else recorded is evaluated and the tensor keeps its record."""
    u = _t(8, 2, seed=24)
    with LW.lowering():
        (a,) = _leaves(u)
        e = a * 3.0
        d = a * 2.0
        node = d._insr_node
        d.requires_grad_(True)
        assert e._insr_node.real is None and d._insr_node is node


def test_augmented_assignment_is_a_write():
    """u += 1 / u *= 2 on a Lazy tensor (Tensor.__iadd__ / __imul__): writes, in eager order; int() / iter()
    are reads (nothing else recorded is evaluated)."""
    base, t = _t(8, 2, seed=25), _t(8, 2, grad=False, seed=26)

    def body(u, t):
        d = u - t
        u += 1.0
        u *= 2.0
        return torch.mean(d ** 2) + torch.mean(u ** 2)

    ref = body(base * 1.0, t)
    with LW.lowering():
        (a,) = _leaves(base * 1.0)
        lz = body(a, t)
        e = a * 3.0
        rows = [r for r in lz.reshape(1)]
        assert e._insr_node.real is None and len(rows) == 1
        assert a.mul_(1.0) is a and isinstance(a, LW.Lazy)
    assert torch.allclose(LW.materialize(lz), ref, rtol=1e-6)


def test_plain_tensor_written_with_a_lazy_value():
    """x[:, 0] = u[:, 1] (a plain tensor written from a Lazy one) after d = x - u was recorded: d keeps the
    old x, as in eager code."""
    base, x0 = _t(8, 2, seed=27), _t(8, 2, grad=False, seed=28)

    def body(u, x):
        d = x - u
        x[:, 0] = u[:, 1].detach()
        return torch.mean(d ** 2) + torch.mean((x - u) ** 2)

    ref = body(base * 1.0, x0.clone())
    with LW.lowering():
        (a,) = _leaves(base * 1.0)
        lz = body(a, x0.clone())
    assert torch.allclose(LW.materialize(lz), ref, rtol=1e-6)


def test_ready_sampler_leaf_rescale_is_one_op_and_cached():
    """A sampler's draw (base/lower.py sampler_api: a READY leaf) rescaled as the reference advection body
    does (advection/model.py:27: sample_random(...).requires_grad_(True) * length / 2) evaluates as one
    multiply by the folded scalar, with autograd, is cached, and reading the draw itself returns its tensor."""
    torch.manual_seed(3)
    draw = torch.rand(16, 1) * 2 - 1
    with LW.lowering():
        n = LW._Node("leaf", real=draw, shape=tuple(draw.shape))
        n.ready = True
        x = LW._wrap(n, draw.dtype, draw.device, False)
        xg = x.requires_grad_(True)
        assert xg is x and x.requires_grad and draw.requires_grad
        y = x * 4.0 / 2
        assert isinstance(y, LW.Lazy) and y.requires_grad
        before = LW.LOWERED["materialized"]
        r = LW.materialize(y)
        assert LW.LOWERED["materialized"] == before + 1  # one evaluation for the whole chain
        assert torch.equal(r, draw * 2.0) and r.requires_grad and r.grad_fn is not None
        assert LW.materialize(y) is r and LW.materialize(x) is draw
        r.sum().backward()
        assert torch.equal(draw.grad, torch.full_like(draw, 2.0))


def _el2d_loss(Jz, Fl, Fr, T, torch_mod=torch):
    """elasticity/model.py:143-183 with energy = [arap, constraint, constraint_right, volume] (el2D)."""
    U, S, V = torch.svd(Jz)
    E_arap = 1.0 * torch.sum((S - 1.0) ** 2)
    E_volume = 1e3 * torch.sum((torch.prod(S, dim=1) - 1) ** 2)
    loss = 0
    loss = loss + E_arap
    loss = loss + 1e4 * torch.sum((Fl - 0) ** 2)
    loss = loss + 1e4 * torch.sum((Fr - T) ** 2)
    loss = loss + E_volume
    return loss


def test_elasticity_energy_plan():
    """The unchanged elasticity body's energy (svd of J + I, the arap / volume sums over its singular values,
    the positional constraints): energy_plan finds one singular-value energy per term and the constraints as
    sum-of-squares terms, records nothing eagerly, and the materialised Lazy loss is the eager expression."""
    from base import _jet  # noqa: F401  (deferred_jets opens a fused_forwards scope)
    n = 40
    Jraw, f, x = _t(n, 2, 2, seed=4), _t(n, 2, seed=5), _t(n, 2, grad=False, seed=6)
    Fl, Fr, T = _t(7, 2, seed=7), _t(7, 2, seed=8), _t(7, 2, grad=False, seed=9)
    with torch.no_grad():
        Jraw.mul_(0.2)
    ref = _el2d_loss(Jraw + torch.eye(2), Fl, Fr, T)
    mat0 = LW.LOWERED["materialized"]
    with LW.lowering(), LW.deferred_jets():
        Jz = LW.eye_add(Jraw, (None, f, x))
        lz = _el2d_loss(Jz, *_leaves(Fl, Fr), T)
        assert isinstance(lz, LW.Lazy) and LW.LOWERED["materialized"] == mat0  # nothing evaluated while recording
        ep = LW.energy_plan(lz._insr_node)
        assert ep is not None
        kinds = [(k, w) for k, w, _ in ep]
        assert kinds == [("energy", 1.0), ("sq", 1e4), ("sq", 1e4), ("energy", 1e3)]
        assert [p[0] for k, _, p in ep if k == "energy"] == ["arap", "volume"]
        sq = [w * _eval_plan(p) for k, w, p in ep if k == "sq"]
        assert all(p[0] == "combo" and p[4] == "sum" for k, _, p in ep if k == "sq")
        assert torch.allclose(sq[0], 1e4 * torch.sum(Fl ** 2)) and torch.allclose(sq[1], 1e4 * torch.sum((Fr - T) ** 2))
        m = LW.materialize(lz)
    assert torch.allclose(m, ref, rtol=1e-6)
    g, g_ref = _grads(m, [Jraw, Fl, Fr]), _grads(ref, [Jraw, Fl, Fr])
    for a, b in zip(g, g_ref):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)


def test_kinematics_is_a_sum_of_squares_term():
    """E_kinematics = r sum((qdot - qdot_prev)^2), qdot = (q - q_prev) / dt, q = f + x (elasticity/model.py:
    137-148): the x terms cancel exactly and the residual is one 3-operand combo (f, f_prev, f_pp)."""
    n, dt = 30, 0.1
    f, fp, fpp, x = _t(n, 3, seed=1), _t(n, 3, grad=False, seed=2), _t(n, 3, grad=False, seed=3), _t(n, 3, grad=False, seed=4)

    def body(f, fp, fpp, x):
        q, q_prev, q_pp = f + x, fp + x, fpp + x
        qdot = (q - q_prev) / dt
        qdot_prev = (q_prev - q_pp) / dt
        return 1.0 * torch.sum((qdot - qdot_prev) ** 2)
    ref = body(f, fp, fpp, x)
    with LW.lowering():
        lz = body(*_leaves(f, fp, fpp, x))
    p = LW.plan(lz._insr_node)
    assert p is not None and p[0] == "combo" and p[4] == "sum"
    assert sum(t is not None for t in p[1]) == 3
    assert torch.allclose(_eval_plan(p), ref, rtol=1e-5)
