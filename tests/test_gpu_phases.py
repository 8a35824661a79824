"""Phase-level parity: the HIP path against vectors recorded from the REFERENCE itself
(tests/golden/ref_phases.npz, made by tests/golden/make_golden.py on identical weights
and samples).  Covers the loss dict of every phase body, the parameter gradients after
loss.backward(), and two full optimiser iterations (Adam + plateau) per phase.

Tolerances: losses 1e-5 relative; gradients 1e-5 normwise per network.  After Adam,
parameter *updates* are compared on entries whose reference gradient is well away from
zero (|g| > 1e-3 max|g|): Adam's first step is ~lr*sign(g), so entries with |g| at the
fp32 noise floor may legitimately flip sign.
"""
import os
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_phases.npz")
TOL = 1e-5


@pytest.fixture(scope="module")
def ph():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return dict(np.load(GOLD))


def nerr(a, b):
    a = torch.as_tensor(np.asarray(a, np.float64))
    b = torch.as_tensor(np.asarray(b, np.float64))
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def set_flat(net, vec):
    with torch.no_grad():
        net.flat_params().copy_(torch.from_numpy(np.asarray(vec, np.float32)).cuda())


def flat_grad(net):
    return net.flat_grad_buffer().detach().cpu().numpy() if net.grad_touched() else np.zeros(net.param_count)


def flat(net):
    return net.flat_params().detach().cpu().numpy()


def check_update(after_hip, before, after_ref, g_ref):
    d_hip, d_ref = after_hip - before, after_ref - before
    mask = np.abs(g_ref) > 1e-3 * np.abs(g_ref).max()
    assert mask.sum() > 0.5 * mask.size
    assert nerr(d_hip[mask], d_ref[mask]) < 1e-3
    # everything else moved by at most ~2 lr per step (sign flips at the noise floor)
    assert np.abs(d_hip - d_ref).max() <= 2 * 2 * 1e-4 * 1.01


from base import _jet  # noqa: E402


def _cfg(pde, **kw):
    from pde.config import make_config
    kw.setdefault("insr_progress", False)
    kw.setdefault("early_stop", False)
    kw.setdefault("max_n_iters", 2)
    kw.setdefault("lr", 1e-4)
    return make_config(pde, proj_dir="/tmp/insr_test", **kw)


@pytest.mark.parametrize("fused", [True, False])
def test_fluid_phases(ph, fused):
    from pde.fluid import Fluid2DModel
    cfg = _cfg("fluid", num_hidden_layers=4, hidden_features=128, sample_resolution=32, dt=0.05,
               insr_fuse_forwards=fused)
    model = Fluid2DModel(cfg)
    T = lambda k: torch.from_numpy(ph[k]).cuda()  # noqa: E731
    nets = {"vel": model.velocity_field, "vel_prev": model.velocity_field_prev, "pres": model.pressure_field}

    def reset():
        for k, n in nets.items():
            set_flat(n, ph[f"fluid/{k}/params0"])

    def patch(it):
        model._sample_in_training = lambda: T(f"fluid/x{it}").clone().requires_grad_(True)
        model._boundary_pair = lambda n: (T(f"fluid/bcx{it}").clone().requires_grad_(True),
                                          T(f"fluid/bcy{it}").clone().requires_grad_(True))

    for phase in ("_advect_velocity", "_solve_pressure", "_projection"):
        body = getattr(Fluid2DModel, phase)._insr_phase
        reset()
        patch(0)
        model._reset_optimizer()
        ld = body(model)
        for k, v in ld.items():
            ref = float(ph[f"fluid/{phase}/loss_{k}"])
            assert abs(float(v) - ref) <= TOL * abs(ref) + 1e-12, (phase, k, float(v), ref)
        model.optimizer.zero_grad()
        sum(ld.values()).backward()
        gv = ph[f"fluid/{phase}/grad_vel"]
        if np.abs(gv).max() > 0:
            assert nerr(flat_grad(model.velocity_field), gv) < TOL, phase
        gp = ph[f"fluid/{phase}/grad_pres"]
        if np.abs(gp).max() > 0:
            assert nerr(flat_grad(model.pressure_field), gp) < TOL, phase
        else:
            assert not model.pressure_field.grad_touched()
        if np.abs(ph[f"fluid/{phase}/grad_vel"]).max() == 0:
            assert not model.velocity_field.grad_touched()
        # two reference iterations: phase + _update_network (Adam + plateau)
        reset()
        model._reset_optimizer()
        trace = []
        owner = types.SimpleNamespace()  # jet-mode hints: iteration 1 replays iteration 0's diff ops
        for it in range(2):
            patch(it)
            with _jet.call_scope(owner):
                ld = body(model)
            model._update_network(ld)
            trace.append([float(ld[k]) for k in sorted(ld)])
        assert nerr(np.array(trace), ph[f"fluid/{phase}/loss_trace"]) < TOL
        if phase != "_advect_velocity":  # divergence / laplace / gradient of network values
            assert owner._insr_jet_hints, phase
        for key, net, g_ref in (("vel", model.velocity_field, ph[f"fluid/{phase}/grad_vel"]),
                                ("pres", model.pressure_field, gp)):
            if np.abs(g_ref).max() > 0:
                check_update(flat(net), ph[f"fluid/{key}/params0"], ph[f"fluid/{phase}/{key}_after"], g_ref)
            else:  # no gradient reaches this network in this phase: torch skips it, so do we
                assert np.array_equal(flat(net), ph[f"fluid/{key}/params0"])


def test_advect_phase(ph):
    import pde.advection as adv
    cfg = _cfg("advection", num_hidden_layers=3, hidden_features=64, sample_resolution=512, dt=0.05, vel=0.25,
               length=4.0)
    model = adv.Advection1DModel(cfg)
    set_flat(model.field, ph["advect/field/params0"])
    set_flat(model.field_prev, ph["advect/field_prev/params0"])
    T = lambda k: torch.from_numpy(ph[k]).cuda()  # noqa: E731
    orig = adv.sample_boundary

    def patch(it):
        model._sample_in_training = lambda: T(f"advect/x{it}").clone().requires_grad_(True)
        adv.sample_boundary = lambda n, sdim, device=None, **k: T(f"advect/bc{it}") / 2.0

    try:
        body = adv.Advection1DModel._advect._insr_phase
        patch(0)
        model._reset_optimizer()
        ld = body(model)
        for k, v in ld.items():
            ref = float(ph[f"advect/_advect/loss_{k}"])
            assert abs(float(v) - ref) <= TOL * abs(ref) + 1e-12, (k, float(v), ref)
        model.optimizer.zero_grad()
        sum(ld.values()).backward()
        assert nerr(flat_grad(model.field), ph["advect/_advect/grad_field"]) < TOL
        set_flat(model.field, ph["advect/field/params0"])
        model._reset_optimizer()
        trace = []
        owner = types.SimpleNamespace()  # jet-mode hints: iteration 1 replays iteration 0's diff ops
        for it in range(2):
            patch(it)
            with _jet.call_scope(owner):
                ld = body(model)
            model._update_network(ld)
            trace.append([float(ld[k]) for k in sorted(ld)])
        assert nerr(np.array(trace), ph["advect/_advect/loss_trace"]) < TOL
        check_update(flat(model.field), ph["advect/field/params0"], ph["advect/_advect/field_after"],
                     ph["advect/_advect/grad_field"])
    finally:
        adv.sample_boundary = orig


def test_elasticity_phase(ph):
    from pde.elasticity import ElasticityModel
    energy = [str(e) for e in ph["el2d/cfg_energy"]]
    cfg = _cfg("elasticity", num_hidden_layers=5, hidden_features=128, sample_resolution=16, dt=0.1, dim=2,
               energy=energy, ratio_constraint=1e4, ratio_volume=1e3, ratio_arap=1.0, ratio_collide=1e2,
               ratio_kinematics=1.0, external_force_timesteps=5, external_force_y=-1.0,
               constraint_right_offset_x=2.0, plane_height=-0.9)
    model = ElasticityModel(cfg)
    model.timestep = 1
    for k, n in (("f", model.deformation_field), ("f_prev", model.deformation_field_prev),
                 ("f_pp", model.deformation_field_prev_prev)):
        set_flat(n, ph[f"el2d/{k}/params0"])
    T = lambda k: torch.from_numpy(ph[k]).cuda()  # noqa: E731

    def patch(it):
        model._sample_in_training = lambda res: T(f"el2d/x{it}").clone().requires_grad_(True)
        model._sample_fixed_in_training = lambda res: (T(f"el2d/fixed_l{it}").clone().requires_grad_(True),
                                                       T(f"el2d/fixed_r{it}").clone().requires_grad_(True))

    body = ElasticityModel._solve_deformation._insr_phase
    patch(0)
    model._reset_optimizer()
    ld = body(model)
    ref = float(ph["el2d/_solve_deformation/loss_main"])
    assert abs(float(ld["main"]) - ref) <= TOL * abs(ref)
    model.optimizer.zero_grad()
    ld["main"].backward()
    assert nerr(flat_grad(model.deformation_field), ph["el2d/_solve_deformation/grad_f"]) < TOL
    set_flat(model.deformation_field, ph["el2d/f/params0"])
    model._reset_optimizer()
    trace = []
    owner = types.SimpleNamespace()  # jet-mode hints: iteration 1 replays iteration 0's diff ops
    for it in range(2):
        patch(it)
        with _jet.call_scope(owner):
            ld = body(model)
        model._update_network(ld)
        trace.append([float(ld[k]) for k in sorted(ld)])
    assert nerr(np.array(trace), ph["el2d/_solve_deformation/loss_trace"]) < TOL
    check_update(flat(model.deformation_field), ph["el2d/f/params0"], ph["el2d/_solve_deformation/f_after"],
                 ph["el2d/_solve_deformation/grad_f"])


def test_elasticity3d_phase(ph):
    """3-D energies (3x3 singular values via the fused HIP SVD kernel, plane and sphere
    collisions, external force, kinematics) against the reference's 3-D phase."""
    from pde.elasticity import ElasticityModel
    g3 = dict(np.load(GOLD.replace("ref_phases.npz", "ref_phases_el3d.npz")))
    energy = [str(e) for e in g3["el3d/cfg_energy"]]
    cfg = _cfg("elasticity", num_hidden_layers=2, hidden_features=64, sample_resolution=6, dt=0.1, dim=3,
               energy=energy, ratio_constraint=1e4, ratio_volume=1e3, ratio_arap=1e2, ratio_collide=1e3,
               ratio_kinematics=1.0, external_force_timesteps=5, external_force_x=0.0, external_force_y=0.0,
               external_force_z=-1e2, constraint_right_offset_x=0.0, plane_height=-0.5, collide_circle_x=0.0,
               collide_circle_y=-1.6, collide_circle_z=0.0, collide_circle_radius=1.0)
    model = ElasticityModel(cfg)
    model.timestep = 1
    for k, n in (("f", model.deformation_field), ("f_prev", model.deformation_field_prev),
                 ("f_pp", model.deformation_field_prev_prev)):
        set_flat(n, g3[f"el3d/{k}/params0"])
    T = lambda k: torch.from_numpy(g3[k]).cuda()  # noqa: E731

    def patch(it):
        model._sample_in_training = lambda res: T(f"el3d/x{it}").clone().requires_grad_(True)

    body = ElasticityModel._solve_deformation._insr_phase
    patch(0)
    model._reset_optimizer()
    ld = body(model)
    ref = float(g3["el3d/_solve_deformation/loss_main"])
    assert abs(float(ld["main"]) - ref) <= TOL * abs(ref), (float(ld["main"]), ref)
    model.optimizer.zero_grad()
    ld["main"].backward()
    assert nerr(flat_grad(model.deformation_field), g3["el3d/_solve_deformation/grad_f"]) < TOL
    set_flat(model.deformation_field, g3["el3d/f/params0"])
    model._reset_optimizer()
    trace = []
    owner = types.SimpleNamespace()
    for it in range(2):
        patch(it)
        with _jet.call_scope(owner):
            ld = body(model)
        model._update_network(ld)
        trace.append([float(ld[k]) for k in sorted(ld)])
    assert nerr(np.array(trace), g3["el3d/_solve_deformation/loss_trace"]) < TOL
    check_update(flat(model.deformation_field), g3["el3d/f/params0"], g3["el3d/_solve_deformation/f_after"],
                 g3["el3d/_solve_deformation/grad_f"])


INIT = {"advect": ("advection", "pde.advection", "Advection1DModel", "field",
                   dict(num_hidden_layers=3, hidden_features=64, sample_resolution=512, dt=0.05, vel=0.25, length=4.0,
                        init_cond="example1"), False),
        "fluid": ("fluid", "pde.fluid", "Fluid2DModel", "velocity_field",
                  dict(num_hidden_layers=4, hidden_features=128, sample_resolution=32, dt=0.05,
                       init_cond="taylorgreen"), False),
        "el2d": ("elasticity", "pde.elasticity", "ElasticityModel", "deformation_field",
                 dict(num_hidden_layers=5, hidden_features=128, sample_resolution=16, dt=0.1, dim=2,
                      energy=["arap"]), True)}


@pytest.mark.parametrize("name", sorted(INIT))
def test_initialize_phase(name):
    """The `_initialize` phases (advection/model.py:43-52, fluid/model.py:42-51,
    elasticity/model.py:109-117) vs the reference's own vectors (tests/golden/ref_init.npz):
    loss, parameter gradients, and 2 iterations of phase + Adam + plateau."""
    import importlib
    from pde.examples import get_examples
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = dict(np.load(GOLD.replace("ref_phases.npz", "ref_init.npz")))
    pde, mod, cls_name, attr, kw, takes_res = INIT[name]
    cls = getattr(importlib.import_module(mod), cls_name)
    model = cls(_cfg(pde, **kw))
    model.timestep = 0
    if "init_cond" in kw:
        model.init_cond_func = get_examples(kw["init_cond"])
    net = getattr(model, attr)
    T = lambda k: torch.from_numpy(g[k]).cuda()  # noqa: E731

    def patch(it):
        x = lambda *a: T(f"init/{name}/x{it}").clone().requires_grad_(True)  # noqa: E731
        model._sample_in_training = x

    body = cls._initialize._insr_phase
    set_flat(net, g[f"init/{name}/params0"])
    patch(0)
    model._reset_optimizer()
    ld = body(model)
    ref = float(g[f"init/{name}/loss_main"])
    assert abs(float(ld["main"]) - ref) <= TOL * abs(ref), (float(ld["main"]), ref)
    model.optimizer.zero_grad()
    ld["main"].backward()
    assert nerr(flat_grad(net), g[f"init/{name}/grad"]) < TOL
    set_flat(net, g[f"init/{name}/params0"])
    model._reset_optimizer()
    trace = []
    for it in range(2):
        patch(it)
        ld = body(model)
        model._update_network(ld)
        trace.append([float(ld[k]) for k in sorted(ld)])
    assert nerr(np.array(trace), g[f"init/{name}/loss_trace"]) < TOL
    check_update(flat(net), g[f"init/{name}/params0"], g[f"init/{name}/after"], g[f"init/{name}/grad"])


@pytest.mark.parametrize("fused", [True, False])
def test_training_loop_graph_matches_eager(ph, fused):
    """insr_graph=True (hipGraph replay) gives the same trajectory as eager execution (fused
    mixed launches and the unfused per-jet path)."""
    from pde.fluid import Fluid2DModel
    res = {}
    for graph in (False, True):
        torch.manual_seed(0)
        cfg = _cfg("fluid", num_hidden_layers=4, hidden_features=128, sample_resolution=32, max_n_iters=6,
                   insr_graph=graph, insr_sync_every=3, insr_fuse_forwards=fused)
        model = Fluid2DModel(cfg)
        set_flat(model.velocity_field, ph["fluid/vel/params0"])
        set_flat(model.velocity_field_prev, ph["fluid/vel_prev/params0"])
        set_flat(model.pressure_field, ph["fluid/pres/params0"])
        xs = [torch.from_numpy(ph["fluid/x0"]).cuda(), torch.from_numpy(ph["fluid/x1"]).cuda()]
        static_x = xs[0].clone()
        static_bx = torch.from_numpy(ph["fluid/bcx0"]).cuda()
        static_by = torch.from_numpy(ph["fluid/bcy0"]).cuda()
        model._sample_in_training = lambda: static_x.clone().requires_grad_(True)
        model._boundary_pair = lambda n: (static_bx.clone().requires_grad_(True), static_by.clone().requires_grad_(True))
        model.timestep = 1
        model._solve_pressure()
        if graph:  # the capture succeeded (a failed capture silently stays eager)
            assert getattr(model, "_insr_capture_error", None) is None
        res[graph] = (flat(model.pressure_field), float(model.optimizer.state[0]),
                      float(model.optimizer.state[1]))
    assert res[True][2] == res[False][2] == 6.0
    assert nerr(res[True][0], res[False][0]) < 1e-6


def test_training_loop_unrolled_graph_matches(ph):
    """insr_graph_unroll = U: groups of U iterations replayed as ONE graph (between the loop's host
    reads) -- the same kernels in the same order as one replay per iteration, on the product sampler
    path (each iteration's device draw advances the Philox stream inside the graph): parameters, step
    count and the device sampler position bit for bit equal to U = 1, and the losses the loop reads."""
    from pde.fluid import Fluid2DModel
    res = {}
    for U in (1, 2, 4):
        torch.manual_seed(0)
        # (frozen work ahead off: it evaluates the group's frozen jets in one launch, whose fp16 scale tiles
        # differ from the per-iteration launches -- tests/test_gpu_frozen_ahead.py compares the two)
        cfg = _cfg("fluid", num_hidden_layers=4, hidden_features=128, sample_resolution=32, max_n_iters=10,
                   insr_graph=True, insr_sync_every=4, insr_graph_unroll=U, insr_frozen_ahead=False)
        model = Fluid2DModel(cfg)
        set_flat(model.velocity_field, ph["fluid/vel/params0"])
        set_flat(model.velocity_field_prev, ph["fluid/vel_prev/params0"])
        set_flat(model.pressure_field, ph["fluid/pres/params0"])
        model.timestep = 1
        seen = []
        model.tb = type("TB", (), {"add_scalars": lambda self, tag, vals, global_step: seen.append(
            (global_step, vals["main"]))})()
        model._solve_pressure()
        assert getattr(model, "_insr_capture_error", None) is None
        res[U] = (flat(model.pressure_field), float(model.optimizer.state[1]), seen)
    for U in (2, 4):
        assert res[U][1] == res[1][1] == 10.0
        assert np.array_equal(res[U][0], res[1][0]), U
        assert res[U][2] == res[1][2], U  # the same iterations read, the same losses


@pytest.mark.parametrize("policy", [None, 5])
@pytest.mark.parametrize("graph", [False, True])
def test_fused_sums_adam_bit_identical(ph, graph, policy):
    """base._jet.defer_reductions: a reverse jet's sums run inside the Adam launch -- a fused-path
    value backward's partial rows (insr_adam_step_partials; default policy) and, under policy 5, the
    resident sweep's dW sums of every jet (insr_siren_jet_bwd_grad_adam phase 2, the pressure
    Laplacian jet included) -- the same sums in the same order and the same update, so the advect /
    pressure / projection loops end with parameters, optimiser moments and state, and the flat .grad
    bit for bit equal to the separate sums + Adam launches (DEFER_REDUCE off), eager and
    graph-replayed."""
    import contextlib
    from pde.fluid import Fluid2DModel
    import base
    res = {}
    for defer in (False, True):
        _jet.DEFER_REDUCE = defer
        scope = base._native.knobs(policy=policy) if policy is not None else contextlib.nullcontext()
        try:
            with scope:
                torch.manual_seed(0)
                # (without in-kernel loss seeds, which need the deferred sums: the loss values and the
                # plateau state come from the same launches in both runs; tests/test_gpu_seeds.py)
                cfg = _cfg("fluid", num_hidden_layers=4, hidden_features=128, sample_resolution=32, max_n_iters=6,
                           insr_graph=graph, insr_sync_every=3, insr_seed_in_bwd=False)
                model = Fluid2DModel(cfg)
                set_flat(model.velocity_field, ph["fluid/vel/params0"])
                set_flat(model.velocity_field_prev, ph["fluid/vel_prev/params0"])
                set_flat(model.pressure_field, ph["fluid/pres/params0"])
                model.timestep = 1
                out = []
                for phase in ("_advect_velocity", "_solve_pressure", "_projection"):
                    getattr(model, phase)()
                    assert getattr(model, "_insr_capture_error", None) is None
                    torch.cuda.synchronize()
                    opt = model.optimizer
                    fused = getattr(opt, "partials_steps", 0) > 0
                    assert fused == defer or (phase == "_solve_pressure" and policy is None and not fused)
                    out += [opt._nets[0][1].cpu().numpy(), opt._nets[0][2].cpu().numpy(), opt._nets[1][1].cpu().numpy(),
                            opt._nets[1][2].cpu().numpy(), opt.state.cpu().numpy()]
                out += [flat(model.velocity_field), flat(model.pressure_field), flat_grad(model.velocity_field),
                        flat_grad(model.pressure_field)]
                res[defer] = out
                for net in (model.velocity_field, model.pressure_field):
                    assert "_insr_pending_reduce" not in net.__dict__
        finally:
            _jet.DEFER_REDUCE = True
    for a, b in zip(res[False], res[True]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("dim", [2, 3])
def test_plain_elasticity_body_through_lowering(ph, dim):
    """The reference's elasticity body as written (pde/elasticity_plain.py: q = f(x) + x, jacobian, torch.svd,
    torch energy sums, separate constraint calls) run the way the loop runs an unchanged model file -- inside
    base.lower's lowering() + deferred_jets() scopes.  None of its energies is lowered (no mean squares): every
    expression runs eagerly through the Lazy tensors' fallback, and the deferred jets are launched at the first
    read.  Losses, gradients and two Adam + plateau iterations against the reference's golden vectors."""
    from base import lower as LW
    from pde.elasticity_plain import ElasticityPlainModel
    if dim == 2:
        g = ph
        energy = [str(e) for e in g["el2d/cfg_energy"]]
        cfg = _cfg("elasticity", num_hidden_layers=5, hidden_features=128, sample_resolution=16, dt=0.1, dim=2,
                   energy=energy, ratio_constraint=1e4, ratio_volume=1e3, ratio_arap=1.0, ratio_collide=1e2,
                   ratio_kinematics=1.0, external_force_timesteps=5, external_force_y=-1.0,
                   constraint_right_offset_x=2.0, plane_height=-0.9)
        pre = "el2d"
    else:
        g = dict(np.load(GOLD.replace("ref_phases.npz", "ref_phases_el3d.npz")))
        energy = [str(e) for e in g["el3d/cfg_energy"]]
        cfg = _cfg("elasticity", num_hidden_layers=2, hidden_features=64, sample_resolution=6, dt=0.1, dim=3,
                   energy=energy, ratio_constraint=1e4, ratio_volume=1e3, ratio_arap=1e2, ratio_collide=1e3,
                   ratio_kinematics=1.0, external_force_timesteps=5, external_force_x=0.0, external_force_y=0.0,
                   external_force_z=-1e2, constraint_right_offset_x=0.0, plane_height=-0.5, collide_circle_x=0.0,
                   collide_circle_y=-1.6, collide_circle_z=0.0, collide_circle_radius=1.0)
        pre = "el3d"
    model = ElasticityPlainModel(cfg)
    model.timestep = 1
    for k, n in (("f", model.deformation_field), ("f_prev", model.deformation_field_prev),
                 ("f_pp", model.deformation_field_prev_prev)):
        set_flat(n, g[f"{pre}/{k}/params0"])
    T = lambda k: torch.from_numpy(g[k]).cuda()  # noqa: E731

    def patch(it):
        model._sample_in_training = lambda res: T(f"{pre}/x{it}").clone().requires_grad_(True)
        if dim == 2:
            model._sample_fixed_in_training = lambda res: (T(f"el2d/fixed_l{it}").clone().requires_grad_(True),
                                                           T(f"el2d/fixed_r{it}").clone().requires_grad_(True))

    body = ElasticityPlainModel._solve_deformation._insr_phase
    assert model._lower_on() and model._defer_on()

    def run():
        with LW.lowering(model._lower_on()), LW.deferred_jets(model._defer_on()):
            ld = body(model)
        return LW.lower_losses(ld)

    patch(0)
    model._reset_optimizer()
    ld = run()
    ref = float(g[f"{pre}/_solve_deformation/loss_main"])
    assert abs(float(ld["main"]) - ref) <= TOL * abs(ref), (float(ld["main"]), ref)
    model.optimizer.zero_grad()
    model._backward(ld)
    assert nerr(flat_grad(model.deformation_field), g[f"{pre}/_solve_deformation/grad_f"]) < TOL
    set_flat(model.deformation_field, g[f"{pre}/f/params0"])
    model._reset_optimizer()
    trace = []
    owner = types.SimpleNamespace()
    for it in range(2):
        patch(it)
        with _jet.call_scope(owner):
            ld = run()
        model._update_network(ld)
        trace.append([float(ld[k]) for k in sorted(ld)])
    assert nerr(np.array(trace), g[f"{pre}/_solve_deformation/loss_trace"]) < TOL
    check_update(flat(model.deformation_field), g[f"{pre}/f/params0"], g[f"{pre}/_solve_deformation/f_after"],
                 g[f"{pre}/_solve_deformation/grad_f"])
