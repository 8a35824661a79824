"""Pin the CPU oracle against golden vectors recorded from the reference itself.

Fixtures: tests/golden/ref_ops.npz, ref_phases.npz (made by tests/golden/make_golden.py,
which imports /root/reference in the build container).  These tests need only numpy +
torch and run on the CPU.
"""
import os

import numpy as np
import pytest
import torch

from oracle import siren_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def ops():
    return dict(np.load(os.path.join(GOLD, "ref_ops.npz")))


@pytest.fixture(scope="module")
def phases():
    return dict(np.load(os.path.join(GOLD, "ref_phases.npz")))


def nrm(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


def seeded(din, dout, L, W, seed):
    torch.manual_seed(int(seed))
    return O.OracleSiren(din, dout, L, W)


def set_flat(net, vec):
    off = 0
    with torch.no_grad():
        for p in net.parameters():
            n = p.numel()
            p.copy_(torch.from_numpy(np.asarray(vec[off:off + n])).view_as(p))
            off += n


CASES = ["advect", "fluid_vel", "fluid_pres", "el2d", "el3d"]


@pytest.mark.parametrize("name", CASES)
def test_init_bit_exact(ops, name):
    din, dout, L, W = ops[f"{name}/shape"]
    net = seeded(din, dout, L, W, ops[f"{name}/seed"])
    stride = int(ops[f"{name}/param_stride"])
    got = O.flat_params(net).numpy()[::stride]
    assert np.array_equal(got, ops[f"{name}/params"])
    # state_dict keys identical to the reference layout net.{0,2,..}.{weight,bias}
    keys = list(net.state_dict().keys())
    assert keys[0] == "net.0.weight" and keys[-1] == f"net.{2 * (L + 1)}.bias"


@pytest.mark.parametrize("name", CASES)
def test_diff_ops_and_param_grads(ops, name):
    din, dout, L, W = ops[f"{name}/shape"]
    net = seeded(din, dout, L, W, ops[f"{name}/seed"])
    stride = int(ops[f"{name}/param_stride"])
    x = torch.from_numpy(ops[f"{name}/x"]).requires_grad_(True)
    y = net(x)
    assert nrm(y.detach(), ops[f"{name}/y"]) < 1e-6
    fns = {"gradient": lambda: O.op_gradient(y, x), "divergence": lambda: O.op_divergence(y, x),
           "laplace": lambda: O.op_laplace(y, x), "jacobian": lambda: O.op_jacobian(y, x)[0]}
    for op, fn in fns.items():
        if f"{name}/{op}" not in ops:
            continue
        val = fn()
        assert nrm(val.detach(), ops[f"{name}/{op}"]) < 1e-6, op
        net.zero_grad(set_to_none=True)
        (val * torch.from_numpy(ops[f"{name}/{op}_R"])).sum().backward(retain_graph=True)
        assert nrm(O.flat_grads(net).numpy()[::stride], ops[f"{name}/{op}_pgrad"]) < 1e-6, op
    if f"{name}/hessian" in ops:
        x3 = x.detach()[None].clone().requires_grad_(True)
        h, st = O.op_hessian(net(x3), x3)
        assert st == int(ops[f"{name}/hessian_status"])
        assert nrm(h.detach(), ops[f"{name}/hessian"]) < 1e-6
    net.zero_grad(set_to_none=True)
    (net(x) * torch.from_numpy(ops[f"{name}/value_R"])).sum().backward()
    assert nrm(O.flat_grads(net).numpy()[::stride], ops[f"{name}/value_pgrad"]) < 1e-6


def test_samplers(ops):
    assert np.array_equal(O.sample_uniform(8, 2).numpy(), ops["sampling/uniform_8_2"])
    assert np.array_equal(O.sample_uniform(5, 1).numpy(), ops["sampling/uniform_5_1"])
    assert np.array_equal(O.sample_uniform(4, 3).numpy(), ops["sampling/uniform_4_3"])
    torch.manual_seed(6)
    assert np.array_equal(O.sample_random(100, 2).numpy(), ops["sampling/random_seed6_100x2"])
    torch.manual_seed(8)
    assert np.array_equal(O.sample_boundary2d_side(20, "horizontal").numpy(), ops["sampling/bnd2d_h_seed8_20"])
    torch.manual_seed(9)
    assert np.array_equal(O.sample_boundary1d(20).numpy(), ops["sampling/bnd1d_seed9_20"])


def _nets(ph, prefix, specs):
    nets = {}
    for name, (din, dout, L, W) in specs.items():
        n = O.OracleSiren(din, dout, L, W)
        set_flat(n, ph[f"{prefix}/{name}/params0"])
        nets[name] = n
    return nets


def _run(nets, trainable, loss_fn, n_iters, lr=1e-4):
    opt = O.OracleAdam([p for k in trainable for p in nets[k].parameters()], lr=lr)
    trace = []
    for it in range(n_iters):
        ld = loss_fn(it)
        O.update_step([nets[k] for k in trainable], ld, opt)
        trace.append([float(ld[k]) for k in sorted(ld)])
    return np.array(trace)


def test_fluid_phases(phases):
    ph = phases
    specs = {"vel": (2, 2, 4, 128), "vel_prev": (2, 2, 4, 128), "pres": (2, 1, 4, 128)}
    T = lambda k: torch.from_numpy(ph[k])  # noqa: E731
    X = lambda it: T(f"fluid/x{it}").clone().requires_grad_(True)  # noqa: E731
    BX = lambda it: T(f"fluid/bcx{it}").clone().requires_grad_(True)  # noqa: E731
    BY = lambda it: T(f"fluid/bcy{it}").clone().requires_grad_(True)  # noqa: E731
    fns = {
        "_advect_velocity": lambda n, it: O.fluid_advect_loss(n["vel"], n["vel_prev"], X(it), BX(it), BY(it), 0.05),
        "_solve_pressure": lambda n, it: O.fluid_pressure_loss(n["vel"], n["pres"], X(it), BX(it), BY(it)),
        "_projection": lambda n, it: O.fluid_projection_loss(n["vel"], n["vel_prev"], n["pres"], X(it), BX(it),
                                                             BY(it)),
    }
    for phase, fn in fns.items():
        nets = _nets(ph, "fluid", specs)
        ld = fn(nets, 0)
        for k, v in ld.items():
            assert abs(float(v) - float(ph[f"fluid/{phase}/loss_{k}"])) <= 1e-6 * abs(
                float(ph[f"fluid/{phase}/loss_{k}"])) + 1e-12, (phase, k)
        sum(ld.values()).backward()
        assert nrm(O.flat_grads(nets["vel"]), ph[f"fluid/{phase}/grad_vel"]) < 1e-5, phase
        if np.abs(ph[f"fluid/{phase}/grad_pres"]).max() > 0:
            assert nrm(O.flat_grads(nets["pres"]), ph[f"fluid/{phase}/grad_pres"]) < 1e-5, phase
        nets = _nets(ph, "fluid", specs)
        trace = _run(nets, ["vel", "pres"], lambda it: fn(nets, it), 2)
        assert nrm(trace, ph[f"fluid/{phase}/loss_trace"]) < 1e-5
        # after Adam: compare the update (p - p0) normwise, scaled to lr
        for k, key in (("vel", "vel_after"), ("pres", "pres_after")):
            d_ref = ph[f"fluid/{phase}/{key}"] - ph[f"fluid/{k}/params0"]
            d_got = O.flat_params(nets[k]).numpy() - ph[f"fluid/{k}/params0"]
            if np.abs(d_ref).max() > 0:
                assert nrm(d_got, d_ref) < 1e-3, (phase, k)


def test_advect_phase(phases):
    ph = phases
    specs = {"field": (1, 1, 3, 64), "field_prev": (1, 1, 3, 64)}
    X = lambda it: torch.from_numpy(ph[f"advect/x{it}"]).clone().requires_grad_(True)  # noqa: E731
    B = lambda it: torch.from_numpy(ph[f"advect/bc{it}"]).clone()  # noqa: E731
    nets = _nets(ph, "advect", specs)
    ld = O.advect1d_loss(nets["field"], nets["field_prev"], X(0), B(0), 0.05, 0.25)
    for k, v in ld.items():
        assert abs(float(v) - float(ph[f"advect/_advect/loss_{k}"])) <= 1e-6 * abs(float(v)) + 1e-12
    sum(ld.values()).backward()
    assert nrm(O.flat_grads(nets["field"]), ph["advect/_advect/grad_field"]) < 1e-5
    nets = _nets(ph, "advect", specs)
    trace = _run(nets, ["field"], lambda it: O.advect1d_loss(nets["field"], nets["field_prev"], X(it), B(it),
                                                             0.05, 0.25), 2)
    assert nrm(trace, ph["advect/_advect/loss_trace"]) < 1e-5
    d_ref = ph["advect/_advect/field_after"] - ph["advect/field/params0"]
    d_got = O.flat_params(nets["field"]).numpy() - ph["advect/field/params0"]
    assert nrm(d_got, d_ref) < 1e-3


def el2d_cfg(energy):
    return dict(dt=0.1, energy=list(energy), ratio_arap=1.0, ratio_volume=1e3, ratio_kinematics=1.0,
                ratio_constraint=1e4, ratio_collide=1e2, plane_height=-0.9, external_force=[0.0, -1.0],
                constraint_offset_right=[2.0, 0.0], circle_center=[0.0, -2.0], circle_radius=1.0,
                external_force_timesteps=5)


def test_elasticity_phase(phases):
    ph = phases
    specs = {"f": (2, 2, 5, 128), "f_prev": (2, 2, 5, 128), "f_pp": (2, 2, 5, 128)}
    cfg = el2d_cfg([str(e) for e in ph["el2d/cfg_energy"]])
    X = lambda it: torch.from_numpy(ph[f"el2d/x{it}"]).clone().requires_grad_(True)  # noqa: E731
    FL = lambda it: torch.from_numpy(ph[f"el2d/fixed_l{it}"]).clone().requires_grad_(True)  # noqa: E731
    FR = lambda it: torch.from_numpy(ph[f"el2d/fixed_r{it}"]).clone().requires_grad_(True)  # noqa: E731
    nets = _nets(ph, "el2d", specs)
    ld = O.elasticity_loss(nets["f"], nets["f_prev"], nets["f_pp"], X(0), FL(0), FR(0), cfg, timestep=1)
    ref = float(ph["el2d/_solve_deformation/loss_main"])
    assert abs(float(ld["main"]) - ref) <= 1e-5 * abs(ref)
    ld["main"].backward()
    assert nrm(O.flat_grads(nets["f"]), ph["el2d/_solve_deformation/grad_f"]) < 1e-5
    nets = _nets(ph, "el2d", specs)
    trace = _run(nets, ["f"], lambda it: O.elasticity_loss(nets["f"], nets["f_prev"], nets["f_pp"], X(it), FL(it),
                                                           FR(it), cfg, timestep=1), 2)
    assert nrm(trace, ph["el2d/_solve_deformation/loss_trace"]) < 1e-5


def test_elasticity3d_phase():
    """The 3-D energy set (3x3 singular values, plane + sphere collisions incl. the
    reference's (K, K, 3) sphere-force broadcast, external force, kinematics)."""
    ph = dict(np.load(os.path.join(GOLD, "ref_phases_el3d.npz")))
    specs = {"f": (3, 3, 2, 64), "f_prev": (3, 3, 2, 64), "f_pp": (3, 3, 2, 64)}
    cfg = dict(dt=0.1, energy=[str(e) for e in ph["el3d/cfg_energy"]], ratio_arap=1e2, ratio_volume=1e3,
               ratio_kinematics=1.0, ratio_constraint=1e4, ratio_collide=1e3, plane_height=-0.5,
               external_force=[0.0, 0.0, -1e2], constraint_offset_right=[0.0, 0.0, 0.0],
               circle_center=[0.0, -1.6, 0.0], circle_radius=1.0, external_force_timesteps=5)
    X = lambda it: torch.from_numpy(ph[f"el3d/x{it}"]).clone().requires_grad_(True)  # noqa: E731
    nets = _nets(ph, "el3d", specs)
    ld = O.elasticity_loss(nets["f"], nets["f_prev"], nets["f_pp"], X(0), None, None, cfg, timestep=1)
    ref = float(ph["el3d/_solve_deformation/loss_main"])
    assert abs(float(ld["main"]) - ref) <= 1e-5 * abs(ref)
    ld["main"].backward()
    assert nrm(O.flat_grads(nets["f"]), ph["el3d/_solve_deformation/grad_f"]) < 1e-5
    nets = _nets(ph, "el3d", specs)
    trace = _run(nets, ["f"], lambda it: O.elasticity_loss(nets["f"], nets["f_prev"], nets["f_pp"], X(it), None,
                                                           None, cfg, timestep=1), 2)
    assert nrm(trace, ph["el3d/_solve_deformation/loss_trace"]) < 1e-5


INIT_CASES = {"advect": ((1, 1, 3, 64), O.advect1d_init_loss), "fluid": ((2, 2, 4, 128), O.fluid_init_loss),
              "el2d": ((2, 2, 5, 128), O.elasticity_init_loss)}


@pytest.mark.parametrize("name", sorted(INIT_CASES))
def test_initialize_phases(name):
    """The `_initialize` phases (advection/model.py:43-52, fluid/model.py:42-51,
    elasticity/model.py:109-117) vs tests/golden/ref_init.npz: loss, parameter gradients, and
    the loss trace + update of 2 reference iterations."""
    ph = dict(np.load(os.path.join(GOLD, "ref_init.npz")))
    shape, fn = INIT_CASES[name]
    X = lambda it: torch.from_numpy(ph[f"init/{name}/x{it}"]).clone().requires_grad_(True)  # noqa: E731
    nets = _nets(ph, "init", {name: shape})
    ld = fn(nets[name], X(0))
    ref = float(ph[f"init/{name}/loss_main"])
    assert abs(float(ld["main"]) - ref) <= 1e-6 * abs(ref)
    ld["main"].backward()
    assert nrm(O.flat_grads(nets[name]), ph[f"init/{name}/grad"]) < 1e-5
    nets = _nets(ph, "init", {name: shape})
    trace = _run(nets, [name], lambda it: fn(nets[name], X(it)), 2)
    assert nrm(trace, ph[f"init/{name}/loss_trace"]) < 1e-5
    d_ref = ph[f"init/{name}/after"] - ph[f"init/{name}/params0"]
    d_got = O.flat_params(nets[name]).numpy() - ph[f"init/{name}/params0"]
    assert nrm(d_got, d_ref) < 1e-3


def test_plateau_matches_torch():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1e-4)
    sch = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, factor=0.1, patience=3, min_lr=1e-8)
    mine = O.OraclePlateau(1e-4, factor=0.1, patience=3, min_lr=1e-8)
    rng = np.random.default_rng(0)
    vals = list(rng.random(40)) + [1.0] * 40
    for v in vals:
        sch.step(v)
        lr = mine.step(v)
        assert lr == opt.param_groups[0]["lr"]
