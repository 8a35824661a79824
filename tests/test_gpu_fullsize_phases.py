"""One full iteration of the headline models at their BASELINE.json sizes, against the CPU
oracle (oracle/siren_oracle.py, pinned to the reference's own vectors by
tests/test_oracle_golden.py) on the SAME points:

  * fluid2Dtlgn   fused pde/fluid.py phases at 128^2 = 16,384 interior points + 2 x 162 bands
  * fluid2DtlgnM  the same at 256^2 = 65,536 + 2 x 654
  * elasticity2Dstretch  _solve_deformation at 20,000 points (SIREN 5x128) + 2 x 200 fixed
  * advect1D     _advect at 4,096 interior + 2 x 20 band points (SIREN 3x64)
  * the reference's own bodies (pde/fluid_plain.py, pde/advection_plain.py, pde/elasticity_plain.py) at the
    fluid2Dtlgn, advect1D and elasticity2Dstretch sizes, through the training loop's loss lowering and
    deferred jets (the drop-in path)

The GPU runs the product path exactly as bench.py does -- device sampler into the merged
[interior; bands] buffer (fluid) / the persistent box batch (elasticity), mixed launches,
loss groups, the fused energy, Adam + plateau in one launch -- and the test reads back the
points that path drew and hands them to the oracle (fluid/model.py:72-151,
elasticity/model.py:127-189, base/baseModel.py:73-81).  A second fluid2Dtlgn case feeds
recorded samples through the _sample_in_training / _boundary_pair hooks (as
test_gpu_phases.py does at 32^2).

Checks per phase: every loss (1e-5 relative), every parameter tensor's gradient (1e-5
normwise, each weight and bias on its own), and the parameters after the Adam step (updates
compared on entries whose gradient is well above the noise floor, as test_gpu_phases)."""
import numpy as np
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
    torch.set_num_threads(min(16, torch.get_num_threads()))
    return base


def nerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def seeded(din, dout, L, W, seed):
    torch.manual_seed(seed)
    return O.OracleSiren(din, dout, L, W)


def load(net, ref):
    with torch.no_grad():
        net.flat_params().copy_(O.flat_params(ref).cuda())


def per_tensor(flat, ref):
    """Split a flat vector in the reference's state_dict order: {name: array}."""
    out, off = {}, 0
    for k, p in ref.named_parameters():
        out[k] = flat[off:off + p.numel()]
        off += p.numel()
    return out


def check_grads(net, ref, what):
    got = net.flat_grad_buffer().detach().cpu().numpy() if net.grad_touched() else np.zeros(net.param_count)
    want = O.flat_grads(ref).numpy()
    if np.abs(want).max() == 0:
        assert not net.grad_touched(), what
        return
    g, w = per_tensor(got, ref), per_tensor(want, ref)
    for k in w:
        if np.abs(w[k]).max() > 0:
            assert nerr(g[k], w[k]) < TOL, (what, k, nerr(g[k], w[k]))
        else:
            assert np.abs(g[k]).max() == 0, (what, k)


def check_update(net, ref, p0, lr):
    got = net.flat_params().detach().cpu().numpy() - p0
    want = O.flat_params(ref).numpy() - p0
    g = O.flat_grads(ref).numpy()
    if np.abs(g).max() == 0:
        assert np.abs(got).max() == 0
        return
    mask = np.abs(g) > 1e-3 * np.abs(g).max()
    assert mask.sum() > 0.5 * mask.size
    assert nerr(got[mask], want[mask]) < 1e-3
    assert np.abs(got - want).max() <= 2 * lr * 1.01  # noise-floor entries may flip sign


# ---------------------------------------------------------------------------------------------
def _fluid(B, config, hooks, plain=False, **over):
    from pde.config import baseline_config
    from pde.fluid import Fluid2DModel
    from pde.fluid_plain import Fluid2DPlainModel
    import pde.fluid as fl
    import pde.fluid_plain as fp
    from base import lower as LW
    cfg = baseline_config(config, proj_dir="/tmp/insr_fullsize_phases", insr_progress=False, early_stop=False,
                          max_n_iters=1, insr_graph=False, insr_sync_every=1, **over)
    cls = Fluid2DPlainModel if plain else Fluid2DModel
    m = cls(cfg)
    m.timestep = 1
    refs = {"vel": seeded(2, 2, 4, 128, 201), "vel_prev": seeded(2, 2, 4, 128, 202), "pres": seeded(2, 1, 4, 128, 203)}
    nets = {"vel": m.velocity_field, "vel_prev": m.velocity_field_prev, "pres": m.pressure_field}
    N = getattr(cfg, "insr_points_per_rank", None) or cfg.sample_resolution ** 2
    nb = N // 100
    gen = torch.Generator().manual_seed(301)
    drawn = {}
    if hooks:
        x = torch.rand(N, 2, generator=gen) * 2 - 1
        bx = O.sample_boundary2d_side(nb, "horizontal", generator=gen)
        by = O.sample_boundary2d_side(nb, "vertical", generator=gen)
        m._sample_in_training = lambda: x.cuda().requires_grad_(True)
        m._boundary_pair = lambda n: (bx.cuda().requires_grad_(True), by.cuda().requires_grad_(True))
        drawn["pts"] = (x, bx, by)
        if plain:  # the reference bodies' separate band samplers (x-faces, then y-faces)
            orig_sep = fp.sample_boundary2D_separate
            fp.sample_boundary2D_separate = lambda n, side, device=None: (bx if side == "horizontal" else by).cuda()
            drawn["restore"] = lambda: setattr(fp, "sample_boundary2D_separate", orig_sep)
    else:  # the product sampler: record the merged buffer it draws
        orig = fl.sample_random_and_bands2D

        def rec(n, n_band, **kw):
            buf = orig(n, n_band, **kw)
            h = (buf.shape[0] - n) // 2
            b = buf.detach().cpu()
            drawn["pts"] = (b[:n].clone(), b[n:n + h].clone(), b[n + h:].clone())
            return buf
        fl.sample_random_and_bands2D = rec
        drawn["restore"] = lambda: setattr(fl, "sample_random_and_bands2D", orig)
    oracle = {
        "_advect_velocity": lambda r, x, bx, by: O.fluid_advect_loss(r["vel"], r["vel_prev"], x, bx, by, cfg.dt),
        "_solve_pressure": lambda r, x, bx, by: O.fluid_pressure_loss(r["vel"], r["pres"], x, bx, by),
        "_projection": lambda r, x, bx, by: O.fluid_projection_loss(r["vel"], r["vel_prev"], r["pres"], x, bx, by),
    }
    try:
        for phase, fn in oracle.items():
            for k in nets:
                load(nets[k], refs[k])
            p0 = {k: O.flat_params(refs[k]).numpy().copy() for k in ("vel", "pres")}
            m._reset_optimizer()
            body = getattr(cls, phase)._insr_phase
            if plain:  # as the training loop runs an unchanged model file: lowered, jets deferred
                with LW.lowering(m._lower_on()), LW.deferred_jets(m._defer_on()):
                    ld = body(m)
                ld = LW.lower_losses(ld)
            else:
                ld = body(m)
            m._update_network(ld)
            torch.cuda.synchronize()
            assert len(ld) == 2
            x, bx, by = drawn["pts"]
            assert x.shape[0] == N and bx.shape[0] == by.shape[0] == 2 * (nb // 2)
            r = {k: seeded(*s, seed) for k, s, seed in (("vel", (2, 2, 4, 128), 201), ("vel_prev", (2, 2, 4, 128), 202),
                                                         ("pres", (2, 1, 4, 128), 203))}
            for p in r["vel_prev"].parameters():
                p.requires_grad_(False)
            opt = O.OracleAdam([p for k in ("vel", "pres") for p in r[k].parameters()], lr=cfg.lr)
            ldo = fn(r, x.clone().requires_grad_(True), bx.clone().requires_grad_(True), by.clone().requires_grad_(True))
            O.update_step([r["vel"], r["pres"]], ldo, opt)
            for k, v in ldo.items():
                assert abs(float(ld[k]) - float(v)) <= TOL * abs(float(v)) + 1e-12, (phase, k, float(ld[k]), float(v))
            for k in ("vel", "pres"):
                check_grads(nets[k], r[k], (phase, k))
                check_update(nets[k], r[k], p0[k], cfg.lr)
    finally:
        if "restore" in drawn:
            drawn["restore"]()


def test_fluid2dtlgn_phases_full_size(B):
    _fluid(B, "fluid2Dtlgn", hooks=False)


def test_fluid2dtlgn_phases_full_size_recorded_samples(B):
    _fluid(B, "fluid2Dtlgn", hooks=True)


def test_fluid2dtlgn_plain_phases_full_size(B):
    """The reference's fluid bodies as written (pde/fluid_plain.py) at the headline size, through the
    training loop's loss lowering and deferred jets -- the drop-in path of bench.py --api plain -- against
    the oracle on the same 16,384 + 2 x 162 points."""
    _fluid(B, "fluid2Dtlgn", hooks=True, plain=True)


def test_fluid2dtlgnM_phases_full_size(B):
    _fluid(B, "fluid2DtlgnM", hooks=False)


def test_fluid2dtlgnM_rank_shard_size(B):
    """One rank's batch of the 8-rank strong-scaling fluid2DtlgnM run (bench.py --shard-of 8):
    65,536 / 8 = 8,192 interior + 2 x 82 band points (the tile count -- 523 tiles of 16 on 256 CUs --
    is the shard's quantisation case)."""
    _fluid(B, "fluid2DtlgnM", hooks=False, insr_points_per_rank=8192)


def test_elasticity2dstretch_full_size(B):
    """elasticity2Dstretch (scripts/elasticity2Dstretch.sh: SIREN 5x128, sample_resolution 100,
    arap + constraint + constraint_right + volume): one iteration on the 20,000 interior + 400
    fixed points the persistent box batch draws, vs the oracle's energy on the same points."""
    from pde.config import baseline_config
    from pde.elasticity import ElasticityModel
    cfg = baseline_config("elasticity2Dstretch", proj_dir="/tmp/insr_fullsize_el2d", insr_progress=False,
                          early_stop=False, max_n_iters=1, insr_graph=False, insr_sync_every=1)
    m = ElasticityModel(cfg)
    m.timestep = 1
    refs = {"f": seeded(2, 2, 5, 128, 211), "f_prev": seeded(2, 2, 5, 128, 212), "f_pp": seeded(2, 2, 5, 128, 213)}
    for k, net in (("f", m.deformation_field), ("f_prev", m.deformation_field_prev),
                   ("f_pp", m.deformation_field_prev_prev)):
        load(net, refs[k])
    p0 = O.flat_params(refs["f"]).numpy().copy()
    m._reset_optimizer()
    ld = ElasticityModel._solve_deformation._insr_phase(m)
    m._update_network(ld)
    torch.cuda.synchronize()
    (buf, _, x, fixed_l, fixed_r), = m.__dict__["_insr_box_batch"].values()
    x, fl_, fr_ = (t.detach().cpu().clone() for t in (x, fixed_l, fixed_r))
    assert x.shape[0] == 20000 and fl_.shape[0] == fr_.shape[0] == 200
    ecfg = dict(dt=cfg.dt, energy=list(cfg.energy), ratio_arap=cfg.ratio_arap, ratio_volume=cfg.ratio_volume,
                ratio_kinematics=cfg.ratio_kinematics, ratio_constraint=cfg.ratio_constraint,
                ratio_collide=cfg.ratio_collide, plane_height=cfg.plane_height,
                external_force=[cfg.external_force_x, cfg.external_force_y],
                constraint_offset_right=[cfg.constraint_right_offset_x, cfg.constraint_right_offset_y],
                circle_center=[cfg.collide_circle_x, cfg.collide_circle_y], circle_radius=cfg.collide_circle_radius,
                external_force_timesteps=cfg.external_force_timesteps)
    r = {k: seeded(2, 2, 5, 128, s) for k, s in (("f", 211), ("f_prev", 212), ("f_pp", 213))}
    for k in ("f_prev", "f_pp"):
        for p in r[k].parameters():
            p.requires_grad_(False)
    opt = O.OracleAdam(list(r["f"].parameters()), lr=cfg.lr)
    ldo = O.elasticity_loss(r["f"], r["f_prev"], r["f_pp"], x.requires_grad_(True), fl_.requires_grad_(True),
                            fr_.requires_grad_(True), ecfg, timestep=1)
    O.update_step([r["f"]], ldo, opt)
    assert abs(float(ld["main"]) - float(ldo["main"])) <= TOL * abs(float(ldo["main"])), (float(ld["main"]),
                                                                                             float(ldo["main"]))
    check_grads(m.deformation_field, r["f"], "el2d")
    check_update(m.deformation_field, r["f"], p0, cfg.lr)


def test_elasticity3d_sphere_collision(B):
    """A 3-D box scene whose energy holds collision_sphere (elasticity/losses.py:22-39: the reference's
    dist[:, None, None] * dir broadcast makes the 3-D term -dt r_c (sum dist) (sum qdot . dir)), one
    iteration through the fused energy launch and its gradient pass, vs the oracle's literal broadcast on
    the same points.  The sphere is placed inside the box so that a large share of the points collide."""
    from pde.config import make_config
    from pde.elasticity import ElasticityModel
    energy = ["arap", "kinematics", "collision_sphere", "external", "volume"]
    cfg = make_config("elasticity", proj_dir="/tmp/insr_el3d_sphere", insr_progress=False, early_stop=False,
                      max_n_iters=1, insr_graph=False, insr_sync_every=1, dim=3, num_hidden_layers=3,
                      hidden_features=64, sample_resolution=12, dt=0.1, energy=energy, ratio_collide=1e3,
                      collide_circle_x=0.1, collide_circle_y=-0.4, collide_circle_z=0.2, collide_circle_radius=0.8)
    m = ElasticityModel(cfg)
    m.timestep = 1
    refs = {"f": seeded(3, 3, 3, 64, 221), "f_prev": seeded(3, 3, 3, 64, 222), "f_pp": seeded(3, 3, 3, 64, 223)}
    for k, net in (("f", m.deformation_field), ("f_prev", m.deformation_field_prev),
                   ("f_pp", m.deformation_field_prev_prev)):
        load(net, refs[k])
    p0 = O.flat_params(refs["f"]).numpy().copy()
    m._reset_optimizer()
    ld = ElasticityModel._solve_deformation._insr_phase(m)
    m._update_network(ld)
    torch.cuda.synchronize()
    (buf, _, x, _, _), = m.__dict__["_insr_box_batch"].values()
    x = x.detach().cpu().clone()
    dist = (x - torch.tensor([0.1, -0.4, 0.2])).norm(dim=1)
    assert x.shape[1] == 3 and int((dist < 0.8).sum()) > 0.1 * x.shape[0]
    ecfg = dict(dt=cfg.dt, energy=energy, ratio_arap=cfg.ratio_arap, ratio_volume=cfg.ratio_volume,
                ratio_kinematics=cfg.ratio_kinematics, ratio_constraint=cfg.ratio_constraint,
                ratio_collide=cfg.ratio_collide, plane_height=cfg.plane_height,
                external_force=[cfg.external_force_x, cfg.external_force_y, cfg.external_force_z],
                constraint_offset_right=[cfg.constraint_right_offset_x, cfg.constraint_right_offset_y,
                                         cfg.constraint_right_offset_z],
                circle_center=[0.1, -0.4, 0.2], circle_radius=0.8,
                external_force_timesteps=cfg.external_force_timesteps)
    r = {k: seeded(3, 3, 3, 64, s) for k, s in (("f", 221), ("f_prev", 222), ("f_pp", 223))}
    for k in ("f_prev", "f_pp"):
        for p in r[k].parameters():
            p.requires_grad_(False)
    opt = O.OracleAdam(list(r["f"].parameters()), lr=cfg.lr)
    empty = torch.zeros(0, 3)
    ldo = O.elasticity_loss(r["f"], r["f_prev"], r["f_pp"], x.requires_grad_(True), empty, empty, ecfg, timestep=1)
    O.update_step([r["f"]], ldo, opt)
    assert abs(float(ld["main"]) - float(ldo["main"])) <= TOL * abs(float(ldo["main"])), (float(ld["main"]),
                                                                                             float(ldo["main"]))
    check_grads(m.deformation_field, r["f"], "el3d sphere")
    check_update(m.deformation_field, r["f"], p0, cfg.lr)


@pytest.mark.parametrize("fused", [False, True])
def test_advect1d_full_size(B, fused):
    """advect1D (BASELINE.json configs[0]: SIREN 3x64, sample_resolution 4,096): one _advect iteration
    on the product path -- fused=False: ONE insr_sample_boxes launch writes the 4,096 interior points and the
    2 x 20 band points at +-L/2 into the merged buffer (pde/advection.py _advect_points), the frozen and
    the trainable field run as one fused jet launch, the loss is fused_mse, Adam + plateau one launch;
    fused=True (the default, round 6): the whole iteration but the sums as ONE insr_advect1d_iteration
    launch (base/advect_iter.py), its rows summed by the Adam launch -- vs the oracle's
    advection/model.py:68-91 loss on the points the launch drew: both losses, every parameter gradient, the
    Adam update."""
    import pde.advection as adv
    from base import advect_iter
    from pde.config import baseline_config
    cfg = baseline_config("advect1D", proj_dir="/tmp/insr_fullsize_adv", insr_progress=False, early_stop=False,
                          max_n_iters=1, insr_graph=False, insr_sync_every=1, insr_advect_fused=fused)
    m = adv.Advection1DModel(cfg)
    m.timestep = 1
    refs = {"f": seeded(1, 1, 3, 64, 221), "f_prev": seeded(1, 1, 3, 64, 222)}
    load(m.field, refs["f"])
    load(m.field_prev, refs["f_prev"])
    p0 = O.flat_params(refs["f"]).numpy().copy()
    drawn = {}
    orig = adv.sample_boxes

    def rec(boxes, d, **kw):
        buf = orig(boxes, d, **kw)
        drawn["buf"] = buf.detach().cpu().clone()
        drawn["n"] = [b[0] for b in boxes]
        return buf
    adv.sample_boxes = rec
    if fused:
        m._insr_points_out = torch.empty(4096 + 40, device="cuda")
    it0 = advect_iter.STATS["iterations"]
    try:
        m._reset_optimizer()
        ld = adv.Advection1DModel._advect._insr_phase(m)
        m._update_network(ld)
        torch.cuda.synchronize()
    finally:
        adv.sample_boxes = orig
    assert advect_iter.STATS["iterations"] - it0 == (1 if fused else 0)
    if fused:
        assert "buf" not in drawn  # no sampler launch: the iteration kernel drew the points
        drawn["buf"], drawn["n"] = m._insr_points_out.detach().cpu().view(-1, 1).clone(), [4096, 20, 20]
    n, h, h2 = drawn["n"]
    assert (n, h, h2) == (4096, 20, 20)
    buf = drawn["buf"]
    x, bc = buf[:n], buf[n:]
    half = cfg.length / 2
    assert float(x.min()) >= -half and float(x.max()) < half
    assert (bc.abs() > half * (1 - 1.01e-4)).all() and (bc.abs() < half * (1 + 1.01e-4)).all()
    r = {k: seeded(1, 1, 3, 64, s) for k, s in (("f", 221), ("f_prev", 222))}
    for p in r["f_prev"].parameters():
        p.requires_grad_(False)
    opt = O.OracleAdam(list(r["f"].parameters()), lr=cfg.lr)
    ldo = O.advect1d_loss(r["f"], r["f_prev"], x.clone().requires_grad_(True), bc.clone().requires_grad_(True),
                          cfg.dt, cfg.vel)
    O.update_step([r["f"]], ldo, opt)
    assert set(ld) == set(ldo) == {"main", "bc"}
    for k, v in ldo.items():
        assert abs(float(ld[k]) - float(v)) <= TOL * abs(float(v)) + 1e-12, (k, float(ld[k]), float(v))
    check_grads(m.field, r["f"], "advect1D")
    check_update(m.field, r["f"], p0, cfg.lr)


def test_advect1d_plain_full_size(B):
    """The reference's advection body as written (pde/advection_plain.py) at the advect1D size (4,096 +
    2 x 20 points), through the training loop's loss lowering and deferred jets, vs the oracle on the same
    points: both losses, every parameter gradient, the Adam update."""
    import pde.advection_plain as ap
    from base import lower as LW
    from pde.config import baseline_config
    cfg = baseline_config("advect1D", proj_dir="/tmp/insr_fullsize_adv_plain", insr_progress=False, early_stop=False,
                          max_n_iters=1, insr_graph=False, insr_sync_every=1)
    m = ap.Advection1DPlainModel(cfg)
    m.timestep = 1
    refs = {"f": seeded(1, 1, 3, 64, 231), "f_prev": seeded(1, 1, 3, 64, 232)}
    load(m.field, refs["f"])
    load(m.field_prev, refs["f_prev"])
    p0 = O.flat_params(refs["f"]).numpy().copy()
    gen = torch.Generator().manual_seed(233)
    half = cfg.length / 2
    x = (torch.rand(4096, 1, generator=gen) * 2 - 1) * half
    eps = 1e-4
    bu = torch.cat([-1 + eps * (torch.rand(20, 1, generator=gen) * 2 - 1), 1 + eps * (torch.rand(20, 1, generator=gen) * 2 - 1)])
    m._sample_in_training = lambda: x.cuda().requires_grad_(True)
    orig = ap.sample_boundary
    ap.sample_boundary = lambda n, d, device=None: bu.cuda()
    try:
        m._reset_optimizer()
        with LW.lowering(m._lower_on()), LW.deferred_jets(m._defer_on()):
            ld = ap.Advection1DPlainModel._advect._insr_phase(m)
        ld = LW.lower_losses(ld)
        m._update_network(ld)
        torch.cuda.synchronize()
    finally:
        ap.sample_boundary = orig
    bc = (bu.cuda() * cfg.length / 2).cpu()  # the body's own scaling, in its op order
    r = {k: seeded(1, 1, 3, 64, s) for k, s in (("f", 231), ("f_prev", 232))}
    for p in r["f_prev"].parameters():
        p.requires_grad_(False)
    opt = O.OracleAdam(list(r["f"].parameters()), lr=cfg.lr)
    ldo = O.advect1d_loss(r["f"], r["f_prev"], x.clone().requires_grad_(True), bc.clone().requires_grad_(True),
                          cfg.dt, cfg.vel)
    O.update_step([r["f"]], ldo, opt)
    assert set(ld) == set(ldo) == {"main", "bc"}
    for k, v in ldo.items():
        assert abs(float(ld[k]) - float(v)) <= TOL * abs(float(v)) + 1e-12, (k, float(ld[k]), float(v))
    check_grads(m.field, r["f"], "advect1D plain")
    check_update(m.field, r["f"], p0, cfg.lr)


def test_elasticity2dstretch_plain_full_size(B):
    """The reference's elastodynamics body as written (pde/elasticity_plain.py: q = f(x) + x, jacobian,
    torch.svd, the energies as torch sums, separate constraint calls) at the elasticity2Dstretch size
    (20,000 + 2 x 200 points), through the training loop's lowering scopes, vs the oracle on the same points."""
    from base import lower as LW
    from pde.config import baseline_config
    from pde.elasticity_plain import ElasticityPlainModel
    cfg = baseline_config("elasticity2Dstretch", proj_dir="/tmp/insr_fullsize_el2d_plain", insr_progress=False,
                          early_stop=False, max_n_iters=1, insr_graph=False, insr_sync_every=1)
    m = ElasticityPlainModel(cfg)
    m.timestep = 1
    for k, s, net in (("f", 241, m.deformation_field), ("f_prev", 242, m.deformation_field_prev),
                      ("f_pp", 243, m.deformation_field_prev_prev)):
        load(net, seeded(2, 2, 5, 128, s))
    p0 = O.flat_params(seeded(2, 2, 5, 128, 241)).numpy().copy()
    gen = torch.Generator().manual_seed(244)
    x = torch.rand(20000, 2, generator=gen) * 2 - 1
    fl_ = torch.rand(200, 2, generator=gen) * 0.02 - 1.0
    fr_ = torch.rand(200, 2, generator=gen) * 0.02 + 0.98
    m._sample_in_training = lambda resolution: x.cuda().requires_grad_(True)
    m._sample_fixed_in_training = lambda resolution: (fl_.cuda().requires_grad_(True), fr_.cuda().requires_grad_(True))
    m._reset_optimizer()
    e0 = LW.LOWERED["energies"]
    with LW.lowering(m._lower_on()), LW.deferred_jets(m._defer_on()):
        ld = ElasticityPlainModel._solve_deformation._insr_phase(m)
    ld = LW.lower_losses(ld)
    # the svd energies went through ONE insr_elastic_energy launch, the constraints through a loss group
    assert LW.LOWERED["energies"] == e0 + 1
    m._update_network(ld)
    torch.cuda.synchronize()
    ecfg = dict(dt=cfg.dt, energy=list(cfg.energy), ratio_arap=cfg.ratio_arap, ratio_volume=cfg.ratio_volume,
                ratio_kinematics=cfg.ratio_kinematics, ratio_constraint=cfg.ratio_constraint,
                ratio_collide=cfg.ratio_collide, plane_height=cfg.plane_height,
                external_force=[cfg.external_force_x, cfg.external_force_y],
                constraint_offset_right=[cfg.constraint_right_offset_x, cfg.constraint_right_offset_y],
                circle_center=[cfg.collide_circle_x, cfg.collide_circle_y], circle_radius=cfg.collide_circle_radius,
                external_force_timesteps=cfg.external_force_timesteps)
    r = {k: seeded(2, 2, 5, 128, s) for k, s in (("f", 241), ("f_prev", 242), ("f_pp", 243))}
    for k in ("f_prev", "f_pp"):
        for p in r[k].parameters():
            p.requires_grad_(False)
    opt = O.OracleAdam(list(r["f"].parameters()), lr=cfg.lr)
    ldo = O.elasticity_loss(r["f"], r["f_prev"], r["f_pp"], x.clone().requires_grad_(True),
                            fl_.clone().requires_grad_(True), fr_.clone().requires_grad_(True), ecfg, timestep=1)
    O.update_step([r["f"]], ldo, opt)
    assert abs(float(ld["main"]) - float(ldo["main"])) <= TOL * abs(float(ldo["main"])), (float(ld["main"]),
                                                                                             float(ldo["main"]))
    check_grads(m.deformation_field, r["f"], "el2d plain")
    check_update(m.deformation_field, r["f"], p0, cfg.lr)


def test_elasticity2dstretch_plain_loop_is_captured(B):
    """The unchanged elasticity body through the real training loop with hipGraph replay (U = 4 groups): no
    host read inside an iteration any more (jacobian()'s NaN status is a Lazy value nobody reads, the svd
    energies lowered), so every iteration after the first is captured and replayed; the energy decreases."""
    import warnings
    from base import lower as LW
    from pde.config import baseline_config
    from pde.elasticity_plain import ElasticityPlainModel
    cfg = baseline_config("elasticity2Dstretch", proj_dir="/tmp/insr_el2d_plain_loop", insr_progress=False,
                          early_stop=False, max_n_iters=7, insr_graph=True, insr_graph_unroll=4, insr_sync_every=1000)
    torch.manual_seed(0)
    m = ElasticityPlainModel(cfg)
    m.timestep = 1
    seen = []
    m.tb = type("TB", (), {"add_scalars": lambda self, tag, vals, global_step: seen.append(vals["main"])})()
    e0 = LW.LOWERED["energies"]
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)  # a capture fallback warns
        m._solve_deformation()
    torch.cuda.synchronize()
    assert getattr(m, "_insr_capture_error", None) is None, m._insr_capture_error
    assert LW.LOWERED["energies"] >= e0 + 3  # iteration 0, the captured iteration 1, the group graph's bodies
    assert len(seen) == 2 and np.isfinite(seen).all() and seen[1] < seen[0]
