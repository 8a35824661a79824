"""Generate golden vectors by running the REFERENCE (qingxu-thu/INSR-PDE) on the CPU.

Run in the build container only (needs /root/reference, which does not exist on
the GPU box):   python tests/golden/make_golden.py

What it does, and nothing else:
* imports the reference's own `base` package and the advection / fluid /
  elasticity model classes from /root/reference.  Four third-party modules the
  reference imports at module top but never calls on these paths are absent
  from the image (pytorch3d.ops -- vortex kNN, base/networks.py:4; tensorboardX
  -- logging, base/baseModel.py:5; meshio -- mesh files, elasticity/model.py:13;
  open3d -- .ply output, elasticity/visualize.py:5); they get empty placeholder
  modules so the import succeeds.  No reference function is replaced.
* forces the CPU (the reference hard-codes cuda:0, base/baseModel.py:25) and
  drops ReduceLROnPlateau's removed `verbose` kwarg (torch 2.10).
* builds reference MLPs from fixed torch seeds, evaluates the reference diff
  ops on fixed samples, and runs the reference phase bodies (pulled out of the
  `_training_loop` closure) + the reference `_update_network` (backward + Adam)
  on fixed samples.
* writes the inputs and outputs to tests/golden/*.npz (fixtures = data only).
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _placeholder_modules():
    class _Unused:
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, name):
            return lambda *a, **k: None

    p3d = types.ModuleType("pytorch3d")
    p3d_ops = types.ModuleType("pytorch3d.ops")
    p3d_ops.knn_points = p3d_ops.knn_gather = None
    p3d.ops = p3d_ops
    tbx = types.ModuleType("tensorboardX")
    tbx.SummaryWriter = _Unused
    sys.modules.update({"pytorch3d": p3d, "pytorch3d.ops": p3d_ops, "tensorboardX": tbx,
                        "meshio": types.ModuleType("meshio"), "open3d": types.ModuleType("open3d")})


def load_reference():
    _placeholder_modules()
    import matplotlib
    matplotlib.use("Agg")
    sys.path.insert(0, REF)
    import base  # noqa: E402  (reference package)
    import base.baseModel as bm

    orig_init = bm.BaseModel.__init__

    def cpu_init(self, cfg):
        orig_init(self, cfg)
        self.device = torch.device("cpu")

    bm.BaseModel.__init__ = cpu_init
    orig_plateau = torch.optim.lr_scheduler.ReduceLROnPlateau

    class Plateau(orig_plateau):
        def __init__(self, *a, verbose=None, **k):
            super().__init__(*a, **k)

    torch.optim.lr_scheduler.ReduceLROnPlateau = Plateau
    torch.Tensor.cuda = lambda self, *a, **k: self
    torch.nn.Module.cuda = lambda self, *a, **k: self
    return base


def raw_phase(cls, name):
    """Unwrap the BaseModel._training_loop closure to the phase body."""
    loop = getattr(cls, name)
    for cell in loop.__closure__:
        if callable(cell.cell_contents) and getattr(cell.cell_contents, "__name__", "") == name:
            return cell.cell_contents
    raise KeyError(name)


class Cfg(types.SimpleNamespace):
    pass


def base_cfg(**kw):
    c = Cfg(exp_dir="/tmp/golden_exp", log_dir="/tmp/golden_exp/log", model_dir="/tmp/golden_exp/model",
            dt=0.05, max_n_iters=3, sample_resolution=32, vis_resolution=8, lr=1e-4, network="siren",
            num_hidden_layers=3, hidden_features=64, nonlinearity="sine", vis_frequency=10**9,
            early_stop=False, init_cond=None)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def flat(net):
    return torch.cat([p.detach().reshape(-1) for p in net.parameters()]).numpy().copy()


def flat_grad(net):
    return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                      for p in net.parameters()]).detach().numpy().copy()


def set_flat(net, vec):
    off = 0
    with torch.no_grad():
        for p in net.parameters():
            n = p.numel()
            p.copy_(torch.from_numpy(vec[off:off + n]).view_as(p))
            off += n


def seeded_net(base, d_in, d_out, L, W, seed):
    torch.manual_seed(seed)
    return base.MLP(d_in, d_out, L, W, nonlinearity="sine")


# ---------------------------------------------------------------------------
def gen_networks_and_ops(base):
    """Init bit-pattern + every diff op + param-grads of a fixed functional."""
    cases = {"advect": (1, 1, 3, 64), "fluid_vel": (2, 2, 4, 128), "fluid_pres": (2, 1, 4, 128),
             "el2d": (2, 2, 5, 128), "el3d": (3, 3, 5, 256)}
    out = {}
    for i, (name, (din, dout, L, W)) in enumerate(cases.items()):
        seed = 100 + i
        net = seeded_net(base, din, dout, L, W, seed)
        out[f"{name}/seed"] = np.array(seed)
        out[f"{name}/shape"] = np.array([din, dout, L, W])
        stride = 61 if W == 256 else 1  # el3d: strided subsample keeps the fixture small
        out[f"{name}/param_stride"] = np.array(stride)
        out[f"{name}/params"] = flat(net)[::stride]
        g = torch.Generator().manual_seed(1000 + i)
        n_pts = 64 if W == 256 else 256
        x = (torch.rand(n_pts, din, generator=g) * 2 - 1).requires_grad_(True)
        out[f"{name}/x"] = x.detach().numpy().copy()
        y = net(x)
        out[f"{name}/y"] = y.detach().numpy().copy()
        ops = {}
        if W < 256:
            ops["gradient"] = base.gradient(y, x)
            if dout == din:
                ops["divergence"] = base.divergence(y, x)
            ops["laplace"] = base.laplace(y, x)
        jac, st = base.jacobian(y, x)
        ops["jacobian"] = jac
        out[f"{name}/jacobian_status"] = np.array(st)
        if W <= 128 and din <= 2:
            # reference hessian wants (meta_batch, obs, ch) / (meta_batch, obs, dim)
            x3 = x.detach()[None].clone().requires_grad_(True)
            hes, st = base.hessian(net(x3), x3)
            ops["hessian"] = hes
            out[f"{name}/hessian_status"] = np.array(st)
        for op, val in ops.items():
            out[f"{name}/{op}"] = val.detach().numpy().copy()
            r = torch.randn(val.shape, generator=g)
            out[f"{name}/{op}_R"] = r.numpy().copy()
            net.zero_grad(set_to_none=True)
            (val * r).sum().backward(retain_graph=True)
            out[f"{name}/{op}_pgrad"] = flat_grad(net)[::stride]
        # trainable value functional
        r = torch.randn(y.shape, generator=g)
        out[f"{name}/value_R"] = r.numpy().copy()
        net.zero_grad(set_to_none=True)
        (net(x) * r).sum().backward()
        out[f"{name}/value_pgrad"] = flat_grad(net)[::stride]
    return out


# ---------------------------------------------------------------------------
def run_phase(model, cls, phase, n_iters, samples_fn, patches):
    """Reset the optimiser, then n_iters x (phase body + _update_network)."""
    body = raw_phase(cls, phase)
    model._reset_optimizer()
    rec = []
    for it in range(n_iters):
        for mod, attr, fn in patches(it):
            setattr(mod, attr, fn)
        model._sample_in_training = samples_fn(it)
        loss_dict = body(model)
        model._update_network(loss_dict)
        rec.append({k: float(v.detach()) for k, v in loss_dict.items()})
    return rec


def gen_fluid(base):
    import fluid.model as fm
    from fluid.model import Fluid2DModel
    cfg = base_cfg(num_hidden_layers=4, hidden_features=128, sample_resolution=32, dt=0.05,
                   init_cond="taylorgreen")
    torch.manual_seed(7)
    model = Fluid2DModel(cfg)
    out = {}
    # distinct, seeded weights for current / prev / pressure
    for name, net, seed in (("vel", model.velocity_field, 11), ("vel_prev", model.velocity_field_prev, 12),
                            ("pres", model.pressure_field, 13)):
        set_flat(net, flat(seeded_net(base, 2, net.net[-1].out_features, 4, 128, seed)))
        out[f"fluid/{name}/params0"] = flat(net)
    N = cfg.sample_resolution ** 2
    nb = N // 100
    g = torch.Generator().manual_seed(2024)
    iters = 2
    xs = [(torch.rand(N, 2, generator=g) * 2 - 1) for _ in range(iters)]
    bxs = [base.sample_boundary2D_separate(nb, "horizontal") for _ in range(iters)]
    bys = [base.sample_boundary2D_separate(nb, "vertical") for _ in range(iters)]
    for it in range(iters):
        out[f"fluid/x{it}"] = xs[it].numpy()
        out[f"fluid/bcx{it}"] = bxs[it].numpy()
        out[f"fluid/bcy{it}"] = bys[it].numpy()

    def samples_fn(it):
        return lambda: xs[it].clone().requires_grad_(True)

    def patches(it):
        seq = iter([bxs[it], bys[it]])
        return [(fm, "sample_boundary2D_separate", lambda n, side, device=None, **k: next(seq).clone())]

    state0 = {n: flat(getattr(model, a)) for n, a in
              (("vel", "velocity_field"), ("vel_prev", "velocity_field_prev"), ("pres", "pressure_field"))}
    for phase in ("_advect_velocity", "_solve_pressure", "_projection"):
        for n, a in (("vel", "velocity_field"), ("vel_prev", "velocity_field_prev"), ("pres", "pressure_field")):
            set_flat(getattr(model, a), state0[n])
        # single iteration: loss + grads
        body = raw_phase(Fluid2DModel, phase)
        model._reset_optimizer()
        for mod, attr, fn in patches(0):
            setattr(mod, attr, fn)
        model._sample_in_training = samples_fn(0)
        ld = body(model)
        for k, v in ld.items():
            out[f"fluid/{phase}/loss_{k}"] = np.array(float(v.detach()))
        loss = sum(ld.values())
        model.optimizer.zero_grad()
        loss.backward()
        out[f"fluid/{phase}/grad_vel"] = flat_grad(model.velocity_field)
        out[f"fluid/{phase}/grad_pres"] = flat_grad(model.pressure_field)
        # full iterations through the reference update
        for n, a in (("vel", "velocity_field"), ("vel_prev", "velocity_field_prev"), ("pres", "pressure_field")):
            set_flat(getattr(model, a), state0[n])
        rec = run_phase(model, Fluid2DModel, phase, iters, samples_fn, patches)
        out[f"fluid/{phase}/loss_trace"] = np.array([[r[k] for k in sorted(r)] for r in rec])
        out[f"fluid/{phase}/vel_after"] = flat(model.velocity_field)
        out[f"fluid/{phase}/pres_after"] = flat(model.pressure_field)
    return out


def gen_advect(base):
    import advection.model as am
    from advection.model import Advection1DModel
    cfg = base_cfg(num_hidden_layers=3, hidden_features=64, sample_resolution=512, dt=0.05, vel=0.25,
                   length=4.0, init_cond="example1")
    model = Advection1DModel(cfg)
    out = {}
    for name, net, seed in (("field", model.field, 21), ("field_prev", model.field_prev, 22)):
        set_flat(net, flat(seeded_net(base, 1, 1, 3, 64, seed)))
        out[f"advect/{name}/params0"] = flat(net)
    g = torch.Generator().manual_seed(77)
    iters = 2
    xs = [(torch.rand(cfg.sample_resolution, 1, generator=g) * 2 - 1) * cfg.length / 2 for _ in range(iters)]
    nb = max(cfg.sample_resolution // 100, 10)
    bs = [base.sample_boundary(nb, 1) * cfg.length / 2 for _ in range(iters)]
    for it in range(iters):
        out[f"advect/x{it}"] = xs[it].numpy()
        out[f"advect/bc{it}"] = bs[it].numpy()

    def samples_fn(it):
        return lambda: xs[it].clone().requires_grad_(True)

    def patches(it):
        # reference multiplies the band by length/2 itself (advection/model.py:86)
        return [(am, "sample_boundary", lambda n, sdim, device=None, **k: bs[it] / (cfg.length / 2))]

    s0 = {"field": flat(model.field), "field_prev": flat(model.field_prev)}
    body = raw_phase(Advection1DModel, "_advect")
    model._reset_optimizer()
    for mod, attr, fn in patches(0):
        setattr(mod, attr, fn)
    model._sample_in_training = samples_fn(0)
    ld = body(model)
    for k, v in ld.items():
        out[f"advect/_advect/loss_{k}"] = np.array(float(v.detach()))
    model.optimizer.zero_grad()
    sum(ld.values()).backward()
    out["advect/_advect/grad_field"] = flat_grad(model.field)
    set_flat(model.field, s0["field"])
    rec = run_phase(model, Advection1DModel, "_advect", iters, samples_fn, patches)
    out["advect/_advect/loss_trace"] = np.array([[r[k] for k in sorted(r)] for r in rec])
    out["advect/_advect/field_after"] = flat(model.field)
    return out


def gen_elasticity(base):
    from elasticity.model import ElasticityModel
    cfg = base_cfg(num_hidden_layers=5, hidden_features=128, sample_resolution=16, dt=0.1, lr=1e-4, dim=2,
                   energy=["arap", "constraint", "constraint_right", "volume", "kinematics", "external",
                           "collision"],
                   sample_pattern=["random", "uniform"], ratio_constraint=1e4, ratio_volume=1e3, ratio_arap=1.0,
                   ratio_collide=1e2, ratio_kinematics=1.0, use_mesh=False, mesh_path="",
                   external_force_timesteps=5, external_force_x=0.0, external_force_y=-1.0,
                   external_force_z=0.0, constraint_right_offset_x=2.0, constraint_right_offset_y=0.0,
                   constraint_right_offset_z=0.0, plane_height=-0.9, collide_circle_x=0.0,
                   collide_circle_y=-2.0, collide_circle_z=0.0, collide_circle_radius=1.0)
    model = ElasticityModel(cfg)
    model.timestep = 1
    out = {}
    for name, net, seed in (("f", model.deformation_field, 31), ("f_prev", model.deformation_field_prev, 32),
                            ("f_pp", model.deformation_field_prev_prev, 33)):
        set_flat(net, flat(seeded_net(base, 2, 2, 5, 128, seed)))
        out[f"el2d/{name}/params0"] = flat(net)
    g = torch.Generator().manual_seed(55)
    R = cfg.sample_resolution
    iters = 2
    xs, fl, fr = [], [], []
    for it in range(iters):
        rnd = torch.rand(R * R, 2, generator=g) * 2 - 1
        xs.append(torch.cat([rnd, base.sample_uniform(R, 2)], 0))
        fl.append(torch.cat([torch.cat([-torch.ones(R, 1), torch.rand(R, 1, generator=g) * 2 - 1], 1),
                             torch.cat([-torch.ones(R, 1), base.sample_uniform(R, 1)], 1)], 0))
        fr.append(torch.cat([torch.cat([torch.ones(R, 1), torch.rand(R, 1, generator=g) * 2 - 1], 1),
                             torch.cat([torch.ones(R, 1), base.sample_uniform(R, 1)], 1)], 0))
        out[f"el2d/x{it}"] = xs[it].numpy()
        out[f"el2d/fixed_l{it}"] = fl[it].numpy()
        out[f"el2d/fixed_r{it}"] = fr[it].numpy()

    def samples_fn(it):
        return lambda res: xs[it].clone().requires_grad_(True)

    def patches(it):
        return [(model, "_sample_fixed_in_training",
                 lambda res: (fl[it].clone().requires_grad_(True), fr[it].clone().requires_grad_(True)))]

    s0 = flat(model.deformation_field)
    body = raw_phase(ElasticityModel, "_solve_deformation")
    model._reset_optimizer()
    for mod, attr, fn in patches(0):
        setattr(mod, attr, fn)
    model._sample_in_training = samples_fn(0)
    ld = body(model)
    out["el2d/_solve_deformation/loss_main"] = np.array(float(ld["main"].detach()))
    model.optimizer.zero_grad()
    ld["main"].backward()
    out["el2d/_solve_deformation/grad_f"] = flat_grad(model.deformation_field)
    set_flat(model.deformation_field, s0)
    rec = run_phase(model, ElasticityModel, "_solve_deformation", iters, samples_fn, patches)
    out["el2d/_solve_deformation/loss_trace"] = np.array([[r[k] for k in sorted(r)] for r in rec])
    out["el2d/_solve_deformation/f_after"] = flat(model.deformation_field)
    out["el2d/cfg_energy"] = np.array(cfg.energy)
    return out


def gen_elasticity3d(base):
    """3-D phase (the elasticity3Dbunny energy set on the box geometry, plus the sphere
    collider): singular values of 3x3 blocks, plane/sphere collisions, external force,
    kinematics.  A small 3 -> 3, 2 x 64 net keeps the fixture small; the 5 x 256 width is
    covered by the el3d operator vectors above."""
    from elasticity.model import ElasticityModel
    cfg = base_cfg(num_hidden_layers=2, hidden_features=64, sample_resolution=6, dt=0.1, lr=1e-4, dim=3,
                   energy=["arap", "kinematics", "external", "volume", "collision", "collision_sphere"],
                   sample_pattern=["random", "uniform"], ratio_constraint=1e4, ratio_volume=1e3, ratio_arap=1e2,
                   ratio_collide=1e3, ratio_kinematics=1.0, use_mesh=False, mesh_path="",
                   external_force_timesteps=5, external_force_x=0.0, external_force_y=0.0,
                   external_force_z=-1e2, constraint_right_offset_x=0.0, constraint_right_offset_y=0.0,
                   constraint_right_offset_z=0.0, plane_height=-0.5, collide_circle_x=0.0,
                   collide_circle_y=-1.6, collide_circle_z=0.0, collide_circle_radius=1.0)
    model = ElasticityModel(cfg)
    model.timestep = 1
    out = {}
    for name, net, seed in (("f", model.deformation_field, 41), ("f_prev", model.deformation_field_prev, 42),
                            ("f_pp", model.deformation_field_prev_prev, 43)):
        set_flat(net, flat(seeded_net(base, 3, 3, 2, 64, seed)))
        out[f"el3d/{name}/params0"] = flat(net)
    g = torch.Generator().manual_seed(66)
    R = cfg.sample_resolution
    iters = 2
    xs = []
    for it in range(iters):
        xs.append(torch.cat([torch.rand(R ** 3, 3, generator=g) * 2 - 1, base.sample_uniform(R, 3)], 0))
        out[f"el3d/x{it}"] = xs[it].numpy()

    def samples_fn(it):
        return lambda res: xs[it].clone().requires_grad_(True)

    def patches(it):
        return []

    s0 = flat(model.deformation_field)
    body = raw_phase(ElasticityModel, "_solve_deformation")
    model._reset_optimizer()
    model._sample_in_training = samples_fn(0)
    ld = body(model)
    out["el3d/_solve_deformation/loss_main"] = np.array(float(ld["main"].detach()))
    model.optimizer.zero_grad()
    ld["main"].backward()
    out["el3d/_solve_deformation/grad_f"] = flat_grad(model.deformation_field)
    set_flat(model.deformation_field, s0)
    rec = run_phase(model, ElasticityModel, "_solve_deformation", iters, samples_fn, patches)
    out["el3d/_solve_deformation/loss_trace"] = np.array([[r[k] for k in sorted(r)] for r in rec])
    out["el3d/_solve_deformation/f_after"] = flat(model.deformation_field)
    out["el3d/cfg_energy"] = np.array(cfg.energy)
    return out


def gen_init(base):
    """ref_init.npz: the three `_initialize` phases (the t = 0 fits every run starts with):
    advection/model.py:43-52 (mse to the 'example1' Gaussian), fluid/model.py:42-51 (mse to
    'taylorgreen'), elasticity/model.py:109-117 (mean(f(x)^2)) -- loss, parameter gradients
    of one backward, and the loss trace + parameters after 2 reference iterations (phase body
    + _update_network) on explicit samples."""
    from advection.model import Advection1DModel
    from fluid.model import Fluid2DModel
    from elasticity.model import ElasticityModel
    out = {}
    iters = 2
    cases = [
        ("advect", Advection1DModel, "field",
         base_cfg(num_hidden_layers=3, hidden_features=64, sample_resolution=512, dt=0.05, vel=0.25, length=4.0,
                  init_cond="example1"), (1, 1, 3, 64), 61,
         lambda g: [(torch.rand(512, 1, generator=g) * 2 - 1) * 2.0 for _ in range(iters)], False),
        ("fluid", Fluid2DModel, "velocity_field",
         base_cfg(num_hidden_layers=4, hidden_features=128, sample_resolution=32, dt=0.05, init_cond="taylorgreen"),
         (2, 2, 4, 128), 62, lambda g: [torch.rand(1024, 2, generator=g) * 2 - 1 for _ in range(iters)], False),
        ("el2d", ElasticityModel, "deformation_field",
         base_cfg(num_hidden_layers=5, hidden_features=128, sample_resolution=16, dt=0.1, dim=2, energy=["arap"],
                  sample_pattern=["random", "uniform"], ratio_constraint=1e4, ratio_volume=1e3, ratio_arap=1.0,
                  ratio_collide=1e2, ratio_kinematics=1.0, use_mesh=False, mesh_path="",
                  external_force_timesteps=5, external_force_x=0.0, external_force_y=-1.0, external_force_z=0.0,
                  constraint_right_offset_x=2.0, constraint_right_offset_y=0.0, constraint_right_offset_z=0.0,
                  plane_height=-0.9, collide_circle_x=0.0, collide_circle_y=-2.0, collide_circle_z=0.0,
                  collide_circle_radius=1.0),
         (2, 2, 5, 128), 63,
         lambda g: [torch.cat([torch.rand(512, 2, generator=g) * 2 - 1, base.sample_uniform(16, 2)]) for _ in
                    range(iters)], True),
    ]
    for name, cls, attr, cfg, (din, dout, L, W), seed, draw, takes_res in cases:
        model = cls(cfg)
        model.timestep = 0
        if name != "el2d":
            model.init_cond_func = __import__(cls.__module__.split(".")[0] + ".examples",
                                              fromlist=["get_examples"]).get_examples(cfg.init_cond)
        net = getattr(model, attr)
        set_flat(net, flat(seeded_net(base, din, dout, L, W, seed)))
        p0 = flat(net)
        out[f"init/{name}/params0"] = p0
        xs = draw(torch.Generator().manual_seed(seed + 1000))
        for it in range(iters):
            out[f"init/{name}/x{it}"] = xs[it].numpy()

        def samples_fn(it):
            return (lambda res: xs[it].clone().requires_grad_(True)) if takes_res else \
                (lambda: xs[it].clone().requires_grad_(True))

        body = raw_phase(cls, "_initialize")
        model._reset_optimizer()
        model._sample_in_training = samples_fn(0)
        ld = body(model)
        out[f"init/{name}/loss_main"] = np.array(float(ld["main"].detach()))
        model.optimizer.zero_grad()
        ld["main"].backward()
        out[f"init/{name}/grad"] = flat_grad(net)
        set_flat(net, p0)
        rec = run_phase(model, cls, "_initialize", iters, samples_fn, lambda it: [])
        out[f"init/{name}/loss_trace"] = np.array([[r[k] for k in sorted(r)] for r in rec])
        out[f"init/{name}/after"] = flat(net)
    return out


def gen_samplers(base):
    torch.manual_seed(5)
    out = {"sampling/uniform_8_2": base.sample_uniform(8, 2).numpy(),
           "sampling/uniform_5_1": base.sample_uniform(5, 1).numpy(),
           "sampling/uniform_4_3": base.sample_uniform(4, 3).numpy()}
    torch.manual_seed(6)
    out["sampling/random_seed6_100x2"] = base.sample_random(100, 2).numpy()
    torch.manual_seed(8)
    out["sampling/bnd2d_h_seed8_20"] = base.sample_boundary2D_separate(20, "horizontal").numpy()
    torch.manual_seed(9)
    out["sampling/bnd1d_seed9_20"] = base.sample_boundary(20, 1).numpy()
    return out


def gen_extra(base):
    """ref_extra.npz: the reference's initial conditions (fluid/examples.py:17-51) on grid +
    random points (incl. the blend gaps), and more of its samplers (base/sampling.py:4-64)."""
    sys.path.insert(0, os.path.join(REF, "fluid"))
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_fluid_examples", os.path.join(REF, "fluid", "examples.py"))
    ex = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ex)
    g = torch.Generator().manual_seed(40)
    grid = base.sample_uniform(64, 2)
    rnd = torch.rand(4096, 2, generator=g) * 2 - 1
    gaps = torch.cat([torch.rand(512, 2, generator=g) * 0.2 - 0.1 + 0.05,          # around the (0.05, 0.05) corner
                      torch.rand(512, 2, generator=g) * 0.1 + 0.7])                 # around p - gap_ = 0.725
    x = torch.cat([grid, rnd, gaps])
    out = {"examples/x": x.numpy(),
           "examples/taylorgreen_multi": ex.taylorgreen_multi_velocity(x).numpy(),
           "examples/taylorgreen": ex.get_examples("taylorgreen")(x).numpy()}
    torch.manual_seed(10)
    out["sampling/bnd2d_v_seed10_20"] = base.sample_boundary2D_separate(20, "vertical").numpy()
    torch.manual_seed(11)
    out["sampling/bnd2d_box_seed11_40"] = base.sample_boundary(40, 2).numpy()
    torch.manual_seed(12)
    out["sampling/random_seed12_50x3"] = base.sample_random(50, 3).numpy()
    return out


def gen_other_nets(base):
    """ref_nets.npz: the reference MLP's other configurations (base/networks.py:30-71) -- relu / elu
    networks, outermost_linear=False, a SIREN wider than the kernels' 256 -- seeded init bit patterns,
    the value and gradient (autograd create_graph, base/diff_ops.py:53-58) on fixed points, and the
    parameter gradients of a fixed functional of both."""
    cases = {"relu": (2, 1, 3, 64, True, "relu"), "elu": (2, 2, 2, 32, True, "elu"),
             "sine_nonlinear_out": (2, 1, 2, 32, False, "sine"), "relu_nonlinear_out": (1, 2, 2, 16, False, "relu"),
             "sine_w300": (1, 1, 1, 300, True, "sine")}
    out = {}
    for i, (name, (din, dout, L, W, olin, nl)) in enumerate(cases.items()):
        seed = 700 + i
        torch.manual_seed(seed)
        net = base.MLP(din, dout, L, W, outermost_linear=olin, nonlinearity=nl)
        out[f"{name}/seed"] = np.array(seed)
        out[f"{name}/shape"] = np.array([din, dout, L, W, int(olin)])
        out[f"{name}/nonlinearity"] = np.array(nl)
        out[f"{name}/params"] = flat(net)
        g = torch.Generator().manual_seed(7000 + i)
        x = (torch.rand(128, din, generator=g) * 2 - 1).requires_grad_(True)
        out[f"{name}/x"] = x.detach().numpy().copy()
        y = net(x)
        gr = base.gradient(y, x)
        out[f"{name}/y"] = y.detach().numpy().copy()
        out[f"{name}/gradient"] = gr.detach().numpy().copy()
        ry, rg = torch.randn(y.shape, generator=g), torch.randn(gr.shape, generator=g)
        out[f"{name}/y_R"], out[f"{name}/gradient_R"] = ry.numpy().copy(), rg.numpy().copy()
        net.zero_grad(set_to_none=True)
        ((y * ry).sum() + (gr * rg).sum()).backward()
        out[f"{name}/pgrad"] = flat_grad(net)
    return out


def main():
    torch.set_num_threads(8)
    base = load_reference()
    if "--nets" in sys.argv:  # relu / elu / outermost_linear=False / wide networks (ref_nets.npz)
        np.savez_compressed(os.path.join(OUT, "ref_nets.npz"), **gen_other_nets(base))
        print("ref_nets.npz", os.path.getsize(os.path.join(OUT, "ref_nets.npz")) / 1e6, "MB")
        return
    if "--extra" in sys.argv:  # initial conditions + more samplers (ref_extra.npz)
        np.savez_compressed(os.path.join(OUT, "ref_extra.npz"), **gen_extra(base))
        print("ref_extra.npz", os.path.getsize(os.path.join(OUT, "ref_extra.npz")) / 1e6, "MB")
        return
    if "--init" in sys.argv:  # the three _initialize phases (ref_init.npz)
        np.savez_compressed(os.path.join(OUT, "ref_init.npz"), **gen_init(base))
        print("ref_init.npz", os.path.getsize(os.path.join(OUT, "ref_init.npz")) / 1e6, "MB")
        return
    if "--el3d" in sys.argv:  # the 3-D elasticity phase vectors alone (ref_phases_el3d.npz)
        np.savez_compressed(os.path.join(OUT, "ref_phases_el3d.npz"), **gen_elasticity3d(base))
        print("ref_phases_el3d.npz", os.path.getsize(os.path.join(OUT, "ref_phases_el3d.npz")) / 1e6, "MB")
        return
    data = {}
    data.update(gen_samplers(base))
    data.update(gen_networks_and_ops(base))
    np.savez_compressed(os.path.join(OUT, "ref_ops.npz"), **data)
    phases = {}
    phases.update(gen_advect(base))
    phases.update(gen_fluid(base))
    phases.update(gen_elasticity(base))
    np.savez_compressed(os.path.join(OUT, "ref_phases.npz"), **phases)
    for f in ("ref_ops.npz", "ref_phases.npz"):
        print(f, os.path.getsize(os.path.join(OUT, f)) / 1e6, "MB")


if __name__ == "__main__":
    main()
