"""Elastodynamics by energy minimisation on a deformation field q = x + f(x)
(the reference's ElasticityModel, elasticity/model.py:15-250, losses from
elasticity/losses.py:6-39), on the insr-pde_amd `base` API.

Energy terms (all SUMS over collocation points, as in the reference):
  arap        r_a  sum (sigma_i - 1)^2         sigma = singular values of dq/dx
  volume      r_v  sum (prod sigma_i - 1)^2
  kinematics  r_k  sum |qdot - qdot_prev|^2     qdot = (q - q_prev)/dt
  external    -dt  sum qdot . f_ext             (first T_ext timesteps)
  constraint(_right[_compress]) r_c sum |f(x_fixed) - target|^2
  collision(_sphere)  -dt sum qdot . penalty force on penetrating points (3-D sphere: the
              reference's broadcast makes it -dt r_c (sum dist) (sum qdot . dir), reproduced as is)

Geometry: the synthetic box [-1, 1]^d (use_mesh=False), or a tet / triangle mesh
(use_mesh=True, cfg.mesh_path: MEDIT .mesh or .obj; pde/mesh.py): volume-weighted
random points ('random') and the mesh vertices ('uniform'), as elasticity/model.py:198-207.
"""
import os

import numpy as np
import torch

from base import BaseModel, elastic_energy, fused_forwards, merge_samples, sample_random, sample_uniform
from base.sampling import sample_boxes_into
from base.diff_ops import jacobian_only



class ElasticityModel(BaseModel):
    _dp_loss_reduction = 'sum'
    _insr_lower = False  # written against the fused helpers (no expression lowering, base/lower.py)

    def __init__(self, cfg):
        super().__init__(cfg)
        self.dim = cfg.dim
        self.deformation_field = self._create_network(self.dim, self.dim)
        self.deformation_field_prev = self._create_network(self.dim, self.dim)
        self.deformation_field_prev_prev = self._create_network(self.dim, self.dim)
        self._set_require_grads(self.deformation_field_prev, False)
        self._set_require_grads(self.deformation_field_prev_prev, False)
        with torch.no_grad():
            self.deformation_field_prev.load_state_dict(self.deformation_field.state_dict())
            self.deformation_field_prev_prev.load_state_dict(self.deformation_field.state_dict())
        self._init_params(cfg)

    def _init_params(self, cfg):
        d, dev = self.dim, self.device
        self.energy = list(cfg.energy)
        self.use_mesh = bool(getattr(cfg, "use_mesh", False))
        if self.use_mesh:
            self._init_mesh(cfg.mesh_path)
        self.sample_pattern = list(cfg.sample_pattern)
        self.ratio_arap, self.ratio_volume = cfg.ratio_arap, cfg.ratio_volume
        self.ratio_kinematics, self.ratio_constraint = cfg.ratio_kinematics, cfg.ratio_constraint
        self.ratio_collide = cfg.ratio_collide
        self.external_force_timesteps = cfg.external_force_timesteps
        self.plane_height = cfg.plane_height
        self.circle_radius = cfg.collide_circle_radius
        vec = lambda *v: torch.tensor(v[:d], dtype=torch.float32, device=dev)  # noqa: E731
        self.external_force = vec(cfg.external_force_x, cfg.external_force_y, cfg.external_force_z)
        self.constraint_offset_right = vec(cfg.constraint_right_offset_x, cfg.constraint_right_offset_y,
                                           cfg.constraint_right_offset_z)
        self.circle_center = vec(cfg.collide_circle_x, cfg.collide_circle_y, cfg.collide_circle_z)
        self.sample_resolution_init = self.sample_resolution if self.use_mesh else {2: 500, 3: 100}[d]

    def _init_mesh(self, path):
        """elasticity/model.py:75-93 (meshio + torchgp restated in pde/mesh.py)."""
        from .mesh import MeshSampler, load_mesh
        V, E, SF = load_mesh(path, self.dim, device=self.device)
        self.mesh_V, self.mesh_F, self.mesh_SF = V, E, SF
        self.mesh_sampler = MeshSampler(V.double().cpu(), E, device=self.device)
        self.surface_sampler = MeshSampler(V.double().cpu(), SF, device=self.device) if self.dim == 3 else \
            self.mesh_sampler

    @property
    def _trainable_networks(self):
        return {'deformation': self.deformation_field}

    # ---- sampling ------------------------------------------------------------
    # Data parallelism.  Strong scaling (the default under torch.distributed): rank r of K draws ONLY its
    # share of every part of the global batch -- rows [r n / K, (r + 1) n / K) of each 'uniform' part
    # (grid / mesh vertices: the same rows the global draw would hold) and as many fresh rows of each
    # 'random' part (independent uniform draws: the union over ranks has the global batch's size and
    # distribution; no rank draws the world-sized batch).  cfg.insr_dp_weak: every rank draws the whole
    # batch (weak scaling).  cfg.insr_shard = (r, K): one process runs rank r's share of a K-rank strong
    # run (bench.py --shard-of K measures exactly this code).  Ranks draw independent points: the device
    # samplers fold the rank into their key (base.sampling.sampler_seed); a sharded rank's mesh draw takes
    # its uniforms from the same device stream (_mesh_draw; on the CPU a generator keyed alike).
    def _shard(self):
        """(r, K): this process's share of the global batch (K = 1: the whole batch)."""
        emu = getattr(self.cfg, "insr_shard", None)
        if emu:
            return int(emu[0]), int(emu[1])
        world = self._dp_world()
        if world == 1 or getattr(self.cfg, "insr_dp_weak", False):
            return 0, 1
        return torch.distributed.get_rank(), world

    def _rows(self, n):
        """(first, count) of this process's rows of a part of n global rows."""
        r, k = self._shard()
        a, b = r * n // k, (r + 1) * n // k
        return a, b - a

    def _mesh_draw(self, sampler, n):
        """n volume-weighted mesh points (elasticity/model.py:200-207).  One unsharded rank: torch's default
        generator, as the reference (a hipGraph capture registers it).  A rank of a sharded run on the GPU:
        the uniforms come from the rank-keyed device Philox sampler (base.sampling.sample_boxes, the box
        scenes' stream) -- capturable, each replay draws fresh points, and ranks seeded alike draw
        independent points.  (A private torch.Generator is not registered with the capture: the strong
        path's graph came out empty and the phase ran eagerly, round 5.)  On the CPU: _mesh_generator."""
        r, k = self._shard()
        if (k == 1 and self._dp_world() == 1) or torch.device(self.device).type != "cuda":
            return sampler.sample(n, generator=self._mesh_generator())
        from base.sampling import sample_boxes
        m = sampler.uniforms_per_point()  # 6 (tets) or 4 (triangles): n * m / 2 rows of 2 or 3 coordinates
        dim = 3 if m % 3 == 0 else 2
        u = sample_boxes([(n * m // dim, (0.0,) * dim, (1.0,) * dim)], dim, device=self.device) if n > 0 else \
            torch.zeros(0, dim, device=self.device)
        return sampler.sample(n, uniforms=u.view(n, m))

    def _mesh_generator(self):
        """None (the default generator, as the reference) on one unsharded rank; else (a CPU rank of a
        sharded run) a generator keyed by the torch seed with the rank folded in (base.sampling.sampler_seed),
        re-made when torch is re-seeded -- ranks seeded alike still draw independent mesh points."""
        r, k = self._shard()
        world = self._dp_world()
        if k == 1 and world == 1:
            return None
        from base.sampling import reseed_epoch, sampler_seed
        rank = r if k > 1 else torch.distributed.get_rank()
        dev = torch.device(self.device)
        if dev.type == "cuda":
            idx = dev.index if dev.index is not None else torch.cuda.current_device()
            seed = torch.cuda.default_generators[idx].initial_seed()
        else:
            seed = torch.initial_seed()
        key = (seed, reseed_epoch(), rank)
        cached = self.__dict__.get("_insr_mesh_gen")
        if cached is None or cached[0] != key:
            g = torch.Generator(device=dev)
            g.manual_seed(sampler_seed(seed, rank) & 0x7FFFFFFFFFFFFFFF)
            cached = self.__dict__["_insr_mesh_gen"] = (key, g)
        return cached[1]

    def _sample_in_training(self, resolution):
        """elasticity/model.py:198-220, this process's share of it (see above)."""
        d, parts = self.dim, []
        for s in self.sample_pattern:
            if s == 'random':
                n = self._rows(resolution ** d)[1]
                if self.use_mesh:  # elasticity/model.py:200-207: volume-weighted points of the mesh
                    parts.append(self._mesh_draw(self.mesh_sampler, n)[:, :d])
                else:
                    parts.append(sample_random(n, d, device=self.device).requires_grad_(True))
            elif s == 'uniform':
                full = self.mesh_V[:, :d] if self.use_mesh else self._uniform_grid(resolution, d)
                a, n = self._rows(full.shape[0])
                parts.append(full if n == full.shape[0] else full[a:a + n])
            else:
                raise NotImplementedError(s)
        x = torch.cat(parts, dim=0)
        return x.requires_grad_(True) if x.is_leaf else x

    def _uniform_grid(self, resolution, d):
        """sample_uniform(resolution, d) -- the same cell-centred grid every iteration (no RNG):
        built once per (resolution, d) instead of ~5 launches per iteration (a leaf that
        requires grad, as the reference's; consumers only read it)."""
        cache = self.__dict__.setdefault("_insr_grids", {})
        key = (resolution, d)
        if key not in cache:
            cache[key] = sample_uniform(resolution, d, device=self.device).requires_grad_(True)
        return cache[key]

    def _sample_fixed_in_training(self, resolution):
        """Points on the x = -1 face (left) and x = +1 face (right), this process's share of each part;
        none on a mesh (the reference's mesh scenes use no positional constraint, elasticity/model.py:228)."""
        d, left, right = self.dim, [], []
        if self.use_mesh:
            empty = torch.zeros(0, d, device=self.device).requires_grad_(True)
            return empty, empty
        for s in self.sample_pattern:
            if s == 'random':
                n = self._rows(resolution)[1]
                faces = [sample_random(n, d - 1, device=self.device) for _ in range(2)]
            elif s == 'uniform':
                g = self._uniform_grid(resolution, d - 1).detach()
                a, n = self._rows(g.shape[0])
                faces = [g[a:a + n], g[a:a + n]]
            else:
                raise NotImplementedError(s)
            one = torch.ones(faces[0].shape[0], 1, device=self.device)
            left.append(torch.cat([-one, faces[0]], 1))
            right.append(torch.cat([one, faces[1]], 1))
        return torch.cat(left, 0).requires_grad_(True), torch.cat(right, 0).requires_grad_(True)

    # ---- timestepping ----------------------------------------------------------
    @BaseModel._timestepping
    def initialize(self):
        self._initialize()
        self.deformation_field_prev_prev.load_state_dict(self.deformation_field.state_dict())
        self.deformation_field_prev.load_state_dict(self.deformation_field.state_dict())

    @BaseModel._training_loop
    def _initialize(self):
        """mean(f(x)^2) over the GLOBAL batch (elasticity/model.py:109-117): a sum over this
        rank's shard / the global element count, so the 'sum' all-reduce of _dp_sync gives
        the reference's mean at any world size."""
        x = self._sample_in_training(self.sample_resolution_init)
        y = self.deformation_field(x)
        world = self._dp_world()
        if world == 1:
            return {'main': torch.mean(y ** 2)}
        count = y.numel() * (world if getattr(self.cfg, "insr_dp_weak", False) else 1)
        if not getattr(self.cfg, "insr_dp_weak", False):
            count = self._global_rows(self.sample_resolution_init) * y.shape[1]
        return {'main': torch.sum(y ** 2) / count}

    def _global_rows(self, resolution):
        """Rows of the global draw _sample_in_training shards."""
        if self.use_mesh:
            return sum(resolution ** self.dim if s == 'random' else self.mesh_V.shape[0] for s in self.sample_pattern)
        return len(self.sample_pattern) * resolution ** self.dim

    @BaseModel._timestepping
    def step(self):
        self.deformation_field_prev_prev.load_state_dict(self.deformation_field_prev.state_dict())
        self.deformation_field_prev.load_state_dict(self.deformation_field.state_dict())
        self._solve_deformation()

    @BaseModel._training_loop
    def _solve_deformation(self):
        fast = self._box_batch(self.sample_resolution)
        if fast is not None:
            xa, x, fixed_l, fixed_r = fast
            return {'main': self.energy_of(x, fixed_l, fixed_r, xa=xa)}
        x = self._sample_in_training(self.sample_resolution)
        fixed_l, fixed_r = self._sample_fixed_in_training(self.sample_resolution)
        return {'main': self.energy_of(x, fixed_l, fixed_r)}

    def _box_batch(self, resolution):
        """The box scene's iteration batch on the GPU (one rank, or weak scaling): the merged
        jet input [x; fixed_l; fixed_r] (each in sample_pattern order, rows as
        _sample_in_training / _sample_fixed_in_training / merge_samples lay them out) as ONE
        persistent leaf buffer -- the 'uniform' grid rows are written once, the 'random' rows
        are redrawn in place by ONE device sampler launch (base.sample_boxes_into) instead of
        ~17 draw / fill / cat launches.  Same distributions; None where it does not apply."""
        if self.use_mesh or torch.device(self.device).type != "cuda":
            return None
        if "_sample_in_training" in self.__dict__ or "_sample_fixed_in_training" in self.__dict__:
            return None  # an instance-level sampler (tests pass recorded samples) takes precedence
        d = self.dim
        use_l = 'constraint' in self.energy
        use_r = any(t in self.energy for t in ('constraint_right', 'constraint_right_compress'))
        shard = self._shard()
        key = (resolution, use_l, use_r, shard)
        cache = self.__dict__.setdefault("_insr_box_batch", {})
        if key not in cache:
            rows, boxes, fill = 0, [], []

            def put(kind, n, lo, hi, const):
                """One part of the batch: this process's share of its n global rows."""
                nonlocal rows
                a, m = self._rows(n)
                if kind == 'random':
                    boxes.append((rows, m, lo, hi))
                elif kind == 'uniform':
                    fill.append((rows, const[a:a + m]))
                else:
                    raise NotImplementedError(kind)
                rows += m
            for s in self.sample_pattern:
                put(s, resolution ** d, [-1.0] * d, [1.0] * d,
                    sample_uniform(resolution, d, device=self.device) if s == 'uniform' else None)
            n = rows
            sides = ([-1.0] if use_l else []) + ([1.0] if use_r else [])
            nside = []
            for side in sides:
                r0 = rows
                for s in self.sample_pattern:
                    m = resolution if s == 'random' else resolution ** (d - 1)
                    g = None
                    if s == 'uniform':
                        g = sample_uniform(resolution, d - 1, device=self.device)
                        g = torch.cat([torch.full((g.shape[0], 1), side, device=self.device), g], 1)
                    put(s, m, [side] + [-1.0] * (d - 1), [side] + [1.0] * (d - 1), g)
                nside.append(rows - r0)
            buf = torch.empty(rows, d, device=self.device)
            with torch.no_grad():
                for r0, g in fill:
                    buf[r0:r0 + g.shape[0]].copy_(g)
            buf.requires_grad_(True)
            nl = nside[0] if use_l else 0
            nr = nside[-1] if use_r else 0
            empty = torch.zeros(0, d, device=self.device)
            fixed_l = buf[n:n + nl] if use_l else empty
            fixed_r = buf[n + nl:n + nl + nr] if use_r else empty
            cache[key] = (buf, [b for b in boxes if b[1] > 0], buf[:n], fixed_l, fixed_r)
        buf, boxes, x, fixed_l, fixed_r = cache[key]
        if boxes:
            sample_boxes_into(buf.detach(), boxes)
        return buf, x, fixed_l, fixed_r

    def energy_of(self, x, fixed_l, fixed_r, xa=None):
        """elasticity/model.py:131-189.  The interior points and the fixed points the
        constraint terms need go through ONE jet launch of the deformation field
        (base.merge_samples, or the caller's merged buffer xa); every term reads its rows."""
        dt, n = self.dt, x.shape[0]
        if self.dim == 3 and 'collision_sphere' in self.energy and self._shard()[1] > 1 and \
                not self.__dict__.get("_insr_sphere_warned"):
            self._insr_sphere_warned = True
            import warnings
            warnings.warn("elasticity: the 3-D collision_sphere term is a product of two sums over the batch "
                          "(elasticity/losses.py:35); a rank of a strong-scaling run forms it from its own shard's "
                          "sums, so the all-reduced energy is not the single-process one (DESIGN.md §7)",
                          RuntimeWarning, stacklevel=2)
        use_l = 'constraint' in self.energy
        use_r = any(t in self.energy for t in ('constraint_right', 'constraint_right_compress'))
        parts = [x] + ([fixed_l] if use_l else []) + ([fixed_r] if use_r else [])
        if xa is None:
            xa = merge_samples(*parts) if len(parts) > 1 else x
        row_l = n
        row_r = n + (fixed_l.shape[0] if use_l else 0)
        # the two frozen fields' value jets at x are independent of each other and of the
        # trainable field's jet: one fused launch for the two value jets (the trainable one,
        # a Jacobian jet after iteration 0, is grouped by itself)
        with fused_forwards():
            with torch.no_grad():
                f_prev = self.deformation_field_prev(x)
                f_pp = self.deformation_field_prev_prev(x)
            fa = self.deformation_field(xa)
        # every term in ONE launch with its unit-seed gradient (base.elastic_energy): the
        # singular values of dq/dx = J + I, kinematics, external force, collisions and the
        # positional constraints; J is the Jacobian jet of the same field launch
        J = jacobian_only(fa, xa) if ('arap' in self.energy or 'volume' in self.energy) else None
        sign = -1.0 if 'constraint_right_compress' in self.energy else 1.0
        ratios = {'arap': self.ratio_arap, 'volume': self.ratio_volume, 'kinematics': self.ratio_kinematics,
                  'constraint': self.ratio_constraint, 'constraint_right': self.ratio_constraint,
                  'constraint_right_compress': self.ratio_constraint, 'collision': self.ratio_collide,
                  'collision_sphere': self.ratio_collide}
        total, _ = elastic_energy(
            fa, J, x, f_prev, f_pp, n=n, dt=dt, energy=self.energy, ratios=ratios,
            ext=self._host_vec('external_force'), external_on=self.timestep <= self.external_force_timesteps,
            rows_l=(row_l, fixed_l.shape[0] if use_l else 0), rows_r=(row_r, fixed_r.shape[0] if use_r else 0),
            target=[sign * v for v in self._host_vec('constraint_offset_right')], plane_height=self.plane_height,
            center=self._host_vec('circle_center'), radius=self.circle_radius)
        return total

    def _host_vec(self, name):
        """A cfg vector (external force, offsets, sphere centre) as host floats, cached."""
        cache = self.__dict__.setdefault("_insr_host_vecs", {})
        if name not in cache:
            cache[name] = [float(v) for v in getattr(self, name).cpu()]
        return cache[name]

    # ---- output (host side; PNG figures are out of scope) ---------------------------
    def sample_visualization(self, resolution):
        """elasticity/model.py:255-270: the box grid + both fixed faces, or on a mesh the
        surface samples + the mesh vertices."""
        d, dev = self.dim, self.device
        if self.use_mesh:
            return torch.cat([self.surface_sampler.sample(resolution)[:, :d], self.mesh_V[:, :d]], dim=0)
        pts = sample_uniform(resolution, d, device=dev)
        face = sample_uniform(resolution, d - 1, device=dev)
        one = torch.ones(face.shape[0], 1, device=dev)
        return torch.cat([pts, torch.cat([-one, face], 1), torch.cat([one, face], 1)], dim=0)

    def deformed_points(self, resolution=None):
        """q = x + f(x) at the visualisation samples (elasticity/model.py:277-288)."""
        if getattr(self, "_vis_samples", None) is None:
            self._vis_samples = self.sample_visualization(resolution or self.vis_resolution)
        x = self._vis_samples
        with torch.no_grad():
            return (self.deformation_field(x) + x).detach()

    def write_output(self, output_folder):
        """elasticity/model.py:311-317: t###_deformation.ply (ASCII point cloud, 2-D lifted to
        z = 0, as write_pointcloud_to_file) and t###_deformation.npy."""
        q = self.deformed_points().cpu().numpy().astype(np.float64)
        os.makedirs(output_folder, exist_ok=True)
        np.save(os.path.join(output_folder, f"t{self.timestep:03d}_deformation.npy"), q)
        write_ply(os.path.join(output_folder, f"t{self.timestep:03d}_deformation.ply"), q)


def write_ply(path, points):
    """ASCII PLY point cloud (x y z per vertex; 2-D points get z = 0)."""
    if points.shape[1] == 2:
        points = np.hstack([points, np.zeros((points.shape[0], 1))])
    with open(path, "w") as f:
        f.write("ply\nformat ascii 1.0\nelement vertex %d\nproperty double x\nproperty double y\n"
                "property double z\nend_header\n" % points.shape[0])
        np.savetxt(f, points, fmt="%.9g")
