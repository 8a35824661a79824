"""2-D inviscid Navier-Stokes on [-1, 1]^2 by operator splitting (the reference's
Fluid2DModel, fluid/model.py:11-151), written against the insr-pde_amd `base` API.

One timestep = three inner optimisation phases:
  _advect_velocity  semi-Lagrangian: u(x) ~ u_prev(clamp(x - u_prev(x) dt))  (:72-101)
  _solve_pressure   Poisson: lap p = div u, Neumann grad p . n = 0          (:103-125)
  _projection       u ~ u_prev - grad p, no-slip-normal boundary            (:127-151)

Under data parallelism each rank draws N / world collocation points (and its
share of the boundary bands); the HIP jets and the RCCL gradient all-reduce
in BaseModel._update_network make the step equal to one on the global batch.
"""
import os

import numpy as np
import torch

from base import (BaseModel, advect_target, axpy_clamp, divergence, fused_forwards, fused_mse, gradient, jacobian,
                  laplace,
                  merge_samples, mse_term, sample_boundary2D_pair, sample_boundary2D_separate, sample_random,
                  sample_random_and_bands2D, sample_uniform, sq_losses, wall_mse, wall_term)
from base.diff_ops import jacobian_only
from base.sampling import frozen_ahead, frozen_join

from .examples import get_examples


class Fluid2DModel(BaseModel):
    """inviscid Navier-Stokes equation. 2D fluid. [-1, 1]^2."""
    # every loss below is a mean over the GLOBAL point count (BaseModel._dp_total): the ranks' losses
    # and gradients sum to the global means, so the all-reduce needs no 1/world pass
    _dp_loss_reduction = 'sum'
    # the phase bodies return their sq_losses outputs and read the jet outputs those losses read nowhere
    # else: the loss groups ride in the reverse jets (base/losses.py lazy_losses)
    _insr_lazy_losses = True
    # written against the fused helpers already (merged batches, loss groups): no expression lowering
    _insr_lower = False

    def __init__(self, cfg):
        super().__init__(cfg)
        self.velocity_field = self._create_network(2, 2)
        self.velocity_field_prev = self._create_network(2, 2)
        self.pressure_field = self._create_network(2, 1)
        self._set_require_grads(self.velocity_field_prev, False)

    @property
    def _trainable_networks(self):
        return {'velocity': self.velocity_field, 'pressure': self.pressure_field}

    # ---- sampling ------------------------------------------------------------
    def _n_interior(self):
        """Points per rank: sample_resolution^2 split over ranks (strong scaling), or
        cfg.insr_points_per_rank when set (weak scaling)."""
        fixed = getattr(self.cfg, "insr_points_per_rank", None)
        return int(fixed) if fixed else max(1, self.sample_resolution ** 2 // self._dp_world())

    def _sample_in_training(self):
        """The interior batch.  On the GPU the iteration's wall bands come from the same
        launch (sample_random_and_bands2D) into the same buffer [interior; bands]: x is its
        first rows, and _merged(x) hands the whole buffer to the jets that take both."""
        n = self._n_interior()
        if torch.device(self.device).type == "cuda":
            buf = sample_random_and_bands2D(n, n // 100, device=self.device, merged=True).requires_grad_(True)
            x = buf[:n]
            self._insr_merged = (buf, x, (buf.shape[0] - n) // 2)
            return x
        return sample_random(n, 2, device=self.device).requires_grad_(True)

    def _merged(self, x):
        """([x; bands] as one leaf, n interior rows, nb rows per band pair): the sampler's
        buffer when x came from it, else x and _boundary_bands(n) concatenated."""
        n = x.shape[0]
        pre = self.__dict__.pop("_insr_merged", None)
        if pre is not None and pre[1] is x and "_boundary_pair" not in self.__dict__:
            return pre[0], n, pre[2]
        bxy, nb = self._boundary_bands(n)
        return merge_samples(x, bxy), n, nb

    def _boundary_pair(self, n_interior):
        nb = n_interior // 100
        bx = sample_boundary2D_separate(nb, side='horizontal', device=self.device).requires_grad_(True)
        by = sample_boundary2D_separate(nb, side='vertical', device=self.device).requires_grad_(True)
        return bx, by

    def _boundary_bands(self, n_interior):
        """Both band pairs as one (2 nb, 2) tensor [x-face bands; y-face bands] and nb.
        One sampler draw and one jet launch for both (a band is ~1% of the points, so
        these launches are latency-bound).  An instance-level `_boundary_pair` hook
        (tests pass recorded samples) takes precedence."""
        if "_boundary_pair" in self.__dict__:
            bx, by = self._boundary_pair(n_interior)
            return torch.cat([bx, by]), bx.shape[0]
        pre = self.__dict__.pop("_insr_merged", None)
        if pre is not None and pre[1].shape[0] == n_interior:
            return pre[0][n_interior:].detach().requires_grad_(True), pre[2]
        bxy = sample_boundary2D_pair(n_interior // 100, device=self.device).requires_grad_(True)
        return bxy, bxy.shape[0] // 2

    def sample_field(self, resolution, return_samples=False):
        grid = sample_uniform(resolution, 2, device=self.device, flatten=False).requires_grad_(True)
        u = self.velocity_field(grid)
        return (u, grid) if return_samples else u

    # ---- timestepping ----------------------------------------------------------
    @BaseModel._timestepping
    def initialize(self):
        if not hasattr(self, "init_cond_func"):
            self.init_cond_func = get_examples(self.cfg.init_cond)
        self._initialize()

    @BaseModel._training_loop
    def _initialize(self):
        x = self._sample_in_training()
        target = self.init_cond_func(x)
        return {'main': fused_mse(self.velocity_field(x), target, total=self._dp_total(target.numel()))}

    @BaseModel._timestepping
    def step(self):
        self.velocity_field_prev.load_state_dict(self.velocity_field.state_dict())
        self._advect_velocity()
        self._solve_pressure()
        self.velocity_field_prev.load_state_dict(self.velocity_field.state_dict())
        self._projection()

    # The wall terms evaluate the network on the boundary bands (~1% of the points).  In the
    # fused path (default) they are rows of the merged [interior; bands] batch; the unfused
    # path (cfg.insr_fuse_forwards = False) evaluates them in jets of their own.  (Measured and
    # removed: band / no-grad jets on a side stream -- 1.031 vs 1.009 ms per step, 46.3 vs 48.0
    # M pts/s: the interior jets hold every CU's registers / LDS, so nothing co-resides.)
    def _wall_loss(self, n_interior):
        """u_x = 0 on the x-faces, u_y = 0 on the y-faces: mean(u_x^2) + mean(u_y^2)
        (fluid/model.py:90-94) as one jet launch and one fused loss launch."""
        bxy, nb = self._boundary_bands(n_interior)
        return wall_mse(self.velocity_field(bxy), nb, total=self._dp_total(nb))

    def _pressure_wall_loss(self, n_interior):
        """mean(dp/dx^2) + mean(dp/dy^2) on the bands (fluid/model.py:116-120)."""
        bxy, nb = self._boundary_bands(n_interior)  # one jet launch for both bands
        gp = gradient(self.pressure_field(bxy), bxy)
        return wall_mse(gp, nb, total=self._dp_total(nb))

    def _advect_target(self, x):
        with torch.no_grad():
            u_prev = self.velocity_field_prev(x).detach()
            foot = axpy_clamp(x.detach(), u_prev, -self.cfg.dt, -1.0, 1.0)  # clamp(x - dt u_prev, -1, 1)
            return self.velocity_field_prev(foot)

    def _velocity_divergence(self, x):
        with torch.no_grad():  # the reference detaches div u: no reverse jet, no saved streams
            return divergence(self.velocity_field(x), x)

    def _projection_target(self, x):
        with torch.no_grad():  # both detached in the reference as well
            return self.velocity_field_prev(x).detach(), gradient(self.pressure_field(x), x)

    # Horizontal fusion (cfg.insr_fuse_forwards, default on):
    # the frozen field's value jet and the trainable field's value jet at the same points
    # are independent -- ONE insr_siren_jet_fwd_multi launch holds two blocks per CU
    # instead of two latency-bound launches of one block per CU each.
    def _fused_pair(self):
        return getattr(self.cfg, "insr_fuse_forwards", True)

    # Frozen work ahead (cfg.insr_frozen_ahead, default OFF: measured slower, below).  Inside a group of U
    # iterations replayed as one hipGraph (base/_loop.py run_group; their points drawn by ONE sampler launch,
    # base.sampling.draw_ahead), what a phase evaluates on networks it does not train -- the advection's
    # semi-Lagrangian target on u_prev, the pressure phase's div u, the projection's u_prev and grad p -- does
    # not depend on any iteration's update: with it on, that runs ONCE for all U iterations' points
    # (base.sampling.frozen_ahead), and each iteration's forward launch holds only the trained network's jet.
    # Same-box A/B (profiles/r06/frozen_ahead/, 40-step lines, two rounds): headline 100.9 / 101.3 M pts/s on
    # vs 108.0 / 108.2 M off, fluid2DtlgnM 8-way DP-path shard 0.344 / 0.345 vs 0.322 / 0.322 ms -- the mixed
    # launch already runs the frozen job beside the trained one for free (both latency-bound); a batch of
    # its own is one more launch.  Side stream: 102.2 / 102.5 M, 0.344 ms; pipelined: 91.4 / 92.1 M, 0.378 ms.
    # cfg.insr_frozen_stream (default off): that evaluation runs on a side stream, overlapping the group's first
    # trained-network forward; _join makes the main stream wait before the first loss reads it.
    # cfg.insr_frozen_ahead = "pipe": per iteration on the side stream, one iteration ahead (under the previous
    # iteration's reverse jets, all-reduce and Adam step; base.sampling.frozen_ahead).
    def _ahead(self, name, x, fn):
        mode = getattr(self.cfg, "insr_frozen_ahead", False)
        if not mode:
            return None
        pipe = mode == "pipe"
        side = None
        if pipe or getattr(self.cfg, "insr_frozen_stream", False):
            side = self.__dict__.get("_insr_frozen_side")
            if side is None:
                side = self._insr_frozen_side = torch.cuda.Stream(device=self.device)
        return frozen_ahead(name, x, fn, stream=side, pipe=pipe)

    @staticmethod
    def _join(name):
        frozen_join(name)

    def _target_all(self, X):
        return (advect_target(self.velocity_field_prev, X, self.cfg.dt, -1.0, 1.0)[0],)

    def _div_all(self, X):
        return (jacobian_only(self.velocity_field(X), X),)

    def _projection_all(self, X):
        with fused_forwards():
            u_prev = self.velocity_field_prev(X)
            grad_p = gradient(self.pressure_field(X), X)
        return u_prev, grad_p

    @BaseModel._training_loop
    def _advect_velocity(self):
        x = self._sample_in_training()
        if self._fused_pair():
            xa, n, nb = self._merged(x)
            pre = self._ahead("advect", x, self._target_all)
            if pre is not None:  # the group's targets, computed once (_ahead)
                u_target, = pre
                ua = self.velocity_field(xa)
                self._join("advect")
            else:
                # the frozen field's semi-Lagrangian target u_prev(clamp(x - dt u_prev(x), -1, 1))
                # (two value jets and the foot, point-local: one job) beside the trainable field's
                # value jet over [x; bands]: one mixed launch
                with fused_forwards():
                    u_target, _ = advect_target(self.velocity_field_prev, x, self.cfg.dt, -1.0, 1.0)
                    ua = self.velocity_field(xa)
            # mean((u - u_target)^2) over the interior rows and the wall terms on the band rows,
            # one launch
            main, bc = sq_losses(mse_term(ua, u_target, count=u_target.numel(), total=self._dp_total(u_target.numel())),
                                 wall_term(ua, nb, row0=n, total=self._dp_total(nb)))
            return {'main': main, 'bc': bc}
        bc = self._wall_loss(x.shape[0])
        u_target = self._advect_target(x)
        return {'main': fused_mse(self.velocity_field(x), u_target, total=self._dp_total(u_target.numel())), 'bc': bc}

    @BaseModel._training_loop
    def _solve_pressure(self):
        x = self._sample_in_training()
        if self._fused_pair():
            # The wall term needs grad p on the bands, which the Laplacian jet carries anyway
            # (its tangent streams): ONE pressure jet over [interior; bands] (base.merge_samples)
            # instead of a separate gradient jet + reverse jet for 2% of the points.  The
            # Laplacian rows of the band points get zero adjoint.
            xa, n, nb = self._merged(x)
            pre = self._ahead("pressure", x, self._div_all)
            if pre is not None:  # the group's velocity Jacobians, computed once (_ahead)
                Ju, = pre
                lap_p, grad_p = laplace(self.pressure_field(xa), xa, return_grad=True)
                self._join("pressure")
            else:
                # the velocity's Jacobian jet and the pressure's Laplacian jet are independent: one
                # mixed-mode launch (base.fused_forwards); outputs are read after the scope
                with fused_forwards():
                    with torch.no_grad():  # div u = du/dx + dv/dy, read off the velocity's Jacobian
                        Ju = jacobian_only(self.velocity_field(x), x)
                    lap_p, grad_p = laplace(self.pressure_field(xa), xa, return_grad=True)
            # mean((lap p - du/dx - dv/dy)^2) over the interior rows (= mean((div u - lap p)^2))
            # and the wall terms, one launch; the diagonal of J is read in place (stride 4)
            main, bc = sq_losses(mse_term(lap_p, Ju[:, 0, 0], Ju[:, 1, 1], alpha=1.0, beta=-1.0, gamma=-1.0, count=n,
                                          total=self._dp_total(n)),
                                 wall_term(grad_p, nb, row0=n, total=self._dp_total(nb)))
            return {'main': main, 'bc': bc}
        bc = self._pressure_wall_loss(x.shape[0])
        div_u = self._velocity_divergence(x)
        main = fused_mse(div_u, laplace(self.pressure_field(x), x), total=self._dp_total(div_u.numel()))  # rho = 1
        return {'main': main, 'bc': bc}

    @BaseModel._training_loop
    def _projection(self):
        x = self._sample_in_training()
        if self._fused_pair():
            xa, n, nb = self._merged(x)
            pre = self._ahead("projection", x, self._projection_all)
            if pre is not None:  # the group's u_prev and grad p, computed once (_ahead)
                u_prev, grad_p = pre
                ua = self.velocity_field(xa)
                self._join("projection")
            else:
                # frozen velocity (value), pressure gradient (detached) and the trainable velocity
                # over [x; bands]: independent jets, one mixed-mode launch
                with fused_forwards():
                    with torch.no_grad():
                        u_prev = self.velocity_field_prev(x)
                        grad_p = gradient(self.pressure_field(x), x)
                    ua = self.velocity_field(xa)
            u_prev = u_prev.detach()
            main, bc = sq_losses(mse_term(ua, None, u_prev, grad_p, gamma=-1.0, delta=-1.0, count=u_prev.numel(),
                                          total=self._dp_total(u_prev.numel())),
                                 wall_term(ua, nb, row0=n, total=self._dp_total(nb)))
            return {'main': main, 'bc': bc}
        bc = self._wall_loss(x.shape[0])
        u_prev, grad_p = self._projection_target(x)
        # mean((u - (u_prev - grad_p))^2): r = 1*(u + 0) + (-1)*(u_prev + (-1)*grad_p)
        main = fused_mse(self.velocity_field(x), None, u_prev, grad_p, gamma=-1.0, delta=-1.0,
                         total=self._dp_total(u_prev.numel()))
        return {'main': main, 'bc': bc}

    # ---- output (host side; PNG figures are out of scope) ---------------------
    def field_quantities(self, resolution):
        """The fields fluid/model.py:207-217 writes, on the (R, R) cell-centred grid:
        velocity u (R, R, 2), speed |u| (R, R) and vorticity curl u = dv/dx - du/dy (R, R)
        from ONE gradient jet of the velocity net (no autograd passes)."""
        grid = sample_uniform(resolution, 2, device=self.device, flatten=False).requires_grad_(True)
        with torch.no_grad():  # no parameter gradients: no saved streams
            u = self.velocity_field(grid)
            jac, _ = jacobian(u, grid)  # (R, R, 2, 2)
        u_mag = torch.sqrt(torch.sum(u ** 2, dim=-1))
        u_curl = jac[..., 1, 0] - jac[..., 0, 1]
        return u.detach(), u_mag.detach(), u_curl.detach(), grid.detach()

    def write_output(self, output_folder):
        """fluid/model.py:207-232: t###.npy = the velocity grid (as the reference), plus the
        speed and curl arrays its PNGs are drawn from (t###_mag.npy, t###_curl.npy)."""
        u, mag, curl, _ = self.field_quantities(self.vis_resolution)
        os.makedirs(output_folder, exist_ok=True)
        np.save(os.path.join(output_folder, f"t{self.timestep:03d}.npy"), u.cpu().numpy())
        np.save(os.path.join(output_folder, f"t{self.timestep:03d}_mag.npy"), mag.cpu().numpy())
        np.save(os.path.join(output_folder, f"t{self.timestep:03d}_curl.npy"), curl.cpu().numpy())
