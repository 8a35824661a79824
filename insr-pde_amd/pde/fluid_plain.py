"""The fluid phases written ONLY against the reference's public `base` API -- what an
unchanged user model file (fluid/model.py:72-151 style) runs on this package: plain torch
expressions for the residuals (torch.mean((a - b) ** 2), F.mse_loss), the separate band
samplers sample_boundary2D_separate, and one MLP call per point set.  None of the fused
helpers of pde/fluid.py (merged batches, loss groups, fused_forwards, the device sampler).

It exists to measure (bench.py --api plain) and test (tests/test_gpu_plain_api.py) the
drop-in claim: the jets behind gradient / divergence / laplace and the HIP backward still
run, and the graph-replayed loop still applies; only the model-side fusions are absent.
"""
import torch
import torch.nn.functional as F

from base import BaseModel, divergence, gradient, laplace, sample_boundary2D_separate, sample_random

from .fluid import Fluid2DModel


def _bands(n, device):
    """The two band pairs of a wall term: n // 100 points around the x-faces, then the y-faces."""
    m = n // 100
    return (sample_boundary2D_separate(m, side='horizontal', device=device).requires_grad_(True),
            sample_boundary2D_separate(m, side='vertical', device=device).requires_grad_(True))


class Fluid2DPlainModel(Fluid2DModel):
    """Fluid2DModel with phase bodies that use the reference API only (same losses)."""
    _dp_loss_reduction = 'mean'  # torch.mean over this rank's points: the all-reduce averages
    _insr_lazy_losses = False  # the reference bodies: torch expressions, no loss groups
    # ... which the loop lowers (base/lower.py) -- as for any model file that does not opt out
    _insr_lower = True

    def _sample_in_training(self):
        return sample_random(self._n_interior(), 2, device=self.device).requires_grad_(True)

    def _no_slip(self, n):
        """mean(u_x^2) on the x-face bands + mean(u_y^2) on the y-face bands."""
        bx, by = _bands(n, self.device)
        ux = self.velocity_field(bx)[..., 0]
        uy = self.velocity_field(by)[..., 1]
        return (torch.mean(ux ** 2) + torch.mean(uy ** 2)) * 1.0

    @BaseModel._training_loop
    def _initialize(self):
        x = self._sample_in_training()
        return {'main': F.mse_loss(self.velocity_field(x), self.init_cond_func(x))}

    @BaseModel._training_loop
    def _advect_velocity(self):
        x = self._sample_in_training()
        with torch.no_grad():
            u_old = self.velocity_field_prev(x).detach()
        u = self.velocity_field(x)
        foot = torch.clamp(x - u_old * self.cfg.dt, min=-1.0, max=1.0)
        with torch.no_grad():
            target = self.velocity_field_prev(foot).detach()
        return {'main': torch.mean((u - target) ** 2), 'bc': self._no_slip(x.shape[0])}

    @BaseModel._training_loop
    def _solve_pressure(self):
        x = self._sample_in_training()
        div_u = divergence(self.velocity_field(x), x).detach()
        lap_p = laplace(self.pressure_field(x), x)
        bx, by = _bands(self._n_interior(), self.device)
        dpx = gradient(self.pressure_field(bx), bx)[..., 0]
        dpy = gradient(self.pressure_field(by), by)[..., 1]
        return {'main': torch.mean((div_u - lap_p) ** 2), 'bc': torch.mean(dpx ** 2) + torch.mean(dpy ** 2)}

    @BaseModel._training_loop
    def _projection(self):
        x = self._sample_in_training()
        with torch.no_grad():
            u_old = self.velocity_field_prev(x).detach()
        grad_p = gradient(self.pressure_field(x), x).detach()
        u = self.velocity_field(x)
        return {'main': torch.mean((u - (u_old - grad_p)) ** 2), 'bc': self._no_slip(x.shape[0])}
