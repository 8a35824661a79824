"""The advection phase written ONLY against the reference's public `base` API -- what an unchanged
user model file (advection/model.py:68-91 style) runs on this package: plain torch expressions for
the midpoint residual and the Dirichlet band term, a separate boundary sampler, one network call per
point set.  None of the fused helpers of pde/advection.py (merged batches, fused_forwards, fused_mse).

The training loop lowers its residual expressions (base/lower.py): both losses of an iteration are
one fused loss-group launch.  It exists to measure (bench.py --config advect1D --api plain) and test
(tests/test_gpu_plain_api.py) the drop-in claim for the 1-D model as pde/fluid_plain.py does for fluid.
"""
import torch
import torch.nn.functional as F

from base import BaseModel, gradient, sample_boundary, sample_random

from .advection import Advection1DModel


class Advection1DPlainModel(Advection1DModel):
    """Advection1DModel with the reference's phase bodies (same losses)."""
    _dp_loss_reduction = 'mean'  # torch.mean over this rank's points: the all-reduce averages
    _insr_lower = True  # the reference bodies' torch expressions, lowered by the loop (base/lower.py)

    def _sample_in_training(self):
        return sample_random(self._n_interior(), 1, device=self.device).requires_grad_(True) * self.length / 2

    @BaseModel._training_loop
    def _initialize(self):
        samples = self._sample_in_training()
        ref = self.init_cond_func(samples)
        return {'main': F.mse_loss(self.field(samples), ref)}

    @BaseModel._training_loop
    def _advect(self):
        samples = self._sample_in_training()
        prev_u = self.field_prev(samples)
        curr_u = self.field(samples)
        dudt = (curr_u - prev_u) / self.dt
        grad_u = gradient(curr_u, samples)
        grad_u0 = gradient(prev_u, samples).detach()
        loss = torch.mean((dudt + self.vel * (grad_u + grad_u0) / 2.) ** 2)
        boundary_samples = sample_boundary(max(self._n_interior() // 100, 10), 1, device=self.device) * self.length / 2
        bound_u = self.field(boundary_samples)
        return {'main': loss, 'bc': torch.mean(bound_u ** 2) * 1.}
