"""insr-pde_amd `base`: drop-in for the reference's base package (base/__init__.py:1-4).

    from base import BaseModel, gradient, divergence, laplace, jacobian, \
        sample_random, sample_uniform, sample_boundary, sample_boundary2D_separate, get_network

The hot path runs on libinsr_hip.so (gfx950); see DESIGN.md.
"""
from .baseModel import BaseModel
from .diff_ops import *  # noqa: F401,F403
from .sampling import *  # noqa: F401,F403
from .networks import *  # noqa: F401,F403
from .networks import MLP, Sine, get_network  # noqa: F401
from .optim import DevicePlateau, FusedAdam  # noqa: F401
from .losses import axpy_clamp, elastic_energy, fused_mse, mse_term, sq_losses, svd_energy, wall_mse, wall_term  # noqa: F401
from ._jet import UnsupportedPattern, advect_target, fused_forwards  # noqa: F401
from ._native import NativeUnavailable, NativeError  # noqa: F401
from . import sampling as _sampling
from .lower import sampler_api as _sampler_api

# the samplers a model file imports from `base` hand their draws to the loss lowering as ready leaves
# (base/lower.py sampler_api; outside lowering() they are the plain functions)
sample_random = _sampler_api(_sampling.sample_random)
sample_uniform = _sampler_api(_sampling.sample_uniform)
sample_boundary = _sampler_api(_sampling.sample_boundary)
sample_boundary2D_separate = _sampler_api(_sampling.sample_boundary2D_separate)
