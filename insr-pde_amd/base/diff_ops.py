"""Spatial differential operators, drop-in for base/diff_ops.py:6-82 of the reference.

Same names, signatures, return shapes and status semantics.  Instead of
torch.autograd.grad(..., create_graph=True) passes, each operator asks the HIP
library for ONE forward Taylor jet of the SIREN that produced `y` (see
base/_jet.py) and assembles the requested quantity from its streams:

  reference (base/diff_ops.py)            here
  gradient   :53-58  d(sum_c g_c y_c)/dx   sum_c g_c J[c, :]           (GRAD jet)
  divergence :44-50  sum_i dy_i/dx_i       trace of J                  (GRAD jet)
  jacobian   :61-82  (N, dy, dx), status   J (+ I if y = f(x) + x)    (GRAD jet)
  laplace    :33-41  div(grad y)           sum_c Lap y_c              (LAP jet, d_in <= 3)
  hessian    :6-30   (.., dy, dx, dx)      not on the INSR-PDE path: raises

All results stay differentiable w.r.t. the network parameters (loss.backward()
runs the HIP reverse jet).  `status` is returned, never raised (-1 on NaN).
"""
import torch

from . import _jet
from . import _native as nat

__all__ = ["hessian", "laplace", "divergence", "gradient", "jacobian"]


def _resolve(y, x, opname):
    m = _jet.match(y, x)
    if m is None:
        gsrc = getattr(y, "_insr_gradient_of", None)
        if gsrc is not None and gsrc[1] is x and opname == "divergence":
            return ("gradient-of",) + gsrc
        raise _jet.UnsupportedPattern(
            f"{opname}(y, x): y is not a SIREN output of x (or f(x) + x) produced by base.MLP; "
            "the HIP path only differentiates recognised SIREN graphs")
    return m


def gradient(y, x, grad_outputs=None):
    """d(sum_c grad_outputs_c * y_c)/dx, shape x.shape (base/diff_ops.py:53-58)."""
    mlp, value, affine = _resolve(y, x, "gradient")
    _, J, _ = _jet.jet_of(mlp, value, x, nat.MODE_GRAD)  # (..., dout, din)
    if grad_outputs is None:
        # scalar net: a view (no launch, and its backward is a view too)
        g = J.squeeze(-2) if J.shape[-2] == 1 else J.sum(dim=-2)
        if affine:
            g = g + 1.0
    else:
        go = grad_outputs
        g = (go.unsqueeze(-1) * J).sum(dim=-2)
        if affine:
            g = g + go
    g._insr_gradient_of = (mlp, x, value, affine, grad_outputs is None)
    return g


def divergence(y, x):
    """sum_i dy_i/dx_i, shape (..., 1) (base/diff_ops.py:44-50)."""
    r = _resolve(y, x, "divergence")
    if r[0] == "gradient-of":
        # divergence(gradient(f, x), x) with unit grad_outputs == laplace(f, x)
        _, mlp, _, value, affine, unit = r
        if not unit:
            raise _jet.UnsupportedPattern("divergence of a weighted gradient is not fused")
        _, _, lap = _jet.jet_of(mlp, value, x, nat.MODE_LAP)
        return lap if lap.shape[-1] == 1 else lap.sum(dim=-1, keepdim=True)
    mlp, value, affine = r
    _, J, _ = _jet.jet_of(mlp, value, x, nat.MODE_GRAD)
    k = min(J.shape[-2], J.shape[-1])
    if k == 1:
        div = J[..., 0, :1]
    elif k == 2:  # one fused add instead of diagonal + reduction
        div = J[..., 0, 0:1] + J[..., 1, 1:2]
    else:
        div = torch.diagonal(J[..., :k, :k], dim1=-2, dim2=-1).sum(dim=-1, keepdim=True)
    if affine:
        div = div + float(k)
    return div


def laplace(y, x, normalize=False, eps=0., return_grad=False):
    """div(grad y) (base/diff_ops.py:33-41).  normalize=True is not fused."""
    if normalize:
        raise _jet.UnsupportedPattern("laplace(normalize=True) is not on the INSR-PDE path")
    mlp, value, affine = _resolve(y, x, "laplace")
    _, J, lap = _jet.jet_of(mlp, value, x, nat.MODE_LAP)
    # the identity part of f(x)+x has zero Laplacian; a scalar net needs no reduction launch
    div = lap if lap.shape[-1] == 1 else lap.sum(dim=-1, keepdim=True)
    if return_grad:
        g = J.squeeze(-2) if J.shape[-2] == 1 else J.sum(dim=-2)
        if affine:
            g = g + 1.0
        return div, g
    return div


def jacobian(y: torch.FloatTensor, x: torch.FloatTensor):
    """(N, dim_y, dim_x) Jacobian and status (-1 if NaN) (base/diff_ops.py:61-82)."""
    mlp, value, affine = _resolve(y, x, "jacobian")
    _, J, _ = _jet.jet_of(mlp, value, x, nat.MODE_GRAD)
    if affine:
        J = J + torch.eye(J.shape[-1], device=J.device, dtype=J.dtype)
    status = -1 if bool(torch.isnan(J).any()) else 0
    return J, status


def jacobian_nosync(y, x):
    """jacobian() without the NaN status host sync (returns the device flag instead)."""
    J = jacobian_only(y, x)
    return J, torch.isnan(J).any()


def jacobian_only(y, x):
    """The (N, dim_y, dim_x) Jacobian of jacobian() alone: no status (no NaN scan launches)."""
    mlp, value, affine = _resolve(y, x, "jacobian")
    _, J, _ = _jet.jet_of(mlp, value, x, nat.MODE_GRAD)
    if affine:
        J = J + torch.eye(J.shape[-1], device=J.device, dtype=J.dtype)
    return J


def hessian(y, x):
    """base/diff_ops.py:6-30 -- defined by the reference but never called by any model."""
    raise _jet.UnsupportedPattern("hessian is not on the INSR-PDE training path (the reference never calls it)")
