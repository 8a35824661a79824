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
  hessian    :6-30   (.., dy, dx, dx)      d_in = 1: the Laplacian stream; d_in = 2: Laplacian
                                           jets of the field and of f(x + s v) for three
                                           directions v (polarisation), d_in <= 2

All results stay differentiable w.r.t. the network parameters (loss.backward()
runs the HIP reverse jet).  `status` is returned, never raised (-1 on NaN).
"""
import torch

from . import _jet
from . import _native as nat
from .networks import MLP

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
    """div(grad y) (base/diff_ops.py:33-41).  normalize=True: div(g / (|g| + eps)), g = grad y,
    = tr(H) / (|g| + eps) - g.H g / (|g| (|g| + eps)^2) with H the Hessian of sum_c y_c
    (hessian(): d_in <= 2)."""
    if normalize:
        return _laplace_normalized(y, x, eps, return_grad)
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


def _laplace_normalized(y, x, eps, return_grad):
    g = gradient(y, x)
    H = _hessian_core(y, x, "laplace(normalize=True)").sum(dim=-3)  # Hessian of sum_c y_c
    gn = g.norm(dim=-1, keepdim=True)
    gHg = torch.einsum("...i,...ij,...j->...", g, H, g).unsqueeze(-1)
    tr = laplace(y, x)  # tr(H) straight from the Laplacian stream (no polarisation error)
    div = tr / (gn + eps) - gHg / (gn * (gn + eps) ** 2)
    if return_grad:
        return div, g / (gn + eps)
    return div


def _aug_net(mlp, v, device):
    """The SIREN f(x + s v) of one extra input s (first-layer column W0 v appended), kept per
    (network, direction); its weights are rewritten for each call (_AugLaplacian).  Built under
    a forked RNG: the reference's seeded streams are not disturbed."""
    nets = mlp.__dict__.setdefault("_insr_aug", {})  # not a submodule: mlp.parameters() unchanged
    if v not in nets:
        with torch.random.fork_rng(devices=[]):
            nets[v] = MLP(mlp.in_features + 1, mlp.out_features, mlp.num_hidden_layers, mlp.hidden_features,
                          nonlinearity="sine", precision=mlp.precision).to(device)
    return nets[v]


class _AugLaplacian(torch.autograd.Function):
    """Per-channel Laplacian of g(x, s) = f(x + s v) over (x, s) at s = 0, i.e. tr(H) + v.H v:
    ONE Laplacian jet of the augmented network (first layer [W0 | W0 v]).  Backward: that
    network's reverse jet, its first-layer gradient folded back (dW0 = G[:, :d] + G[:, d] v^T)."""

    @staticmethod
    def forward(ctx, x2, v, mlp, *params):
        aug = _aug_net(mlp, v, x2.device)
        ps = list(mlp.parameters())
        vt = torch.tensor(v, dtype=ps[0].dtype, device=ps[0].device)
        with torch.no_grad():
            qs = list(aug.parameters())
            qs[0].copy_(torch.cat([ps[0], ps[0] @ vt[:, None]], dim=1))
            for q, p in zip(qs[1:], ps[1:]):
                q.copy_(p)
        with torch.enable_grad():
            xa = torch.cat([x2.detach(), torch.zeros_like(x2[:, :1])], dim=1).requires_grad_(True)
            _, _, lap = _jet.run_jet(aug, xa, nat.MODE_LAP)
        # the reverse jet reads the network's weights: keep this call's (a later call rewrites them)
        ctx.lap, ctx.aug, ctx.vt, ctx.snap = lap, aug, vt, aug.flat_params().detach().clone()
        return lap.detach()

    @staticmethod
    def backward(ctx, glap):
        aug = ctx.aug
        with torch.no_grad():
            aug.flat_params().copy_(ctx.snap)
        aug.zero_grad(set_to_none=True)
        with _jet.immediate_backward():  # aug's .grad is read right below
            torch.autograd.backward(ctx.lap, glap.contiguous(), retain_graph=True)
        gq = [q.grad if q.grad is not None else torch.zeros_like(q) for q in aug.parameters()]
        d = gq[0].shape[1] - 1
        g0 = gq[0][:, :d] + gq[0][:, d:] * ctx.vt[None, :]
        return (None, None, None, g0, *[g.clone() for g in gq[1:]])


def _hessian_core(y, x, opname):
    """(..., d_out, d_in, d_in) Hessian of each output channel (no status)."""
    mlp, value, affine = _resolve(y, x, opname)
    if _jet._Fused.pending is not None:
        raise _jet.UnsupportedPattern(f"{opname} inside a fused_forwards scope (its jets' values are read at once)")
    d = mlp.in_features
    _, _, L0 = _jet.jet_of(mlp, value, x, nat.MODE_LAP)  # (..., c): tr(H)
    if d == 1:
        return L0[..., None, None]
    if d != 2:
        raise _jet.UnsupportedPattern(f"{opname}: Hessians of d_in = {d} inputs (d_in <= 2: the augmented "
                                      "Laplacian jet of f(x + s v) has d_in + 1 <= 3 inputs)")
    x2, lead = _jet._flatten_x(x, d)
    params = tuple(mlp.parameters())
    L0f = L0.reshape(-1, L0.shape[-1])
    # v.H v = (Lap_aug(a v) - tr H) / a^2 with a = 8 (exact in fp32): the directional term
    # outweighs tr H 64-fold, so the difference keeps its digits
    a = 8.0
    q = [(_AugLaplacian.apply(x2, (a * v0, a * v1), mlp, *params) - L0f) * (1.0 / (a * a))
         for v0, v1 in ((1.0, 0.0), (0.0, 1.0), (1.0, 1.0))]
    h11, h22 = q[0], q[1]
    h12 = 0.5 * (q[2] - h11 - h22)
    H = torch.stack([torch.stack([h11, h12], -1), torch.stack([h12, h22], -1)], -2)  # (n, c, 2, 2)
    return H.reshape(*L0.shape, 2, 2)


def hessian(y, x):
    """base/diff_ops.py:6-30: y (meta, obs, channels), x (meta, obs, dim) -> the Hessian
    (meta, obs, channels, dim, dim) and status (-1 if NaN); 2-D y, x give (N, channels, dim, dim).
    d_in <= 2 (the reference never calls it on the INSR-PDE path).  The identity part of
    f(x) + x has zero Hessian."""
    H = _hessian_core(y, x, "hessian")
    status = -1 if bool(torch.isnan(H).any()) else 0
    return H, status
