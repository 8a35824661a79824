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

Reference-semantics fallback.  A graph the jet path does not serve -- y post-processed
before differentiation (2 * net(x), net(x)[..., :1] ** 2, a sum of two networks), the
divergence of a weighted or normalised gradient, Hessians of d_in = 3 inputs, widths or
shapes without a compiled kernel -- takes the reference's own route: torch.autograd.grad(...,
create_graph=True) through y's graph (_ref_* below, restating base/diff_ops.py:6-82).  The jet
nodes in that graph differentiate themselves with torch ops on the device (base/_jet.py
torch_jet), so the result is exact to any order and differentiable for loss.backward(); it
is slower, and counted in FALLBACKS.  CPU tensors still raise NativeUnavailable (the
networks' forwards are HIP-only).
"""
import warnings

import torch

from . import _jet
from . import _native as nat
from . import lower as _lower
from .lower import api as _lower_api


def _api(fn):
    return _lower_api(fn, operand_first=True)
from .networks import MLP

__all__ = ["hessian", "laplace", "divergence", "gradient", "jacobian"]

FALLBACKS = {}  # op name -> calls served by the reference-semantics route


def _fallback(opname, why):
    """Book-keeping of one reference-semantics call (a warning on the first one per op)."""
    if _lower.deferring():  # the loop's deferred jets (base/lower.py): the route reads values -- launch them
        _lower.flush()
    elif _jet._Fused.pending is not None:
        raise _jet.UnsupportedPattern(f"{opname} of an unfused graph inside a fused_forwards scope: its jets have "
                                      "no values until the scope exits")
    FALLBACKS[opname] = FALLBACKS.get(opname, 0) + 1
    if FALLBACKS[opname] == 1:
        warnings.warn(f"{opname}: {why}; using the reference-semantics autograd route (torch ops, slower)",
                      stacklevel=3)


# ---- the reference's definitions (base/diff_ops.py:6-82), used when the jet path does not apply ----
def _ref_grad(y, x, grad_outputs):
    """autograd.grad(y, [x], grad_outputs, create_graph=True)[0] (base/diff_ops.py:53-58)."""
    return torch.autograd.grad(y, [x], grad_outputs=grad_outputs, create_graph=True)[0]


def _ref_gradient(y, x, grad_outputs=None):
    return _ref_grad(y, x, torch.ones_like(y) if grad_outputs is None else grad_outputs)


def _ref_divergence(y, x):
    """sum_i d y_i / d x_i, one reverse pass per component (base/diff_ops.py:44-50)."""
    div = 0.
    for i in range(y.shape[-1]):
        yi = y[..., i]
        div = div + _ref_grad(yi, x, torch.ones_like(yi))[..., i:i + 1]
    return div


def _ref_jacobian_rows(y, x):
    """(..., dim_y, dim_x) from dim_y reverse passes (base/diff_ops.py:61-82, without the status)."""
    rows = []
    for i in range(y.shape[-1]):
        yi = y[..., i]
        rows.append(_ref_grad(yi, x, torch.ones_like(yi)))
    return torch.stack(rows, dim=-2)


def _ref_hessian(y, x):
    """(..., channels, dim, dim): row j of channel i = d(d y_i / d x_j)/dx (base/diff_ops.py:6-30)."""
    out = []
    for i in range(y.shape[-1]):
        yi = y[..., i]
        g = _ref_grad(yi, x, torch.ones_like(yi))
        out.append(torch.stack([_ref_grad(g[..., j], x, torch.ones_like(g[..., j])) for j in range(x.shape[-1])],
                               dim=-2))
    return torch.stack(out, dim=-3)


def _resolve(y, x, opname):
    """(mlp, holder, affine) of a recognised SIREN graph, ("gradient-of", ...) for the divergence of a
    jet gradient, or None (the reference-semantics route)."""
    m = _jet.match(y, x)
    if m is not None and _lower.affine_operand():  # f of a recorded q = f(x) + x (base/lower.py api)
        m = (m[0], m[1], True)
    if m is None:
        gsrc = getattr(y, "_insr_gradient_of", None)
        if gsrc is not None and gsrc[1] is x and opname == "divergence":
            return ("gradient-of",) + gsrc
        return None
    return m


def _jet_or_none(mlp, holder, x, mode):
    """The fused jet, or None when no kernel serves this network in `mode` (fallback)."""
    try:
        return _jet.jet_of(mlp, holder, x, mode)
    except _jet.UnsupportedPattern:
        return None


@_api
def gradient(y, x, grad_outputs=None):
    """d(sum_c grad_outputs_c * y_c)/dx, shape x.shape (base/diff_ops.py:53-58)."""
    r = _resolve(y, x, "gradient")
    res = _jet_or_none(r[0], r[1], x, nat.MODE_GRAD) if r is not None else None
    if res is None:
        _fallback("gradient", "y is not a fused SIREN output of x" if r is None else "no kernel for this network")
        return _ref_gradient(y, x, grad_outputs)
    mlp, value, affine = r
    _, J, _ = res  # (..., dout, din)
    if J.shape[-2] != 1 or affine or grad_outputs is not None:
        _lower.flush()  # a reduction / add over the jet's outputs: their values first (deferred jets)
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


@_api
def divergence(y, x):
    """sum_i dy_i/dx_i, shape (..., 1) (base/diff_ops.py:44-50)."""
    r = _resolve(y, x, "divergence")
    if r is not None and r[0] == "gradient-of":
        # divergence(gradient(f, x), x) with unit grad_outputs == laplace(f, x)
        _, mlp, _, value, affine, unit = r
        res = _jet_or_none(mlp, value, x, nat.MODE_LAP) if unit else None
        if res is None:
            _fallback("divergence", "the divergence of a weighted gradient" if not unit else "no Laplacian kernel")
            return _ref_divergence(y, x)
        lap = res[2]
        if lap.shape[-1] != 1:
            _lower.flush()
        return lap if lap.shape[-1] == 1 else lap.sum(dim=-1, keepdim=True)
    res = _jet_or_none(r[0], r[1], x, nat.MODE_GRAD) if r is not None else None
    if res is None:
        _fallback("divergence", "y is not a fused SIREN output of x" if r is None else "no kernel for this network")
        return _ref_divergence(y, x)
    mlp, value, affine = r
    _, J, _ = res
    k = min(J.shape[-2], J.shape[-1])
    if k == 1:
        div = J[..., 0, :1]
    elif k == 2:  # one fused add instead of diagonal + reduction (recorded while jets are deferred)
        div = _lower.add_views(J[..., 0, 0:1], J[..., 1, 1:2])
    else:
        _lower.flush()
        div = torch.diagonal(J[..., :k, :k], dim1=-2, dim2=-1).sum(dim=-1, keepdim=True)
    if affine:
        div = div + float(k)
    return div


@_api
def laplace(y, x, normalize=False, eps=0., return_grad=False):
    """div(grad y) (base/diff_ops.py:33-41).  normalize=True: div(g / (|g| + eps)), g = grad y,
    = tr(H) / (|g| + eps) - g.H g / (|g| (|g| + eps)^2) with H the Hessian of sum_c y_c
    (hessian(): d_in <= 2; otherwise the reference's route)."""
    if normalize:
        return _laplace_normalized(y, x, eps, return_grad)
    r = _resolve(y, x, "laplace")
    res = _jet_or_none(r[0], r[1], x, nat.MODE_LAP) if r is not None else None
    if res is None:
        _fallback("laplace", "y is not a fused SIREN output of x" if r is None else "no Laplacian kernel")
        g = gradient(y, x)
        div = _ref_divergence(g, x)
        return (div, g) if return_grad else div
    mlp, value, affine = r
    _, J, lap = res
    if lap.shape[-1] != 1 or (return_grad and (J.shape[-2] != 1 or affine)):
        _lower.flush()  # reductions over the jet's outputs: their values first (deferred jets)
    # the identity part of f(x)+x has zero Laplacian; a scalar net needs no reduction launch
    div = lap if lap.shape[-1] == 1 else lap.sum(dim=-1, keepdim=True)
    if return_grad:
        g = J.squeeze(-2) if J.shape[-2] == 1 else J.sum(dim=-2)
        if affine:
            g = g + 1.0
        return div, g
    return div


@_api
def jacobian(y: torch.FloatTensor, x: torch.FloatTensor):
    """(N, dim_y, dim_x) Jacobian and status (-1 if NaN) (base/diff_ops.py:61-82)."""
    J = jacobian_only(y, x)
    if _lower.deferring():
        # the reference's NaN status (a host read) as a Lazy 0-dim tensor computed only when a body reads it:
        # no launch, no sync, and the iteration stays capturable (elasticity/model.py:143 discards it)
        return J, _lower.lazy_call(_nan_status, (J,), (), torch.int64, J.device)
    _lower.flush()  # the status reads the values
    status = -1 if bool(torch.isnan(J).any()) else 0
    return J, status


def _nan_status(J):
    return torch.where(torch.isnan(J).any(), -1, 0)


@_api
def jacobian_nosync(y, x):
    """jacobian() without the NaN status host sync (returns the device flag instead)."""
    J = jacobian_only(y, x)
    _lower.flush()
    return J, torch.isnan(J).any()


@_api
def jacobian_only(y, x):
    """The (N, dim_y, dim_x) Jacobian of jacobian() alone: no status (no NaN scan launches)."""
    r = _resolve(y, x, "jacobian")
    res = _jet_or_none(r[0], r[1], x, nat.MODE_GRAD) if r is not None else None
    if res is None:
        _fallback("jacobian", "y is not a fused SIREN output of x" if r is None else "no kernel for this network")
        return _ref_jacobian_rows(y, x)
    mlp, value, affine = r
    _, J, _ = res
    if affine:  # J + I: recorded while jets are deferred (an energy lowering reads J itself, base/lower.py)
        return _lower.eye_add(J, (mlp, res[0], x))
    return J


def _laplace_normalized(y, x, eps, return_grad):
    with _lower.immediate():  # reads its jets' values in this call
        return _laplace_normalized_now(y, x, eps, return_grad)


def _laplace_normalized_now(y, x, eps, return_grad):
    g = gradient(y, x)
    try:
        H = _hessian_core(y, x, "laplace(normalize=True)").sum(dim=-3)  # Hessian of sum_c y_c
    except _jet.UnsupportedPattern:
        if _jet._Fused.pending is not None:
            raise
        # base/diff_ops.py:33-41 as written: div(g / (|g| + eps))
        _fallback("laplace", "normalize=True beyond the polarised Hessian jets")
        gn = g / (g.norm(dim=-1, keepdim=True) + eps)
        div = _ref_divergence(gn, x)
        return (div, gn) if return_grad else div
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
    """(..., d_out, d_in, d_in) Hessian of each output channel (no status); UnsupportedPattern where the
    polarised jets do not apply (the callers fall back)."""
    r = _resolve(y, x, opname)
    if r is None or r[0] == "gradient-of":
        raise _jet.UnsupportedPattern(f"{opname}: y is not a fused SIREN output of x")
    mlp, value, affine = r
    if _jet._Fused.pending is not None:
        raise _jet.UnsupportedPattern(f"{opname} inside a fused_forwards scope (its jets' values are read at once)")
    d = mlp.in_features
    if d > 2:
        raise _jet.UnsupportedPattern(f"{opname}: Hessians of d_in = {d} inputs (d_in <= 2: the augmented "
                                      "Laplacian jet of f(x + s v) has d_in + 1 <= 3 inputs)")
    _, _, L0 = _jet.jet_of(mlp, value, x, nat.MODE_LAP)  # (..., c): tr(H)
    if d == 1:
        return L0[..., None, None]
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


@_api
def hessian(y, x):
    """base/diff_ops.py:6-30: y (meta, obs, channels), x (meta, obs, dim) -> the Hessian
    (meta, obs, channels, dim, dim) and status (-1 if NaN); 2-D y, x give (N, channels, dim, dim).
    The polarised jets serve d_in <= 2; other inputs (and unfused graphs) take the reference's
    route.  The identity part of f(x) + x has zero Hessian."""
    try:
        with _lower.immediate():  # the polarised jets' values are read in this call
            H = _hessian_core(y, x, "hessian")
    except _jet.UnsupportedPattern:
        if _jet._Fused.pending is not None:
            raise
        _fallback("hessian", "beyond the polarised Hessian jets (d_in <= 2 SIREN outputs)")
        H = _ref_hessian(y, x)
    status = -1 if bool(torch.isnan(H).any()) else 0
    return H, status
