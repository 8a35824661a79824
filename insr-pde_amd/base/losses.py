"""Fused squared-residual losses (HIP, one launch forward + one backward).

    fused_mse(a, b=None, c=None, d=None, alpha=1.0, beta=-1.0, gamma=1.0, delta=1.0)
        == torch.mean((alpha * (a + beta * b) + gamma * (c + delta * d)) ** 2)
        (missing tensors are zero; evaluated in that order, so the usual residuals
        round exactly like the reference's expressions)
    wall_mse(y, n)
        == torch.mean(y[:n, 0] ** 2) + torch.mean(y[n:2n, 1] ** 2)

They close the PDE residuals of the model phases (fluid/model.py:96-101,121-125,
147-151 and the wall terms :90-94,129-133; advection/model.py:78-91), which the
reference spells as 3-5 aten launches forward and as many backward.  Gradients flow
to every input that requires them.  GPU only (the product path has no CPU fallback).
"""
import torch

from . import _native as nat

_WORK = {}  # device index -> partials buffer of the (large-n) two-launch reduction


def _workspace(dev):
    """One partials buffer per device (loss launches are ordered on the caller's
    stream).  Created on the first eager call -- phase loops always run iteration 0
    eagerly before capturing -- so it lives outside any graph pool."""
    key = dev.index
    if key not in _WORK:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("fused loss workspace must be created before graph capture (run one eager call)")
        _WORK[key] = torch.empty(nat.lib().insr_sq_loss_work_floats(), device=dev, dtype=torch.float32)
    return _WORK[key]


def _prep(t):
    if t is None:
        return None
    if not t.is_cuda or t.dtype != torch.float32:
        raise nat.NativeUnavailable("fused losses run on fp32 GPU tensors only")
    return t if t.is_contiguous() else t.contiguous()


class _SqLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, kind, n, m, coef, scale, a, b, c, d):
        lib = nat.lib()
        dev = a.device
        work = _workspace(dev)
        out = torch.empty((), device=dev, dtype=torch.float32)
        rc = lib.insr_sq_loss_fwd(kind, nat.ptr(a), nat.ptr(b), nat.ptr(c), nat.ptr(d), n, m, *coef, scale,
                                  nat.ptr(out), nat.ptr(work), nat.stream_of(dev))
        nat.check(rc, "insr_sq_loss_fwd")
        ctx.save_for_backward(a, b, c, d)
        ctx.args = (kind, n, m, coef, scale)
        return out

    @staticmethod
    def backward(ctx, gout):
        a, b, c, d = ctx.saved_tensors
        kind, n, m, coef, scale = ctx.args
        need = ctx.needs_input_grad[5:9]
        if not any(need):
            return (None,) * 9
        grads = [torch.empty_like(t) if (t is not None and nd) else None for t, nd in zip((a, b, c, d), need)]
        g = gout.reshape(1) if gout.is_contiguous() else gout.contiguous().reshape(1)
        rc = nat.lib().insr_sq_loss_bwd(kind, nat.ptr(a), nat.ptr(b), nat.ptr(c), nat.ptr(d), n, m, *coef, scale,
                                        nat.ptr(g), *[nat.ptr(t) for t in grads], nat.stream_of(a.device))
        nat.check(rc, "insr_sq_loss_bwd")
        return (None, None, None, None, None, *grads)


def fused_mse(a, b=None, c=None, d=None, alpha=1.0, beta=-1.0, gamma=1.0, delta=1.0):
    """mean((alpha*(a + beta*b) + gamma*(c + delta*d))**2) over all elements; b, c, d are
    None or the shape of a (d needs c).  fused_mse(u, target) == F.mse_loss(u, target)."""
    for t in (b, c, d):
        if t is not None and t.shape != a.shape:
            raise ValueError(f"fused_mse: shape mismatch {tuple(t.shape)} vs {tuple(a.shape)}")
    if d is not None and c is None:
        raise ValueError("fused_mse: d needs c")
    a, b, c, d = _prep(a), _prep(b), _prep(c), _prep(d)
    n = a.numel()
    coef = (float(alpha), float(beta), float(gamma), float(delta))
    return _SqLoss.apply(nat.LOSS_COMBO, n, 1, coef, 1.0 / max(n, 1), a, b, c, d)


def wall_mse(y, n):
    """mean(y[:n, 0]**2) + mean(y[n:2n, 1]**2) for y of shape (2n, m), m >= 2 (the
    normal-component wall terms of both boundary bands in one launch)."""
    if y.dim() != 2 or y.shape[0] != 2 * n or y.shape[1] < 2:
        raise ValueError(f"wall_mse: expected (2*{n}, m>=2), got {tuple(y.shape)}")
    y = _prep(y)
    return _SqLoss.apply(nat.LOSS_BANDS, n, y.shape[1], (0.0, 0.0, 0.0, 0.0), 1.0 / max(n, 1), y, None, None, None)


_SVD_WORK = {}  # device index -> partials buffer of the SVD-energy reduction


class _SvdEnergy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, J, ratio_arap, ratio_volume):
        lib = nat.lib()
        dev = J.device
        if dev.index not in _SVD_WORK:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("SVD-energy workspace must be created before graph capture (run one eager call)")
            _SVD_WORK[dev.index] = torch.empty(lib.insr_svd_energy_work_floats(), device=dev, dtype=torch.float32)
        out = torch.empty((), device=dev, dtype=torch.float32)
        n, d = J.shape[0], J.shape[-1]
        rc = lib.insr_svd_energy_fwd(nat.ptr(J), n, d, float(ratio_arap), float(ratio_volume), nat.ptr(out),
                                     nat.ptr(_SVD_WORK[dev.index]), nat.stream_of(dev))
        nat.check(rc, "insr_svd_energy_fwd")
        ctx.save_for_backward(J)
        ctx.ratios = (float(ratio_arap), float(ratio_volume))
        return out

    @staticmethod
    def backward(ctx, gout):
        (J,) = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None
        gJ = torch.empty_like(J)
        g = gout.reshape(1) if gout.is_contiguous() else gout.contiguous().reshape(1)
        rc = nat.lib().insr_svd_energy_bwd(nat.ptr(J), J.shape[0], J.shape[-1], *ctx.ratios, nat.ptr(g), nat.ptr(gJ),
                                           nat.stream_of(J.device))
        nat.check(rc, "insr_svd_energy_bwd")
        return gJ, None, None


def svd_energy(J, ratio_arap=1.0, ratio_volume=0.0):
    """sum over points of ratio_arap * sum_i (s_i - 1)^2 + ratio_volume * (prod_i s_i - 1)^2,
    s = singular values of each J[n] (d x d, d = 2 or 3) -- the ARAP and volume terms of
    elasticity/model.py:143-163 in one launch (torch.svd's gradient U diag(dE/ds) V^T in
    one backward launch)."""
    if J.dim() != 3 or J.shape[-1] != J.shape[-2] or J.shape[-1] not in (2, 3):
        raise ValueError(f"svd_energy: expected (N, d, d) with d in (2, 3), got {tuple(J.shape)}")
    return _SvdEnergy.apply(_prep(J), ratio_arap, ratio_volume)
