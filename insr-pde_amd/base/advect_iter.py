"""One advection iteration in one launch (csrc/advect_iter.hip, insr_advect1d_iteration).

The reference's Advection1DModel._advect (advection/model.py:68-91) per iteration: draw the interior
collocation points and the Dirichlet band (base/sampling.py:14-30), the value and x-derivative of the frozen
field and of the trainable one (MLP.forward + gradient, base/diff_ops.py:44-58), the midpoint residual and
the band term, then loss.backward() (base/baseModel.py:73-78).  For the 1 -> 1 SIREN of width 64 the
advection configuration trains, all of that is ONE kernel here: each block draws its tiles' points, runs
both fields' jets, forms the residuals and their adjoint seeds and the reverse jet, and writes one
partial-gradient row; its last block finishes the two loss values.  advect1d_iteration returns (main, bc)
as loss tensors whose backward costs no launch -- it hands the rows to the network's held-back sums
(base/_jet.py PendingSums), which the Adam launch consumes (FusedAdam + DevicePlateau: sums + Adam +
plateau in one launch).  An iteration is two launches instead of five.

Same distributions as the generic path, bit-identical draws (the device Philox stream of
insr_sample_boxes with the same three boxes); exact fp32 products (tests/test_gpu_advect_iter.py: the
oracle at 1e-5 on the points the kernel drew, one and several Adam iterations, graph replay).
"""
import ctypes

import torch

from . import _jet
from . import _native as nat
from .networks import MLP

WIDTH = 64  # the kernel's hidden width (4 waves x 16 neuron rows)


def supported(field, field_prev):
    """Whether insr_advect1d_iteration serves this pair of fields: packed sine MLPs 1 -> 1 of width 64 and
    1..3 hidden layers (the staged weights fill the LDS) on one CUDA device, the same architecture."""
    for f in (field, field_prev):
        if type(f) is not MLP or f.in_features != 1 or f.out_features != 1 or f.kernel_width != WIDTH or \
                f.hidden_features != WIDTH or not (1 <= f.num_hidden_layers <= 3):
            return False
        if getattr(f, "nonlinearity", "sine") != "sine":
            return False
        p = f.flat_params()
        if not p.is_cuda or p.dtype != torch.float32:
            return False
    return field.num_hidden_layers == field_prev.num_hidden_layers and \
        field.flat_params().device == field_prev.flat_params().device


class _AdvectLosses(torch.autograd.Function):
    """(main, bc) of one fused iteration.  The gradient was computed by the forward launch itself (unit
    seeds: the training loop's loss backward, BaseModel._unit_seed); backward only hands its partial rows to
    the network's sums (held back for the Adam launch inside BaseModel._update_network)."""

    @staticmethod
    def forward(ctx, losses, job, *params):
        ctx.job = job
        ctx.set_materialize_grads(False)
        return losses[0], losses[1]

    @staticmethod
    def backward(ctx, g_main, g_bc):
        from .losses import _UNIT_SEEDS
        field, part, nb, stride, npts = ctx.job
        none = (None, None) + (None,) * len(field.plist())
        for gr in (g_main, g_bc):
            if gr is not None and not (gr.numel() == 1 and gr.data_ptr() in _UNIT_SEEDS):
                raise _jet.UnsupportedPattern(
                    "advect1d_iteration: its gradient is formed in the forward launch for unit loss seeds "
                    "(the training loop's backward); scale the learning rate instead of the losses")
        if g_main is None and g_bc is None:
            return none
        job = _RowsJob(field, part, nb, stride, npts, torch.cuda.current_stream(part.device))
        queue = _jet._BwdBatch.queue_for(job)
        if queue is not None:  # the loop's batched_backward scope: registered at its exit, on the caller's
            queue.append(job)  # thread (autograd runs this node on its device thread; defer_reductions is
        else:                  # the caller thread's state)
            job.run()
        return none


class _RowsJob:
    """The partial rows of one fused iteration, handed to the network's sums: held back for the Adam launch
    inside defer_reductions (insr_adam_step_partials: sums + Adam + plateau, one launch), else summed now."""
    __slots__ = ("field", "part", "nb", "stride", "npts", "cur")

    def __init__(self, field, part, nb, stride, npts, cur):
        self.field, self.part, self.nb, self.stride, self.npts, self.cur = field, part, nb, stride, npts, cur

    def run(self):
        field, cur = self.field, self.cur
        gflat, accumulate = field.grad_for_backward()
        field.grad_write_begin(cur)
        pr = _jet.PendingSums("rows", self.part, self.nb, self.stride, field, gflat, accumulate, cur,
                              (nat.MODE_GRAD, self.npts, WIDTH, (1, 1, field.num_hidden_layers)))
        if getattr(_jet._Defer, "depth", 0) > 0 and 0 < self.nb < 1024:
            field.set_pending_reduce(pr)
            _jet._Defer.nets.append(field)
        else:
            pr.launch()
        field.grad_write_end(cur)


STATS = {"iterations": 0}


def advect1d_iteration(field, field_prev, n, n_band_half, half, eps, dt, vel, main_total, bc_total,
                       points=None):
    """(main, bc) of one advection iteration (advection/model.py:68-91) in one launch: n interior points
    U[-half, half), n_band_half points in each band U[(-1 -+ eps) half), U[(1 -+ eps) half); main =
    sum(((u - u0) / dt + vel (u_x + u0_x) / 2)^2) / main_total, bc = sum(u_band^2) / bc_total.  points: a
    contiguous (n + 2 n_band_half,) fp32 tensor that receives the drawn points (None: not stored)."""
    from .sampling import _sampler
    lib = nat.lib()
    field.ensure_packed()
    field.ensure_wsplit()  # (the Adam launch keeps the trainable field's weight planes current)
    field_prev.ensure_packed()
    prm, prev = field.flat_params(), field_prev.flat_params()
    dev = prm.device
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    L = field.num_hidden_layers
    npts = int(n) + 2 * int(n_band_half)
    nb = lib.insr_advect1d_rows(npts)
    stride = lib.insr_jet_partial_stride(1, 1, L, WIDTH)
    part = torch.empty(nb * stride, device=dev, dtype=torch.float32)
    lpart = torch.empty(nb * nat.SEED_MAX, device=dev, dtype=torch.float32)
    losses = torch.empty(2, device=dev, dtype=torch.float32)
    if points is not None and (points.numel() != npts or not points.is_contiguous() or points.dtype != torch.float32):
        raise ValueError("advect1d_iteration: points must be a contiguous fp32 tensor of n + 2 n_band_half values")
    lo = (ctypes.c_float * 3)(-half, (-1 - eps) * half, (1 - eps) * half)
    hi = (ctypes.c_float * 3)(half, (-1 + eps) * half, (1 + eps) * half)
    state, seed = _sampler(dev)
    with _jet._timed("iter", nat.MODE_GRAD, npts, WIDTH, (1, 1, L)):  # (bench.py's roofline leg)
        rc = lib.insr_advect1d_iteration(nat.ptr(prm), nat.ptr(prev), L, WIDTH, int(n), int(n_band_half), lo, hi,
                                         float(dt), float(vel), float(main_total), float(bc_total), seed,
                                         nat.ptr(state), None if points is None else nat.ptr(points),
                                         nat.ptr(part), stride, nat.ptr(lpart), nat.ptr(losses), nat.stream_of(dev))
    nat.check(rc if rc < 0 else 0, "insr_advect1d_iteration")
    STATS["iterations"] += 1
    params = tuple(field.plist())
    if torch.is_grad_enabled() and any(p.requires_grad for p in params):
        return _AdvectLosses.apply(losses, (field, part, nb, stride, npts), *params)
    return losses[0], losses[1]
