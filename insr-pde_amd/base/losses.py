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
import ctypes
import threading

import torch

from . import _native as nat

_WORK = {}  # (device index, stream handle) -> partials buffer of the large-n in-launch reduction


def _stream_key(dev, stream=None):
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    return (dev.index, s.cuda_stream)


def prepare_workspaces(stream):
    """Create the reduction workspaces of `stream` (before a graph capture on it)."""
    dev = stream.device
    for table, floats, zero in ((_WORK, nat.lib().insr_sq_loss_work_floats(), True),
                                (_SVD_WORK, nat.lib().insr_svd_energy_work_floats(), False),
                                (_EL_WORK, nat.lib().insr_elastic_work_floats(), True)):
        key = _stream_key(dev, stream)
        if key not in table:
            table[key] = (torch.zeros if zero else torch.empty)(floats, device=dev, dtype=torch.float32)


def _workspace(dev):
    """One partials buffer per (device, stream): launches on one stream are ordered, launches
    on two streams (a side-stream band loss next to the interior loss, two models on two
    streams) never share one.  Created on the first eager call on that stream, or by
    prepare_workspaces() before a capture -- never inside a capture (a graph-pool buffer)."""
    key = _stream_key(dev)
    if key not in _WORK:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("fused loss workspace must be created before graph capture "
                               "(base.losses.prepare_workspaces(stream) or one eager call on the stream)")
        # zeros: the tail word is the in-launch combine's ticket (every launch leaves it 0)
        _WORK[key] = torch.zeros(nat.lib().insr_sq_loss_work_floats(), device=dev, dtype=torch.float32)
    return _WORK[key]


def _prep(t):
    if t is None:
        return None
    if not t.is_cuda or t.dtype != torch.float32:
        raise nat.NativeUnavailable("fused losses run on fp32 GPU tensors only")
    return t if t.is_contiguous() else t.contiguous()


def _at(t, off):
    """Device pointer to element `off` of t (None stays None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr() + 4 * int(off))


def _grad_like(t, n_used):
    """Gradient buffer of an input of which the loss reads n_used elements: elements the
    loss does not read (the other rows of a merged jet launch) get zero gradient."""
    return torch.empty_like(t) if t.numel() == n_used else torch.zeros_like(t)


# Unit seeds: 1-element tensors holding 1.0 that the training loop passes as the gradient of
# every loss (BaseModel._unit_seed).  A loss whose backward receives one of them returns the
# gradient its forward launch already wrote -- no backward launch.
# data_ptr -> the seed tensor itself: the registry holds a reference, so a registered address
# can never be recycled by the caching allocator for another (non-unit) gradient tensor
_UNIT_SEEDS = {}


def register_unit_seed(t):
    """Declare `t` (a tensor of ones the caller never modifies) a unit seed for loss backwards."""
    if t.numel() == 1:
        _UNIT_SEEDS[t.data_ptr()] = t
    return t


def _prep_strided(t):
    """(tensor, element stride) of a b / c / d input: contiguous tensors and 1-D (or (n, 1))
    strided views are read in place (e.g. the diagonal of a Jacobian, J[:, i, i])."""
    if t is None:
        return None, 1
    if not t.is_cuda or t.dtype != torch.float32:
        raise nat.NativeUnavailable("fused losses run on fp32 GPU tensors only")
    if t.is_contiguous():
        return t, 1
    if t.dim() == 1 or (t.dim() == 2 and t.shape[1] == 1):
        return t, t.stride(0)
    return t.contiguous(), 1


class LossSpec:
    """One squared-residual loss, not yet launched (see sq_losses)."""

    def __init__(self, kind, n, m, coef, scale, a, b, c, d, a_off, strides=(1, 1, 1)):
        self.meta = (kind, int(n), int(m), tuple(float(v) for v in coef), float(scale), int(a_off),
                     tuple(int(v) for v in strides))
        self.tensors = (a, b, c, d)

    def a_range(self):
        """Elements of `a` the loss reads: [a_off, a_off + terms) (BANDS: 2n rows of m; n rows when the
        second band is a tensor of its own, b)."""
        kind, n, m, _, _, a_off, _ = self.meta
        if kind == nat.LOSS_COMBO:
            return a_off, a_off + n
        return a_off, a_off + (1 if self.tensors[1] is not None else 2) * n * m


def _mse_spec(a, b=None, c=None, d=None, alpha=1.0, beta=-1.0, gamma=1.0, delta=1.0, count=None, a_row0=0,
              reduction="mean", total=None, weight=1.0):
    if count is None:
        for t in (b, c, d):
            if t is not None and t.shape != a.shape:
                raise ValueError(f"fused_mse: shape mismatch {tuple(t.shape)} vs {tuple(a.shape)}")
        count, a_off = a.numel(), 0
    else:
        row = a.numel() // max(a.shape[0], 1) if a.dim() > 0 else 1
        a_off = int(a_row0) * row
        if a_off + count > a.numel() or any(t is not None and t.numel() < count for t in (b, c, d)):
            raise ValueError(f"fused_mse: count {count} (a from element {a_off}) exceeds an input")
    if d is not None and c is None:
        raise ValueError("fused_mse: d needs c")
    if reduction not in ("mean", "sum"):
        raise ValueError(reduction)
    # total: the denominator of the mean (default: the terms summed here) -- under data parallelism the
    # GLOBAL term count, so the ranks' losses and gradients sum to the global mean (no 1/world pass)
    scale = 1.0 / max(count if total is None else total, 1) if reduction == "mean" else 1.0
    if weight != 1.0:  # weight * the loss (base/lower.py: a reference loss scaled by a constant)
        scale = float(weight) * scale
    (b, sb), (c, sc), (d, sd) = _prep_strided(b), _prep_strided(c), _prep_strided(d)
    return LossSpec(nat.LOSS_COMBO, count, 1, (alpha, beta, gamma, delta), scale, _prep(a), b, c, d, a_off,
                    (sb, sc, sd))


def _wall_spec(y, n, row0=0, total=None):
    if y.dim() != 2 or y.shape[0] < row0 + 2 * n or y.shape[1] < 2 or (row0 == 0 and y.shape[0] != 2 * n):
        raise ValueError(f"wall_mse: expected ({row0} + 2*{n} rows, m>=2), got {tuple(y.shape)}")
    return LossSpec(nat.LOSS_BANDS, n, y.shape[1], (0.0, 0.0, 0.0, 0.0), 1.0 / max(n if total is None else total, 1),
                    _prep(y), None, None, None, int(row0) * y.shape[1])


def wall_term2(ya, yb, weight=1.0):
    """weight * (mean(ya[:, 0] ** 2) + mean(yb[:, 1] ** 2)) for two (n, m) tensors of their own (the
    reference's separate band calls, fluid/model.py:96-98,119-122), unlaunched: an argument of sq_losses()."""
    if ya.dim() != 2 or ya.shape != yb.shape or ya.shape[1] < 2:
        raise ValueError(f"wall_term2: expected two (n, m >= 2) tensors, got {tuple(ya.shape)}, {tuple(yb.shape)}")
    if not yb.is_contiguous():
        raise ValueError("wall_term2: the second band must be contiguous")
    n = ya.shape[0]
    return LossSpec(nat.LOSS_BANDS, n, ya.shape[1], (0.0, 0.0, 0.0, 0.0), float(weight) / max(n, 1), _prep(ya),
                    _prep(yb), None, None, 0)


def mse_term(*args, **kwargs):
    """The loss of fused_mse(*args, **kwargs), unlaunched: an argument of sq_losses()."""
    return _mse_spec(*args, **kwargs)


def wall_term(y, n, row0=0, total=None):
    """The loss of wall_mse(y, n, row0, total), unlaunched: an argument of sq_losses()."""
    return _wall_spec(y, n, row0, total)


def _shared_a(specs):
    """For each loss, the index of the earlier loss whose `a` (the same tensor) it shares a
    gradient buffer with, or None.  Sharing needs disjoint ranges that together cover the whole
    tensor (e.g. a merged jet's interior rows and its band rows)."""
    owner = [None] * len(specs)
    groups = {}
    for i, sp in enumerate(specs):
        groups.setdefault(id(sp.tensors[0]), []).append(i)
    for idx in groups.values():
        if len(idx) < 2:
            continue
        rs = sorted(specs[i].a_range() for i in idx)
        numel = specs[idx[0]].tensors[0].numel()
        if rs[0][0] != 0 or rs[-1][1] != numel or any(rs[k][1] != rs[k + 1][0] for k in range(len(rs) - 1)):
            continue
        for i in idx[1:]:
            owner[i] = idx[0]
    return owner


# ---- adjoint seeds inside the reverse jet (round 5) ------------------------------------------------
# A loss group formed inside lazy_losses() -- opened by the training loop around a phase body that opts
# in (BaseModel._insr_lazy_losses: the body returns its sq_losses outputs and nothing else consumes the
# jet outputs they read) -- holds its launch back.  Its unit-seeded backward hands out the gradient
# buffers unfilled; the reverse jet that receives them (base/_jet.py _launch_bwd) evaluates the loss
# terms itself (insr_siren_jet_bwd_seeded: bit for bit the gradient the group launch writes) and the
# sums launch after it finishes the loss values (InsrLossFin) -- one launch fewer per iteration.  Any
# other consumer launches the group first (LazyGroup.materialize), and settle_lazy() (after the
# backward, BaseModel._update_network) launches every group no reverse jet took.
class _LazyState(threading.local):
    depth = 0
    groups = None  # the lazy groups formed on this thread since the last settle_lazy()


_Lazy = _LazyState()
_LAZY = {}  # data_ptr of a handed-out gradient buffer -> (LazyGroup, index of the loss that owns it)
_LAZY_LOCK = threading.Lock()  # (reverse jets may run on autograd's device thread)


class lazy_losses:
    """`with lazy_losses(on): body()` -- loss groups formed inside defer their launch (see above)."""

    def __init__(self, on=True):
        self.on = bool(on)

    def __enter__(self):
        if self.on:
            _Lazy.depth += 1
        return self

    def __exit__(self, *exc):
        if self.on:
            _Lazy.depth -= 1
        return False


class LazyGroup:
    """A loss group whose launch is held back: state 'pending' (formed), 'handed' (its unit-seeded
    backward gave out the unfilled gradient buffers), 'seeded' (a reverse jet took them), 'launched'."""
    __slots__ = ("arr", "k", "work", "dev", "outs", "metas", "owner", "real_a", "tensors", "grads", "state",
                 "bufs", "over", "__weakref__")

    def materialize(self, stream=None):
        """Launch the group now (its losses and gradients, as the eager path) -- before anything reads them."""
        if self.state in ("pending", "handed"):
            st = nat.stream_of(self.dev) if stream is None else ctypes.c_void_p(stream.cuda_stream)
            nat.check(nat.lib().insr_sq_loss_group(self.arr, self.k, nat.ptr(self.work), st), "insr_sq_loss_group")
            self.state = "launched"
        self._forget()

    def _forget(self):
        with _LAZY_LOCK:
            for p in self.bufs:
                _LAZY.pop(p, None)
        self.bufs = []

    def seeds_for(self, streams):
        """The InsrSeed terms of this group for a reverse jet whose adjoint streams are
        streams = {stream id: (gradient tensor or None, the jet's output data_ptr, its numel)}: every loss of
        the group must seed one of them from its own output buffer; None when that does not hold."""
        if self.state != "handed":
            return None
        terms = []
        covered = set()
        for sid, (g, out_ptr, out_numel) in streams.items():
            if g is None or g.data_ptr() not in self.bufs:
                continue
            o = self.bufs.index(g.data_ptr())
            owner_idx = [i for i in range(self.k) if (self.owner[i] if self.owner[i] is not None else i) == o]
            for i in owner_idx:
                kind, n, m, coef, scale, a_off, (sb, sc, sd) = self.metas[i]
                a = self.real_a[i]
                if a.data_ptr() != out_ptr or a.numel() != out_numel:
                    return None
                b, c, d = self.tensors[4 * i + 1:4 * i + 4]
                terms.append(nat.Seed(kind, m, sid, i, n, a_off, a.data_ptr(), nat.ptr(b), nat.ptr(c), nat.ptr(d),
                                      sb, sc, sd, *coef, scale))
                covered.add(i)
        if covered != set(range(self.k)) or len(terms) > nat.SEED_MAX:
            return None
        return terms

    def fin(self, part, rows):
        """The InsrLossFin that finishes this group's loss values from a seeded backward's rows."""
        f = nat.LossFin()
        f.part, f.rows, f.nloss = part.data_ptr(), rows, self.k
        for i in range(self.k):
            f.scale[i] = self.metas[i][4]
            f.out[i] = self.over[i] if self.over[i] is not None else self.outs[i].data_ptr()
        return f

    def redirect(self, i, address):
        """Finish loss i's value at `address` (a device float) instead of its own output tensor -- e.g. the
        data-parallel arena's loss slot (BaseModel._dp_pack); the output tensor is then not written."""
        self.over[i] = address


def lazy_output(t):
    """(LazyGroup, index) when t is a loss output of a lazy group formed on this thread, else None."""
    for g in _Lazy.groups or ():
        for i, o in enumerate(g.outs):
            if o is t:
                return g, i
    return None


def lazy_group_of(t):
    """The LazyGroup whose handed-out gradient buffer t is (None: an ordinary tensor)."""
    if t is None or not _LAZY:
        return None
    with _LAZY_LOCK:
        ent = _LAZY.get(t.data_ptr())
    return None if ent is None else ent[0]


def materialize_for(*ts):
    """Launch the lazy groups any of ts came from (a consumer that reads them as data)."""
    for t in ts:
        g = lazy_group_of(t)
        if g is not None:
            g.materialize()


def settle_lazy():
    """After the backward: launch every lazy group of this thread that no reverse jet took (its losses
    are read later); a group whose buffers were handed out but reached no reverse jet was read as data
    by something else -- that is an error of the phase body's opt-in, raised."""
    gs, _Lazy.groups = (_Lazy.groups or []), None
    bad = False
    for g in gs:
        if g.state == "handed":
            bad = True
        if g.state in ("pending", "handed"):
            g.materialize()
        g._forget()
    if bad:
        raise RuntimeError("a lazy loss group's gradients were consumed outside the reverse jets (the phase "
                           "body reads a jet output its sq_losses reads): do not open lazy_losses around it")


_VIEW_NODES = frozenset(("ViewBackward0", "UnsafeViewBackward0", "ReshapeAliasBackward0", "AliasBackward0",
                         "SqueezeBackward0", "SqueezeBackward1", "SqueezeBackward2", "SqueezeBackward3",
                         "UnsqueezeBackward0"))


def _lazy_ok(metas, owner, real_a, need):
    """Whether a group may hold its launch back: every loss's trained operand is its `a` (b, c, d carry no
    gradient), every `a` requires grad, and is a jet output (or a view of one) -- the reverse jet that
    receives its gradient evaluates the terms."""
    for i in range(len(metas)):
        o = owner[i] if owner[i] is not None else i
        if not need[4 * o] or any(need[4 * i + q] for q in (1, 2, 3)):
            return False
        a = real_a[i]
        fn = a.grad_fn
        # a view of a jet output (e.g. the scalar net's gradient J.squeeze(-2), diff_ops.gradient): its
        # backward is a view of the incoming gradient -- the reverse jet receives the handed-out buffer itself
        while fn is not None and type(fn).__name__ in _VIEW_NODES:
            fn = fn.next_functions[0][0] if fn.next_functions else None
        if fn is None or "_SirenJet" not in type(fn).__name__:
            return False
    return True


class _SqLossGroup(torch.autograd.Function):
    """Up to LOSS_GROUP_MAX losses in ONE launch forward (insr_sq_loss_group), each with the
    gradient for a unit seed written by the same launch; inputs: 4 tensor slots per loss (a
    loss that shares its `a` with an earlier one passes None there: one gradient buffer)."""

    @staticmethod
    def forward(ctx, metas, owner, real_a, *tensors):
        lib = nat.lib()
        k = len(metas)
        dev = next(t for t in tensors if t is not None).device
        need = ctx.needs_input_grad[3:]
        outs = [torch.empty((), device=dev, dtype=torch.float32) for _ in range(k)]
        arr = (nat.Loss * k)()
        grads = []
        multi = False
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        for i, (kind, n, m, coef, scale, a_off, (sb, sc, sd)) in enumerate(metas):
            slot = list(tensors[4 * i:4 * i + 4])
            nd = list(need[4 * i:4 * i + 4])
            if owner[i] is not None:  # a shared with loss owner[i]: write into its buffer
                slot[0], nd[0] = real_a[i], need[4 * owner[i]]
            g = [torch.empty_like(t) if (t is not None and q) else None for t, q in zip(slot, nd)]
            if owner[i] is not None:
                g[0] = grads[4 * owner[i]]
            grads.extend(g)
            terms = n if kind == nat.LOSS_COMBO else 2 * n
            a_rows = terms if (kind == nat.LOSS_COMBO or slot[1] is None) else n  # BANDS with b: a holds n rows
            a_lo, a_hi = (a_off, a_off + a_rows * (1 if kind == nat.LOSS_COMBO else m))
            shared = owner[i] is not None or any(o == i for o in owner)
            lo, hi = (a_lo, a_hi) if shared else (0, 0 if g[0] is None else g[0].numel())
            lens = [0 if t is None else t.numel() for t in g[1:]]
            span = max([hi - lo] + lens + [terms])
            multi = multi or span > 1024
            a, b, c, d = slot
            arr[i] = nat.Loss(kind, m, n, p(a), p(b), p(c), p(d), sb, sc, sd, *coef, scale, outs[i].data_ptr(),
                              p(g[0]), lo, hi, a_off, p(g[1]), p(g[2]), p(g[3]), *lens)
        work = _workspace(dev) if multi else None
        ctx.lazy = None
        # (a BANDS term with its second band in a tensor of its own is never seeded in-kernel)
        bands2 = any(mt[0] == nat.LOSS_BANDS and tensors[4 * i + 1] is not None for i, mt in enumerate(metas))
        if _Lazy.depth > 0 and not bands2 and _lazy_ok(metas, owner, real_a, need):
            lz = LazyGroup()
            lz.arr, lz.k, lz.work, lz.dev, lz.outs, lz.metas, lz.owner = arr, k, work, dev, outs, metas, owner
            lz.real_a, lz.tensors, lz.grads, lz.state, lz.bufs = list(real_a), list(tensors), grads, "pending", []
            lz.over = [None] * k
            ctx.lazy = lz
            if _Lazy.groups is None:
                _Lazy.groups = []
            _Lazy.groups.append(lz)
        else:
            nat.check(lib.insr_sq_loss_group(arr, k, nat.ptr(work), nat.stream_of(dev)), "insr_sq_loss_group")
        ctx.save_for_backward(*[real_a[i] if owner[i] is not None and j == 0 else t
                                for i in range(k) for j, t in enumerate(tensors[4 * i:4 * i + 4])])
        ctx.metas, ctx.owner = metas, owner
        ctx.pre = [None if (owner[i // 4] is not None and i % 4 == 0) else g for i, g in enumerate(grads)]
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        tensors = ctx.saved_tensors
        need = ctx.needs_input_grad[3:]
        owner = ctx.owner
        k = len(ctx.metas)
        res = [None] * len(tensors)
        unit = [g is not None and g.numel() == 1 and g.data_ptr() in _UNIT_SEEDS for g in gouts]
        lz = ctx.lazy
        if lz is not None:
            if all(unit) and lz.state == "pending" and not getattr(ctx, "pre_used", False):
                # the first unit-seeded backward: hand out the unfilled a-gradient buffers (a reverse jet
                # evaluates them, or materialize() fills them before anything else reads them)
                lz.state = "handed"
                with _LAZY_LOCK:
                    for o in range(k):
                        if owner[o] is None and ctx.pre[4 * o] is not None:
                            lz.bufs.append(ctx.pre[4 * o].data_ptr())
                            _LAZY[ctx.pre[4 * o].data_ptr()] = (lz, o)
                # (bufs in owner order: seeds_for maps a buffer back to the losses that share it)
                lz.bufs = [ctx.pre[4 * o].data_ptr() if (owner[o] is None and ctx.pre[4 * o] is not None) else -1
                           for o in range(k)]
            else:
                lz.materialize()
        # the forward's precomputed gradients are handed out once; a repeated backward
        # (retain_graph=True) gets copies, so nothing downstream can alias the kept buffers
        pre = ctx.pre if not getattr(ctx, "pre_used", False) else [None if g is None else g.clone() for g in ctx.pre]
        ctx.pre_used = True
        for o in range(k):
            if owner[o] is not None:
                continue
            members = [o] + [j for j in range(k) if owner[j] == o]
            if all(unit[j] for j in members):  # the forward wrote exactly these gradients
                res[4 * o:4 * o + 4] = pre[4 * o:4 * o + 4]
                for j in members[1:]:
                    res[4 * j + 1:4 * j + 4] = pre[4 * j + 1:4 * j + 4]
                continue
            for j in members:  # general seeds: one backward launch per loss, a-gradients summed
                if gouts[j] is None:
                    continue
                kind, n, m, coef, scale, a_off, strides = ctx.metas[j]
                a, b, c, d = tensors[4 * j:4 * j + 4]
                nd = [need[4 * o]] + list(need[4 * j + 1:4 * j + 4])
                used = n if kind == nat.LOSS_COMBO else 2 * n * m
                g = [_grad_like(t, used) if (t is not None and q) else None for t, q in zip((a, b, c, d), nd)]
                b, c, d = [None if t is None else (t if s_ == 1 else t.contiguous()) for t, s_ in zip((b, c, d), strides)]
                go = gouts[j].reshape(1) if gouts[j].is_contiguous() else gouts[j].contiguous().reshape(1)
                rc = nat.lib().insr_sq_loss_bwd(kind, _at(a, a_off), _at(b, 0), _at(c, 0), _at(d, 0), n, m, *coef,
                                                scale, nat.ptr(go), _at(g[0], a_off), _at(g[1], 0), _at(g[2], 0),
                                                _at(g[3], 0), nat.stream_of(a.device))
                nat.check(rc, "insr_sq_loss_bwd")
                if g[0] is not None:
                    res[4 * o] = g[0] if res[4 * o] is None else res[4 * o] + g[0]
                res[4 * j + 1:4 * j + 4] = g[1:]
        return (None, None, None, *res)


def sq_losses(*specs):
    """Launch every loss term of `specs` (mse_term / wall_term) in ONE kernel; returns their
    scalar losses in order (each differentiable; a unit-seeded backward costs no launch)."""
    if not 1 <= len(specs) <= nat.LOSS_GROUP_MAX:
        raise ValueError(f"sq_losses: 1..{nat.LOSS_GROUP_MAX} losses")
    metas = tuple(sp.meta for sp in specs)
    owner = _shared_a(specs)
    real_a = [sp.tensors[0] for sp in specs]
    tensors = [None if (owner[i] is not None and j == 0) else t
               for i, sp in enumerate(specs) for j, t in enumerate(sp.tensors)]
    return _SqLossGroup.apply(metas, owner, real_a, *tensors)


def fused_mse(a, b=None, c=None, d=None, alpha=1.0, beta=-1.0, gamma=1.0, delta=1.0, count=None, a_row0=0,
              reduction="mean", total=None):
    """mean((alpha*(a + beta*b) + gamma*(c + delta*d))**2) over all elements; b, c, d are
    None or the shape of a (d needs c).  fused_mse(u, target) == F.mse_loss(u, target).

    Merged jet launches (interior + boundary points of one network in one launch):
    count = number of terms; every tensor is read from its first element except `a`,
    which starts at row a_row0; elements outside the range get zero gradient.
    reduction="sum" returns the sum instead of the mean; total = the mean's denominator when it is not
    the number of terms summed here (a data-parallel rank's share of a global mean)."""
    return sq_losses(_mse_spec(a, b, c, d, alpha, beta, gamma, delta, count, a_row0, reduction, total))[0]


def wall_mse(y, n, row0=0, total=None):
    """mean(y[r:r+n, 0]**2) + mean(y[r+n:r+2n, 1]**2), r = row0, for y of shape (R, m),
    m >= 2, R >= r + 2n (the normal-component wall terms of both boundary bands in one
    launch; the other rows -- a merged launch's interior points -- get zero gradient);
    total = the means' denominator (default n)."""
    return sq_losses(_wall_spec(y, n, row0, total))[0]


def axpy_clamp(x, y, alpha, lo, hi):
    """clamp(x + alpha y, lo, hi) in one launch (no autograd: the fluid advection's foot,
    computed under no_grad, fluid/model.py:97)."""
    x, y = _prep(x), _prep(y)
    if x.shape != y.shape:
        raise ValueError(f"axpy_clamp: {tuple(x.shape)} vs {tuple(y.shape)}")
    out = torch.empty_like(x)
    nat.check(nat.lib().insr_axpy_clamp(nat.ptr(x), nat.ptr(y), float(alpha), float(lo), float(hi), nat.ptr(out),
                                        x.numel(), nat.stream_of(x.device)), "insr_axpy_clamp")
    return out


_SVD_WORK = {}  # (device index, stream handle) -> partials buffer of the SVD-energy reduction


class _SvdEnergy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, J, ratio_arap, ratio_volume, n):
        lib = nat.lib()
        dev = J.device
        key = _stream_key(dev)
        if key not in _SVD_WORK:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("SVD-energy workspace must be created before graph capture (run one eager call)")
            _SVD_WORK[key] = torch.empty(lib.insr_svd_energy_work_floats(), device=dev, dtype=torch.float32)
        out = torch.empty((), device=dev, dtype=torch.float32)
        d = J.shape[-1]
        rc = lib.insr_svd_energy_fwd(nat.ptr(J), n, d, float(ratio_arap), float(ratio_volume), nat.ptr(out),
                                     nat.ptr(_SVD_WORK[key]), nat.stream_of(dev))
        nat.check(rc, "insr_svd_energy_fwd")
        ctx.save_for_backward(J)
        ctx.args = (float(ratio_arap), float(ratio_volume), n)
        return out

    @staticmethod
    def backward(ctx, gout):
        (J,) = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None, None
        ra, rv, n = ctx.args
        gJ = torch.empty_like(J) if n == J.shape[0] else torch.zeros_like(J)
        g = gout.reshape(1) if gout.is_contiguous() else gout.contiguous().reshape(1)
        rc = nat.lib().insr_svd_energy_bwd(nat.ptr(J), n, J.shape[-1], ra, rv, nat.ptr(g), nat.ptr(gJ),
                                           nat.stream_of(J.device))
        nat.check(rc, "insr_svd_energy_bwd")
        return gJ, None, None, None


def svd_energy(J, ratio_arap=1.0, ratio_volume=0.0, count=None):
    """sum over points of ratio_arap * sum_i (s_i - 1)^2 + ratio_volume * (prod_i s_i - 1)^2,
    s = singular values of each J[n] (d x d, d = 2 or 3) -- the ARAP and volume terms of
    elasticity/model.py:143-163 in one launch (torch.svd's gradient U diag(dE/ds) V^T in
    one backward launch).  count: only the first `count` blocks (the interior rows of a
    merged jet launch; the other blocks get zero gradient)."""
    if J.dim() != 3 or J.shape[-1] != J.shape[-2] or J.shape[-1] not in (2, 3):
        raise ValueError(f"svd_energy: expected (N, d, d) with d in (2, 3), got {tuple(J.shape)}")
    n = J.shape[0] if count is None else int(count)
    if n > J.shape[0] or n < 0:
        raise ValueError(f"svd_energy: count {n} > {J.shape[0]} blocks")
    return _SvdEnergy.apply(_prep(J), ratio_arap, ratio_volume, n)


_EL_WORK = {}  # (device index, stream handle) -> per-term partials + ticket of insr_elastic_energy


class _ElasticEnergy(torch.autograd.Function):
    """insr_elastic_energy: the energy and, in the same launch, its gradient for a unit seed
    w.r.t. the field rows f and the Jacobian J (the backward of a unit-seeded loss costs no
    launch; any other seed scales the written gradients)."""

    @staticmethod
    def forward(ctx, f, J, spec, consts):
        x, f_prev, f_pp = consts
        dev = f.device
        key = _stream_key(dev)
        if key not in _EL_WORK:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("elastic-energy workspace must be created before graph capture "
                                   "(base.losses.prepare_workspaces(stream) or one eager call on the stream)")
            _EL_WORK[key] = torch.zeros(nat.lib().insr_elastic_work_floats(), device=dev, dtype=torch.float32)
        out = torch.empty((), device=dev, dtype=torch.float32)
        terms = torch.empty(nat.EL_TERMS, device=dev, dtype=torch.float32)
        need_f, need_J = ctx.needs_input_grad[0], J is not None and ctx.needs_input_grad[1]
        gf = torch.empty_like(f) if need_f else None
        # the kernel writes dE/dJ only when an SVD term (arap / volume) has a nonzero ratio
        # (svd_energy.hip); otherwise the gradient w.r.t. J is exactly zero
        svd_on = any(spec["ratio"].get(nat.EL_IDS[t], 0.0) != 0.0 for t in ("arap", "volume"))
        gJ = (torch.empty_like(J) if svd_on else torch.zeros_like(J)) if need_J else None
        e = nat.Elastic()
        d = f.shape[1]
        e.d, e.n, e.rows = d, spec["n"], f.shape[0]
        e.f, e.J, e.x, e.f_prev, e.f_pp = nat.ptr(f), nat.ptr(J), nat.ptr(x), nat.ptr(f_prev), nat.ptr(f_pp)
        e.dt = spec["dt"]
        for t, r in spec["ratio"].items():
            e.ratio[t] = r
        for k in range(d):
            e.ext[k], e.target[k], e.center[k] = spec["ext"][k], spec["target"][k], spec["center"][k]
        e.plane_height, e.radius = spec["plane_height"], spec["radius"]
        e.row_l, e.n_l, e.row_r, e.n_r = spec["rows_l"] + spec["rows_r"]
        e.n_order = len(spec["order"])
        for k, t in enumerate(spec["order"]):
            e.order[k] = t
        e.out, e.terms, e.gf, e.gJ = nat.ptr(out), nat.ptr(terms), nat.ptr(gf), nat.ptr(gJ)
        nat.check(nat.lib().insr_elastic_energy(ctypes.byref(e), nat.ptr(_EL_WORK[key]), nat.stream_of(dev)),
                  "insr_elastic_energy")
        ctx.pre = (gf, gJ)
        ctx.mark_non_differentiable(terms)
        ctx.set_materialize_grads(False)  # the unused terms output: no zero-filled gradient launch
        return out, terms

    @staticmethod
    def backward(ctx, gtotal, _gterms):
        gf, gJ = ctx.pre  # kept (retain_graph=True may run the backward again)
        if gtotal is None:
            return None, None, None, None
        if not (gtotal.numel() == 1 and gtotal.data_ptr() in _UNIT_SEEDS):
            gf = None if gf is None else gf * gtotal
            gJ = None if gJ is None else gJ * gtotal
        return gf, gJ, None, None


def elastic_energy(f, J, x, f_prev, f_pp, *, n, dt, energy, ratios, ext=(0.0, 0.0, 0.0), external_on=True,
                   rows_l=(0, 0), rows_r=(0, 0), target=(0.0, 0.0, 0.0), plane_height=0.0, center=(0.0, 0.0, 0.0),
                   radius=0.0):
    """The elastodynamics energy of elasticity/model.py:131-186 in ONE launch (insr_elastic_energy).

    f: (rows, d) trainable field values of one merged jet launch -- rows [0, n) at the interior
    points x, rows_l = (first row, count) / rows_r the fixed points of the positional
    constraints; J: (rows, d, d) the field's Jacobian df/dx (None without arap / volume);
    f_prev, f_pp: the frozen fields at x.  energy: cfg.energy (terms are added in that order);
    ratios: {term: ratio}.  Returns (total, terms) -- total differentiable w.r.t. f and J,
    terms (8 floats, non-differentiable) the per-term values (index INSR_EL_*, base._native.EL_IDS)."""
    ids = nat.EL_IDS
    order, ratio = [], {}
    if "constraint_right" in energy and "constraint_right_compress" in energy:
        # the reference adds two terms with opposite targets; the fused launch has one slot
        raise _unsupported("constraint_right and constraint_right_compress together are not fused")
    for term in energy:
        if term == "constraint_right_compress":
            t = ids["constraint_right"]
        elif term in ids:
            t = ids[term]
        else:
            raise NotImplementedError(term)
        if term == "external" and not external_on:
            continue
        order.append(t)
        ratio[t] = 1.0 if term == "external" else float(ratios[term])
    spec = {"n": int(n), "dt": float(dt), "ratio": ratio, "order": order, "ext": [float(v) for v in ext],
            "target": [float(v) for v in target], "center": [float(v) for v in center],
            "plane_height": float(plane_height), "radius": float(radius),
            "rows_l": tuple(int(v) for v in rows_l), "rows_r": tuple(int(v) for v in rows_r)}
    f = _prep(f)
    J = None if J is None else _prep(J)
    x, f_prev, f_pp = _prep(x.detach()), _prep(f_prev.detach()), _prep(f_pp.detach())
    return _ElasticEnergy.apply(f, J, spec, (x, f_prev, f_pp))


def _unsupported(msg):
    from ._jet import UnsupportedPattern
    return UnsupportedPattern(msg)
