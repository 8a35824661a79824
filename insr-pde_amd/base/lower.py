"""Loss lowering for unchanged model files: the reference phase bodies' torch residual expressions
(fluid/model.py:72-151, advection/model.py:68-91) become ONE loss-group launch per iteration.

A reference phase body spells each loss as a chain of aten ops on the network outputs --
torch.mean((u - target) ** 2), (torch.mean(ux[..., 0] ** 2) + torch.mean(uy[..., 1] ** 2)) * 1.0,
F.mse_loss(u, ref) -- about 25 small launches forward and backward per phase iteration, which
cost more than they compute (profiles/r03/plain_glue_attribution.txt).  While the training loop
runs a phase body inside `lowering()` (base/_loop.py, models that do not opt out), every network
and diff-op output is handed to the body as a `Lazy` tensor: a storage-less wrapper whose
arithmetic is RECORDED instead of launched.  When the body returns, `lower_losses` reads each
loss of its dict as a sum of mean squares of linear combinations of network / diff-op outputs
and ordinary tensors and maps it onto the fused loss group (base/losses.py):

    mean((c1 T1 + c2 T2 + c3 T3 + c4 T4) ** 2)              -> one COMBO term (r = alpha (a + beta b)
                                                               + gamma (c + delta d))
    w (mean(A[..., 0] ** 2) + mean(B[..., 1] ** 2))          -> one BANDS term over two tensors

so that every loss of the iteration is ONE insr_sq_loss_group launch whose unit-seeded backward
costs nothing.  The semi-Lagrangian foot clamp(x - dt u, lo, hi) a no-grad jet consumes is one
insr_axpy_clamp launch.  Inside `deferred_jets()` (opened with it) the body's network / diff-op calls
are queued and launched together at the first read of a value (below).

Anything else is EAGER, exactly as written: an op the recorder does not know, or any use of a
Lazy tensor's value (float(), .cpu(), an unsupported torch function, a network input, ...),
materialises it -- the recorded torch calls replayed on the real tensors, in the grad mode they
were recorded in, with their autograd history (cached: one replay per node).  A loss the lowering
does not recognise is materialised the same way.  So the lowering changes launch counts and fp32
rounding order (a mean as scale * sum, c x / dt as (c / dt) x), never semantics; the unchanged
reference bodies are pinned to the reference golden vectors through it
(tests/test_gpu_plain_api.py).
"""
import threading

import torch

__all__ = ["Lazy", "lowering", "deferred_jets", "deferring", "flush", "immediate", "add_views", "eye_add", "lazy_call",
           "suspended", "api", "sampler_api", "active", "leaf", "materialize", "plan", "energy_plan", "lower_losses",
           "LOWERED"]

LOWERED = {"groups": 0, "terms": 0, "eager_losses": 0, "materialized": 0, "energies": 0}  # counters (tests, docs)


class _State(threading.local):
    affine = False  # the running diff op's operand is f of a recorded f(x) + x (api, _affine_operand)
    depth = 0
    defer = 0  # > 0: network / diff-op jets are queued (a fused_forwards scope) and launched at the first read
    nodes = None  # the recorded nodes of the open scope (evaluated before an in-place op, see _pin_all)


_S = _State()


class lowering:
    """`with lowering(on): body()` -- network / diff-op outputs created inside are Lazy."""

    def __init__(self, on=True):
        self.on = bool(on)

    def __enter__(self):
        if self.on:
            _S.depth += 1
        return self

    def __exit__(self, *exc):
        if self.on:
            _S.depth -= 1
            if _S.depth == 0:
                _S.nodes = None
        return False


def active():
    return _S.depth > 0


# ---- deferred jets ------------------------------------------------------------------------------
# Inside `deferred_jets()` (opened by the loop with lowering()) the forward jets the body asks for are
# QUEUED, as in a base.fused_forwards scope (base/_jet.py): the phase body gets Lazy leaves of their
# (not yet written) outputs, and the queue is launched -- jets of one architecture as ONE multi / mixed
# launch -- at the first read of any value (materialize), before a diff op that needs values, and at the
# scope's exit.  So the reference's separate calls (the interior batch and each wall band, the frozen and
# the trainable field) share launches as the hand-fused model files arrange them.
class deferred_jets:
    """`with deferred_jets(on): body()` -- see above."""

    def __init__(self, on=True):
        self.on = bool(on)

    def __enter__(self):
        if self.on:
            from . import _jet
            self.ff = _jet.fused_forwards()
            self.ff.__enter__()
            _S.defer += 1
        return self

    def __exit__(self, *exc):
        if self.on:
            _S.defer -= 1
            self.ff.__exit__(*exc)
        return False


def deferring():
    """Whether jets are being queued right now (a deferred_jets scope with its fused scope open)."""
    if _S.defer <= 0:
        return False
    from . import _jet
    return _jet._Fused.pending is not None


def flush():
    """Launch the queued jets now (the scope stays open for the next ones)."""
    if _S.defer <= 0:
        return
    from . import _jet
    jobs = _jet._Fused.pending
    if jobs:
        _jet._Fused.pending = []
        _jet._launch_fused(jobs)


class immediate:
    """`with immediate():` -- jets launched at once inside (the queue flushed first): a diff-op route that
    reads its jets' values in the same call (Hessian polarisation, the reference-semantics fallback)."""

    def __enter__(self):
        from . import _jet
        self.saved = None
        if _S.defer > 0 and _jet._Fused.pending is not None:
            flush()
            self.saved, _jet._Fused.pending = _jet._Fused.pending, None
        return self

    def __exit__(self, *exc):
        if self.saved is not None:
            from . import _jet
            _jet._Fused.pending = self.saved
        return False


def add_views(a, b):
    """a + b of two views of queued jet outputs (the divergence's J[..., 0, 0:1] + J[..., 1, 1:2]): recorded
    as a Lazy sum while jets are deferred (its operands have no values yet), else added now."""
    if not deferring():
        return a + b
    n = _Node("lin", (_Node("leaf", real=a, shape=tuple(a.shape)), _Node("leaf", real=b, shape=tuple(b.shape))),
              coef=(1.0, 1.0), call=(torch.add, (a, b), {}), shape=tuple(a.shape))
    n.grad_mode = torch.is_grad_enabled()
    _register(n)
    return _wrap(n, a.dtype, a.device, torch.is_grad_enabled() and (a.requires_grad or b.requires_grad))


# ---- the recorded graph ------------------------------------------------------------------------
# node kinds: 'leaf' (a real tensor), 'lin' (sum of coefficient x node), 'sq' (x ** 2), 'mean' (all
# elements), 'sel' (x[..., k] of a 2-D x), 'detach', 'clamp' (scalar bounds).  Every node keeps the
# torch call that made it (func, args, kwargs, grad mode): materialisation replays exactly that.
#
# In-place writes.  A recorded expression is evaluated later than eager code would evaluate it, so a
# tensor it reads must not change in between.  An in-place op on a Lazy tensor (add_, __setitem__,
# out=, ...) first evaluates every node recorded so far in the scope (_pin_all: their values are the
# ones eager code computed before the write), then writes the real tensor, and the Lazy tensor stands
# for the written tensor from then on.  Every leaf keeps its tensor's version counter: a loss whose
# leaves were written since they were recorded is not lowered (its cached / replayed values are used),
# and a replay that would read a tensor written behind the recorder's back (an in-place op on a plain
# tensor a recorded expression reads) raises instead of computing with the new values.
class _Node:
    __slots__ = ("kind", "kids", "coef", "k", "lo", "hi", "real", "real_ng", "call", "shape", "grad_mode", "ver",
                 "ready", "meta")

    def __init__(self, kind, kids=(), coef=None, k=None, lo=None, hi=None, real=None, call=None, shape=None):
        self.kind, self.kids, self.coef, self.k, self.lo, self.hi = kind, tuple(kids), coef, k, lo, hi
        self.real, self.real_ng, self.call, self.shape = real, None, call, shape
        self.ready = False  # real holds final values no queued jet writes (a sampler's draw, or c times one)
        self.meta = None  # (eyeadd) the Jacobian jet's provenance: (mlp, value f, x)
        self.grad_mode = torch.is_grad_enabled()
        self.ver = real._version if real is not None else None


def _register(n):
    if _S.depth > 0:
        if _S.nodes is None:
            _S.nodes = []
        _S.nodes.append(n)


def _stale(n, through=True, seen=None):
    """Whether a leaf under n was written since it was recorded.  through=False stops at evaluated nodes
    (a replay reads their cached values); through=True looks through them (a plan reads the leaves)."""
    seen = set() if seen is None else seen
    if id(n) in seen:
        return False
    seen.add(id(n))
    if n.kind == "leaf":
        return n.real._version != n.ver
    if not through and n.real is not None:
        return False
    return any(_stale(k, through, seen) for k in n.kids)


_INPLACE_DUNDER = frozenset("__%s__" % n for n in ("setitem", "iadd", "isub", "imul", "itruediv", "ifloordiv", "imod",
                                                  "ipow", "iand", "ior", "ixor", "ilshift", "irshift", "imatmul"))


def _mutated(name, args, kwargs):
    """The tensors an op writes in place (empty for a functional op)."""
    out = []
    if "out" in kwargs:
        o = kwargs["out"]
        out.extend(o if isinstance(o, (list, tuple)) else [o])
    if args and (name in _INPLACE_DUNDER or
                 (name.endswith("_") and not name.startswith("_") and name != "requires_grad_")):
        out.append(args[0])
    return [t for t in out if isinstance(t, torch.Tensor)]


def _pin_all():
    """Evaluate every node recorded in the open scope that is not evaluated yet (before an in-place op)."""
    flush()  # (a node may read a queued jet's output directly, e.g. add_views)
    for n in list(_S.nodes or ()):
        if n.real is None and n.call is not None:
            _eval(n)


_META = {"numel", "dim", "size", "__len__", "is_floating_point", "nelement", "element_size", "ndimension",
         "get_device"}
# properties a Lazy tensor answers from its own metadata; every other attribute (data, grad_fn, is_leaf,
# grad, T, ...) is read off the materialised tensor
_META_ATTRS = {"shape", "dtype", "device", "requires_grad", "is_cuda", "ndim", "layout", "is_sparse", "is_quantized",
               "is_meta", "is_nested", "is_mkldnn", "is_complex"}


class Lazy(torch.Tensor):
    """A recorded (not yet computed) tensor: shape, dtype, device and requires_grad are real; any
    use of its value materialises it (see the module docstring)."""

    @staticmethod
    def __new__(cls, node, dtype, device, requires_grad):
        t = torch.Tensor._make_wrapper_subclass(cls, node.shape, dtype=dtype, device=device,
                                                requires_grad=bool(requires_grad))
        t._insr_node = node
        return t

    def __repr__(self):  # what eager code would print: the value
        return repr(materialize(self))

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = getattr(func, "__name__", "")
        if name in _META or (name == "__get__" and getattr(getattr(func, "__self__", None), "__name__", "")
                             in _META_ATTRS):
            with torch._C.DisableTorchFunctionSubclass():
                return func(*args, **kwargs)
        written = _mutated(name, args, kwargs)
        if written:  # (a plain tensor written with a Lazy operand, x[:, 0] = u, may be read by a record too)
            _pin_all()
            r = func(*_real_tree(args), **_real_tree(kwargs))
            for t in written:  # a written Lazy tensor now stands for its written real tensor
                if not isinstance(t, Lazy):
                    continue
                real = materialize(t)
                t._insr_node = _Node("leaf", real=real, shape=tuple(real.shape))
                if r is real:  # u.add_(1) / u += 1 return u itself, as in eager code
                    r = t
            return r
        r = _record(name, func, args, kwargs)
        if r is not None:
            return r
        return func(*_real_tree(args), **_real_tree(kwargs))

    @classmethod
    def __torch_dispatch__(cls, func, types, args=(), kwargs=None):
        # below autograd (a path that bypassed __torch_function__): compute on the real tensors
        return func(*_real_tree(args), **_real_tree(kwargs or {}))


def _wrap(node, like_dtype, like_device, requires_grad):
    return Lazy(node, like_dtype, like_device, requires_grad)


def leaf(t):
    """A network / diff-op output as a Lazy leaf (inside lowering(); otherwise t itself)."""
    if not active() or not isinstance(t, torch.Tensor) or isinstance(t, Lazy) or t.dtype != torch.float32:
        return t
    return _wrap(_Node("leaf", real=t, shape=tuple(t.shape)), t.dtype, t.device, t.requires_grad)


def sampler_api(fn):
    """A sampler of the base API (sample_random, sample_boundary, ...).  Inside lowering() its GPU result is
    a READY Lazy leaf -- a drawn tensor, which no queued jet writes: handing it to a network or diff op
    launches nothing, and a body's scalar rescale of its samples (advection/model.py:27,86:
    sample_random(...).requires_grad_(True) * self.length / 2) is recorded and evaluated as ONE launch
    instead of one per operator."""
    import functools

    @functools.wraps(fn)
    def w(*args, **kwargs):
        r = fn(*_real_tree(args), **_real_tree(kwargs))
        if not active() or not isinstance(r, torch.Tensor) or isinstance(r, Lazy) or r.dtype != torch.float32 \
                or not r.is_cuda:
            return r
        n = _Node("leaf", real=r, shape=tuple(r.shape))
        n.ready = True
        return _wrap(n, r.dtype, r.device, r.requires_grad)
    return w


class suspended:
    """`with suspended():` -- no Lazy outputs inside (a base-API call's own nested calls)."""

    def __enter__(self):
        self.depth, _S.depth = _S.depth, 0
        return self

    def __exit__(self, *exc):
        _S.depth = self.depth
        return False


def api(fn, operand_first=False):
    """Decorator of the base API entry points (the networks' forward, the diff ops): Lazy arguments are
    materialised, the call runs unlowered, and its tensor results come back as Lazy leaves while
    lowering() is active.  operand_first (the diff ops): the first argument -- the differentiated output,
    read for its provenance, not its values -- is handed over without launching the queued jets when it
    is a Lazy leaf."""
    import functools

    @functools.wraps(fn)
    def w(*args, **kwargs):
        if not operand_first and len(args) == 2 and not kwargs and isinstance(args[1], Lazy) and deferring() \
                and not torch.is_grad_enabled():  # a network call at the advection foot
            r = _advect_target(args[0], args[1])
            if r is not None:
                return leaf(r)
        affine = False
        if operand_first and args:
            rest = tuple(_real_tree(a) for a in args[1:])
            f = _affine_operand(args[0], rest[0] if rest else None)
            if f is not None:  # q = f(x) + x still recorded: the diff op takes f with the identity added
                args, affine = (f,) + rest, True
            else:
                args = (_api_tree(args[0]),) + rest
        else:
            args = _real_tree(args)
        kwargs = _real_tree(kwargs)
        if not active():
            return fn(*args, **kwargs)
        _S.affine = affine
        try:
            with suspended():
                r = fn(*args, **kwargs)
        finally:
            _S.affine = False
        if isinstance(r, tuple):
            return tuple(leaf(v) for v in r)
        return leaf(r)
    return w


def _affine_operand(v, x):
    """f when v is the recorded q = f + x (x + f) of a network output f at x (elasticity/model.py:137), else None."""
    if not isinstance(v, Lazy) or x is None:
        return None
    n = v._insr_node
    if n.kind != "lin" or len(n.kids) != 2 or tuple(n.coef) != (1.0, 1.0) or any(k.kind != "leaf" for k in n.kids):
        return None
    a, b = n.kids
    for f, y in ((a, b), (b, a)):
        src = getattr(f.real, "_insr_src", None)
        if y.real is x and src is not None and src[1] is x and f.real.shape == x.shape and not _stale(n):
            return f.real
    return None


def affine_operand():
    """Whether the diff op running now was handed f of a recorded f(x) + x (its result adds the identity)."""
    return getattr(_S, "affine", False)


def _advect_target(mlp, foot):
    """f(clamp(x - dt f(x), lo, hi)) of a frozen field f asked for (no_grad) while f(x) is still a queued
    value jet of the same network at the same x (fluid/model.py:79-87 as written): ONE advection-target job
    of the mixed launch (base._jet.advect_target) that also writes f(x) into the queued jet's output, whose
    own job is dropped -- the hand-fused model's launch (pde/fluid.py).  None when the pattern does not hold."""
    from . import _jet
    n = foot._insr_node
    if n.kind != "clamp" or not hasattr(mlp, "flat_params") or _jet._Fused.pending is None:
        return None
    at = _atoms(n.kids[0])
    if at is None or len(at) != 2:
        return None
    (cx, ax), (cy, ay) = at.values()
    if cx != 1.0:
        (cx, ax), (cy, ay) = (cy, ay), (cx, ax)
    if cx != 1.0 or ax.kind != "leaf" or ay.kind != "leaf":
        return None
    x, u = ax.base, ay.base
    if x.dim() != 2 or u.shape != x.shape or not x.is_contiguous():
        return None
    flat = mlp.flat_params()
    for i, (key, job) in enumerate(_jet._Fused.pending):
        if len(job) == 8 and job[2] is u and job[1] is flat and job[3] is None and job[5] is None and \
                job[0].data_ptr() == x.data_ptr() and job[0].shape == x.shape and \
                (key[3] & 0xF) == 0:  # a VALUE jet (INSR_MODE_VALUE)
            try:
                y, _ = _jet.advect_target(mlp, x, -cy, n.lo, n.hi, up=u)
            except _jet.UnsupportedPattern:
                return None
            del _jet._Fused.pending[i]  # f(x) now comes from the target job
            return y
    return None


def _scalar(v):
    """A Python float of a number or a 0-dim CPU tensor, else None (never a device read)."""
    if isinstance(v, bool):
        return None
    if isinstance(v, (int, float)):
        return float(v)
    if isinstance(v, torch.Tensor) and not isinstance(v, Lazy) and v.dim() == 0 and v.device.type == "cpu":
        return float(v)
    return None


def _operand(v):
    """The node of a tensor operand of a recorded op (a real tensor becomes a leaf), None otherwise."""
    if isinstance(v, Lazy):
        return v._insr_node
    if isinstance(v, torch.Tensor) and v.dtype == torch.float32:
        return _Node("leaf", real=v, shape=tuple(v.shape))
    return None


def _req(*vals):
    return torch.is_grad_enabled() and any(isinstance(v, torch.Tensor) and v.requires_grad for v in vals)


def _lazy_of(kind, kids, call, shape, like, req, **kw):
    n = _Node(kind, kids, call=call, shape=tuple(shape), **kw)
    _register(n)
    return _wrap(n, like.dtype, like.device, req)


def _record(name, func, args, kwargs):
    """A Lazy result of func(*args, **kwargs) when it is an op the lowering knows, else None."""
    call = (func, args, kwargs)
    tens = [a for a in args if isinstance(a, torch.Tensor)]
    like = next((a for a in tens if isinstance(a, Lazy)), None)
    if like is None or like.dtype != torch.float32:
        return None
    if name in ("add", "sub", "__radd__", "__rsub__") and len(args) == 2 and set(kwargs) <= {"alpha"} and \
            isinstance(args[0], Lazy) and _scalar(args[1]) is not None and _scalar(kwargs.get("alpha", 1.0)) is not None:
        # x + c, x - c (S - 1.0, q_fixed - 0: elasticity/model.py:146-147, losses.py:7), c + x, c - x
        x, c = args[0], _scalar(args[1]) * _scalar(kwargs.get("alpha", 1.0))
        nx = x._insr_node
        if name == "__rsub__":
            nx = _Node("lin", (nx,), coef=(-1.0,), call=None, shape=nx.shape)
        return _lazy_of("off", (nx,), call, nx.shape, like, _req(x), lo=(-c if name == "sub" else c))
    if name == "prod" and isinstance(args[0], Lazy) and len(args[0]._insr_node.shape) == 2 and \
            ((len(args) == 2 and not kwargs) or (len(args) == 1 and set(kwargs) == {"dim"})):
        x = args[0]
        dim = args[1] if len(args) == 2 else kwargs["dim"]
        if not isinstance(dim, int) or dim % 2 != 1:
            return None
        return _lazy_of("prod", (x._insr_node,), call, x._insr_node.shape[:1], like, _req(x), k=1)
    if name == "mul" and len(args) == 2 and not kwargs and _scalar(args[0]) is None and _scalar(args[1]) is None:
        # x * T with a constant tensor T of x's shape (elasticity/model.py:149's external-force product)
        x, y = args
        if not isinstance(x, Lazy):
            x, y = y, x
        if isinstance(x, Lazy) and isinstance(y, torch.Tensor) and not isinstance(y, Lazy) and not y.requires_grad:
            ny = _operand(y)
            if ny is not None and ny.shape == x._insr_node.shape:
                return _lazy_of("mulT", (x._insr_node, ny), call, x._insr_node.shape, like, _req(x, y))
        return None
    if name == "svd" and len(args) == 1 and not kwargs and isinstance(args[0], Lazy) and \
            len(args[0]._insr_node.shape) == 3 and args[0]._insr_node.shape[1] == args[0]._insr_node.shape[2]:
        # torch.svd(J) of a batch of square Jacobians (elasticity/model.py:144): three Lazy parts of ONE svd
        # node, evaluated (torch.svd) only when a part's value is read
        x = args[0]
        nd = x._insr_node
        parent = _Node("svd", (nd,), call=call, shape=nd.shape)
        _register(parent)
        req = _req(x)
        shapes = (nd.shape, nd.shape[:2], nd.shape)
        return tuple(_lazy_of("svdpart", (parent,), (_svd_part, (parent, i), {}), shapes[i], like, req, k=i)
                     for i in range(3))
    if name in ("add", "sub") and len(args) == 2 and set(kwargs) <= {"alpha"}:
        x, y = args
        nx, ny = _operand(x), _operand(y)
        alpha = _scalar(kwargs.get("alpha", 1.0))
        if nx is None or ny is None or alpha is None or nx.shape != ny.shape:
            return None  # scalar offsets (no constant term in a residual) and broadcasting stay eager
        sgn = alpha if name == "add" else -alpha
        return _lazy_of("lin", (nx, ny), call, nx.shape, like, _req(x, y), coef=(1.0, sgn))
    if name in ("mul", "div") and len(args) == 2 and not kwargs:
        x, y = args
        if name == "mul" and isinstance(x, Lazy) and x is y:
            return _lazy_of("sq", (x._insr_node,), call, x._insr_node.shape, like, _req(x))
        if not isinstance(x, Lazy) and name == "mul":
            x, y = y, x
        c = _scalar(y)
        if not isinstance(x, Lazy) or c is None:
            return None
        if name == "div":
            if c == 0.0:
                return None
            c = 1.0 / c
        return _lazy_of("lin", (x._insr_node,), call, x._insr_node.shape, like, _req(x), coef=(c,))
    if name == "neg" and len(args) == 1 and not kwargs:
        x = args[0]
        return _lazy_of("lin", (x._insr_node,), call, x._insr_node.shape, like, _req(x), coef=(-1.0,))
    if name in ("pow", "square") and not kwargs and isinstance(args[0], Lazy):
        e = 2.0 if name == "square" else (_scalar(args[1]) if len(args) == 2 else None)
        if e != 2.0:
            return None
        x = args[0]
        return _lazy_of("sq", (x._insr_node,), call, x._insr_node.shape, like, _req(x))
    if name in ("mean", "sum") and len(args) == 1 and not kwargs and isinstance(args[0], Lazy):
        x = args[0]
        return _lazy_of(name, (x._insr_node,), call, (), like, _req(x))
    if name == "mse_loss" and len(args) == 2 and set(kwargs) <= {"reduction", "size_average", "reduce", "weight"} \
            and kwargs.get("reduction", "mean") in ("mean", "sum") and all(kwargs.get(k) is None for k in
                                                                             ("size_average", "reduce", "weight")):
        x, y = args
        nx, ny = _operand(x), _operand(y)
        if nx is None or ny is None or nx.shape != ny.shape:
            return None
        r = _req(x, y)
        d = _Node("lin", (nx, ny), coef=(1.0, -1.0), call=None, shape=nx.shape)
        s = _Node("sq", (d,), call=None, shape=nx.shape)
        return _lazy_of(kwargs.get("reduction", "mean"), (s,), call, (), like, r)
    if name == "__getitem__" and len(args) == 2 and isinstance(args[0], Lazy):
        x, idx = args
        n = x._insr_node
        if len(n.shape) == 2 and isinstance(idx, tuple) and len(idx) == 2 and isinstance(idx[1], int) and \
                (idx[0] is Ellipsis or idx[0] == slice(None)) and -n.shape[1] <= idx[1] < n.shape[1]:
            k = idx[1] % n.shape[1]
            return _lazy_of("sel", (n,), call, (n.shape[0],), like, x.requires_grad, k=k)
        return None
    if name == "requires_grad_" and isinstance(args[0], Lazy) and args[0]._insr_node.kind == "leaf" and \
            args[0]._insr_node.ready and len(args) <= 2 and set(kwargs) <= {"requires_grad"}:
        x = args[0]  # a sampler's leaf: flag its tensor and the wrapper, as eager code flags the tensor
        flag = bool(args[1]) if len(args) == 2 else bool(kwargs.get("requires_grad", True))
        x._insr_node.real.requires_grad_(flag)
        with torch._C.DisableTorchFunctionSubclass():
            torch.Tensor.requires_grad_(x, flag)
        return x
    if name == "detach" and len(args) == 1 and not kwargs:
        x = args[0]
        return _lazy_of("detach", (x._insr_node,), call, x._insr_node.shape, like, False)
    if name == "clamp" and isinstance(args[0], Lazy):
        lo = kwargs.get("min", args[1] if len(args) > 1 else None)
        hi = kwargs.get("max", args[2] if len(args) > 2 else None)
        if _scalar(lo) is None or _scalar(hi) is None or len(args) > 3 or set(kwargs) - {"min", "max"}:
            return None
        x = args[0]
        return _lazy_of("clamp", (x._insr_node,), call, x._insr_node.shape, like, _req(x), lo=_scalar(lo),
                        hi=_scalar(hi))
    return None


def _svd_part(parent, i):
    """Part i (U, S, V) of a recorded torch.svd, the decomposition computed once."""
    return _eval(parent)[i]


_EYES = {}


def _eye(d, device, dtype):
    """torch.eye(d) on `device`, made once (two fill launches each time otherwise); read-only."""
    key = (d, str(device), dtype)
    e = _EYES.get(key)
    if e is None:
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return torch.eye(d, device=device, dtype=dtype)  # (no allocation kept from a capture pool)
        e = _EYES[key] = torch.eye(d, device=device, dtype=dtype)
    return e


def eye_add(J, meta):
    """J + I of a Jacobian jet J (the affine f(x) + x of elasticity/model.py:137,143): recorded while jets are
    deferred (J has no values yet; an energy lowering reads J itself), else added now.  meta = (mlp, value,
    x) of the jet."""
    eye = _eye(J.shape[-1], J.device, J.dtype)
    if not deferring():
        return J + eye
    leafJ = _Node("leaf", real=J, shape=tuple(J.shape))
    n = _Node("eyeadd", (leafJ,), call=(torch.add, (J, eye), {}), shape=tuple(J.shape))
    n.meta = meta
    _register(n)
    return _wrap(n, J.dtype, J.device, torch.is_grad_enabled() and J.requires_grad)


def lazy_call(fn, args, shape, dtype, device):
    """A Lazy result of fn(*args) with no autograd, computed only when its value is read (the NaN status of
    jacobian(): the reference's host read, elasticity/model.py:143, which no body uses)."""
    n = _Node("call", (), call=(fn, args, {}), shape=tuple(shape))
    _register(n)
    return _wrap(n, dtype, device, False)


# ---- materialisation --------------------------------------------------------------------------
def _api_tree(v):
    """A diff op's operand: a Lazy LEAF is handed over as its real tensor without launching the queued jets
    (the diff ops read its provenance, not its values -- they flush where they do); any other Lazy tensor
    is materialised."""
    if isinstance(v, Lazy) and v._insr_node.kind == "leaf":
        return v._insr_node.real
    return materialize(v)


def _real_tree(v):
    if isinstance(v, Lazy):
        return materialize(v)
    if isinstance(v, (list, tuple)):
        r = [_real_tree(a) for a in v]
        return type(v)(r) if isinstance(v, list) else tuple(r)
    if isinstance(v, dict):
        return {k: _real_tree(a) for k, a in v.items()}
    return v


def _eval(n):
    """The real tensor of node n: its recorded torch call replayed (in its recorded grad mode)."""
    if n.real is not None:
        return n.real
    if n.call is None:  # an internal node (F.mse_loss's parts): evaluated by the enclosing call
        raise RuntimeError("internal lazy node has no call of its own")
    if _stale(n, through=False):
        raise RuntimeError("base/lower.py: a tensor read by a recorded expression was written in place after "
                           "the expression was recorded (an in-place op on a plain tensor); evaluating it now "
                           "would read the new values. Run this model unlowered (cfg.insr_lower = False).")
    sc = _ready_scale(n)
    if sc is not None:  # c x of a ready leaf (a chain of scalar multiplies / divides): one launch
        c, base = sc
        with torch.set_grad_enabled(n.grad_mode):
            n.real = base * c
        n.ready = True
        LOWERED["materialized"] += 1
        return n.real
    func, args, kwargs = n.call
    a, k = _real_tree(args), _real_tree(kwargs)
    with torch.set_grad_enabled(n.grad_mode):
        n.real = func(*a, **k)
    LOWERED["materialized"] += 1
    return n.real


def _ready_scale(n):
    """(c, tensor) when n is c times a ready value (a sampler's draw, or an evaluated rescale of one) through
    single-operand scalar 'lin' nodes, else None."""
    c, m = 1.0, n
    while m.kind == "lin" and len(m.kids) == 1 and m.real is None:
        c *= m.coef[0]
        m = m.kids[0]
    if m is n or m.real is None or not m.ready:
        return None
    return c, m.real


def _axpy_clamp_fast(n):
    """clamp(x + alpha y, lo, hi) of two real same-shape fp32 GPU tensors as one launch (no autograd:
    the consumer runs without gradients), or None."""
    if n.kind != "clamp":
        return None
    at = _atoms(n.kids[0])
    if at is None or len(at) != 2 or any(a.kind == "sel" for _, a in at.values()):
        return None
    (cx, ax), (cy, ay) = at.values()
    if cx != 1.0:
        (cx, ax), (cy, ay) = (cy, ay), (cx, ax)
    if cx != 1.0:
        return None
    x, y = ax.base, ay.base
    if not (x.is_cuda and y.is_cuda and x.shape == y.shape and x.is_contiguous() and y.is_contiguous()):
        return None
    from .losses import axpy_clamp
    return axpy_clamp(x.detach(), y.detach(), cy, n.lo, n.hi)


def materialize(t):
    """The real tensor of t (t itself when it is not Lazy).  Under no_grad a clamp(x + a y) node takes
    the one-launch axpy_clamp (cached apart from the autograd-carrying replay).  Queued jets are
    launched first (their outputs are what the value reads)."""
    if not isinstance(t, Lazy):
        return t
    n = getattr(t, "_insr_node", None)
    if n is None:
        raise RuntimeError("a storage-less Lazy tensor without its record (made by torch from a Lazy tensor "
                           "below __torch_function__): base/lower.py cannot compute it")
    if n.ready and n.real is not None:  # a sampler's draw, or c times one: no queued jet's output in it
        return n.real
    if n.real is None and _ready_scale(n) is not None:
        return _eval(n)
    flush()
    if not torch.is_grad_enabled() and n.real is None:
        if n.real_ng is None:
            n.real_ng = _axpy_clamp_fast(n)
        if n.real_ng is not None:
            return n.real_ng
    return _eval(n)


# ---- lowering of the loss dict ----------------------------------------------------------------
def _ms_terms(n, w=1.0):
    """n as [(w_i, E_i, red_i)] with n = sum_i w_i red_i(E_i ** 2), red = 'mean' or 'sum', or None."""
    if n.kind in ("mean", "sum") and n.kids[0].kind == "sq":
        return [(w, n.kids[0].kids[0], n.kind)]
    if n.kind == "lin":
        out = []
        for c, kid in zip(n.coef, n.kids):
            t = _ms_terms(kid, w * c)
            if t is None:
                return None
            out.extend(t)
        return out
    return None


class _Atom:
    """An operand of a linear residual: a leaf tensor or a column of one (sel), possibly detached."""
    __slots__ = ("kind", "k", "base", "det")

    def __init__(self, kind, k, base, det):
        self.kind, self.k, self.base, self.det = kind, k, base, det


def _atoms(n, c=1.0, acc=None, det=False):
    """E as {key: (coefficient, _Atom)} over leaf / sel operands (first-appearance order; a detach anywhere
    above an operand detaches it: detach(sum c_i T_i) = sum c_i detach(T_i)), or None."""
    acc = {} if acc is None else acc
    if n.kind == "lin":
        for ci, kid in zip(n.coef, n.kids):
            if _atoms(kid, c * ci, acc, det) is None:
                return None
        return acc
    if n.kind == "detach":
        return _atoms(n.kids[0], c, acc, True)
    if n.kind == "off" and n.lo == 0.0:  # x - 0 (a positional constraint's zero target)
        return _atoms(n.kids[0], c, acc, det)
    if n.kind == "sel":
        base = n.kids[0]
        while base.kind == "detach":
            det, base = True, base.kids[0]
        if base.kind != "leaf":
            return None
        a = _Atom("sel", n.k, base.real, det)
    elif n.kind == "leaf":
        a = _Atom("leaf", None, n.real, det)
    else:
        return None
    key = (a.kind, a.k, id(a.base), a.det)
    acc[key] = (acc[key][0] + c, a) if key in acc else (c, a)
    return acc


def _atom_tensor(a):
    """The real tensor (or view) an atom reads: no launch (views, detach)."""
    t = a.base if a.kind == "leaf" else a.base[..., a.k]
    return t.detach() if a.det else t


def plan(n):
    """The fused form of loss node n, or None (eager):
      ("combo", (a, b, c, d), (alpha, beta, gamma, delta), w, red): w red((alpha (a + beta b) + gamma (c + delta d))^2),
                                                                   red = 'mean' or 'sum'
      ("bands2", (A, B), w):                                   w (mean(A[:, 0]^2) + mean(B[:, 1]^2))
    (a contiguous; b, c, d None or same-shape tensors / 1-D strided views; no launch is made here)."""
    if _stale(n):  # a leaf written since it was recorded: the recorded values are the cached ones (eager)
        return None
    terms = _ms_terms(n)
    if not terms or any(w == 0.0 for w, _, _ in terms):
        return None
    if len(terms) == 2:  # w (mean(A[..., 0]^2) + mean(B[..., 1]^2)): one BANDS term over two tensors
        (w0, e0, r0), (w1, e1, r1) = terms
        if r0 != "mean" or r1 != "mean":
            return None
        at = [_atoms(e) for e in (e0, e1)]
        if w0 != w1 or any(a is None or len(a) != 1 for a in at):
            return None
        (c0, a0), = at[0].values()
        (c1, a1), = at[1].values()
        if abs(c0) != 1.0 or abs(c1) != 1.0 or a0.kind != "sel" or a1.kind != "sel":
            return None
        if (a0.k, a1.k) == (1, 0):
            a0, a1 = a1, a0
        A = a0.base.detach() if a0.det else a0.base
        B = a1.base.detach() if a1.det else a1.base
        if (a0.k, a1.k) != (0, 1) or A.dim() != 2 or A.shape != B.shape or A.shape[1] < 2 or \
                not (A.is_contiguous() and B.is_contiguous()) or A.device != B.device:
            return None
        return ("bands2", (A, B), w0)
    if len(terms) != 1:
        return None
    (w, e, red), = terms
    at = _atoms(e)
    if at is None or not 1 <= len(at) <= 4:
        return None
    ops = [(c, _atom_tensor(a)) for c, a in at.values() if c != 0.0]
    if not ops:
        return None
    shape, dev = ops[0][1].shape, ops[0][1].device
    if any(t.shape != shape or t.device != dev for _, t in ops):
        return None
    # `a` must be contiguous (b, c, d may be 1-D strided views): a contiguous operand first
    first = next((i for i, (_, t) in enumerate(ops) if t.is_contiguous()), None)
    if first is None:
        return None
    ops = [ops[first]] + ops[:first] + ops[first + 1:]
    while len(ops) < 4:
        ops.append((0.0, None))
    (c1, a), (c2, b), (c3, c), (c4, d) = ops
    alpha, beta = c1, (c2 / c1 if b is not None else -1.0)
    gamma, delta = (1.0, 1.0) if c is None else (c3, (c4 / c3 if d is not None else 1.0))
    return ("combo", (a, b, c, d), (alpha, beta, gamma, delta), w, red)


def _spec(n):
    """The LossSpec (base/losses.py) of loss node n, or None (eager)."""
    from . import losses as L
    p = plan(n)
    if p is None or not all(t is None or t.is_cuda for t in p[1]):
        return None
    if p[0] == "bands2":
        (A, B), w = p[1], p[2]
        return L.wall_term2(A, B, weight=w)
    (a, b, c, d), (alpha, beta, gamma, delta), w, red = p[1], p[2], p[3], p[4]
    # w mean(r^2): the loss's scale is w / count (w = 1 for the reference's losses; * 1.0 is exact); w sum(r^2): w
    return L.mse_term(a, b, c, d, alpha=alpha, beta=beta, gamma=gamma, delta=delta, reduction=red, weight=w)


# ---- elastodynamics energies (elasticity/model.py:127-189, losses.py:6-8) ----------------------------
def _lin_terms(n, w=1.0, out=None):
    """n as [(w_i, T_i)] with n = sum_i w_i T_i through 'lin' nodes and zero offsets (loss = 0; loss = loss + E)."""
    out = [] if out is None else out
    if n.kind == "lin":
        for c, kid in zip(n.coef, n.kids):
            _lin_terms(kid, w * c, out)
    elif n.kind == "off" and n.lo == 0.0:
        _lin_terms(n.kids[0], w, out)
    else:
        out.append((w, n))
    return out


def _svd_of(n):
    """The svd node whose singular values n is (an 'svdpart' k = 1), or None."""
    return n.kids[0] if n.kind == "svdpart" and n.k == 1 else None


def _energy_term(T):
    """('arap' | 'volume', svd node) when T = sum((S - 1)^2) / sum((prod(S, 1) - 1)^2) over the singular values S
    of a recorded torch.svd, else None."""
    if T.kind != "sum" or T.kids[0].kind != "sq":
        return None
    X = T.kids[0].kids[0]
    if X.kind != "off" or X.lo != -1.0:
        return None
    Y = X.kids[0]
    sv = _svd_of(Y)
    if sv is not None:
        return "arap", sv
    if Y.kind == "prod" and Y.k == 1:
        sv = _svd_of(Y.kids[0])
        if sv is not None:
            return "volume", sv
    return None


def energy_plan(n):
    """The loss node of an unchanged elasticity body as [(kind, weight, payload)], or None:
      ('energy', w, (term, svd node))   w * E_term from the singular values of J + I (one insr_elastic_energy
                                         launch for every such term: arap, volume)
      ('sq', w, plan)                    w * a sum / mean of squares of a linear residual (the positional
                                         constraints, kinematics): one term of the loss group
      ('eager', w, node)                 anything else, materialised as written
    The singular values must be those of the Jacobian jet of f(x) + x (jacobian(q, x), an eyeadd node)."""
    if _stale(n):
        return None
    terms = _lin_terms(n)
    out, svds = [], set()
    for w, T in terms:
        e = _energy_term(T)
        if e is not None:
            J = e[1].kids[0]
            if J.kind != "eyeadd" or J.meta is None:
                return None
            svds.add(id(e[1]))
            out.append(("energy", w, e))
            continue
        p = plan(T) if T.kind in ("sum", "mean") else None
        if p is not None and p[0] == "combo":
            out.append(("sq", w, p))
        else:
            out.append(("eager", w, T))
    if not any(k == "energy" for k, _, _ in out) or len(svds) != 1:
        return None
    return out


def _energy_loss(ep):
    """Evaluate an energy_plan: ONE insr_elastic_energy launch for the singular-value terms, ONE loss-group
    launch for the squared residuals, the rest eager; their sum."""
    from .losses import elastic_energy, mse_term, sq_losses
    parts = []
    order, ratios, svd = [], {}, None
    for kind, w, pay in ep:
        if kind == "energy":
            term, svd = pay
            if term in ratios:  # the same term twice: weights add (the kernel has one slot per term)
                ratios[term] += w
            else:
                order.append(term)
                ratios[term] = w
    Jn = svd.kids[0]
    mlp, f, x = Jn.meta
    Jraw = Jn.kids[0].real
    flush()
    n = f.shape[0]
    total, _ = elastic_energy(f, Jraw, x, f.detach(), f.detach(), n=n, dt=1.0, energy=order, ratios=ratios)
    parts.append(total)
    specs = []
    for kind, w, pay in ep:
        if kind == "sq":
            (a, b, c, d), (alpha, beta, gamma, delta), w2, red = pay[1], pay[2], pay[3], pay[4]
            specs.append(mse_term(a, b, c, d, alpha=alpha, beta=beta, gamma=gamma, delta=delta, reduction=red,
                                  weight=w * w2))
        elif kind == "eager":
            LOWERED["eager_losses"] += 1
            v = _eval(pay) if pay.real is None else pay.real
            parts.append(v * w if w != 1.0 else v)
    from . import _native as nat
    for i in range(0, len(specs), nat.LOSS_GROUP_MAX):
        parts.extend(sq_losses(*specs[i:i + nat.LOSS_GROUP_MAX]))
        LOWERED["groups"] += 1
    LOWERED["energies"] = LOWERED.get("energies", 0) + 1
    LOWERED["terms"] += len(order) + len(specs)
    res = parts[0]
    for v in parts[1:]:
        res = res + v
    return res


def lower_losses(loss_dict):
    """The loss dict a phase body returned inside lowering(), with every recognised Lazy loss computed by
    ONE fused loss-group launch (per LOSS_GROUP_MAX losses) and every other Lazy loss materialised."""
    if not isinstance(loss_dict, dict) or not any(isinstance(v, Lazy) for v in loss_dict.values()):
        return loss_dict
    flush()  # (the loop calls this after its deferred scope closed: nothing is queued any more)
    from . import _native as nat
    from .losses import sq_losses
    specs, slot, energies = [], {}, {}
    for k, v in loss_dict.items():
        if isinstance(v, Lazy):
            sp = _spec(v._insr_node)
            if sp is not None:
                slot[k] = len(specs)
                specs.append(sp)
            else:
                ep = energy_plan(v._insr_node)
                if ep is not None and all(
                        all(t is None or t.is_cuda for t in p[1]) for kind, _, p in ep if kind == "sq") and \
                        all(p[1].kids[0].kids[0].real.is_cuda for kind, _, p in ep if kind == "energy"):
                    energies[k] = ep
    outs = []
    for i in range(0, len(specs), nat.LOSS_GROUP_MAX):
        outs.extend(sq_losses(*specs[i:i + nat.LOSS_GROUP_MAX]))
        LOWERED["groups"] += 1
    LOWERED["terms"] += len(specs)
    res = {}
    for k, v in loss_dict.items():
        if k in slot:
            res[k] = outs[slot[k]]
        elif k in energies:
            res[k] = _energy_loss(energies[k])
        elif isinstance(v, Lazy):
            LOWERED["eager_losses"] += 1
            res[k] = materialize(v)
        else:
            res[k] = v
    return res
