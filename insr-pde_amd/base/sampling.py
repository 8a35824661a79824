"""Collocation samplers, drop-in for base/sampling.py:4-64 of the reference.

Same signatures (including `device=`) and distributions.  On the CPU the torch
RNG is consumed exactly as the reference does, so a seeded CPU generator yields
the reference's points bit for bit.  On a GPU device each sampler is ONE
insr_sample_boxes launch (the device Philox-4x32-10 stream, graph-capturable: the
kernel advances its own stream position, so a replayed graph draws fresh points
with no host-side generator update), instead of up to 13 launches for a pair of
boundary bands: same distributions, another stream -- parity tests pass explicit
sample tensors.
"""
import ctypes
import os

import torch

_AFFINE = {}  # (N, side-key, epsilon, device) -> (scale, shift) constant tensors

__all__ = ["sample_uniform", "sample_random", "sample_boundary", "sample_boundary2D_separate",
           "sample_boundary2D_pair", "sample_random_and_bands2D", "sample_boxes", "sample_boxes_into",
           "merge_samples"]


def sample_uniform(resolution, sdim=1, device="cpu", flatten=True):
    """Cell-centred grid (i + 0.5)/R * 2 - 1 per axis, 'ij' order (base/sampling.py:4-11)."""
    axis = torch.linspace(0.5, resolution - 0.5, resolution, device=device) / resolution * 2 - 1
    grid = torch.stack(torch.meshgrid(*([axis] * sdim), indexing='ij'), dim=-1)
    return grid.reshape(resolution ** sdim, sdim) if flatten else grid


def sample_random(N, sdim=1, device="cpu"):
    """N points uniform in [-1, 1)^sdim (base/sampling.py:14-18).  On the GPU: one
    insr_sample_boxes launch (the device Philox stream, advanced by the kernel itself -- inside a
    replayed hipGraph torch's generator would add a seed / offset fill and copy per replay); before
    that stream exists and while a capture runs, one uniform_ draw (== rand * 2 - 1)."""
    dev = torch.device(device)
    if dev.type == "cuda":
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        if N > 0 and 1 <= sdim <= 3 and (dev.index in _SAMPLER or not torch.cuda.is_current_stream_capturing()):
            return sample_boxes([(N, (-1.0,) * sdim, (1.0,) * sdim)], sdim, device=dev)
        return torch.empty(N, sdim, device=dev).uniform_(-1.0, 1.0)
    return torch.rand(N, sdim, device=device) * 2 - 1


def _fused_bands(n_per, faces, key, device):
    """len(faces) bands of n_per points on the GPU: ONE insr_sample_boxes launch (the device Philox
    stream of sample_random_and_bands2D), rows in face order; before that stream exists and a
    hipGraph capture is running, one rand draw + one fused multiply-add instead."""
    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    if n_per == 0:
        return torch.empty(0, len(faces[0]), device=dev)
    if dev.index in _SAMPLER or not torch.cuda.is_current_stream_capturing():
        return sample_boxes([(n_per, tuple(r[0] for r in f), tuple(r[1] for r in f)) for f in faces], len(faces[0]),
                            device=dev)
    k = (n_per, key, dev)
    if k not in _AFFINE:
        d = len(faces[0])
        lo = torch.tensor([[f[j][0] for j in range(d)] for f in faces], dtype=torch.float32)
        hi = torch.tensor([[f[j][1] for j in range(d)] for f in faces], dtype=torch.float32)
        _AFFINE[k] = ((hi - lo).repeat_interleave(n_per, 0).to(device), lo.repeat_interleave(n_per, 0).to(device))
    scale, shift = _AFFINE[k]
    u = torch.rand(scale.shape, device=device)
    return torch.addcmul(shift, u, scale)


def _band(n, ranges, device):
    """n points, coordinate k uniform in ranges[k] = (lo, hi)."""
    pts = torch.empty(n, len(ranges), device=device)
    for k, (lo, hi) in enumerate(ranges):
        pts[:, k] = torch.rand(n, device=device) * (hi - lo) + lo
    return pts


def sample_boundary(N, sdim, epsilon=1e-4, device='cpu'):
    """Random points in thin bands around the box faces (base/sampling.py:21-42)."""
    if sdim == 1:
        if torch.device(device).type == "cuda":  # both bands in one device Philox launch
            return _fused_bands(N // 2, [((-1 - epsilon, -1 + epsilon),), ((1 - epsilon, 1 + epsilon),)],
                                ("box1", epsilon), device)
        left = (torch.rand(N // 2, 1, device=device) * 2 - 1) * epsilon - 1.
        right = (torch.rand(N // 2, 1, device=device) * 2 - 1) * epsilon + 1.
        return torch.cat([left, right], dim=0)
    if sdim == 2:
        full, lo, hi = (-1, 1), (-1 - epsilon, -1 + epsilon), (1 - epsilon, 1 + epsilon)
        faces = [(full, lo), (full, hi), (lo, full), (hi, full)]
        if torch.device(device).type == "cuda":
            return _fused_bands(N // 4, faces, ("box2", epsilon), device)
        return torch.cat([_band(N // 4, f, device) for f in faces], dim=0)
    raise NotImplementedError


def sample_boundary2D_separate(N, side, epsilon=1e-4, device='cpu'):
    """Bands on the two x-faces ('horizontal') or the two y-faces ('vertical'),
    N//2 random points each (base/sampling.py:45-64)."""
    full, lo, hi = (-1, 1), (-1 - epsilon, -1 + epsilon), (1 - epsilon, 1 + epsilon)
    if side == 'horizontal':
        faces = [(lo, full), (hi, full)]
    elif side == 'vertical':
        faces = [(full, lo), (full, hi)]
    else:
        raise RuntimeError
    if torch.device(device).type == "cuda":
        return _fused_bands(N // 2, faces, (side, epsilon), device)
    return torch.cat([_band(N // 2, f, device) for f in faces], dim=0)


def sample_boundary2D_pair(N, epsilon=1e-4, device='cpu'):
    """torch.cat([sample_boundary2D_separate(N, 'horizontal'), sample_boundary2D_separate(N,
    'vertical')]) -- the x-face bands then the y-face bands, N//2 points per face -- as
    one draw (the fluid wall terms use both band pairs together, fluid/model.py:90-94)."""
    full, lo, hi = (-1, 1), (-1 - epsilon, -1 + epsilon), (1 - epsilon, 1 + epsilon)
    faces = [(lo, full), (hi, full), (full, lo), (full, hi)]
    if torch.device(device).type == "cuda":
        return _fused_bands(N // 2, faces, ("pair", epsilon), device)
    return torch.cat([_band(N // 2, f, device) for f in faces], dim=0)


def merge_samples(*parts):
    """One leaf sample tensor holding several point sets of ONE network (interior points,
    boundary bands, fixed points): the model evaluates the network once, so the HIP path
    runs one jet launch each way instead of one per set -- a band of a few hundred points
    would otherwise be a latency-bound launch of its own.  Row order = argument order."""
    return torch.cat([p.detach() for p in parts]).requires_grad_(True)


_SAMPLER = {}  # device index -> (Philox stream position on the device, key, torch seed, reseed epoch)


def sampler_seed(torch_seed, rank):
    """Philox key of the fused sampler: the device's torch seed with the data-parallel rank
    folded in (golden-ratio stride), so ranks seeded alike (identical weights need it) still
    draw independent collocation points."""
    return (int(torch_seed) + int(rank) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF


def _dp_rank():
    d = torch.distributed
    return d.get_rank() if (d.is_available() and d.is_initialized()) else 0


# Re-seed detection.  Every torch re-seed (torch.manual_seed / torch.cuda.manual_seed[_all], the same
# seed again included) restarts the fused sampler's stream, so seeded runs repeat their draws as the
# reference's torch samplers do.  The seeding functions are wrapped once (at import) to count
# re-seeds; nothing reads or writes torch's generator state (its offset and every other torch
# random stream stay untouched).  A seed CHANGE made any other way (a generator object's own
# manual_seed) is still seen through torch.cuda.initial_seed(); a same-seed re-seed through an
# unwrapped reference taken before `base` was imported is not.
_RESEED = [0]


def reseed_epoch():
    """Number of torch re-seeds seen so far (the fused and mesh samplers restart when it moves)."""
    return _RESEED[0]


def _wrap_seeder(mod, name):
    fn = getattr(mod, name, None)
    if fn is None or getattr(fn, "_insr_reseed_hook", False):
        return

    def seeded(*a, **k):
        out = fn(*a, **k)
        _RESEED[0] += 1
        return out
    seeded._insr_reseed_hook = True
    seeded.__doc__, seeded.__name__, seeded.__wrapped__ = fn.__doc__, fn.__name__, fn
    setattr(mod, name, seeded)


def _seeder_sites():
    import torch.cuda.random as cr
    import torch.random as tr
    return ((torch, ("manual_seed", "seed")), (tr, ("manual_seed", "seed")),
            (torch.cuda, ("manual_seed", "manual_seed_all", "seed", "seed_all")),
            (cr, ("manual_seed", "manual_seed_all", "seed", "seed_all")))


def install_reseed_hooks():
    """Wrap torch's seeding functions to count re-seeds (done once at import unless the environment sets
    INSR_NO_RESEED_HOOKS=1).  The wrappers call the original and add one to reseed_epoch(); each keeps the
    original as `__wrapped__`.  Idempotent."""
    for mod, names in _seeder_sites():
        for name in names:
            _wrap_seeder(mod, name)


def uninstall_reseed_hooks():
    """Put torch's own seeding functions back (undoes install_reseed_hooks; idempotent).  Without the hooks
    a same-seed re-seed no longer restarts the fused sampler's stream -- a seed CHANGE still does (the
    sampler compares torch.cuda.initial_seed())."""
    for mod, names in _seeder_sites():
        for name in names:
            fn = getattr(mod, name, None)
            if fn is not None and getattr(fn, "_insr_reseed_hook", False):
                setattr(mod, name, fn.__wrapped__)


if os.environ.get("INSR_NO_RESEED_HOOKS", "0") in ("", "0"):
    install_reseed_hooks()


def _sampler(dev):
    """Per-device Philox state of the fused sampler (insr_sample_boxes): (stream position on
    the device, key).  The key is the device's torch seed with the distributed rank folded in.
    A torch re-seed (reseed_epoch) or a changed seed restarts the stream.  Created / restarted on
    an eager call -- phase loops always run iteration 0 eagerly before capturing (a capture keeps
    the current stream)."""
    from . import _native as nat
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    ent = _SAMPLER.get(key)
    if torch.cuda.is_current_stream_capturing():
        if ent is None:
            raise RuntimeError("sampler state must be created before graph capture (run one eager call)")
        return ent[:2]
    torch.cuda.init()
    seed = torch.cuda.default_generators[key].initial_seed()  # host-side state, no device sync
    epoch = _RESEED[0]
    if ent is None or ent[2] != seed or ent[3] != epoch:
        state = ent[0].zero_() if ent is not None else torch.zeros(nat.lib().insr_sampler_state_bytes() // 8,
                                                                    device=dev, dtype=torch.int64)
        ent = _SAMPLER[key] = (state, sampler_seed(seed, _dp_rank()), seed, epoch)
    return ent[:2]


def sample_random_and_bands2D(N, n_band, epsilon=1e-4, device="cuda", merged=False):
    """(sample_random(N, 2), sample_boundary2D_pair(n_band)) -- the interior batch and the
    four wall bands of one fluid phase iteration (fluid/model.py:74,90-91,105,116-117) --
    drawn in ONE device launch (insr_sample_boxes: 3 launches -> 1).  Same distributions;
    the device stream is Philox-4x32-10, not torch's (GPU only: the CPU samplers above
    reproduce the reference bit for bit).  merged=True returns the one (N + 2 (n_band // 2) * 2, 2)
    buffer [interior; bands] instead (both are consecutive rows of it)."""
    from . import _native as nat
    dev = torch.device(device)
    if dev.type != "cuda":
        raise nat.NativeUnavailable("sample_random_and_bands2D draws on the GPU only")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    h = n_band // 2
    rows = N + 4 * h
    ahead = draw_ahead.active
    if merged and ahead is not None:
        buf = ahead.take((N, h, float(epsilon), dev.index), rows, dev, lambda out, reps: _draw_fluid(
            out, N, h, epsilon, dev, reps))
        if buf is not None:
            return buf
    buf = torch.empty(rows, 2, device=dev)  # [interior; bands]: one jet can take both (merged=True)
    _draw_fluid(buf, N, h, epsilon, dev, 1)
    if merged:
        return buf
    return buf[:N], buf[N:]


def _draw_fluid(out, N, h, epsilon, dev, reps):
    """The interior box and the four wall bands of sample_random_and_bands2D into `out` -- (reps, N + 4 h,
    2) for reps consecutive iterations, one launch either way (insr_sample_boxes_rep)."""
    from . import _native as nat
    state, seed = _sampler(dev)
    full, lo, hi = (-1.0, 1.0), (-1 - epsilon, -1 + epsilon), (1 - epsilon, 1 + epsilon)
    faces = [(lo, full), (hi, full), (full, lo), (full, hi)]  # sample_boundary2D_pair's order
    f3 = nat._F * 3
    base = out.data_ptr()
    boxes = (nat.Box * 5)()
    boxes[0] = nat.Box(base, N, f3(-1.0, -1.0, 0.0), f3(1.0, 1.0, 0.0))
    for k, (rx, ry) in enumerate(faces):  # face k: rows [N + k h, N + (k + 1) h), 8 bytes a row
        boxes[1 + k] = nat.Box(base + 8 * (N + h * k), h, f3(rx[0], ry[0], 0.0), f3(rx[1], ry[1], 0.0))
    strides = (ctypes.c_long * 5)(*([2 * (N + 4 * h)] * 5))
    nat.check(nat.lib().insr_sample_boxes_rep(boxes, 5, 2, reps, strides, seed, nat.ptr(state), nat.stream_of(dev)),
              "insr_sample_boxes_rep")


class draw_ahead:
    """`with draw_ahead(U):` around U consecutive iterations that hold no host read between them (the
    U-iteration hipGraph of base/_loop.py PhaseLoop.run_group): the first merged fluid draw
    (sample_random_and_bands2D(merged=True)) draws the buffers of all U iterations in ONE launch
    (insr_sample_boxes_rep) and the next U - 1 calls of the same shape take theirs -- 4 sampler launches
    per phase and replay -> 1.  Independent uniform draws made earlier: which Philox numbers an
    iteration gets changes, not their distribution (the points never depend on the network).  A call
    of another shape, or a (U + 1)-th call, draws on its own."""

    active = None

    def __init__(self, reps):
        self.reps = max(1, int(reps))

    def __enter__(self):
        self.saved, self.store, self.key, self.pos = draw_ahead.active, None, None, 0
        self.frozen = {}  # frozen_ahead results of this group, by name
        draw_ahead.active = self if self.reps > 1 else None
        return self

    def __exit__(self, *exc):
        draw_ahead.active = self.saved
        return False

    def group_of(self, buf):
        """(store, k) when `buf` is (a leading-row view of) iteration k's buffer of this group's draw, else None."""
        st = self.store
        if st is None or buf.dim() != 2 or buf.shape[1] != st.shape[2] or buf.dtype != st.dtype:
            return None
        off = buf.data_ptr() - st.data_ptr()
        rb = st.shape[1] * st.shape[2] * st.element_size()
        if off < 0 or off % rb or off // rb >= st.shape[0] or not buf.is_contiguous():
            return None
        return st, off // rb

    def take(self, key, rows, dev, draw):
        if self.store is None:
            self.store = torch.empty(self.reps, rows, 2, device=dev)
            self.key = key
            draw(self.store, self.reps)
        if key != self.key or self.pos >= self.reps:
            return None
        buf = self.store[self.pos]
        self.pos += 1
        return buf


def frozen_ahead(name, x, fn, stream=None, pipe=False):
    """Work on FROZEN networks for the iterations of a draw_ahead group, ahead of the iterations themselves.
    `x` is an iteration's merged draw (or its leading rows) from the group's store; `fn(X)` evaluates the
    frozen networks at points X (no autograd) and returns a tuple of tensors whose rows follow X's.  Exact for
    networks no iteration of the group trains (the previous-step field, the other field of a phase): their
    outputs at the group's points do not depend on any iteration's update.  Returns iteration k's outputs
    (rows [:x.shape[0]]), or None outside a group (U = 1, eager iterations): the caller computes its own.

      batched (pipe=False): on the group's first call of `name` fn runs ONCE on all U buffers (U x rows points:
          one launch per jet instead of U latency-bound shares of a mixed launch; the band rows and the other
          iterations' rows are computed too).  stream: run it on this side stream (forked after the group's
          draw), overlapping the first iteration's trained-network forward.
      pipelined (pipe=True, stream required): fn runs per iteration on its own points, on the side stream, one
          iteration AHEAD: frozen_join(name) (called by the body after its trained-network forward) waits for
          iteration k's outputs and issues iteration k + 1's, which then run under iteration k's reverse jets,
          gradient all-reduce and Adam step -- the latency-bound tail of a backward launch and the collective
          leave most CUs idle.
    The caller calls frozen_join(name) before the first read of the outputs whenever a stream is given (a group
    runs under hipGraph capture: the forks and joins become graph edges)."""
    da = draw_ahead.active
    if da is None:
        return None
    hit = da.group_of(x)
    if hit is None:
        return None
    st, k = hit
    U, rows, n = st.shape[0], st.shape[1], x.shape[0]
    if pipe and stream is not None:
        ent = da.frozen.get(name)
        if ent is None:  # iteration 0: its own outputs, on the side stream, forked here
            ent = da.frozen[name] = {"fn": fn, "stream": stream, "n": n, "outs": {}, "ev": {}}
            _frozen_issue(da, name, 0)
        if k not in ent["outs"]:
            raise RuntimeError(f"frozen_ahead({name!r}): iteration {k}'s outputs were not issued (frozen_join "
                               "must follow every iteration's call)")
        ent["cur"] = k
        return ent["outs"][k]
    outs = da.frozen.get(name)
    if outs is None:
        X = st.view(-1, st.shape[2]).detach().requires_grad_(True)
        if stream is not None:
            stream.wait_stream(torch.cuda.current_stream(st.device))
            with torch.cuda.stream(stream), torch.no_grad():
                outs = tuple(fn(X))
            ev = torch.cuda.Event()
            ev.record(stream)
            da.frozen[name + "/join"] = ev
        else:
            with torch.no_grad():
                outs = tuple(fn(X))
        da.frozen[name] = outs
    return tuple(o.view(U, rows, *o.shape[1:])[k, :n] for o in outs)


def _frozen_issue(da, name, k):
    """Pipelined frozen_ahead: iteration k's frozen outputs on the side stream, forked from the current stream
    now (so they run after everything issued so far, beside everything issued later)."""
    ent = da.frozen[name]
    st, side = da.store, ent["stream"]
    X = st[k, :ent["n"]].detach().requires_grad_(True)
    side.wait_stream(torch.cuda.current_stream(st.device))
    with torch.cuda.stream(side), torch.no_grad():
        ent["outs"][k] = tuple(ent["fn"](X))
    ev = torch.cuda.Event()
    ev.record(side)
    ent["ev"][k] = ev


def frozen_join(name):
    """Before the first read of frozen_ahead(name, ...)'s outputs when they run on a side stream: the current
    stream waits for them (batched: once per group); pipelined: waits for iteration k's and issues k + 1's."""
    da = draw_ahead.active
    if da is None:
        return
    ent = da.frozen.get(name)
    if isinstance(ent, dict):  # pipelined
        k = ent.get("cur")
        ev = ent["ev"].pop(k, None)
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        if k is not None and k + 1 < da.store.shape[0] and k + 1 not in ent["outs"]:
            _frozen_issue(da, name, k + 1)
        return
    ev = da.frozen.pop(name + "/join", None)
    if ev is not None:
        torch.cuda.current_stream().wait_event(ev)


class draw_plan:
    """`with draw_plan(owner):` around one iteration of a phase body (base/_loop.py).  The
    sampler calls of an iteration (sample_random, the band samplers) are recorded on `owner`;
    on the next iteration the FIRST call draws every request the previous iteration made, in
    ONE insr_sample_boxes launch (each request its own output tensor), and the later calls
    take their pre-drawn tensors as long as they ask for the same (dim, boxes) in the same
    order -- the reference's phase bodies call the samplers 3 times per iteration
    (fluid/model.py:75,94-95): 3 launches -> 1.  Independent uniform draws, so drawing them
    early changes which Philox numbers a request gets, not its distribution.  A request that
    departs from the plan draws on its own (and ends the plan for that iteration)."""

    active = None  # the innermost scope's state

    def __init__(self, owner):
        self.owner = owner

    def __enter__(self):
        self.saved = draw_plan.active
        self.prev = self.owner.__dict__.get("_insr_draw_plan")
        self.rec, self.pos, self.ready = [], 0, None
        draw_plan.active = self
        return self

    def __exit__(self, *exc):
        draw_plan.active = self.saved
        if exc[0] is None:
            self.owner._insr_draw_plan = self.rec
        return False

    def take(self, key, dev):
        """The pre-drawn tensor for request `key` = (dim, boxes, device index), or None (draw it now)."""
        from . import _native as nat
        pos, self.pos = self.pos, self.pos + 1
        self.rec.append(key)
        plan = self.prev
        if not plan or pos >= len(plan) or plan[pos] != key:
            self.prev = None  # off the plan: every later request draws on its own
            return None
        if pos == 0:
            if len(plan) < 2 or len({(k[0], k[2]) for k in plan}) != 1 or sum(len(k[1]) for k in plan) > nat.MAX_BOXES:
                self.prev = None
                return None
            outs = [torch.empty(sum(int(b[0]) for b in k[1]), k[0], device=dev) for k in plan]
            _launch_boxes([(o, k[1]) for o, k in zip(outs, plan)], key[0], dev)
            self.ready = outs
        return self.ready[pos] if self.ready is not None else None


def _launch_boxes(reqs, dim, dev):
    """One insr_sample_boxes launch: reqs = [(out tensor (sum n, dim), boxes), ...]; the boxes of
    a request fill its tensor's rows in order."""
    from . import _native as nat
    state, seed = _sampler(dev)
    f3 = nat._F * 3
    nbox = sum(len(b) for _, b in reqs)
    arr = (nat.Box * nbox)()
    k, pad = 0, [0.0] * (3 - dim)
    for out, boxes in reqs:
        row = 0
        for n, lo, hi in boxes:
            arr[k] = nat.Box(out.data_ptr() + 4 * dim * row, int(n), f3(*(list(lo) + pad)), f3(*(list(hi) + pad)))
            row, k = row + int(n), k + 1
    nat.check(nat.lib().insr_sample_boxes(arr, nbox, dim, seed, nat.ptr(state), nat.stream_of(dev)),
              "insr_sample_boxes")


def sample_boxes(boxes, dim, device="cuda"):
    """ONE device launch drawing every box of an iteration into one (sum n, dim) tensor,
    rows in box order: boxes = [(n, lo[dim], hi[dim]), ...], coordinate j of box k uniform
    in [lo[j], hi[j]) (insr_sample_boxes, the device stream of sample_random_and_bands2D).
    Inside a phase loop's draw_plan the tensor may have been drawn by the iteration's first
    sampler call (same distribution)."""
    from . import _native as nat
    dev = torch.device(device)
    if dev.type != "cuda":
        raise nat.NativeUnavailable("sample_boxes draws on the GPU only")
    if not 1 <= len(boxes) <= nat.MAX_BOXES:
        raise ValueError(f"sample_boxes: 1..{nat.MAX_BOXES} boxes")
    plan = draw_plan.active
    if plan is not None:
        key = (dim, tuple((int(n), tuple(float(v) for v in lo), tuple(float(v) for v in hi)) for n, lo, hi in boxes),
               dev.index)
        out = plan.take(key, dev)
        if out is not None:
            return out
    out = torch.empty(sum(int(b[0]) for b in boxes), dim, device=dev)
    _launch_boxes([(out, boxes)], dim, dev)
    return out


def sample_boxes_into(buf, boxes):
    """sample_boxes, written in place into row ranges of an existing (R, dim) fp32 device buffer
    (rows the boxes do not cover keep their contents -- e.g. constant grid rows of a persistent
    batch): boxes = [(row0, n, lo[dim], hi[dim]), ...], ONE launch (insr_sample_boxes)."""
    from . import _native as nat
    if not buf.is_cuda or buf.dtype != torch.float32 or not buf.is_contiguous() or buf.dim() != 2:
        raise nat.NativeUnavailable("sample_boxes_into: a contiguous (R, dim) fp32 GPU buffer")
    dim = buf.shape[1]
    if not 1 <= len(boxes) <= nat.MAX_BOXES:
        raise ValueError(f"sample_boxes_into: 1..{nat.MAX_BOXES} boxes")
    state, seed = _sampler(buf.device)
    f3 = nat._F * 3
    arr = (nat.Box * len(boxes))()
    for k, (row0, n, lo, hi) in enumerate(boxes):
        if row0 < 0 or row0 + n > buf.shape[0]:
            raise ValueError(f"sample_boxes_into: rows [{row0}, {row0 + n}) outside {buf.shape[0]}")
        pad = [0.0] * (3 - dim)
        arr[k] = nat.Box(buf.data_ptr() + 4 * dim * int(row0), int(n), f3(*(list(lo) + pad)), f3(*(list(hi) + pad)))
    nat.check(nat.lib().insr_sample_boxes(arr, len(boxes), dim, seed, nat.ptr(state), nat.stream_of(buf.device)),
              "insr_sample_boxes")
    return buf
