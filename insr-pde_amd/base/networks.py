"""SIREN field network, drop-in for base/networks.py:12-93 of the reference.

`get_network(cfg, in, out)` / `MLP(...)` keep the reference's module tree
(`.net` = Sequential[Linear, Sine, (Linear, Sine) x L, Linear]), its init RNG
order (so a torch seed gives the reference's weights bit for bit), and its
state_dict keys (net.0.weight ... net.{2L+2}.bias), so checkpoints and
`load_state_dict` interoperate with the reference unchanged.

What differs is storage and execution:
  * all parameters are views into ONE flat fp32 buffer in state_dict order --
    the layout the HIP kernels and the fused Adam consume directly (see
    include/insr_siren.h); `.grad` tensors are views into one flat gradient;
  * any hidden width W <= 256 is served: the kernels are compiled for widths
    32 / 64 / 128 / 256, and a net of another width (the paper scripts use 20, 66
    and 68: scripts/advect1D.sh:5, elasticity3Dbunny.sh:4, elasticity2Dstretch.sh:4)
    is stored ZERO-PADDED to the next compiled width Wp: the flat buffer has the
    layout of an SIREN of width Wp, and each parameter is the (W-row, W-column)
    corner view of its padded block.  Padding is exact: a padded neuron has zero
    weights and bias, so z = 0, sin(0) = 0 and every derivative stream is 0; its
    outgoing weights are 0, so it adds nothing downstream; every padded gradient
    entry is exactly 0, so Adam leaves the padding at 0;
  * `forward` runs the fused HIP jet kernel (value stream) instead of the
    aten addmm/sin chain, and tags its output with its provenance so the
    diff ops (base/diff_ops.py) can dispatch derivative jets.
"""
import copy
import math
import weakref

import numpy as np
import torch
import torch.nn as nn

from . import _jet
from . import lower

OMEGA = 30.0
KERNEL_WIDTHS = (32, 64, 128, 256)  # hidden widths the HIP jets are compiled for


def get_network(cfg, in_features, out_features):
    """base/networks.py:12-17: cfg.network 'siren' -> MLP(..., nonlinearity=cfg.nonlinearity) (a relu /
    elu one, or a width above 256, is the reference's plain torch network: TorchMLP).
    cfg.insr_precision (optional, default None = the library default, fp32-accurate split-bf16)
    selects the matrix-core precision of the net's jets: 'fp32', 'bf16x6', 'bf16x3' or 'bf16'."""
    if cfg.network == 'siren':
        return MLP(in_features, out_features, cfg.num_hidden_layers, cfg.hidden_features,
                   nonlinearity=cfg.nonlinearity, precision=getattr(cfg, "insr_precision", None))
    raise NotImplementedError(cfg.network)


class Sine(nn.Module):
    """sin(30 x) (base/networks.py:21-27).  Only used when `.net` is called directly;
    MLP.forward never runs it (the HIP kernel fuses it)."""

    def forward(self, input):
        return torch.sin(OMEGA * input)


def _sine_init(m):
    # base/networks.py:80-85
    with torch.no_grad():
        if hasattr(m, 'weight'):
            fan_in = m.weight.size(-1)
            b = np.sqrt(6 / fan_in) / OMEGA
            m.weight.uniform_(-b, b)


def _first_layer_sine_init(m):
    # base/networks.py:88-93
    with torch.no_grad():
        if hasattr(m, 'weight'):
            fan_in = m.weight.size(-1)
            m.weight.uniform_(-1 / fan_in, 1 / fan_in)


def kernel_width(width):
    """The compiled width a net of hidden width `width` runs at (zero-padded up to it)."""
    for w in KERNEL_WIDTHS:
        if width <= w:
            return w
    raise NotImplementedError(f"hidden width {width} > {KERNEL_WIDTHS[-1]}: no HIP kernel")


# 'mixed' (BASELINE.json configs[4] "mixed fp32/bf16 MFMA"): the forward / backward precision pair
# measured fastest within 1e-2 normwise on every op and parameter gradient (profiles/r03/prec_*).
MIXED_PRECISION = "bf16x3/bf16"


def _parse_precision(precision):
    """None, a name of _native.PRECISIONS, 'fwd/bwd' names or 'mixed' -> (fwd, bwd) ints or None."""
    from ._native import PRECISIONS
    if precision is None:
        return None
    name = MIXED_PRECISION if precision == "mixed" else precision
    parts = name.split("/")
    if len(parts) == 1:
        parts = parts * 2
    if len(parts) != 2 or any(p not in PRECISIONS for p in parts):
        raise ValueError(f"precision {precision!r}: one of {sorted(PRECISIONS)}, 'fwd/bwd' of those, 'mixed' or None")
    return PRECISIONS[parts[0]], PRECISIONS[parts[1]]


# flat storage address -> the MLP that owns it (load_state_dict's one-copy snapshot)
_FLAT_OWNERS = weakref.WeakValueDictionary()


def _kaiming_relu_init(m):
    # base/networks.py:74-77 (relu networks)
    if type(m) is nn.Linear:
        nn.init.kaiming_normal_(m.weight, a=0.0, nonlinearity='relu', mode='fan_in')


def _elu_init(m):
    # base/networks.py:96-100 (elu networks)
    if type(m) is nn.Linear:
        nn.init.normal_(m.weight, std=math.sqrt(1.5505188080679277) / math.sqrt(m.weight.size(-1)))


def hip_served(nonlinearity, outermost_linear, hidden_features):
    """Whether the HIP jets serve this network: a SIREN ('sine') with a linear output layer and a hidden
    width the kernels are compiled for (<= 256, zero-padded up to 32 / 64 / 128 / 256)."""
    return nonlinearity == 'sine' and bool(outermost_linear) and hidden_features <= KERNEL_WIDTHS[-1]


class TorchMLP(nn.Module):
    """The reference's MLP (base/networks.py:30-71) as plain torch modules on the device, for the
    configurations the HIP jets do not serve -- relu / elu networks, outermost_linear=False, SIRENs
    wider than 256 -- none of which the INSR-PDE models build (they all use get_network's SIREN).  Same
    module tree, init order (a seed gives the reference's weights bit for bit) and state_dict keys;
    its derivatives take the reference's autograd route in base/diff_ops.py.  Off the hot path: a
    warning says so once per configuration."""

    _warned = set()

    def __init__(self, in_features, out_features, num_hidden_layers, hidden_features,
                 outermost_linear=True, nonlinearity='relu', weight_init=None):
        super().__init__()
        acts = {'sine': (Sine, _sine_init, _first_layer_sine_init), 'relu': (lambda: nn.ReLU(inplace=True),
                                                                             _kaiming_relu_init, None),
                'elu': (lambda: nn.ELU(inplace=True), _elu_init, None)}
        if nonlinearity not in acts:
            raise KeyError(nonlinearity)
        make, init, first = acts[nonlinearity]
        act = make()  # one module shared by every layer, as the reference's
        self.in_features, self.out_features = in_features, out_features
        self.num_hidden_layers, self.hidden_features = num_hidden_layers, hidden_features
        self.first_layer_init = None
        layers = [nn.Linear(in_features, hidden_features), act]
        for _ in range(num_hidden_layers):
            layers += [nn.Linear(hidden_features, hidden_features), act]
        layers.append(nn.Linear(hidden_features, out_features))
        if not outermost_linear:
            layers.append(act)
        self.net = nn.Sequential(*layers)
        self.weight_init = weight_init if weight_init is not None else init
        if self.weight_init is not None:
            self.net.apply(self.weight_init)
        if first is not None:
            self.net[0].apply(first)
        key = (nonlinearity, bool(outermost_linear), hidden_features > KERNEL_WIDTHS[-1])
        if key not in TorchMLP._warned:
            TorchMLP._warned.add(key)
            import warnings
            warnings.warn(f"MLP({nonlinearity}, outermost_linear={outermost_linear}, width {hidden_features}): no "
                          "HIP jet serves it; running plain torch ops (off the INSR-PDE hot path)", stacklevel=3)

    @lower.api
    def forward(self, coords, weights=None):
        out = self.net(coords)
        return out * weights if weights is not None else out


class _MLPArgs:
    """MLP's constructor arguments by name (the signature of MLP.__init__), for __new__'s dispatch."""

    def __init__(self, in_features, out_features, num_hidden_layers, hidden_features,
                 outermost_linear=True, nonlinearity='relu', weight_init=None, precision=None):
        self.in_features, self.out_features = in_features, out_features
        self.num_hidden_layers, self.hidden_features = num_hidden_layers, hidden_features
        self.outermost_linear, self.nonlinearity, self.weight_init = outermost_linear, nonlinearity, weight_init


class MLP(nn.Module):
    """SIREN MLP with flat parameter storage and a HIP forward (base/networks.py:30-71).  A
    configuration the kernels do not serve (hip_served) is built as TorchMLP instead."""

    def __new__(cls, *args, **kwargs):
        # copy.deepcopy / pickle rebuild through cls.__new__(cls) with no arguments: plain allocation then
        if cls is MLP and (args or kwargs):
            a = _MLPArgs(*args, **kwargs)
            if not hip_served(a.nonlinearity, a.outermost_linear, a.hidden_features):
                return TorchMLP(a.in_features, a.out_features, a.num_hidden_layers, a.hidden_features,
                                outermost_linear=a.outermost_linear, nonlinearity=a.nonlinearity,
                                weight_init=a.weight_init)
        return super().__new__(cls)

    def __init__(self, in_features, out_features, num_hidden_layers, hidden_features,
                 outermost_linear=True, nonlinearity='relu', weight_init=None, precision=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.num_hidden_layers, self.hidden_features = num_hidden_layers, hidden_features
        self.kernel_width = kernel_width(hidden_features)
        self.set_precision(precision)
        layers = [nn.Linear(in_features, hidden_features), Sine()]
        for _ in range(num_hidden_layers):
            layers += [nn.Linear(hidden_features, hidden_features), Sine()]
        layers.append(nn.Linear(hidden_features, out_features))
        self.net = nn.Sequential(*layers)
        self.weight_init = weight_init if weight_init is not None else _sine_init
        self.net.apply(self.weight_init)
        self.net[0].apply(_first_layer_sine_init)
        self.first_layer_init = None
        self._flat = None
        self._flat_grad = None
        self._wsplit_stamp = None
        self._repack()
        self.register_load_state_dict_post_hook(lambda m, keys: m.refresh_wsplit())

    # ---- matrix-core precision ------------------------------------------------
    def set_precision(self, precision):
        """None (the library default: fp32-accurate split-bf16), one of 'fp32', 'bf16x6', 'bf16x3',
        'bf16' for every jet of this network (include/insr_siren.h INSR_PREC_*), 'fwd/bwd' with one
        name per direction (e.g. 'bf16x3/bf16'), or 'mixed' (= MIXED_PRECISION: the fastest
        forward/backward pair measured within 1e-2 normwise, tools/prec_errors.py)."""
        self._prec_pair = _parse_precision(precision)
        self.precision = precision

    def call_mode(self, mode):
        """The jet `mode` argument of this network's library calls (precision bits added; the
        flat buffer carries the pre-split weight planes: INSR_MODE_WSPLIT)."""
        from ._native import _PREC_BITS, MODE_WSPLIT, jet_bprec, jet_prec, scope_bits
        mode |= MODE_WSPLIT | scope_bits()  # + the caller's knob scope (_native.knobs)
        if self._prec_pair is None:
            return mode
        pf, pb = self._prec_pair
        return (mode & ~_PREC_BITS) | jet_prec(pf) | (jet_bprec(pb) if pb != pf else 0)

    # ---- pre-split weight planes (include/insr_siren.h insr_siren_wsplit) -----------
    # The flat storage is [parameters | pad to 16 B | planes]: every hidden weight split in three
    # bf16 terms in the matrix-core fragment order (forward W rows, backward W^T rows), so the
    # split-bf16 kernels read fragments instead of re-splitting W in every block.  The planes
    # are derived data: rewritten after every parameter change -- by FusedAdam.step (captured
    # with it in a hipGraph), after load_state_dict, and before a jet whenever the parameters'
    # version counters moved (any torch in-place write).
    def wsplit_offset(self):
        return (self.param_count + 3) & ~3

    def wsplit_floats(self):
        # bf16 x 3 + fp16 x 2 planes, both orientations each, then the status quad
        # (include/insr_siren.h insr_siren_wsplit_floats; tests/test_capi.py pins the two together)
        return 5 * self.num_hidden_layers * self.kernel_width ** 2 + 4

    def plist(self):
        """list(self.parameters()) without the module-tree walk (the checks before every jet and
        snapshot read it): the (module, name) slots holding parameters are found once, the
        parameters re-read from them on every call (a replaced Parameter is seen)."""
        slots = self.__dict__.get("_insr_pslots")
        if slots is None:
            slots, seen = [], set()
            for mname, m in self.named_modules():
                for pname, q in m._parameters.items():
                    if q is not None and id(q) not in seen:
                        seen.add(id(q))
                        slots.append((m, pname, f"{mname}.{pname}" if mname else pname))
            self.__dict__["_insr_pslots"] = slots
        return [m._parameters[n] for m, n, _ in slots]

    def _param_names(self):
        self.plist()
        return [k for *_, k in self.__dict__["_insr_pslots"]]

    def _param_versions(self):
        return (self._flat.data_ptr(), self._flat._version) + tuple(p._version for p in self.plist())

    def refresh_wsplit(self, stream=None):
        """Rewrite the planes from the parameters now (one launch on `stream` / the current one)."""
        if self._flat is None or not self._flat.is_cuda or self.num_hidden_layers == 0:
            return
        from . import _native as nat
        W, L = self.kernel_width, self.num_hidden_layers
        st = stream.cuda_stream if stream is not None else nat.stream_of(self._flat.device)
        nat.check(nat.lib().insr_siren_wsplit(nat.ptr(self._flat), self.in_features, self.out_features, L, W, st),
                  "insr_siren_wsplit")
        self._wsplit_stamp = self._param_versions()

    def uses_f16_planes(self):
        """Whether this network's jets read the fp16 weight planes: an f16x3 forward (the default) or a
        bf16x6-contract backward with fp16 products (the default INSR_JET_BWD_F16 mask)."""
        from ._native import PREC_BF16X6, PREC_F16X3, bwd_f16_mask, scope_bits
        if self._prec_pair is None:
            bits = scope_bits()
            pf = ((bits >> 4) & 0xF) - 1
            return pf < 0 or pf == PREC_F16X3 or bwd_f16_mask() != 0
        pf, pb = self._prec_pair
        return pf == PREC_F16X3 or (pb in (PREC_BF16X6, PREC_F16X3) and bwd_f16_mask() != 0)

    def check_weight_planes(self):
        """Host sync point (the training loop's loss reads): raise NativeError when a hidden weight left
        the fp16 planes' range (|w| >= 255, include/insr_siren.h insr_siren_wsplit_status) while this
        network's jets read those planes -- the f16x3 products would not be the network's.  Remedy:
        MLP(precision='bf16x6') with INSR_JET_BWD_F16(0) (fp32's range everywhere)."""
        if self._flat is None or not self._flat.is_cuda or self.num_hidden_layers == 0 or not self.uses_f16_planes():
            return
        from . import _native as nat
        rc = nat.lib().insr_siren_wsplit_status(nat.ptr(self._flat), self.in_features, self.out_features,
                                                self.num_hidden_layers, self.kernel_width,
                                                nat.stream_of(self._flat.device))
        if rc == nat.ERANGE:
            raise nat.NativeError("a hidden weight reached |w| >= 255: outside the fp16 weight planes' range "
                                  "(f16x3 products); run this network at precision='bf16x6' with bwd_f16=0")
        nat.check(rc, "insr_siren_wsplit_status")

    def _status_word(self):
        """The fp16 planes' range status quad's first word (a view into the flat storage, as int32), or
        None when this network's jets do not read the fp16 planes (insr_siren_wsplit_status's word)."""
        if self._flat is None or not self._flat.is_cuda or self.num_hidden_layers == 0 or not self.uses_f16_planes():
            return None
        off = self.wsplit_offset() + 5 * self.num_hidden_layers * self.kernel_width ** 2
        return self._store[off:off + 1].view(torch.int32)

    @staticmethod
    def check_weight_planes_all(nets):
        """check_weight_planes of several networks with ONE device-to-host read of their status words
        (the training loop's sync points: one small copy instead of a stream sync + copy per network)."""
        words = [(n, w) for n in nets if isinstance(n, MLP) for w in (n._status_word(),) if w is not None]
        if not words:
            return
        vals = torch.cat([w for _, w in words]).cpu()
        for (net, _), v in zip(words, vals.tolist()):
            if v:
                from . import _native as nat
                raise nat.NativeError("a hidden weight reached |w| >= 255: outside the fp16 weight planes' range "
                                      "(f16x3 products); run this network at precision='bf16x6' with bwd_f16=0")

    def mark_wsplit_current(self):
        """The planes were rewritten with the parameters (insr_adam_step_nets)."""
        self._wsplit_stamp = self._param_versions()

    def ensure_wsplit(self):
        """Before a jet: refresh the planes if the parameters changed behind our back."""
        if self._wsplit_stamp != self._param_versions():
            self.refresh_wsplit()

    # ---- flat storage ------------------------------------------------------
    @property
    def param_count(self):
        """Floats of the flat buffer (= the parameter count, plus the zero padding of a
        net whose width is not a compiled one)."""
        W, L, din, dout = self.kernel_width, self.num_hidden_layers, self.in_features, self.out_features
        return W * din + W + L * (W * W + W) + dout * W + dout

    def flat_params(self):
        return self._flat

    def _layout(self):
        """(offset, padded shape, corner) of every parameter in the flat buffer, in
        parameters() order: Linear weights are (out, in) row-major blocks of the padded
        width, biases padded vectors; `corner` = the parameter's own (rows, cols)."""
        W, din, dout = self.kernel_width, self.in_features, self.out_features
        out, off = [], 0
        for i, p in enumerate(self.plist()):
            layer = i // 2
            rows = W if layer <= self.num_hidden_layers else dout
            cols = din if layer == 0 else W
            shape = (rows, cols) if p.dim() == 2 else (rows,)
            out.append((off, shape, tuple(p.shape)))
            off += int(np.prod(shape))
        return out

    def _view(self, buf, entry):
        off, shape, corner = entry
        block = buf[off:off + int(np.prod(shape))].view(*shape)
        return block[tuple(slice(0, c) for c in corner)]

    def _repack(self):
        """Move every parameter into one flat (zero-padded) buffer (Parameter identity kept)."""
        params = self.plist()
        if not params:
            return
        dev, dt = params[0].device, params[0].dtype
        lay = self._layout()
        store = torch.zeros(self.wsplit_offset() + self.wsplit_floats(), device=dev, dtype=dt)
        flat = store[:self.param_count]  # parameters; the pre-split weight planes follow
        grads_present = any(p.grad is not None for p in params)
        gflat = torch.zeros_like(flat) if grads_present else None
        for p, e in zip(params, lay):
            view = self._view(flat, e)
            view.copy_(p.data)
            p.data = view
            if gflat is not None:
                gv = self._view(gflat, e)
                if p.grad is not None:
                    gv.copy_(p.grad)
                p.grad = gv
        self._flat = flat
        self._store = store
        self._flat_grad = gflat
        self._wsplit_stamp = None
        _FLAT_OWNERS[flat.data_ptr()] = self

    def __deepcopy__(self, memo):
        """nn.Module's deep copy (Parameters cloned one by one), then the copy's parameters moved into
        a flat buffer of its own, so the copy is a packed MLP like the original (a model file keeping a
        previous-step copy of its network with copy.deepcopy)."""
        cls = type(self)
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            if k in ("_flat", "_store", "_flat_grad"):  # rebuilt by _repack below
                continue
            new.__dict__[k] = copy.deepcopy(v, memo)
        new._flat = new._store = new._flat_grad = None
        new._repack()
        if new._flat.is_cuda:
            new.refresh_wsplit()
        return new

    # ---- snapshots: prev = net.state_dict() ----------------------------------------
    def _snapshot_source(self, state_dict):
        """The MLP whose live parameters `state_dict` holds (net.state_dict() of a packed net of
        this geometry with current weight planes), else None."""
        keys = list(state_dict.keys()) if hasattr(state_dict, "keys") else None
        own = self._param_names()
        if keys != own or self._flat is None or not all(torch.is_tensor(v) for v in state_dict.values()):
            return None
        src = _FLAT_OWNERS.get(state_dict[own[0]].data_ptr())
        geo = ("in_features", "out_features", "num_hidden_layers", "hidden_features", "kernel_width")
        if (src is None or src is self or type(src) is not type(self)
                or any(getattr(src, a) != getattr(self, a) for a in geo)
                or src._flat is None or src._flat.device != self._flat.device or src._flat.dtype != self._flat.dtype
                or not src._is_packed() or src._wsplit_stamp != src._param_versions()):
            return None
        if not all(self._sig_of(state_dict[k]) == sg for k, sg in zip(own, src._view_sigs(src._flat))):
            return None
        return src

    def load_state_dict(self, state_dict, strict=True, assign=False):
        """torch's load_state_dict; when `state_dict` is another packed net's live state_dict()
        (the timestep snapshot prev.load_state_dict(net.state_dict()), fluid/model.py:64,69,
        advection/model.py:64) the parameters AND their pre-split weight planes are copied as
        ONE device copy of the flat storage (instead of a copy per tensor + a plane rewrite)."""
        src = None if assign else self._snapshot_source(state_dict)
        if src is None:
            return super().load_state_dict(state_dict, strict=strict, assign=assign)
        self.ensure_packed()
        with torch.no_grad():
            self._store.copy_(src._store)
        self._wsplit_stamp = self._param_versions()
        return nn.modules.module._IncompatibleKeys([], [])

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._repack()
        return out

    def _is_view_of(self, t, buf, entry):
        v = self._view(buf, entry)
        return t.data_ptr() == v.data_ptr() and t.stride() == v.stride() and t.shape == v.shape

    def _view_sigs(self, buf):
        """(data_ptr, stride, shape) of every parameter's view into `buf` -- cached per buffer
        (the checks run at every timestep snapshot and jet call; building the views is the cost)."""
        key = (buf.data_ptr(), buf.numel())
        cache = self.__dict__.get("_insr_sigs")
        if cache is None or cache[0] != key:
            sigs = [(v.data_ptr(), v.stride(), tuple(v.shape)) for v in (self._view(buf, e) for e in self._layout())]
            cache = self.__dict__["_insr_sigs"] = (key, sigs)
        return cache[1]

    @staticmethod
    def _sig_of(t):
        return (t.data_ptr(), t.stride(), tuple(t.shape))

    def _is_packed(self):
        params = self.plist()
        if self._flat is None or not params or self._flat.numel() != self.param_count:
            return False
        # (the parameters' own metadata: the same as p.data's, without building a tensor per parameter)
        return all(self._sig_of(p) == sg for p, sg in zip(params, self._view_sigs(self._flat)))

    def ensure_packed(self):
        if not self._is_packed():
            self._repack()

    # ---- flat gradient ---------------------------------------------------------
    # state 'stale': zero_grad() ran; the buffer holds garbage and the first
    # backward overwrites it (no memset launch).  'live': it holds the sum of
    # the backward passes since then.
    def _attach_grad_views(self, fold_foreign):
        params = self.plist()
        g = self._flat_grad
        if g is None or g.device != self._flat.device or g.numel() != self._flat.numel():
            g = torch.zeros_like(self._flat)
            self._flat_grad = g
        folded = False
        for p, e in zip(params, self._layout()):
            if p.grad is None or not self._is_view_of(p.grad, g, e):
                view = self._view(g, e)
                if fold_foreign and p.grad is not None:
                    view.copy_(p.grad)
                    folded = True
                elif fold_foreign:
                    view.zero_()
                    folded = True
                p.grad = view
        return g, folded

    # A fused-path backward's partial-gradient rows whose sums are held back for the Adam launch that
    # follows (base/_jet.py defer_reductions: insr_adam_step_partials sums them into .grad and steps in
    # one launch).  Anything else that touches the flat gradient first lands the sums
    # (flush_pending_reduce) -- or drops them when the gradient is being discarded (mark_grad_stale).
    def set_pending_reduce(self, args):
        self.__dict__['_insr_pending_reduce'] = args

    def take_pending_reduce(self):
        return self.__dict__.pop('_insr_pending_reduce', None)

    def flush_pending_reduce(self):
        """Land held-back sums now, on the stream their reverse jet ran on -- ordered after any
        earlier .grad write made on another stream, and recorded as the last write, so a reader
        on another stream (grad_read_sync) waits for the sums, not only for the sweep."""
        pr = self.take_pending_reduce()
        if pr is not None:
            self.grad_write_begin(pr.cur)
            _jet.launch_reduce(pr)
            self.grad_write_end(pr.cur)

    def mark_grad_stale(self, set_to_none=True):
        self.take_pending_reduce()  # zero_grad: the held-back sums would write a discarded gradient
        self.ensure_packed()
        if set_to_none:
            for p in self.plist():
                p.grad = None
        else:
            g, _ = self._attach_grad_views(fold_foreign=False)
            g.zero_()
        self._grad_state = 'stale'
        self._grad_event_stream = None  # a new iteration: earlier writes are ordered already

    def grad_for_backward(self):
        """(flat grad buffer, accumulate flag) for the next HIP backward."""
        self.flush_pending_reduce()  # an earlier write of this iteration lands first
        self.ensure_packed()
        if getattr(self, '_grad_state', 'stale') == 'stale' and all(p.grad is None for p in self.plist()):
            g, _ = self._attach_grad_views(fold_foreign=False)
            self._grad_state = 'live'
            return g, 0
        if getattr(self, '_grad_state', 'stale') == 'stale':
            # set_to_none=False zeroing already happened; or foreign grads: fold them
            g, _ = self._attach_grad_views(fold_foreign=True)
            self._grad_state = 'live'
            return g, 1
        g, _ = self._attach_grad_views(fold_foreign=True)
        return g, 1

    def bind_flat_grad(self, buf):
        """Make `buf` (a 1-D fp32 tensor of param_count elements, e.g. a slice of a model's
        data-parallel gradient arena) this network's flat .grad storage; the current
        gradient values move into it."""
        self.flush_pending_reduce()
        self.ensure_packed()
        if buf.numel() != self._flat.numel() or buf.dtype != self._flat.dtype or buf.device != self._flat.device:
            raise ValueError("bind_flat_grad: buffer does not match the flat parameters")
        live = any(p.grad is not None for p in self.plist())
        if live:
            old, _ = self._attach_grad_views(fold_foreign=True)
            buf.copy_(old)
        self._flat_grad = buf
        if live:
            self._attach_grad_views(fold_foreign=False)

    # ---- cross-stream ordering of the flat-gradient writes ---------------------------
    # A model may run some jets on a side stream (fluid boundary bands); autograd then runs
    # their backward on that stream too.  The HIP backward writes the flat .grad directly
    # (overwrite on the first write of an iteration, accumulate after), so the writers and
    # the readers (Adam, the DP all-reduce) are chained with an event when they are on
    # different streams.  Works under hipGraph capture (event record / wait = graph edges).
    def grad_write_begin(self, stream):
        """Before a write of .grad on `stream`: wait for this iteration's previous write if it
        was made on another stream (iterations start ordered: zero_grad clears the chain, so
        a graph capture never waits on an event recorded outside it)."""
        ev = getattr(self, "_grad_event", None)
        last = getattr(self, "_grad_event_stream", None)
        if ev is not None and last is not None and last != stream:
            stream.wait_event(ev)

    def grad_write_end(self, stream):
        ev = getattr(self, "_grad_event", None)
        if ev is None:
            ev = self._grad_event = torch.cuda.Event()
        ev.record(stream)
        self._grad_event_stream = stream

    def grad_read_sync(self, stream):
        """Make `stream` wait for the last gradient write when it happened on another stream."""
        self.grad_write_begin(stream)

    def grad_touched(self):
        return getattr(self, '_grad_state', 'stale') == 'live' or any(p.grad is not None for p in self.plist())

    def flat_grad_buffer(self):
        """Flat gradient with every parameter's .grad attached to it (None grads -> 0); held-back
        sums land first."""
        self.flush_pending_reduce()
        return self._flat_grad_buffer()

    def _flat_grad_buffer(self):
        """Flat gradient with every parameter's .grad attached to it (None grads -> 0)."""
        self.ensure_packed()
        if self._flat_grad is None or any(p.grad is None for p in self.plist()):
            g, _ = self._attach_grad_views(fold_foreign=True)
            self._grad_state = 'live'
            return g
        g, _ = self._attach_grad_views(fold_foreign=True)
        return g

    # ---- forward -------------------------------------------------------------
    @lower.api
    def forward(self, coords, weights=None):
        out = _jet.siren_value(self, coords)
        if weights is not None:
            out = out * weights
        return out

    def extra_repr(self):
        pad = "" if self.kernel_width == self.hidden_features else f" (kernel width {self.kernel_width}, zero-padded)"
        prec = "" if self.precision is None else f", precision={self.precision}"
        return (f"in={self.in_features}, out={self.out_features}, hidden_layers={self.num_hidden_layers}, "
                f"width={self.hidden_features}{pad}{prec}, backend=hip")
