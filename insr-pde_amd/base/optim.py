"""Device-resident Adam + ReduceLROnPlateau over flat parameter buffers.

Drop-in for what base/baseModel.py:55-62,79-81 builds: torch.optim.Adam
(betas (0.9, 0.999), eps 1e-8, no weight decay; one param group per trainable
network, lr = cfg.lr) and ReduceLROnPlateau(factor=0.1, patience=500,
min_lr=1e-8).  lr, step count and plateau state live in one small device
tensor, so an iteration needs no host round trip (hipGraph-replayable):

    ONE multi-tensor Adam launch over every network's flat buffer (bias
    corrections computed in-kernel from t + 1) -> ONE plateau launch that also
    advances t.

Reading `param_groups[i]['lr']` synchronises (as the reference's early-stop
check does, base/baseModel.py:132).
"""
import math
import weakref

import torch

from . import _native as nat


class _Group(dict):
    """A torch-style param group whose 'lr' reads the device state."""

    def __init__(self, opt, params, lr):
        super().__init__(params=params)
        self._opt = weakref.ref(opt)
        self._lr0 = lr

    def __getitem__(self, k):
        if k == 'lr':
            return self._opt().lr
        return super().__getitem__(k)

    def get(self, k, default=None):
        return self[k] if (k == 'lr' or k in self) else default


class FusedAdam:
    """Adam over whole networks (their flat buffers) + generic tensors."""

    def __init__(self, groups, betas=(0.9, 0.999), eps=1e-8):
        self.betas, self.eps = betas, eps
        self.param_groups = []
        self._nets = []     # (mlp, m, v)
        self._loose = []    # (param, m, v)
        dev = None
        lr = None
        for grp in groups:
            params = list(grp["params"]) if not hasattr(grp["params"], "flat_params") else grp["params"]
            lr = grp.get("lr", lr)
            self.param_groups.append(_Group(self, params, lr))
            owner = grp.get("module")
            if owner is not None and hasattr(owner, "flat_params"):
                owner.ensure_packed()
                flat = owner.flat_params()
                self._nets.append((owner, torch.zeros_like(flat), torch.zeros_like(flat)))
                dev = flat.device
            else:
                for p in params:
                    self._loose.append((p, torch.zeros_like(p), torch.zeros_like(p)))
                    dev = p.device
        if dev is None:
            raise ValueError("FusedAdam got no parameters")
        self.device = dev
        self.state = torch.zeros(nat.OPT_NFLOATS, device=dev, dtype=torch.float32)
        self.state[nat.OPT_LR] = lr
        self.state[nat.OPT_BEST] = math.inf
        self.state[nat.OPT_FACTOR] = 0.1
        self.state[nat.OPT_MINLR] = 0.0
        self._pending_advance = False

    @property
    def lr(self):
        return float(self.state[nat.OPT_LR])

    def zero_grad(self, set_to_none=True):
        for mlp, _, _ in self._nets:
            mlp.mark_grad_stale(set_to_none)
        for p, _, _ in self._loose:
            if p.grad is not None:
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.zero_()

    def _advance_pending(self):
        """t += 1 for a step() whose scheduler step never came (no scheduler / repeat step)."""
        if self._pending_advance:
            nat.check(nat.lib().insr_plateau_step(nat.ptr(self.state), None, 0, 1, nat.stream_of(self.device)),
                      "insr_plateau_step(advance)")
            self._pending_advance = False

    @torch.no_grad()
    def step(self, plateau=None):
        """One Adam update of every buffer whose grad exists, in ONE launch.
        Uses t = state[STEP] + 1; the step counter itself is advanced by the
        scheduler's plateau launch that follows (or lazily, without one).
        plateau = (DevicePlateau, metric): its step runs in the same launch (last block)."""
        import ctypes
        lib = nat.lib()
        self._advance_pending()
        if self._step_partials(plateau):
            return
        bufs = []
        stepped = []
        cur = torch.cuda.current_stream(self.device)
        for mlp, m, v in self._nets:
            if mlp.grad_touched():  # torch skips params whose .grad is None
                g = mlp.flat_grad_buffer()  # held-back sums land first (their write is recorded) ...
                mlp.grad_read_sync(cur)  # ... then wait for the last .grad write if it ran on a side stream
                bufs.append((mlp.flat_params(), g, m, v,
                             (mlp.in_features, mlp.out_features, mlp.num_hidden_layers, mlp.kernel_width)))
                stepped.append(mlp)
        for p, m, v in self._loose:
            if p.grad is not None:
                bufs.append((p.data, p.grad if p.grad.is_contiguous() else p.grad.contiguous(), m, v, (0, 0, 0, 0)))
        b1, b2 = self.betas
        st = nat.stream_of(self.device)
        chunks = [bufs[i:i + nat.ADAM_MAX_TENSORS] for i in range(0, len(bufs), nat.ADAM_MAX_TENSORS)]
        metric = plateau[0]._metric(plateau[1]) if plateau is not None else None
        if metric is not None and not chunks:
            plateau[0].step(plateau[1])
            metric = None
        for ci, chunk in enumerate(chunks):
            k = len(chunk)
            arr = lambda j: (ctypes.c_void_p * k)(*[c[j].data_ptr() for c in chunk])  # noqa: E731
            sizes = (ctypes.c_long * k)(*[c[0].numel() for c in chunk])
            # network buffers: the same launch rewrites their pre-split weight planes
            shapes = (ctypes.c_int * (4 * k))(*[v for c in chunk for v in c[4]])
            if metric is not None and ci == len(chunks) - 1:  # + the scheduler step (advances t)
                nat.check(lib.insr_adam_plateau_step_nets(k, arr(0), arr(1), arr(2), arr(3), sizes, shapes,
                                                          nat.ptr(self.state), b1, b2, self.eps, nat.ptr(metric),
                                                          plateau[0].patience, st), "insr_adam_plateau_step_nets")
            else:
                nat.check(lib.insr_adam_step_nets(k, arr(0), arr(1), arr(2), arr(3), sizes, shapes,
                                                  nat.ptr(self.state), b1, b2, self.eps, 1, st), "insr_adam_step_nets")
        for mlp in stepped:  # planes current: no refresh before the next jet
            mlp.mark_wsplit_current()
        self._pending_advance = plateau is None


    def _step_partials(self, plateau):
        """The step of a single network whose whole gradient is one reverse jet whose sums
        base._jet.defer_reductions held back: sums + Adam (+ plateau) in ONE launch
        (insr_adam_step_partials / insr_siren_jet_bwd_grad_adam phase 2: the same sums and update
        bit for bit).  False: not that case (the regular launch runs, landing held-back sums first)."""
        pend = [(mlp, m, v) for mlp, m, v in self._nets if "_insr_pending_reduce" in mlp.__dict__]
        if len(pend) != 1 or any(p.grad is not None for p, _, _ in self._loose):
            return False
        mlp, m, v = pend[0]
        if any(o is not mlp and o.grad_touched() for o, _, _ in self._nets):
            return False
        pr = mlp.__dict__["_insr_pending_reduce"]
        if pr.cur.cuda_stream != torch.cuda.current_stream(self.device).cuda_stream:
            return False
        mlp.take_pending_reduce()
        b1, b2 = self.betas
        metric = plateau[0]._metric(plateau[1]) if plateau is not None else None
        pr.launch(adam=(mlp.flat_params(), m, v, self.state, b1, b2, self.eps, metric,
                        plateau[0].patience if plateau is not None else 0))
        mlp.mark_wsplit_current()
        self._pending_advance = plateau is None
        self.partials_steps = getattr(self, "partials_steps", 0) + 1  # (tests: the fused path ran)
        return True


class DevicePlateau:
    """ReduceLROnPlateau(mode='min', threshold=1e-4 rel, cooldown=0, eps=1e-8) on the device."""
    fusable = True  # FusedAdam.step(plateau=(self, metric)) runs this step in the Adam launch

    def __init__(self, optimizer, factor=0.1, patience=10, min_lr=0.0, verbose=None):
        self.optimizer = optimizer
        self.patience = int(patience)
        with torch.no_grad():
            optimizer.state[nat.OPT_FACTOR] = factor
            optimizer.state[nat.OPT_MINLR] = min_lr
        self._scratch = torch.zeros(1, device=optimizer.device)

    def _metric(self, metrics):
        """The metric as a 1-element fp32 device tensor."""
        if isinstance(metrics, torch.Tensor) and metrics.is_cuda:
            m = metrics.detach().reshape(1)
            return m if m.dtype == torch.float32 else m.float()
        self._scratch.fill_(float(metrics))
        return self._scratch

    def step(self, metrics):
        m = self._metric(metrics)
        opt = self.optimizer
        adv = 1 if opt._pending_advance else 0
        nat.check(nat.lib().insr_plateau_step(nat.ptr(opt.state), nat.ptr(m), self.patience, adv,
                                              nat.stream_of(opt.device)), "insr_plateau_step")
        opt._pending_advance = False
