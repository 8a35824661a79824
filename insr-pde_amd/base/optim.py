"""Device-resident Adam + ReduceLROnPlateau over flat parameter buffers.

Drop-in for what base/baseModel.py:55-62,79-81 builds: torch.optim.Adam
(betas (0.9, 0.999), eps 1e-8, no weight decay; one param group per trainable
network, lr = cfg.lr) and ReduceLROnPlateau(factor=0.1, patience=500,
min_lr=1e-8).  lr, step count and plateau state live in one small device
tensor, so an iteration needs no host round trip (hipGraph-replayable):

    prepare (t += 1, bias corrections)  -> one Adam launch per network's flat
    buffer -> plateau step on the device-resident loss.

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

    @torch.no_grad()
    def step(self):
        lib = nat.lib()
        b1, b2 = self.betas
        st = nat.stream_of(self.device)
        nat.check(lib.insr_adam_prepare(nat.ptr(self.state), b1, b2, st), "insr_adam_prepare")
        for mlp, m, v in self._nets:
            if not mlp.grad_touched():
                continue  # torch skips params whose .grad is None
            flat, g = mlp.flat_params(), mlp.flat_grad_buffer()
            nat.check(lib.insr_adam_step(nat.ptr(flat), nat.ptr(g), nat.ptr(m), nat.ptr(v), flat.numel(),
                                         nat.ptr(self.state), b1, b2, self.eps, st), "insr_adam_step")
        for p, m, v in self._loose:
            if p.grad is None:
                continue
            g = p.grad.contiguous()
            nat.check(lib.insr_adam_step(nat.ptr(p.data), nat.ptr(g), nat.ptr(m), nat.ptr(v), p.numel(),
                                         nat.ptr(self.state), b1, b2, self.eps, st), "insr_adam_step")


class DevicePlateau:
    """ReduceLROnPlateau(mode='min', threshold=1e-4 rel, cooldown=0, eps=1e-8) on the device."""

    def __init__(self, optimizer, factor=0.1, patience=10, min_lr=0.0, verbose=None):
        self.optimizer = optimizer
        self.patience = int(patience)
        with torch.no_grad():
            optimizer.state[nat.OPT_FACTOR] = factor
            optimizer.state[nat.OPT_MINLR] = min_lr
        self._scratch = torch.zeros(1, device=optimizer.device)

    def step(self, metrics):
        if isinstance(metrics, torch.Tensor) and metrics.is_cuda:
            m = metrics.detach().reshape(1)
            if m.dtype != torch.float32:
                m = m.float()
        else:
            self._scratch.fill_(float(metrics))
            m = self._scratch
        nat.check(nat.lib().insr_plateau_step(nat.ptr(self.optimizer.state), nat.ptr(m), self.patience,
                                              nat.stream_of(self.optimizer.device)), "insr_plateau_step")
