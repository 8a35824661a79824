"""Training-loop framework, drop-in for base/baseModel.py:10-162 of the reference.

Same abstract members (_trainable_networks, _sample_in_training, initialize,
step), decorators (_timestepping, _training_loop), helpers (_update_network,
_reset_optimizer, _create_network, _set_require_grads, _create_tb,
save_ckpt, load_ckpt) and attributes (device, dt, max_n_iters,
sample_resolution, vis_resolution, timestep, train_step, optimizer,
scheduler, tb).  Model files written for the reference run unchanged.

MI355X-specific behaviour (all opt-in through cfg attributes, defaults keep
the reference's semantics except where noted):
  * the optimiser is base.optim.FusedAdam (flat buffers, device-resident lr /
    step / plateau state) -- same update rule as torch.optim.Adam;
  * cfg.insr_sync_every (default 1): the loop reads the loss values (tqdm /
    tensorboard / early stop) every k iterations instead of every iteration;
  * cfg.insr_graph (default False): after one eager iteration the phase body +
    update is captured into a hipGraph (torch.cuda.CUDAGraph) and replayed;
    falls back to eager if the phase is not capturable;
  * data parallel: when torch.distributed is initialised, _update_network
    all-reduces the flat gradients (RCCL) before the Adam step and the losses
    before the plateau step (mean or sum per `_dp_loss_reduction`).
"""
import contextlib
import os
import shutil
from abc import ABC, abstractmethod

import torch

from . import _jet
from .losses import settle_lazy
from .networks import get_network
from .optim import DevicePlateau, FusedAdam

try:  # tensorboardX is optional (not installed on the MI355X image)
    from tensorboardX import SummaryWriter
except Exception:  # pragma: no cover - depends on the environment
    SummaryWriter = None

try:
    from tqdm import tqdm
except Exception:  # pragma: no cover
    tqdm = None


class _NullWriter:
    def __init__(self, *a, **k):
        pass

    def add_scalars(self, *a, **k):
        pass

    def add_scalar(self, *a, **k):
        pass

    def add_figure(self, *a, **k):
        pass

    def close(self):
        pass


def _local_device():
    rank = int(os.environ.get("LOCAL_RANK", "0"))
    return torch.device("cuda", rank)


class BaseModel(ABC):
    _dp_loss_reduction = 'mean'  # how per-rank losses combine under data parallelism

    def __init__(self, cfg):
        self.cfg = cfg
        self.exp_dir = cfg.exp_dir
        self.dt = cfg.dt
        self.max_n_iters = cfg.max_n_iters
        self.sample_resolution = cfg.sample_resolution
        self.vis_resolution = cfg.vis_resolution
        self.timestep = -1

        self.tb = None
        self.min_lr = 1.1e-8
        self.early_stop_plateau = 500
        self.train_step = 0
        self.optimizer = None
        self.scheduler = None

        self.device = _local_device()

    def _create_network(self, input_dim, output_dim):
        return get_network(self.cfg, input_dim, output_dim).to(self.device)

    @property
    @abstractmethod
    def _trainable_networks(self):
        """return a dict of trainable networks"""
        raise NotImplementedError

    @abstractmethod
    def _sample_in_training(self):
        """sampling points in each training step"""
        raise NotImplementedError

    @abstractmethod
    def initialize(self):
        """fit network to initial condition (timestep = 0). NOTE: warp with _timestepping."""
        raise NotImplementedError

    @abstractmethod
    def step(self):
        """step the system by one time step (timestep >= 1). NOTE: warp with _timestepping."""
        raise NotImplementedError

    def write_output(self, output_folder):
        """write visulized/discrete output"""
        pass

    # ------------------------------------------------------------------ optimiser
    def _reset_optimizer(self, use_scheduler=True, gamma=0.1, patience=500, min_lr=1e-8):
        """Adam (one group per trainable network) + ReduceLROnPlateau (base/baseModel.py:55-62)."""
        groups = [{"params": list(net.parameters()), "lr": self.cfg.lr, "module": net}
                  for net in self._trainable_networks.values()]
        self.optimizer = FusedAdam(groups)
        self.scheduler = DevicePlateau(self.optimizer, factor=gamma, patience=patience,
                                       min_lr=min_lr) if use_scheduler else None

    def _create_tb(self, name, overwrite=True):
        """create tensorboard log (a no-op writer when tensorboardX is absent)"""
        self.log_path = os.path.join(self.cfg.log_dir, name)
        if os.path.exists(self.log_path) and overwrite:
            shutil.rmtree(self.log_path, ignore_errors=True)
        if self.tb is not None:
            self.tb.close()
        self.tb = SummaryWriter(self.log_path) if SummaryWriter is not None else _NullWriter()

    def _dp_world(self):
        d = torch.distributed
        return d.get_world_size() if (d.is_available() and d.is_initialized()) else 1

    def _dp_total(self, count):
        """The denominator of a mean over `count` local terms: under data parallelism the global count
        (every rank holds an equal share), so the ranks' means -- values and gradients -- SUM to the global
        mean (models whose losses use it declare _dp_loss_reduction = 'sum': no 1/world pass)."""
        return count * self._dp_world() if self._dp_active() else count

    def _dp_active(self):
        """Whether iterations take the data-parallel path (gradient arena + all-reduce): world > 1, or
        cfg.insr_dp_always with a process group of any size (bench.py --dp-path: one rank's DP step,
        world-1 all-reduce included, measured on one GPU)."""
        if self._dp_world() > 1:
            return True
        d = torch.distributed
        return bool(getattr(getattr(self, "cfg", None), "insr_dp_always", False)) and d.is_available() and \
            d.is_initialized()

    def _dp_sync(self, loss_dict):
        """All-reduce gradients and losses across ranks: ONE RCCL call per iteration over the
        model's gradient arena -- every trainable network's flat .grad is a view into it (bound
        on the first call), followed by one slot per loss -- so there is no concatenation and
        no copy-back.  A network no gradient reached this iteration contributes zeros (one
        memset) and stays untouched for Adam (torch skips params whose .grad is None).

        Three pieces, so that the graph-replayed loop (base/_loop.py) issues only the collective
        eagerly: _dp_pack (device ops: zero-fill + the losses into the arena tail; captured with
        the phase and its backward), _dp_allreduce (the RCCL call), _dp_finish (the 1/world of a
        mean reduction; captured with Adam + plateau, which read the arena in place)."""
        if not self._dp_active():
            return loss_dict
        synced = self._dp_pack(loss_dict)
        self._dp_allreduce()
        self._dp_finish()
        return synced

    def _dp_allreduce(self):
        d = torch.distributed
        d.all_reduce(self._insr_dp_red, op=d.ReduceOp.SUM)

    def _dp_finish(self):
        if self._dp_loss_reduction == 'mean':
            self._insr_dp_red.div_(self._dp_world())

    def _dp_pack(self, loss_dict):
        """The iteration's gradients and losses as one contiguous arena slice (self._insr_dp_red);
        returns the losses as views of their arena slots (the values after _dp_allreduce/_dp_finish).

        Arena layout [net 0 | loss slots | net 1 | net 2 ...] (each network's flat .grad bound to its
        slice on the first call): the slice reduced is the smallest contiguous span covering the loss
        slots and every network this iteration's backward reached -- a phase that trains one of two
        networks (every fluid phase) all-reduces [its gradient | losses] only, with no zero-fill of the
        other network (untouched networks inside the span are zero-filled: they add nothing)."""
        if not self._dp_active():
            return loss_dict
        nets = list(self._trainable_networks.values())
        keys = list(loss_dict.keys())
        dev = nets[0].flat_params().device
        if torch.device(dev).type == "cuda" and torch.cuda.is_available():
            cur = torch.cuda.current_stream(dev)
            for net in nets:
                if hasattr(net, "grad_read_sync"):
                    net.grad_read_sync(cur)
        sizes = [net.param_count for net in nets]
        nslots = max(len(keys), 8)
        arena = self.__dict__.get("_insr_dp_arena")
        if arena is None or arena.numel() < sum(sizes) + nslots or arena.device != dev:
            arena = torch.zeros(sum(sizes) + nslots, device=dev, dtype=torch.float32)
            self._insr_dp_arena = arena
            offs, off = [], 0
            for i, (net, n) in enumerate(zip(nets, sizes)):
                if i == 1:
                    off += nslots  # the loss slots sit between the first and the second network
                offs.append(off)
                net.bind_flat_grad(arena[off:off + n])
                off += n
            self._insr_dp_offs, self._insr_dp_loss_off, self._insr_dp_nslots = offs, sizes[0], nslots
        offs, loss_off = self._insr_dp_offs, self._insr_dp_loss_off
        touched = [net.grad_touched() for net in nets]
        lo = min([loss_off] + [o for o, t in zip(offs, touched) if t])
        hi = max([loss_off + len(keys)] + [o + n for o, n, t in zip(offs, sizes, touched) if t])
        for o, n, t in zip(offs, sizes, touched):
            if not t and lo <= o < hi:
                arena[o:o + n].zero_()
        tail = arena[loss_off:loss_off + len(keys)]
        # losses a seeded reverse jet's sums launch already finished in their slots (_dp_redirect) need no copy
        direct = self.__dict__.pop("_insr_dp_direct", {})
        rest = [i for i, k in enumerate(keys) if not (k in direct and direct[k].state == "seeded")]
        if len(rest) == len(keys):
            torch.stack([torch.as_tensor(loss_dict[k], device=dev).detach().float().reshape(()) for k in keys], out=tail)
        else:
            for i in rest:
                tail[i].copy_(torch.as_tensor(loss_dict[keys[i]], device=dev).detach().float().reshape(()))
        self._insr_dp_red = arena[lo:hi]
        return {k: tail[i] for i, k in enumerate(keys)}

    def _dp_redirect(self, loss_dict):
        """Before the backward of a data-parallel iteration: the losses of lazy loss groups are finished by
        their seeded reverse jet's sums launch straight into their arena slots (the arena exists from the
        first iteration on), so _dp_pack copies only the others."""
        from .losses import lazy_output
        loss_off = self.__dict__.get("_insr_dp_loss_off")
        arena = self.__dict__.get("_insr_dp_arena")
        if not self._dp_active() or arena is None or loss_off is None:
            return
        if len(loss_dict) > self.__dict__.get("_insr_dp_nslots", 0):
            return  # more losses than the arena has slots: _dp_pack grows the arena and copies every loss
        direct = {}
        for i, (k, v) in enumerate(loss_dict.items()):
            hit = lazy_output(v)
            if hit is not None:
                g, j = hit
                g.redirect(j, arena.data_ptr() + 4 * (loss_off + i))
                direct[k] = g
        self._insr_dp_direct = direct

    # A phase body that returns its sq_losses outputs and reads no jet output they read elsewhere may let
    # its loss groups ride in the reverse jets (base/losses.py lazy_losses): the model classes that are
    # written that way set this (pde/fluid.py, pde/advection.py); cfg.insr_seed_in_bwd = False turns it off
    _insr_lazy_losses = False

    def _lazy_losses_on(self):
        """Whether the loop may open lazy_losses() around this model's phase body (opted in): the loss
        values are finished by the sums launch of the reverse jet that took the group -- inside the Adam
        launch (deferred sums), or right after the jet (data parallelism: before the arena pack)."""
        return self._insr_lazy_losses and getattr(self.cfg, "insr_seed_in_bwd", True)

    # Loss lowering (base/lower.py): the loop runs the phase body with network / diff-op outputs as Lazy
    # tensors and computes the losses it recognises -- the reference's torch.mean((a - b) ** 2) residuals
    # and wall terms as written -- in ONE fused loss-group launch.  On for every model (an unchanged
    # reference model file); the model classes written against the fused helpers (pde/fluid.py, ...) turn
    # it off; cfg.insr_lower = False turns it off for a run
    _insr_lower = True

    def _lower_on(self):
        return self._insr_lower and getattr(self.cfg, "insr_lower", True)

    def _defer_on(self):
        """With lowering: the body's forward jets are queued and launched together at the first read of a
        value (base/lower.py deferred_jets); cfg.insr_defer_jets = False launches each call at once."""
        return self._lower_on() and getattr(self.cfg, "insr_defer_jets", True)

    def _update_network(self, loss_dict):
        """update network by back propagation (base/baseModel.py:73-81).  backward of
        sum(loss_dict.values()) is run as backward of every term with a persistent unit
        seed: the same gradients without the add and ones-fill launches."""
        self.optimizer.zero_grad()
        self._dp_redirect(loss_dict)  # data parallel: lazy groups' losses straight into the arena slots
        # one process with the fused optimiser: a fused-path backward's row sums run inside the Adam
        # launch (base/_jet.py defer_reductions; under data parallelism the all-reduce needs them first)
        defer = _jet.DEFER_REDUCE and isinstance(self.optimizer, FusedAdam) and not self._dp_active()
        with (_jet.defer_reductions() if defer else contextlib.nullcontext()):
            self._backward(loss_dict)
            settle_lazy()  # lazy loss groups no reverse jet evaluated: launched now (base/losses.py)
            synced = self._dp_sync(loss_dict)
            if self.scheduler is not None and getattr(self.scheduler, "fusable", False):
                self.optimizer.step(plateau=(self.scheduler, synced['main']))  # Adam + plateau: one launch
            else:
                self.optimizer.step()
                if self.scheduler is not None:
                    self.scheduler.step(synced['main'])
        return synced

    def _backward(self, loss_dict):
        terms = [v for v in loss_dict.values() if v.requires_grad]
        if terms:
            # the reverse jets of one network (its interior batch and boundary bands from separate
            # calls) launch together when autograd is done with the pass (_jet.batched_backward)
            with _jet.batched_backward():
                torch.autograd.backward(terms, grad_tensors=[self._unit_seed(v) for v in terms])
            # join .grad writes a side-stream backward made (fluid boundary bands): the
            # caller's stream -- and a hipGraph capture -- must see them
            cur = torch.cuda.current_stream(self.device) if (torch.device(self.device).type == "cuda"
                                                             and torch.cuda.is_available()) else None
            if cur is not None:
                for net in self._trainable_networks.values():
                    if hasattr(net, "grad_read_sync"):
                        net.grad_read_sync(cur)

    def _unit_seed(self, v):
        seeds = self.__dict__.setdefault("_insr_seeds", {})
        key = (v.device, v.dtype, tuple(v.shape))
        if key not in seeds:
            from .losses import register_unit_seed
            seeds[key] = register_unit_seed(torch.ones(v.shape, device=v.device, dtype=v.dtype))
        return seeds[key]

    def _set_require_grads(self, model, require_grad):
        for p in model.parameters():
            p.requires_grad_(require_grad)

    # ------------------------------------------------------------------ decorators
    @classmethod
    def _timestepping(cls, func):
        def warp(self):
            self.timestep += 1
            self._create_tb(f"t{self.timestep:03d}")
            func(self)
            self.save_ckpt()
        return warp

    @classmethod
    def _training_loop(cls, func):
        """Wrap a phase body (returns a loss dict with key 'main') in the inner
        optimisation loop (base/baseModel.py:96-135)."""
        tag = func.__name__

        def loop(self, *args, **kwargs):
            from ._loop import PhaseLoop
            PhaseLoop(self, func, tag, args, kwargs).run()
        loop.__name__ = tag
        loop._insr_phase = func
        return loop

    # ------------------------------------------------------------------ checkpoints
    def save_ckpt(self, name=None):
        """save checkpoint for future restore (keys as base/baseModel.py:137-150)"""
        if name is None:
            save_path = os.path.join(self.cfg.model_dir, f"ckpt_step_t{self.timestep:03d}.pth")
        else:
            save_path = os.path.join(self.cfg.model_dir, f"ckpt_{name}.pth")
        save_dict = {}
        for key, net in self._trainable_networks.items():
            save_dict[f'net_{key}'] = {k: v.detach().cpu() for k, v in net.state_dict().items()}
        save_dict['timestep'] = self.timestep
        d = torch.distributed
        if not (d.is_available() and d.is_initialized()) or d.get_rank() == 0:  # one writer under DP
            os.makedirs(os.path.dirname(save_path), exist_ok=True)
            torch.save(save_dict, save_path)

    def load_ckpt(self, name):
        """load saved checkpoint (base/baseModel.py:152-162)"""
        if type(name) is int:
            load_path = os.path.join(self.cfg.model_dir, f"ckpt_step_t{name:03d}.pth")
        else:
            load_path = os.path.join(self.cfg.model_dir, f"ckpt_{name}.pth")
        checkpoint = torch.load(load_path, map_location=self.device, weights_only=True)
        for key, net in self._trainable_networks.items():
            net.load_state_dict(checkpoint[f'net_{key}'])
        self.timestep = checkpoint['timestep']
