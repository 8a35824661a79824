"""The inner optimisation loop of one phase (base/baseModel.py:96-135 semantics).

  reset optimiser -> for i < max_n_iters: loss_dict = phase(); update();
                     log losses; optional vis; early stop when lr <= 1.1e-8

Differences, all controlled by cfg attributes:
  insr_sync_every (int, default 1) -- losses/lr are read on the host every k
      iterations (the reference reads them every iteration, which costs two
      device->host syncs per iteration).  Early stop is checked at those reads.
  insr_graph (bool, default False) -- iteration 0 runs eagerly (warm-up,
      allocator settle); iteration 1 is captured into a hipGraph and every
      later iteration is one graph replay.  If capture fails (e.g. a phase
      with data-dependent shapes or host syncs) the loop stays eager.
      Under data parallelism with RCCL the all-reduce is captured too: one graph per
      iteration.  A backend whose collective cannot be captured (gloo) or
      cfg.insr_dp_capture = False gives two graphs -- [phase + backward + the
      gradients' and losses' arena pack] and [1/world + Adam + plateau, which read
      the arena in place] -- with the single all-reduce of that arena issued
      eagerly between them.
  insr_graph_unroll (int, default 1) -- single process or captured collectives: U > 1 also captures U
      consecutive iterations into ONE graph and replays that for every group of U
      iterations that holds no host read (sync / vis point) before its last one.  Each
      iteration inside is a full one (its own collocation points, backward, Adam + plateau
      step; the U iterations' points come from ONE sampler launch at the group's start,
      base.sampling.draw_ahead); it also saves the host's replay call per iteration (under a kernel
      trace, whose per-launch host work makes the host the bottleneck, ~8.7 us of idle
      device between two replays; without a profiler the host stays ahead and U = 1 and
      U = 4 measure the same, profiles/r04/final_v1/unroll_ab_*).
"""
import torch

from . import _jet
from .networks import MLP
from .losses import lazy_losses, settle_lazy
from .lower import deferred_jets, lower_losses, lowering
from .sampling import draw_ahead, draw_plan

try:
    from tqdm import tqdm
except Exception:  # pragma: no cover
    tqdm = None


class PhaseLoop:
    def __init__(self, model, func, tag, args, kwargs):
        self.m, self.func, self.tag = model, func, tag
        self.args, self.kwargs = args, kwargs
        cfg = model.cfg
        self.sync_every = max(1, int(getattr(cfg, "insr_sync_every", 1)))
        self.use_graph = bool(getattr(cfg, "insr_graph", False))
        self.vis_every = int(getattr(cfg, "vis_frequency", 1000))
        self.early_stop = bool(getattr(cfg, "early_stop", True))
        self.show = bool(getattr(cfg, "insr_progress", True)) and tqdm is not None
        self.graph = self.graph2 = None
        self.static = None
        self.static_main = None
        self.unroll = max(1, int(getattr(cfg, "insr_graph_unroll", 1)))
        self.graphU = None
        self.staticU = None

    def start(self):
        """Fresh optimiser + scheduler for this phase (base/baseModel.py:106)."""
        self.m._reset_optimizer()
        self.opt, self.sched = self.m.optimizer, self.m.scheduler
        self.graph, self.graph2, self.static = None, None, None
        self.graphU, self.staticU = None, None

    def _body(self):
        self.m.optimizer, self.m.scheduler = self.opt, self.sched
        # lazy_losses: the body's loss groups ride in the reverse jets (BaseModel._lazy_losses_on)
        with _jet.call_scope(self), draw_plan(self), lazy_losses(self.m._lazy_losses_on()):
            # lowering: an unchanged reference body's residual expressions -> one loss-group launch (base/lower.py)
            with lowering(self.m._lower_on()), deferred_jets(self.m._defer_on()):
                loss_dict = self.func(self.m, *self.args, **self.kwargs)
            loss_dict = lower_losses(loss_dict)
        synced = self.m._update_network(loss_dict)
        return synced if isinstance(synced, dict) else loss_dict

    # ---- data-parallel split: [phase + backward + arena pack] graph | eager RCCL all-reduce |
    # [1/world + Adam + plateau] graph -- the collective is the only eager launch of an iteration
    def _stage1(self):
        m = self.m
        m.optimizer, m.scheduler = self.opt, self.sched
        with _jet.call_scope(self), draw_plan(self), lazy_losses(m._lazy_losses_on()):
            with lowering(m._lower_on()), deferred_jets(m._defer_on()):
                loss_dict = self.func(m, *self.args, **self.kwargs)
            loss_dict = lower_losses(loss_dict)
        m.optimizer.zero_grad()
        m._dp_redirect(loss_dict)  # lazy groups' losses finished straight into the arena's loss slots
        m._backward(loss_dict)
        settle_lazy()  # (the seeded jets' sums launches finished the loss values the pack reads)
        packed = m._dp_pack(loss_dict)  # gradients + losses in the arena (views of its tail)
        self.static_main = packed['main'].detach().reshape(1)
        return packed

    def _stage2(self):
        m = self.m
        m._dp_finish()
        if m.scheduler is not None and getattr(m.scheduler, "fusable", False):
            m.optimizer.step(plateau=(m.scheduler, self.static_main))  # Adam + plateau: one launch
        else:
            m.optimizer.step()
            if m.scheduler is not None:
                m.scheduler.step(self.static_main)

    def _dp_step_eager(self):
        packed = self._stage1()
        self.m._dp_allreduce()
        self._stage2()
        return packed

    def _capture_graph(self, fn):
        from .losses import prepare_workspaces
        m = self.m
        # one capture stream per model (its loss workspaces are created once, before capture)
        side = m.__dict__.get("_insr_capture_stream")
        if side is None:
            side = m._insr_capture_stream = torch.cuda.Stream(device=m.device)
        prepare_workspaces(side)
        side.wait_stream(torch.cuda.current_stream(m.device))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                out = fn()
        torch.cuda.current_stream(m.device).wait_stream(side)
        return g, out

    _warned = set()

    def _capture_failed(self, e, fallback):
        """Record a failed hipGraph capture on the model (`_insr_capture_error`: tests assert it is None)
        and warn once per (model class, phase, error type) -- a phase that silently ran eagerly had hidden
        the round-5 el3D strong-path failure."""
        self.capture_error = repr(e)
        self.m._insr_capture_error = self.capture_error  # visible after run() (tests, logs)
        key = (type(self.m).__name__, self.tag, type(e).__name__)
        if key not in PhaseLoop._warned:
            PhaseLoop._warned.add(key)
            import warnings
            warnings.warn(f"{type(self.m).__name__}.{self.tag}: hipGraph capture failed ({self.capture_error}); "
                          f"{fallback}", RuntimeWarning, stacklevel=3)

    def _dp_split(self):
        """Whether a data-parallel iteration is replayed as two graphs around an EAGER all-reduce: the
        collective cannot be captured (gloo: host-side) or cfg.insr_dp_capture is off.  With RCCL
        (backend 'nccl') the all-reduce is captured with the rest of the iteration: ONE graph per
        iteration (or per group of insr_graph_unroll iterations), no host round trip between the
        backward and the optimiser step (profiles/r05: two host gaps of ~18 + ~9 us per iteration in
        the split form)."""
        if not self.m._dp_active():
            return False
        if not getattr(self.m.cfg, "insr_dp_capture", True):
            return True
        d = torch.distributed
        return d.get_backend() != "nccl" or torch.device(self.m.device).type != "cuda"

    def _capture(self):
        try:
            if self._dp_split():
                g1, out = self._capture_graph(self._stage1)
                g2, _ = self._capture_graph(self._stage2)
                self.graph, self.graph2 = g1, g2
            else:
                self.graph, out = self._capture_graph(self._body)
                self.graph2 = None
        except Exception as e:  # not capturable: stay eager
            torch.cuda.synchronize(self.m.device)
            self.use_graph = False
            self._capture_failed(e, "the phase runs eagerly")
            self.graph = self.graph2 = None
            return None
        self.static = {k: v.detach() for k, v in out.items()}
        return self.static

    def _bodies(self):
        out = None
        with draw_ahead(self.unroll):  # the group's collocation draws: one sampler launch up front
            for _ in range(self.unroll):
                out = self._body()
        return out

    def can_group(self):
        """Whether run_group() may serve the next `unroll` iterations (graph mode, one process,
        the single-iteration graph already captured: iterations 0 and 1 ran)."""
        return (self.unroll > 1 and self.use_graph and self.graph is not None and self.graph2 is None
                and not self._dp_split())

    def run_group(self):
        """`unroll` consecutive iterations as ONE graph replay (captured on first use -- a capture
        records, the replay that follows runs); returns the device loss dict of the group's last
        iteration."""
        if self.graphU is None:
            try:
                self.graphU, out = self._capture_graph(self._bodies)
            except Exception as e:  # not capturable as a group: iterate singly from now on
                torch.cuda.synchronize(self.m.device)
                self.unroll = 1
                self._capture_failed(e, "iterations replay one graph each")
                self.graphU = None
                return None
            self.staticU = {k: v.detach() for k, v in out.items()}
        self.graphU.replay()
        return self.staticU

    def run_iters(self, i0, k):
        """Iterations i0 .. i0 + k - 1 (no host reads in between): groups of `unroll` as one
        replay where possible, the rest one by one.  Returns the last iteration's loss dict."""
        out, i = None, i0
        while i < i0 + k:
            if i0 + k - i >= self.unroll and i >= 2 and self.can_group():
                out = self.run_group()
                if out is not None:
                    i += self.unroll
                    continue
            out = self.step(i)
            i += 1
        return out

    def step(self, i):
        """Run iteration i; returns the device loss dict of that iteration."""
        dp = self._dp_split()
        if self.use_graph and i >= 1:
            if self.graph is None and self._capture() is None:
                return self._dp_step_eager() if dp else self._body()
            self.graph.replay()
            if self.graph2 is None:
                return self.static
            self.m._dp_allreduce()  # one RCCL all-reduce, eager (the arena the graphs read in place)
            self.graph2.replay()
            return self.static
        return self._dp_step_eager() if dp else self._body()

    def run(self):
        m = self.m
        self.start()
        m.train_step = 0
        pbar = tqdm(range(m.max_n_iters), desc=f"{self.tag}[{m.timestep}]", disable=not self.show) \
            if tqdm is not None else range(m.max_n_iters)
        min_loss, accum = float("inf"), 0
        U = self.unroll
        skip = 0
        for i in pbar:
            if skip:  # inside a group run_group() already executed
                skip -= 1
                m.train_step += 1
                if skip:
                    continue
                # the group's last iteration: loss_dict is its losses -- read below as usual
            else:
                def host_reads(q):
                    return (q + 1) % self.sync_every == 0 or q == m.max_n_iters - 1 or q == 0 or \
                        (q + 1) % self.vis_every == 0
                grouped = None
                if (U > 1 and i >= 2 and i + U <= m.max_n_iters and self.can_group()
                        and not any(host_reads(q) for q in range(i, i + U - 1))):
                    grouped = self.run_group()
                if grouped is not None:
                    loss_dict, skip = grouped, U - 1
                    m.train_step += 1
                    continue
                loss_dict = self.step(i)
                m.train_step += 1
            last = (i == m.max_n_iters - 1)
            if (i + 1) % self.sync_every == 0 or last or i == 0:
                vals = {k: float(v) for k, v in loss_dict.items()}
                # the fp16 weight planes' range guard: one device-to-host read for every network
                MLP.check_weight_planes_all(m._trainable_networks.values())
                if m.tb is not None:
                    m.tb.add_scalars(self.tag, vals, global_step=i)
                if tqdm is not None and hasattr(pbar, "set_postfix"):
                    pbar.set_postfix(vals)
                if vals["main"] < min_loss:
                    min_loss, accum = vals["main"], 0
                else:
                    accum += 1
                if self.early_stop and m.optimizer.param_groups[0]['lr'] <= m.min_lr:
                    if tqdm is not None:
                        tqdm.write(f"early stopping at iteration {i}")
                    break
            if (i == 0 or (i + 1) % self.vis_every == 0) and hasattr(m, f"_vis{self.tag}"):
                getattr(m, f"_vis{self.tag}")()
        # the fp16 weight planes' range guard at the phase's end too, whatever insr_sync_every is (a
        # loop that never syncs -- bench.py's 1e9 -- is still checked once per phase)
        MLP.check_weight_planes_all(m._trainable_networks.values())
        self.graph = self.graph2 = None
        self.static = None
