"""DevicePlateau + early stop against torch's own scheduler (base/baseModel.py:55-62,
80-81, 132-134): the device-resident ReduceLROnPlateau follows
torch.optim.lr_scheduler.ReduceLROnPlateau(factor, patience, min_lr) step for step on a
scripted loss sequence that crosses the patience, the relative threshold (1e-4) and the
min_lr clamp; and PhaseLoop stops a phase at the iteration the reference's loop does
(lr <= 1.1e-8 after ReduceLROnPlateau(factor 0.1, patience 500, min_lr 1e-8))."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def B():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    base._native.load()
    return base


def scripted_losses():
    seq = [1.0, 0.9, 0.8]                      # improving
    seq += [0.8 * (1 - 5e-5)] * 3              # below the 1e-4 relative threshold: not an improvement
    seq += [0.5]                               # improvement
    seq += [0.5] * 4                           # plateau > patience 3: lr 1e-4 -> 1e-5
    seq += [0.4, 0.4, 0.4, 0.4, 0.4]           # one improvement, then patience again -> 1e-6
    seq += [0.4] * 16                          # -> 1e-7 -> 1e-8 -> clamped at min_lr (no further change)
    return seq


@pytest.mark.parametrize("fused", [False, True])
def test_device_plateau_follows_torch_scheduler(B, fused):
    """fused: FusedAdam.step(plateau=...) -- the scheduler step in the Adam launch's last block
    (insr_adam_plateau_step_nets), as BaseModel._update_network issues it."""
    torch.manual_seed(0)
    net = B.MLP(2, 1, 1, 32, nonlinearity="sine").cuda()
    opt = B.FusedAdam([{"params": list(net.parameters()), "lr": 1e-4, "module": net}])
    sched = B.DevicePlateau(opt, factor=0.1, patience=3, min_lr=1e-8)
    dummy = torch.nn.Parameter(torch.zeros(1))
    topt = torch.optim.SGD([dummy], lr=1e-4)
    tsched = torch.optim.lr_scheduler.ReduceLROnPlateau(topt, factor=0.1, patience=3, min_lr=1e-8)
    lrs, tlrs = [], []
    for v in scripted_losses():
        net.flat_grad_buffer().normal_()
        if fused:
            opt.step(plateau=(sched, torch.tensor([v], device="cuda")))
        else:
            opt.step()
            sched.step(torch.tensor([v], device="cuda"))
        tsched.step(v)
        st = opt.state.cpu()
        lrs.append(float(st[B._native.OPT_LR]))
        tlrs.append(topt.param_groups[0]["lr"])
        assert int(st[B._native.OPT_BAD]) == tsched.num_bad_epochs
        assert float(st[B._native.OPT_BEST]) == pytest.approx(tsched.best, rel=1e-7)
    for a, b in zip(lrs, tlrs):
        assert a == pytest.approx(b, rel=1e-6)
    assert min(tlrs) == pytest.approx(1e-8) and len(set(round(math.log10(v)) for v in tlrs)) == 5
    assert int(opt.state[B._native.OPT_STEP]) == len(lrs)


def _expected_stop():
    """Iteration at which the reference's loop breaks for a constant loss."""
    dummy = torch.nn.Parameter(torch.zeros(1))
    topt = torch.optim.SGD([dummy], lr=1e-4)
    ts = torch.optim.lr_scheduler.ReduceLROnPlateau(topt, factor=0.1, patience=500, min_lr=1e-8)
    for i in range(10 ** 5):
        ts.step(0.25)
        if topt.param_groups[0]["lr"] <= 1.1e-8:
            return i
    raise AssertionError


@pytest.mark.parametrize("graph", [False, True])
def test_phase_loop_early_stop(B, graph):
    from pde.config import make_config

    class Const(B.BaseModel):
        """A phase whose loss never improves (its gradient is exactly zero)."""
        def __init__(self, cfg):
            super().__init__(cfg)
            self.field = self._create_network(1, 1)
            self.x = torch.linspace(-1, 1, 64, device=self.device).reshape(-1, 1).requires_grad_(True)

        @property
        def _trainable_networks(self):
            return {"field": self.field}

        def _sample_in_training(self):
            return self.x

        def initialize(self):
            pass

        def step(self):
            pass

        @B.BaseModel._training_loop
        def _fit(self):
            y = self.field(self._sample_in_training())
            return {"main": B.fused_mse(y, None, y.detach(), None, gamma=-1.0) + 0.25}

    cfg = make_config("advection", proj_dir="/tmp/insr_test_es", insr_progress=False, max_n_iters=5000,
                      num_hidden_layers=1, hidden_features=32, insr_graph=graph)
    torch.manual_seed(0)
    m = Const(cfg)
    m._fit()
    assert m.train_step == _expected_stop() + 1
    assert m.optimizer.param_groups[0]["lr"] <= 1.1e-8


@pytest.mark.parametrize("shape", [(2, 2, 2, 64), (1, 1, 1, 32)])  # 34 blocks; 5 (< 8 ticket shards)
def test_fused_adam_plateau_equals_two_launches(B, shape):
    """Parameters, moments and optimiser state after 12 fused Adam + plateau launches equal the
    separate insr_adam_step_nets + insr_plateau_step launches bit for bit; the two-level ticket's
    nine words are back at zero."""
    out = []
    for fused in (False, True):
        torch.manual_seed(1)
        net = B.MLP(shape[0], shape[1], shape[2], shape[3], nonlinearity="sine").cuda()
        opt = B.FusedAdam([{"params": list(net.parameters()), "lr": 1e-3, "module": net}])
        sched = B.DevicePlateau(opt, factor=0.5, patience=2, min_lr=1e-6)
        g = torch.Generator(device="cuda").manual_seed(2)
        for v in scripted_losses()[:12]:
            net.flat_grad_buffer().copy_(torch.randn(net.param_count, device="cuda", generator=g))
            loss = torch.tensor([v], device="cuda")
            if fused:
                opt.step(plateau=(sched, loss))
            else:
                opt.step()
                sched.step(loss)
        torch.cuda.synchronize()
        out.append((net.flat_params().clone(), opt._nets[0][1].clone(), opt._nets[0][2].clone(),
                    opt.state[:B._native.OPT_TICKET].clone(),
                    opt.state[B._native.OPT_TICKET:B._native.OPT_NFLOATS].view(torch.int32).abs().sum().item()))
    for u, v in zip(out[0][:4], out[1][:4]):
        assert torch.equal(u, v)
    assert out[1][4] == 0  # the ticket words are left at zero
