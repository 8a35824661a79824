"""Re-entrancy of the C ABI ("re-entrant for distinct streams", no
process-global mutable state): every knob of a jet call -- precision, backward path, fp16 backward
products, tiles per block -- rides in its own `mode` argument (include/insr_siren.h
INSR_JET_PREC / INSR_JET_POLICY / INSR_JET_BWD_F16 / INSR_JET_TILES).  Two host threads drive
two HIP streams at once with different precisions and backward paths; each stream's outputs and
parameter gradients must equal, bit for bit, the same calls run alone on one stream.

Calls through the library directly (ctypes): the pressure net of fluid/model.py:111 (2 -> 1,
4 x 128) in its Laplacian jet, forward + backward into a gradient buffer.
"""
import ctypes
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu

N = 4111  # not a multiple of a tile: ragged last tile on every path


@pytest.fixture(scope="module")
def setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    nat = base._native
    lib = nat.load()
    torch.manual_seed(51)
    net = base.MLP(2, 1, 4, 128, nonlinearity="sine").cuda()
    net.refresh_wsplit()
    x = (torch.rand(N, 2, generator=torch.Generator().manual_seed(52)) * 2 - 1).cuda()
    g = torch.Generator().manual_seed(53)
    gy, gdy, glap = (torch.randn(N, 1, generator=g).cuda(), torch.randn(N, 1, 2, generator=g).cuda(),
                     torch.randn(N, 1, generator=g).cuda())
    return nat, lib, net, x, (gy, gdy, glap)


# (name, mode bits): default f16x3 forward + two-kernel f16x3 backward; bf16x6 forward + recompute
# backward; bf16x6 forward + resident bf16x6 backward; exact-fp32 forward and backward
CONFIGS = {
    "f16x3_twokernel": lambda nat: nat.jet_policy(2),
    "bf16x6_recompute": lambda nat: nat.jet_prec(nat.PREC_BF16X6) | nat.jet_policy(4),
    "bf16x6_resident": lambda nat: nat.jet_prec(nat.PREC_BF16X6) | nat.jet_policy(3) | nat.jet_bwd_f16(0),
    "fp32_fused_t2": lambda nat: nat.jet_prec(nat.PREC_F32) | nat.jet_tiles(2, 2),
}


class Run:
    """One configuration's buffers and its forward + backward on a given stream."""

    def __init__(self, setup, name):
        nat, lib, net, x, (gy, gdy, glap) = setup
        self.nat, self.lib, self.net, self.x = nat, lib, net, x
        self.gy, self.gdy, self.glap = gy, gdy, glap
        self.mode = nat.MODE_LAP | nat.MODE_WSPLIT | CONFIGS[name](nat)
        self.path = lib.insr_jet_bwd_path(N, 2, 1, 4, 128, self.mode)
        self.y, self.dy, self.lap = (torch.empty(N, 1, device="cuda"), torch.empty(N, 1, 2, device="cuda"),
                                     torch.empty(N, 1, device="cuda"))
        ab = lib.insr_jet_act_bytes(N, 2, 4, 128, self.mode)
        self.act = None if self.path == 3 else torch.empty(ab // 4, device="cuda")
        wb = lib.insr_jet_bwd_work_bytes(N, 2, 1, 4, 128, self.mode)
        if self.path == 0:
            wb = lib.insr_jet_partial_bytes(N, 2, 1, 4, 128, self.mode)
        self.work = torch.empty(max(wb // 4, 1), device="cuda")
        self.grad = torch.empty(net.param_count, device="cuda")

    def step(self, stream):
        nat, lib = self.nat, self.lib
        st = ctypes.c_void_p(stream.cuda_stream)
        flat = self.net.flat_params()
        rc = lib.insr_siren_jet_fwd(nat.ptr(self.x), N, 2, 1, 4, 128, self.mode, nat.ptr(flat), nat.ptr(self.y),
                                    nat.ptr(self.dy), nat.ptr(self.lap), nat.ptr(self.act), st)
        assert rc == 0
        if self.path > 0:
            rc = lib.insr_siren_jet_bwd_grad(nat.ptr(self.x), N, 2, 1, 4, 128, self.mode, nat.ptr(flat),
                                             nat.ptr(self.act), nat.ptr(self.gy), nat.ptr(self.gdy),
                                             nat.ptr(self.glap), nat.ptr(self.work), nat.ptr(self.grad), 0, st)
            assert rc == 0
        else:
            rc = lib.insr_siren_jet_bwd(nat.ptr(self.x), N, 2, 1, 4, 128, self.mode, nat.ptr(flat), nat.ptr(self.act),
                                        nat.ptr(self.gy), nat.ptr(self.gdy), nat.ptr(self.glap), nat.ptr(self.work), st)
            assert rc == 0
            rc = lib.insr_reduce_partials_strided(nat.ptr(self.work), lib.insr_jet_partial_blocks(N, 2, 128, self.mode),
                                                  self.net.param_count, lib.insr_jet_partial_stride(2, 1, 4, 128),
                                                  nat.ptr(self.grad), 0, st)
            assert rc == 0

    def result(self):
        return [t.clone() for t in (self.y, self.dy, self.lap, self.grad)]


def test_configs_take_their_own_paths(setup):
    """The knobs select different kernels: the four configurations run four backward paths."""
    paths = {name: Run(setup, name).path for name in CONFIGS}
    assert paths == {"f16x3_twokernel": 1, "bf16x6_recompute": 3, "bf16x6_resident": 2, "fp32_fused_t2": 0}


@pytest.mark.parametrize("pair", [("f16x3_twokernel", "bf16x6_recompute"), ("bf16x6_resident", "fp32_fused_t2"),
                                  ("f16x3_twokernel", "fp32_fused_t2")])
def test_two_streams_concurrently_match_single_stream(setup, pair):
    """Two threads, two streams, different precisions and backward paths, 6 forward + backward steps
    each, interleaved on the device: every output and gradient equals its single-stream run."""
    runs = [Run(setup, name) for name in pair]
    ref = []
    s0 = torch.cuda.Stream()
    for r in runs:  # alone, one after the other
        r.step(s0)
        s0.synchronize()
        ref.append(r.result())
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    errors = []
    start = threading.Barrier(2)

    def drive(k):
        try:
            start.wait()
            for _ in range(6):
                runs[k].step(streams[k])
            streams[k].synchronize()
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append(e)

    threads = [threading.Thread(target=drive, args=(k,)) for k in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in threads)
    assert not errors, errors
    torch.cuda.synchronize()
    for r, want in zip(runs, ref):
        for a, b in zip(r.result(), want):
            assert torch.isfinite(a).all()
            assert torch.equal(a, b)


@pytest.mark.parametrize("kind", ["value", "lap"])
def test_deferred_backward_on_side_stream_then_step(setup, kind):
    """A reverse jet run on a side stream inside defer_reductions holds its sums back; the optimiser
    step on the default stream cannot fuse them (other stream), so it lands them on their own stream
    (MLP.flush_pending_reduce records that write) and waits for it before Adam reads .grad
    (grad_read_sync after the flush).  Parameters and .grad equal the same sequence run on one stream
    bit for bit -- value jets (fused-path partial rows) and the Laplacian jet (split sums)."""
    import base
    from base import _jet
    res = []
    for side in (False, True):
        torch.manual_seed(61)
        net = base.MLP(2, 2 if kind == "value" else 1, 4, 128, nonlinearity="sine").cuda()
        opt = base.FusedAdam([{"params": list(net.parameters()), "lr": 1e-3, "module": net}])
        x = (torch.rand(3000, 2, generator=torch.Generator().manual_seed(62)) * 2 - 1).cuda().requires_grad_(True)
        s = torch.cuda.Stream() if side else torch.cuda.current_stream()
        s.wait_stream(torch.cuda.current_stream())
        opt.zero_grad()
        with _jet.defer_reductions():
            with torch.cuda.stream(s):
                y = net(x)
                v = y if kind == "value" else base.laplace(y, x)
                with _jet.batched_backward():
                    (v ** 2).sum().backward()
                # a long queue on the side stream: the sums would still be running if unordered
                for _ in range(20):
                    torch.matmul(torch.empty(512, 512, device="cuda"), torch.empty(512, 512, device="cuda"))
            assert "_insr_pending_reduce" in net.__dict__  # held back for the step
            opt.step()
        torch.cuda.synchronize()
        res.append((torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cpu(),
                    torch.cat([p.grad.reshape(-1) for p in net.parameters()]).cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
