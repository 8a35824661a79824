"""Pre-split weight planes (include/insr_siren.h insr_siren_wsplit, INSR_MODE_WSPLIT).

The split-bf16 kernels read every hidden weight as three bf16 terms that live after the
parameters in the flat storage.  They are derived data, so every way a parameter can change
must leave them current: FusedAdam (eager and captured), load_state_dict, a torch in-place
write; and a raw C-ABI call without the bit splits into a per-stream scratch copy instead.
Each check compares a jet against a fresh network holding the same parameters -- bit for bit.
"""
import ctypes

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


def _twin(B, net):
    """A fresh network with net's parameters (its planes built from scratch)."""
    t = B.MLP(net.in_features, net.out_features, net.num_hidden_layers, net.hidden_features,
              nonlinearity="sine").cuda()
    t.load_state_dict({k: v.clone() for k, v in net.state_dict().items()})  # clones: planes from scratch
    return t


def _lap(B, net, x):
    xg = x.clone().requires_grad_(True)
    return B.laplace(net(xg), xg).detach()


def test_planes_after_adam_steps(B):
    torch.manual_seed(0)
    net = B.MLP(2, 1, 3, 128, nonlinearity="sine").cuda()
    opt = B.FusedAdam([{"params": net.parameters(), "module": net, "lr": 1e-3}])
    x = torch.rand(3000, 2, device="cuda") * 2 - 1
    for _ in range(3):
        opt.zero_grad()
        xg = x.clone().requires_grad_(True)
        (B.laplace(net(xg), xg) ** 2).mean().backward()
        opt.step()
    assert torch.equal(_lap(B, net, x), _lap(B, _twin(B, net), x))


def test_planes_after_load_state_dict_and_inplace_write(B):
    torch.manual_seed(1)
    a = B.MLP(2, 2, 3, 128, nonlinearity="sine").cuda()
    b = B.MLP(2, 2, 3, 128, nonlinearity="sine").cuda()
    x = torch.rand(2000, 2, device="cuda") * 2 - 1
    b(x)  # planes of b's initial weights
    b.load_state_dict(a.state_dict())
    assert torch.equal(b(x), a(x))
    with torch.no_grad():
        b.net[2].weight.mul_(0.5)  # a torch in-place write: the version counter moves
    ref = _twin(B, b)
    assert torch.equal(b(x), ref(x))
    assert not torch.equal(b(x), a(x))


def test_raw_call_without_the_bit_uses_a_scratch_split(B):
    """insr_siren_jet_fwd on a bare parameter buffer (no planes, no INSR_MODE_WSPLIT) equals
    the network's own call with planes."""
    nat = B._native
    lib = nat.lib()
    torch.manual_seed(2)
    net = B.MLP(2, 1, 3, 128, nonlinearity="sine").cuda()
    n = 1500
    x = (torch.rand(n, 2, device="cuda") * 2 - 1).contiguous()
    bare = net.flat_params().clone()  # parameters only: no room for planes
    outs = []
    for buf, bit in ((bare, 0), (net.flat_params(), nat.MODE_WSPLIT)):
        if bit:
            net.refresh_wsplit()
        y = torch.empty(n, 1, device="cuda")
        dy = torch.empty(n, 1, 2, device="cuda")
        lap = torch.empty(n, 1, device="cuda")
        nat.check(lib.insr_siren_jet_fwd(nat.ptr(x), n, 2, 1, 3, 128, nat.MODE_LAP | bit, nat.ptr(buf), nat.ptr(y),
                                         nat.ptr(dy), nat.ptr(lap), None, nat.stream_of(x.device)), "fwd")
        outs.append((y, dy, lap))
    torch.cuda.synchronize()
    for u, v in zip(*outs):
        assert torch.equal(u, v)


def test_wsplit_planes_are_the_exact_three_term_split(B):
    """The planes hold bf16 terms h, m, l with h + m + l == w to 2^-24 relative (the split of
    jet_x6.hpp), for both orientations."""
    nat = B._native
    torch.manual_seed(3)
    net = B.MLP(2, 2, 2, 64, nonlinearity="sine").cuda()
    net.refresh_wsplit()
    torch.cuda.synchronize()
    store = net.flat_params()._base
    planes = store[net.wsplit_offset():].view(torch.int32).cpu()
    W, L, NT, KC = 64, 2, 4, 2
    vecs = L * W * W * 3 // 8

    def term(u):  # bf16 halves of an int32 word -> (lo, hi) floats
        lo = (u << 16).view(torch.float32)
        hi = (u & -65536).view(torch.float32)
        return lo, hi

    for o in (0, 1):
        for j in (1, 2):
            Wj = net.net[2 * j].weight.detach().cpu()
            for rt in range(NT):
                for kc in range(KC):
                    base = (o * vecs + (((j - 1) * NT + rt) * KC + kc) * 3 * 64) * 4
                    for lane in (0, 17, 63):
                        g, c = lane >> 4, lane & 15
                        tot = torch.zeros(8, dtype=torch.float64)
                        for q in range(3):
                            words = planes[base + (q * 64 + lane) * 4: base + (q * 64 + lane) * 4 + 4]
                            lo, hi = term(words)
                            tot += torch.stack([lo, hi], 1).reshape(8).double()
                        idx = [32 * kc + 8 * g + jj for jj in range(8)]
                        want = Wj[16 * rt + c, idx] if o == 0 else Wj[idx, 16 * rt + c]
                        assert torch.allclose(tot, want.double(), rtol=2.0 ** -23, atol=0), (o, j, rt, kc, lane)


def test_wsplit_fp16_planes_are_the_scaled_two_term_split(B):
    """The fp16 planes (INSR_PREC_F16X3, after both bf16 orientations) hold 2^8 w as fp16 terms
    h + l == 2^8 w to 2^-22 relative, in the forward (W_j rows) and then the backward (W_j^T rows)
    fragment order -- written by insr_siren_wsplit and, after an optimiser step, by the Adam launch."""
    torch.manual_seed(4)
    net = B.MLP(2, 2, 2, 64, nonlinearity="sine").cuda()
    opt = B.FusedAdam([{"params": net.parameters(), "module": net, "lr": 1e-2}])
    x = torch.rand(500, 2, device="cuda") * 2 - 1
    W, L, NT, KC = 64, 2, 4, 2
    for step in range(2):
        if step:
            opt.zero_grad()
            (net(x) ** 2).mean().backward()
            opt.step()  # the planes now come from adam_wsplit
        else:
            net.refresh_wsplit()
        torch.cuda.synchronize()
        store = net.flat_params()._base
        for o in (0, 1):
            h16 = store[net.wsplit_offset() + (3 + o) * L * W * W:].view(torch.float16).cpu().double()
            for j in (1, 2):
                Wj = net.net[2 * j].weight.detach().cpu().double() * 256.0
                if o:
                    Wj = Wj.t()
                for rt in range(NT):
                    for kc in range(KC):
                        fr = ((j - 1) * NT + rt) * KC + kc
                        for lane in (0, 17, 63):
                            g, c = lane >> 4, lane & 15
                            hi = h16[((fr * 2) * 64 + lane) * 8:((fr * 2) * 64 + lane) * 8 + 8]
                            lo = h16[((fr * 2 + 1) * 64 + lane) * 8:((fr * 2 + 1) * 64 + lane) * 8 + 8]
                            want = Wj[16 * rt + c, [32 * kc + 8 * g + jj for jj in range(8)]]
                            assert torch.allclose(hi + lo, want, rtol=2.0 ** -21, atol=2.0 ** -24), \
                                (step, o, j, rt, kc, lane)


@pytest.mark.parametrize("w0_scale", [1.0, 10.0, 40.0])
def test_f16x3_forward_matches_x6_to_fp32_level(B, w0_scale):
    """The f16x3 forward (MLP(precision='f16x3'), the default) against the bf16x6 forward of the
    same weights: value, gradient and Laplacian jets agree to 1e-5 normwise -- also with the first
    layer scaled x10 / x40 (tangents ~10-40x, Laplacians ~100-1600x the init's: the per-tile
    dynamic scale of the Laplacian planes keeps fp16 in range; the static 2^-4 of the first
    version overflowed to inf there)."""
    torch.manual_seed(5)
    a = B.MLP(2, 1, 4, 128, nonlinearity="sine", precision="bf16x6").cuda()
    b = B.MLP(2, 1, 4, 128, nonlinearity="sine", precision="f16x3").cuda()
    with torch.no_grad():
        a.net[0].weight.mul_(w0_scale)
    b.load_state_dict({k: v.clone() for k, v in a.state_dict().items()})
    x = torch.rand(3000, 2, device="cuda") * 2 - 1
    for net_out in (lambda n: n(x), lambda n: B.gradient(n(x.requires_grad_(True)), x),
                    lambda n: B.laplace(n(x.requires_grad_(True)), x)):
        u, v = net_out(a).detach(), net_out(b).detach()
        assert torch.isfinite(v).all()
        assert float((u - v).abs().max() / u.abs().max()) < 1e-5


def test_snapshot_copies_flat_storage_once(B):
    """prev.load_state_dict(net.state_dict()) -- the per-timestep snapshot of the reference
    (fluid/model.py:64,69) -- copies the parameters and the current planes as ONE flat copy; the
    result equals a net whose planes were built from scratch, bit for bit.  With net's planes
    stale (a torch in-place write and no jet since) it takes the per-tensor path + a rewrite."""
    torch.manual_seed(3)
    net = B.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    prev = B.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    opt = B.FusedAdam([{"params": net.parameters(), "module": net, "lr": 1e-3}])
    x = torch.rand(2000, 2, device="cuda") * 2 - 1
    for _ in range(2):
        opt.zero_grad()
        (net(x) ** 2).mean().backward()
        opt.step()
    assert prev._snapshot_source(net.state_dict()) is net
    prev.load_state_dict(net.state_dict())
    assert torch.equal(prev._store, _twin(B, net)._store)
    assert torch.equal(prev(x), net(x))
    with torch.no_grad():
        net.net[2].weight.mul_(0.5)  # planes of net now stale
    assert prev._snapshot_source(net.state_dict()) is None
    prev.load_state_dict(net.state_dict())
    assert torch.equal(prev._store, _twin(B, net)._store)
    assert torch.equal(prev(x), net(x))
