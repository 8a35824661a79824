"""Fused collocation sampler (insr_sample_boxes / base.sample_random_and_bands2D).

The device stream is Philox-4x32-10: a numpy restatement here is pinned to the Random123
known-answer vector, and the kernel's draws must equal it bit for bit (value v of a
launch = Philox(seed, base + v // 4)[v % 4] -> lo + (hi - lo) * (bits >> 8) * 2^-24).
Distribution checks cover the reference samplers' boxes (base/sampling.py:14-64).
"""
import ctypes

import numpy as np
import pytest
import torch

M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85


def philox4x32_10(key, ctr):
    """numpy Philox-4x32-10; key (k0, k1), ctr (N, 4) uint32 -> (N, 4) uint32."""
    c = np.array(ctr, dtype=np.uint64)
    k0, k1 = np.uint64(key[0]), np.uint64(key[1])
    mask = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(M0) * c[:, 0]
        p1 = np.uint64(M1) * c[:, 2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        c = np.stack([hi1 ^ c[:, 1] ^ k0, lo1, hi0 ^ c[:, 3] ^ k1, lo0], axis=1)
        k0, k1 = (k0 + np.uint64(W0)) & mask, (k1 + np.uint64(W1)) & mask
    return c.astype(np.uint32)


def test_numpy_philox_known_answer():
    # Random123 kat_vectors: philox4x32 10 rounds, ctr = key = 0 and ctr = key = all ones
    assert philox4x32_10((0, 0), [[0, 0, 0, 0]]).tolist() == [[0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]]
    f = 0xFFFFFFFF
    assert philox4x32_10((f, f), [[f, f, f, f]]).tolist() == [[0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]]


@pytest.fixture(scope="module")
def B():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    base._native.load()
    return base


def _draw(B, boxes, dim, seed, state):
    nat = B._native
    arr = (nat.Box * len(boxes))()
    f3 = nat._F * 3
    outs = []
    for k, (n, lo, hi) in enumerate(boxes):
        t = torch.empty(n, dim, device="cuda")
        outs.append(t)
        arr[k] = nat.Box(t.data_ptr(), n, f3(*(list(lo) + [0.0] * (3 - dim))), f3(*(list(hi) + [0.0] * (3 - dim))))
    nat.check(nat.lib().insr_sample_boxes(arr, len(boxes), dim, seed, nat.ptr(state), nat.stream_of(0)), "sample")
    return outs


def _expected(boxes, dim, seed, base):
    total = sum(n * dim for n, _, _ in boxes)
    nthreads = (total + 3) // 4
    ctr = np.zeros((nthreads, 4), dtype=np.uint64)
    g = np.arange(nthreads, dtype=np.uint64) + np.uint64(base)
    ctr[:, 0], ctr[:, 1] = g & np.uint64(0xFFFFFFFF), g >> np.uint64(32)
    bits = philox4x32_10((seed & 0xFFFFFFFF, seed >> 32), ctr).reshape(-1)[:total]
    u = (bits >> 8).astype(np.float32) * np.float32(2.0 ** -24)
    out, v = [], 0
    for n, lo, hi in boxes:
        uu = u[v:v + n * dim].reshape(n, dim)
        lo32, hi32 = np.array(lo, np.float32), np.array(hi, np.float32)
        out.append(lo32 + (hi32 - lo32) * uu)
        v += n * dim
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [1, 2, 3])
def test_kernel_equals_philox_restatement_and_advances(B, dim):
    boxes = [(1000, [-1.0] * dim, [1.0] * dim), (7, [0.5] * dim, [0.75] * dim), (0, [0.0] * dim, [1.0] * dim),
             (333, [-2.0 + j for j in range(dim)], [-1.0 + 2 * j for j in range(dim)])]
    seed = 0x123456789ABCDEF
    state = torch.zeros(2, dtype=torch.int64, device="cuda")
    state[0] = (1 << 32) - 5  # counter carry into the high word inside the launch
    base = int(state[0])
    for _ in range(2):
        got = _draw(B, boxes, dim, seed, state)
        exp = _expected(boxes, dim, seed, base)
        for g, e in zip(got, exp):
            assert np.array_equal(g.cpu().numpy(), e)
        total = sum(n * dim for n, _, _ in boxes)
        assert int(state[0]) == base + (total + 3) // 4 and int(state[1]) == 0  # advanced; ticket reset
        base = int(state[0])


@pytest.mark.gpu
def test_fluid_draw_boxes_and_moments(B):
    torch.manual_seed(0)
    x, bxy = B.sample_random_and_bands2D(1 << 20, 2000, epsilon=1e-4, device="cuda")
    assert x.shape == (1 << 20, 2) and bxy.shape == (4000, 2)
    xc = x.double().cpu()
    assert float(xc.min()) >= -1.0 and float(xc.max()) < 1.0
    assert abs(float(xc.mean())) < 3e-3 and abs(float(xc.var()) - 1.0 / 3.0) < 3e-3
    b = bxy.cpu().view(4, 1000, 2)
    eps = 1e-4
    # face order of sample_boundary2D_pair: x = -1, x = +1, y = -1, y = +1 bands
    for k, (axis, c) in enumerate([(0, -1.0), (0, 1.0), (1, -1.0), (1, 1.0)]):
        assert float((b[k, :, axis] - c).abs().max()) <= eps + 2.5e-7  # fp32 rounding of 1 +- eps
        other = b[k, :, 1 - axis]
        assert float(other.min()) >= -1.0 and float(other.max()) < 1.0 and float(other.std()) > 0.5


@pytest.mark.gpu
def test_graph_replay_draws_fresh_points(B):
    x0, _ = B.sample_random_and_bands2D(4096, 40, device="cuda")  # eager: creates the state
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            xg, bg = B.sample_random_and_bands2D(4096, 40, device="cuda")
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a = xg.clone()
    g.replay()
    torch.cuda.synchronize()
    assert not torch.equal(a, xg) and not torch.equal(a, x0)
    assert float(xg.abs().max()) <= 1.0


@pytest.mark.gpu
def test_sample_boxes_rows_in_box_order(B):
    out = B.sample_boxes([(5000, [-2.0], [2.0]), (20, [-2.0002], [-1.9998]), (20, [1.9998], [2.0002])], 1)
    assert out.shape == (5040, 1)
    o = out.cpu()
    assert float(o[:5000].min()) >= -2.0 and float(o[:5000].max()) < 2.0 and float(o[:5000].std()) > 1.0
    assert float((o[5000:5020] + 2.0).abs().max()) <= 2e-4 + 5e-7
    assert float((o[5020:] - 2.0).abs().max()) <= 2e-4 + 5e-7


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_advection_device_sampler_phase_runs(B, graph):
    """advect1D on the GPU draws x and the Dirichlet bands in one launch (rows of one xa
    buffer) and fuses the frozen / trainable gradient jets; eager and graph replay train."""
    from pde.advection import Advection1DModel
    from pde.config import make_config
    torch.manual_seed(0)
    cfg = make_config("advection", proj_dir="/tmp/insr_test", insr_progress=False, early_stop=False,
                      max_n_iters=8, lr=1e-4, insr_graph=graph, insr_sync_every=4, init_cond="example1")
    model = Advection1DModel(cfg)
    model.timestep = 1
    model.initialize()
    before = model.field.flat_params().detach().clone()
    model.step()
    after = model.field.flat_params().detach()
    assert torch.isfinite(after).all() and not torch.equal(before, after)
    if graph:
        assert getattr(model, "_insr_capture_error", None) is None


@pytest.mark.gpu
def test_reference_band_samplers_on_the_device(B):
    """The reference's band samplers called with a cuda device (base/sampling.py:21-64: what an
    unchanged model file calls) draw through ONE insr_sample_boxes launch: face k in rows
    [k n, (k + 1) n), each coordinate uniform in its face's range, a fresh draw per call."""
    eps = 1e-4
    lo, hi, full = (-1 - eps, -1 + eps), (1 - eps, 1 + eps), (-1.0, 1.0)
    cases = [
        (lambda: B.sample_boundary2D_separate(4000, side="horizontal", device="cuda"), [(lo, full), (hi, full)]),
        (lambda: B.sample_boundary2D_separate(4000, side="vertical", device="cuda"), [(full, lo), (full, hi)]),
        (lambda: B.sample_boundary(8000, 2, device="cuda"), [(full, lo), (full, hi), (lo, full), (hi, full)]),
        (lambda: B.sample_boundary2D_pair(4000, device="cuda"), [(lo, full), (hi, full), (full, lo), (full, hi)]),
        (lambda: B.sample_boundary(4000, 1, device="cuda"), [(lo,), (hi,)]),  # advection/model.py:86
    ]
    for draw, faces in cases:
        a, b = draw(), draw()
        n = 2000
        assert a.shape == (n * len(faces), len(faces[0])) and a.is_cuda and a.dtype == torch.float32
        assert not torch.equal(a, b)
        for k, face in enumerate(faces):
            rows = a[k * n:(k + 1) * n].cpu().double()
            for j, (l, h) in enumerate(face):
                col = rows[:, j]
                assert float(col.min()) >= np.float32(l) and float(col.max()) <= np.float32(h), (k, j)
                assert abs(float(col.mean()) - (l + h) / 2) < 0.05 * (h - l), (k, j)
    assert B.sample_boundary2D_separate(1, side="horizontal", device="cuda").shape == (0, 2)


@pytest.mark.gpu
def test_sample_random_on_the_device(B):
    """sample_random(N, d, device='cuda') (base/sampling.py:14-18): one insr_sample_boxes launch,
    uniform in [-1, 1)^d, fresh per call."""
    for d in (1, 2, 3):
        a, b = B.sample_random(20000, d, device="cuda"), B.sample_random(20000, d, device="cuda")
        assert a.shape == (20000, d) and a.is_cuda and not torch.equal(a, b)
        assert float(a.min()) >= -1.0 and float(a.max()) < 1.0
        assert abs(float(a.mean())) < 0.02 and abs(float(a.var()) - 1 / 3) < 0.02
    assert B.sample_random(0, 2, device="cuda").shape == (0, 2)


@pytest.mark.gpu
def test_draw_plan_one_launch_per_iteration(B):
    """Inside a phase loop's draw_plan (base/_loop.py) the reference's per-iteration sampler calls
    (fluid/model.py:75,94-95: sample_random + two sample_boundary2D_separate) draw in ONE
    insr_sample_boxes launch from the second iteration on: same shapes and boxes, fresh points
    every iteration, every request its own tensor; a request off the recorded plan draws alone."""
    from base import _native as nat
    from base.sampling import draw_plan
    lib = nat.lib()
    orig, calls = lib.insr_sample_boxes, []

    def counting(*a):
        calls.append(a[1])
        return orig(*a)

    class Owner:
        pass

    eps = 1e-4
    lo, hi, full = (-1 - eps, -1 + eps), (1 - eps, 1 + eps), (-1.0, 1.0)
    owner, seen = Owner(), []
    lib.insr_sample_boxes = counting
    try:
        for it in range(3):
            calls.clear()
            with draw_plan(owner):
                x = B.sample_random(16384, 2, device="cuda").requires_grad_(True)
                bx = B.sample_boundary2D_separate(163, side="horizontal", device="cuda").requires_grad_(True)
                by = B.sample_boundary2D_separate(163, side="vertical", device="cuda").requires_grad_(True)
            assert calls == ([1, 2, 2] if it == 0 else [5]), (it, calls)
            assert x.shape == (16384, 2) and bx.shape == (162, 2) and by.shape == (162, 2)
            assert x.is_leaf and bx.is_leaf and by.is_leaf
            assert float(x.min()) >= -1.0 and float(x.max()) < 1.0 and abs(float(x.mean())) < 0.03
            for t, faces in ((bx, [(lo, full), (hi, full)]), (by, [(full, lo), (full, hi)])):
                for k, face in enumerate(faces):
                    rows = t[k * 81:(k + 1) * 81].detach().cpu().double()
                    for j, (l, h) in enumerate(face):
                        assert float(rows[:, j].min()) >= np.float32(l) and float(rows[:, j].max()) <= np.float32(h)
            seen.append(x.detach().clone())
        assert not torch.equal(seen[1], seen[2]) and not torch.equal(seen[0], seen[1])
        # off the plan: another size draws alone, and so does every later request of that iteration
        calls.clear()
        with draw_plan(owner):
            B.sample_random(8192, 2, device="cuda")
            B.sample_boundary2D_separate(163, side="horizontal", device="cuda")
        assert calls == [1, 2], calls
    finally:
        lib.insr_sample_boxes = orig


@pytest.mark.gpu
def test_same_seed_reseed_repeats_draws(B):
    """Re-seeding torch with the SAME seed restarts the device sampler's stream, as the reference's
    torch samplers repeat their draws (base/sampling.py:14-18); torch's own CUDA draws in between
    (which only advance torch's generator) do not restart it."""
    for reseed in (torch.manual_seed, torch.cuda.manual_seed):
        reseed(0)
        a = B.sample_random(1000, 2, device="cuda")
        a2 = B.sample_random(1000, 2, device="cuda")
        reseed(0)
        b = B.sample_random(1000, 2, device="cuda")
        torch.rand(10, device="cuda")  # torch's own CUDA RNG in between
        b2 = B.sample_random(1000, 2, device="cuda")
        assert torch.equal(a, b) and not torch.equal(a, a2)
        assert not torch.equal(b, b2)
    torch.manual_seed(1)
    c = B.sample_random(1000, 2, device="cuda")
    assert not torch.equal(a, c)


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [1, 2, 3])
def test_repeated_draw_equals_consecutive_draws(B, dim):
    """insr_sample_boxes_rep (base.sampling.draw_ahead: the U iterations of a replayed group drawn by
    one launch): repetition r of every box is bit for bit the r-th of U single launches -- each
    repetition starts at the Philox group where that launch would start, odd value counts included --
    and the stream position advances exactly as far."""
    nat = B._native
    boxes = [(101, [-1.0] * dim, [1.0] * dim), (3, [0.5] * dim, [0.75] * dim), (40, [-2.0] * dim, [0.0] * dim)]
    seed, U = 0xBADC0FFEE, 4
    per = sum(n for n, _, _ in boxes)
    st1 = torch.zeros(2, dtype=torch.int64, device="cuda")
    singles = [torch.cat(_draw(B, boxes, dim, seed, st1)) for _ in range(U)]
    st2 = torch.zeros(2, dtype=torch.int64, device="cuda")
    big = torch.full((U, per, dim), float("nan"), device="cuda")
    f3 = nat._F * 3
    arr = (nat.Box * len(boxes))()
    row = 0
    for k, (n, lo, hi) in enumerate(boxes):
        arr[k] = nat.Box(big.data_ptr() + 4 * dim * row, n, f3(*(list(lo) + [0.0] * (3 - dim))),
                         f3(*(list(hi) + [0.0] * (3 - dim))))
        row += n
    strides = (ctypes.c_long * len(boxes))(*([per * dim] * len(boxes)))
    nat.check(nat.lib().insr_sample_boxes_rep(arr, len(boxes), dim, U, strides, seed, nat.ptr(st2),
                                              nat.stream_of(0)), "rep")
    torch.cuda.synchronize()
    for r in range(U):
        assert torch.equal(big[r], singles[r]), r
    assert int(st2[0]) == int(st1[0]) and int(st2[1]) == 0
    # overlapping repetitions are refused
    bad = (ctypes.c_long * len(boxes))(*([1] * len(boxes)))
    assert nat.lib().insr_sample_boxes_rep(arr, len(boxes), dim, U, bad, seed, nat.ptr(st2), nat.stream_of(0)) != 0


@pytest.mark.gpu
def test_draw_ahead_one_launch_per_group(B):
    """Inside draw_ahead(U) the merged fluid draws of U iterations come from one launch, each iteration's
    buffer equal to what its own draw would have been (sample_random_and_bands2D(merged=True))."""
    lib = B._native.lib()
    from base.sampling import draw_ahead
    torch.manual_seed(5)
    ref = [B.sample_random_and_bands2D(1000, 10, merged=True).clone() for _ in range(4)]
    calls = []
    orig = lib.insr_sample_boxes_rep

    def spy(*a):
        calls.append(a[3])
        return orig(*a)
    lib.insr_sample_boxes_rep = spy
    try:
        torch.manual_seed(5)
        with draw_ahead(4):
            got = [B.sample_random_and_bands2D(1000, 10, merged=True) for _ in range(4)]
            extra = B.sample_random_and_bands2D(1000, 10, merged=True)  # a 5th call draws on its own
    finally:
        lib.insr_sample_boxes_rep = orig
    assert calls == [4, 1], calls
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    assert extra.shape == ref[0].shape
