"""Parity at the BASELINE.json sizes (SURVEY.md §8 d): the HIP jets against the CPU oracle
on the full fluid2Dtlgn batch (16384 points, SIREN 4x128: pressure Laplacian jet, velocity
divergence) and on a 32768-point shard of elasticity3Dbunny (SIREN 5x256 Jacobian jet, the
two-kernel W = 256 backward), including the parameter gradients of a loss of each.
Tolerance (north_star): 1e-5 relative, normwise per tensor (max |hip - ref| / max |ref|)."""
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-5


def nerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope="module")
def base():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base as B
    B._native.load()
    return B


def pair(B, din, dout, L, W, seed):
    torch.manual_seed(seed)
    ref = O.OracleSiren(din, dout, L, W)
    torch.manual_seed(seed)
    net = B.MLP(din, dout, L, W, nonlinearity="sine").cuda()
    return ref, net


def grads(net):
    return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1).cpu()
                      for p in net.parameters()])


def test_fluid2dtlgn_pressure_full_batch(base):
    """fluid/model.py:110-125 at 128^2 points: lap p, and d/dtheta mean((g - lap p)^2)."""
    ref, net = pair(base, 2, 1, 4, 128, 11)
    torch.manual_seed(5)
    x = torch.rand(16384, 2) * 2 - 1
    g = torch.randn(16384, 1)
    xr = x.clone().requires_grad_(True)
    lr_ = O.op_laplace(ref(xr), xr)
    ((g - lr_) ** 2).mean().backward()
    xg = x.cuda().requires_grad_(True)
    lg = base.laplace(net(xg), xg)
    ((g.cuda() - lg) ** 2).mean().backward()
    assert nerr(lg, lr_) < TOL
    assert nerr(grads(net), grads(ref)) < TOL


def test_fluid2dtlgn_velocity_divergence_full_batch(base):
    ref, net = pair(base, 2, 2, 4, 128, 12)
    x = torch.rand(16384, 2, generator=torch.Generator().manual_seed(6)) * 2 - 1
    xr = x.clone().requires_grad_(True)
    dr = O.op_divergence(ref(xr), xr)
    xg = x.cuda().requires_grad_(True)
    with torch.no_grad():
        dg = base.divergence(net(xg), xg)
    assert nerr(dg, dr) < TOL


def test_elasticity3d_jacobian_shard(base):
    """elasticity/model.py:137-147 on a 32768-point shard (8-GPU strong scaling of 64^3):
    J of q = f(x) + x and the parameter gradient of sum(J^2) (W = 256 two-kernel backward)."""
    ref, net = pair(base, 3, 3, 5, 256, 13)
    x = torch.rand(32768, 3, generator=torch.Generator().manual_seed(7)) * 2 - 1
    xr = x.clone().requires_grad_(True)
    Jr, _ = O.op_jacobian(ref(xr) + xr, xr)
    (Jr ** 2).sum().backward()
    xg = x.cuda().requires_grad_(True)
    Jg, st = base.jacobian(net(xg) + xg, xg)
    (Jg ** 2).sum().backward()
    assert st == 0
    assert nerr(Jg, Jr) < TOL
    assert nerr(grads(net), grads(ref)) < TOL


# ---- fluid2DtlgnM (BASELINE.json configs[4]): 256^2 = 65,536 points, default kernel routing ----
def test_fluid2dtlgnM_pressure_laplacian_65536(base):
    """fluid/model.py:110-125 at 256^2 points: the W = 128 Laplacian backward takes the
    two-kernel path by default at this size (propagation kernel + split-K dW GEMM over
    K = 65,536 x 4); lap p and d/dtheta mean((g - lap p)^2) vs the oracle."""
    lib = base._native.lib()
    assert lib.insr_jet_bwd_is_wide(65536, 2, 128, base._native.MODE_LAP) == 1  # default routing
    ref, net = pair(base, 2, 1, 4, 128, 31)
    torch.manual_seed(32)
    x = torch.rand(65536, 2) * 2 - 1
    g = torch.randn(65536, 1)
    xr = x.clone().requires_grad_(True)
    lr_ = O.op_laplace(ref(xr), xr)
    ((g - lr_) ** 2).mean().backward()
    xg = x.cuda().requires_grad_(True)
    lg = base.laplace(net(xg), xg)
    ((g.cuda() - lg) ** 2).mean().backward()
    assert nerr(lg, lr_) < TOL
    assert nerr(grads(net), grads(ref)) < TOL
    for (k, a), b in zip(ref.named_parameters(), net.parameters()):  # every tensor on its own
        ga = a.grad if a.grad is not None else torch.zeros_like(a)
        gb = b.grad if b.grad is not None else torch.zeros_like(b)
        if ga.abs().max() > 0:
            assert nerr(gb, ga) < TOL, k


def test_fluid2dtlgnM_velocity_jets_65536(base):
    """divergence (detached, fluid/model.py:109) and the trainable value + gradient jet of the
    velocity net (wall terms / projection) at 65,536 points, with parameter gradients."""
    ref, net = pair(base, 2, 2, 4, 128, 33)
    x = torch.rand(65536, 2, generator=torch.Generator().manual_seed(34)) * 2 - 1
    xr = x.clone().requires_grad_(True)
    dr = O.op_divergence(ref(xr), xr)
    xg = x.cuda().requires_grad_(True)
    with torch.no_grad():
        dg = base.divergence(net(xg), xg)
    assert nerr(dg, dr) < TOL
    R = torch.randn(65536, 2, generator=torch.Generator().manual_seed(35))
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    Gr = O.op_gradient(yr, xr)
    ((yr * R).sum() + (Gr * R).sum()).backward()
    xg = x.cuda().requires_grad_(True)
    y = net(xg)
    G = base.gradient(y, xg)
    ((y * R.cuda()).sum() + (G * R.cuda()).sum()).backward()
    assert nerr(G, Gr) < TOL and nerr(y, yr) < TOL
    assert nerr(grads(net), grads(ref)) < TOL


def test_taylorgreen_multi_on_device():
    """pde.examples.taylor_green_multi on the GPU vs the reference's own values
    (fluid/examples.py:34-51, tests/golden/ref_extra.npz)."""
    import os
    import numpy as np
    from pde.examples import get_examples
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_extra.npz"))
    got = get_examples("taylorgreen_multi")(torch.from_numpy(d["examples/x"]).cuda()).cpu().numpy()
    want = d["examples/taylorgreen_multi"]
    assert np.abs(got - want).max() <= 1e-6 * np.abs(want).max()


def _fluidM(graph):
    from pde.config import baseline_config
    from pde.fluid import Fluid2DModel
    cfg = baseline_config("fluid2DtlgnM", proj_dir="/tmp/insr_test_m", insr_progress=False, early_stop=False,
                          max_n_iters=6, insr_graph=graph, insr_sync_every=1)
    torch.manual_seed(7)
    m = Fluid2DModel(cfg)
    m.timestep = 1
    torch.manual_seed(8)
    m.velocity_field_prev.load_state_dict({k: v + 1e-3 * torch.randn_like(v)
                                           for k, v in m.velocity_field.state_dict().items()})
    return m


def test_fluid2dtlgnM_full_phases_graph_equals_eager(base):
    """One fluid2DtlgnM timestep's three phases at 65,536 points (+ 2 x 654 band points),
    6 iterations each, device sampler: hipGraph replay equals eager execution bit for bit,
    every loss finite, and the pressure fit decreasing."""
    from base import sampling
    res = {}
    for graph in (False, True):
        sampling._SAMPLER.clear()  # the same Philox draws in both runs
        m = _fluidM(graph)
        trace = {}
        for phase in ("_advect_velocity", "_solve_pressure", "_projection"):
            rec = []
            m.tb = type("TB", (), {"add_scalars": lambda self, tag, vals, global_step: rec.append(vals)})()
            getattr(m, phase)()
            assert getattr(m, "_insr_capture_error", None) is None
            trace[phase] = rec
        torch.cuda.synchronize()
        res[graph] = (m.velocity_field.flat_params().detach().cpu(), m.pressure_field.flat_params().detach().cpu(),
                      trace)
    assert torch.equal(res[True][0], res[False][0]) and torch.equal(res[True][1], res[False][1])
    for phase, rec in res[True][2].items():
        assert len(rec) == 6 and rec == res[False][2][phase], phase
        assert all(torch.isfinite(torch.tensor(list(r.values()))).all() for r in rec), phase
    pres = [r["main"] for r in res[True][2]["_solve_pressure"]]
    assert pres[-1] < pres[0]


@pytest.mark.parametrize("case", ["value16708", "value20400"])
def test_balanced_launch_shapes(base, case):
    """Batches just above a multiple of the resident block slots run balanced blocks of T + 1
    tiles (16384 interior + 324 band points: value jets 4 -> 5 tiles per block, gradient jets
    2 -> 3 in the forward): values, derivatives and parameter gradients vs the oracle."""
    mode, n = case[:-5], int(case[-5:])
    lib = base._native.lib()
    m = base._native.MODE_VALUE if mode == "value" else base._native.MODE_GRAD
    T_fwd, T_bwd = lib.insr_jet_split_tiles(n, 2, 128, m, 0), lib.insr_jet_split_tiles(n, 2, 128, m, 1)
    assert {T_fwd, T_bwd} & {3, 5}, (T_fwd, T_bwd)  # the case runs a balanced shape
    ref, net = pair(base, 2, 2, 4, 128, 41)
    x = torch.rand(n, 2, generator=torch.Generator().manual_seed(42)) * 2 - 1
    R = torch.randn(n, 2, 2, generator=torch.Generator().manual_seed(43))
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    vr = yr if mode == "value" else O.op_jacobian(yr, xr)[0]
    (vr * (R[..., 0] if mode == "value" else R)).sum().backward()
    xg = x.cuda().requires_grad_(True)
    y = net(xg)
    v = y if mode == "value" else base.jacobian(y, xg)[0]
    (v * (R[..., 0] if mode == "value" else R).cuda()).sum().backward()
    assert nerr(v, vr) < TOL
    assert nerr(grads(net), grads(ref)) < TOL


def test_fused_multi_five_tile_blocks(base):
    """The fluid advection's fused forward: the frozen field at 16384 interior points and the
    trainable one at 16384 + 324 band points in one launch of 5-tile blocks (518 four-tile
    blocks would overflow the 512 resident slots): both outputs and the trainable field's
    parameter gradients vs the oracle."""
    refp, prev = pair(base, 2, 2, 4, 128, 51)
    refc, cur = pair(base, 2, 2, 4, 128, 52)
    for p in prev.parameters():
        p.requires_grad_(False)
    buf = torch.rand(16708, 2, generator=torch.Generator().manual_seed(53)) * 2 - 1
    R = torch.randn(16708, 2, generator=torch.Generator().manual_seed(54))
    xb = buf.cuda().requires_grad_(True)
    with base.fused_forwards():
        with torch.no_grad():
            up = prev(xb[:16384])
        ua = cur(xb)
    (ua * R.cuda()).sum().backward()
    assert nerr(up, refp(buf[:16384])) < TOL
    xr = buf.clone().requires_grad_(True)
    yr = refc(xr)
    (yr * R).sum().backward()
    assert nerr(ua, yr) < TOL
    assert nerr(grads(cur), grads(refc)) < TOL


@pytest.mark.parametrize("shape,n", [((3, 1, 4, 128), 10000), ((3, 2, 3, 256), 4096)])
def test_laplacian_3d_input(base, shape, n):
    """laplace with a 3-d input (5-stream jet; base/diff_ops.py:33-41): values and parameter
    gradients vs the oracle, through the default routing (W = 128 from 8,192 points and W = 256:
    the two-kernel backward)."""
    din, dout, L, W = shape
    ref, net = pair(base, din, dout, L, W, 21)
    x = torch.rand(n, din, generator=torch.Generator().manual_seed(7)) * 2 - 1
    g = torch.randn(n, 1, generator=torch.Generator().manual_seed(8))
    xr = x.clone().requires_grad_(True)
    lr_ = O.op_laplace(ref(xr), xr)
    ((g - lr_) ** 2).mean().backward()
    xg = x.cuda().requires_grad_(True)
    lg = base.laplace(net(xg), xg)
    ((g.cuda() - lg) ** 2).mean().backward()
    assert nerr(lg, lr_) < TOL
    assert nerr(grads(net), grads(ref)) < TOL
