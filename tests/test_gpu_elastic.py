"""The fused elasticity energy (base.elastic_energy -> insr_elastic_energy, one launch with the
unit-seed gradient) against the reference's energy expressions (elasticity/model.py:131-186,
elasticity/losses.py:6-39, restated in oracle/siren_oracle.py:281-356) evaluated in fp64 torch
on the same tensors.  Tolerances: total 1e-5 of the largest term; every term 1e-5 relative to fp64 or
within 3x the error of the reference's own fp32 evaluation (qdot = (q - q_prev)/dt cancels); gradients w.r.t. f 1e-5 and w.r.t. J 1e-4 normwise (a singular
value's gradient is ill-conditioned near repeated values, as in test_gpu_losses.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ALL2 = ["arap", "kinematics", "collision_sphere", "external", "volume", "constraint", "constraint_right"]
ALL3 = ["arap", "kinematics", "collision", "external", "volume", "constraint", "constraint_right_compress"]
SPH3 = ["arap", "kinematics", "collision_sphere", "external", "volume"]


@pytest.fixture(scope="module")
def B():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    return base


def rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def reference_terms(f, J, x, fp, fpp, n, rows_l, rows_r, cfg):
    """fp64 restatement of elasticity/model.py:131-186 on tensors (q = f + x, svdvals of J + I)."""
    d = x.shape[1]
    dt = cfg["dt"]
    q = f[:n] + x
    q_prev, q_pp = fp + x, fpp + x
    qdot = (q - q_prev) / dt
    qdot_prev = (q_prev - q_pp) / dt
    S = torch.linalg.svdvals(J[:n] + torch.eye(d, dtype=J.dtype))
    t = {}
    t["arap"] = cfg["ra"] * torch.sum((S - 1.0) ** 2)
    t["volume"] = cfg["rv"] * torch.sum((torch.prod(S, dim=1) - 1) ** 2)
    t["kinematics"] = cfg["rk"] * torch.sum((qdot - qdot_prev) ** 2)
    t["external"] = -dt * torch.sum(qdot * torch.tensor(cfg["ext"][:d], dtype=x.dtype))
    fl = f[rows_l[0]:rows_l[0] + rows_l[1]]
    fr = f[rows_r[0]:rows_r[0] + rows_r[1]]
    off = torch.tensor(cfg["offset"][:d], dtype=x.dtype)
    t["constraint"] = cfg["rc"] * torch.sum(fl ** 2)
    t["constraint_right"] = cfg["rc"] * torch.sum((fr - off) ** 2)
    t["constraint_right_compress"] = cfg["rc"] * torch.sum((fr + off) ** 2)
    hit = (q[:, -1] < cfg["h"]).to(x.dtype)
    t["collision"] = -dt * torch.sum(qdot[:, -1] * cfg["rcol"] * (cfg["h"] - q[:, -1]) * hit)
    vec = q - torch.tensor(cfg["center"][:d], dtype=x.dtype)
    dist = torch.sqrt(torch.sum(vec ** 2, dim=1))
    hs = (dist < cfg["radius"]).to(x.dtype)
    if d == 2:
        t["collision_sphere"] = -dt * torch.sum(qdot * (cfg["rcol"] * dist[:, None] * (vec / dist[:, None])) *
                                                hs[:, None])
    else:  # elasticity/losses.py:35-38: dist[:, None, None] * dir broadcasts to (K, K, 3) -- a product of sums
        hit = hs.bool()
        dh, dirh = dist[hit], vec[hit] / dist[hit][:, None]
        if int(hit.sum()) <= 3000:  # the reference's expression as written
            force = cfg["rcol"] * dh[:, None, None] * dirh
            t["collision_sphere"] = -dt * torch.sum(torch.mul(qdot[hit], force))
        else:  # the same sum without the K x K x 3 tensor
            t["collision_sphere"] = -dt * cfg["rcol"] * torch.sum(dh) * torch.sum(qdot[hit] * dirh)
    return t


def make_case(d, n, n_l, n_r, seed):
    g = torch.Generator().manual_seed(seed)
    rows = n + n_l + n_r
    f = 0.3 * torch.randn(rows, d, generator=g)
    J = 0.3 * torch.randn(rows, d, d, generator=g)
    x = torch.rand(n, d, generator=g) * 2 - 1
    fp = f[:n] + 0.05 * torch.randn(n, d, generator=g)
    fpp = fp + 0.05 * torch.randn(n, d, generator=g)
    cfg = dict(dt=0.1, ra=20.0, rv=1e3, rk=10.0, rc=1e4, rcol=1e4, ext=(0.3, -2e2, -1e2), offset=(2.0, 0.5, -0.25),
               h=-0.4, center=(0.1, -0.2, 0.0), radius=0.6)
    return f, J, x, fp, fpp, (n, n_l), (n + n_l, n_r), cfg


@pytest.mark.parametrize("d,energy", [(2, ALL2), (3, ALL3), (2, ["arap", "constraint", "constraint_right", "volume"]),
                                      (3, ["arap", "kinematics", "collision", "external", "volume"]),
                                      (3, SPH3), (3, ["collision_sphere"]),
                                      (2, ["kinematics", "external"])])
@pytest.mark.parametrize("n", [5, 3000, 70000])
def test_elastic_energy_matches_reference(B, d, energy, n):
    n_l = 40 if "constraint" in energy else 0
    n_r = 40 if any(e.startswith("constraint_right") for e in energy) else 0
    f, J, x, fp, fpp, rows_l, rows_r, cfg = make_case(d, n, n_l, n_r, 10 * n + d)
    use_svd = "arap" in energy or "volume" in energy
    f64, J64 = f.double().requires_grad_(True), J.double().requires_grad_(True)
    terms = reference_terms(f64, J64, x.double(), fp.double(), fpp.double(), n, rows_l, rows_r, cfg)
    # the reference's own fp32 evaluation: q - q_prev cancels (qdot), so the fp32 terms carry
    # rounding error of their own; a term must be within 1e-5 of fp64 or within 3x that error
    terms32 = reference_terms(f, J, x, fp, fpp, n, rows_l, rows_r, cfg)
    total64 = 0
    for e in energy:
        total64 = total64 + terms[e]
    gf64, gJ64 = torch.autograd.grad(total64, (f64, J64), allow_unused=True)
    fg, Jg = f.cuda().requires_grad_(True), J.cuda().requires_grad_(True)
    ratios = {"arap": cfg["ra"], "volume": cfg["rv"], "kinematics": cfg["rk"], "constraint": cfg["rc"],
              "constraint_right": cfg["rc"], "constraint_right_compress": cfg["rc"], "collision": cfg["rcol"],
              "collision_sphere": cfg["rcol"]}
    sign = -1.0 if "constraint_right_compress" in energy else 1.0
    total, per = B.elastic_energy(fg, Jg if use_svd else None, x.cuda(), fp.cuda(), fpp.cuda(), n=n, dt=cfg["dt"],
                                  energy=energy, ratios=ratios, ext=cfg["ext"][:d], rows_l=rows_l, rows_r=rows_r,
                                  target=[sign * v for v in cfg["offset"][:d]], plane_height=cfg["h"],
                                  center=cfg["center"][:d], radius=cfg["radius"])
    scale = max(abs(float(terms[e])) for e in energy)
    assert abs(float(total) - float(total64)) <= 1e-5 * scale, (float(total), float(total64))
    ids = B._native.EL_IDS
    for e in energy:
        t = ids["constraint_right" if e == "constraint_right_compress" else e]
        err32 = abs(float(terms32[e]) - float(terms[e]))
        tol = max(1e-5 * max(abs(float(terms[e])), 1e-6 * scale), 3 * err32)
        assert abs(float(per[t]) - float(terms[e])) <= tol, (e, float(per[t]), float(terms[e]), err32)
    # unit seed (the training loop's): gradients written by the forward launch
    seed = B.losses.register_unit_seed(torch.ones((), device="cuda"))
    gf, gJ = torch.autograd.grad(total, (fg, Jg), grad_outputs=seed, allow_unused=True, retain_graph=True)
    assert rel(gf, gf64) < 1e-5
    if use_svd:
        assert rel(gJ, gJ64) < 1e-4 and float(gJ[n:].abs().sum()) == 0.0
    else:
        assert gJ is None
    # a non-unit seed scales them
    gf2, = torch.autograd.grad(total * 3.0, (fg,))
    assert rel(gf2 / 3.0, gf64) < 1e-5


def test_elastic_energy_rejects(B):
    with pytest.raises(B.NativeUnavailable):
        B.elastic_energy(torch.zeros(10, 2), None, torch.zeros(10, 2), torch.zeros(10, 2), torch.zeros(10, 2), n=10,
                         dt=0.1, energy=["kinematics"], ratios={"kinematics": 1.0})


def test_svd_terms_with_zero_ratio_give_zero_jacobian_gradient(B):
    """arap / volume listed with ratio 0: the kernel writes no dE/dJ, the gradient is exactly zero
    (not uninitialised memory), and constraint_right with _compress together is refused."""
    f, J, x, fp, fpp, rows_l, rows_r, cfg = make_case(2, 3000, 0, 0, 77)
    fg, Jg = f.cuda().requires_grad_(True), J.cuda().requires_grad_(True)
    torch.empty(8 << 20, device="cuda").fill_(float("nan"))  # dirty the caching allocator's blocks
    total, _ = B.elastic_energy(fg, Jg, x.cuda(), fp.cuda(), fpp.cuda(), n=3000, dt=0.1,
                                energy=["arap", "volume", "kinematics"],
                                ratios={"arap": 0.0, "volume": 0.0, "kinematics": 2.0})
    seed = B.losses.register_unit_seed(torch.ones((), device="cuda"))
    gf, gJ = torch.autograd.grad(total, (fg, Jg), grad_outputs=seed)
    assert float(gJ.abs().sum()) == 0.0 and torch.isfinite(gf).all()
    with pytest.raises(B.UnsupportedPattern):
        B.elastic_energy(fg, None, x.cuda(), fp.cuda(), fpp.cuda(), n=3000, dt=0.1,
                         energy=["constraint_right", "constraint_right_compress"],
                         ratios={"constraint_right": 1.0, "constraint_right_compress": 1.0})


def test_box_batch_layout_and_energy(B):
    """ElasticityModel._box_batch (one sampler launch into a persistent [x; fixed_l; fixed_r]
    buffer): the layout _sample_in_training / _sample_fixed_in_training / merge_samples give --
    random rows in the box / on the faces, grid rows equal to sample_uniform, fresh draws every
    iteration -- and the energy on it equals energy_of on the same points merged by merge_samples."""
    from pde.config import baseline_config
    from pde.elasticity import ElasticityModel
    cfg = baseline_config("elasticity2Dstretch", proj_dir="/tmp/insr_test", insr_progress=False, sample_resolution=20,
                          num_hidden_layers=2, hidden_features=64)
    torch.manual_seed(0)
    m = ElasticityModel(cfg)
    m.timestep = 1
    xa, x, fl, fr = m._box_batch(20)
    n = 2 * 400
    assert x.shape == (n, 2) and fl.shape == (40, 2) and fr.shape == (40, 2) and xa.shape == (n + 80, 2)
    a = xa.detach().clone()
    grid = B.sample_uniform(20, 2, device="cuda")
    assert torch.equal(a[400:800], grid)
    assert float(a[:400].abs().max()) <= 1.0
    assert torch.equal(a[n:n + 20, 0], torch.full((20,), -1.0, device="cuda"))
    assert torch.equal(a[n + 20:n + 40, 1], B.sample_uniform(20, 1, device="cuda")[:, 0])
    assert torch.equal(a[n + 40:, 0], torch.full((40,), 1.0, device="cuda"))
    xa2 = m._box_batch(20)[0]
    assert xa2 is xa and not torch.equal(xa.detach()[:400], a[:400]) and torch.equal(xa.detach()[400:800], grid)
    e_fast = m.energy_of(x, fl, fr, xa=xa)
    xs, fls, frs = (t.detach().clone().requires_grad_(True) for t in (x, fl, fr))
    e_ref = m.energy_of(xs, fls, frs)
    assert float(e_fast) == float(e_ref)
