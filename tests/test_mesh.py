"""Mesh input (pde/mesh.py; the reference's meshio + torchgp path, elasticity/model.py:75-93,
198-207, elasticity/torchgp/*.py).  CPU tests: a MEDIT cube written here (exact volumes,
faces and sample moments), and -- when /root/reference is present (build container only)
-- the reference's own bunny.mesh, whose file carries the surface triangles that
boundary_faces() must reproduce from the tets.  Sampling parity is distributional (the
reference draws with numpy / torch.distributions): checked by exact containment and
moment tests."""
import os

import numpy as np
import pytest
import torch

from pde import mesh as M

# unit cube [-1, 1]^3 split into 6 tets around the main diagonal (0 -> 6)
CUBE_V = np.array([[x, y, z] for z in (-1, 1) for y in (-1, 1) for x in (-1, 1)], np.float64)
CUBE_T = np.array([[0, 1, 3, 7], [0, 1, 5, 7], [0, 2, 3, 7], [0, 2, 6, 7], [0, 4, 5, 7], [0, 4, 6, 7]])


def write_medit(path, V, T, F=None):
    with open(path, "w") as f:
        f.write("MeshVersionFormatted 1\nDimension 3\nVertices\n%d\n" % len(V))
        for v in V:
            f.write("%.17g %.17g %.17g 1\n" % tuple(v))
        if F is not None:
            f.write("Triangles\n%d\n" % len(F))
            for t in F:
                f.write("%d %d %d 1\n" % tuple(t + 1))
        f.write("Tetrahedra\n%d\n" % len(T))
        for t in T:
            f.write("%d %d %d %d 1\n" % tuple(t + 1))
        f.write("End\n")


@pytest.fixture
def cube(tmp_path):
    p = tmp_path / "cube.mesh"
    write_medit(str(p), CUBE_V, CUBE_T)
    return str(p)


def test_read_medit_cube(cube):
    V, blocks = M.read_medit(cube)
    assert V.shape == (8, 3) and np.array_equal(V, CUBE_V)
    assert np.array_equal(blocks["Tetrahedra"], CUBE_T)  # 1-based file -> 0-based, tag dropped


def test_volumes_and_boundary(cube):
    V, blocks = M.read_medit(cube)
    vol = M.tet_volumes(torch.as_tensor(V), torch.as_tensor(blocks["Tetrahedra"]))
    assert torch.allclose(vol, torch.full((6,), 8.0 / 6.0, dtype=vol.dtype))
    SF = M.boundary_faces(blocks["Tetrahedra"])
    assert SF.shape == (12, 3)  # 6 cube faces x 2 triangles; interior faces appear twice
    # every boundary triangle lies in one cube face (one coordinate constant at +-1)
    tri = CUBE_V[SF]
    assert all(np.any(np.all(np.abs(t - t[0]) == 0, axis=0) & (np.abs(t[0]) == 1)) for t in tri)


def test_normalize_matches_reference_rule():
    V = torch.tensor([[0.0, 0.0, 0.0], [2.0, 4.0, 0.0], [1.0, 0.0, 6.0]], dtype=torch.float64)
    N = M.normalize(V)
    c = V - torch.tensor([1.0, 2.0, 3.0], dtype=torch.float64)  # bbox centre
    assert torch.allclose(N, c / c.norm(dim=1).max())
    assert abs(float(N.norm(dim=1).max()) - 1.0) < 1e-15


def test_volume_sampler_uniform_in_cube():
    s = M.MeshSampler(CUBE_V, CUBE_T)
    g = torch.Generator().manual_seed(0)
    x = s.sample(200000, generator=g).double()
    assert x.shape == (200000, 3)
    assert float(x.abs().max()) <= 1.0 + 1e-6
    # uniform on [-1, 1]^3: mean 0, variance 1/3, and each of the 6 equal tets gets 1/6
    assert torch.allclose(x.mean(0), torch.zeros(3, dtype=x.dtype), atol=6e-3)
    assert torch.allclose(x.var(0), torch.full((3,), 1.0 / 3.0, dtype=x.dtype), atol=6e-3)
    octant = ((x > 0).long() * torch.tensor([1, 2, 4])).sum(1)
    frac = torch.bincount(octant, minlength=8).double() / x.shape[0]
    assert torch.allclose(frac, torch.full((8,), 0.125, dtype=frac.dtype), atol=5e-3)


def test_volume_sampler_weights_by_volume():
    # two tets sharing a face, volumes 1/6 and 3/6: 25% / 75% of the samples
    V = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1], [0, 0, -3]], np.float64)
    T = np.array([[0, 1, 2, 3], [0, 1, 2, 4]])
    s = M.MeshSampler(V, T)
    x = s.sample(100000, generator=torch.Generator().manual_seed(1))
    assert abs(float((x[:, 2] > 0).double().mean()) - 0.25) < 6e-3
    # containment: barycentric coordinates of every sample are >= 0 in its tet
    up = x[x[:, 2] > 0].double()
    assert float(up.min()) >= -1e-6 and float(up.sum(1).max()) <= 1.0 + 1e-6


def test_triangle_sampler_area_weighted():
    V = np.array([[0, 0], [1, 0], [0, 1], [-2, 0]], np.float64)  # areas 0.5 and 1.0
    F = np.array([[0, 1, 2], [0, 2, 3]])
    s = M.MeshSampler(V, F)
    x = s.sample(90000, generator=torch.Generator().manual_seed(2))
    assert abs(float((x[:, 0] > 0).double().mean()) - 1.0 / 3.0) < 6e-3
    right = x[x[:, 0] > 0].double()
    assert torch.allclose(right.mean(0), torch.tensor([1 / 3, 1 / 3], dtype=right.dtype), atol=5e-3)  # centroid


@pytest.mark.gpu
def test_elasticity_model_mesh_phase(cube):
    """The model on a mesh (GPU: the product path has no CPU fallback): samples inside the
    normalised mesh, the mesh vertices as the 'uniform' set, and one _solve_deformation
    iteration (jets + fused SVD energy + Adam) with a finite loss that matches the oracle's
    on the same samples."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base
    from oracle import siren_oracle as O
    from pde.config import make_config
    from pde.elasticity import ElasticityModel
    cfg = make_config("elasticity", dim=3, use_mesh=True, mesh_path=cube, sample_resolution=8,
                      sample_pattern=["random", "uniform"], num_hidden_layers=1, hidden_features=32,
                      energy=["arap", "kinematics", "external", "volume"], external_force_z=-1.0,
                      proj_dir="/tmp/insr_test_mesh")
    model = ElasticityModel(cfg)
    x = model._sample_in_training(8)
    assert x.shape == (8 ** 3 + 8, 3) and x.requires_grad
    r = 2.0 / np.sqrt(3.0)  # normalised cube (farthest vertex at 1) scaled by 2
    assert float(x.abs().max()) <= r + 1e-5
    assert torch.allclose(x[-8:].detach().cpu().double(), torch.as_tensor(CUBE_V) * r, atol=1e-6)
    fl, fr = model._sample_fixed_in_training(8)
    assert fl.shape == (0, 3) and fr.shape == (0, 3)
    base._native.load()
    model.timestep = 1
    xs = x.detach().clone()
    model._sample_in_training = lambda res: xs.clone().requires_grad_(True)
    body = ElasticityModel._solve_deformation._insr_phase
    model._reset_optimizer()
    ld = body(model)
    ecfg = dict(dt=cfg.dt, energy=list(cfg.energy), ratio_arap=cfg.ratio_arap, ratio_volume=cfg.ratio_volume,
                ratio_kinematics=cfg.ratio_kinematics, ratio_constraint=cfg.ratio_constraint,
                ratio_collide=cfg.ratio_collide, plane_height=cfg.plane_height,
                external_force=[cfg.external_force_x, cfg.external_force_y, cfg.external_force_z],
                constraint_offset_right=[0.0, 0.0, 0.0], circle_center=[0.0, 0.0, 0.0], circle_radius=1.0,
                external_force_timesteps=cfg.external_force_timesteps)
    nets = []
    for net in (model.deformation_field, model.deformation_field_prev, model.deformation_field_prev_prev):
        o = O.OracleSiren(3, 3, 1, 32)
        with torch.no_grad():
            for po, pn in zip(o.parameters(), net.parameters()):
                po.copy_(pn.detach().cpu())
        nets.append(o)
    xr = xs.cpu().requires_grad_(True)
    ref = O.elasticity_loss(nets[0], nets[1], nets[2], xr, None, None, ecfg)["main"]
    assert np.isfinite(float(ld["main"]))
    assert abs(float(ld["main"]) - float(ref)) <= 1e-5 * abs(float(ref)) + 1e-6


REF_BUNNY = "/root/reference/elasticity/data/bunny.mesh"


@pytest.mark.skipif(not os.path.exists(REF_BUNNY), reason="reference tree not mounted")
def test_reference_bunny_mesh():
    V, blocks = M.read_medit(REF_BUNNY)
    T, F = blocks["Tetrahedra"], blocks["Triangles"]
    assert V.shape == (18592, 3) and T.shape == (76854, 4) and F.shape == (20522, 3)
    assert T.min() == 0 and T.max() == V.shape[0] - 1
    SF = M.boundary_faces(T)
    # the file's surface triangles are exactly the tets' boundary faces (as sets of vertices)
    key = lambda A: set(map(tuple, np.sort(A, axis=1)))  # noqa: E731
    assert key(SF) == key(F)
    vol = M.tet_volumes(torch.as_tensor(V), torch.as_tensor(T))
    assert bool(torch.all(vol > 0))
    Vn, E, _ = M.load_mesh(REF_BUNNY, 3)
    assert abs(float(Vn.norm(dim=1).max()) - 2.0) < 1e-5


BUNNY_NPZ = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bunny_mesh.npz")


def test_bunny_fixture_loads_like_the_reference_mesh():
    """The derived fixture (tests/golden/make_bunny_fixture.py) is what the elasticity3Dbunny
    bench trains on: same vertex / tet counts as the reference's bunny.mesh, positive tet
    volumes, normalised radius 2, and -- where the reference tree is mounted -- the same
    loaded arrays as reading the .mesh itself."""
    Vn, E, SF = M.load_mesh(BUNNY_NPZ, 3)
    assert Vn.shape == (18592, 3) and E.shape == (76854, 4) and SF.shape == (20522, 3)
    assert abs(float(Vn.norm(dim=1).max()) - 2.0) < 1e-5
    vol = M.tet_volumes(Vn.double(), torch.as_tensor(E))
    assert bool(torch.all(vol > 0))
    if os.path.exists(REF_BUNNY):
        Vr, Er, SFr = M.load_mesh(REF_BUNNY, 3)
        assert torch.equal(Vn, Vr) and np.array_equal(E, Er) and np.array_equal(SF, SFr)
