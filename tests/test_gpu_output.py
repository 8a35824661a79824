"""Output path (SURVEY.md §8 f row 4): the quantities write_output exports, against the
oracle on the same weights -- fluid velocity / speed / curl on the visualisation grid
(fluid/model.py:207-232) and the deformed elasticity samples (elasticity/model.py:277-317)."""
import os

import numpy as np
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-5


def nerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def oracle_copy(net, din, dout, L, W):
    o = O.OracleSiren(din, dout, L, W)
    with torch.no_grad():
        for po, pn in zip(o.parameters(), net.parameters()):
            po.copy_(pn.detach().cpu())
    return o


@pytest.fixture(scope="module")
def base():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import base as B
    B._native.load()
    return B


def test_fluid_output(base, tmp_path):
    from pde.config import make_config
    from pde.fluid import Fluid2DModel
    torch.manual_seed(3)
    cfg = make_config("fluid", num_hidden_layers=2, hidden_features=64, vis_resolution=40,
                      proj_dir=str(tmp_path))
    model = Fluid2DModel(cfg)
    model.timestep = 7
    u, mag, curl, grid = model.field_quantities(40)
    ref = oracle_copy(model.velocity_field, 2, 2, 2, 64)
    g = grid.cpu().reshape(-1, 2).requires_grad_(True)
    ur = ref(g)
    J, _ = O.op_jacobian(ur, g)
    assert nerr(u.cpu().reshape(-1, 2), ur.detach()) < TOL
    assert nerr(mag.cpu().reshape(-1), ur.detach().norm(dim=-1)) < TOL
    assert nerr(curl.cpu().reshape(-1), (J[:, 1, 0] - J[:, 0, 1]).detach()) < TOL
    out = tmp_path / "results"
    model.write_output(str(out))
    arr = np.load(out / "t007.npy")
    assert arr.shape == (40, 40, 2) and nerr(arr.reshape(-1, 2), ur.detach().numpy()) < TOL
    assert np.load(out / "t007_curl.npy").shape == (40, 40)


def test_elasticity_output(base, tmp_path):
    from pde.config import make_config
    from pde.elasticity import ElasticityModel
    torch.manual_seed(4)
    cfg = make_config("elasticity", dim=2, num_hidden_layers=2, hidden_features=64, vis_resolution=20,
                      proj_dir=str(tmp_path))
    model = ElasticityModel(cfg)
    model.timestep = 2
    q = model.deformed_points(20)
    x = model.sample_visualization(20).cpu()
    assert x.shape == (20 * 20 + 2 * 20, 2)
    ref = oracle_copy(model.deformation_field, 2, 2, 2, 64)
    qr = (ref(x) + x).detach()
    assert nerr(q.cpu(), qr) < TOL
    out = tmp_path / "results"
    model.write_output(str(out))
    ply = open(out / "t002_deformation.ply").read().split("end_header\n")
    pts = np.loadtxt(ply[1].splitlines())
    assert pts.shape == (440, 3) and np.all(pts[:, 2] == 0) and nerr(pts[:, :2], qr.numpy()) < 1e-6


@pytest.mark.parametrize("pde,kw,nets", [
    ("fluid", dict(num_hidden_layers=4, hidden_features=128), {"velocity": (2, 2), "pressure": (2, 1)}),
    ("elasticity", dict(dim=2, num_hidden_layers=3, hidden_features=68), {"deformation": (2, 2)}),  # padded width
])
def test_model_checkpoint_roundtrip(base, tmp_path, pde, kw, nets):
    """BaseModel.save_ckpt / load_ckpt (base/baseModel.py:137-162): the file holds the reference's
    layout ({'net_<name>': state_dict with the reference MLP's keys and shapes, 'timestep'}), a
    reference network loads it and computes the same field, and load_ckpt into a fresh model
    restores the parameters bit for bit (jets included: the weight planes follow the load)."""
    from pde.config import make_config
    import pde.fluid as F
    import pde.elasticity as E
    M = F.Fluid2DModel if pde == "fluid" else E.ElasticityModel
    cfg = make_config(pde, proj_dir=str(tmp_path), insr_progress=False, **kw)
    torch.manual_seed(3)
    a = M(cfg)
    a.timestep = 7
    a.save_ckpt("rt")
    path = os.path.join(cfg.model_dir, "ckpt_rt.pth")
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert sorted(ck) == sorted([f"net_{k}" for k in nets] + ["timestep"]) and ck["timestep"] == 7
    x = torch.rand(300, 2) * 2 - 1
    L, W = kw["num_hidden_layers"], kw["hidden_features"]
    for key, (din, dout) in nets.items():
        ref = O.OracleSiren(din, dout, L, W)
        assert [(k, tuple(v.shape)) for k, v in ck[f"net_{key}"].items()] == \
            [(k, tuple(v.shape)) for k, v in ref.state_dict().items()]
        ref.load_state_dict(ck[f"net_{key}"])
        net = a._trainable_networks[key]
        with torch.no_grad():
            assert nerr(net(x.cuda()).cpu(), ref(x)) < TOL
    torch.manual_seed(4)
    b = M(cfg)
    b.load_ckpt("rt")
    assert b.timestep == 7
    for key in nets:
        na, nb = a._trainable_networks[key], b._trainable_networks[key]
        assert torch.equal(na.flat_params(), nb.flat_params())
        xg = x.cuda().requires_grad_(True)
        assert torch.equal(base.jacobian(na(xg), xg)[0], base.jacobian(nb(xg), xg)[0])
