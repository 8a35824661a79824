"""The reference MLP's configurations the HIP jets do not serve (base/networks.py:30-71: relu / elu
networks, outermost_linear=False, a SIREN wider than 256): base.MLP builds them as TorchMLP -- the
reference's module tree in plain torch ops -- and their derivatives take the reference's autograd
route.  Pinned to tests/golden/ref_nets.npz, made by running the reference itself
(tests/golden/make_golden.py --nets): init bit for bit, value, gradient and the parameter gradients of
a fixed functional at 1e-5 normwise.  CPU here; tests/test_gpu_fallback.py repeats it on the GPU."""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_nets.npz")
NAMES = ["relu", "elu", "sine_nonlinear_out", "relu_nonlinear_out", "sine_w300"]


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLD) as z:
        return {k: z[k] for k in z.files}


def _nw(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def check_net(base, gold, name, device):
    din, dout, L, W, olin = [int(v) for v in gold[f"{name}/shape"]]
    nl = str(gold[f"{name}/nonlinearity"])
    torch.manual_seed(int(gold[f"{name}/seed"]))
    net = base.MLP(din, dout, L, W, outermost_linear=bool(olin), nonlinearity=nl)
    assert type(net).__name__ == "TorchMLP"
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).numpy()
    assert np.array_equal(flat, gold[f"{name}/params"])  # the reference's init, bit for bit
    net = net.to(device)
    x = torch.from_numpy(gold[f"{name}/x"]).to(device).requires_grad_(True)
    y = net(x)
    g = base.gradient(y, x)
    assert _nw(y.detach().cpu(), gold[f"{name}/y"]) < 1e-5
    assert _nw(g.detach().cpu(), gold[f"{name}/gradient"]) < 1e-5
    ry = torch.from_numpy(gold[f"{name}/y_R"]).to(device)
    rg = torch.from_numpy(gold[f"{name}/gradient_R"]).to(device)
    ((y * ry).sum() + (g * rg).sum()).backward()
    pg = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in net.parameters()])
    ref = gold[f"{name}/pgrad"]
    if np.abs(ref).max() > 0:
        assert _nw(pg.detach().cpu(), ref) < 1e-5
    sd = net.state_dict()
    assert list(sd)[0] == "net.0.weight" and list(sd)[-1] == f"net.{2 * (L + 1)}.bias"


@pytest.mark.parametrize("name", NAMES)
def test_other_networks_match_reference(gold, name):
    import base
    check_net(base, gold, name, "cpu")


def test_siren_stays_on_the_hip_path():
    import base
    net = base.MLP(2, 1, 4, 128, nonlinearity="sine")
    assert isinstance(net, base.MLP) and net.kernel_width == 128
    with pytest.raises(base._native.NativeUnavailable):
        net(torch.zeros(4, 2))  # the SIREN hot path has no CPU route
