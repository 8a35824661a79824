"""base.MLP storage on the CPU (no kernel calls): reference init bit for bit, state_dict
keys and shapes, the flat (zero-padded) layout of widths that are not compiled, and the
checkpoint round trip in the reference's layout (base/baseModel.py:137-162)."""
import pytest
import torch

from oracle import siren_oracle as O


@pytest.fixture(scope="module")
def B():
    import base
    return base


@pytest.mark.parametrize("shape", [(1, 1, 2, 20), (2, 2, 3, 68), (3, 3, 3, 66), (2, 1, 4, 128), (2, 3, 1, 40)])
def test_padded_layout_matches_reference_init(B, shape):
    din, dout, L, W = shape
    torch.manual_seed(3)
    ref = O.OracleSiren(din, dout, L, W)
    torch.manual_seed(3)
    net = B.MLP(din, dout, L, W, nonlinearity="sine")
    Wp = B.networks.kernel_width(W)
    assert net.kernel_width == Wp and Wp in (32, 64, 128, 256) and Wp >= W
    sd, rsd = net.state_dict(), ref.state_dict()
    assert list(sd) == list(rsd)
    for k in sd:
        assert sd[k].shape == rsd[k].shape and torch.equal(sd[k], rsd[k]), k
    flat = net.flat_params()
    assert flat.numel() == net.param_count == Wp * din + Wp + L * (Wp * Wp + Wp) + dout * Wp + dout
    # the flat buffer is the padded SIREN of width Wp: padding exactly zero, parameters in place
    lay = net._layout()
    mask = torch.zeros_like(flat, dtype=torch.bool)
    for p, (off, pshape, corner) in zip(net.parameters(), lay):
        block = flat[off:off + int(torch.tensor(pshape).prod())].view(*pshape)
        inner = block[tuple(slice(0, c) for c in corner)]
        assert inner.data_ptr() == p.data_ptr() and torch.equal(inner, p.detach())
        mask[off:off + block.numel()].view(*pshape)[tuple(slice(0, c) for c in corner)] = True
    assert int(mask.sum()) == sum(p.numel() for p in ref.parameters())
    assert bool((flat[~mask] == 0).all())


def test_load_state_dict_and_checkpoint_roundtrip(B, tmp_path):
    torch.manual_seed(0)
    a = B.MLP(2, 2, 3, 68, nonlinearity="sine")
    torch.manual_seed(1)
    b = B.MLP(2, 2, 3, 68, nonlinearity="sine")
    b.load_state_dict(a.state_dict())
    assert torch.equal(a.flat_params(), b.flat_params())
    # reference checkpoint layout: {'net_<name>': state_dict, 'timestep': t}
    path = tmp_path / "ckpt_step_t003.pth"
    torch.save({"net_deformation": {k: v.detach().cpu() for k, v in a.state_dict().items()}, "timestep": 3}, path)
    ck = torch.load(path, weights_only=True)
    torch.manual_seed(2)
    c = B.MLP(2, 2, 3, 68, nonlinearity="sine")
    c.load_state_dict(ck["net_deformation"])
    assert torch.equal(c.flat_params(), a.flat_params())
    # and a reference-built network reads it unchanged
    ref = O.OracleSiren(2, 2, 3, 68)
    ref.load_state_dict(ck["net_deformation"])
    for p, q in zip(ref.parameters(), a.parameters()):
        assert torch.equal(p.detach(), q.detach())


def test_grad_views_follow_the_padded_layout(B):
    torch.manual_seed(0)
    net = B.MLP(1, 1, 2, 20, nonlinearity="sine")
    g = net.flat_grad_buffer()
    g.copy_(torch.arange(g.numel(), dtype=torch.float32))
    for p, e in zip(net.parameters(), net._layout()):
        assert torch.equal(p.grad, net._view(g, e))


def test_width_above_256_is_the_torch_network(B):
    """No kernel is compiled above width 256: such a SIREN is the reference's plain torch network
    (TorchMLP; tests/test_other_nets.py pins it to the reference's outputs)."""
    net = B.MLP(2, 2, 1, 300, nonlinearity="sine")
    assert type(net).__name__ == "TorchMLP" and not isinstance(net, B.MLP)
    with pytest.raises(NotImplementedError):
        B.networks.kernel_width(300)


@pytest.mark.parametrize("shape", [(2, 1, 3, 128), (3, 3, 4, 256), (1, 1, 2, 32), (2, 3, 1, 64)])
def test_weight_planes_follow_the_parameters(B, shape):
    """The flat storage reserves the pre-split weight planes right after the parameters, at the
    offset and size the library computes (insr_siren_wsplit_offset / _floats), and the
    parameter views never reach into them."""
    din, dout, L, W = shape
    net = B.MLP(din, dout, L, W, nonlinearity="sine")
    lib = B._native.lib()
    assert net.wsplit_offset() == lib.insr_siren_wsplit_offset(din, dout, L, W)
    assert net.wsplit_floats() == lib.insr_siren_wsplit_floats(L, W) == 5 * L * W * W + 4  # + the status quad
    flat = net.flat_params()
    store = flat._base if flat._base is not None else flat
    assert store.numel() == net.wsplit_offset() + net.wsplit_floats()
    assert flat.numel() == net.param_count and net.wsplit_offset() % 4 == 0
    end = flat.data_ptr() + 4 * net.param_count
    for p in net.parameters():
        assert p.data_ptr() >= flat.data_ptr() and p.data_ptr() + 4 * p.numel() <= end


def test_reference_import_surface(B):
    """Every name the reference's model packages import from `base` (advection/model.py:5,
    fluid/model.py:5-6, fluid/visualize.py, elasticity/model.py:5-11, base/networks.py
    `from .diff_ops import *`) resolves here -- the model files' import lines run unchanged.
    (Random_Basis_Function*: the kNN random-basis solver, pytorch3d, out of scope: DESIGN §8.)"""
    names = ["BaseModel", "gradient", "divergence", "laplace", "jacobian", "hessian", "sample_random",
             "sample_uniform", "sample_boundary", "sample_boundary2D_separate", "MLP", "Sine", "get_network"]
    for n in names:
        assert hasattr(B, n), n


def test_deepcopy_round_trip(B):
    """copy.deepcopy rebuilds through MLP.__new__(cls) with no arguments (a model file keeping a
    previous-step copy of its network): the copy is an MLP with equal parameters on storage of its
    own, still one flat buffer; a TorchMLP deep-copies as well."""
    import copy
    torch.manual_seed(0)
    a = B.MLP(2, 1, 2, 64, nonlinearity="sine")
    b = copy.deepcopy(a)
    assert type(b) is type(a)
    assert torch.equal(a.flat_params(), b.flat_params())
    assert b.flat_params().data_ptr() != a.flat_params().data_ptr()
    for p in b.parameters():  # the copy's parameters are views of the copy's flat buffer
        assert b.flat_params().data_ptr() <= p.data_ptr() < b.flat_params().data_ptr() + 4 * b.param_count
    with torch.no_grad():
        next(b.parameters()).add_(1.0)
    assert not torch.equal(a.flat_params(), b.flat_params())
    t = copy.deepcopy(B.MLP(2, 1, 2, 64, nonlinearity="relu"))
    assert type(t).__name__ == "TorchMLP"


def test_reseed_hooks_reversible():
    """base.sampling's re-seed counters wrap torch's seeding functions reversibly: uninstall
    puts the originals back, install wraps them again, and a re-seed is counted only while installed."""
    import torch
    from base import sampling as S
    orig = torch.manual_seed.__wrapped__ if hasattr(torch.manual_seed, "_insr_reseed_hook") else torch.manual_seed
    try:
        S.uninstall_reseed_hooks()
        assert torch.manual_seed is orig and not hasattr(torch.cuda.manual_seed_all, "_insr_reseed_hook")
        e = S.reseed_epoch()
        torch.manual_seed(3)
        assert S.reseed_epoch() == e
        S.install_reseed_hooks()
        S.install_reseed_hooks()  # idempotent: no wrapper of a wrapper
        assert torch.manual_seed.__wrapped__ is orig
        torch.manual_seed(3)
        assert S.reseed_epoch() > e
    finally:
        S.install_reseed_hooks()
