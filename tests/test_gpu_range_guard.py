"""Range guard of the fp16 weight planes (include/insr_siren.h insr_siren_wsplit_status): 2^8 w in
two fp16 terms needs |w| < 255.  insr_siren_wsplit and the Adam launch that keeps the planes current
flag a hidden weight outside that range (and clamp its fp16 terms: nothing overflows), the flag is a
clean INSR_ERANGE at the host's sync point, and base.MLP.check_weight_planes -- called by the
training loop where it reads the losses -- raises instead of training on f16x3 products that are
not the network's.  A network at precision='bf16x6' with INSR_JET_BWD_F16(0) reads only the bf16
planes (fp32's range).
"""
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


def status(B, net):
    nat = B._native
    return nat.lib().insr_siren_wsplit_status(nat.ptr(net.flat_params()), net.in_features, net.out_features,
                                              net.num_hidden_layers, net.kernel_width,
                                              nat.stream_of(torch.device("cuda")))


def test_wsplit_flags_and_clears(B):
    nat = B._native
    torch.manual_seed(61)
    net = B.MLP(2, 1, 4, 128, nonlinearity="sine").cuda()
    net.refresh_wsplit()
    assert status(B, net) == 0
    net.check_weight_planes()
    with torch.no_grad():
        net.net[4].weight[3, 7] = 300.0  # hidden layer 2
    net.refresh_wsplit()
    assert status(B, net) == nat.ERANGE
    with pytest.raises(nat.NativeError):
        net.check_weight_planes()
    # the clamped planes keep every jet finite (the flag says the products are not the network's)
    x = (torch.rand(500, 2) * 2 - 1).cuda().requires_grad_(True)
    lp = B.laplace(net(x), x)
    assert torch.isfinite(lp).all()
    with torch.no_grad():
        net.net[4].weight[3, 7] = 0.01
    net.refresh_wsplit()  # a split of in-range weights clears the flag
    assert status(B, net) == 0


def test_adam_flags_sticky(B):
    """The Adam launch that rewrites the planes flags an update that leaves the range."""
    nat = B._native
    torch.manual_seed(62)
    net = B.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    opt = B.FusedAdam([{"params": net, "module": net, "lr": 400.0}])
    x = (torch.rand(256, 2) * 2 - 1).cuda()
    net(x).sum().backward()
    opt.step()  # |dw| ~ lr = 400 on the first Adam step: hidden weights leave the planes' range
    assert status(B, net) == nat.ERANGE
    with pytest.raises(nat.NativeError):
        net.check_weight_planes()


def test_bf16x6_network_ignores_the_fp16_planes(B):
    """One hidden weight at 300: outside the fp16 planes' range.  At precision='bf16x6' with no fp16
    backward products the network never reads the fp16 planes: no error from the guard, finite jets
    and gradients.  (No oracle comparison here: sin(30 z) with |z| ~ 10^3 is ill-conditioned at fp32
    for every implementation, the reference's included.)"""
    nat = B._native
    torch.manual_seed(63)
    net = B.MLP(2, 1, 4, 128, nonlinearity="sine", precision="bf16x6").cuda()
    with torch.no_grad():
        net.net[4].weight[3, 7] = 300.0
    x = (torch.rand(700, 2, generator=torch.Generator().manual_seed(64)) * 2 - 1).cuda().requires_grad_(True)
    with nat.knobs(bwd_f16=0):
        assert not net.uses_f16_planes()
        lp = B.laplace(net(x), x)
        lp.square().sum().backward()
        torch.cuda.synchronize()
        net.check_weight_planes()  # not read by this network's jets: no error
    assert status(B, net) == nat.ERANGE  # ... though the planes are flagged
    assert torch.isfinite(lp).all()
    for q in net.parameters():
        assert q.grad is None or torch.isfinite(q.grad).all()


def test_batched_check_of_several_networks(B):
    """MLP.check_weight_planes_all (the training loop's sync points and phase end): one read of every
    network's status word; raises when any network's planes are flagged, passes otherwise, skips networks
    that do not read the fp16 planes and non-kernel networks."""
    nat = B._native
    torch.manual_seed(63)
    a = B.MLP(2, 1, 4, 128, nonlinearity="sine").cuda()
    b = B.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    t = B.MLP(2, 1, 2, 16, nonlinearity="relu").cuda()  # TorchMLP: no planes
    for n in (a, b):
        n.refresh_wsplit()
    B.MLP.check_weight_planes_all([a, b, t])
    with torch.no_grad():
        b.net[2].weight[0, 0] = -400.0
    b.refresh_wsplit()
    assert status(B, b) == nat.ERANGE
    with pytest.raises(nat.NativeError):
        B.MLP.check_weight_planes_all([a, b, t])
    B.MLP.check_weight_planes_all([a, t])
