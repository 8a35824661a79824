"""Bitwise repeatability of the jet launches the fluid phases issue (balanced / 5-tile shapes):
the same inputs twice must give the same outputs and parameter gradients."""
import sys
sys.path[:0] = ['.', 'insr-pde_amd']
import torch
import base
base._native.load()


def once(n, merged_extra, seed=0):
    torch.manual_seed(seed)
    prev = base.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    cur = base.MLP(2, 2, 4, 128, nonlinearity="sine").cuda()
    for p in prev.parameters():
        p.requires_grad_(False)
    g = torch.Generator(device="cuda").manual_seed(5)
    buf = (torch.rand(n + merged_extra, 2, device="cuda", generator=g) * 2 - 1).requires_grad_(True)
    x = buf[:n]
    with base.fused_forwards():
        with torch.no_grad():
            up = prev(x)
        ua = cur(buf)
    tgt = torch.rand(n, 2, device="cuda", generator=g)
    main, bc = base.sq_losses(base.mse_term(ua, tgt, count=2 * n), base.wall_term(ua, merged_extra // 2, row0=n))
    one = torch.ones((), device="cuda")
    torch.autograd.backward([main, bc], grad_tensors=[one, one])
    torch.cuda.synchronize()
    return up.clone(), ua.detach().clone(), main.detach().clone(), bc.detach().clone(), cur.flat_grad_buffer().clone()


for n, e in ((16384, 324), (65536, 1308)):
    a, b = once(n, e), once(n, e)
    print(n, e, [bool(torch.equal(u, v)) for u, v in zip(a, b)],
          [float((u - v).abs().max()) for u, v in zip(a, b)])
    lib = base._native.lib()
    print("  shapes fwd T", lib.insr_jet_split_tiles(n + e, 2, 128, 0, 0), "bwd T", lib.insr_jet_split_tiles(n + e, 2, 128, 0, 1),
          "bwd blocks", lib.insr_jet_partial_blocks(n + e, 2, 128, 0))
