"""Initial conditions used by the INSR-PDE experiments.

advection 'example1'        advection/examples.py:6-16   Gaussian bump at -1.5, sigma 0.1
fluid 'taylorgreen'         fluid/examples.py:17-31      Taylor-Green vortex, scaled by 1/pi
fluid 'taylorgreen_multi'   fluid/examples.py:34-51      two blended Taylor-Green patches
"""
import math

import torch


def gaussian_bump(x, mu=-1.5, sigma=0.1):
    return torch.exp(-0.5 * (x - mu) ** 2 / (sigma ** 2))


def taylor_green(p, rescale=False):
    """u = sin(X) cos(Y), v = -cos(X) sin(Y) with X, Y = pi (p + 1)."""
    X = math.pi * (p[..., 0] + 1)
    Y = math.pi * (p[..., 1] + 1)
    u = torch.sin(X) * torch.cos(Y)
    v = -(torch.cos(X) * torch.sin(Y))
    if rescale:
        return torch.stack([u / math.pi, v / math.pi], dim=-1)
    return torch.stack([u, v], dim=-1)


def taylor_green_multi(p, scale=8):
    """A unit vortex in the lower-left quadrant and a 1/scale vortex in the upper-right
    corner, each faded to zero across a thin gap (fluid/examples.py:34-51)."""
    gap = 0.05
    out = torch.zeros_like(p)
    low = (p[..., 0] <= gap) & (p[..., 1] <= gap)
    q = p[low]
    fade = 1.0 - q.clamp(0, gap).norm(dim=-1) / gap
    out[low] = taylor_green((q * 2 + 1).clamp(-1, 1)) * fade[:, None]
    corner = 1 - 2 / scale
    g2 = 2 * gap / scale
    high = (p[..., 0] > corner - g2) & (p[..., 1] > corner - g2)
    q = p[high]
    fade = 1.0 - (corner - q).clamp(0, g2).norm(dim=-1) / g2
    out[high] = taylor_green((q * scale + (1 - scale)).clamp(-1, 1)) * fade[:, None]
    return out


def get_examples(src, **kwargs):
    table = {
        'example1': lambda x: gaussian_bump(x, mu=-1.5),
        'taylorgreen': lambda p: taylor_green(p, rescale=True),
        'taylorgreen_multi': taylor_green_multi,
    }
    if src not in table:
        raise NotImplementedError(src)
    return table[src]
