"""Collocation samplers, drop-in for base/sampling.py:4-64 of the reference.

Same signatures (including `device=`) and the same torch RNG consumption, so a
seeded generator state yields the reference's points.  On a GPU device the
points come from torch's device RNG (graph-capturable); parity tests therefore
pass explicit sample tensors rather than relying on identical RNG streams.
"""
import torch

__all__ = ["sample_uniform", "sample_random", "sample_boundary", "sample_boundary2D_separate"]


def sample_uniform(resolution, sdim=1, device="cpu", flatten=True):
    """Cell-centred grid (i + 0.5)/R * 2 - 1 per axis, 'ij' order (base/sampling.py:4-11)."""
    axis = torch.linspace(0.5, resolution - 0.5, resolution, device=device) / resolution * 2 - 1
    grid = torch.stack(torch.meshgrid(*([axis] * sdim), indexing='ij'), dim=-1)
    return grid.reshape(resolution ** sdim, sdim) if flatten else grid


def sample_random(N, sdim=1, device="cpu"):
    """N points uniform in [-1, 1)^sdim (base/sampling.py:14-18)."""
    return torch.rand(N, sdim, device=device) * 2 - 1


def _band(n, ranges, device):
    """n points, coordinate k uniform in ranges[k] = (lo, hi)."""
    pts = torch.empty(n, len(ranges), device=device)
    for k, (lo, hi) in enumerate(ranges):
        pts[:, k] = torch.rand(n, device=device) * (hi - lo) + lo
    return pts


def sample_boundary(N, sdim, epsilon=1e-4, device='cpu'):
    """Random points in thin bands around the box faces (base/sampling.py:21-42)."""
    if sdim == 1:
        left = (torch.rand(N // 2, 1, device=device) * 2 - 1) * epsilon - 1.
        right = (torch.rand(N // 2, 1, device=device) * 2 - 1) * epsilon + 1.
        return torch.cat([left, right], dim=0)
    if sdim == 2:
        full, lo, hi = (-1, 1), (-1 - epsilon, -1 + epsilon), (1 - epsilon, 1 + epsilon)
        faces = [(full, lo), (full, hi), (lo, full), (hi, full)]
        return torch.cat([_band(N // 4, f, device) for f in faces], dim=0)
    raise NotImplementedError


def sample_boundary2D_separate(N, side, epsilon=1e-4, device='cpu'):
    """Bands on the two x-faces ('horizontal') or the two y-faces ('vertical'),
    N//2 random points each (base/sampling.py:45-64)."""
    full, lo, hi = (-1, 1), (-1 - epsilon, -1 + epsilon), (1 - epsilon, 1 + epsilon)
    if side == 'horizontal':
        faces = [(lo, full), (hi, full)]
    elif side == 'vertical':
        faces = [(full, lo), (full, hi)]
    else:
        raise RuntimeError
    return torch.cat([_band(N // 2, f, device) for f in faces], dim=0)
