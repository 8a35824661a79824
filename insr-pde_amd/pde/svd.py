"""Singular values of batched 2x2 / 3x3 deformation gradients (elasticity/model.py:144).

The reference calls torch.svd(J) and only uses S; dE/dJ = U diag(dE/dS) V^T.
  2x2: closed form (differentiable torch ops, no solver launch):
       E=(a+d)/2, F=(a-d)/2, G=(c+b)/2, H=(c-b)/2, Q=|(E,H)|, R=|(F,G)|,
       s1 = Q + R, s2 = |Q - R|  (descending, non-negative like torch.svd).
       A 1e-30 guard under the square roots keeps the gradient finite at the
       exact rotation / reflection points (value change < 1e-15).
  3x3: torch.linalg.svdvals (rocSOLVER) -- a fused HIP small-SVD kernel is
       SURVEY.md §8(f) row 1 (next).
"""
import torch


def singular_values(J):
    if J.shape[-2:] == (2, 2):
        a, b = J[..., 0, 0], J[..., 0, 1]
        c, d = J[..., 1, 0], J[..., 1, 1]
        E, F = (a + d) * 0.5, (a - d) * 0.5
        G, H = (c + b) * 0.5, (c - b) * 0.5
        Q = torch.sqrt(E * E + H * H + 1e-30)
        R = torch.sqrt(F * F + G * G + 1e-30)
        return torch.stack([Q + R, torch.abs(Q - R)], dim=-1)
    return torch.linalg.svdvals(J)
