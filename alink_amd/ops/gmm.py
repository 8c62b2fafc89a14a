"""GMM E-step (``csrc/gmm.hip``): one GEMM for all components' Mahalanobis projections plus a
fused log-density / log-sum-exp / responsibility kernel.

``estep(X0, mu0, W, logdet, rank, logw)`` -> ``(R [n, k], sum_i lse_i)`` where ``X0 = X - xbar`` and
``mu0 = mu - xbar`` (centred by one global vector so ``x W - mu W`` loses no precision), ``W [k, d, d]`` the
pseudo-inverse roots of the covariances.  ``estep_torch`` is the per-component torch formula
(``MultivariateGaussian.logpdf``); CPU tensors and k > 64 take it.
"""
from __future__ import annotations

import math
from typing import Tuple

import torch

from . import _lib

__all__ = ["estep", "estep_torch", "KMAX"]

KMAX = 64
_CHUNK_BYTES = 1 << 30       # Z chunk of at most 1 GiB (rows x k*d fp64)


def estep_torch(X0, mu0, W, logdet, rank, logw) -> Tuple[torch.Tensor, torch.Tensor]:
    n, k = X0.shape[0], mu0.shape[0]
    lp = torch.empty((n, k), dtype=X0.dtype, device=X0.device)
    for j in range(k):
        z = (X0 - mu0[j]) @ W[j]
        lp[:, j] = -0.5 * (rank[j] * math.log(2 * math.pi) + logdet[j]) - 0.5 * (z * z).sum(1)
    lp = lp + logw[None, :]
    lse = torch.logsumexp(lp, dim=1)
    return torch.exp(lp - lse[:, None]), lse.sum()


def estep(X0, mu0, W, logdet, rank, logw) -> Tuple[torch.Tensor, torch.Tensor]:
    k, d = mu0.shape
    if not (X0.is_cuda and X0.dtype == torch.float64 and k <= KMAX) or \
            (not _lib.available() and _lib.torch_fallback_allowed()):
        return estep_torch(X0, mu0, W, logdet, rank, logw)
    L = _lib.require()
    n = X0.shape[0]
    dev = X0.device
    Wcat = W.permute(1, 0, 2).reshape(d, k * d).contiguous()          # [d, k*d]: column block j is W_j
    C = torch.einsum("kd,kde->ke", mu0, W).contiguous()                # mu0_j W_j
    cst = (-0.5 * (rank * math.log(2 * math.pi) + logdet) + logw).to(torch.float64).contiguous()
    R = torch.empty((n, k), dtype=torch.float64, device=dev)
    rows = max(1, min(n, _CHUNK_BYTES // (8 * k * d)))
    total = torch.zeros((), dtype=torch.float64, device=dev)
    for s in range(0, n, rows):
        e = min(n, s + rows)
        Z = X0[s:e] @ Wcat
        part = torch.empty(L.alink_gmm_grid(e - s), dtype=torch.float64, device=dev)
        rc = L.alink_gmm_estep_f64(Z.data_ptr(), e - s, k, d, C.data_ptr(), cst.data_ptr(), R[s:e].data_ptr(),
                                   part.data_ptr(), _lib.stream_ptr(dev))
        if rc != 0:
            raise RuntimeError(f"alink_gmm_estep_f64 failed: {rc}")
        total = total + part.sum()
    return R, total
