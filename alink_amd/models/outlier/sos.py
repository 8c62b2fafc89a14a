"""Stochastic Outlier Selection (SOS).

Reference: ``A/operator/common/outlier/SOSImpl.java`` — dissimilarity = squared Euclidean distance (cross
product :39-73), per-row bisection for the Gaussian precision ``beta`` matching the perplexity
(``solveForBeta`` :75-108, 100 iterations, tolerance 1e-2 on log-perplexity), binding probabilities
:133-172, outlier probability = prod_i (1 - b_ij) :174-203; ``SosBatchOp.java``.

MI355X-first: the n x n dissimilarity matrix is ONE GEMM (``|x|^2 + |y|^2 - 2 X X^T``) on the device, the
bisection runs for all rows at once (vectorised state with per-row convergence masks, so every row follows
exactly the reference's iteration sequence), and the column products are a log-sum reduction — rows are
processed in blocks so memory stays bounded.
"""
from __future__ import annotations

import math

import torch

__all__ = ["sos_scores"]

MAX_ITER = 100
TOL = 1.0e-2


def _log_h(D: torch.Tensor, beta: torch.Tensor, self_mask: torch.Tensor) -> torch.Tensor:
    A = torch.exp(-beta[:, None] * D).masked_fill(self_mask, 0.0)
    s = A.sum(1)
    return (A * D).sum(1) * (beta / s) + torch.log(s)


def sos_scores(X: torch.Tensor, perplexity: float, block: int = 4096) -> torch.Tensor:
    """Outlier probability of every row of X [n, d] (float64)."""
    n = X.shape[0]
    X = X.to(torch.float64)
    sq = (X * X).sum(1)
    logh = math.log(perplexity)
    log_keep = torch.zeros(n, dtype=torch.float64, device=X.device)   # sum_i log(1 - b_ij)
    for s in range(0, n, block):
        e = min(n, s + block)
        D = (sq[s:e, None] + sq[None, :] - 2.0 * (X[s:e] @ X.T)).clamp_min(0.0)
        rows = torch.arange(s, e, device=X.device)
        self_mask = torch.zeros_like(D, dtype=torch.bool)
        self_mask[torch.arange(e - s, device=X.device), rows] = True
        beta = torch.ones(e - s, dtype=torch.float64, device=X.device)
        bmin = torch.zeros_like(beta)
        bmax = torch.full_like(beta, float("inf"))
        err = _log_h(D, beta, self_mask) - logh
        for _ in range(MAX_ITER):
            active = torch.isnan(err) | (err.abs() > TOL)
            if not bool(active.any()):
                break
            nan = torch.isnan(err)
            pos = (~nan) & (err > 0)
            neg = (~nan) & (err <= 0)
            unbounded = torch.isinf(bmax)
            nb = beta.clone()
            nb = torch.where(active & nan, beta / 10.0, nb)
            nb = torch.where(active & pos & unbounded, beta * 2.0, nb)
            nb = torch.where(active & pos & ~unbounded, 0.5 * (beta + bmax), nb)
            nbmin = torch.where(active & pos, beta, bmin)
            nbmax = torch.where(active & neg, beta, bmax)
            nb = torch.where(active & neg, 0.5 * (bmin + beta), nb)
            beta, bmin, bmax = nb, nbmin, nbmax
            err = torch.where(active, _log_h(D, beta, self_mask) - logh, err)
        A = torch.exp(-beta[:, None] * D).masked_fill(self_mask, 0.0)
        B = A / A.sum(1, keepdim=True)
        log_keep += torch.log1p(-B.clamp(max=1.0)).sum(0)
    return torch.exp(log_keep)
