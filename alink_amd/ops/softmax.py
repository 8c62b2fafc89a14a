"""Fused softmax-loss epilogues (``csrc/softmax.hip``).

``softmax_grad(eta, y, w)`` -> ``(R, loss)``: ``R = w * (softmax(eta | pivot 0) - onehot(y))`` ([n, k1], the
right-hand side of the ``X^T R`` gradient GEMM) and the weighted loss sum, from one pass over the logits.
``softmax_search(ec, ed, y, w, beta, nsteps)`` -> the weighted loss at each of ``nsteps`` trial steps
``ec - s * beta * ed`` from one read of ``ec`` / ``ed``.  Reference: ``SoftmaxObjFunc.java``.
CPU tensors (and k1 > 32) use the torch formulas.
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _lib

__all__ = ["softmax_grad", "softmax_grad_torch", "softmax_search", "softmax_search_torch", "KMAX"]

KMAX = 32


def _lse_pivot(eta: torch.Tensor) -> torch.Tensor:
    z = torch.zeros((eta.shape[0], 1), dtype=eta.dtype, device=eta.device)
    return torch.logsumexp(torch.cat([eta, z], 1), 1)


def _lin(eta, y):
    k1 = eta.shape[1]
    yk = y.long()
    return torch.where(yk < k1, eta.gather(1, yk.clamp(max=k1 - 1)[:, None])[:, 0], torch.zeros_like(y))


def softmax_grad_torch(eta, y, w) -> Tuple[torch.Tensor, torch.Tensor]:
    lse = _lse_pivot(eta)
    phi = torch.exp(eta - lse[:, None])
    yk = y.long()
    rows = torch.nonzero(yk < eta.shape[1]).reshape(-1)
    phi[rows, yk[rows]] -= 1.0
    return phi * w[:, None], ((lse - _lin(eta, y)) * w).sum()


def softmax_search_torch(ec, ed, y, w, beta: float, nsteps: int) -> torch.Tensor:
    d = ed * beta
    out = []
    for s in range(nsteps):
        e = ec - s * d
        out.append(((_lse_pivot(e) - _lin(e, y)) * w).sum())
    return torch.stack(out)


def _kernel_ok(eta: torch.Tensor) -> bool:
    return eta.is_cuda and eta.dtype == torch.float64 and eta.dim() == 2 and 0 < eta.shape[1] <= KMAX and \
        (_lib.available() or not _lib.torch_fallback_allowed())


def softmax_grad(eta, y, w) -> Tuple[torch.Tensor, torch.Tensor]:
    if not _kernel_ok(eta):
        return softmax_grad_torch(eta, y, w)
    L = _lib.require()
    n, k1 = eta.shape
    eta = eta.contiguous()
    y = y.to(torch.float64).contiguous()
    w = w.to(torch.float64).contiguous()
    assert y.numel() == n and w.numel() == n
    R = torch.empty_like(eta)
    part = torch.zeros(max(1, L.alink_softmax_grid(n)), dtype=torch.float64, device=eta.device)
    rc = L.alink_softmax_grad_f64(eta.data_ptr(), y.data_ptr(), w.data_ptr(), n, k1, R.data_ptr(), part.data_ptr(),
                                  _lib.stream_ptr(eta.device))
    if rc != 0:
        raise RuntimeError(f"alink_softmax_grad_f64 failed: {rc}")
    return R, part.sum()


def softmax_search(ec, ed, y, w, beta: float, nsteps: int) -> torch.Tensor:
    if not _kernel_ok(ec) or nsteps > 64:
        return softmax_search_torch(ec, ed, y, w, beta, nsteps)
    L = _lib.require()
    n, k1 = ec.shape
    assert ed.shape == ec.shape
    ec, ed = ec.contiguous(), ed.to(torch.float64).contiguous()
    y = y.to(torch.float64).contiguous()
    w = w.to(torch.float64).contiguous()
    part = torch.zeros((max(1, L.alink_softmax_grid(n)), nsteps), dtype=torch.float64, device=ec.device)
    rc = L.alink_softmax_search_f64(ec.data_ptr(), ed.data_ptr(), y.data_ptr(), w.data_ptr(), n, k1, float(beta),
                                    int(nsteps), part.data_ptr(), _lib.stream_ptr(ec.device))
    if rc != 0:
        raise RuntimeError(f"alink_softmax_search_f64 failed: {rc}")
    return part.sum(0)


def softmax_full_grad_torch(z, y, w) -> Tuple[torch.Tensor, torch.Tensor]:
    """No pivot class: ``w * (softmax(z) - onehot(y))`` and ``sum w (lse - z[y])`` (the MLP output layer)."""
    lse = torch.logsumexp(z, 1)
    P = torch.exp(z - lse[:, None])
    yk = y.long()
    P[torch.arange(z.shape[0], device=z.device), yk] -= 1.0
    return P * w[:, None], ((lse - z.gather(1, yk[:, None])[:, 0]) * w).sum()
