"""Linear-model hot path: fused one-pass loss gradient (kernel K12) — ``csrc/linear.hip``.

``linear_grad(X, y, w, coef, loss)`` returns ``(sum_i w_i l'(x_i.coef, y_i) x_i, sum_i w_i l(.), sum_i w_i)``
with ONE read of the dense fp64 shard (the torch form reads it twice: ``X @ coef`` then ``X^T g``).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from . import _lib

__all__ = ["linear_grad_hip", "loss_code", "hip_linear_supported", "sparse_grad_hip", "hip_sparse_supported",
           "search_losses_hip"]

_SLABS: Dict[Tuple, torch.Tensor] = {}


def loss_code(unary) -> Optional[Tuple[int, float]]:
    from ..models.linear import objfunc as O
    t = type(unary)
    if t is O.LogLossFunc:
        return 0, 0.0
    if t is O.LogisticLossFunc:
        return 1, 0.0
    if t is O.SquareLossFunc:
        return 2, 0.0
    if t is O.HingeLossFunc:
        return 3, 0.0
    if t is O.SmoothHingeLossFunc:
        return 4, 0.0
    if t is O.PerceptronLossFunc:
        return 5, 0.0
    if t is O.ExponentialLossFunc:
        return 6, 0.0
    if t is O.HuberLossFunc:
        return 7, unary.delta
    if t is O.SvrLossFunc:
        return 8, unary.epsilon
    return None


MAX_D = 1024     # d <= 32: lane-per-row kernel; 32 < d <= 1024: lanes-over-columns kernel (csrc/linear.hip)


def hip_linear_supported(X: torch.Tensor) -> bool:
    return (X is not None and X.is_cuda and X.dtype == torch.float64 and X.dim() == 2 and 0 < X.shape[1] <= MAX_D
            and X.shape[0] > 0 and X.is_contiguous())


def linear_grad_hip(X: torch.Tensor, y: torch.Tensor, w: torch.Tensor, coef: torch.Tensor, code: int,
                    prm: float = 0.0) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    L = _lib.require()
    if not hip_linear_supported(X):
        raise ValueError(f"linear_grad_hip needs a contiguous fp64 [n, d<={MAX_D}] CUDA tensor")
    n, d = X.shape
    dev = X.device
    y = y.to(device=dev, dtype=torch.float64).contiguous()
    w = w.to(device=dev, dtype=torch.float64).contiguous()
    c = coef[:d].to(device=dev, dtype=torch.float64).contiguous()
    if y.shape[0] != n or w.shape[0] != n:
        raise ValueError("label / weight length mismatch")
    pad = int(L.alink_linear_grad_pad(d))
    wide = d > 32
    # narrow: one row per lane (256 rows per block); wide: one row group per wave, 2 blocks per CU resident
    nblk = max(1, min((n + 255) // 256, 2048)) if not wide else max(1, min((n + 7) // 8, 1024))
    key = (dev.index, nblk, pad)
    if key not in _SLABS:
        _SLABS[key] = torch.empty(nblk * (pad + 2), dtype=torch.float64, device=dev)
    out = torch.empty(d + 2, dtype=torch.float64, device=dev)
    fn = L.alink_linear_grad_wide_f64 if wide else L.alink_linear_grad_f64
    rc = fn(X.data_ptr(), y.data_ptr(), w.data_ptr(), c.data_ptr(), n, d, int(code), float(prm),
            _SLABS[key].data_ptr(), nblk, out.data_ptr(), _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_linear_grad{'_wide' if wide else ''}_f64 failed: {rc}")
    g = out[:d]
    if coef.shape[0] > d:
        g = torch.cat([g, torch.zeros(coef.shape[0] - d, dtype=g.dtype, device=dev)])
    return g, out[d], out[d + 1]


SEARCH_MAX_STEPS = 16


def k14_disabled() -> bool:
    """``ALINK_DISABLE_K14=1``: line search through the torch GEMM form (A/B diagnostics, tools/lr_train_bench.py)."""
    import os
    return os.environ.get("ALINK_DISABLE_K14", "0") == "1"


def search_losses_hip(X: torch.Tensor, y: torch.Tensor, w: torch.Tensor, coef: torch.Tensor, dirv: torch.Tensor,
                      code: int, prm: float, beta: float, nsteps: int) -> torch.Tensor:
    """K14: ``[sum_i w_i l(x_i.coef - s beta x_i.dir, y_i) for s < nsteps]`` in one pass over the dense fp64 X
    (``csrc/linear.hip`` linear_search_kernel; the torch form is an [n,d]x[d,2] fp64 GEMM plus elementwise)."""
    L = _lib.require()
    if not hip_linear_supported(X) or not 1 <= nsteps <= SEARCH_MAX_STEPS:
        raise ValueError("search_losses_hip needs a contiguous fp64 [n, d<=1024] CUDA tensor and <= 16 steps")
    n, d = X.shape
    dev = X.device
    y = y.to(device=dev, dtype=torch.float64).contiguous()
    w = w.to(device=dev, dtype=torch.float64).contiguous()
    c = coef[:d].to(device=dev, dtype=torch.float64).contiguous()
    dv = dirv[:d].to(device=dev, dtype=torch.float64).contiguous()
    nblk = max(1, min((n + 7) // 8, 1024))
    key = (dev.index, nblk, "search")
    if key not in _SLABS:
        _SLABS[key] = torch.empty(nblk * (SEARCH_MAX_STEPS + 2), dtype=torch.float64, device=dev)
    out = torch.empty(SEARCH_MAX_STEPS, dtype=torch.float64, device=dev)
    rc = L.alink_linear_search_f64(X.data_ptr(), y.data_ptr(), w.data_ptr(), c.data_ptr(), dv.data_ptr(), n, d,
                                   int(code), float(prm), float(beta), int(nsteps), _SLABS[key].data_ptr(), nblk,
                                   out.data_ptr(), _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_linear_search_f64 failed: {rc}")
    return out[:nsteps]


def hip_sparse_supported(fm) -> bool:
    return fm is not None and getattr(fm, "is_sparse", False) and fm.val.is_cuda and \
        (_lib.available() or not _lib.torch_fallback_allowed())


def _csc(fm):
    """CSC copy of a CSR FeatureMatrix (built once, cached on the matrix): column pointers, row ids, values."""
    c = getattr(fm, "_csc_cache", None)
    if c is not None:
        return c
    n = fm.nrows
    dev = fm.val.device
    rows = torch.repeat_interleave(torch.arange(n, device=dev), fm.crow[1:] - fm.crow[:-1])
    cols = fm.col.to(torch.int64)
    key, order = torch.sort(cols, stable=True)
    d = int(fm.ncols)
    cptr = torch.zeros(d + 1, dtype=torch.int64, device=dev)
    torch.cumsum(torch.bincount(key, minlength=d)[:d], 0, out=cptr[1:])
    c = (cptr, rows[order].contiguous(), fm.val.to(torch.float64)[order].contiguous(),
         fm.col.to(torch.int32).contiguous(), fm.val.to(torch.float64).contiguous())
    fm._csc_cache = c
    return c


def sparse_grad_hip(fm, y: torch.Tensor, w: torch.Tensor, coef: torch.Tensor, code: int, prm: float = 0.0):
    """(sum_i w_i l'(x_i.coef, y_i) x_i [d], sum_i w_i l(.), sum_i w_i) over a CSR FeatureMatrix on the GPU:
    row pass (wave per row) + column gather over the cached CSC copy (wave per column), no atomics."""
    L = _lib.require()
    dev = fm.val.device
    n = fm.nrows
    cptr, rows_of, cval, col32, val64 = _csc(fm)
    d = int(fm.ncols)
    y = y.to(device=dev, dtype=torch.float64).contiguous()
    w = w.to(device=dev, dtype=torch.float64).contiguous()
    c = torch.zeros(max(d, coef.shape[0]), dtype=torch.float64, device=dev)
    c[:coef.shape[0]] = coef.to(device=dev, dtype=torch.float64)
    g = torch.empty(n, dtype=torch.float64, device=dev)
    lw = torch.empty(n, dtype=torch.float64, device=dev)
    st = _lib.stream_ptr(dev)
    crow = fm.crow.to(torch.int64).contiguous()
    rc = L.alink_csr_row_deriv_f64(crow.data_ptr(), col32.data_ptr(), val64.data_ptr(), y.data_ptr(), w.data_ptr(),
                                   c.data_ptr(), n, int(code), float(prm), g.data_ptr(), lw.data_ptr(), st)
    if rc != 0:
        raise RuntimeError(f"alink_csr_row_deriv_f64 failed: {rc}")
    grad = torch.zeros(coef.shape[0], dtype=torch.float64, device=dev)
    out = torch.empty(d, dtype=torch.float64, device=dev)
    rc = L.alink_csc_gather_f64(cptr.data_ptr(), rows_of.data_ptr(), cval.data_ptr(), g.data_ptr(), d,
                                out.data_ptr(), st)
    if rc != 0:
        raise RuntimeError(f"alink_csc_gather_f64 failed: {rc}")
    m = min(d, coef.shape[0])
    grad[:m] = out[:m]
    return grad, lw.sum(), w.sum()
