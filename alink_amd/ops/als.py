"""ALS normal equations + batched solves.

``normal_equations(indptr, nbr, rating, Y, implicit, alpha)`` -> ``(A [m, r, r], b [m, r])`` with
``A_u = sum c y y^T`` and ``b_u = sum w y`` over the CSR row ``u`` (reference ``NormalEquation.add`` called
from ``AlsTrain.UpdateFactorsFunc``).  GPU: the HIP kernel in ``csrc/als.hip`` (one wavefront per row,
register-blocked 8x8 tiles, LDS-staged neighbour factors); CPU: chunked fp64 ``index_add_``.

``solve(A, b, nonnegative)``: batched SPD Cholesky solves (rocSOLVER via torch) in fp64 chunks, or a batched
projected coordinate-descent NNLS (reference ``NNLSSolver``) for the non-negative variant.
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["normal_equations", "normal_equations_torch", "solve", "nnls"]


def normal_equations_torch(indptr, nbr, rating, Y, implicit: bool, alpha: float):
    m = indptr.numel() - 1
    r = Y.shape[1]
    dev = Y.device
    A = torch.zeros((m, r, r), dtype=torch.float64, device=dev)
    b = torch.zeros((m, r), dtype=torch.float64, device=dev)
    nnz = nbr.numel()
    if m == 0 or nnz == 0:
        return A, b
    counts = (indptr[1:] - indptr[:-1]).long()
    rows = torch.repeat_interleave(torch.arange(m, device=dev), counts)
    rt = rating.to(torch.float64)
    if implicit:
        c = torch.where(rt > 0, alpha * rt, torch.zeros_like(rt))
        w = torch.where(rt > 0, 1.0 + c, torch.zeros_like(rt))
    else:
        c = torch.ones_like(rt)
        w = rt
    chunk = max(1, (1 << 24) // max(1, r * r))
    for s in range(0, nnz, chunk):
        y = Y[nbr[s:s + chunk].long()].to(torch.float64)
        A.index_add_(0, rows[s:s + chunk], (c[s:s + chunk, None, None] * y[:, :, None] * y[:, None, :]))
        b.index_add_(0, rows[s:s + chunk], w[s:s + chunk, None] * y)
    return A, b


def normal_equations(indptr: torch.Tensor, nbr: torch.Tensor, rating: torch.Tensor, Y: torch.Tensor,
                     implicit: bool = False, alpha: float = 0.0):
    r = Y.shape[1]
    if not Y.is_cuda or r > 64 or (not _lib.available() and _lib.torch_fallback_allowed()):
        return normal_equations_torch(indptr, nbr, rating, Y, implicit, alpha)
    L = _lib.require()
    m = indptr.numel() - 1
    indptr = indptr.to(torch.int64).contiguous()
    nbr = nbr.to(torch.int32).contiguous()
    rating = rating.to(torch.float32).contiguous()
    Yf = Y.to(torch.float32).contiguous()
    if nbr.numel() and int(nbr.max()) >= Yf.shape[0]:
        raise ValueError("neighbour index out of range")
    A = torch.empty((m, r, r), dtype=torch.float32, device=Y.device)
    b = torch.empty((m, r), dtype=torch.float32, device=Y.device)
    if m == 0:
        return A, b
    rc = L.alink_als_gram_f32(indptr.data_ptr(), nbr.data_ptr(), rating.data_ptr(), Yf.data_ptr(), m, r,
                              int(bool(implicit)), float(alpha), A.data_ptr(), b.data_ptr(),
                              _lib.stream_ptr(Y.device))
    if rc != 0:
        raise RuntimeError(f"alink_als_gram_f32 failed: {rc}")
    return A, b


def nnls(A: torch.Tensor, b: torch.Tensor, sweeps: int = 200, tol: float = 1e-10) -> torch.Tensor:
    """Batched non-negative least squares min 1/2 x'Ax - b'x, x >= 0 (projected coordinate descent)."""
    m, r = b.shape
    x = torch.zeros_like(b)
    diag = torch.diagonal(A, dim1=1, dim2=2).clamp_min(1e-300)
    g = -b.clone()                              # gradient A x - b
    for _ in range(sweeps):
        delta_max = torch.zeros(m, dtype=b.dtype, device=b.device)
        for i in range(r):
            xi = x[:, i]
            new = (xi - g[:, i] / diag[:, i]).clamp_min(0.0)
            d = new - xi
            x[:, i] = new
            g += d[:, None] * A[:, :, i]
            delta_max = torch.maximum(delta_max, d.abs())
        if float(delta_max.max()) < tol:
            break
    return x


def solve(A: torch.Tensor, b: torch.Tensor, nonnegative: bool = False, chunk: int = None) -> torch.Tensor:
    """x_u = A_u^{-1} b_u for every u (fp64), returned as float32."""
    m, r = b.shape
    out = torch.empty((m, r), dtype=torch.float32, device=b.device)
    if m == 0:
        return out
    chunk = chunk or max(1, (1 << 26) // max(1, r * r))
    for s in range(0, m, chunk):
        Ad = A[s:s + chunk].to(torch.float64)
        bd = b[s:s + chunk].to(torch.float64)
        if nonnegative:
            x = nnls(Ad, bd)
        else:
            Lc, info = torch.linalg.cholesky_ex(Ad)
            x = torch.cholesky_solve(bd[:, :, None], Lc)[:, :, 0]
            bad = info != 0
            if bool(bad.any()):
                x[bad] = (torch.linalg.pinv(Ad[bad]) @ bd[bad][:, :, None])[:, :, 0]
        out[s:s + chunk] = x.to(torch.float32)
    return out
