"""ALS normal equations + batched solves.

``normal_equations(indptr, nbr, rating, Y, implicit, alpha)`` -> ``(A [m, r, r], b [m, r])`` with
``A_u = sum c y y^T`` and ``b_u = sum w y`` over the CSR row ``u`` (reference ``NormalEquation.add`` called
from ``AlsTrain.UpdateFactorsFunc``).  GPU: the HIP kernel in ``csrc/als.hip`` (one wavefront per row,
register-blocked 8x8 tiles, LDS-staged neighbour factors); CPU: chunked fp64 ``index_add_``.

``solve(A, b, nonnegative)``: batched SPD Cholesky solves (rocSOLVER via torch) in fp64 chunks, or a batched
projected coordinate-descent NNLS (reference ``NNLSSolver``) for the non-negative variant.

``fused_solve(...)``: the GPU default for the unconstrained solve — ``alink_als_fused_solve`` builds each row's
normal equations in registers (fp64), factors and solves them in LDS, one wave per row; the ``[m, r, r]``
matrices never touch HBM.  Rows whose matrix is not SPD are re-solved with ``pinv`` on the host side.  At rank
33..64 the light rows run ``alink_als_mfma_solve`` instead: Gram and block LDL^T on the f64 matrix cores
(``v_mfma_f64_16x16x4``), no LDS; explicit rows with <= 32 ratings take the push-through m x m solve and rows with
> 16384 ratings the split heavy path.
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["normal_equations", "normal_equations_torch", "solve", "nnls", "fused_solve", "fused_supported"]


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


HEAVY_DEGREE = 16384     # rows with more neighbours are split across waves (partial Grams)
HEAVY_CHUNK = 4096
# rank 33..64: heavy rows' partial Grams on the matrix cores (als_heavy_gram_mfma: exact bf16 x3 split, fp64
# folding per 32 neighbours); 0 keeps the fp64 VALU kernel
HEAVY_MFMA = int(__import__("os").environ.get("ALINK_ALS_HEAVY_MFMA", "1"))
# explicit rows with <= 8 / 16 / 32 neighbours (below the padded rank): m x m push-through solve
# (alink_als_woodbury_solve) instead of the r x r system; 0 disables
WOODBURY = int(__import__("os").environ.get("ALINK_ALS_WOODBURY", "1"))
# rank 33..64 light rows: the normal-equation Gram and the block LDL^T solve on the f64 matrix cores
# (alink_als_mfma_solve); 0 keeps the VALU Gram + Gauss-Jordan kernel (alink_als_fused_solve)
MFMA_LIGHT = int(__import__("os").environ.get("ALINK_ALS_MFMA_LIGHT", "1"))
# explicit rows with 9..16 ratings: Gram / solve / Y^T a of the push-through identity on the f64 matrix cores
# (alink_als_woodbury16_mfma); 0 keeps the LDS-staged kernel
WOODBURY_MFMA = int(__import__("os").environ.get("ALINK_ALS_WOODBURY_MFMA", "0"))
WOODBURY_BUCKETS = tuple(int(x) for x in __import__("os").environ.get("ALINK_ALS_WOODBURY_BUCKETS", "8,16,32")
                         .split(","))


def fused_supported(Y: torch.Tensor) -> bool:
    return Y.is_cuda and Y.shape[1] <= 64 and (_lib.available() or not _lib.torch_fallback_allowed())


_PLANS = {}


def _row_plan(indptr: torch.Tensor, nbr: torch.Tensor, n_factors: int, buckets: tuple) -> dict:
    """The row partition of a CSR rating matrix for ``fused_solve`` -- heavy rows and their chunking, the
    Woodbury buckets, the light rows -- and the neighbour-range check, computed once per (CSR, bucket set):
    ALS re-solves the same two CSR matrices every iteration, so the per-sweep deg / nonzero / max passes (and
    their host synchronisations) are paid on the first sweep only.  Keyed by the tensors' identity and version."""
    import weakref
    key = (indptr.data_ptr(), indptr.numel(), indptr._version, nbr.data_ptr(), nbr.numel(), nbr._version, n_factors,
           buckets, HEAVY_DEGREE, HEAVY_CHUNK)
    hit = _PLANS.get(key)
    if hit is not None and hit[0]() is indptr and hit[1]() is nbr:
        return hit[2]
    if nbr.numel() and int(nbr.max()) >= n_factors:
        raise ValueError("neighbour index out of range")
    dev = indptr.device
    deg = indptr[1:] - indptr[:-1]
    heavy = torch.nonzero(deg > HEAVY_DEGREE, as_tuple=False).reshape(-1)
    small = torch.zeros_like(deg, dtype=torch.bool)
    lo, ids_list = -1, []
    for P in buckets:
        sel = (deg > lo) & (deg <= P)
        small |= sel
        ids_list.append(torch.nonzero(sel, as_tuple=False).reshape(-1))
        lo = P
    light = torch.nonzero((deg <= HEAVY_DEGREE) & ~small, as_tuple=False).reshape(-1) \
        if (heavy.numel() or buckets) else None
    plan = {"heavy": heavy, "buckets": ids_list, "light": light, "chunk_row": None, "chunk_start": None}
    if heavy.numel():
        hd = deg[heavy]
        nck = (hd + HEAVY_CHUNK - 1) // HEAVY_CHUNK
        chunk_row = torch.repeat_interleave(torch.arange(heavy.numel(), device=dev), nck)
        first = torch.cumsum(nck, 0) - nck
        chunk_start = indptr[:-1][heavy][chunk_row] + (torch.arange(int(nck.sum()), device=dev) - first[chunk_row]) \
            * HEAVY_CHUNK
        plan["chunk_row"], plan["chunk_start"] = chunk_row.contiguous(), chunk_start.contiguous()
    if len(_PLANS) >= 8:
        _PLANS.clear()
    _PLANS[key] = (weakref.ref(indptr), weakref.ref(nbr), plan)
    return plan


def fused_solve(indptr: torch.Tensor, nbr: torch.Tensor, rating: torch.Tensor, Y: torch.Tensor, reg: torch.Tensor,
                implicit: bool = False, alpha: float = 0.0, YtY: torch.Tensor = None) -> torch.Tensor:
    """x_u (float32 [m, r]) of ``(sum c y y^T + reg_u I [+ YtY]) x = sum w y`` for every CSR row u (GPU)."""
    L = _lib.require()
    m = indptr.numel() - 1
    r = Y.shape[1]
    dev = Y.device
    X = torch.empty((max(m, 0), r), dtype=torch.float32, device=dev)
    if m <= 0:
        return X
    indptr = indptr.to(device=dev, dtype=torch.int64).contiguous()
    nbr = nbr.to(device=dev, dtype=torch.int32).contiguous()
    rating = rating.to(device=dev, dtype=torch.float32).contiguous()
    Yf = Y.to(torch.float32).contiguous()
    regd = reg.to(device=dev, dtype=torch.float64).contiguous()
    yty = None if YtY is None else YtY.to(device=dev, dtype=torch.float64).contiguous()
    status = torch.zeros(m, dtype=torch.int32, device=dev)
    st = _lib.stream_ptr(dev)
    RP = int(L.alink_als_padded_rank(r))
    buckets = [P for P in WOODBURY_BUCKETS if WOODBURY and not implicit and yty is None and P < RP]
    plan = _row_plan(indptr, nbr, Yf.shape[0], tuple(buckets))
    heavy, light = plan["heavy"], plan["light"]
    for P, ids in zip(buckets, plan["buckets"]):
        if ids.numel():
            if P == 16 and WOODBURY_MFMA:
                rc = L.alink_als_woodbury16_mfma(indptr.data_ptr(), nbr.data_ptr(), rating.data_ptr(), Yf.data_ptr(),
                                                 ids.numel(), r, regd.data_ptr(), ids.data_ptr(), X.data_ptr(),
                                                 status.data_ptr(), st)
            else:
                rc = L.alink_als_woodbury_solve(indptr.data_ptr(), nbr.data_ptr(), rating.data_ptr(), Yf.data_ptr(),
                                                ids.numel(), r, regd.data_ptr(), ids.data_ptr(), P, X.data_ptr(),
                                                status.data_ptr(), st)
            if rc != 0:
                raise RuntimeError(f"alink_als_woodbury_solve failed: {rc}")
    nl = m if light is None else light.numel()
    if nl:
        fn = L.alink_als_mfma_solve if (MFMA_LIGHT and RP == 64) else L.alink_als_fused_solve
        rc = fn(indptr.data_ptr(), nbr.data_ptr(), rating.data_ptr(), Yf.data_ptr(), nl, r, int(bool(implicit)),
                float(alpha), regd.data_ptr(), None if yty is None else yty.data_ptr(),
                None if light is None else light.data_ptr(), X.data_ptr(), status.data_ptr(), st)
        if rc != 0:
            raise RuntimeError(f"{fn.__name__} failed: {rc}")
    if heavy.numel():
        # popular items: the neighbour list is split into HEAVY_CHUNK pieces, one wave each (partial Grams
        # summed in fp64), then one wave per row solves
        chunk_row, chunk_start = plan["chunk_row"], plan["chunk_start"]
        G = torch.zeros((heavy.numel(), RP, RP), dtype=torch.float64, device=dev)
        B = torch.zeros((heavy.numel(), RP), dtype=torch.float64, device=dev)
        rc = L.alink_als_heavy_solve(indptr.data_ptr(), nbr.data_ptr(), rating.data_ptr(), Yf.data_ptr(), r,
                                     int(bool(implicit)), float(alpha), regd.data_ptr(),
                                     None if yty is None else yty.data_ptr(), heavy.data_ptr(), heavy.numel(),
                                     chunk_row.contiguous().data_ptr(), chunk_start.contiguous().data_ptr(),
                                     chunk_row.numel(), HEAVY_CHUNK, G.data_ptr(), B.data_ptr(), X.data_ptr(),
                                     status.data_ptr(), HEAVY_MFMA, st)
        if rc != 0:
            raise RuntimeError(f"alink_als_heavy_solve failed: {rc}")
    bad = torch.nonzero(status != 0, as_tuple=False).reshape(-1)
    if bad.numel():                         # singular / indefinite rows: pinv like the chunked solver
        starts, ends = indptr[:-1][bad], indptr[1:][bad]
        cnt = ends - starts
        sub = torch.zeros(bad.numel() + 1, dtype=torch.int64, device=dev)
        sub[1:] = torch.cumsum(cnt, 0)
        pos = torch.repeat_interleave(starts - sub[:-1], cnt) + torch.arange(int(sub[-1]), device=dev)
        A, b = normal_equations_torch(sub, nbr[pos], rating[pos], Yf, implicit, alpha)
        if yty is not None:
            A = A + yty[None]
        A = A + regd[bad][:, None, None] * torch.eye(r, dtype=A.dtype, device=dev)[None]
        # symmetric pinv (eigh) on the host: rocSOLVER's batched SVD does not converge on rank-deficient systems,
        # and these rows are rare
        Ah = torch.linalg.pinv(A.cpu(), hermitian=True)
        X[bad] = (Ah @ b.cpu()[:, :, None])[:, :, 0].to(device=dev, dtype=torch.float32)
    return X
