"""Fused elementwise HIP kernels (``csrc/elementwise.hip``).

* ``gbdt_grad_stats(pred, y, w, algo)`` -> ``[n, 4]`` fp32 row records ``{g*g, g, h, 1}`` for the histogram kernel
  (least squares ``algo=0`` / logistic ``algo=1``), bit-identical to the torch chain it replaces
  (``ConstructLocalBin.java:116-131,185-205``).
* ``gbdt_leaf_update(pred, codes, vals)``: ``pred += vals[-1-code]`` for rows that ended in a leaf, in fp64 and
  rounded to fp32 (``Split.java`` predBuf).
* ``col_transform(X, mode, a, b, lo, hi)``: standard / min-max / max-abs scaling, NaN imputation and binarisation of
  a dense ``[n, d]`` (or ``[n]``) fp32/fp64 block into fp64 in one pass (``*ScalerModelMapper``,
  ``ImputerModelMapper``, ``BinarizerMapper``).

CPU tensors take the torch reference (``*_torch``); on a GPU the HIP kernels run, and a missing library raises
unless ``ALINK_ALLOW_TORCH_FALLBACK=1``.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import _lib

__all__ = ["gbdt_grad_stats", "gbdt_grad_stats_torch", "gbdt_leaf_update", "gbdt_leaf_update_torch",
           "col_transform", "col_transform_torch", "MODES"]

MODES = {"standard": 0, "minmax": 1, "maxabs": 2, "impute": 3, "binarize": 4}


def _use_kernel(t: torch.Tensor) -> bool:
    return t.is_cuda and (_lib.available() or not _lib.torch_fallback_allowed())


def _check(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{name} failed: {rc}")


# ---------------------------------------------------------------------------------------------------- K6
def gbdt_grad_stats_torch(pred: torch.Tensor, y: torch.Tensor, w: Optional[torch.Tensor], algo: int) -> torch.Tensor:
    if algo == 1:
        p = torch.sigmoid(pred.double())
        g = (p - y.double()).float()
        h = (p * (1.0 - p)).float()
    else:
        g = pred - y
        h = torch.ones_like(g)
    if w is not None:
        g, h = g * w, h * w
    return torch.stack([g * g, g, h, torch.ones_like(g)], dim=1)


def gbdt_grad_stats(pred: torch.Tensor, y: torch.Tensor, w: Optional[torch.Tensor], algo: int) -> torch.Tensor:
    if not _use_kernel(pred):
        return gbdt_grad_stats_torch(pred, y, w, algo)
    L = _lib.require()
    n = pred.numel()
    assert pred.dtype == y.dtype == torch.float32 and y.numel() == n and (w is None or w.numel() == n)
    pred, y = pred.contiguous(), y.contiguous()
    if w is not None:
        assert w.dtype == torch.float32
        w = w.contiguous()
    out = torch.empty((n, 4), dtype=torch.float32, device=pred.device)
    _check(L.alink_gbdt_grad_stats(pred.data_ptr(), y.data_ptr(), w.data_ptr() if w is not None else None, n,
                                   int(algo), out.data_ptr(), _lib.stream_ptr(pred.device)), "alink_gbdt_grad_stats")
    return out


RANK_MAX_POSITION = 10000       # the reference's kMaxPosition (ConstructLocalBin.java:46): longest query
_DISC = {}


def dcg_discount(device) -> torch.Tensor:
    """The reference's float discount table (float)(log 2 / log(2 + r)), r < 10000 (ConstructLocalBin.java:46-50)."""
    key = str(device)
    if key not in _DISC:
        r = np.arange(RANK_MAX_POSITION, dtype=np.float64)
        _DISC[key] = torch.from_numpy((np.log(2.0) / np.log(2.0 + r)).astype(np.float32)).to(device)
    return _DISC[key]


def gbdt_rank_stats(pred: torch.Tensor, gain: torch.Tensor, w: Optional[torch.Tensor], offsets: torch.Tensor,
                    algo: int) -> torch.Tensor:
    """K6 ranking variant: {g*g, g, h, 1} float32 row records of LambdaMART-NDCG (algo 2), LambdaMART-DCG (3) or
    GBRank (4) over contiguous queries (``offsets`` int64 [Q+1], every query <= 10000 rows).  GPU: one workgroup
    per query (``csrc/gbdt_rank.hip``); CPU: the reference's pair loop in C++ (``_native.gbdt_rank_grad``)."""
    n = pred.numel()
    assert pred.dtype == gain.dtype == torch.float32 and gain.numel() == n
    sizes = offsets[1:] - offsets[:-1]
    if sizes.numel() and int(sizes.max()) > RANK_MAX_POSITION:
        raise ValueError(f"a query has more than {RANK_MAX_POSITION} rows (the reference's kMaxPosition)")
    if _use_kernel(pred):
        L = _lib.require()
        pred, gain = pred.contiguous(), gain.contiguous()
        off = offsets.to(device=pred.device, dtype=torch.int64).contiguous()
        if w is not None:
            w = w.to(torch.float32).contiguous()
        out = torch.empty((n, 4), dtype=torch.float32, device=pred.device)
        rs = torch.empty(n, dtype=torch.int32, device=pred.device)
        ss = torch.empty(n, dtype=torch.float32, device=pred.device)
        _check(L.alink_gbdt_rank_stats(pred.data_ptr(), gain.data_ptr(), None if w is None else w.data_ptr(),
                                       off.data_ptr(), off.numel() - 1, dcg_discount(pred.device).data_ptr(),
                                       int(algo), rs.data_ptr(), ss.data_ptr(), out.data_ptr(),
                                       _lib.stream_ptr(pred.device)), "alink_gbdt_rank_stats")
        return out
    from .. import _native
    res = _native.gbdt_rank_grad(pred.detach().cpu().numpy(), gain.detach().cpu().numpy(),
                                 offsets.detach().cpu().numpy(), dcg_discount("cpu").numpy(), int(algo))
    if res is None:
        raise RuntimeError("GBDT ranking gradients need the host library (python build_native.py)")
    g, h = (torch.from_numpy(a).to(pred.device) for a in res)
    if w is not None:
        g, h = g * w.to(torch.float32), h * w.to(torch.float32)
    return torch.stack([g * g, g, h, torch.ones_like(g)], dim=1)


def gbdt_leaf_update_torch(pred: torch.Tensor, codes: torch.Tensor, vals: torch.Tensor) -> torch.Tensor:
    leaf = (-1 - codes.long()).clamp(min=0, max=vals.numel() - 1)
    inc = torch.where(codes < 0, vals[leaf], torch.zeros_like(vals[leaf]))
    return (pred.double() + inc).float()


def gbdt_leaf_update(pred: torch.Tensor, codes: torch.Tensor, vals: torch.Tensor) -> torch.Tensor:
    """Returns the updated prediction (in place on the GPU path)."""
    if not _use_kernel(pred):
        return gbdt_leaf_update_torch(pred, codes, vals)
    L = _lib.require()
    assert pred.dtype == torch.float32 and pred.is_contiguous() and codes.dtype == torch.int32
    assert codes.numel() == pred.numel() and vals.numel() >= 1
    codes = codes.contiguous()
    vals = vals.to(device=pred.device, dtype=torch.float64).contiguous()
    _check(L.alink_gbdt_leaf_update(pred.data_ptr(), codes.data_ptr(), vals.data_ptr(), vals.numel(), pred.numel(),
                                    _lib.stream_ptr(pred.device)), "alink_gbdt_leaf_update")
    return pred


# ---------------------------------------------------------------------------------------------------- K27
def col_transform_torch(X: torch.Tensor, mode: str, a=None, b=None, lo: float = 0.0, hi: float = 1.0) -> torch.Tensor:
    X = X.double()
    a = a.double() if a is not None else None
    b = b.double() if b is not None else None
    if mode == "standard":
        return torch.where(b > 0, (X - a) / torch.where(b > 0, b, torch.ones_like(b)), torch.zeros_like(X))
    if mode == "minmax":
        rng = b - a
        return torch.where(rng != 0, (X - a) / torch.where(rng != 0, rng, torch.ones_like(rng)) * (hi - lo) + lo,
                           torch.full_like(X, 0.5 * (hi + lo)))
    if mode == "maxabs":
        return torch.where(a == 0, X, X / torch.where(a == 0, torch.ones_like(a), a))
    if mode == "impute":
        return torch.where(torch.isnan(X), a.expand_as(X), X)
    if mode == "binarize":
        return (X > lo).double()
    raise ValueError(mode)


def col_transform(X: torch.Tensor, mode: str, a: Optional[torch.Tensor] = None, b: Optional[torch.Tensor] = None,
                  lo: float = 0.0, hi: float = 1.0) -> torch.Tensor:
    """``X`` [n, d] or [n] fp32/fp64; ``a``/``b`` fp64 per-column parameters of length d (see module doc)."""
    if not _use_kernel(X) or X.dtype not in (torch.float32, torch.float64):
        return col_transform_torch(X, mode, a, b, lo, hi)
    L = _lib.require()
    X = X.contiguous()
    d = X.shape[1] if X.dim() == 2 else 1
    n = X.shape[0]
    dev = X.device

    def prm(v):
        if v is None:
            return torch.zeros(d, dtype=torch.float64, device=dev)
        v = torch.as_tensor(v, dtype=torch.float64, device=dev).reshape(-1)
        assert v.numel() >= d, "per-column parameter shorter than the column count"
        return v[:d].contiguous()

    pa, pb = prm(a), prm(b)
    out = torch.empty(X.shape, dtype=torch.float64, device=dev)
    _check(L.alink_col_transform(X.data_ptr(), n, d, 0 if X.dtype == torch.float32 else 1, MODES[mode],
                                 pa.data_ptr(), pb.data_ptr(), float(lo), float(hi), out.data_ptr(),
                                 _lib.stream_ptr(dev)), "alink_col_transform")
    return out
