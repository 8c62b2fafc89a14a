"""Column statistics of a dense device matrix in one pass (``csrc/colstats.hip``).

``colstats(X)`` -> dict of fp64 [d] tensors ``sum, sum2, l1, min, max, nnz`` over the rows of ``X`` [n, d]
(fp32 / fp64 / bf16, read in place).  Reference: ``DenseVectorSummarizer.visit``
(``A/common/statistics/basicstatistic/DenseVectorSummarizer.java:78-120``).  CPU tensors use torch.
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["colstats", "colstats_torch", "kernel_supported"]

_DT = {torch.float32: 0, torch.float64: 1, torch.bfloat16: 2}
TB = 256


def kernel_supported(X: torch.Tensor) -> bool:
    return X.is_cuda and X.dim() == 2 and X.dtype in _DT and (_lib.available() or not _lib.torch_fallback_allowed())


def colstats_torch(X: torch.Tensor) -> dict:
    Xd = X.double()
    d = X.shape[1]
    if X.shape[0]:
        mn, mx = Xd.min(0).values, Xd.max(0).values
    else:
        mn = torch.full((d,), float("inf"), dtype=torch.float64, device=X.device)
        mx = -mn
    return {"sum": Xd.sum(0), "sum2": (Xd * Xd).sum(0), "l1": Xd.abs().sum(0), "min": mn, "max": mx,
            "nnz": (Xd != 0).sum(0).double()}


def colstats(X: torch.Tensor, use_kernel: bool = None) -> dict:
    if use_kernel is None:
        use_kernel = kernel_supported(X)
    if not use_kernel:
        return colstats_torch(X)
    L = _lib.require()
    X = X.contiguous()
    n, d = X.shape
    chunks = (d + TB - 1) // TB
    phases = max(1, TB // min(d, TB))
    slabs = int(max(1, min((n + 4 * phases - 1) // (4 * phases), max(1, 2048 // chunks))))
    part = torch.empty((slabs, 6, d), dtype=torch.float64, device=X.device)
    rc = L.alink_colstats(X.data_ptr(), n, d, _DT[X.dtype], slabs, part.data_ptr(), _lib.stream_ptr(X.device))
    if rc != 0:
        raise RuntimeError(f"alink_colstats failed: {rc}")
    tot = part[:, [0, 1, 2, 5]].sum(0)
    return {"sum": tot[0], "sum2": tot[1], "l1": tot[2], "min": part[:, 3].amin(0), "max": part[:, 4].amax(0),
            "nnz": tot[3]}
