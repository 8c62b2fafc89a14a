"""Hogwild FTRL-proximal micro-batch update on the GPU (kernel K19) — ``csrc/ftrl.hip``.

``ftrl_hogwild(indptr, idx, val, label, w, n, z, ...)`` applies the FTRL-proximal rule of
``FtrlTrainStreamOp.java:423-485`` to every CSR row of a micro-batch, one wave per sample, in place on the
device-resident ``w, n, z`` (fp64).  ``n`` and ``z`` receive exact sums of every sample's contribution; the
weights a sample reads may be stale, as in the reference's asynchronous feedback loop.
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["ftrl_hogwild"]


def ftrl_hogwild(indptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, label: torch.Tensor, w: torch.Tensor,
                 n: torch.Tensor, z: torch.Tensor, alpha: float, beta: float, l1: float, l2: float) -> None:
    L = _lib.require()
    dev = w.device
    if not (w.is_cuda and w.dtype == torch.float64 and n.shape == w.shape and z.shape == w.shape):
        raise ValueError("ftrl_hogwild needs fp64 CUDA state vectors of one shape")
    if not (w.is_contiguous() and n.is_contiguous() and z.is_contiguous()):
        raise ValueError("ftrl_hogwild needs contiguous state vectors")
    indptr = indptr.to(device=dev, dtype=torch.int64).contiguous()
    idx = idx.to(device=dev, dtype=torch.int32).contiguous()
    val = val.to(device=dev, dtype=torch.float64).contiguous()
    label = label.to(device=dev, dtype=torch.float64).contiguous()
    nrows = indptr.shape[0] - 1
    if nrows <= 0:
        return
    nnz = int(indptr[-1].item())
    if nnz != idx.shape[0] or nnz != val.shape[0] or label.shape[0] != nrows:
        raise ValueError("CSR arrays do not match the row pointer")
    st = _lib.stream_ptr(dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = L.alink_ftrl_check_indices(idx.data_ptr(), nnz, w.shape[0], bad.data_ptr(), 1024, st)
    if rc != 0:
        raise RuntimeError(f"alink_ftrl_check_indices failed: {rc}")
    if int(bad.item()) != 0:
        raise ValueError("feature index out of range of the model")
    grid = max(1, min((nrows + 3) // 4, 2048))
    rc = L.alink_ftrl_hogwild_f64(indptr.data_ptr(), idx.data_ptr(), val.data_ptr(), label.data_ptr(), nrows,
                                  w.data_ptr(), n.data_ptr(), z.data_ptr(), float(alpha), float(beta), float(l1),
                                  float(l2), grid, st)
    if rc != 0:
        raise RuntimeError(f"alink_ftrl_hogwild_f64 failed: {rc}")
