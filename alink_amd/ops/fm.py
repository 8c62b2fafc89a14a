"""Factorization-machine micro-batch kernels (``csrc/fm.hip``).

``fm_forward(crow, col, val, w, V, bias)`` -> ``(y [n], vx [n, k])``: one wave per CSR row.
``fm_coord_update(...)``: AdaGrad on the coordinates a micro-batch touches, one wave per coordinate segment of the
coordinate-sorted entries (deterministic, no atomics; untouched coordinates are never read or written).
Reference: ``FmOptimizer.calcY`` / ``UpdateLocalModel.updateFactors``
(``A/operator/common/optim/FmOptimizer.java:389-437``).
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["kernel_supported", "fm_forward", "fm_coord_update"]

EPS = 1.0e-8


def kernel_supported(fm, k: int) -> bool:
    return fm.is_sparse and fm.val.is_cuda and 1 <= k <= 64 and (_lib.available() or not _lib.torch_fallback_allowed())


def _csr(fm):
    return (fm.crow.to(torch.int64).contiguous(), fm.col.to(torch.int32).contiguous(),
            fm.val.to(torch.float64).contiguous())


def fm_forward(fm, w, V, bias: float, want_vx: bool = True):
    L = _lib.require()
    crow, col, val = _csr(fm)
    n = fm.nrows
    k = V.shape[1]
    dev = val.device
    y = torch.empty(n, dtype=torch.float64, device=dev)
    vx = torch.empty((n, k), dtype=torch.float64, device=dev) if want_vx else None
    rc = L.alink_fm_forward_f64(crow.data_ptr(), col.data_ptr(), val.data_ptr(), n, k,
                                None if w is None else w.data_ptr(), V.data_ptr(), float(bias), y.data_ptr(),
                                None if vx is None else vx.data_ptr(), _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_fm_forward_f64 failed: {rc}")
    return y, vx


def fm_coord_update(fm, g, vx, sw_rows, w, sg_w, V, sg_V, use, lr: float, lam1: float, lam2: float):
    """In place on ``w, sg_w, V, sg_V, use`` (fp64, contiguous; ``w``/``sg_w`` may be None)."""
    L = _lib.require()
    crow, col, val = _csr(fm)
    if val.numel() == 0:
        return
    dev = val.device
    rows = torch.repeat_interleave(torch.arange(fm.nrows, device=dev, dtype=torch.int64), crow[1:] - crow[:-1])
    keys, perm = torch.sort(col.to(torch.int64), stable=True)
    coord, counts = torch.unique_consecutive(keys, return_counts=True)
    seg = torch.zeros(counts.numel() + 1, dtype=torch.int64, device=dev)
    torch.cumsum(counts, 0, out=seg[1:])
    ent_row = rows[perm].contiguous()
    ent_val = val[perm].contiguous()
    k = V.shape[1]
    rc = L.alink_fm_coord_update_f64(seg.data_ptr(), counts.numel(), coord.contiguous().data_ptr(),
                                     ent_row.data_ptr(), ent_val.data_ptr(), g.contiguous().data_ptr(),
                                     vx.contiguous().data_ptr(), sw_rows.to(torch.float64).contiguous().data_ptr(), k,
                                     None if w is None else w.data_ptr(), None if sg_w is None else sg_w.data_ptr(),
                                     V.data_ptr(), sg_V.data_ptr(), use.data_ptr(), float(lr), float(lam1),
                                     float(lam2), EPS, _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_fm_coord_update_f64 failed: {rc}")
