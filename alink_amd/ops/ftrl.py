"""Hogwild FTRL-proximal micro-batch update on the GPU (kernel K19) — ``csrc/ftrl.hip``.

``ftrl_hogwild(indptr, idx, val, label, w, n, z, ...)`` applies the FTRL-proximal rule of
``FtrlTrainStreamOp.java:423-485`` to every CSR row of a micro-batch, one wave per sample, in place on the
device-resident ``w, n, z`` (fp64).  ``n`` and ``z`` receive exact sums of every sample's contribution; the
weights a sample reads may be stale, as in the reference's asynchronous feedback loop.  A prox pass then makes
``w`` consistent with the final ``n, z``.

The feature-sharded micro-batch update (updateMode SHARDED) is ``ftrl_partial_margin_hip`` (per-rank
partial margins, all-reduced by the caller) + ``ftrl_shard_update_hip`` (per-coordinate replay in sample order).
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["ftrl_hogwild", "ftrl_prox_hip", "ftrl_partial_margin_hip", "ftrl_shard_update_hip", "ftrl_dp_gradients",
           "ftrl_dp_update"]


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
    # the racing w stores are last-writer-wins: re-derive w = prox(z, n) of every touched coordinate from the
    # exact atomic n/z sums (same stream, after the update kernel)
    ftrl_prox_hip(w, n, z, alpha, beta, l1, l2, coords=torch.unique(idx))


LONG_SEGMENT = 256
# segments with more entries (the intercept: every sample) take the whole-segment speculative block scan
# (ftrl_coord_scan_kernel) instead of the one-wave chunk walk
_FOREIGN = 1 << 62          # sort key of entries another shard owns (after every coordinate)
SCAN_SEGMENT = int(__import__("os").environ.get("ALINK_FTRL_SCAN_SEGMENT", "4096"))


def _grid(n: int, per: int, cap: int = 4096) -> int:
    return max(1, min((n + per - 1) // per, cap))


def ftrl_prox_hip(w: torch.Tensor, n: torch.Tensor, z: torch.Tensor, alpha: float, beta: float, l1: float, l2: float,
                  coords: torch.Tensor = None) -> None:
    """``w_i = prox(z_i, n_i)`` on the device for ``coords`` (int32) or every coordinate."""
    L = _lib.require()
    m = w.shape[0] if coords is None else coords.shape[0]
    if coords is not None:
        coords = coords.to(device=w.device, dtype=torch.int32).contiguous()
    rc = L.alink_ftrl_prox_f64(None if coords is None else coords.data_ptr(), m, w.data_ptr(), n.data_ptr(),
                               z.data_ptr(), float(alpha), float(beta), float(l1), float(l2), _grid(m, 256),
                               _lib.stream_ptr(w.device))
    if rc != 0:
        raise RuntimeError(f"alink_ftrl_prox_f64 failed: {rc}")


def ftrl_partial_margin_hip(indptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, w: torch.Tensor, lo: int,
                            hi: int) -> torch.Tensor:
    """Per-row ``sum_{lo <= i < hi} x_i w_i`` (``w`` = the owned shard) — one wave per row."""
    L = _lib.require()
    dev = w.device
    nrows = indptr.shape[0] - 1
    out = torch.zeros(max(nrows, 0), dtype=torch.float64, device=dev)
    if nrows <= 0:
        return out
    rc = L.alink_ftrl_partial_margin_f64(indptr.data_ptr(), idx.data_ptr(), val.data_ptr(), nrows, w.data_ptr(),
                                         int(lo), int(hi), out.data_ptr(), _grid(nrows, 4), _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_ftrl_partial_margin_f64 failed: {rc}")
    return out


def ftrl_shard_update_hip(indptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, err: torch.Tensor,
                          w: torch.Tensor, n: torch.Tensor, z: torch.Tensor, lo: int, hi: int, alpha: float,
                          beta: float, l1: float, l2: float) -> None:
    """Owned coordinates [lo, hi) replay their entries in sample order with ``err = p - y`` fixed for the
    micro-batch: entries stably sorted by coordinate on the device (entries of other shards keyed past every
    coordinate), one lane per coordinate segment (``ftrl_coord_update_kernel``), one wave per segment longer than
    ``LONG_SEGMENT`` (``ftrl_coord_long_kernel``), one 512-thread speculative scan per segment longer than
    ``SCAN_SEGMENT`` (``ftrl_coord_scan_kernel``).  Segment boundaries, the long-segment lists and their lengths
    stay on the device (the kernels read the counts there): no host synchronisation in the whole update."""
    L = _lib.require()
    dev = w.device
    nrows = indptr.shape[0] - 1
    nnz = idx.numel()
    if nrows <= 0 or nnz == 0:
        return
    st = _lib.stream_ptr(dev)
    lens = indptr[1:] - indptr[:-1]
    erow = torch.repeat_interleave(torch.arange(nrows, device=dev, dtype=torch.int64), lens, output_size=nnz)
    ii = idx.to(torch.int64)
    keys = torch.where((ii >= lo) & (ii < hi), ii, torch.full_like(ii, _FOREIGN))
    keys, ent = torch.sort(keys, stable=True)
    g = (err[erow[ent]] * val[ent]).contiguous()          # per-entry gradient, in coordinate-sorted order
    ar = torch.arange(nnz, device=dev, dtype=torch.int64)
    head = torch.ones(nnz, dtype=torch.bool, device=dev)
    torch.ne(keys[1:], keys[:-1], out=head[1:])
    sid = torch.cumsum(head, 0) - 1
    nseg = sid[-1:] + 1                                    # device scalar
    seg = torch.empty(nnz + 2, dtype=torch.int64, device=dev)
    seg.index_put_((torch.where(head, sid, nnz + 1),), ar)     # seg[q] = first entry of segment q (nnz + 1: dummy)
    seg.index_put_((nseg,), torch.full((1,), nnz, dtype=torch.int64, device=dev))
    first = seg[:nnz].clamp(0, nnz - 1)                    # slots past nseg hold garbage: never read as segments
    coord = keys[first].contiguous()
    cnt = seg[1:nnz + 1] - seg[:nnz]
    live = (ar < nseg) & (coord < hi)
    rc = L.alink_ftrl_coord_update_f64(seg.data_ptr(), nnz, nseg.data_ptr(), coord.data_ptr(), g.data_ptr(),
                                       w.data_ptr(), n.data_ptr(), z.data_ptr(), int(lo), int(hi), float(alpha),
                                       float(beta), float(l1), float(l2), LONG_SEGMENT, _grid(nnz, 256), st)
    if rc != 0:
        raise RuntimeError(f"alink_ftrl_coord_update_f64 failed: {rc}")
    # segments longer than LONG_SEGMENT (the intercept, hot categorical values): compacted id lists + counts on
    # the device; the kernels stride over them from a fixed grid
    for fn, sel, grid in ((L.alink_ftrl_coord_long_f64, live & (cnt > LONG_SEGMENT) & (cnt <= SCAN_SEGMENT), 256),
                          (L.alink_ftrl_coord_scan_f64, live & (cnt > SCAN_SEGMENT), 16)):
        pos = torch.cumsum(sel, 0) - 1
        lst = torch.empty(nnz + 1, dtype=torch.int64, device=dev)
        lst.index_put_((torch.where(sel, pos, nnz),), ar)
        num = pos[-1:] + 1
        rc = fn(seg.data_ptr(), coord.data_ptr(), lst.data_ptr(), nnz, num.data_ptr(), g.data_ptr(), w.data_ptr(),
                n.data_ptr(), z.data_ptr(), int(lo), float(alpha), float(beta), float(l1), float(l2), grid, st)
        if rc != 0:
            raise RuntimeError(f"{fn.__name__} failed: {rc}")


def ftrl_dp_gradients(indptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, label: torch.Tensor,
                      w: torch.Tensor):
    """DATA_PARALLEL mini-batch: margins of the local samples with the current w, and the per-coordinate
    gradient sums ``gq = [sum g, sum g^2]`` ([2, dim] fp64, g = (sigmoid(margin) - y) x) — the one dense buffer
    the ranks all-reduce per step.  Returns (gq, margin).

    No atomics: a click stream puts the intercept and a few hot values in every sample, and fp64 atomic adds on
    one address serialise (torch ``index_add_`` took ~1.3 s per 65536-sample batch).  Margins come from the
    row-parallel HIP kernel on GPU; gradient sums are segmented reductions over the entries sorted (stably, so
    the summation order is deterministic) by coordinate."""
    dev = w.device
    dim = w.numel()
    gq = torch.zeros((2, dim), dtype=torch.float64, device=dev)
    nrow = indptr.numel() - 1
    if nrow <= 0 or idx.numel() == 0:
        return gq, torch.zeros(max(nrow, 0), dtype=torch.float64, device=dev)
    if w.is_cuda:
        margin = ftrl_partial_margin_hip(indptr, idx, val, w, 0, dim)
    else:
        rows = torch.repeat_interleave(torch.arange(nrow, device=dev), indptr[1:] - indptr[:-1])
        margin = torch.zeros(nrow, dtype=torch.float64, device=dev)
        margin.index_add_(0, rows, w[idx.to(torch.int64)] * val)
    err = torch.sigmoid(margin) - label.to(torch.float64)
    rows = torch.repeat_interleave(torch.arange(nrow, device=dev), indptr[1:] - indptr[:-1])
    g = err[rows] * val
    il = idx.to(torch.int64)
    order = torch.argsort(il, stable=True)
    ils, gs = il[order], g[order]
    uniq, counts = torch.unique_consecutive(ils, return_counts=True)
    gq[0, uniq] = torch.segment_reduce(gs, "sum", lengths=counts)
    gq[1, uniq] = torch.segment_reduce(gs * gs, "sum", lengths=counts)
    return gq, margin


def ftrl_dp_update(gq: torch.Tensor, w: torch.Tensor, n: torch.Tensor, z: torch.Tensor, alpha: float, beta: float,
                   l1: float, l2: float) -> None:
    """Mini-batch FTRL-proximal step from the (all-reduced) gradient sums, in place on w, n, z: for every touched
    coordinate sigma = (sqrt(n + sum g^2) - sqrt(n)) / alpha, z += sum g - sigma w, n += sum g^2,
    w = prox(z, n) (reference per-sample rule FtrlTrainStreamOp.java:396-420 applied once per mini-batch)."""
    touched = gq[1] > 0
    sigma = (torch.sqrt(n + gq[1]) - torch.sqrt(n)) / alpha
    z += torch.where(touched, gq[0] - sigma * w, torch.zeros_like(z))
    n += gq[1]
    denom = (beta + torch.sqrt(n)) / alpha + l2
    neww = torch.where(z.abs() <= l1, torch.zeros_like(z), -(z - torch.sign(z) * l1) / denom)
    w.copy_(torch.where(touched, neww, w))
