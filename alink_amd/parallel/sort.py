"""Distributed sample sort / range partitioning (pattern P9).

Reference: ``SortUtils.pSort`` (``A/operator/common/dataproc/SortUtils.java:38``) — sample splitters, range
partition, local sort — and Flink's ``partitionByRange`` used by isotonic regression
(``IsotonicRegTrainBatchOp.java:101-103``).  Here: every rank contributes a uniform sample of its keys, the
``P-1`` splitters are chosen from the all-gathered sample, rows move with ONE tensor all-to-all
(``all_to_all_single`` over RCCL on GPUs, gloo on CPU) and each rank sorts what it received, so rank ``r``
ends up holding the ``r``-th key range in sorted order.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import comm

__all__ = ["range_partition", "sample_sort"]


def _splitters(keys: torch.Tensor, ws: int, samples_per_rank: int = 256) -> torch.Tensor:
    n = keys.shape[0]
    if n:
        idx = torch.linspace(0, n - 1, steps=min(samples_per_rank, n)).round().long().to(keys.device)
        smp = torch.sort(keys)[0][idx]
    else:
        smp = keys[:0]
    allsmp = torch.sort(comm.all_gather_varlen(smp.to(torch.float64)).cpu())[0]
    if allsmp.numel() == 0:
        return torch.zeros(0, dtype=torch.float64)
    q = torch.linspace(0, allsmp.numel() - 1, steps=ws + 1)[1:-1].round().long()
    return allsmp[q]


def range_partition(keys: torch.Tensor, payload: Sequence[torch.Tensor]) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """Move rows so rank r holds the r-th key range; returns (keys, payload) of this rank (unsorted)."""
    ws = comm.get_world_size()
    if ws == 1:
        return keys, list(payload)
    spl = _splitters(keys, ws).to(keys.device, keys.dtype)
    dest = torch.bucketize(keys, spl, right=True) if spl.numel() else torch.zeros_like(keys, dtype=torch.long)
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=ws).tolist()
    cols = [keys.to(torch.float64)] + [p.to(torch.float64) for p in payload]
    packed = torch.stack(cols, 1)[order]
    parts = list(torch.split(packed, counts))
    recv = torch.cat(comm.all_to_all_tensors(parts))
    return recv[:, 0].to(keys.dtype), [recv[:, 1 + i].to(p.dtype) for i, p in enumerate(payload)]


def sample_sort(keys: torch.Tensor, payload: Sequence[torch.Tensor] = (), secondary: torch.Tensor = None):
    """Globally sorted (by key, then ``secondary``) rows, range-partitioned over ranks."""
    pay = list(payload) + ([secondary] if secondary is not None else [])
    k, p = range_partition(keys, pay)
    if secondary is not None:
        sec = p[-1]
        o2 = torch.argsort(sec, stable=True)
        o1 = torch.argsort(k[o2], stable=True)
        order = o2[o1]
        p = p[:-1]
    else:
        order = torch.argsort(k, stable=True)
    return k[order], [x[order] for x in p]
