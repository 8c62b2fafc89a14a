"""Distributed sample sort / range partitioning (pattern P9).

Reference: ``SortUtils.pSort`` (``A/operator/common/dataproc/SortUtils.java:38``) — sample splitters, range
partition, local sort — and Flink's ``partitionByRange`` used by isotonic regression
(``IsotonicRegTrainBatchOp.java:101-103``).  Here: every rank contributes a uniform sample of its keys, the
``P-1`` splitters are chosen from the all-gathered sample, rows move with ONE tensor all-to-all
(``all_to_all_single`` over RCCL on GPUs, gloo on CPU) and each rank sorts what it received, so rank ``r``
ends up holding the ``r``-th key range in sorted order.
"""
from __future__ import annotations

from typing import Any, List, Sequence, Tuple

import numpy as np
import torch

from . import comm

__all__ = ["range_partition", "sample_sort", "global_average_ranks", "global_order_statistics", "merged_vocabulary"]


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
    # every column travels as its exact 64-bit pattern (int64 keys / payload keep all their bits)
    cols = [_as_bits(keys)] + [_as_bits(p) for p in payload]
    packed = torch.stack(cols, 1)[order]
    parts = list(torch.split(packed, counts))
    recv = torch.cat(comm.all_to_all_tensors(parts))
    return _from_bits(recv[:, 0], keys.dtype), [_from_bits(recv[:, 1 + i], p.dtype) for i, p in enumerate(payload)]


def _as_bits(t: torch.Tensor) -> torch.Tensor:
    if t.dtype == torch.int64:
        return t
    if t.dtype == torch.float64:
        return t.contiguous().view(torch.int64)
    return (t.to(torch.float64) if t.is_floating_point() else t.to(torch.int64)).contiguous().view(torch.int64) \
        if t.is_floating_point() else t.to(torch.int64)


def _from_bits(b: torch.Tensor, dtype) -> torch.Tensor:
    if dtype == torch.int64:
        return b.contiguous()
    if dtype == torch.float64:
        return b.contiguous().view(torch.float64)
    if dtype.is_floating_point:
        return b.contiguous().view(torch.float64).to(dtype)
    return b.to(dtype)


def total_order_key(v: torch.Tensor) -> torch.Tensor:
    """int64 keys ordering float64 values like Java's ``Double.compare`` (-0.0 < 0.0); ``from_total_order_key``
    inverts it exactly."""
    b = v.to(torch.float64).contiguous().view(torch.int64)
    return torch.where(b < 0, b ^ 0x7FFFFFFFFFFFFFFF, b)


def from_total_order_key(k: torch.Tensor) -> torch.Tensor:
    return torch.where(k < 0, k ^ 0x7FFFFFFFFFFFFFFF, k).contiguous().view(torch.float64)


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


def _counts(n: int) -> List[int]:
    return [int(c) for c in comm.all_gather_tensor(torch.tensor([int(n)], dtype=torch.int64)).tolist()]


def _run_average_ranks(s: torch.Tensor, offset: int) -> torch.Tensor:
    """1-based average ranks of an ascending-sorted vector (ties averaged), shifted by ``offset`` rows."""
    n = s.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.float64, device=s.device)
    new = torch.ones(n, dtype=torch.bool, device=s.device)
    new[1:] = s[1:] != s[:-1]
    run = torch.cumsum(new.to(torch.int64), 0) - 1
    starts = torch.nonzero(new).reshape(-1)
    ends = torch.cat([starts[1:], torch.tensor([n], device=s.device)])
    avg = (starts + ends + 1).to(torch.float64) * 0.5 + float(offset)     # mean of (start+1 .. end)
    return avg[run]


def global_average_ranks(v: torch.Tensor) -> torch.Tensor:
    """Average ranks (1-based, ties averaged: scipy ``rankdata(method='average')``) of this rank's values within
    the GLOBAL column (every rank's rows), in this rank's row order.  Distributed: ``sample_sort`` (the reference's
    ``SortUtils.pSort``) — the range partition sends equal keys to the same rank, so every tie run is local after
    the exchange — then each rank ranks its range from its global offset and the ranks travel back to their rows'
    owners in one all-to-all.  Nothing is gathered whole on any rank."""
    v = v.to(torch.float64)
    n = v.shape[0]
    if comm.get_world_size() == 1:
        order = torch.sort(v, stable=True).indices
        out = torch.empty(n, dtype=torch.float64, device=v.device)
        out[order] = _run_average_ranks(v[order], 0)
        return out
    me, ws = comm.get_rank(), comm.get_world_size()
    origin = torch.full((n,), float(me), dtype=torch.float64, device=v.device)
    idx = torch.arange(n, dtype=torch.float64, device=v.device)
    k, (org, li) = sample_sort(v, [origin, idx])
    off = sum(_counts(k.shape[0])[:me])
    r = _run_average_ranks(k, off)
    dest = org.to(torch.int64)
    order = torch.argsort(dest, stable=True)
    cnt = torch.bincount(dest, minlength=ws).tolist()
    packed = torch.stack([li, r], 1)[order]
    recv = torch.cat(comm.all_to_all_tensors(list(torch.split(packed, cnt))))
    out = torch.empty(n, dtype=torch.float64, device=v.device)
    out[recv[:, 0].to(torch.int64)] = recv[:, 1]
    return out


def global_order_statistics(v: torch.Tensor, positions_fn) -> Tuple[int, np.ndarray]:
    """(N, values) where N is the global number of values (all ranks) and ``values[j]`` the element at 0-based
    global sorted position ``positions_fn(N)[j]`` — exact quantiles without gathering the column: a device sort on
    one rank, ``sample_sort`` + a count prefix on several (each rank fills the positions inside its range, one
    SUM all-reduce assembles them)."""
    # sorted in Java's Double.compare order (-0.0 before 0.0) through exact int64 total-order keys, so the
    # value at a position is the same on any number of ranks, sign of zero included
    key = total_order_key(v)
    N = sum(_counts(v.shape[0])) if comm.get_world_size() > 1 else int(v.shape[0])
    pos = [int(p) for p in positions_fn(N)]
    if not pos or N == 0:
        return N, np.zeros(len(pos))
    if comm.get_world_size() == 1:
        s = torch.sort(key).values
        return N, from_total_order_key(s[torch.as_tensor(pos, device=v.device)]).cpu().numpy()
    k, _ = sample_sort(key)
    off = sum(_counts(k.shape[0])[:comm.get_rank()])
    # exactly one rank owns each position: a SUM of the owners' keys (zeros elsewhere) is exact in int64
    buf = torch.zeros(len(pos), dtype=torch.int64, device=v.device)
    p = torch.as_tensor(pos, dtype=torch.int64, device=v.device)
    mine = (p >= off) & (p < off + k.shape[0])
    buf[mine] = k[p[mine] - off]
    comm.all_reduce(buf, "sum")
    return N, from_total_order_key(buf).cpu().numpy()


def merged_vocabulary(local: dict, keep=None) -> List[Tuple[str, Any]]:
    """Global (word, value) pairs from per-rank partial counts (``local``: word -> int count or tuple of int
    counts, summed elementwise), in the reference's vocabulary order: first value descending, ties by word
    ascending (``SortUtils.pSort`` on the count, ``Word2VecTrainBatchOp.java:145``,
    ``DocCountVectorizerTrainBatchOp.java:77``).  Every word is reduced on ONE owner rank (hash exchange of packed
    UTF-8 + int64 counts, not a gather of every rank's dictionary), filtered there by ``keep(word, value)``, and
    only the surviving merged entries are all-gathered (the model needs the whole vocabulary on every rank)."""
    ws = comm.get_world_size()
    items = list(local.items())
    tup = bool(items) and isinstance(items[0][1], tuple)
    if ws > 1:
        width = max(comm.all_gather_object(len(items[0][1]) if tup else (1 if items else 0)))
        tup = tup or width > 1
        from ..common.strings import StringBlock
        import zlib
        dest = [zlib.crc32(w.encode("utf-8")) % ws for w, _ in items]
        words = [[] for _ in range(ws)]
        vals = [[] for _ in range(ws)]
        for (w, c), d in zip(items, dest):
            words[d].append(w)
            vals[d].append(c if tup else (c,))
        got_w = comm.all_to_all_strings([StringBlock.from_list(p) for p in words])
        got_v = comm.all_to_all_tensors([torch.tensor(v, dtype=torch.int64).reshape(-1, max(width, 1))
                                         for v in vals])
        merged: dict = {}
        for wb, vb in zip(got_w, got_v):
            for w, row in zip(wb.to_list(), vb.tolist()):
                prev = merged.get(w)
                merged[w] = tuple(row) if prev is None else tuple(a + b for a, b in zip(prev, row))
        if not tup:
            merged = {w: c[0] for w, c in merged.items()}
        local_keep = [(w, c) for w, c in merged.items() if keep is None or keep(w, c)]
        parts = comm.all_gather_object(local_keep)
        allv = [x for p in parts for x in p]
    else:
        allv = [(w, c) for w, c in items if keep is None or keep(w, c)]
    if not allv:
        return []
    first = np.asarray([c[0] if isinstance(c, tuple) else c for _, c in allv], dtype=np.int64)
    wordarr = np.asarray([w for w, _ in allv], dtype=object)
    order = np.lexsort((wordarr.astype(str), -first))
    return [allv[i] for i in order.tolist()]
