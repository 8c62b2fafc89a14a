"""Hash shuffle of table partitions (the relational half of pattern P9).

Reference: ``BatchSqlOperators.java:51-388`` runs distinct / groupBy / join / set operations as Flink SQL
jobs, i.e. a hash repartition on the key followed by per-partition evaluation.  Here the same plan runs over
the SPMD ranks: every row gets a deterministic key hash (Guava murmur3 of the key values' Java strings — the
same bits on every process; Python's ``hash`` is salted per process), rows move to ``hash % P`` with ONE
all-to-all per column (tensor columns through ``all_to_all_single`` — RCCL on GPUs, gloo on CPUs; object
columns through one pickled all-to-all, O(N) total instead of the O(N * P) of gathering every partition to
every rank), and the operator then evaluates locally on co-partitioned data.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from ..common.javafmt import java_str
from ..common.table import Column, MTable
from . import comm

__all__ = ["key_hash", "hash_partition", "exchange"]


def _key_strings(mt: MTable, cols: Sequence[int]) -> List[str]:
    from ..common.linalg import Vector, VectorUtil
    vals = [mt.cols[c].to_list() for c in cols]
    out = []
    for row in zip(*vals) if vals else [() for _ in range(mt.num_rows)]:
        parts = []
        for v in row:
            if v is None:
                parts.append("\x00null")
            elif isinstance(v, Vector):
                parts.append(VectorUtil.toString(v))
            elif isinstance(v, bool):
                parts.append(java_str(v))
            elif isinstance(v, (float, np.floating)) and float(v).is_integer():
                parts.append(str(int(v)))          # 1.0 and 1 compare equal locally -> same partition
            elif isinstance(v, (int, np.integer)):
                parts.append(str(int(v)))
            else:
                parts.append(java_str(v))
        out.append("\x01".join(parts))
    return out


def key_hash(mt: MTable, cols: Sequence[int]) -> np.ndarray:
    """int64 non-negative hash of the key columns of every row (identical on every rank)."""
    from .. import _native
    keys = _key_strings(mt, cols)
    h = _native.murmur3_utf16(keys) if keys else np.zeros(0, dtype=np.int64)
    if h is None:
        from ..models.feature.encoders import _murmur3_py
        h = np.array([_murmur3_py(k) for k in keys], dtype=np.int64)
    return np.asarray(h, dtype=np.int64) & 0x7FFFFFFF


def exchange(mt: MTable, dest: np.ndarray) -> MTable:
    """Send row i to rank ``dest[i]``; returns the rows this rank received (source-rank order, stable)."""
    ws = comm.get_world_size()
    if ws == 1:
        return mt
    dest = np.asarray(dest, dtype=np.int64)
    order = np.argsort(dest, kind="stable")
    counts = np.bincount(dest, minlength=ws)
    bounds = np.concatenate([[0], np.cumsum(counts)])
    srt = mt.take(order)
    cols = []
    for c in srt.cols:
        v = c.values
        if isinstance(v, torch.Tensor):
            parts = [v[bounds[j]:bounds[j + 1]] for j in range(ws)]
            flat = [p.reshape(p.shape[0], -1) if p.dim() > 1 else p[:, None] for p in parts]
            recv = torch.cat(comm.all_to_all_tensors([f.contiguous() for f in flat]))
            val = recv.reshape((recv.shape[0],) + tuple(v.shape[1:])) if v.dim() > 1 else recv[:, 0]
            nulls = None
            if c.nulls is not None:
                nparts = [c.nulls[bounds[j]:bounds[j + 1]].to(torch.uint8)[:, None].cpu() for j in range(ws)]
                nulls = torch.cat(comm.all_to_all_tensors(nparts))[:, 0].to(torch.bool).to(v.device)
            cols.append(Column(val.to(v.device), nulls))
        else:
            lst = c.to_list()
            parts = [lst[bounds[j]:bounds[j + 1]] for j in range(ws)]
            got = comm.all_to_all_objects(parts)
            cols.append(Column([x for part in got for x in part]))
    return MTable(mt.schema, cols, False)


def hash_partition(mt: MTable, cols: Sequence[int]) -> MTable:
    """Co-partition ``mt`` by the key columns: equal keys end up on the same rank."""
    ws = comm.get_world_size()
    if ws == 1 or mt.replicated:
        return mt
    return exchange(mt, key_hash(mt, cols) % ws)
