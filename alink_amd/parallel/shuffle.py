"""Hash shuffle of table partitions (the relational half of pattern P9).

Reference: ``BatchSqlOperators.java:51-388`` runs distinct / groupBy / join / set operations as Flink SQL
jobs, i.e. a hash repartition on the key followed by per-partition evaluation.  Here the same plan runs over
the SPMD ranks:

* every row gets a deterministic key hash, computed column-wise in bulk where the column lives: numeric /
  boolean columns by a 64-bit mix of the value (integral values hashed as integers, so ``1`` and ``1.0``
  co-locate) in torch on the host or the GPU; string columns by MurmurHash3 over their packed UTF-8 bytes
  (``ops/strings.py``: HIP kernel for device blocks, the C++ twin on the host); other objects through their
  string form.  The bits are identical on every process (Python's ``hash`` is salted per process);
* rows move to ``hash % P``: numeric columns with one ``all_to_all_single`` each (RCCL on GPUs, gloo on CPUs),
  string columns as packed UTF-8 — one lengths and one bytes all-to-all, received as a ``StringBlock`` — so
  each rank sends and receives only its rows' bytes (about N/P of them with a balanced key);
* the operator then evaluates locally on co-partitioned data.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch

from ..common.strings import StringBlock
from ..common.table import Column, MTable
from . import comm

__all__ = ["key_hash", "hash_partition", "exchange", "ShuffleStats", "STATS"]


class ShuffleStats:
    """Per-process counters of the last / all exchanges (tests assert received bytes ~ N/P)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.rows_sent = 0
        self.rows_recv = 0
        self.string_bytes_sent = 0
        self.string_bytes_recv = 0
        self.tensor_bytes_sent = 0
        self.tensor_bytes_recv = 0


STATS = ShuffleStats()

_M32 = 0xFFFFFFFF
_NULL_HASH = 0x5BD1E995


def _s64(x: int) -> int:
    return x - (1 << 64) if x >= (1 << 63) else x


_C1, _C2 = _s64(0xff51afd7ed558ccd), _s64(0xc4ceb9fe1a85ec53)


def _lshr(k: torch.Tensor, r: int) -> torch.Tensor:
    return (k >> r) & ((1 << (64 - r)) - 1)


def _mix64(k: torch.Tensor) -> torch.Tensor:
    """MurmurHash3 fmix64 in wrapping int64 arithmetic; returns the low 32 bits (as int64 >= 0)."""
    k = k ^ _lshr(k, 33)
    k = k * _C1
    k = k ^ _lshr(k, 33)
    k = k * _C2
    k = k ^ _lshr(k, 33)
    return k & _M32


def _numeric_hash(v: torch.Tensor) -> torch.Tensor:
    if v.dtype == torch.bool:
        return _mix64(v.to(torch.int64))
    if not v.dtype.is_floating_point:
        return _mix64(v.to(torch.int64))
    x = v.to(torch.float64)
    integral = torch.isfinite(x) & (x == torch.floor(x)) & (x.abs() < 9.2e18)
    key = torch.where(integral, torch.where(integral, x, torch.zeros_like(x)).to(torch.int64), x.view(torch.int64))
    return _mix64(key)


def _object_strings(vals) -> StringBlock:
    from ..common.javafmt import java_str
    from ..common.linalg import Vector, VectorUtil
    out = []
    for v in vals:
        if v is None:
            out.append(None)
        elif isinstance(v, Vector):
            out.append(VectorUtil.toString(v))
        elif isinstance(v, (bytes, bytearray)):
            out.append(bytes(v).hex())
        else:
            out.append(java_str(v))
    return StringBlock.from_list(out)


def _is_num(x) -> bool:
    return isinstance(x, (int, float, np.integer, np.floating)) and not isinstance(x, bool)


def _hash_kind(c: Column) -> str:
    """How this rank's part of a column would hash on its own: ``num`` (numeric tensor, or numbers in an object
    column), ``str`` (strings), ``null`` (nothing but NULLs: compatible with any kind) or ``obj`` (mixed)."""
    v = c.values
    if isinstance(v, torch.Tensor) and v.dim() == 1:
        return "num"
    if isinstance(v, StringBlock):
        return "str"
    vals = c.to_list()
    if all(x is None for x in vals):
        return "null"
    if all(x is None or isinstance(x, str) for x in vals):
        return "str"
    if all(x is None or _is_num(x) for x in vals):
        return "num"
    return "obj"


def _agree_kind(kinds) -> str:
    """One hash kind every rank uses for a column (equal keys must hash equally wherever they live)."""
    ks = {k for k in kinds if k != "null"}
    if not ks:
        return "num"
    return ks.pop() if len(ks) == 1 else "obj"


def _column_hash(c: Column, kind: str = None) -> torch.Tensor:
    """int64 [n] in [0, 2^32) on the column's device; NULL rows hash to a constant.  ``kind`` (agreed across
    ranks by ``key_hash``) forces the hash family; None = this column's own ``_hash_kind``."""
    from ..ops.strings import hash_bytes
    kind = kind or _hash_kind(c)
    if kind == "null":
        kind = "num"
    v = c.values
    if kind == "num" and isinstance(v, torch.Tensor) and v.dim() == 1:
        h = _numeric_hash(v)
        nulls = c.nulls.to(h.device) if c.nulls is not None else None
    elif kind == "num":
        # numbers in an object column hash as numbers (same bits as a numeric column of those values)
        vals = c.to_list()
        h = _numeric_hash(torch.tensor([0.0 if x is None else float(x) for x in vals], dtype=torch.float64))
        nulls = torch.tensor([x is None for x in vals], dtype=torch.bool)
    else:
        if kind == "str" and isinstance(v, StringBlock):
            blk = v
        elif kind == "str":
            blk = StringBlock.from_list(c.to_list())
        else:
            # mixed on some rank: every rank hashes the Java string form of every value
            blk = v if isinstance(v, StringBlock) else _object_strings(c.to_list())
        h = hash_bytes(blk).to(torch.int64) & _M32
        nulls = blk.nulls
    if nulls is not None:
        h = torch.where(nulls.to(h.device), torch.full_like(h, _NULL_HASH), h)
    return h


def key_hash(mt: MTable, cols: Sequence[int]) -> np.ndarray:
    """int64 non-negative hash of the key columns of every row (identical on every rank).  Collective when the
    job is distributed: the per-column hash family is agreed across ranks first."""
    n = mt.num_rows
    kinds = [_hash_kind(mt.cols[c]) for c in cols]
    if comm.is_distributed():
        everyone = comm.all_gather_object(kinds)
        kinds = [_agree_kind([k[i] for k in everyone]) for i in range(len(cols))]
    h = torch.zeros(n, dtype=torch.int64)
    for c, kind in zip(cols, kinds):
        hc = _column_hash(mt.cols[c], kind).cpu()
        h = (h * 31 + hc) & _M32
    return (h & 0x7FFFFFFF).numpy()


def _is_string_column(c: Column) -> bool:
    if isinstance(c.values, StringBlock):
        return True
    return isinstance(c.values, list) and all(x is None or isinstance(x, str) for x in c.values)


def exchange(mt: MTable, dest: np.ndarray) -> MTable:
    """Send row i to rank ``dest[i]``; returns the rows this rank received (source-rank order, stable)."""
    ws = comm.get_world_size()
    if ws == 1:
        return mt
    dest = np.asarray(dest, dtype=np.int64)
    order = np.argsort(dest, kind="stable")
    counts = np.bincount(dest, minlength=ws)
    bounds = np.concatenate([[0], np.cumsum(counts)])
    me = comm.get_rank()
    STATS.rows_sent += int(mt.num_rows - counts[me])
    # the string decision and the presence of a NULL mask must agree across ranks (a column may be all-None, or
    # NULL-free, on some ranks only): ONE object gather of both, so every rank issues the same collectives
    local = [(_is_string_column(c), c.nulls is not None) for c in mt.cols]
    agreed = comm.all_gather_object(local)
    is_str = [all(a[i][0] for a in agreed) for i in range(len(mt.cols))]
    any_nulls = [any(a[i][1] for a in agreed) for i in range(len(mt.cols))]
    cols = []
    for ci, c in enumerate(mt.cols):
        v = c.values
        if isinstance(v, torch.Tensor):
            srt = v[torch.as_tensor(order, device=v.device)]
            parts = [srt[bounds[j]:bounds[j + 1]] for j in range(ws)]
            flat = [p.reshape(p.shape[0], -1) if p.dim() > 1 else p[:, None] for p in parts]
            recv = torch.cat(comm.all_to_all_tensors([f.contiguous() for f in flat]))
            STATS.tensor_bytes_sent += int(sum(f.numel() * f.element_size() for j, f in enumerate(flat) if j != me))
            STATS.tensor_bytes_recv += int(recv.numel() * recv.element_size())
            val = recv.reshape((recv.shape[0],) + tuple(v.shape[1:])) if v.dim() > 1 else recv[:, 0]
            nulls = None
            if any_nulls[ci]:
                nm = c.nulls if c.nulls is not None else torch.zeros(v.shape[0], dtype=torch.bool)
                nm = nm.cpu()[torch.as_tensor(order)]
                nparts = [nm[bounds[j]:bounds[j + 1]].to(torch.uint8)[:, None] for j in range(ws)]
                nulls = torch.cat(comm.all_to_all_tensors(nparts))[:, 0].to(torch.bool).to(v.device)
                if not bool(nulls.any()):
                    nulls = None
            cols.append(Column(val.to(v.device), nulls))
        elif is_str[ci]:
            blk = v if isinstance(v, StringBlock) else StringBlock.from_list(c.to_list())
            srt = blk.take(torch.as_tensor(order, device=blk.device))
            parts = [srt.take(slice(int(bounds[j]), int(bounds[j + 1]))) for j in range(ws)]
            got = comm.all_to_all_strings(parts)
            STATS.string_bytes_sent += int(sum(p.nbytes for j, p in enumerate(parts) if j != me))
            recv = StringBlock.concat(got)
            STATS.string_bytes_recv += recv.nbytes
            cols.append(Column(recv))
        else:
            lst = c.to_list()
            lst = [lst[i] for i in order]
            parts = [lst[bounds[j]:bounds[j + 1]] for j in range(ws)]
            got = comm.all_to_all_objects(parts)
            cols.append(Column([x for part in got for x in part]))
    out = MTable(mt.schema, cols, False)
    STATS.rows_recv += int(out.num_rows)
    return out


def hash_partition(mt: MTable, cols: Sequence[int]) -> MTable:
    """Co-partition ``mt`` by the key columns: equal keys end up on the same rank."""
    ws = comm.get_world_size()
    if ws == 1 or mt.replicated:
        return mt
    return exchange(mt, key_hash(mt, cols) % ws)
