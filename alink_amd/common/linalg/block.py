"""Columnar sparse-vector block: a whole vector column as one CSR triple of tensors.

A ``Column`` whose values are a ``SparseBlock`` carries ``n`` sparse vectors as ``crow [n+1] int64``,
``col [nnz] int32``, ``val [nnz] float64`` (row-sorted, unique indices) on the rank's device, instead of ``n``
Python ``SparseVector`` objects.  It is what the GPU feature path produces (FeatureHasher / OneHot /
VectorAssembler, ``ops/csrc/feature.hip``) and what ``extract_features`` hands to the linear / FTRL kernels
without touching the host.

It behaves like a read-only sequence of vectors (``len``, ``iter``, ``[i]``) so row-wise code (mappers, sinks,
printing, the model-table writers) keeps working: rows materialise lazily as ``SparseVector`` — or as
``DenseVector`` when ``dense_ratio`` is set and ``nnz * dense_ratio > size`` (the VectorAssembler rule,
reference ``VectorAssemblerMapper.java:94-99``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from .vector import DenseVector, SparseVector

__all__ = ["SparseBlock"]


class SparseBlock:
    __slots__ = ("crow", "col", "val", "size", "dense_ratio", "_host")

    def __init__(self, crow: torch.Tensor, col: torch.Tensor, val: torch.Tensor, size: int,
                 dense_ratio: Optional[float] = None):
        if crow.dim() != 1 or col.shape != val.shape:
            raise ValueError("SparseBlock needs crow [n+1] and col/val [nnz]")
        self.crow = crow.to(torch.int64)
        self.col = col.to(torch.int32)
        self.val = val.to(torch.float64)
        self.size = int(size)
        self.dense_ratio = dense_ratio
        self._host = None

    # ---------------------------------------------------------------- sequence protocol
    def __len__(self) -> int:
        return int(self.crow.shape[0]) - 1

    @property
    def device(self):
        return self.val.device

    @property
    def nnz(self) -> int:
        return int(self.col.shape[0])

    def _np(self):
        if self._host is None:
            self._host = (self.crow.cpu().numpy(), self.col.cpu().numpy(), self.val.cpu().numpy())
        return self._host

    def _vec(self, crow, col, val, i):
        s, e = int(crow[i]), int(crow[i + 1])
        if self.dense_ratio is not None and (e - s) * self.dense_ratio > self.size:
            d = np.zeros(self.size, dtype=np.float64)
            d[col[s:e]] = val[s:e]
            return DenseVector(d)
        v = SparseVector.__new__(SparseVector)
        v.n = self.size
        v.indices = col[s:e].astype(np.int32)
        v.values = val[s:e].copy()
        return v

    def __iter__(self):
        crow, col, val = self._np()
        for i in range(len(self)):
            yield self._vec(crow, col, val, i)

    def __getitem__(self, i):
        if isinstance(i, (int, np.integer)):
            n = len(self)
            i = int(i) + n if i < 0 else int(i)
            if not 0 <= i < n:
                raise IndexError(i)
            return self._vec(*self._np(), i)
        return self.take(i)

    def to_list(self) -> List:
        return list(self)

    # ---------------------------------------------------------------- block ops (stay on the device)
    def to(self, device) -> "SparseBlock":
        return SparseBlock(self.crow.to(device), self.col.to(device), self.val.to(device), self.size,
                           self.dense_ratio)

    def take(self, idx) -> "SparseBlock":
        """Row selection (slice, index list/tensor or boolean mask), gathered on the block's device."""
        dev = self.crow.device
        n = len(self)
        if isinstance(idx, slice):
            s, e, st = idx.indices(n)
            if st == 1:
                lo, hi = int(self.crow[s]), int(self.crow[max(s, e)])
                return SparseBlock(self.crow[s:max(s, e) + 1] - lo, self.col[lo:hi], self.val[lo:hi], self.size,
                                   self.dense_ratio)
            rows = torch.arange(s, e, st, device=dev)
        elif isinstance(idx, torch.Tensor):
            rows = idx.to(dev)
            if rows.dtype == torch.bool:
                rows = torch.nonzero(rows, as_tuple=False).reshape(-1)
        else:
            a = np.asarray(idx)
            if a.dtype == bool:
                a = np.nonzero(a)[0]
            rows = torch.as_tensor(a.astype(np.int64), device=dev)
        rows = rows.to(torch.int64)
        starts = self.crow[rows]
        lens = self.crow[rows + 1] - starts
        crow = torch.zeros(rows.shape[0] + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=crow[1:])
        total = int(crow[-1]) if rows.shape[0] else 0
        if total == 0:
            return SparseBlock(crow, self.col[:0], self.val[:0], self.size, self.dense_ratio)
        rid = torch.repeat_interleave(torch.arange(rows.shape[0], device=dev), lens)
        src = starts[rid] + (torch.arange(total, device=dev) - crow[:-1][rid])
        return SparseBlock(crow, self.col[src], self.val[src], self.size, self.dense_ratio)

    @staticmethod
    def concat(blocks: Sequence["SparseBlock"]) -> "SparseBlock":
        blocks = list(blocks)
        dev = blocks[0].device
        crows, off = [torch.zeros(1, dtype=torch.int64, device=dev)], 0
        for b in blocks:
            crows.append(b.crow[1:].to(dev) + off)
            off += b.nnz
        return SparseBlock(torch.cat(crows), torch.cat([b.col.to(dev) for b in blocks]),
                           torch.cat([b.val.to(dev) for b in blocks]), max(b.size for b in blocks),
                           blocks[0].dense_ratio)

    @staticmethod
    def from_vectors(vecs: Sequence, size: Optional[int] = None, device=None) -> "SparseBlock":
        counts, idx, vals, d = [], [], [], 0
        for v in vecs:
            if v is None:
                counts.append(0)
                continue
            if isinstance(v, SparseVector):
                idx.append(np.asarray(v.indices, np.int32))
                vals.append(np.asarray(v.values, np.float64))
                d = max(d, v.size())
            else:
                a = np.asarray(v.data, np.float64)
                nz = np.nonzero(a)[0]
                idx.append(nz.astype(np.int32))
                vals.append(a[nz])
                d = max(d, a.shape[0])
            counts.append(len(idx[-1]))
        crow = np.zeros(len(counts) + 1, np.int64)
        crow[1:] = np.cumsum(counts)
        col = np.concatenate(idx) if idx else np.zeros(0, np.int32)
        val = np.concatenate(vals) if vals else np.zeros(0, np.float64)
        return SparseBlock(torch.from_numpy(crow).to(device or "cpu"), torch.from_numpy(col).to(device or "cpu"),
                           torch.from_numpy(val).to(device or "cpu"), size if size is not None else d)

    def to_dense(self, dtype=torch.float64) -> torch.Tensor:
        n = len(self)
        out = torch.zeros((n, self.size), dtype=dtype, device=self.device)
        if self.nnz:
            rid = torch.repeat_interleave(torch.arange(n, device=self.device), self.crow[1:] - self.crow[:-1])
            out.index_put_((rid, self.col.to(torch.int64)), self.val.to(dtype), accumulate=True)
        return out

    def __repr__(self):
        return f"SparseBlock(n={len(self)}, size={self.size}, nnz={self.nnz}, device={self.device})"
