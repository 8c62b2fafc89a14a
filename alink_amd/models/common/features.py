"""Device-resident feature matrices shared by the learning algorithms.

The reference moves training samples around as ``Tuple3<weight, label, Vector>`` records and evaluates
losses/gradients one ``Vector`` at a time (``A/operator/common/optim/objfunc/OptimObjFunc.java:126-231``,
``A/common/linalg/MatVecOp.java``).  Here a partition's samples are ONE matrix on the rank's device:

* ``dense``  — ``[n, d]`` float64 tensor (row-major; GEMV/GEMM via rocBLAS on MI355X);
* ``sparse`` — CSR (``crow [n+1]``, ``col [nnz]``, ``val [nnz]``) with the same operations implemented as
  gather/segment-sum (``index_add_``) kernels.

``FeatureMatrix`` offers exactly the products the optimizers need: ``X @ v`` (margins), ``X @ V``
(several directions at once — the line-search trick of ``UnaryLossObjFunc.calcSearchValues``),
``X^T g`` (gradients) and ``X^T diag(h) X`` (Newton Hessians).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...ops.gemm import tn_matmul
from ...common.linalg import DenseVector, SparseBlock, SparseVector, VectorUtil
from ...common.table import MTable
from ...common.types import Types, is_numeric
from ...parallel import comm

__all__ = ["FeatureMatrix", "extract_features", "column_stats", "global_vector_size"]


class FeatureMatrix:
    """Dense or CSR sample matrix (one partition)."""

    def __init__(self, dense: Optional[torch.Tensor] = None, crow=None, col=None, val=None, ncols: int = 0):
        self.dense = dense
        self.crow, self.col, self.val = crow, col, val
        self._ncols = int(dense.shape[1]) if dense is not None else int(ncols)
        self._row_ids = None

    # -- info --
    @property
    def is_sparse(self) -> bool:
        return self.dense is None

    @property
    def device(self):
        return self.dense.device if self.dense is not None else self.val.device

    @property
    def nrows(self) -> int:
        return int(self.dense.shape[0]) if self.dense is not None else int(self.crow.shape[0]) - 1

    @property
    def ncols(self) -> int:
        return self._ncols

    def __len__(self):
        return self.nrows

    def row_ids(self) -> torch.Tensor:
        if self._row_ids is None:
            counts = self.crow[1:] - self.crow[:-1]
            # output_size: the entry count is known on the host, so no device->host sync for the result size
            self._row_ids = torch.repeat_interleave(torch.arange(self.nrows, device=self.val.device), counts,
                                                    output_size=int(self.col.numel()))
        return self._row_ids

    def set_ncols(self, d: int) -> "FeatureMatrix":
        if self.dense is not None:
            if d > self._ncols:
                self.dense = torch.nn.functional.pad(self.dense, (0, d - self._ncols))
            self._ncols = int(self.dense.shape[1])
        else:
            self._ncols = max(self._ncols, int(d))
        return self

    def __getitem__(self, sl: slice) -> "FeatureMatrix":
        lo, hi, _ = sl.indices(self.nrows)
        if self.dense is not None:
            return FeatureMatrix(self.dense[lo:hi])
        a, b = int(self.crow[lo]), int(self.crow[hi])
        return FeatureMatrix(crow=self.crow[lo:hi + 1] - a, col=self.col[a:b], val=self.val[a:b], ncols=self._ncols)

    def take(self, idx: torch.Tensor) -> "FeatureMatrix":
        if self.dense is not None:
            return FeatureMatrix(self.dense[idx])
        idx = idx.to(self.crow.device)
        starts, ends = self.crow[idx], self.crow[idx + 1]
        counts = ends - starts
        crow = torch.zeros(idx.shape[0] + 1, dtype=torch.int64, device=self.crow.device)
        crow[1:] = torch.cumsum(counts, 0)
        if int(crow[-1]) == 0:
            return FeatureMatrix(crow=crow, col=self.col[:0], val=self.val[:0], ncols=self._ncols)
        rep = torch.repeat_interleave(starts - crow[:-1], counts)
        pos = torch.arange(int(crow[-1]), device=self.crow.device) + rep
        return FeatureMatrix(crow=crow, col=self.col[pos], val=self.val[pos], ncols=self._ncols)

    def to(self, device) -> "FeatureMatrix":
        if self.dense is not None:
            return FeatureMatrix(self.dense.to(device))
        return FeatureMatrix(crow=self.crow.to(device), col=self.col.to(device), val=self.val.to(device),
                             ncols=self._ncols)

    # -- products --
    def mv(self, v: torch.Tensor) -> torch.Tensor:
        """X @ v  -> [n]  (v may be longer than ncols: extra entries ignored)."""
        if self.dense is not None:
            return self.dense @ v[: self._ncols]
        if self.val.numel() == 0:
            return torch.zeros(self.nrows, dtype=v.dtype, device=v.device)
        if v.is_cuda and v.dtype == torch.float64 and self.val.dtype == torch.float64:
            from ...ops.feature import csr_mv         # HIP: G lanes per row, fixed-order sum, no atomics
            return csr_mv(self.crow, self.col, self.val, v)
        prod = self.val * v[self.col]
        out = torch.zeros(self.nrows, dtype=v.dtype, device=v.device)
        return out.index_add_(0, self.row_ids(), prod)

    def mm(self, V: torch.Tensor) -> torch.Tensor:
        """X @ V for V [d, k] -> [n, k]."""
        if self.dense is not None:
            return self.dense @ V[: self._ncols]
        out = torch.zeros((self.nrows, V.shape[1]), dtype=V.dtype, device=V.device)
        if self.val.numel() == 0:
            return out
        return out.index_add_(0, self.row_ids(), self.val[:, None] * V[self.col])

    def rmv(self, g: torch.Tensor, d: Optional[int] = None) -> torch.Tensor:
        """X^T g -> [d]."""
        d = self._ncols if d is None else d
        if self.dense is not None:
            out = tn_matmul(self.dense, g)
            return out if d == self._ncols else torch.nn.functional.pad(out, (0, d - self._ncols))
        out = torch.zeros(d, dtype=g.dtype, device=g.device)
        if self.val.numel() == 0:
            return out
        return out.index_add_(0, self.col, self.val * g[self.row_ids()])

    def rmm(self, G: torch.Tensor, d: Optional[int] = None) -> torch.Tensor:
        """X^T G for G [n, k] -> [d, k]."""
        d = self._ncols if d is None else d
        if self.dense is not None:
            out = tn_matmul(self.dense, G)
            return out if d == self._ncols else torch.nn.functional.pad(out, (0, 0, 0, d - self._ncols))
        out = torch.zeros((d, G.shape[1]), dtype=G.dtype, device=G.device)
        if self.val.numel() == 0:
            return out
        return out.index_add_(0, self.col, self.val[:, None] * G[self.row_ids()])

    def gram(self, h: torch.Tensor, d: Optional[int] = None) -> torch.Tensor:
        """X^T diag(h) X -> [d, d]."""
        d = self._ncols if d is None else d
        if self.dense is not None:
            Xd = self.dense
            out = tn_matmul(Xd, Xd * h[:, None])
            return out if d == self._ncols else torch.nn.functional.pad(out, (0, d - self._ncols, 0, d - self._ncols))
        D = self.to_dense(d)
        return tn_matmul(D, D * h[:, None])

    # -- transforms --
    def to_dense(self, d: Optional[int] = None) -> torch.Tensor:
        d = self._ncols if d is None else d
        if self.dense is not None:
            return self.dense if d == self._ncols else torch.nn.functional.pad(self.dense, (0, d - self._ncols))
        out = torch.zeros((self.nrows, d), dtype=self.val.dtype, device=self.val.device)
        if self.val.numel():
            out.index_put_((self.row_ids(), self.col), self.val, accumulate=True)
        return out

    def prefix_one(self) -> "FeatureMatrix":
        """Prepend a constant-1 column (``Vector.prefix(1.0)``: intercept at index 0)."""
        if self.dense is not None:
            ones = torch.ones((self.nrows, 1), dtype=self.dense.dtype, device=self.dense.device)
            return FeatureMatrix(torch.cat([ones, self.dense], 1))
        # every row gains one leading entry: entry i of row r moves to i + r + 1, the new entry sits at the row's
        # new start — pure index arithmetic, sizes known on the host (no device->host sync, no boolean mask)
        n = self.nrows
        m = int(self.col.numel())
        counts = self.crow[1:] - self.crow[:-1] + 1
        crow = torch.zeros(n + 1, dtype=torch.int64, device=self.crow.device)
        crow[1:] = torch.cumsum(counts, 0)
        nnz = m + n
        col = torch.empty(nnz, dtype=self.col.dtype, device=self.col.device)
        val = torch.empty(nnz, dtype=self.val.dtype, device=self.val.device)
        first = crow[:-1]
        col[first] = 0
        val[first] = 1.0
        if m:
            pos = torch.arange(m, device=self.col.device) + self.row_ids() + 1
            col[pos] = self.col + 1
            val[pos] = self.val
        return FeatureMatrix(crow=crow, col=col, val=val, ncols=self._ncols + 1)

    def standardize(self, mean: torch.Tensor, std: torch.Tensor, center: bool) -> "FeatureMatrix":
        """(x - mean)/std (dense, center) or x/std; sparse data is only ever scaled (mean is zero)."""
        if self.dense is not None:
            X = self.dense
            if center:
                X = X - mean[None, : X.shape[1]]
            return FeatureMatrix(X / std[None, : X.shape[1]])
        return FeatureMatrix(crow=self.crow, col=self.col, val=(self.val - (mean[self.col] if center else 0.0))
                             / std[self.col], ncols=self._ncols)


def _vectors_to_matrix(vals: Sequence, dtype, device, size: Optional[int]) -> FeatureMatrix:
    vecs = [VectorUtil.getVector(v) if v is not None else None for v in vals]
    if any(isinstance(v, SparseVector) for v in vecs):
        idx, vv, counts = [], [], []
        d = 0
        for v in vecs:
            if v is None:
                counts.append(0)
                continue
            if isinstance(v, SparseVector):
                idx.append(np.asarray(v.indices, dtype=np.int64))
                vv.append(np.asarray(v.values, dtype=np.float64))
                counts.append(len(v.indices))
                d = max(d, v.size() if v.size() >= 0 else (int(v.indices[-1]) + 1 if len(v.indices) else 0))
            else:
                a = np.asarray(v.data, dtype=np.float64)
                nz = np.nonzero(a)[0]
                idx.append(nz.astype(np.int64))
                vv.append(a[nz])
                counts.append(len(nz))
                d = max(d, a.shape[0])
        crow = np.zeros(len(vecs) + 1, dtype=np.int64)
        crow[1:] = np.cumsum(counts)
        col = np.concatenate(idx) if idx else np.zeros(0, dtype=np.int64)
        val = np.concatenate(vv) if vv else np.zeros(0, dtype=np.float64)
        if size is not None:
            d = max(d, size)
        return FeatureMatrix(crow=torch.from_numpy(crow).to(device), col=torch.from_numpy(col).to(device),
                             val=torch.from_numpy(val).to(device=device, dtype=dtype), ncols=d)
    d = max((v.size() for v in vecs if v is not None), default=0)
    if size is not None:
        d = max(d, size)
    out = np.zeros((len(vecs), d), dtype=np.float64)
    for i, v in enumerate(vecs):
        if v is not None:
            out[i, : v.size()] = v.data
    return FeatureMatrix(torch.from_numpy(out).to(device=device, dtype=dtype))


def extract_features(mt: MTable, feature_cols: Optional[Sequence[str]], vector_col: Optional[str], device,
                     dtype=torch.float64, vector_size: Optional[int] = None) -> FeatureMatrix:
    """This rank's samples as a FeatureMatrix: numeric ``featureCols`` stacked, or a vector column
    (dense tensor block, dense/sparse vectors or vector strings)."""
    if vector_col:
        c = mt.col(vector_col)
        v = c.values
        if isinstance(v, SparseBlock):       # columnar CSR (GPU feature path): no host round trip
            d = max(v.size, vector_size or 0)
            return FeatureMatrix(crow=v.crow.to(device), col=v.col.to(device=device, dtype=torch.int64),
                                 val=v.val.to(device=device, dtype=dtype), ncols=d)
        if isinstance(v, torch.Tensor) and v.dim() == 2:
            fm = FeatureMatrix(v.to(device=device, dtype=dtype))
            return fm.set_ncols(vector_size) if vector_size else fm
        return _vectors_to_matrix(list(v) if not isinstance(v, torch.Tensor) else v.tolist(), dtype, device,
                                  vector_size)
    cols = []
    for name in feature_cols or []:
        c = mt.col(name)
        if isinstance(c.values, torch.Tensor):
            t = c.values.to(device=device, dtype=dtype)
            if c.nulls is not None:
                t = t.masked_fill(c.nulls.to(device), 0.0)
        else:
            t = torch.tensor([0.0 if x is None else float(x) for x in c.values], dtype=dtype, device=device)
        cols.append(t.reshape(-1))
    if not cols:
        return FeatureMatrix(torch.zeros((mt.num_rows, 0), dtype=dtype, device=device))
    return FeatureMatrix(torch.stack(cols, 1))


def global_vector_size(fm: FeatureMatrix) -> int:
    return max(comm.all_gather_object(int(fm.ncols)))


def column_stats(fm: FeatureMatrix, d: Optional[int] = None, weights: Optional[torch.Tensor] = None):
    """Global (all ranks) per-column count / mean / sample std / min / max / maxAbs / nnz.

    Mirrors the ``DenseVectorSummarizer``/``SparseVectorSummarizer`` moments the reference computes in
    ``StatisticsHelper.summary`` (``A/operator/common/statistics/basicstatistic/*``); for sparse inputs min/max
    include the implicit zeros of rows that do not store a column.
    """
    d = fm.ncols if d is None else d
    dev = fm.device
    n_local = fm.nrows
    l1_local = None
    if fm.is_sparse:
        s = torch.zeros(d, dtype=torch.float64, device=dev).index_add_(0, fm.col, fm.val.double())
        s2 = torch.zeros(d, dtype=torch.float64, device=dev).index_add_(0, fm.col, fm.val.double() ** 2)
        nnz = torch.zeros(d, dtype=torch.float64, device=dev).index_add_(
            0, fm.col, (fm.val != 0).double())
        l1_local = torch.zeros(d, dtype=torch.float64, device=dev).index_add_(0, fm.col, fm.val.double().abs())
        stored = torch.zeros(d, dtype=torch.float64, device=dev).index_add_(
            0, fm.col, torch.ones_like(fm.val, dtype=torch.float64))
        big = torch.full((d,), float("inf"), dtype=torch.float64, device=dev)
        mn = big.clone().scatter_reduce_(0, fm.col, fm.val.double(), "amin")
        mx = (-big).scatter_reduce_(0, fm.col, fm.val.double(), "amax")
        has_zero = stored < n_local
        mn = torch.where(has_zero, torch.minimum(mn, torch.zeros_like(mn)), mn)
        mx = torch.where(has_zero, torch.maximum(mx, torch.zeros_like(mx)), mx)
    else:
        from ...ops import stats as sops
        X = fm.dense
        if X.shape[1] < d:
            X = torch.nn.functional.pad(X, (0, d - X.shape[1]))
        # one pass over the native-dtype matrix (HIP K23 on the GPU), fp64 moments
        cs = sops.colstats(X) if X.shape[1] else sops.colstats_torch(X)
        s, s2, nnz, mn, mx = cs["sum"], cs["sum2"], cs["nnz"], cs["min"], cs["max"]
        l1_local = cs["l1"]
    cnt = torch.tensor([float(n_local)], dtype=torch.float64, device=dev)
    buf = torch.cat([cnt, s, s2, nnz, l1_local])
    comm.all_reduce(buf, "sum")
    comm.all_reduce(mn, "min")
    comm.all_reduce(mx, "max")
    n = float(buf[0].item())
    s, s2, nnz, l1 = buf[1:1 + d], buf[1 + d:1 + 2 * d], buf[1 + 2 * d:1 + 3 * d], buf[1 + 3 * d:]
    mean = s / max(n, 1.0)
    var = (s2 - s * mean) / max(n - 1.0, 1.0) if n > 1 else torch.zeros_like(s)
    std = torch.sqrt(torch.clamp(var, min=0.0))
    return {"count": n, "sum": s, "sum2": s2, "mean": mean, "std": std, "min": mn, "max": mx,
            "maxAbs": torch.maximum(mn.abs(), mx.abs()), "nnz": nnz, "variance": var, "l1": l1}
