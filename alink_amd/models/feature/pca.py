"""PCA (reference ``A/operator/batch/feature/PcaTrainBatchOp.java``, ``A/operator/common/feature/pca/*``).

Training = one pass of sufficient statistics (count, sum, sum of squares and the Gram matrix ``X^T X`` — a
single rocBLAS SYRK/GEMM on the device — all-reduced across ranks), then the covariance / correlation
eigen-decomposition on the host (``d x d``).  Constant columns are dropped (``idxNonEqual``), as the reference.
Model: meta ``{featureCols, vectorCol, calculationType}`` + one ``PcaModelData`` JSON row.
Prediction: ``((x - mean) / std) . coef_k`` with ``SIMPLE`` (no centring), ``SUBMEAN`` or ``NORMALIZATION``
(scores divided by their standard deviation), the CORR type dividing by the column std.

Eigenvector signs: each component is oriented so that its entry of largest magnitude is positive.
"""
from __future__ import annotations

import json
from typing import List, Optional

import numpy as np
import torch

from ...ops.gemm import tn_matmul
from ...common.javafmt import gson_dumps
from ...common.linalg import DenseVector, VectorUtil
from ...common.mapper import ModelMapper, OutputColsHelper, find_col_index
from ...common.model.converter import SimpleModelDataConverter
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import Types
from ...parallel import comm
from ..common.features import extract_features, global_vector_size

__all__ = ["train_pca", "PcaModelMapper"]


def _pget(p: Params, name, default=None):
    try:
        if p.contains(name):
            v = p.get(name)
            return default if v is None else v
    except KeyError:
        pass
    return default


def _ename(v, default):
    return default if v is None else str(getattr(v, "name", v)).upper()


class _PcaModelData:
    __gson_fields__ = ("featureColNames", "vectorColName", "pcaType", "nameX", "means", "stddevs", "p", "lambda",
                       "coef", "cov", "idxNonEqual", "nx")
    __gson_skip_nulls__ = True

    def __init__(self, **kw):
        for f in self.__gson_fields__:
            setattr(self, f, kw.get(f))


def train_pca(mt: MTable, params: Params, env) -> List[tuple]:
    dev = env.device
    k = int(params.get("k"))
    ctype = _ename(_pget(params, "calculationType"), "CORR")
    cols = _pget(params, "selectedCols")
    vcol = _pget(params, "vectorCol")
    fm = extract_features(mt, list(cols) if cols and not vcol else None, vcol, dev)
    d = global_vector_size(fm)
    if fm.is_sparse:
        fm.set_ncols(d)
    X = fm.to_dense().to(torch.float64)
    if X.shape[1] < d:
        X = torch.nn.functional.pad(X, (0, d - X.shape[1]))
    n = torch.tensor([float(X.shape[0])], dtype=torch.float64, device=X.device)
    buf = torch.cat([n, X.sum(0), (X * X).sum(0), tn_matmul(X, X).reshape(-1)])
    comm.all_reduce(buf, "sum")
    cnt = float(buf[0])
    s = buf[1:1 + d].cpu().numpy()
    s2 = buf[1 + d:1 + 2 * d].cpu().numpy()
    G = buf[1 + 2 * d:].reshape(d, d).cpu().numpy()
    nonconst = [i for i in range(d) if abs(s2[i] - s[i] * s[i] / cnt) > 1e-10]
    idx = np.asarray(nonconst, dtype=np.int64)
    s, s2, G = s[idx], s2[idx], G[np.ix_(idx, idx)]
    cov = (G - np.outer(s, s) / cnt) / (cnt - 1)
    std = np.sqrt(np.maximum(0.0, (s2 - s * s / cnt) / (cnt - 1)))
    if ctype == "CORR":
        M = cov / np.outer(std, std)
        np.fill_diagonal(M, 1.0)
    else:
        M = cov.copy()
        if ctype == "COVAR_POP":
            if cnt <= 1:
                raise RuntimeError("record num is less than 2!")
            M = M * (cnt / (cnt - 1))
    if k >= M.shape[0]:
        raise RuntimeError(f"k is larger than vector size. k: {k} vectorSize: {M.shape[0]}")
    w, V = np.linalg.eigh(M)
    order = np.argsort(-w)[:k]
    lam, vec = w[order], V[:, order]
    for j in range(vec.shape[1]):
        if vec[np.argmax(np.abs(vec[:, j])), j] < 0:
            vec[:, j] = -vec[:, j]
    model = _PcaModelData(featureColNames=list(cols) if cols and not vcol else None, vectorColName=vcol,
                          pcaType=ctype, means=(s / cnt).tolist(), stddevs=std.tolist(), p=k,
                          **{"lambda": lam.tolist()}, coef=vec.T.tolist(), cov=cov.tolist(),
                          idxNonEqual=[int(i) for i in idx], nx=d)
    meta = Params().set("featureCols", list(cols) if cols and not vcol else None).set("vectorCol", vcol) \
        .set("calculationType", ctype)
    return SimpleModelDataConverter.rows_from(meta, [gson_dumps(model, java_map_order=False)])


class PcaModelMapper(ModelMapper):
    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        p = self.params
        self.helper = OutputColsHelper(dataSchema, [p.get("predictionCol")], [Types.STRING], _pget(p, "reservedCols"))

    def loadModel(self, rows):
        meta, data = SimpleModelDataConverter.split_rows(rows)
        m = json.loads(data[0])
        self.m = m
        self.vcol = _pget(self.params, "vectorCol") or m.get("vectorColName")
        self.fcols = m.get("featureColNames")
        nx = int(m["nx"])
        nne = len(m["idxNonEqual"])
        self.idx = np.asarray(m["idxNonEqual"], dtype=np.int64)
        self.coef = np.asarray(m["coef"], dtype=np.float64)
        mean = np.zeros(nne)
        std = np.ones(nne)
        score_std = np.ones(self.coef.shape[0])
        if str(m["pcaType"]).upper() == "CORR":
            std = np.asarray(m["stddevs"], dtype=np.float64)
        tt = _ename(_pget(self.params, "transformType"), "SIMPLE")
        if tt in ("SUBMEAN", "NORMALIZATION"):
            mean = np.asarray(m["means"], dtype=np.float64)
        if tt == "NORMALIZATION":
            cov = np.asarray(m["cov"], dtype=np.float64)
            score_std = np.sqrt(np.einsum("ij,ik,jk->i", self.coef, self.coef, cov))
        self.mean, self.std, self.score_std = mean, std, score_std
        self.nx = nx

    def _map_columns(self, mt):
        from ..linear.model import _dev
        dev = _dev(mt)
        fm = extract_features(mt, self.fcols if not self.vcol else None, self.vcol, dev)
        if fm.is_sparse:
            fm.set_ncols(self.nx)
        if dev.type == "cuda" and mt.num_rows:
            P = self._project_device(fm.to_dense().double())
        else:
            P = self._project(fm.to_dense().double().numpy())
        from ... import _native
        r = _native.java_double_rows_packed(P, " ") if P.size else None
        if r is None:
            return [Column.from_values([VectorUtil.toString(DenseVector(r)) for r in P], Types.STRING)]
        from ...common.strings import StringBlock
        return [Column(StringBlock(torch.from_numpy(np.ascontiguousarray(r[0])), torch.from_numpy(r[1])))]

    def _project_device(self, X: torch.Tensor) -> np.ndarray:
        """``_project`` in float64 on the input's device (the same operations; matmul rounding may differ)."""
        dev = X.device
        if X.shape[1] < self.nx:
            X = torch.nn.functional.pad(X, (0, self.nx - X.shape[1]))
        t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=dev)  # noqa: E731
        Z = X[:, torch.as_tensor(self.idx, dtype=torch.int64, device=dev)]
        ok = np.abs(self.std) > 1e-12
        std = t(np.where(ok, self.std, 1.0))
        Zs = (Z - t(self.mean)[None, :]) / std[None, :]
        Z = torch.where(torch.as_tensor(ok, device=dev)[None, :], Zs, Z if len(self.idx) == self.nx else torch.zeros_like(Z))
        return (Z @ t(self.coef).T / t(self.score_std)[None, :]).cpu().numpy()

    def _project(self, X: np.ndarray) -> np.ndarray:
        if X.shape[1] < self.nx:
            X = np.pad(X, ((0, 0), (0, self.nx - X.shape[1])))
        Z = X[:, self.idx]
        ok = np.abs(self.std) > 1e-12
        Z = np.where(ok[None, :], (Z - self.mean[None, :]) / np.where(ok, self.std, 1.0)[None, :],
                     np.where(len(self.idx) != self.nx, 0.0, Z))
        return Z @ self.coef.T / self.score_std[None, :]
