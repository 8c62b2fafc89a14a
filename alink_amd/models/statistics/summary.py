"""Column / vector statistics: summarizers, correlation, chi-square tests.

Reference: ``A/operator/common/statistics/basicstatistic/{TableSummary,TableSummarizer,DenseVectorSummary,
SparseVectorSummary,SummaryDataConverter,VectorSummaryDataConverter,CorrelationResult,SpearmanCorrelation}.java``,
``A/operator/common/statistics/{StatisticsHelper,ChiSquareTest,ChiSquareTestResult}.java``.

Moments are column reductions on the device (one fused pass per table) merged with ONE all-reduce
(the reference reduces summarizer objects to a single task); Pearson correlation is a Gram-matrix GEMM
(``X^T X``, the reference's ``DenseVectorSummarizer`` outer product), Spearman ranks each column
(global rank via all-gather of the column, then the same GEMM).
"""
from __future__ import annotations

import json
import math
from typing import Any, List, Optional, Sequence

import numpy as np
import torch

from ...ops.gemm import tn_matmul
from ...common.javafmt import gson_dumps
from ...common.linalg import DenseMatrix, DenseVector, SparseVector, VectorUtil
from ...common.model.converter import SimpleModelDataConverter
from ...common.params import Params
from ...common.table import MTable
from ...common.types import Types, is_numeric
from ...parallel import comm
from ..common.features import column_stats, extract_features

__all__ = ["TableSummary", "VectorSummary", "table_summary", "vector_summary", "SummaryDataConverter",
           "VectorSummaryDataConverter", "CorrelationResult", "correlation", "vector_correlation",
           "chi_square_test", "ChiSquareTestResult"]


def _fmt_table(names, rows):
    from ...operator.base import format_rows
    return format_rows(names, rows)


class _Count(int):
    """The row count: an int that can also be called, as the reference's ``count()`` method."""

    def __call__(self) -> int:
        return int(self)


class TableSummary:
    """count / sum / squareSum / min / max / normL1 / numMissingValue of the selected columns (statistics for
    the numeric ones, counts for all) — ``TableSummary.java``; accessors take a column name."""

    def __init__(self, names, num_idx, count, s, s2, mn, mx, l1, nmv):
        self.colNames = list(names)
        self.numericalColIndices = list(num_idx)
        self.count = _Count(count)
        self._sum, self._s2, self._mn, self._mx, self._l1, self._nmv = s, s2, mn, mx, l1, nmv

    def _idx(self, col):
        i = self.colNames.index(col)
        return self.numericalColIndices.index(i) if i in self.numericalColIndices else -1

    def _num(self, arr, col):
        j = self._idx(col)
        return float(arr[j]) if j >= 0 else float("nan")

    def getColNames(self):
        return list(self.colNames)

    def numMissingValue(self, col):
        return float(self._nmv[self.colNames.index(col)])

    def numValidValue(self, col):
        return self.count - self.numMissingValue(col)

    def sum(self, col):
        return self._num(self._sum, col)

    def mean(self, col):
        if self._idx(col) < 0:
            return float("nan")
        n = self.numValidValue(col)
        return 0.0 if n == 0 else self.sum(col) / n

    def variance(self, col):
        j = self._idx(col)
        if j < 0:
            return float("nan")
        n = self.numValidValue(col)
        if n in (0, 1):
            return 0.0
        s, s2 = float(self._sum[j]), float(self._s2[j])
        return max(0.0, (s2 - s * s / n) / (n - 1))

    def standardDeviation(self, col):
        return math.sqrt(self.variance(col))

    def min(self, col):
        return self._num(self._mn, col)

    def max(self, col):
        return self._num(self._mx, col)

    def normL1(self, col):
        return self._num(self._l1, col)

    def normL2(self, col):
        j = self._idx(col)
        return math.sqrt(float(self._s2[j])) if j >= 0 else float("nan")

    def __str__(self):
        head = ["colName", "count", "numMissingValue", "numValidValue", "sum", "mean", "variance",
                "standardDeviation", "min", "max", "normL1", "normL2"]
        rows = [[c, self.count, self.numMissingValue(c), self.numValidValue(c), self.sum(c), self.mean(c),
                 self.variance(c), self.standardDeviation(c), self.min(c), self.max(c), self.normL1(c),
                 self.normL2(c)] for c in self.colNames]
        return _fmt_table(head, rows)


def _make_summary(names, num_idx, count, s, s2, mn, mx, l1, nmv) -> TableSummary:
    return TableSummary(names, num_idx, count, s, s2, mn, mx, l1, nmv)


def table_summary(mt: MTable, cols: Optional[Sequence[str]] = None, device=None) -> TableSummary:
    """Distributed column summary (``StatisticsHelper.summary`` / ``TableSummarizer``)."""
    cols = list(cols) if cols else list(mt.schema.names)
    num_idx = [i for i, c in enumerate(cols) if is_numeric(mt.col_type(c)) or mt.col_type(c) == Types.BOOLEAN]
    dev = device or torch.device("cpu")
    nnum = len(num_idx)
    n = mt.num_rows
    s = torch.zeros(nnum, dtype=torch.float64, device=dev)
    s2, l1 = torch.zeros_like(s), torch.zeros_like(s)
    mn = torch.full((nnum,), float("inf"), dtype=torch.float64, device=dev)
    mx = torch.full((nnum,), float("-inf"), dtype=torch.float64, device=dev)
    nmv = torch.zeros(len(cols), dtype=torch.float64, device=dev)
    for j, c in enumerate(cols):
        col = mt.col(c)
        if isinstance(col.values, torch.Tensor) and col.values.dim() == 1:
            v = col.values.to(device=dev, dtype=torch.float64)
            valid = ~col.nulls.to(dev) if col.nulls is not None else torch.ones(n, dtype=torch.bool, device=dev)
            valid = valid & ~torch.isnan(v)
        else:
            lst = col.to_list()
            valid = torch.tensor([x is not None and not (isinstance(x, float) and x != x) for x in lst],
                                 dtype=torch.bool, device=dev)
            v = None
            if j in num_idx:
                v = torch.tensor([float(x) if x is not None else 0.0 for x in lst], dtype=torch.float64, device=dev)
        nmv[j] = float(n) - valid.sum().double()
        if j in num_idx:
            k = num_idx.index(j)
            vv = v[valid]
            s[k] = vv.sum()
            s2[k] = (vv * vv).sum()
            l1[k] = vv.abs().sum()
            if vv.numel():
                mn[k] = vv.min()
                mx[k] = vv.max()
    buf = torch.cat([torch.tensor([float(n)], dtype=torch.float64, device=dev), s, s2, l1, nmv])
    comm.all_reduce(buf, "sum")
    comm.all_reduce(mn, "min")
    comm.all_reduce(mx, "max")
    b = buf.cpu().numpy()
    count = int(b[0])
    s_, s2_, l1_, nmv_ = b[1:1 + nnum], b[1 + nnum:1 + 2 * nnum], b[1 + 2 * nnum:1 + 3 * nnum], b[1 + 3 * nnum:]
    mnn, mxx = mn.cpu().numpy(), mx.cpu().numpy()
    mnn = np.where(np.isinf(mnn), np.nan, mnn)
    mxx = np.where(np.isinf(mxx), np.nan, mxx)
    return _make_summary(cols, num_idx, count, s_, s2_, mnn, mxx, l1_, nmv_)


class SummaryDataConverter(SimpleModelDataConverter):
    """Rows of a SummarizerBatchOp output (``SummaryDataConverter.java``)."""

    def serializeModel(self, t: TableSummary):
        data = [gson_dumps(list(t.colNames)), VectorUtil.toString(DenseVector(np.asarray(t._sum))),
                VectorUtil.toString(DenseVector(np.asarray(t._s2))), VectorUtil.toString(DenseVector(np.asarray(t._mn))),
                VectorUtil.toString(DenseVector(np.asarray(t._mx))), VectorUtil.toString(DenseVector(np.asarray(t._l1))),
                VectorUtil.toString(DenseVector(np.asarray(t._nmv))), gson_dumps(list(t.numericalColIndices)),
                str(int(t.count))]
        return Params(), data

    def deserializeModel(self, meta, data):
        it = iter(data)
        names = json.loads(next(it))

        def dv(s):
            return VectorUtil.parseDense(s).data if s else np.zeros(0)
        s, s2, mn, mx, l1, nmv = (dv(next(it)) for _ in range(6))
        idx = json.loads(next(it))
        count = int(next(it))
        return _make_summary(names, idx, count, s, s2, mn, mx, l1, nmv)


class VectorSummary:
    """Vector-column summary (``DenseVectorSummary`` / ``SparseVectorSummary``)."""

    def __init__(self, count, sum_, sum2, mn, mx, l1, nnz, sparse: bool):
        self.count, self._sum, self._s2, self._mn, self._mx, self._l1, self._nnz = \
            _Count(count), sum_, sum2, mn, mx, l1, nnz
        self.sparse = sparse

    def vectorSize(self):
        return len(self._sum)

    def _vec(self, a):
        a = np.asarray(a, dtype=np.float64)
        if self.sparse:
            nz = np.nonzero(a)[0]
            return SparseVector(len(a), nz, a[nz])
        return DenseVector(a.copy())

    @property
    def colNum(self) -> int:
        return len(self._sum)

    def _at(self, arr, idx):
        # every statistic takes an optional column index, as the reference's max(int) / max() pair
        return self._vec(arr) if idx is None else float(np.asarray(arr, dtype=np.float64)[idx])

    def sum(self, idx=None):
        return self._at(self._sum, idx)

    def mean(self, idx=None):
        return self._at(self._sum / max(self.count, 1), idx)

    def _variance(self):
        n = self.count
        if n <= 1:
            return np.zeros_like(np.asarray(self._sum, dtype=np.float64))
        return np.maximum(0.0, (self._s2 - self._sum * self._sum / n) / (n - 1))

    def variance(self, idx=None):
        return self._at(self._variance(), idx)

    def standardDeviation(self, idx=None):
        return self._at(np.sqrt(self._variance()), idx)

    def min(self, idx=None):
        return self._at(self._mn, idx)

    def max(self, idx=None):
        return self._at(self._mx, idx)

    def normL1(self, idx=None):
        return self._at(self._l1, idx)

    def normL2(self, idx=None):
        return self._at(np.sqrt(self._s2), idx)

    def numNonZero(self, idx=None):
        # a DenseVector for sparse summaries too (SparseVectorSummary.numNonZero)
        a = np.asarray(self._nnz, dtype=np.float64)
        return DenseVector(a.copy()) if idx is None else float(a[idx])

    def __str__(self):
        head = ["id", "count", "sum", "mean", "variance", "standardDeviation", "min", "max", "normL1", "normL2"]
        var = np.maximum(0.0, (self._s2 - self._sum ** 2 / max(self.count, 1)) / max(self.count - 1, 1))
        rows = [[i, self.count, self._sum[i], self._sum[i] / max(self.count, 1), var[i], math.sqrt(var[i]),
                 self._mn[i], self._mx[i], self._l1[i], math.sqrt(self._s2[i])] for i in range(len(self._sum))]
        return _fmt_table(head, rows)


def vector_summary(mt: MTable, vector_col: str, device=None) -> VectorSummary:
    fm = extract_features(mt, None, vector_col, device or torch.device("cpu"))
    d = max(comm.all_gather_object(int(fm.ncols)))
    st = column_stats(fm, d)          # one pass (HIP K23 for dense device blocks), one fused all-reduce
    l1 = st["l1"]
    sparse = any(comm.all_gather_object(bool(fm.is_sparse)))
    mn, mx = st["min"].cpu().numpy(), st["max"].cpu().numpy()
    return VectorSummary(st["count"], st["sum"].cpu().numpy(), st["sum2"].cpu().numpy(),
                         np.where(np.isinf(mn), np.nan, mn), np.where(np.isinf(mx), np.nan, mx),
                         l1.cpu().numpy(), st["nnz"].cpu().numpy(), sparse)


class VectorSummaryDataConverter(SimpleModelDataConverter):
    def serializeModel(self, v: VectorSummary):
        meta = Params().set("count", int(v.count)).set("sparse", bool(v.sparse))
        data = [VectorUtil.toString(DenseVector(np.asarray(a, dtype=np.float64)))
                for a in (v._sum, v._s2, v._mn, v._mx, v._l1, v._nnz)]
        return meta, data

    def deserializeModel(self, meta, data):
        arrs = [VectorUtil.parseDense(s).data for s in data]
        return VectorSummary(meta.get("count"), *arrs, sparse=bool(meta.get("sparse")))


class CorrelationResult:
    def __init__(self, matrix: np.ndarray, names: Optional[List[str]] = None):
        self.correlation = DenseMatrix(np.asarray(matrix, dtype=np.float64))
        self.colNames = names

    def getCorrelationMatrix(self):
        return self.correlation

    def getCorrelation(self):
        return self.correlation.toArray() if hasattr(self.correlation, "toArray") else \
            np.asarray(self.correlation.data).reshape(self.correlation.m, self.correlation.n, order="F")

    def getColNames(self):
        return self.colNames

    def __str__(self):
        arr = self.getCorrelation()
        names = self.colNames or [str(i) for i in range(arr.shape[0])]
        return _fmt_table(["colName"] + list(names), [[names[i]] + list(arr[i]) for i in range(arr.shape[0])])


def _is_spearman(method) -> bool:
    """The reference's enum spells it ``SPEAMAN`` (``HasMethod`` of CorrelationBatchOp); accept both spellings."""
    m = str(getattr(method, "name", method)).upper()
    return m in ("SPEAMAN", "SPEARMAN")


def _rank_global(v: torch.Tensor) -> torch.Tensor:
    """Average ranks (1-based, ties averaged) of the GLOBAL column, returned for this rank's rows — the
    distributed sample sort of ``parallel/sort.global_average_ranks`` (reference ``SpearmanCorrelation.java:61``,
    ``SortUtils.pSort``): no rank gathers the column."""
    from ...parallel.sort import global_average_ranks
    return global_average_ranks(v)


def _pearson_pairwise(X: torch.Tensor, valid: torch.Tensor) -> np.ndarray:
    """Pearson correlation over pairwise-complete rows (reference ``TableSummarizer.correlation``: every pair of
    columns uses the rows where both are present).  Five d x d moment matrices from four GEMMs over the masked
    values, all-reduced in one buffer: n_ij, sum x_i, sum x_i^2 (over the pair's rows), sum x_i x_j."""
    M = valid.to(X.dtype)
    A = torch.where(valid, X, torch.zeros_like(X))
    d = X.shape[1]
    mom = torch.stack([tn_matmul(M, M), tn_matmul(A, M), tn_matmul(A * A, M), tn_matmul(A, A)])
    comm.all_reduce(mom, "sum")
    N, Sx, Sxx, Sxy = mom[0], mom[1], mom[2], mom[3]
    Sy, Syy = Sx.T, Sxx.T
    num = N * Sxy - Sx * Sy
    den = torch.sqrt(torch.clamp(N * Sxx - Sx * Sx, min=0.0) * torch.clamp(N * Syy - Sy * Sy, min=0.0))
    corr = torch.where((den == 0) | (N < 2), torch.full_like(num, float("nan")), num / torch.where(den == 0,
                                                                                             torch.ones_like(den), den))
    corr.fill_diagonal_(1.0)
    return corr.cpu().numpy() if d else np.zeros((0, 0))


def _pearson(X: torch.Tensor) -> np.ndarray:
    n_loc = torch.tensor([float(X.shape[0])], dtype=torch.float64, device=X.device)
    s = X.sum(0)
    G = tn_matmul(X, X)
    buf = torch.cat([n_loc, s, G.reshape(-1)])
    comm.all_reduce(buf, "sum")
    d = X.shape[1]
    n = float(buf[0])
    s, G = buf[1:1 + d], buf[1 + d:].reshape(d, d)
    cov = (G - torch.outer(s, s) / n) / max(n - 1, 1.0)
    sd = torch.sqrt(torch.clamp(torch.diagonal(cov), min=0.0))
    corr = cov / torch.outer(sd, sd)
    corr = torch.where(torch.outer(sd, sd) == 0, torch.full_like(corr, float("nan")), corr)
    corr.fill_diagonal_(1.0)
    return corr.cpu().numpy()


def correlation(mt: MTable, cols: Sequence[str], method: str = "PEARSON", device=None) -> CorrelationResult:
    dev = device or torch.device("cpu")
    from ..tree.data import numeric_column
    vals, nulls = zip(*[numeric_column(mt, c, dev) for c in cols]) if cols else ((), ())
    nulls_any = comm.all_gather_object(bool(any(bool(m.any()) for m in nulls)))
    if not any(nulls_any):
        X = extract_features(mt, list(cols), None, dev).dense.double()
        if _is_spearman(method):
            X = torch.stack([_rank_global(X[:, j]) for j in range(X.shape[1])], 1) if X.shape[1] else X
        return CorrelationResult(_pearson(X), list(cols))
    # NULL / NaN cells: pairwise-complete statistics (Spearman ranks the present values of each column)
    X = torch.stack(vals, 1)
    valid = ~torch.stack(nulls, 1)
    if _is_spearman(method):
        X = torch.stack([_rank_present_global(X[:, j], valid[:, j]) for j in range(X.shape[1])], 1)
    return CorrelationResult(_pearson_pairwise(X, valid), list(cols))


def _rank_present_global(v: torch.Tensor, ok: torch.Tensor) -> torch.Tensor:
    """Average ranks among the column's present values (global over ranks); absent cells get 0 (masked)."""
    out = torch.zeros_like(v)
    idx = torch.nonzero(ok).reshape(-1)
    out[idx] = _rank_global(v[idx])
    return out


def vector_correlation(mt: MTable, vector_col: str, method: str = "PEARSON", device=None) -> CorrelationResult:
    dev = device or torch.device("cpu")
    fm = extract_features(mt, None, vector_col, dev)
    d = max(comm.all_gather_object(int(fm.ncols)))
    X = fm.to_dense(d).double()
    if _is_spearman(method):
        X = torch.stack([_rank_global(X[:, j]) for j in range(X.shape[1])], 1)
    return CorrelationResult(_pearson(X), None)


class ChiSquareTestResult:
    __gson_fields__ = ("comment", "df", "p", "value")

    def __init__(self, df, p, value, comment="pearson test", col=None):
        self.df, self.p, self.value, self.comment, self.colName = float(df), float(p), float(value), comment, col

    def getDf(self):
        return self.df

    def getP(self):
        return self.p

    def getValue(self):
        return self.value

    def getColName(self):
        return self.colName


def chi_square_test(pairs_per_col: List[List[tuple]], names: List[str]) -> List[ChiSquareTestResult]:
    """Pearson chi-square independence test of each feature column vs the label (``ChiSquareTest.java``):
    contingency tables are merged across ranks via all-gather of (value, label) -> count maps."""
    from scipy.stats import chi2
    out = []
    for name, pairs in zip(names, pairs_per_col):
        merged = {}
        for part in comm.all_gather_object(pairs):
            for k, c in part:
                merged[k] = merged.get(k, 0) + c
        rows = sorted({k[0] for k in merged}, key=str)
        cols = sorted({k[1] for k in merged}, key=str)
        obs = np.zeros((len(rows), len(cols)))
        ri = {r: i for i, r in enumerate(rows)}
        ci = {c: i for i, c in enumerate(cols)}
        for (a, b), c in merged.items():
            obs[ri[a], ci[b]] += c
        tot = obs.sum()
        exp = np.outer(obs.sum(1), obs.sum(0)) / tot if tot else obs
        with np.errstate(divide="ignore", invalid="ignore"):
            stat = float(np.nansum((obs - exp) ** 2 / np.where(exp == 0, np.nan, exp)))
        df = (len(rows) - 1) * (len(cols) - 1)
        p = float(chi2.sf(stat, df)) if df > 0 else 1.0
        out.append(ChiSquareTestResult(df, p, stat, col=name))
    return out
