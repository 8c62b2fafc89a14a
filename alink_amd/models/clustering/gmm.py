"""Gaussian mixture model, full covariances, EM (reference ``A/operator/batch/clustering/GmmTrainBatchOp.java``,
``A/operator/common/clustering/{GmmModelData,GmmModelDataConverter,GmmModelMapper}.java``,
``A/operator/common/statistics/basicstatistic/MultivariateGaussian.java``).

Semantics kept: initialisation from ``5 k`` samples drawn with replacement, sample ``i`` seeding component
``i mod k`` (mean + diagonal covariance); E-step responsibilities from the previous parameters; M-step
``w = sum r / N``, ``mu = sum r x / sum r``, ``Sigma = sum r x x^T / sum r - mu mu^T``; stop when
``|LL_t - LL_{t-1}| <= tol`` after the first step or at ``maxIter``; densities with the pseudo-inverse /
pseudo-determinant of the covariance (eigenvalues below ``eps * max * d`` dropped).  Covariances are stored
upper-packed column-major (``(1 + j) j / 2 + i``, i <= j).

MI355X design: one EM step = a batched ``[n, k]`` log-density evaluation (``(X - mu_k) W_k`` GEMMs with
``W_k = U diag(lambda^-1/2)``), a log-sum-exp, and the weighted moment sums ``R^T X`` and
``X^T diag(r_k) X`` as GEMMs — all on the device — followed by ONE all-reduce of the
``k (1 + d + d^2) + 1`` statistics buffer (the reference's reduce-to-one + broadcast).
"""
from __future__ import annotations

import json
import math
from typing import List, Optional

import numpy as np
import torch

from ...ops.gemm import tn_matmul
from ...common.javafmt import gson_dumps
from ...common.linalg import DenseVector, VectorUtil
from ...common.mapper import OutputColsHelper, RichModelMapper
from ...common.model.converter import SimpleModelDataConverter
from ...common.params import Params
from ...common.strings import StringBlock
from ...common.table import Column, MTable
from ...common.types import Types
from ...ops import gmm as gmm_ops
from ...parallel import comm
from ..common.features import extract_features, global_vector_size

__all__ = ["train_gmm", "GmmModelMapper", "pack_cov", "unpack_cov", "gaussian_logpdf"]

_EPS = 2.220446049250313e-16


def pack_cov(S: np.ndarray) -> np.ndarray:
    d = S.shape[0]
    out = np.zeros(d * (d + 1) // 2)
    for j in range(d):
        for i in range(j + 1):
            out[(1 + j) * j // 2 + i] = S[i, j]
    return out


def unpack_cov(v, d: int) -> np.ndarray:
    S = np.zeros((d, d))
    for j in range(d):
        for i in range(j + 1):
            S[i, j] = S[j, i] = v[(1 + j) * j // 2 + i]
    return S


def _root_inv(cov: torch.Tensor):
    """(W [k, d, d], log-pseudo-determinant [k], normaliser dimension [k]) with x^T Sigma^+ x = |x W|^2.  The
    (2 pi)^(-k/2) factor uses the full dimension d even for a singular covariance, as the reference
    (``MultivariateGaussian.java:89-115``: ``u = -0.5 * (k * log(2 pi) + logPseudoDet)`` with k = mean size)."""
    lam, U = torch.linalg.eigh(cov)
    tol = _EPS * lam.max(dim=-1, keepdim=True).values * cov.shape[-1]
    keep = lam > tol
    inv_sqrt = torch.where(keep, 1.0 / torch.sqrt(torch.where(keep, lam, torch.ones_like(lam))),
                           torch.zeros_like(lam))
    W = U * inv_sqrt[..., None, :]
    logdet = torch.where(keep, torch.log(torch.where(keep, lam, torch.ones_like(lam))), torch.zeros_like(lam)).sum(-1)
    return W, logdet, torch.full_like(logdet, float(cov.shape[-1]))


def gaussian_logpdf(X: torch.Tensor, mean: torch.Tensor, cov: torch.Tensor) -> torch.Tensor:
    """[n, k] log densities (``MultivariateGaussian.logpdf``)."""
    return _logpdf_root(X, mean, *_root_inv(cov))


def _logpdf_root(X, mean, W, logdet, rank):
    """``gaussian_logpdf`` from the ``_root_inv`` factors (all on X's device)."""
    out = torch.empty((X.shape[0], mean.shape[0]), dtype=X.dtype, device=X.device)
    for j in range(mean.shape[0]):
        z = (X - mean[j]) @ W[j]
        out[:, j] = -0.5 * (rank[j] * math.log(2 * math.pi) + logdet[j]) - 0.5 * (z * z).sum(1)
    return out


class MultivariateGaussian:
    """Gaussian density with a possibly singular covariance (reference
    ``A/operator/common/statistics/basicstatistic/MultivariateGaussian.java``): pseudo-inverse and
    pseudo-determinant over the eigenvalues above ``eps * max * d``, as the GMM E-step uses."""

    def __init__(self, mean, cov):
        mu = mean.getData() if hasattr(mean, "getData") else mean
        sig = cov.getArrayCopy2D() if hasattr(cov, "getArrayCopy2D") else cov
        self.mean = torch.as_tensor(np.asarray(mu, dtype=np.float64))[None, :]
        self.cov = torch.as_tensor(np.asarray(sig, dtype=np.float64))[None, :, :]

    def logpdf(self, x) -> float:
        v = x.getData() if hasattr(x, "getData") else x
        X = torch.as_tensor(np.asarray(v, dtype=np.float64))[None, :]
        return float(gaussian_logpdf(X, self.mean, self.cov)[0, 0])

    def pdf(self, x) -> float:
        return math.exp(self.logpdf(x))


def _weighted_syrk(R: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
    """[k, d, d] = sum_i R[i, k] x_i x_i^T.  On the GPU one [k*d, rows] x [rows, d] hipBLASLt GEMM per row chunk of
    at most ~1 GiB of (R (x) X) operand; the CPU keeps the einsum."""
    n, k = R.shape
    d = X.shape[1]
    if not X.is_cuda:
        return torch.einsum("nk,nd,ne->kde", R, X, X)
    out = torch.zeros((k * d, d), dtype=X.dtype, device=X.device)
    rows = max(1, min(n, (1 << 30) // (8 * max(1, k * d))))
    for s in range(0, n, rows):
        e = min(n, s + rows)
        A = (R[s:e, :, None] * X[s:e, None, :]).reshape(e - s, k * d)
        out += tn_matmul(A, X[s:e])
    return out.reshape(k, d, d)


def train_gmm(mt: MTable, params: Params, env) -> List[tuple]:
    dev = env.device
    vcol = params.get("vectorCol")
    k = int(params.get("k")) if params.contains("k") and params.get("k") is not None else 2
    max_iter = int(params.get("maxIter")) if params.contains("maxIter") and params.get("maxIter") is not None else 100
    tol = float(params.get("tol")) if params.contains("tol") and params.get("tol") is not None else 0.01
    seed = int(params.get("randomSeed")) if params.contains("randomSeed") and params.get("randomSeed") is not None \
        else 0
    fm = extract_features(mt, None, vcol, dev)
    d = global_vector_size(fm)
    if fm.is_sparse:
        fm.set_ncols(d)
    X = fm.to_dense().to(torch.float64)
    if X.shape[1] < d:
        X = torch.nn.functional.pad(X, (0, d - X.shape[1]))
    # init: 5k samples with replacement (gathered to every rank; identical draw everywhere)
    counts = comm.all_gather_object(int(X.shape[0]))
    total = sum(counts)
    rng = np.random.default_rng(seed)
    pick = rng.integers(0, total, size=5 * k)
    offs = np.cumsum([0] + counts)
    me = comm.get_rank()
    local = [(j, int(g - offs[me])) for j, g in enumerate(pick) if offs[me] <= g < offs[me + 1]]
    rows = X[[i for _, i in local]].cpu().numpy() if local else np.zeros((0, d))
    got = {}
    for part in comm.all_gather_object([(j, r.tolist()) for (j, _), r in zip(local, rows)]):
        for j, r in part:
            got[j] = np.asarray(r)
    samples = np.stack([got[j] for j in range(5 * k)])
    means = np.stack([samples[np.arange(5 * k) % k == c].mean(0) for c in range(k)])
    covs = np.stack([np.diag(((samples[np.arange(5 * k) % k == c] - means[c]) ** 2).mean(0)) for c in range(k)])
    weights = np.full(k, 1.0 / k)
    mu = torch.as_tensor(means, device=dev)
    S = torch.as_tensor(covs, device=dev)
    w = torch.as_tensor(weights, device=dev)
    prev = 0.0
    # K22: centre once by the global mean, then every E-step is one GEMM for all components plus one fused
    # log-density / log-sum-exp / responsibility kernel (ops/gmm.py)
    xs_n = torch.cat([X.sum(0), torch.tensor([float(X.shape[0])], dtype=X.dtype, device=dev)])
    comm.all_reduce(xs_n, "sum")
    xbar = xs_n[:d] / xs_n[d].clamp(min=1.0)
    X0 = X - xbar
    for step in range(1, max_iter + 1):
        Wr, logdet, rank = _root_inv(S)
        R, lse_sum = gmm_ops.estep(X0, mu - xbar, Wr, logdet, rank, torch.log(w))
        stats = torch.cat([R.sum(0), tn_matmul(R, X).reshape(-1),
                           _weighted_syrk(R, X).reshape(-1), lse_sum.reshape(1),
                           torch.tensor([float(X.shape[0])], dtype=X.dtype, device=dev)])
        comm.all_reduce(stats, "sum")
        rs = stats[:k]
        xs = stats[k:k + k * d].reshape(k, d)
        xxs = stats[k + k * d:k + k * d + k * d * d].reshape(k, d, d)
        ll = float(stats[-2])
        n = float(stats[-1])
        mu = xs / rs[:, None]
        S = xxs / rs[:, None, None] - mu[:, :, None] * mu[:, None, :]
        w = rs / n
        if step > 1 and abs(ll - prev) <= tol:
            break
        prev = ll
    mu_n, S_n, w_n = mu.cpu().numpy(), S.cpu().numpy(), w.cpu().numpy()
    meta = Params().set("numFeatures", d).set("k", k).set("vectorCol", vcol)
    data = []
    for c in range(k):
        data.append(gson_dumps(_Cluster(c, float(w_n[c]), DenseVector(mu_n[c]), DenseVector(pack_cov(S_n[c]))),
                               java_map_order=False))
    return SimpleModelDataConverter.rows_from(meta, data)


class _Cluster:
    __gson_fields__ = ("clusterId", "weight", "mean", "cov")

    def __init__(self, cid, weight, mean, cov):
        self.clusterId, self.weight, self.mean, self.cov = cid, weight, mean, cov


class GmmModelMapper(RichModelMapper):
    def predResultType(self):
        return Types.LONG

    def loadModel(self, rows):
        meta, data = SimpleModelDataConverter.split_rows(rows)
        self.k = int(meta.get("k"))
        self.d = int(meta.get("numFeatures"))
        cl = sorted((json.loads(s) for s in data), key=lambda c: c["clusterId"])
        self.w = np.asarray([c["weight"] for c in cl])
        self.mu = np.stack([np.asarray(c["mean"]["data"]) for c in cl])
        self.S = np.stack([unpack_cov(c["cov"]["data"], self.d) for c in cl])
        self.vcol = self.params.get("vectorCol") if self.params.contains("vectorCol") and \
            self.params.get("vectorCol") else meta.get("vectorCol")

    def _map_row_values(self, row):
        mt = MTable.from_rows([tuple(row)], self.dataSchema)
        return [c.to_list()[0] for c in self._map_columns(mt)]

    def _map_columns(self, mt):
        from ..linear.model import _dev
        dev = _dev(mt)
        fm = extract_features(mt, None, self.vcol, dev)
        if fm.is_sparse:
            fm.set_ncols(self.d)
        X = fm.to_dense().double()
        f = getattr(self, "_factors", None)
        if f is None or f[0].device != X.device:
            # pseudo-inverse roots once per mapper, on the host (small k x d x d eigh), then kept on X's device
            W, logdet, rank = _root_inv(torch.as_tensor(self.S))
            f = self._factors = tuple(t.to(X.device) for t in (torch.as_tensor(self.mu), W, logdet, rank))
        lp = _logpdf_root(X, *f).cpu().numpy()
        lw = lp + np.log(self.w)[None, :]
        m = lw.max(1, keepdims=True)
        prob = np.exp(lw - m)
        prob = prob / prob.sum(1, keepdims=True)
        pred = prob.argmax(1)
        cols = [Column(torch.from_numpy(pred.astype(np.int64)))]
        if self.detail_col:
            from ... import _native
            r = _native.java_double_rows_packed(prob, " ") if len(prob) else None
            if r is not None:
                cols.append(Column(StringBlock(torch.from_numpy(np.ascontiguousarray(r[0])), torch.from_numpy(r[1]))))
            else:
                cols.append(Column.from_values([VectorUtil.toString(DenseVector(p)) for p in prob], Types.STRING))
        return cols
