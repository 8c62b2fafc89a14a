"""Distance measures of the public API (reference ``A/operator/common/distance/*.java``,
``A/operator/common/similarity/LevenshteinSimilarity.java``, ``A/operator/common/clustering/DistanceType.java``).

Every continuous distance offers the reference's pair form ``calc(a, b)`` (vectors or float arrays) and a block
form ``pairwise(A, B)`` -> ``[len(A), len(B)]`` over stacked rows.  The block form is the MI355X-shaped one: a
torch computation on the rows' device, GEMM-based for Euclidean / cosine (``|a|^2 + |b|^2 - 2 A B^T`` and
``1 - A_n B_n^T``: hipBLASLt on the GPU), which is what the reference's ``FastDistance`` matrix data emulates
with BLAS.  Algorithms that scan huge tables use their own fused kernels (KMeans: ``ops/csrc/kmeans_v10.hip``);
these classes serve user code, mappers and the evaluation / similarity operators.
"""
from __future__ import annotations

import math
from typing import Sequence, Union

import numpy as np
import torch

from .linalg import DenseMatrix, DenseVector, SparseVector, VectorUtil

__all__ = ["ContinuousDistance", "EuclideanDistance", "CosineDistance", "ManHattanDistance", "JaccardDistance",
           "HaversineDistance", "LevenshteinDistance", "LevenshteinSimilarity", "distance_of"]

EARTH_RADIUS = 6371.0


def _dense(v) -> np.ndarray:
    if isinstance(v, str):
        v = VectorUtil.getVector(v)
    if isinstance(v, SparseVector):
        return v.toDenseVector().data
    if isinstance(v, DenseVector):
        return v.data
    return np.asarray(v, dtype=np.float64)


def _pair(a, b):
    x, y = _dense(a), _dense(b)
    if x.shape != y.shape:                        # sparse vectors of unknown size (-1): pad the shorter
        n = max(x.size, y.size)
        x, y = np.pad(x, (0, n - x.size)), np.pad(y, (0, n - y.size))
    return x, y


def _rows(A, device=None) -> torch.Tensor:
    if isinstance(A, torch.Tensor):
        return A.to(torch.float64) if device is None else A.to(device=device, dtype=torch.float64)
    if isinstance(A, DenseMatrix):
        arr = A.getArrayCopy2D()
    else:
        vecs = [_dense(v) for v in A]
        n = max((v.size for v in vecs), default=0)
        arr = np.stack([np.pad(v, (0, n - v.size)) for v in vecs]) if vecs else np.zeros((0, 0))
    return torch.as_tensor(arr, dtype=torch.float64, device=device)


class ContinuousDistance:
    """calc(a, b) for one pair; pairwise(A, B) for row blocks (torch, on ``device``)."""

    def calc(self, a, b) -> float:
        x, y = _pair(a, b)
        return float(self._pair_np(x, y))

    def _pair_np(self, x: np.ndarray, y: np.ndarray) -> float:
        raise NotImplementedError

    def pairwise(self, A, B, device=None) -> torch.Tensor:
        X, Y = _rows(A, device), _rows(B, device)
        d = max(X.shape[1], Y.shape[1])
        X = torch.nn.functional.pad(X, (0, d - X.shape[1]))
        Y = torch.nn.functional.pad(Y, (0, d - Y.shape[1]))
        return self._pairwise(X, Y)

    def _pairwise(self, X: torch.Tensor, Y: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def pairwiseMatrix(self, A, B) -> DenseMatrix:
        return DenseMatrix(self.pairwise(A, B).cpu().numpy())


class EuclideanDistance(ContinuousDistance):
    def _pair_np(self, x, y):
        return math.sqrt(float(((x - y) ** 2).sum()))

    def _pairwise(self, X, Y):
        xn = (X * X).sum(1, keepdim=True)
        yn = (Y * Y).sum(1)[None, :]
        return torch.sqrt((xn + yn - 2.0 * (X @ Y.T)).clamp_min(0.0))


class CosineDistance(ContinuousDistance):
    """1 - a.b / (|a| |b|); 1 when either vector is zero."""

    def _pair_np(self, x, y):
        cross = math.sqrt(float(x @ x) * float(y @ y))
        return 1.0 - (float(x @ y) / cross if cross > 0.0 else 0.0)

    def _pairwise(self, X, Y):
        xn, yn = X.norm(dim=1), Y.norm(dim=1)
        Xn = X / torch.where(xn > 0, xn, torch.ones_like(xn))[:, None]
        Yn = Y / torch.where(yn > 0, yn, torch.ones_like(yn))[:, None]
        return 1.0 - Xn @ Yn.T


class ManHattanDistance(ContinuousDistance):
    """sum |a_i - b_i| (``CITYBLOCK``)."""

    def _pair_np(self, x, y):
        return float(np.abs(x - y).sum())

    def _pairwise(self, X, Y):
        return torch.cdist(X, Y, p=1.0)


class JaccardDistance(ContinuousDistance):
    """1 - |nz(a) & nz(b)| / |nz(a) | nz(b)| over the non-zero coordinates."""

    def _pair_np(self, x, y):
        a, b = x != 0, y != 0
        union = int((a | b).sum())
        return 1.0 - (int((a & b).sum()) / union if union else 0.0)

    def _pairwise(self, X, Y):
        A, B = (X != 0).to(torch.float64), (Y != 0).to(torch.float64)
        inter = A @ B.T
        union = A.sum(1)[:, None] + B.sum(1)[None, :] - inter
        return 1.0 - torch.where(union > 0, inter / torch.where(union > 0, union, torch.ones_like(union)),
                                 torch.zeros_like(inter))


class HaversineDistance(ContinuousDistance):
    """Great-circle distance in km between (latitude, longitude) pairs in degrees."""

    def calc(self, a, b, lat2=None, lon2=None) -> float:
        if lat2 is not None:                      # calc(latitude1, longitude1, latitude2, longitude2)
            return self._pair_np(np.array([a, b], dtype=np.float64), np.array([lat2, lon2], dtype=np.float64))
        return super().calc(a, b)

    def _pair_np(self, x, y):
        lat1, lon1, lat2, lon2 = (math.radians(float(v)) for v in (x[0], x[1], y[0], y[1]))
        h = (1 - math.cos(lat1 - lat2)) / 2 + math.cos(lat1) * math.cos(lat2) * (1 - math.cos(lon1 - lon2)) / 2
        return 2 * EARTH_RADIUS * math.asin(min(1.0, math.sqrt(abs(h))))

    def _pairwise(self, X, Y):
        lat1, lon1 = torch.deg2rad(X[:, 0:1]), torch.deg2rad(X[:, 1:2])
        lat2, lon2 = torch.deg2rad(Y[:, 0])[None, :], torch.deg2rad(Y[:, 1])[None, :]
        h = (1 - torch.cos(lat1 - lat2)) / 2 + torch.cos(lat1) * torch.cos(lat2) * (1 - torch.cos(lon1 - lon2)) / 2
        return 2 * EARTH_RADIUS * torch.asin(torch.sqrt(h.abs()).clamp(max=1.0))


class LevenshteinDistance:
    """Edit distance between two strings or two token lists (insert / delete / substitute, cost 1)."""

    @staticmethod
    def calcDistance(left: Union[str, Sequence], right: Union[str, Sequence]) -> int:
        if len(left) == 0:
            return len(right)
        if len(right) == 0:
            return len(left)
        if len(left) < len(right):
            left, right = right, left
        prev = list(range(len(right) + 1))
        for i in range(1, len(left) + 1):
            cur = [i] + [0] * len(right)
            li = left[i - 1]
            for j in range(1, len(right) + 1):
                cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (0 if li == right[j - 1] else 1))
            prev = cur
        return prev[-1]

    def calc(self, left, right) -> int:
        return self.calcDistance(left, right)


class LevenshteinSimilarity:
    """1 - distance / max(len) (1 for two empty inputs)."""

    def similarity(self, left, right) -> float:
        n = max(len(left), len(right))
        return 1.0 if n == 0 else 1.0 - LevenshteinDistance.calcDistance(left, right) / n

    calc = similarity


def distance_of(name: str) -> ContinuousDistance:
    """The ``DistanceType`` enum's measure by name (EUCLIDEAN, COSINE, CITYBLOCK, HAVERSINE, JACCARD)."""
    key = str(getattr(name, "name", name)).upper()
    table = {"EUCLIDEAN": EuclideanDistance, "COSINE": CosineDistance, "CITYBLOCK": ManHattanDistance,
             "MANHATTAN": ManHattanDistance, "HAVERSINE": HaversineDistance, "JACCARD": JaccardDistance}
    if key not in table:
        raise ValueError(f"unknown distance type {name}")
    return table[key]()
