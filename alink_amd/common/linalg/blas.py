"""Host linear-algebra helpers of the public linalg API: ``BLAS`` (reference ``A/common/linalg/BLAS.java``),
``MatVecOp`` (``MatVecOp.java``) and ``NormalEquation`` (``NormalEquation.java``).

These operate in place on the numpy storage of ``DenseVector`` / ``DenseMatrix`` (per-row utilities for user code,
model mappers and small solves, like the reference's F2J/netlib calls).  Bulk work never goes through them: the
algorithms run their GEMMs and solves on the device (hipBLASLt through torch, ``ops/gemm.py``, ``ops/csrc/als.hip``).
"""
from __future__ import annotations

from typing import Callable

import numpy as np

from .matrix import DenseMatrix
from .vector import DenseVector, SparseVector, Vector

__all__ = ["BLAS", "MatVecOp", "NormalEquation"]


def _check(cond: bool, msg: str):
    if not cond:
        raise ValueError(msg)


class BLAS:
    """Level-1/2/3 kernels with the reference's signatures; results are written into the last argument."""

    @staticmethod
    def asum(x) -> float:
        if isinstance(x, SparseVector):
            return float(np.abs(x.values).sum())
        if isinstance(x, DenseVector):
            return float(np.abs(x.data).sum())
        return float(np.abs(np.asarray(x, dtype=np.float64)).sum())

    @staticmethod
    def axpy(*args):
        """``axpy(a, x, y)``: y += a * x (vectors, dense matrices, or float arrays);
        ``axpy(n, a, x, xOffset, y, yOffset)``: y[yOffset:yOffset+n] += a * x[xOffset:xOffset+n]."""
        if len(args) == 6:
            n, a, x, xo, y, yo = args
            yy = y.data if isinstance(y, DenseVector) else y
            xx = x.data if isinstance(x, DenseVector) else np.asarray(x, dtype=np.float64)
            yy[yo:yo + n] += a * xx[xo:xo + n]
            return
        a, x, y = args
        if isinstance(y, DenseMatrix):
            _check(isinstance(x, DenseMatrix) and x.a.shape == y.a.shape, "matrix size mismatched.")
            y.a += a * x.a
            return
        if isinstance(y, DenseVector):
            _check(x.size() == y.size(), "Vector size mismatched.")
            if isinstance(x, SparseVector):
                np.add.at(y.data, x.indices.astype(np.int64), a * x.values)
            else:
                y.data += a * x.data
            return
        yy = np.asarray(y)
        yy += a * np.asarray(x, dtype=np.float64)

    @staticmethod
    def dot(x, y) -> float:
        if isinstance(x, Vector) and isinstance(y, Vector):
            _check(x.size() == y.size(), "DenseVector size mismatched.")
            return float(x.dot(y))
        x, y = np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)
        _check(x.shape == y.shape, "Array dimension mismatched.")
        return float(x @ y)

    @staticmethod
    def scal(a: float, x):
        if isinstance(x, DenseMatrix):
            x.a *= a
        elif isinstance(x, SparseVector):
            x.values *= a
        elif isinstance(x, DenseVector):
            x.data *= a
        else:
            arr = np.asarray(x)
            arr *= a

    @staticmethod
    def gemm(alpha: float, matA: DenseMatrix, transA: bool, matB: DenseMatrix, transB: bool, beta: float,
             matC: DenseMatrix):
        """C = alpha * op(A) * op(B) + beta * C."""
        A = matA.a.T if transA else matA.a
        B = matB.a.T if transB else matB.a
        _check(A.shape[1] == B.shape[0] and A.shape[0] == matC.a.shape[0] and B.shape[1] == matC.a.shape[1],
               "matrix size mismatched.")
        matC.a[...] = alpha * (A @ B) + (beta * matC.a if beta != 0.0 else 0.0)

    @staticmethod
    def gemv(alpha: float, matA: DenseMatrix, transA: bool, x: Vector, beta: float, y: DenseVector):
        """y = alpha * op(A) * x + beta * y (x dense or sparse)."""
        rows, cols = (matA.a.shape[1], matA.a.shape[0]) if transA else matA.a.shape
        _check(x.size() == cols and y.size() == rows, "Matrix and vector size mismatched.")
        A = matA.a.T if transA else matA.a
        if isinstance(x, SparseVector):
            prod = A[:, x.indices.astype(np.int64)] @ x.values
        else:
            prod = A @ x.data
        y.data[...] = alpha * prod + (beta * y.data if beta != 0.0 else 0.0)


class MatVecOp:
    """Element-wise and reduction helpers over mixed dense / sparse vectors and dense matrices."""

    @staticmethod
    def plus(v1: Vector, v2: Vector) -> Vector:
        return v1.plus(v2)

    @staticmethod
    def minus(v1: Vector, v2: Vector) -> Vector:
        return v1.minus(v2)

    @staticmethod
    def dot(v1: Vector, v2: Vector) -> float:
        return float(v1.dot(v2))

    @staticmethod
    def sumAbsDiff(v1: Vector, v2: Vector) -> float:
        """|| v1 - v2 ||_1"""
        return MatVecOp.applySum(v1, v2, np.subtract, absolute=True)

    @staticmethod
    def sumSquaredDiff(v1: Vector, v2: Vector) -> float:
        """|| v1 - v2 ||_2^2"""
        d = MatVecOp._diff_values(v1, v2)
        return float(d @ d)

    @staticmethod
    def _diff_values(v1: Vector, v2: Vector) -> np.ndarray:
        _check(v1.size() == v2.size(), "x1 and x2 size mismatched.")
        if isinstance(v1, SparseVector) and isinstance(v2, SparseVector):
            r = MatVecOp.apply(v1, v2, lambda a, b: a - b)
            return r.values
        return _dense(v1) - _dense(v2)

    @staticmethod
    def apply(x, y, func: Callable, out=None):
        """Element-wise: ``apply(x, y, f)`` -> y = f(x) for matrices / dense vectors (unary ``f``);
        ``apply(x1, x2, f)`` -> new SparseVector f(x1, x2) over the union of indices for two sparse vectors;
        ``apply(x1, x2, f, out)`` -> out = f(x1, x2) for matrices / dense vectors."""
        if isinstance(x, SparseVector) and isinstance(y, SparseVector):
            _check(x.size() == y.size(), "x1 and x2 size mismatched.")
            idx = np.union1d(x.indices, y.indices).astype(np.int64)
            a = np.zeros(idx.size)
            b = np.zeros(idx.size)
            a[np.searchsorted(idx, x.indices)] = x.values
            b[np.searchsorted(idx, y.indices)] = y.values
            vals = np.fromiter((func(float(p), float(q)) for p, q in zip(a, b)), dtype=np.float64, count=idx.size)
            return SparseVector(x.size(), idx, vals)
        if out is None:
            src, dst = _storage(x), _storage(y)
            _check(src.shape == dst.shape, "x and y size mismatched.")
            dst[...] = np.vectorize(func, otypes=[np.float64])(src)
            return None
        a, b, dst = _storage(x), _storage(y), _storage(out)
        _check(a.shape == b.shape == dst.shape, "x1, x2 and y size mismatched.")
        dst[...] = np.vectorize(func, otypes=[np.float64])(a, b)
        return None

    @staticmethod
    def applySum(x1, x2, func: Callable, absolute: bool = False) -> float:
        """sum_i func(x1_i, x2_i): over the union of stored indices for two sparse vectors, over all entries
        otherwise.  ``func`` may be a numpy ufunc (vectorised) or a scalar function."""
        if isinstance(x1, SparseVector) and isinstance(x2, SparseVector):
            _check(x1.size() == x2.size(), "x1 and x2 size mismatched.")
            idx = np.union1d(x1.indices, x2.indices)
            a = np.zeros(idx.size)
            b = np.zeros(idx.size)
            a[np.searchsorted(idx, x1.indices)] = x1.values
            b[np.searchsorted(idx, x2.indices)] = x2.values
        else:
            a = _dense(x1) if isinstance(x1, Vector) else _storage(x1).reshape(-1)
            b = _dense(x2) if isinstance(x2, Vector) else _storage(x2).reshape(-1)
            _check(a.shape == b.shape, "x1 and x2 size mismatched.")
        if isinstance(func, np.ufunc):
            v = func(a, b)
        else:
            v = np.fromiter((func(float(p), float(q)) for p, q in zip(a, b)), dtype=np.float64, count=a.size)
        if absolute:
            v = np.abs(v)
        return float(v.sum())

    @staticmethod
    def appendVectorToMatrix(matrix: DenseMatrix, trans: bool, index: int, vector: Vector):
        """Write ``vector`` into row ``index`` (trans) or column ``index`` of ``matrix``."""
        size = matrix.numCols() if trans else matrix.numRows()
        if isinstance(vector, DenseVector):
            _check(vector.size() == size, f"Matrix and vector size mismatched, matrix size {size}, "
                                          f"vectorSize {vector.size()}")
            vals = vector.data
        else:
            _check(not len(vector.indices) or int(vector.indices[-1]) < size,
                   f"Index {int(vector.indices[-1]) if len(vector.indices) else -1} out of matrix size {size}!")
            vals = np.zeros(size)
            vals[vector.indices.astype(np.int64)] = vector.values
        if trans:
            matrix.a[index, :] = vals
        else:
            matrix.a[:, index] = vals


def _dense(v: Vector) -> np.ndarray:
    return v.toDenseVector().data if isinstance(v, SparseVector) else v.data


def _storage(x) -> np.ndarray:
    if isinstance(x, DenseMatrix):
        return x.a
    if isinstance(x, DenseVector):
        return x.data
    raise TypeError(f"dense vector or matrix expected, got {type(x).__name__}")


class NormalEquation:
    """Accumulates A^T A and A^T b row by row and solves (A^T A + lambda I) x = A^T b (reference ALS local
    solver; the training path solves batched systems on the device instead, ``ops/csrc/als.hip``)."""

    def __init__(self, n: int):
        self.n = int(n)
        self.ata = DenseMatrix(self.n, self.n)
        self.atb = DenseVector(self.n)

    def add(self, a: DenseVector, b: float, c: float):
        """ata += c * a a^T ; atb += b * a"""
        self.ata.a += c * np.outer(a.data, a.data)
        self.atb.data += b * a.data

    def reset(self):
        self.ata.a[...] = 0.0
        self.atb.data[...] = 0.0

    def merge(self, otherAta: DenseMatrix):
        self.ata.a += otherAta.a

    def regularize(self, lam: float):
        self.ata.a[np.diag_indices(self.n)] += lam

    def solve(self, x: DenseVector, nonNegative: bool = False):
        """Solution into ``x``; the accumulators are reset afterwards (as the reference)."""
        if nonNegative:
            import torch
            from ...ops.als import nnls
            sol = nnls(torch.as_tensor(self.ata.a)[None], torch.as_tensor(self.atb.data)[None])[0].numpy()
        else:
            L = np.linalg.cholesky(self.ata.a)
            sol = np.linalg.solve(L.T, np.linalg.solve(L, self.atb.data))
        x.data[...] = sol
        self.reset()
