"""``DenseMatrix`` (row-level API of ``A/common/linalg/DenseMatrix.java``).

Backed by a 2-D float64 numpy array.  Gson form follows the Java class: ``{"m":..,"n":..,"data":[...]}``
with ``data`` in column-major order.
"""
from __future__ import annotations

import numpy as np

from .vector import DenseVector

__all__ = ["DenseMatrix"]


class DenseMatrix:
    __gson_fields__ = ("m", "n", "data")

    def __init__(self, *args):
        if len(args) == 1:
            a = np.asarray(args[0], dtype=np.float64)
            if a.ndim == 1:
                a = a.reshape(-1, 1)
            self.a = a.copy()
        elif len(args) == 2:
            self.a = np.zeros((int(args[0]), int(args[1])), dtype=np.float64)
        elif len(args) in (3, 4):  # (m, n, data[, inRowMajor]) — column-major unless inRowMajor
            m, n, data = int(args[0]), int(args[1]), args[2]
            arr = np.asarray(data, dtype=np.float64).reshape(-1)
            if arr.size != m * n:
                raise ValueError("Size not match.")
            row_major = bool(args[3]) if len(args) == 4 else False
            self.a = arr.reshape(m, n).copy() if row_major else arr.reshape(n, m).T.copy()
        else:
            self.a = np.zeros((0, 0))

    # gson view
    @property
    def m(self):
        return self.a.shape[0]

    @property
    def n(self):
        return self.a.shape[1]

    @property
    def data(self):
        return self.a.T.reshape(-1)

    @staticmethod
    def eye(m, n=None):
        return DenseMatrix(np.eye(m, m if n is None else n))

    @staticmethod
    def zeros(m, n):
        return DenseMatrix(m, n)

    @staticmethod
    def ones(m, n):
        return DenseMatrix(np.ones((m, n)))

    @staticmethod
    def rand(m, n, seed=None):
        return DenseMatrix(np.random.default_rng(seed).random((m, n)))

    @staticmethod
    def randSymmetric(n, seed=None):
        r = np.random.default_rng(seed).random((n, n))
        return DenseMatrix(np.triu(r) + np.triu(r, 1).T)

    def numRows(self):
        return self.a.shape[0]

    def numCols(self):
        return self.a.shape[1]

    def get(self, i, j):
        return float(self.a[i, j])

    def set(self, i, j, v):
        self.a[i, j] = v

    def add(self, i, j, v):
        self.a[i, j] += v

    def getArrayCopy2D(self):
        return self.a.copy()

    def getArrayCopy1D(self, inRowMajor: bool):
        return (self.a if inRowMajor else self.a.T).reshape(-1).copy()

    def selectRows(self, rows):
        return DenseMatrix(self.a[np.asarray(rows, dtype=np.int64)])

    def getSubMatrix(self, m0, m1, n0, n1):
        """Rows [m0, m1), columns [n0, n1)."""
        return DenseMatrix(self.a[m0:m1, n0:n1])

    def setSubMatrix(self, sub, m0, m1, n0, n1):
        self.a[m0:m1, n0:n1] = sub.a if isinstance(sub, DenseMatrix) else np.asarray(sub)

    def sum(self):
        return float(self.a.sum())

    def getData(self):
        return self.data

    def getRow(self, i):
        return self.a[i].copy()

    def getColumn(self, j):
        return self.a[:, j].copy()

    def transpose(self):
        return DenseMatrix(self.a.T)

    def multiplies(self, o):
        from .vector import SparseVector
        if isinstance(o, DenseMatrix):
            return DenseMatrix(self.a @ o.a)
        if isinstance(o, DenseVector):
            return DenseVector(self.a @ o.data)
        if isinstance(o, SparseVector):
            return DenseVector(self.a[:, o.indices.astype(np.int64)] @ o.values)
        return DenseMatrix(self.a @ np.asarray(o))

    def plus(self, o):
        return DenseMatrix(self.a + (o.a if isinstance(o, DenseMatrix) else o))

    def plusEquals(self, o):
        self.a += o.a if isinstance(o, DenseMatrix) else o

    def minus(self, o):
        return DenseMatrix(self.a - o.a)

    def minusEquals(self, o):
        self.a -= o.a

    def scale(self, v):
        return DenseMatrix(self.a * v)

    def scaleEqual(self, v):
        self.a *= v

    def solve(self, b):
        bb = b.a if isinstance(b, DenseMatrix) else (b.data if isinstance(b, DenseVector) else np.asarray(b))
        x = np.linalg.lstsq(self.a, bb, rcond=None)[0] if self.a.shape[0] != self.a.shape[1] else np.linalg.solve(self.a, bb)
        return DenseMatrix(x) if isinstance(b, DenseMatrix) else DenseVector(x)

    def solveLS(self, b):
        bb = b.a if isinstance(b, DenseMatrix) else b.data
        x = np.linalg.lstsq(self.a, bb, rcond=None)[0]
        return DenseMatrix(x) if isinstance(b, DenseMatrix) else DenseVector(x)

    def inverse(self):
        return DenseMatrix(np.linalg.inv(self.a))

    def pseudoInverse(self):
        return DenseMatrix(np.linalg.pinv(self.a))

    def det(self):
        return float(np.linalg.det(self.a))

    def rank(self):
        return int(np.linalg.matrix_rank(self.a))

    def norm2(self):
        return float(np.linalg.norm(self.a, 2))

    def cond(self):
        """Two-norm condition number (largest / smallest singular value)."""
        sv = np.linalg.svd(self.a, compute_uv=False)
        return float(sv[0] / sv[min(self.a.shape) - 1])

    def normF(self):
        return float(np.linalg.norm(self.a))

    def isSymmetric(self):
        return self.a.shape[0] == self.a.shape[1] and np.allclose(self.a, self.a.T)

    def isSquare(self):
        return self.a.shape[0] == self.a.shape[1]

    def clone(self):
        return DenseMatrix(self.a.copy())

    def __eq__(self, o):
        return isinstance(o, DenseMatrix) and np.array_equal(o.a, self.a)

    def toString(self):
        """``mat[m,n]:`` then one line per row, values as Java ``Double.toString`` (reference ``toString``)."""
        from ..javafmt import java_double_str
        lines = [f"mat[{self.m},{self.n}]:"]
        lines += ["  " + ",".join(java_double_str(float(v)) for v in row) for row in self.a]
        return "\n".join(lines) + "\n"

    __str__ = toString

    def __repr__(self):
        return f"DenseMatrix({self.a.tolist()})"
