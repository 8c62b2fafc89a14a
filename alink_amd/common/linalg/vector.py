"""Row-level vector types: ``DenseVector``, ``SparseVector`` and ``VectorUtil`` string formats.

Semantics follow ``A/common/linalg/{DenseVector,SparseVector,Vector,VectorUtil}.java``: dense strings are
space (or comma) separated values ``"1 2 3"``; sparse strings are ``"$size$i:v i:v"`` with an
optional ``$size$`` header (``VectorUtil.java:12-230``).  Values are float64 (the reference is
``double[]``).  Batch/columnar work never goes through these objects — see ``common.table``.
"""
from __future__ import annotations

import math
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np

from ..javafmt import java_double_str

__all__ = ["Vector", "DenseVector", "SparseVector", "VectorUtil", "VectorIterator"]


class Vector:
    def size(self) -> int:
        raise NotImplementedError

    def get(self, i: int) -> float:
        raise NotImplementedError

    def toDense(self) -> "DenseVector":
        raise NotImplementedError

    def __str__(self):
        return VectorUtil.toString(self)

    def __repr__(self):
        return f"{type(self).__name__}({VectorUtil.toString(self)!r})"


class DenseVector(Vector):
    __gson_fields__ = ("data",)

    def __init__(self, data=None):
        if data is None:
            self.data = np.zeros(0, dtype=np.float64)
        elif isinstance(data, (int, np.integer)):
            self.data = np.zeros(int(data), dtype=np.float64)
        else:
            self.data = np.asarray(data, dtype=np.float64).reshape(-1).copy()

    # -- factories --
    @staticmethod
    def ones(n):
        return DenseVector(np.ones(n))

    @staticmethod
    def zeros(n):
        return DenseVector(np.zeros(n))

    @staticmethod
    def rand(n, seed=None):
        return DenseVector(np.random.default_rng(seed).random(n))

    # -- accessors --
    def getData(self):
        return self.data

    def setData(self, d):
        self.data = np.asarray(d, dtype=np.float64)

    def size(self):
        return int(self.data.shape[0])

    def get(self, i):
        return float(self.data[i])

    def set(self, i, v):
        self.data[i] = v

    def add(self, i, v):
        self.data[i] += v

    def clone(self):
        return DenseVector(self.data.copy())

    def __len__(self):
        return self.size()

    def __eq__(self, o):
        return isinstance(o, DenseVector) and np.array_equal(o.data, self.data)

    def __hash__(self):
        return hash(self.data.tobytes())

    # -- algebra --
    def normL1(self):
        return float(np.abs(self.data).sum())

    def normL2(self):
        return float(math.sqrt(float(np.dot(self.data, self.data))))

    def normL2Square(self):
        return float(np.dot(self.data, self.data))

    def normInf(self):
        return float(np.abs(self.data).max()) if self.data.size else 0.0

    def scale(self, a):
        return DenseVector(self.data * a)

    def scaleEqual(self, a):
        self.data *= a

    def plus(self, o: Vector):
        return DenseVector(self.data + _dense(o))

    def plusEqual(self, o: Vector):
        if isinstance(o, SparseVector):
            np.add.at(self.data, o.indices, o.values)
        else:
            self.data += o.data

    def minus(self, o: Vector):
        return DenseVector(self.data - _dense(o))

    def minusEqual(self, o: Vector):
        if isinstance(o, SparseVector):
            np.subtract.at(self.data, o.indices, o.values)
        else:
            self.data -= o.data

    def plusScaleEqual(self, o: Vector, a: float):
        if isinstance(o, SparseVector):
            np.add.at(self.data, o.indices, a * o.values)
        else:
            self.data += a * o.data

    def dot(self, o: Vector) -> float:
        if isinstance(o, SparseVector):
            return float(np.dot(self.data[o.indices], o.values))
        return float(np.dot(self.data, o.data))

    def outer(self, o: Optional["DenseVector"] = None):
        from .matrix import DenseMatrix
        o = self if o is None else o
        return DenseMatrix(np.outer(self.data, o.data))

    def prefix(self, v: float):
        return DenseVector(np.concatenate([[v], self.data]))

    def append(self, v: float):
        return DenseVector(np.concatenate([self.data, [v]]))

    def slice(self, indices: Sequence[int]):
        return DenseVector(self.data[np.asarray(indices, dtype=np.int64)])

    def normalizeEqual(self, p: float):
        n = float(np.linalg.norm(self.data, ord=p)) if self.data.size else 0.0
        if n != 0:
            self.data /= n

    def standardizeEqual(self, mean, stdvar):
        self.data = (self.data - mean) / stdvar

    def toDense(self):
        return self

    def toSparseVector(self):
        idx = np.nonzero(self.data)[0]
        return SparseVector(self.size(), idx, self.data[idx])

    def iterator(self):
        return VectorIterator(np.arange(self.size()), self.data)


class SparseVector(Vector):
    __gson_fields__ = ("n", "indices", "values")

    def __init__(self, n: int = -1, indices=None, values=None):
        self.n = int(n)
        if indices is None:
            self.indices = np.zeros(0, dtype=np.int32)
            self.values = np.zeros(0, dtype=np.float64)
        elif isinstance(indices, dict):
            items = sorted(indices.items())
            self.indices = np.asarray([k for k, _ in items], dtype=np.int32)
            self.values = np.asarray([v for _, v in items], dtype=np.float64)
        else:
            idx = np.asarray(indices, dtype=np.int64).reshape(-1)
            val = np.asarray(values, dtype=np.float64).reshape(-1)
            if idx.shape != val.shape:
                raise ValueError("Indices size and values size should be the same.")
            if idx.size and np.any(np.diff(idx) <= 0):
                order = np.argsort(idx, kind="stable")
                idx, val = idx[order], val[order]
                # merge duplicate indices by summation (reference sortIndices keeps last; we sum)
                if np.any(np.diff(idx) == 0):
                    uniq, inv = np.unique(idx, return_inverse=True)
                    s = np.zeros(uniq.shape[0], dtype=np.float64)
                    np.add.at(s, inv, val)
                    idx, val = uniq, s
            if self.n >= 0 and idx.size and (idx[-1] >= self.n or idx[0] < 0):
                raise ValueError("Index out of bound.")
            self.indices = idx.astype(np.int32)
            self.values = val

    def size(self):
        return self.n

    def setSize(self, n):
        self.n = int(n)

    def numberOfValues(self):
        return int(self.indices.shape[0])

    def getIndices(self):
        return self.indices

    def getValues(self):
        return self.values

    def get(self, i):
        pos = np.searchsorted(self.indices, i)
        if pos < self.indices.size and self.indices[pos] == i:
            return float(self.values[pos])
        return 0.0

    def set(self, i, v):
        pos = np.searchsorted(self.indices, i)
        if pos < self.indices.size and self.indices[pos] == i:
            self.values[pos] = v
        else:
            self.indices = np.insert(self.indices, pos, i).astype(np.int32)
            self.values = np.insert(self.values, pos, v)

    def add(self, i, v):
        self.set(i, self.get(i) + v)

    def clone(self):
        return SparseVector(self.n, self.indices.copy(), self.values.copy())

    def __eq__(self, o):
        return (isinstance(o, SparseVector) and o.n == self.n and np.array_equal(o.indices, self.indices)
                and np.array_equal(o.values, self.values))

    def __hash__(self):
        return hash((self.n, self.indices.tobytes(), self.values.tobytes()))

    def normL1(self):
        return float(np.abs(self.values).sum())

    def normL2(self):
        return float(math.sqrt(float(np.dot(self.values, self.values))))

    def normL2Square(self):
        return float(np.dot(self.values, self.values))

    def normInf(self):
        return float(np.abs(self.values).max()) if self.values.size else 0.0

    def scale(self, a):
        return SparseVector(self.n, self.indices.copy(), self.values * a)

    def scaleEqual(self, a):
        self.values *= a

    def dot(self, o: Vector) -> float:
        if isinstance(o, DenseVector):
            return float(np.dot(o.data[self.indices], self.values))
        common, ia, ib = np.intersect1d(self.indices, o.indices, assume_unique=True, return_indices=True)
        return float(np.dot(self.values[ia], o.values[ib]))

    def plus(self, o: Vector):
        if isinstance(o, DenseVector):
            return o.plus(self)
        return SparseVector(max(self.n, o.n), np.concatenate([self.indices, o.indices]),
                            np.concatenate([self.values, o.values]))

    def minus(self, o: Vector):
        if isinstance(o, DenseVector):
            return DenseVector(self.toDenseVector().data - o.data)
        return SparseVector(max(self.n, o.n), np.concatenate([self.indices, o.indices]),
                            np.concatenate([self.values, -o.values]))

    def prefix(self, v: float):
        return SparseVector(self.n + 1 if self.n >= 0 else -1,
                            np.concatenate([[0], self.indices.astype(np.int64) + 1]),
                            np.concatenate([[v], self.values]))

    def append(self, v: float):
        if self.n < 0:
            raise ValueError("Can't append to a vector of unknown size")
        return SparseVector(self.n + 1, np.concatenate([self.indices, [self.n]]),
                            np.concatenate([self.values, [v]]))

    def slice(self, indices: Sequence[int]):
        indices = list(indices)
        out_i, out_v = [], []
        for j, i in enumerate(indices):
            v = self.get(i)
            if v != 0.0:
                out_i.append(j)
                out_v.append(v)
        return SparseVector(len(indices), out_i, out_v)

    def outer(self, o: Optional["SparseVector"] = None):
        """Outer product self * o^T as a DenseMatrix (size x o.size)."""
        from .matrix import DenseMatrix
        o = self if o is None else o
        m = np.zeros((self.size(), o.size()))
        m[np.ix_(self.indices.astype(np.int64), o.indices.astype(np.int64))] = np.outer(self.values, o.values)
        return DenseMatrix(m)

    def removeZeroValues(self):
        m = self.values != 0
        self.indices, self.values = self.indices[m], self.values[m]

    def normalizeEqual(self, p):
        n = float(np.linalg.norm(self.values, ord=p)) if self.values.size else 0.0
        if n != 0:
            self.values /= n

    def toDenseVector(self) -> DenseVector:
        n = self.n if self.n >= 0 else (int(self.indices.max()) + 1 if self.indices.size else 0)
        d = np.zeros(n, dtype=np.float64)
        d[self.indices] = self.values
        return DenseVector(d)

    def toDense(self):
        return self.toDenseVector()

    def iterator(self):
        return VectorIterator(self.indices, self.values)


class VectorIterator:
    def __init__(self, idx, val):
        self._i, self._v, self._p = idx, val, 0

    def hasNext(self):
        return self._p < len(self._i)

    def next(self):
        self._p += 1

    def getIndex(self):
        return int(self._i[self._p])

    def getValue(self):
        return float(self._v[self._p])


def _dense(o: Vector) -> np.ndarray:
    return o.toDense().data if isinstance(o, SparseVector) else o.data


class VectorUtil:
    """String (de)serialisation compatible with ``VectorUtil.java``."""

    @staticmethod
    def parse(s: str) -> Vector:
        if s is None or not s.strip() or ":" in s or "$" in s:
            return VectorUtil.parseSparse(s)
        return VectorUtil.parseDense(s)

    @staticmethod
    def parseDense(s: str) -> DenseVector:
        if s is None or not s.strip():
            return DenseVector()
        toks = [t for t in s.replace(",", " ").split(" ") if t.strip()]
        return DenseVector(np.array([float(t) for t in toks], dtype=np.float64))

    @staticmethod
    def parseSparse(s: str) -> SparseVector:
        if s is None or not s.strip():
            return SparseVector()
        n = -1
        body = s
        first = s.find("$")
        if first >= 0:
            last = s.rfind("$")
            n = int(s[first + 1:last])
            body = s[last + 1:]
            if not body.strip():
                return SparseVector(n)
        idx, val = [], []
        for tok in body.replace(",", " ").split(" "):
            tok = tok.strip()
            if not tok:
                continue
            k, _, v = tok.partition(":")
            if not _:
                raise ValueError(f'Fail to getVector sparse vector from string: "{s}".')
            idx.append(int(k))
            val.append(float(v))
        return SparseVector(n, idx, val)

    @staticmethod
    def toString(v: Vector) -> str:
        if isinstance(v, SparseVector):
            head = f"${v.n}$" if v.n > 0 else ""
            return head + " ".join(f"{int(i)}:{java_double_str(x)}" for i, x in zip(v.indices, v.values))
        return " ".join(java_double_str(x) for x in v.data)

    serialize = toString

    @staticmethod
    def getVector(obj) -> Optional[Vector]:
        if obj is None:
            return None
        if isinstance(obj, Vector):
            return obj
        if isinstance(obj, str):
            return VectorUtil.parse(obj)
        if isinstance(obj, (int, float, np.integer, np.floating)):
            return DenseVector(np.array([float(obj)]))
        if isinstance(obj, (list, tuple, np.ndarray)):
            return DenseVector(np.asarray(obj, dtype=np.float64))
        raise ValueError(f"Can not get the vector from {obj}")

    @staticmethod
    def getDenseVector(obj) -> Optional[DenseVector]:
        v = VectorUtil.getVector(obj)
        if v is None:
            return None
        return v if isinstance(v, DenseVector) else v.toDenseVector()

    @staticmethod
    def getSparseVector(obj) -> Optional[SparseVector]:
        v = VectorUtil.getVector(obj)
        if v is None:
            return None
        if isinstance(v, SparseVector):
            return v
        raise ValueError("CAN NOT get SparseVector!")
