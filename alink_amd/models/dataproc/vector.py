"""Vector mappers: VectorAssembler, VectorNormalize, VectorSlice, VectorElementwiseProduct, VectorInteraction,
VectorPolynomialExpand, VectorSizeHint, VectorToColumns, VectorSerialize.

Reference: ``A/operator/common/dataproc/vector/*Mapper.java``.  ``VectorAssemblerMapper.java:50-106``
assembles numbers/vectors/vector strings into a SparseVector that is densified when ``nnz * 1.5 > size``;
null inputs follow ``handleInvalid`` (ERROR raises, SKIP -> null output, otherwise ignored).
The batched path concatenates numeric / dense-block columns directly on the device (K24).
"""
from __future__ import annotations

import math
from typing import List

import numpy as np
import torch

from ...common.linalg import SparseBlock, DenseVector, SparseVector, Vector, VectorUtil
from ...common.mapper import Mapper, MISOMapper, OutputColsHelper, SISOMapper, find_col_index, find_col_indices
from ...common.table import Column, MTable
from ...common.types import Types, is_numeric

RATIO = 1.5


def _append(vec: Vector, items: dict, pos: int) -> int:
    if isinstance(vec, SparseVector):
        for i, v in zip(vec.indices, vec.values):
            items[pos + int(i)] = float(v)
        return pos + vec.size()
    for j in range(vec.size()):
        items[pos + j] = float(vec.data[j])
    return pos + vec.size()


class VectorAssemblerMapper(MISOMapper):
    def outputType(self):
        return Types.VECTOR

    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        hi = self.params.get("handleInvalid") if self.params.contains("handleInvalid") else \
            (self.params.get("handleInvalidMethod") if self.params.contains("handleInvalidMethod") else "ERROR")
        self.handle = str(hi).upper().split(".")[-1]

    def mapColumns(self, vals):
        pos = 0
        items = {}
        for col in vals:
            if col is None:
                if self.handle == "ERROR":
                    raise ValueError("null value is found in vector assembler inputs.")
                if self.handle == "SKIP":
                    return None
                continue
            if isinstance(col, bool):
                items[pos] = float(col)
                pos += 1
            elif isinstance(col, (int, float, np.integer, np.floating)):
                items[pos] = float(col)
                pos += 1
            elif isinstance(col, str):
                pos = _append(VectorUtil.getVector(col), items, pos)
            elif isinstance(col, Vector):
                pos = _append(col, items, pos)
            else:
                raise TypeError("not support type of object.")
        sv = SparseVector(pos, items)
        if len(items) * RATIO > pos:
            return sv.toDenseVector()
        return sv

    def _map_columns(self, mt: MTable):
        cols = [mt.cols[i] for i in self.col_idx]
        fast = all(isinstance(c.values, torch.Tensor) and c.nulls is None for c in cols)
        if fast and cols:
            dev = cols[0].values.device
            # a 1-D column is one value per row (explicit width: reshape(0, -1) of an empty column is ambiguous)
            parts = [c.values.to(dev).reshape(c.values.shape[0], int(np.prod(c.values.shape[1:], dtype=np.int64)))
                     for c in cols]
            dt = torch.float64
            if all(p.dtype in (torch.bfloat16,) for p in parts):
                dt = torch.bfloat16
            elif all(p.dtype in (torch.bfloat16, torch.float32, torch.float16) for p in parts):
                dt = torch.float32
            return [Column(torch.cat([p.to(dt) for p in parts], 1))]
        blocks = [_block_of(c) for c in cols]
        if cols and all(b is not None for b in blocks):
            # columnar path (K24): numeric / dense-vector / sparse / dense-vector-string columns, NULLs handled
            # per handleInvalid (KEEP with a NULL changes that row's vector size: per-row path below)
            anynull = None
            for _, m in blocks:
                if m is not None:
                    anynull = m if anynull is None else (anynull | m)
            blocks = [b for b, _ in blocks]
            if anynull is not None and bool(anynull.any()):
                if self.handle == "ERROR":
                    raise ValueError("null value is found in vector assembler inputs.")
                if self.handle != "SKIP":
                    return super()._map_columns(mt)
            else:
                anynull = None
            from ...ops.feature import vector_assemble
            sb, _ = vector_assemble(blocks, mt.num_rows, skip=anynull, dense_ratio=RATIO)
            return [Column(sb, anynull)]
        return super()._map_columns(mt)


def _block_of(c: Column):
    """(tensor / SparseBlock, null mask or None) of a column for the columnar assembler, or None (per-row
    path): numeric / dense-vector blocks as they are, dense-vector strings of one width parsed natively."""
    v = c.values
    if isinstance(v, (torch.Tensor, SparseBlock)):
        return v, (c.nulls.cpu() if c.nulls is not None else None)
    vals = c.to_list()
    if not vals or not all(isinstance(x, str) or x is None for x in vals):
        return None
    present = [x for x in vals if x is not None]
    if not present:
        return None
    toks = [len(x.replace(",", " ").split()) for x in present]
    d = toks[0]
    if d == 0 or any(t != d for t in toks) or any(x.lstrip().startswith("$") or ":" in x for x in present) \
            or not all(x.isascii() for x in present):
        return None
    from ... import _native
    arr = _native.parse_dense_vectors([x if x is not None else "" for x in vals], d)
    if arr is None:
        return None
    nulls = torch.tensor([x is None for x in vals], dtype=torch.bool)
    return torch.from_numpy(arr), (nulls if bool(nulls.any()) else None)


class VectorNormalizeMapper(SISOMapper):
    def outputType(self):
        return Types.VECTOR

    def mapColumn(self, v):
        if v is None:
            return None
        vec = VectorUtil.getVector(v).clone()
        vec.normalizeEqual(float(self.params.get("p")) if self.params.contains("p") else 2.0)
        return vec

    def _map_columns(self, mt):
        """A dense 2-D tensor column normalised at once, with ``np.linalg.norm``'s per-order reductions along each
        row (the row path's numbers to rounding: its 2-norm is a BLAS dot); other columns row by row."""
        v = mt.cols[self.col_idx].values
        if not (isinstance(v, torch.Tensor) and v.dim() == 2 and not v.is_complex()):
            return super()._map_columns(mt)
        p = float(self.params.get("p")) if self.params.contains("p") else 2.0
        if v.is_cuda and v.shape[1] and p in (1.0, 2.0, float("inf")):
            # on the device: the same orders through torch's row norms (to rounding), float64 like the row path
            X = v.detach().to(torch.float64)
            nrm = torch.linalg.vector_norm(X, ord=p, dim=1, keepdim=True)
            return [Column(torch.where(nrm != 0, X / torch.where(nrm != 0, nrm, torch.ones_like(nrm)), X))]
        X = v.detach().to("cpu", torch.float64).numpy().copy()
        if X.shape[1] == 0:
            return [Column(torch.from_numpy(X))]
        ax = np.abs(X)
        if p == np.inf:
            nrm = ax.max(1)
        elif p == -np.inf:
            nrm = ax.min(1)
        elif p == 0:
            nrm = (X != 0).sum(1).astype(np.float64)
        elif p == 1:
            nrm = np.add.reduce(ax, axis=1)
        elif p == 2:
            nrm = np.sqrt(np.add.reduce(X * X, axis=1))
        else:
            nrm = np.add.reduce(ax ** p, axis=1) ** (1.0 / p)
        nz = nrm != 0
        X[nz] /= nrm[nz, None]
        return [Column(torch.from_numpy(X))]


def _dense_col(mt, i):
    """The 2-D float tensor of a dense vector column (None for any other layout)."""
    v = mt.cols[i].values
    if isinstance(v, torch.Tensor) and v.dim() == 2 and v.is_floating_point():
        return v
    return None


class VectorSliceMapper(SISOMapper):
    def outputType(self):
        return Types.VECTOR

    def mapColumn(self, v):
        if v is None:
            return None
        return VectorUtil.getVector(v).slice(self.params.get("indices"))

    def _map_columns(self, mt):
        X = _dense_col(mt, self.col_idx)
        idx = [int(i) for i in self.params.get("indices")]
        if X is None or any(i < -X.shape[1] or i >= X.shape[1] for i in idx):
            return super()._map_columns(mt)
        return [Column(X.to(torch.float64)[:, torch.as_tensor(idx, dtype=torch.int64, device=X.device)])]


class VectorElementwiseProductMapper(SISOMapper):
    def outputType(self):
        return Types.VECTOR

    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        self.scale = VectorUtil.getVector(self.params.get("scalingVector"))

    def mapColumn(self, v):
        if v is None:
            return None
        vec = VectorUtil.getVector(v)
        s = self.scale.toDense().data
        if isinstance(vec, SparseVector):
            return SparseVector(vec.n, vec.indices.copy(), vec.values * s[vec.indices])
        return DenseVector(vec.data * s[:vec.size()])

    def _map_columns(self, mt):
        X = _dense_col(mt, self.col_idx)
        s = self.scale.toDense().data
        if X is None or s.size < X.shape[1]:
            return super()._map_columns(mt)
        return [Column(X.to(torch.float64) * torch.as_tensor(s[:X.shape[1]], dtype=torch.float64,
                                                             device=X.device)[None, :])]


class VectorInteractionMapper(MISOMapper):
    def outputType(self):
        return Types.VECTOR

    def mapColumns(self, vals):
        """Reference ``VectorInteractionMapper``: dense x dense -> entry i * |b| + j = a_i b_j; sparse x sparse ->
        entry |a| * j + i (the reference's sparse layout); a dense / sparse mix is an error."""
        if len(vals) != 2:
            raise ValueError("VectorInteraction only support two input columns.")
        if any(v is None for v in vals):
            return None
        a, b = VectorUtil.getVector(vals[0]), VectorUtil.getVector(vals[1])
        if isinstance(a, SparseVector) != isinstance(b, SparseVector):
            raise ValueError("Make sure the two input vectors are both dense or sparse.")
        if isinstance(a, SparseVector):
            idx = (a.size() * b.indices.astype(np.int64)[None, :] + a.indices.astype(np.int64)[:, None]).reshape(-1)
            val = np.outer(a.values, b.values).reshape(-1)
            return SparseVector(a.size() * b.size(), idx, val)
        return DenseVector(np.outer(a.data, b.data).reshape(-1))

    def _map_columns(self, mt):
        if len(self.col_idx) != 2:
            return super()._map_columns(mt)
        A, B = _dense_col(mt, self.col_idx[0]), _dense_col(mt, self.col_idx[1])
        if A is None or B is None or A.device != B.device:
            return super()._map_columns(mt)
        A, B = A.to(torch.float64), B.to(torch.float64)
        return [Column((A[:, :, None] * B[:, None, :]).reshape(A.shape[0], -1))]


def poly_size(num_features: int, degree: int) -> int:
    """Number of monomials of total degree <= ``degree`` in ``num_features`` variables, constant included
    (reference ``PolynomialExpansionMapper.getPolySize``)."""
    return math.comb(num_features + degree, degree)


def _expand_dense(vals, last, degree, mult, out, cur):
    # monomial order of the reference (Spark's): recursion over the last feature's power, lower features first
    if mult == 0.0:
        pass
    elif degree == 0 or last < 0:
        if cur >= 0:
            out[cur] = mult
    else:
        v, alpha, start, i = vals[last], mult, cur, 0
        while i <= degree and alpha != 0.0:
            start = _expand_dense(vals, last - 1, degree - i, alpha, out, start)
            i += 1
            alpha *= v
    return cur + poly_size(last + 1, degree)


def _poly_terms(d: int, degree: int):
    """(output position, exponent per feature) of every monomial ``_expand_dense`` writes, in its order."""
    terms = []

    def rec(last, deg, exps, cur):
        if deg == 0 or last < 0:
            if cur >= 0:
                terms.append((cur, tuple(exps)))
        else:
            start = cur
            for i in range(deg + 1):
                e = list(exps)
                e[last] = i
                start = rec(last - 1, deg - i, e, start)
        return cur + poly_size(last + 1, deg)

    rec(d - 1, degree, [0] * d, -1)
    return terms


def _expand_sparse(idx, vals, last, last_feature, degree, mult, out_i, out_v, cur):
    if mult == 0.0:
        pass
    elif degree == 0 or last < 0:
        if cur >= 0:
            out_i.append(cur)
            out_v.append(mult)
    else:
        v, alpha, start, i = vals[last], mult, cur, 0
        last_feature1 = int(idx[last]) - 1
        while i <= degree and alpha != 0.0:
            start = _expand_sparse(idx, vals, last - 1, last_feature1, degree - i, alpha, out_i, out_v, start)
            i += 1
            alpha *= v
    return cur + poly_size(last_feature + 1, degree)


class VectorPolynomialExpandMapper(SISOMapper):
    """All monomials of degree 1..``degree`` (reference ``PolynomialExpansionMapper.java``): dense in, dense out;
    sparse in, sparse out over the stored entries; size ``poly_size(n, degree) - 1``."""

    def outputType(self):
        return Types.VECTOR

    def mapColumn(self, v):
        if v is None:
            return None
        vec = VectorUtil.getVector(v)
        degree = int(self.params.get("degree")) if self.params.contains("degree") else 2
        if isinstance(vec, SparseVector):
            out_i, out_v = [], []
            _expand_sparse(vec.indices, vec.values, len(vec.indices) - 1, vec.size() - 1, degree, 1.0, out_i, out_v,
                           -1)
            return SparseVector(poly_size(vec.size(), degree) - 1, out_i, out_v)
        x = vec.data
        out = np.zeros(poly_size(len(x), degree) - 1)
        _expand_dense(x, len(x) - 1, degree, 1.0, out, -1)
        return DenseVector(out)

    def _map_columns(self, mt):
        """Dense tensor columns at once: each output position's monomial multiplied up in the row path's order
        (last feature first, one factor at a time from 1.0), a product that reached zero on the way kept at
        +0.0 as the recursion stops there -- the row path's values bit for bit."""
        X = _dense_col(mt, self.col_idx)
        degree = int(self.params.get("degree")) if self.params.contains("degree") else 2
        if X is None or poly_size(X.shape[1], degree) > 1 << 16:
            return super()._map_columns(mt)
        X = X.to(torch.float64)
        n, d = X.shape
        out = torch.zeros((n, poly_size(d, degree) - 1), dtype=torch.float64, device=X.device)
        for pos, exps in _poly_terms(d, degree):
            acc = torch.ones(n, dtype=torch.float64, device=X.device)
            dead = torch.zeros(n, dtype=torch.bool, device=X.device)
            for k in range(d - 1, -1, -1):
                for _ in range(exps[k]):
                    acc = acc * X[:, k]
                    dead |= acc == 0
            out[:, pos] = torch.where(dead, torch.zeros_like(acc), acc)
        return [Column(out)]


class VectorSizeHintMapper(SISOMapper):
    def outputType(self):
        return Types.VECTOR

    def mapColumn(self, v):
        if v is None:
            hi = str(self.params.get("handleInvalid")).upper() if self.params.contains("handleInvalid") else "ERROR"
            if "ERROR" in hi:
                raise ValueError("Got null vector in VectorSizeHint")
            return None
        vec = VectorUtil.getVector(v)
        size = self.params.get("size")
        if vec.size() != size:
            hi = str(self.params.get("handleInvalid")).upper() if self.params.contains("handleInvalid") else "ERROR"
            if "ERROR" in hi:
                raise ValueError(f"VectorSizeHint: expect size {size}, got {vec.size()}")
            return None
        return vec

    def _map_columns(self, mt):
        X = _dense_col(mt, self.col_idx)
        if X is None or X.shape[1] != self.params.get("size"):
            return super()._map_columns(mt)
        return [Column(X)]                   # every row already has the hinted size: passed through


class VectorSerializeMapper(Mapper):
    """Vector columns -> their string form (used before CSV/model export)."""

    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        from ...common.types import is_vector, TableSchema
        self.vidx = [i for i, t in enumerate(dataSchema.types) if is_vector(t)]
        names = [dataSchema.names[i] for i in self.vidx]
        self.helper = OutputColsHelper(dataSchema, names, [Types.STRING] * len(names))

    def _map_row_values(self, row):
        return [None if row[i] is None else (VectorUtil.toString(row[i]) if isinstance(row[i], Vector)
                                             else str(row[i])) for i in self.vidx]

    def _map_columns(self, mt):
        """Dense 2-D tensor vector columns formatted by the C++ Double.toString rows (packed); other vector
        columns value by value."""
        from ... import _native
        from ...common.strings import StringBlock
        out = []
        for i in self.vidx:
            X = _dense_col(mt, i)
            r = _native.java_double_rows_packed(X.detach().to("cpu", torch.float64).numpy(), " ") \
                if X is not None and mt.num_rows and X.shape[1] else None
            if r is not None:
                out.append(Column(StringBlock(torch.from_numpy(np.ascontiguousarray(r[0])), torch.from_numpy(r[1]))))
                continue
            vals = mt.cols[i].to_list()
            out.append(Column([None if v is None else (VectorUtil.toString(v) if isinstance(v, Vector) else str(v))
                               for v in vals]))
        return out


class VectorToColumnsMapper(Mapper):
    """``VectorToColumnsMapper`` (``outputCols``) or, when ``schemaStr`` is given instead, the format
    version ``dataproc/format/VectorToColumnsBatchOp`` (``FormatTransMapper`` VECTOR -> COLUMNS)."""

    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        p = self.params
        self._delegate = None
        if not (p.contains("outputCols") and p.get("outputCols")) and p.contains("schemaStr") and p.get("schemaStr"):
            from .format import FormatTransMapper
            q = p.clone()
            q.set("fromFormat", "VECTOR")
            q.set("toFormat", "COLUMNS")
            if not (q.contains("vectorCol") and q.get("vectorCol")):
                q.set("vectorCol", p.get("selectedCol"))
            self._delegate = FormatTransMapper(dataSchema, q)
            self.helper = self._delegate.helper
            return
        self.idx = find_col_index(dataSchema.names, p.get("selectedCol"))
        self.outs = p.get("outputCols")
        reserved = p.get("reservedCols") if p.contains("reservedCols") else None
        self.helper = OutputColsHelper(dataSchema, self.outs, [Types.DOUBLE] * len(self.outs), reserved)

    def _map_row_values(self, row):
        if self._delegate is not None:
            return self._delegate._map_row_values(row)
        v = row[self.idx]
        if v is None:
            return [None] * len(self.outs)
        vec = VectorUtil.getVector(v)
        return [vec.get(i) for i in range(len(self.outs))]

    def _map_columns(self, mt):
        """Whole columns: the format flavour through the format mapper's columnar paths (it was reached only row
        by row -- a Double.toString and a parse per value); the ``outputCols`` flavour slices a dense [n, d] tensor
        column (more output columns than components, or null cells: the row path, which raises as ``Vector.get``
        on the former)."""
        if self._delegate is not None:
            return self._delegate._map_columns(mt)
        c = mt.cols[self.idx]
        v = c.values
        if isinstance(v, torch.Tensor) and v.dim() == 2 and len(self.outs) <= v.shape[1] and \
                (c.nulls is None or not bool(c.nulls.any())):
            V = v.to(torch.float64)
            return [Column(V[:, i].contiguous()) for i in range(len(self.outs))]
        return super()._map_columns(mt)
