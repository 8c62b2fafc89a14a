"""Columnar table (``MTable``) — the unit of data flowing between operators.

Replaces Flink's ``Table``/``DataSet<Row>`` (reference ``A/common/utils/DataSetConversionUtil.java``).
Each rank of an SPMD job holds one *partition* of a table (contiguous block of the global row order),
or — for small tables such as models — a full *replicated* copy.

Columns are stored natively:
  * numeric/boolean -> 1-D ``torch.Tensor`` (+ optional bool null mask), on CPU or the rank's GPU;
  * dense-vector block -> 2-D ``torch.Tensor`` ``[n, d]`` (bf16/fp32/fp64), e.g. GPU-resident features;
  * strings -> Python ``list``, or a packed ``StringBlock`` (UTF-8 bytes + offsets tensors, host or device:
    what shuffles, key hashing and the feature hasher move and read in bulk);
  * everything else (mixed vectors, objects) -> Python ``list`` (``None`` = SQL NULL).
Row-level access (``rows()``/``collect()``) materialises Python values (``DenseVector`` for vector blocks).
"""
from __future__ import annotations

from typing import Any, Iterable, List, Optional, Sequence, Union

import numpy as np
import torch

from .linalg import DenseVector, SparseBlock, SparseVector, Vector, VectorUtil
from .strings import StringBlock
from .detail import DetailBlock
from .types import TableSchema, Types, AlinkType, is_numeric, schema_str_to_schema

__all__ = ["Row", "Column", "MTable", "LazyRows", "infer_type"]


class Row(tuple):
    """Immutable row (Flink ``Row`` analogue)."""

    @staticmethod
    def of(*vals):
        return Row(vals)

    def getField(self, i):
        return self[i]

    def getArity(self):
        return len(self)

    def __repr__(self):
        return "Row(" + ", ".join(repr(v) for v in self) + ")"


def infer_type(v) -> AlinkType:
    if isinstance(v, (bool, np.bool_)):
        return Types.BOOLEAN
    if isinstance(v, (int, np.integer)):
        return Types.LONG
    if isinstance(v, (float, np.floating)):
        return Types.DOUBLE
    if isinstance(v, str):
        return Types.STRING
    if isinstance(v, DenseVector):
        return Types.DENSE_VECTOR
    if isinstance(v, SparseVector):
        return Types.SPARSE_VECTOR
    if isinstance(v, Vector):
        return Types.VECTOR
    if isinstance(v, (bytes, bytearray)):
        return Types.VARBINARY
    return Types.OBJECT


class Column:
    __slots__ = ("values", "nulls")

    def __init__(self, values, nulls: Optional[torch.Tensor] = None):
        self.values = values
        self.nulls = nulls

    # -- constructors --
    @staticmethod
    def from_values(vals: Sequence[Any], t: AlinkType) -> "Column":
        if isinstance(vals, torch.Tensor):
            return Column(vals)
        if isinstance(vals, np.ndarray) and vals.dtype != object and is_numeric_or_bool(t):
            return Column(torch.from_numpy(np.ascontiguousarray(vals)).to(t.torch_dtype))
        vals = list(vals)
        if is_numeric_or_bool(t):
            nulls = [v is None or (isinstance(v, float) and v != v and t not in (Types.DOUBLE, Types.FLOAT))
                     for v in vals]
            has_null = any(v is None for v in vals)
            fill = [0 if v is None else v for v in vals]
            try:
                arr = torch.tensor(fill, dtype=t.torch_dtype)
            except (TypeError, ValueError, RuntimeError):
                arr = torch.tensor([_to_num(v, t) for v in fill], dtype=t.torch_dtype)
            return Column(arr, torch.tensor([v is None for v in vals], dtype=torch.bool) if has_null else None)
        return Column(vals)

    def is_tensor(self):
        return isinstance(self.values, torch.Tensor)

    def __len__(self):
        if isinstance(self.values, torch.Tensor):
            return int(self.values.shape[0])
        return len(self.values)

    def to_list(self) -> List[Any]:
        v = self.values
        if isinstance(v, (StringBlock, DetailBlock)):
            return v.to_list()
        if isinstance(v, SparseBlock):
            lst = v.to_list()
            if self.nulls is not None:
                lst = [None if m else x for x, m in zip(lst, self.nulls.cpu().tolist())]
            return lst
        if isinstance(v, torch.Tensor):
            if v.dim() == 2:
                arr = v.detach().to("cpu", torch.float64).numpy()
                return [DenseVector(r) for r in arr]
            lst = v.detach().cpu().tolist()
            if self.nulls is not None:
                nm = self.nulls.cpu().tolist()
                lst = [None if m else x for x, m in zip(lst, nm)]
            return lst
        return list(v)

    def take(self, idx) -> "Column":
        """Row selection by index tensor/list or boolean mask."""
        v = self.values
        if isinstance(v, (StringBlock, DetailBlock)):
            return Column(v.take(idx))
        if isinstance(v, SparseBlock):
            nn = None
            if self.nulls is not None:
                nn = Column(self.nulls.cpu()).take(idx).values
            return Column(v.take(idx), nn)
        if isinstance(v, torch.Tensor):
            if isinstance(idx, torch.Tensor):
                ii = idx.to(v.device)
            else:
                ii = torch.as_tensor(np.asarray(idx, dtype=np.int64) if not isinstance(idx, slice) else idx, device=v.device) \
                    if not isinstance(idx, slice) else idx
            nv = v[ii]
            nn = None
            if self.nulls is not None:
                nn = self.nulls[ii.to(self.nulls.device) if isinstance(ii, torch.Tensor) else ii]
            return Column(nv, nn)
        if isinstance(idx, slice):
            return Column(v[idx])
        if isinstance(idx, torch.Tensor):
            if idx.dtype == torch.bool:
                idx = torch.nonzero(idx.cpu(), as_tuple=False).reshape(-1)
            idx = idx.cpu().tolist()
        elif isinstance(idx, np.ndarray) and idx.dtype == bool:
            idx = np.nonzero(idx)[0].tolist()
        return Column([v[i] for i in idx])

    @staticmethod
    def concat(cols: List["Column"]) -> "Column":
        if not cols:
            return Column([])
        if all(isinstance(c.values, StringBlock) for c in cols):
            return Column(StringBlock.concat([c.values for c in cols]))
        if all(isinstance(c.values, DetailBlock) for c in cols):
            blk = DetailBlock.concat([c.values for c in cols])
            if blk is not None:
                return Column(blk)
        if all(isinstance(c.values, SparseBlock) for c in cols):
            nulls = None
            if any(c.nulls is not None for c in cols):
                nulls = torch.cat([c.nulls.cpu() if c.nulls is not None else torch.zeros(len(c), dtype=torch.bool)
                                   for c in cols])
            return Column(SparseBlock.concat([c.values for c in cols]), nulls)
        if all(isinstance(c.values, torch.Tensor) for c in cols) and len({c.values.dim() for c in cols}) == 1:
            dev = cols[0].values.device
            vals = torch.cat([c.values.to(dev) for c in cols])
            nulls = None
            if any(c.nulls is not None for c in cols):
                nulls = torch.cat([c.nulls.cpu() if c.nulls is not None else torch.zeros(len(c), dtype=torch.bool)
                                   for c in cols]).to(dev)
            return Column(vals, nulls)
        out = []
        for c in cols:
            out.extend(c.to_list())
        return Column(out)


def is_numeric_or_bool(t: AlinkType) -> bool:
    return is_numeric(t) or t == Types.BOOLEAN


def _to_num(v, t):
    if t == Types.BOOLEAN:
        return bool(v)
    if t in (Types.FLOAT, Types.DOUBLE, Types.DECIMAL):
        return float(v)
    return int(v)


class MTable:
    """A (partition of a) table: schema + columns."""

    def __init__(self, schema: TableSchema, cols: List[Column], replicated: bool = False):
        self.schema = schema
        self.cols = cols
        self.replicated = replicated
        n = {len(c) for c in cols}
        if len(n) > 1:
            raise ValueError(f"column lengths differ: {[len(c) for c in cols]}")

    # -- construction --
    @staticmethod
    def from_rows(rows: Iterable[Sequence[Any]], schema: Union[TableSchema, str, Sequence[str]],
                  replicated: bool = False) -> "MTable":
        rows = [tuple(r) for r in rows]
        if isinstance(schema, str):
            schema = schema_str_to_schema(schema)
        elif not isinstance(schema, TableSchema):
            names = list(schema)
            types = []
            for j in range(len(names)):
                t = Types.STRING
                for r in rows:
                    if r[j] is not None:
                        t = infer_type(r[j])
                        break
                types.append(t)
            schema = TableSchema(names, types)
        ncol = len(schema.names)
        cols = []
        for j in range(ncol):
            vals = [r[j] if j < len(r) else None for r in rows]
            cols.append(Column.from_values(vals, schema.types[j]))
        return MTable(schema, cols, replicated)

    @staticmethod
    def from_columns(names: Sequence[str], types: Sequence[AlinkType], values: Sequence[Any],
                     replicated: bool = False) -> "MTable":
        cols = [v if isinstance(v, Column) else Column.from_values(v, t) for v, t in zip(values, types)]
        return MTable(TableSchema(names, types), cols, replicated)

    @staticmethod
    def empty(schema: TableSchema, replicated=False) -> "MTable":
        return MTable(schema, [Column.from_values([], t) for t in schema.types], replicated)

    # -- info --
    @property
    def num_rows(self) -> int:
        return len(self.cols[0]) if self.cols else 0

    def __len__(self):
        return self.num_rows

    def getColNames(self):
        return list(self.schema.names)

    def getColTypes(self):
        return list(self.schema.types)

    def col_index(self, name: str) -> int:
        try:
            return self.schema.names.index(name)
        except ValueError:
            lower = [n.lower() for n in self.schema.names]
            if name.lower() in lower:
                return lower.index(name.lower())
            raise ValueError(f"Can not find column: {name}, all columns: {self.schema.names}")

    def col(self, name: str) -> Column:
        return self.cols[self.col_index(name)]

    def col_type(self, name: str) -> AlinkType:
        return self.schema.types[self.col_index(name)]

    def column_values(self, name: str) -> List[Any]:
        return self.col(name).to_list()

    # -- row access --
    def lazy_rows(self) -> "LazyRows":
        """The rows as a sequence that builds ``Row`` objects only when indexed / iterated; readers that know it
        (the model-table loaders, ``common/model/converter.py``) take its columns directly."""
        return LazyRows(self)

    def rows(self) -> List[Row]:
        if not self.cols:
            return []
        lists = [c.to_list() for c in self.cols]
        return [Row(vals) for vals in zip(*lists)]

    def row(self, i: int) -> Row:
        return Row(tuple(c.take([i]).to_list()[0] for c in self.cols))

    # -- transforms --
    def select(self, names: Sequence[str]) -> "MTable":
        idx = [self.col_index(n) for n in names]
        return MTable(TableSchema([self.schema.names[i] for i in idx], [self.schema.types[i] for i in idx]),
                      [self.cols[i] for i in idx], self.replicated)

    def take(self, idx) -> "MTable":
        return MTable(self.schema, [c.take(idx) for c in self.cols], self.replicated)

    def slice(self, start: int, end: int) -> "MTable":
        return MTable(self.schema, [c.take(slice(start, end)) for c in self.cols], self.replicated)

    def with_columns(self, names, types, cols) -> "MTable":
        """Append or replace columns."""
        names_out = list(self.schema.names)
        types_out = list(self.schema.types)
        cols_out = list(self.cols)
        for n, t, c in zip(names, types, cols):
            c = c if isinstance(c, Column) else Column.from_values(c, t)
            if n in names_out:
                i = names_out.index(n)
                types_out[i], cols_out[i] = t, c
            else:
                names_out.append(n)
                types_out.append(t)
                cols_out.append(c)
        return MTable(TableSchema(names_out, types_out), cols_out, self.replicated)

    def rename(self, names: Sequence[str]) -> "MTable":
        return MTable(TableSchema(list(names), list(self.schema.types)), self.cols, self.replicated)

    @staticmethod
    def concat(tables: List["MTable"]) -> "MTable":
        tables = [t for t in tables if t is not None]
        if not tables:
            raise ValueError("no tables")
        schema = tables[0].schema
        cols = [Column.concat([t.cols[j] for t in tables]) for j in range(len(schema.names))]
        return MTable(schema, cols, tables[0].replicated)

    # -- vector helpers --
    def vector_block(self, name: str, dtype=torch.float64, device=None, size: Optional[int] = None) -> torch.Tensor:
        """Dense ``[n, d]`` tensor view of a vector (or numeric) column."""
        c = self.col(name)
        v = c.values
        if isinstance(v, torch.Tensor):
            t = v if v.dim() == 2 else v.reshape(-1, 1)
            return t.to(device=device or t.device, dtype=dtype)
        vecs = [VectorUtil.getVector(x) for x in v]
        d = size if size is not None else max((x.size() if x.size() >= 0 else
                                               (int(x.indices.max()) + 1 if len(x.indices) else 0))
                                              for x in vecs if x is not None) if vecs else 0
        out = np.zeros((len(vecs), d), dtype=np.float64)
        for i, x in enumerate(vecs):
            if x is None:
                continue
            if isinstance(x, SparseVector):
                out[i, x.indices] = x.values
            else:
                out[i, :x.size()] = x.data[:d]
        return torch.from_numpy(out).to(device=device or "cpu", dtype=dtype)

    def to_pandas(self):
        import pandas as pd
        return pd.DataFrame({n: c.to_list() for n, c in zip(self.schema.names, self.cols)},
                            columns=self.schema.names)

    def __repr__(self):
        return f"MTable({self.num_rows} rows, {self.schema.to_str()})"


class LazyRows(Sequence):
    """Rows of an ``MTable`` on demand: ``len`` / indexing / iteration behave like the list ``MTable.rows()``
    returns, while ``column(j)`` (python values) and ``int_column(j)`` (int64 numpy, no NULLs) hand a columnar
    reader the data without materialising one ``Row`` per record — a 255k-row tree model table loads in
    milliseconds instead of about a second."""

    def __init__(self, mt: "MTable"):
        self._cols = list(mt.cols)
        self._n = mt.num_rows if mt.cols else 0
        self._lists: dict = {}

    def column(self, j: int) -> List[Any]:
        if j not in self._lists:
            self._lists[j] = self._cols[j].to_list()
        return self._lists[j]

    def int_column(self, j: int) -> Optional[np.ndarray]:
        """int64 array of column j, or None when it is not an integer tensor without NULLs."""
        c = self._cols[j]
        v = c.values
        if isinstance(v, torch.Tensor) and v.dim() == 1 and c.nulls is None and not v.is_floating_point():
            return v.detach().cpu().numpy().astype(np.int64, copy=False)
        vals = self.column(j)
        if any(x is None for x in vals):
            return None
        return np.asarray(vals, dtype=np.int64)

    @property
    def width(self) -> int:
        return len(self._cols)

    def __len__(self) -> int:
        return self._n

    def _row(self, i: int) -> Row:
        return Row(tuple(self.column(j)[i] for j in range(len(self._cols))))

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self._row(k) for k in range(*i.indices(self._n))]
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        return self._row(i)

    def __iter__(self):
        if not self._cols:
            return iter(())
        return (Row(vals) for vals in zip(*[self.column(j) for j in range(len(self._cols))]))

    def __eq__(self, other):
        return list(self) == list(other)
