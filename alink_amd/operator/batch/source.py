"""Batch sources.

Reference: ``A/operator/batch/source/*`` — ``BaseSourceBatchOp`` builds its output lazily on first
``getOutputTable`` (``BaseSourceBatchOp.java:50-55``), ``CsvSourceBatchOp.java:76-116``,
``MemSourceBatchOp``, ``NumSeqSourceBatchOp``, ``TableSourceBatchOp``, ``TextSourceBatchOp``,
``LibSvmSourceBatchOp`` (1-based libsvm indices -> 0-based sparse vectors).

SPMD partitioning: each rank keeps a contiguous block of the global row order, so gathering partitions
in rank order reproduces the source order.  Synthetic sources (``RandomVectorSourceBatchOp``,
``RandomTableSourceBatchOp``) generate each rank's block directly on the rank's device — the path used
for the 1e8-row benchmark tables.
"""
from __future__ import annotations

import io
import os
import urllib.request
from typing import Any, List, Optional, Sequence

import numpy as np
import torch

from ...common.linalg import SparseVector, VectorUtil
from ...common.params import ParamInfo, Params
from ...common.table import Column, MTable, Row
from ...common.types import TableSchema, Types, schema_str_to_schema
from ...parallel import comm
from ..base import BatchOperator, partition_bounds, partition_rows
from ..common.io.csv import CsvParser

__all__ = ["BaseSourceBatchOp", "MemSourceBatchOp", "TableSourceBatchOp", "CsvSourceBatchOp",
           "TextSourceBatchOp", "LibSvmSourceBatchOp", "NumSeqSourceBatchOp", "RandomVectorSourceBatchOp",
           "RandomTableSourceBatchOp", "DataSetWrapperBatchOp", "read_text", "parse_libsvm_line"]


def read_text(path: str) -> str:
    if path.startswith(("http://", "https://")):
        with urllib.request.urlopen(path) as f:  # no egress in the sandbox; kept for parity
            return f.read().decode("utf-8")
    if path.startswith("file://"):
        path = path[len("file://"):]
    with open(path, "r", encoding="utf-8", newline="") as f:
        return f.read()


def read_text_range(path: str, row_delim: str, rank: int, world: int, raw: bool = False):
    """(text of the lines whose first byte lies in this rank's byte range, whether the range holds the file's
    first line) for a local file on a multi-rank job; None when a whole-file read applies (one rank, URLs)."""
    if world <= 1 or path.startswith(("http://", "https://")):
        return None
    if path.startswith("file://"):
        path = path[len("file://"):]
    if not os.path.isfile(path):
        return None
    size = os.path.getsize(path)
    lo, hi = size * rank // world, size * (rank + 1) // world
    d = row_delim.encode("utf-8")
    with open(path, "rb") as f:
        if lo > 0:
            # a line belongs to the range holding its first byte: skip the tail of the previous range's line
            f.seek(lo - len(d) if lo >= len(d) else 0)
            head = f.read(len(d)) if lo >= len(d) else b""
            start = lo
            if head != d:
                f.seek(lo)
                buf = b""
                while True:
                    chunk = f.read(1 << 16)
                    if not chunk:
                        start = size
                        break
                    buf += chunk
                    k = buf.find(d)
                    if k >= 0:
                        start = lo + k + len(d)
                        break
            lo = start
        if lo >= hi:
            return (b"" if raw else ""), rank == 0
        f.seek(lo)
        data = f.read(hi - lo)
        if not data.endswith(d):
            rest = b""
            while True:
                chunk = f.read(1 << 16)
                if not chunk:
                    break
                k = chunk.find(d)
                if k >= 0:
                    rest += chunk[:k + len(d)]
                    break
                rest += chunk
            data += rest
    return (data if raw else data.decode("utf-8")), lo == 0


class BaseSourceBatchOp(BatchOperator):
    @staticmethod
    def of(params):
        """Re-create the registered IO operator named by ``params`` (ioName / ioType, reference ``of(params)``)."""
        from ...common.io_registry import AnnotationUtils, IOType
        return AnnotationUtils.of(params, IOType.SourceBatch)

    _NO_AUTO_PARAMS = False

    def getOutputTable(self) -> MTable:
        if self._output is None:
            self._output = self.initializeDataSource()
        return self._output

    def initializeDataSource(self) -> MTable:
        raise NotImplementedError

    def linkFrom(self, *inputs):
        raise RuntimeError("Source operator does not support linkFrom()")


class TableSourceBatchOp(BaseSourceBatchOp):
    PARAMS = ()

    def __init__(self, table: MTable = None, params: Optional[Params] = None):
        super().__init__(params)
        if table is not None and not isinstance(table, MTable):
            raise TypeError("TableSourceBatchOp expects an MTable")
        self._table = table

    def initializeDataSource(self):
        return self._table


DataSetWrapperBatchOp = TableSourceBatchOp


class MemSourceBatchOp(BaseSourceBatchOp):
    """Rows held in client memory.  Accepted forms (as the Java constructors):
    ``(vals, colName)`` 1-column, ``(rows, colNames)``, ``(rows, TableSchema|schemaStr)``."""
    PARAMS = ()

    def __init__(self, vals=None, schema=None, params: Optional[Params] = None):
        super().__init__(params)
        self._vals = vals
        self._schema = schema

    @staticmethod
    def fromDataframe(df, schemaStr: Optional[str] = None):
        rows = [tuple(None if (isinstance(v, float) and v != v and not isinstance(v, bool)) else
                      (v.item() if hasattr(v, "item") else v) for v in r)
                for r in df.itertuples(index=False, name=None)]
        schema = schemaStr if schemaStr is not None else list(df.columns)
        return MemSourceBatchOp(rows, schema)

    def initializeDataSource(self):
        vals, schema = self._vals, self._schema
        if vals is None:
            raise ValueError("MemSourceBatchOp needs data")
        if hasattr(vals, "itertuples"):
            return MemSourceBatchOp.fromDataframe(vals, schema).getOutputTable()
        if isinstance(schema, str) and "," not in schema and len(schema.split()) == 1:
            rows = [(v,) for v in vals]
            schema = [schema]
        else:
            rows = [tuple(r) if isinstance(r, (list, tuple, Row)) else (r,) for r in vals]
        if isinstance(schema, str):
            schema = schema_str_to_schema(schema)
        rows = partition_rows(rows, self.env)
        if not isinstance(schema, TableSchema):
            # infer types from the full data (every rank sees the same client data)
            full = [tuple(r) if isinstance(r, (list, tuple, Row)) else (r,) for r in vals] \
                if not (isinstance(self._schema, str) and len(self._schema.split()) == 1) else [(v,) for v in vals]
            schema = MTable.from_rows(full[:1000], schema).schema if full else TableSchema(list(schema),
                                                                                         [Types.STRING] * len(schema))
        return MTable.from_rows(rows, schema)


class NumSeqSourceBatchOp(BaseSourceBatchOp):
    PARAMS = ()

    def __init__(self, start: int = 1, end: Optional[int] = None, colName: str = "num",
                 params: Optional[Params] = None):
        super().__init__(params)
        if end is None:
            start, end = 1, start
        self._range = (int(start), int(end))
        self._col = colName

    def initializeDataSource(self):
        a, b = self._range
        n = max(0, b - a + 1)
        lo, hi = partition_bounds(n, self.env)
        return MTable.from_columns([self._col], [Types.LONG], [torch.arange(a + lo, a + hi, dtype=torch.int64)])


class CsvSourceBatchOp(BaseSourceBatchOp):
    def __init__(self, filePath: Optional[str] = None, schemaStr: Optional[str] = None,
                 params: Optional[Params] = None, **kw):
        if isinstance(filePath, Params):
            filePath, params = None, filePath
        super().__init__(params, **kw)
        if filePath is not None:
            self.setFilePath(filePath)
        if schemaStr is not None:
            self.setSchemaStr(schemaStr)

    def initializeDataSource(self):
        schema = schema_str_to_schema(self.getSchemaStr())
        row_delim = self.getRowDelimiter() or "\n"
        path = self.getFilePath()
        quote = self.getParams().get(self._param_infos["quoteChar"])
        delim = self.getFieldDelimiter()
        skip_blank = self.getSkipBlankLine()
        mt = _csv_bytes_table(path, schema, row_delim, delim, quote, skip_blank, self.getIgnoreFirstLine()) \
            if self.env.world_size == comm.get_world_size() else None
        if mt is not None:
            return mt
        ranged = read_text_range(path, row_delim, comm.get_rank(), comm.get_world_size())
        if ranged is not None:
            # byte-range split (CsvSourceBatchOp.java:76-116 / Flink input splits): this rank reads only the
            # lines that start inside its byte range; partitions stay contiguous in file order
            text, first = ranged
        else:
            text, first = read_text(path), True
        lines = text.split(row_delim)
        if lines and lines[-1] == "":
            lines.pop()
        lines = [l[:-1] if l.endswith("\r") and row_delim == "\n" else l for l in lines]
        if self.getIgnoreFirstLine() and lines and first:
            lines = lines[1:]
        if ranged is None:
            lines = partition_rows(lines, self.env)
        mt = _native_parse_csv(lines, schema, delim, quote, skip_blank)
        if mt is not None:
            return mt
        parser = CsvParser(schema.types, delim, quote)
        rows = []
        for line in lines:
            if not line:
                if not skip_blank:
                    rows.append([None] * len(schema.types))
                continue
            ok, r = parser.parse(line)
            if not ok:
                raise RuntimeError(f'Fail to parse line "{line}"')
            rows.append(r)
        return MTable.from_rows(rows, schema)


def _csv_codes(schema):
    codes = []
    for t in schema.types:
        if t in (Types.DOUBLE, Types.FLOAT, Types.DECIMAL):
            codes.append(1)
        elif t in (Types.LONG, Types.INT, Types.SHORT, Types.BYTE):
            codes.append(2)
        elif t == Types.BOOLEAN:
            codes.append(3)
        elif t == Types.STRING:
            codes.append(0)
        else:
            return None
    return codes


def _csv_table(schema, res) -> MTable:
    from ...common.strings import StringBlock
    cols = []
    for t, (vals, nulls) in zip(schema.types, res):
        if isinstance(vals, tuple):
            b, o, nm = vals
            cols.append(Column(StringBlock(torch.from_numpy(b), torch.from_numpy(o),
                                           torch.from_numpy(nm) if nm.any() else None)))
        elif isinstance(vals, list):
            cols.append(Column(vals))
        else:
            tt = torch.from_numpy(vals).to(t.torch_dtype)
            nm = torch.from_numpy(nulls) if nulls is not None and nulls.any() else None
            cols.append(Column(tt, nm))
    return MTable(schema, cols)


def _csv_bytes_table(path, schema, row_delim, delim, quote, skip_blank, ignore_first) -> Optional[MTable]:
    """The CSV source without Python strings: the file (or this rank's byte range) read as bytes, lines found
    with numpy on a one-byte row delimiter, fields parsed in C++ straight from the file buffer
    (``alink_csv_parse_spans``), string columns left packed as ``StringBlock``s.  None (the line path) for
    URLs, multi-byte delimiters, or a single rank of a multi-rank job reading a non-file."""
    from ... import _native
    if _native.lib is None or getattr(_native.lib, "alink_csv_parse_spans", None) is None:
        return None
    d = row_delim.encode("utf-8")
    if len(d) != 1 or len(delim) != 1 or (quote is not None and len(quote) != 1) or \
            path.startswith(("http://", "https://")):
        return None
    codes = _csv_codes(schema)
    if codes is None:
        return None
    fpath = path[len("file://"):] if path.startswith("file://") else path
    if not os.path.isfile(fpath):
        return None
    ws = comm.get_world_size()
    if ws > 1:
        ranged = read_text_range(path, row_delim, comm.get_rank(), ws, raw=True)
        if ranged is None:
            return None
        raw, first = ranged
    else:
        with open(fpath, "rb") as f:
            raw = f.read()
        first = True
    buf = np.frombuffer(raw, dtype=np.uint8)
    ends = np.flatnonzero(buf == d[0])
    starts = np.empty(ends.size + 1, dtype=np.int64)
    starts[0] = 0
    starts[1:] = ends + 1
    ends = np.append(ends, buf.size).astype(np.int64)
    if starts[-1] == buf.size:           # text ending in the delimiter: no trailing empty line
        starts, ends = starts[:-1], ends[:-1]
    if row_delim == "\n" and ends.size:
        cr = (ends > starts) & (buf[np.maximum(ends - 1, 0)] == 13)
        ends = ends - cr
    if ignore_first and first and starts.size:
        starts, ends = starts[1:], ends[1:]
    if skip_blank:
        keep = ends > starts
        if not keep.all():
            starts, ends = starts[keep], ends[keep]
    try:
        res = _native.parse_csv_spans(buf, starts, ends, codes, delim, quote or "", blocks=True)
    except _native._CsvLineError as e:
        line = buf[starts[e.line]:ends[e.line]].tobytes().decode("utf-8", "replace")
        raise RuntimeError(f'Fail to parse line "{line}"') from None
    return None if res is None else _csv_table(schema, res)


def _native_parse_csv(lines, schema, delim, quote, skip_blank) -> Optional[MTable]:
    """Bulk path through the native C++ parser (numeric columns straight into arrays)."""
    try:
        from ... import _native
    except Exception:
        return None
    if _native.lib is None or len(delim) != 1 or (quote is not None and len(quote) != 1):
        return None
    codes = _csv_codes(schema)
    if codes is None:
        return None
    res = _native.parse_csv_lines(lines, codes, delim, quote or "", skip_blank)
    return None if res is None else _csv_table(schema, res)


class TextSourceBatchOp(BaseSourceBatchOp):
    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(params, **kw)

    def initializeDataSource(self):
        text = read_text(self.getFilePath())
        lines = text.split("\n")
        if lines and lines[-1] == "":
            lines.pop()
        if self.getIgnoreFirstLine() and lines:
            lines = lines[1:]
        lines = partition_rows(lines, self.env)
        return MTable.from_columns([self.getTextCol()], [Types.STRING], [lines])


def parse_libsvm_line(line: str):
    if line is None or not line.strip():
        return None, None
    sp = line.find(" ")
    if sp < 0:
        return float(line), VectorUtil.getVector("")
    label = float(line[:sp])
    vec = VectorUtil.getVector(line[sp + 1:])
    if isinstance(vec, SparseVector):
        vec = SparseVector(vec.n, vec.indices.astype(np.int64) - 1, vec.values)
    return label, vec


class LibSvmSourceBatchOp(BaseSourceBatchOp):
    def __init__(self, filePath: Optional[str] = None, params: Optional[Params] = None, **kw):
        super().__init__(params, **kw)
        if filePath is not None:
            self.setFilePath(filePath)

    def initializeDataSource(self):
        lines = [l for l in read_text(self.getFilePath()).split("\n")]
        if lines and lines[-1] == "":
            lines.pop()
        lines = partition_rows(lines, self.env)
        rows = [parse_libsvm_line(l) for l in lines]
        return MTable.from_rows(rows, TableSchema(["label", "features"], [Types.DOUBLE, Types.VECTOR]))


class RandomVectorSourceBatchOp(BaseSourceBatchOp):
    """Synthetic dense-vector table generated on the rank's device (no data files needed).

    With ``numClusters > 0`` rows are drawn from an isotropic Gaussian mixture (the KMeans benchmark
    data); otherwise i.i.d. uniform [0, 1).  ``dtype`` may be ``bf16``/``fp32``/``fp64``.  The global table
    is the concatenation of rank blocks and is identical for any world size (per-block seeding).
    """
    PARAMS = [
        ParamInfo("numRows", int, "number of rows (global)", optional=False),
        ParamInfo("size", int, "vector size", optional=False),
        ParamInfo("idCol", str, "id column name", default=None),
        ParamInfo("outputCol", str, "vector column name", default="vec"),
        ParamInfo("numClusters", int, "mixture components (0 = uniform)", default=0),
        ParamInfo("clusterStd", float, "per-dim std of each component", default=1.0),
        ParamInfo("centerScale", float, "std of the component centres", default=10.0),
        ParamInfo("dtype", str, "bf16 | fp32 | fp64", default="fp64"),
        ParamInfo("seed", int, "random seed", default=0),
        ParamInfo("labelCol", str, "optional true-component column", default=None),
    ]

    BLOCK = 1 << 22

    def initializeDataSource(self):
        n, d = self.getNumRows(), self.getSize()
        k = self.getNumClusters()
        dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64}[self.getDtype().lower()]
        dev = self.env.device
        lo, hi = partition_bounds(n, self.env)
        seed = self.getSeed()
        g = torch.Generator(device="cpu").manual_seed(seed)
        centers = torch.randn(max(k, 1), d, generator=g, dtype=torch.float64) * self.getCenterScale()
        centers = centers.to(dev)
        out = torch.empty((hi - lo, d), dtype=dt, device=dev)
        labels = torch.empty(hi - lo, dtype=torch.int64, device=dev) if self.getLabelCol() else None
        # generate in fixed global blocks so content is independent of the partitioning
        b0 = lo // self.BLOCK
        for b in range(b0, (hi + self.BLOCK - 1) // self.BLOCK if hi > lo else b0):
            s, e = b * self.BLOCK, min(n, (b + 1) * self.BLOCK)
            gb = torch.Generator(device=dev).manual_seed(seed * 1000003 + b + 1)
            if k > 0:
                lab = torch.randint(0, k, (e - s,), generator=gb, device=dev)
                blk = torch.randn((e - s, d), generator=gb, device=dev, dtype=torch.float32) * self.getClusterStd()
                blk = blk + centers[lab].to(torch.float32)
            else:
                lab = None
                blk = torch.rand((e - s, d), generator=gb, device=dev, dtype=torch.float32)
            cs, ce = max(s, lo), min(e, hi)
            out[cs - lo:ce - lo] = blk[cs - s:ce - s].to(dt)
            if labels is not None and lab is not None:
                labels[cs - lo:ce - lo] = lab[cs - s:ce - s]
        names, types, vals = [], [], []
        if self.getIdCol():
            names.append(self.getIdCol())
            types.append(Types.LONG)
            vals.append(torch.arange(lo, hi, dtype=torch.int64))
        names.append(self.getOutputCol())
        types.append(Types.DENSE_VECTOR)
        vals.append(Column(out))
        if labels is not None:
            names.append(self.getLabelCol())
            types.append(Types.LONG)
            vals.append(Column(labels))
        return MTable.from_columns(names, types, vals)


class RandomTableSourceBatchOp(BaseSourceBatchOp):
    """Synthetic numeric table: ``numCols`` double columns ``col0..`` uniform [0,1) (+ optional id)."""
    PARAMS = [
        ParamInfo("numRows", int, "number of rows", optional=False),
        ParamInfo("numCols", int, "number of columns", optional=False),
        ParamInfo("idCol", str, "id column", default=None),
        ParamInfo("seed", int, "seed", default=0),
    ]

    def initializeDataSource(self):
        n, m = self.getNumRows(), self.getNumCols()
        lo, hi = partition_bounds(n, self.env)
        g = torch.Generator().manual_seed(self.getSeed())
        full = torch.rand((n, m), generator=g, dtype=torch.float64)[lo:hi]
        names = ([self.getIdCol()] if self.getIdCol() else []) + [f"col{i}" for i in range(m)]
        types = ([Types.LONG] if self.getIdCol() else []) + [Types.DOUBLE] * m
        vals = ([torch.arange(lo, hi)] if self.getIdCol() else []) + [full[:, j].clone() for j in range(m)]
        return MTable.from_columns(names, types, vals)
