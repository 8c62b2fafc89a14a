"""Batch sinks (reference ``A/operator/batch/sink/*``): CSV, Text, LibSvm.

Every rank formats its partition; rank 0 writes the file (``numFiles == 1``) after gathering, or each rank
writes ``<path>/part-<rank>`` when ``numFiles > 1`` (the Flink "directory of parts" layout).
"""
from __future__ import annotations

import os
from typing import Optional

from ...common.javafmt import java_double_str, java_str
from ...common.linalg import SparseVector, Vector, VectorUtil
from ...common.params import Params
from ...common.types import Types
from ...parallel import comm
from ..base import BatchOperator, gather_table
from ..common.io.csv import CsvFormatter

__all__ = ["BaseSinkBatchOp", "CsvSinkBatchOp", "TextSinkBatchOp", "LibSvmSinkBatchOp", "write_lines"]


def write_lines(path: str, lines, overwrite: bool, num_files: int = 1, row_delim: str = "\n"):
    if path.startswith("file://"):
        path = path[len("file://"):]
    if num_files > 1:
        os.makedirs(path, exist_ok=True)
        fn = os.path.join(path, f"part-{comm.get_rank()}")
        with open(fn, "w", encoding="utf-8") as f:
            for l in lines:
                f.write(l + row_delim)
        return
    all_lines = lines
    if comm.get_world_size() > 1:
        parts = comm.all_gather_object(list(lines))
        all_lines = [l for p in parts for l in p]
    if comm.get_rank() == 0:
        if os.path.exists(path) and not overwrite:
            raise IOError(f"File {path} exists and overwriteSink is false")
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        with open(path, "w", encoding="utf-8") as f:
            for l in all_lines:
                f.write(l + row_delim)
    comm.barrier()


def _write_bytes(path: str, data, overwrite: bool, num_files: int = 1):
    """``write_lines`` for one rank's already assembled UTF-8 bytes (lines and row delimiters included)."""
    if path.startswith("file://"):
        path = path[len("file://"):]
    if num_files > 1:
        os.makedirs(path, exist_ok=True)
        path = os.path.join(path, f"part-{comm.get_rank()}")
    elif os.path.exists(path) and not overwrite:
        raise IOError(f"File {path} exists and overwriteSink is false")
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as f:
        f.write(memoryview(data))


def _csv_bytes(mt, delim: str, quote, rowdelim: str):
    """The CSV file of a table as bytes, column-wise: numeric tensor columns through the C++ Double.toString /
    numpy formatting, packed string columns as their bytes (None -- the row path -- when a string needs quotes),
    other columns through ``CsvFormatter`` one value at a time; lines joined in C++
    (``_native.join_packed_columns``).  Same text as the row path (tests/test_csv.py)."""
    import numpy as np
    import torch
    from ... import _native
    from ...common.strings import StringBlock
    if _native.lib is None or not delim:
        return None
    fmt = CsvFormatter(mt.schema.types, delim, quote)
    q = fmt.quote
    n = mt.num_rows
    packed = []
    for j, t in enumerate(mt.schema.types):
        c = mt.cols[j]
        v = c.values
        nm = c.nulls.cpu().numpy() if c.nulls is not None else None
        if isinstance(v, torch.Tensor) and v.dim() in (1, 2) and t != Types.STRING and v.is_floating_point():
            if v.dim() == 2 and (" " in delim or (q and " " in q)):
                return None
            x = v.detach().cpu().to(torch.float64).numpy()
            r = _native.java_double_rows_packed(x.reshape(n, -1), " ")
            if r is None:
                return None
            b, o = r
            if v.dim() == 2:
                nm = None                              # to_list() keeps every row of a 2-D column
        elif isinstance(v, torch.Tensor) and v.dim() == 1 and t != Types.STRING and not v.is_complex():
            vals = v.detach().cpu().tolist()
            strs = ["true" if e else "false" for e in vals] if v.dtype == torch.bool else list(map(str, vals))
            b, o = _native._pack_utf8(strs)
            b = np.frombuffer(b, dtype=np.uint8)
        elif isinstance(v, StringBlock):
            b, o = v.data.cpu().numpy(), v.offsets.cpu().numpy()
            nm = v.nulls.cpu().numpy() if v.nulls is not None else None   # to_list() reads the block's own nulls
            if q is not None:
                lens = o[1:] - o[:-1]
                live = ~nm if nm is not None else np.ones(n, dtype=bool)
                if bool(((lens == 0) & live).any()):
                    return None                       # "" is quoted on the row path
                if len(delim.encode()) != 1 or len(q.encode()) != 1:
                    return None
                if bool(((b == delim.encode()[0]) | (b == q.encode()[0])).any()):
                    return None
        else:
            strs = [fmt._fmt(e, t) for e in c.to_list()]
            b, o = _native._pack_utf8(strs)
            b = np.frombuffer(b, dtype=np.uint8)
            nm = None                                  # _fmt already wrote "" for None
        if nm is not None and nm.any():               # null cells print as ""
            lens = (o[1:] - o[:-1]).copy()
            lens[nm] = 0
            keep = np.repeat(~nm, o[1:] - o[:-1])
            b = b[keep]
            o = np.zeros(n + 1, dtype=np.int64)
            np.cumsum(lens, out=o[1:])
        packed.append((np.asarray(b, dtype=np.uint8), np.asarray(o, dtype=np.int64)))
    return _native.join_packed_columns(packed, delim, rowdelim)


class BaseSinkBatchOp(BatchOperator):
    @staticmethod
    def of(params):
        """Re-create the registered IO operator named by ``params`` (ioName / ioType, reference ``of(params)``)."""
        from ...common.io_registry import AnnotationUtils, IOType
        return AnnotationUtils.of(params, IOType.SinkBatch)

    def linkFrom(self, *inputs):
        inp = self.checkAndGetFirst(inputs)
        self.sinkFrom(inp)
        self.setOutputTable(inp.getOutputTable())
        return self

    def sinkFrom(self, inp):
        raise NotImplementedError


class CsvSinkBatchOp(BaseSinkBatchOp):
    def __init__(self, filePath: Optional[str] = None, params: Optional[Params] = None, **kw):
        if isinstance(filePath, Params):
            filePath, params = None, filePath
        super().__init__(params, **kw)
        if filePath is not None:
            self.setFilePath(filePath)

    def sinkFrom(self, inp):
        mt = inp.getOutputTable()
        quote = self.getParams().get(self._param_infos["quoteChar"])
        if comm.get_world_size() == 1 and mt.num_rows > 0:
            data = _csv_bytes(mt, self.getFieldDelimiter(), quote, self.getRowDelimiter() or "\n")
            if data is not None:
                _write_bytes(self.getFilePath(), data, self.getOverwriteSink(), self.getNumFiles())
                return
        if mt.replicated and comm.get_rank() != 0:
            rows = []
        else:
            rows = mt.rows()
        fmt = CsvFormatter(mt.schema.types, self.getFieldDelimiter(), quote)
        lines = [fmt.format([VectorUtil.toString(v) if isinstance(v, Vector) else v for v in r]) for r in rows]
        write_lines(self.getFilePath(), lines, self.getOverwriteSink(), self.getNumFiles(),
                    self.getRowDelimiter() or "\n")


class TextSinkBatchOp(BaseSinkBatchOp):
    def sinkFrom(self, inp):
        mt = inp.getOutputTable()
        if len(mt.schema.names) != 1 or mt.schema.types[0] != Types.STRING:
            raise ValueError("TextSinkBatchOp requires a single string column")
        rows = [] if (mt.replicated and comm.get_rank() != 0) else mt.rows()
        write_lines(self.getFilePath(), [("" if r[0] is None else r[0]) for r in rows], self.getOverwriteSink(),
                    self.getNumFiles())


class LibSvmSinkBatchOp(BaseSinkBatchOp):
    def sinkFrom(self, inp):
        mt = inp.getOutputTable()
        rows = [] if (mt.replicated and comm.get_rank() != 0) else mt.rows()
        li = mt.col_index(self.getLabelCol())
        vi = mt.col_index(self.getVectorCol())
        lines = []
        for r in rows:
            v = VectorUtil.getVector(r[vi])
            if isinstance(v, SparseVector):
                body = " ".join(f"{int(i) + 1}:{java_double_str(float(x))}" for i, x in zip(v.indices, v.values))
            else:
                body = " ".join(f"{i + 1}:{java_double_str(float(x))}" for i, x in enumerate(v.data))
            lab = java_str(r[li])
            lines.append(f"{lab} {body}".rstrip())
        write_lines(self.getFilePath(), lines, self.getOverwriteSink())
