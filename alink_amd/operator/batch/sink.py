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
        if mt.replicated and comm.get_rank() != 0:
            rows = []
        else:
            rows = mt.rows()
        quote = self.getParams().get(self._param_infos["quoteChar"])
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
