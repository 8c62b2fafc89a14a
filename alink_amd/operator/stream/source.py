"""Stream sources: a bounded table replayed as micro-batches.

Reference: ``A/operator/stream/source/{CsvSourceStreamOp,MemSourceStreamOp,NumSeqSourceStreamOp,
TableSourceStreamOp,TextSourceStreamOp,LibSvmSourceStreamOp,RandomTableSourceStreamOp}.java`` (Flink
``DataStream`` sources).  Each source reads/generates its rank's row block with the batch reader of the same
name (same Params) and yields it in fixed-size micro-batches (``ALINK_STREAM_BATCH`` rows, default 1024), so
a GPU-resident pipeline processes one device block per micro-batch.
"""
from __future__ import annotations

import os
from typing import Iterator, Optional

import torch

from ...common.params import Params
from ...common.strings import StringBlock
from ...common.table import Column, MTable
from ..batch import source as B
from .base import StreamSourceOp

__all__ = ["TableSourceStreamOp", "MemSourceStreamOp", "CsvSourceStreamOp", "TextSourceStreamOp",
           "LibSvmSourceStreamOp", "NumSeqSourceStreamOp", "RandomTableSourceStreamOp",
           "RandomVectorSourceStreamOp"]


def _batch_rows() -> int:
    return int(os.environ.get("ALINK_STREAM_BATCH", "1024"))


class _TableReplaySource(StreamSourceOp):
    BATCH_OP = None

    def _table(self) -> MTable:
        op = self.BATCH_OP(params=self.getParams().clone())
        op.setMLEnvironmentId(self.getMLEnvironmentId())
        return op.getOutputTable()

    def _ensure_schema(self):
        if self._schema is None:
            self._mt = self._table()
            self._schema = self._mt.schema
        return self._schema

    def getSchema(self):
        return self._ensure_schema()

    def batches(self) -> Iterator[MTable]:
        self._ensure_schema()
        mt = self._mt
        bs = max(1, _batch_rows())
        bounds = list(range(0, mt.num_rows, bs)) + [mt.num_rows]
        # byte offsets of every micro-batch boundary of every string column, read once for the whole stream
        # (slicing a device string block otherwise costs one device-to-host copy per column per micro-batch)
        byte_bounds = {}
        for ci, c in enumerate(mt.cols):
            if isinstance(c.values, StringBlock):
                off = c.values.offsets
                byte_bounds[ci] = off[torch.as_tensor(bounds, device=off.device)].tolist()
        sidx = sorted(byte_bounds)
        for i in range(len(bounds) - 1):
            a, b = bounds[i], bounds[i + 1]
            # every string column's rebased offsets in one multi-tensor launch (torch._foreach_sub) instead of
            # one subtraction kernel per column per micro-batch
            offs = torch._foreach_sub([mt.cols[ci].values.offsets[a:b + 1] for ci in sidx],
                                      [byte_bounds[ci][i] for ci in sidx]) if sidx else []
            rebased = dict(zip(sidx, offs))
            cols = []
            for ci, c in enumerate(mt.cols):
                if ci in rebased:
                    blk = c.values
                    cols.append(Column(StringBlock(blk.data[byte_bounds[ci][i]:byte_bounds[ci][i + 1]], rebased[ci],
                                                   None if blk.nulls is None else blk.nulls[a:b])))
                else:
                    cols.append(c.take(slice(a, b)))
            yield MTable(mt.schema, cols, mt.replicated)


class TableSourceStreamOp(_TableReplaySource):
    _NO_AUTO_PARAMS = True

    def __init__(self, table=None, params: Optional[Params] = None):
        super().__init__(params)
        self._src = table

    def _table(self):
        t = self._src
        return t.getOutputTable() if hasattr(t, "getOutputTable") else t


class MemSourceStreamOp(_TableReplaySource):
    def __init__(self, vals=None, schema=None, params: Optional[Params] = None):
        super().__init__(params)
        self._vals, self._sch = vals, schema

    def _table(self):
        return B.MemSourceBatchOp(self._vals, self._sch).setMLEnvironmentId(self.getMLEnvironmentId()) \
            .getOutputTable()

    @staticmethod
    def fromDataframe(df, schemaStr: Optional[str] = None):
        op = MemSourceStreamOp()
        op._table = lambda: B.MemSourceBatchOp.fromDataframe(df, schemaStr).getOutputTable()
        return op


class CsvSourceStreamOp(_TableReplaySource):
    BATCH_OP = B.CsvSourceBatchOp

    def __init__(self, filePath: Optional[str] = None, schemaStr: Optional[str] = None,
                 params: Optional[Params] = None):
        super().__init__(params)
        if filePath is not None:
            self.setFilePath(filePath)
        if schemaStr is not None:
            self.setSchemaStr(schemaStr)


class TextSourceStreamOp(_TableReplaySource):
    BATCH_OP = B.TextSourceBatchOp


class LibSvmSourceStreamOp(_TableReplaySource):
    BATCH_OP = B.LibSvmSourceBatchOp


class NumSeqSourceStreamOp(_TableReplaySource):
    def __init__(self, start: int = 1, end: Optional[int] = None, colName: str = "num",
                 params: Optional[Params] = None):
        super().__init__(params)
        self._args = (start, end, colName)

    def _table(self):
        s, e, c = self._args
        return B.NumSeqSourceBatchOp(s, e, c).setMLEnvironmentId(self.getMLEnvironmentId()).getOutputTable()


class RandomTableSourceStreamOp(_TableReplaySource):
    BATCH_OP = B.RandomTableSourceBatchOp
    EXTRA_PARAMS = list(B.RandomTableSourceBatchOp.PARAMS)


class RandomVectorSourceStreamOp(_TableReplaySource):
    BATCH_OP = B.RandomVectorSourceBatchOp
    EXTRA_PARAMS = list(B.RandomVectorSourceBatchOp.PARAMS)
