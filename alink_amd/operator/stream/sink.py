"""Stream sinks (reference ``A/operator/stream/sink/{CsvSinkStreamOp,TextSinkStreamOp,LibSvmSinkStreamOp}.java``):
rows of every micro-batch are buffered and written through the batch writer when the stream ends."""
from __future__ import annotations

from typing import List, Optional

from ...common.params import Params
from ...common.table import MTable
from ..batch import sink as BS
from ..batch.source import TableSourceBatchOp
from .utils import StreamSinkOp

__all__ = ["CsvSinkStreamOp", "TextSinkStreamOp", "LibSvmSinkStreamOp"]


class _BufferedSink(StreamSinkOp):
    BATCH_SINK = None

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(params, **kw)
        self._parts: List[MTable] = []

    def on_batch(self, port, mt):
        self._parts.append(mt)

    def _close(self):
        mt = MTable.concat(self._parts) if self._parts else MTable.empty(self._schema)
        mt.replicated = False
        self.BATCH_SINK(self.getParams().clone()).linkFrom(TableSourceBatchOp(mt))
        self._parts = []


class CsvSinkStreamOp(_BufferedSink):
    BATCH_SINK = BS.CsvSinkBatchOp

    def __init__(self, filePath: Optional[str] = None, params: Optional[Params] = None, **kw):
        if isinstance(filePath, Params):
            filePath, params = None, filePath
        super().__init__(params, **kw)
        if filePath is not None:
            self.setFilePath(filePath)


class TextSinkStreamOp(_BufferedSink):
    BATCH_SINK = BS.TextSinkBatchOp


class LibSvmSinkStreamOp(_BufferedSink):
    BATCH_SINK = BS.LibSvmSinkBatchOp
