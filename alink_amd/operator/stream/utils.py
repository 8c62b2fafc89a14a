"""Stream utility ops: Print / Collect sinks (reference ``A/operator/stream/utils/PrintStreamOp.java``)."""
from __future__ import annotations

import sys
from typing import List, Optional

from ...common.params import Params
from ...common.table import MTable, Row
from ..base import format_title, _fmt_val
from .base import StreamOperator, _engine

__all__ = ["PrintStreamOp", "CollectStreamOp", "StreamSinkOp"]


class StreamSinkOp(StreamOperator):
    @staticmethod
    def of(params):
        """Re-create the registered stream sink named by ``params`` (ioName / ioType)."""
        from ...common.io_registry import AnnotationUtils, IOType
        return AnnotationUtils.of(params, IOType.SinkStream)

    def linkFrom(self, *inputs):
        (inp,) = self._connect(*inputs)
        self._schema = inp.getSchema()
        _engine(self.env).register_sink(self)
        return self


class PrintStreamOp(StreamSinkOp):
    PARAMS = ()

    def linkFrom(self, *inputs):
        super().linkFrom(*inputs)
        if self.env.rank == 0:
            print(format_title(self._schema.names))
        return self

    def on_batch(self, port, mt: MTable):
        if self.env.rank == 0:
            for r in mt.rows():
                print("|".join(_fmt_val(v) for v in r))
            sys.stdout.flush()


class CollectStreamOp(StreamSinkOp):
    """Collects every emitted row into a user-supplied list (test / notebook helper)."""
    PARAMS = ()

    def __init__(self, box: Optional[List[Row]] = None, params: Optional[Params] = None):
        super().__init__(params)
        self.box = box if box is not None else []

    def on_batch(self, port, mt: MTable):
        self.box.extend(mt.rows())
