"""Streaming evaluation (reference ``A/operator/stream/evaluation/{EvalBinaryClassStreamOp,EvalMultiClassStreamOp}``,
``BaseEvalClassStreamOp.java:44-90``): for every window (= micro-batch here) two rows are emitted —
``("window", metrics of the window)`` and ``("all", metrics of everything seen so far)`` — in the schema
``(Statistics STRING, Data STRING)``.  The cumulative summary is kept as merged histograms/matrices."""
from __future__ import annotations

import numpy as np

from ...common.detail import DetailBlock
from ...common.table import MTable
from ...common.types import TableSchema, Types
from ...models.evaluation import metrics as M
from .base import StreamOperator

__all__ = ["EvalBinaryClassStreamOp", "EvalMultiClassStreamOp"]

_SCHEMA = TableSchema(["Statistics", "Data"], [Types.STRING, Types.STRING])


def _pget(p, name):
    try:
        return p.get(name) if p.contains(name) else None
    except KeyError:
        return None


class _EvalStream(StreamOperator):
    BINARY = False

    def linkFrom(self, *inputs):
        self._connect(*inputs)
        self._schema = _SCHEMA
        self._acc = None
        self._labels = None
        return self

    def _summary(self, mt):
        p = self.getParams()
        labels = mt.column_values(p.get("labelCol"))
        det_col = _pget(p, "predictionDetailCol")
        pred_col = _pget(p, "predictionCol")
        if det_col:
            dcol = mt.col(det_col)
            if self.BINARY and isinstance(dcol.values, DetailBlock) and len(dcol.values.labels) == 2:
                fast = self._binary_columnar(mt.col(p.get("labelCol")), dcol.values, p)
                if fast is not None:
                    return fast
            dets = mt.column_values(det_col)
            if self._labels is None:
                # the label index is fixed by the first window (its labels and detail keys)
                keys = set()
                for l, d in zip(labels, dets):
                    if l is not None and d is not None:
                        keys.update(M.parse_detail(d).keys())
                        keys.add(str(l))
                self._labels = M.build_label_index(keys, self.BINARY, _pget(p, "positiveLabelValueString"))
            if self.BINARY:
                return ("b",) + M.binary_summary(labels, dets, self._labels)
            return ("m",) + M.multi_summary_from_detail(labels, dets, self._labels)
        preds = mt.column_values(pred_col)
        if self._labels is None:
            self._labels = M.build_label_index({str(x) for x in labels + preds if x is not None}, self.BINARY,
                                               _pget(p, "positiveLabelValueString"))
        return ("m",) + M.multi_summary_from_pred(labels, preds, self._labels)

    def _binary_columnar(self, lcol, blk, p):
        """Binary summary straight from a ``DetailBlock`` (no detail strings; ``metrics.binary_summary_block``)."""
        if self._labels is None:
            self._labels = M.build_label_index(M.detail_block_keys(lcol, blk), True,
                                               _pget(p, "positiveLabelValueString"))
        res = M.binary_summary_block(lcol, blk, self._labels)
        return None if res is None else ("b",) + res

    @staticmethod
    def _metrics(s, labels):
        if s[0] == "b":
            return M.binary_metrics(s[1], s[2], labels, s[3], s[4])
        return M.multi_metrics(s[1], labels, s[2], s[3])

    @staticmethod
    def _merge(a, b):
        if a is None:
            return b
        if a[0] == "b":
            return ("b", a[1] + b[1], a[2] + b[2], a[3] + b[3], a[4] + b[4])
        ll = a[2] + b[2] if a[2] >= 0 and b[2] >= 0 else -1.0
        return ("m", a[1] + b[1], ll, a[3] + b[3])

    def on_batch(self, port, mt):
        if mt.num_rows == 0:
            return
        s = self._summary(mt)
        if s[-1] == 0:
            return
        self._acc = self._merge(self._acc, s)
        rows = [("window", self._metrics(s, self._labels).serialize()[0]),
                ("all", self._metrics(self._acc, self._labels).serialize()[0])]
        self._emit(MTable.from_rows(rows, _SCHEMA))


class EvalBinaryClassStreamOp(_EvalStream):
    BINARY = True


class EvalMultiClassStreamOp(_EvalStream):
    pass
