"""Streaming evaluation (reference ``A/operator/stream/evaluation/{EvalBinaryClassStreamOp,EvalMultiClassStreamOp}``,
``operator/common/evaluation/BaseEvalClassStreamOp.java:44-90``): processing-time windows of ``timeInterval``
seconds (default 3, ``timeWindowAll`` in the reference).  Every micro-batch is reduced to a summary (binned
positive / negative counts, or a confusion matrix) and merged into the open window; when the window has been open
``timeInterval`` seconds — on any rank, agreed over the host group — two rows are emitted: ``("window", metrics of
the window)`` and ``("all", metrics of everything seen so far)``, in the schema ``(Statistics STRING, Data
STRING)``.  The open window is flushed when the stream ends.  ``timeInterval`` 0 emits after every micro-batch."""
from __future__ import annotations

import time

import numpy as np
import torch

from ...common.detail import DetailBlock
from ...common.table import MTable
from ...common.types import TableSchema, Types
from ...models.evaluation import metrics as M
from ...parallel import comm
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
        self._win = None
        self._win_t0 = None
        self._labels = None
        return self

    def _agree_labels(self, keys, p) -> bool:
        """Fix the label index from this micro-batch's label keys (the union over the ranks under a process
        group, so every rank indexes the same labels).  False while no rank has seen an effective row yet."""
        if comm.is_distributed():
            keys = set().union(*[set(part) for part in comm.all_gather_object(sorted(keys))])
        if not keys:
            return False
        self._labels = M.build_label_index(keys, self.BINARY, _pget(p, "positiveLabelValueString"))
        return True

    def _summary(self, mt):
        """This micro-batch's summary over all ranks, or None while no label index exists.  Every collective in
        here runs on every rank, including ranks whose micro-batch is empty (the lockstep runner sends those)."""
        p = self.getParams()
        det_col = _pget(p, "predictionDetailCol")
        pred_col = _pget(p, "predictionCol")
        lcol = mt.col(p.get("labelCol"))
        if det_col:
            dvals = mt.col(det_col).values
            blk = dvals if isinstance(dvals, DetailBlock) else None
            # the columnar / string branch issues different collectives: agree on it first (an empty
            # micro-batch abstains)
            use_block = self.BINARY and ((blk is not None and len(blk.labels) == 2) or mt.num_rows == 0)
            if comm.is_distributed():
                use_block = bool(min(comm.all_gather_object(bool(use_block))))
            if use_block:
                if self._labels is None:
                    keys = M.detail_block_keys(lcol, blk) if blk is not None else set()
                    if not self._agree_labels(keys, p):
                        return None
                res = M.binary_summary_block(lcol, blk, self._labels)
                if res is not None:
                    return ("b",) + res
            labels = mt.column_values(p.get("labelCol"))
            dets = mt.column_values(det_col)
            if self._labels is None:
                # the label index is fixed by the first window (its labels and detail keys)
                keys = set()
                for l, d in zip(labels, dets):
                    if l is not None and d is not None:
                        keys.update(M.parse_detail(d).keys())
                        keys.add(str(l))
                if not self._agree_labels(keys, p):
                    return None
            if self.BINARY:
                return ("b",) + M.binary_summary(labels, dets, self._labels)
            return ("m",) + M.multi_summary_from_detail(labels, dets, self._labels)
        labels = mt.column_values(p.get("labelCol"))
        preds = mt.column_values(pred_col)
        if self._labels is None:
            if not self._agree_labels({str(x) for x in labels + preds if x is not None}, p):
                return None
        return ("m",) + M.multi_summary_from_pred(labels, preds, self._labels)

    @staticmethod
    def _metrics(s, labels):
        if s[0] == "b":
            return M.binary_metrics(s[1], s[2], labels, s[3], s[4])
        return M.multi_metrics(s[1], labels, s[2], s[3])

    @staticmethod
    def _merge(a, b):
        if a is None:
            return b
        if any(isinstance(x, torch.Tensor) for x in a[1:]) != any(isinstance(x, torch.Tensor) for x in b[1:]):
            # a device (GPU columnar) summary meets a host one: merge on the host
            a = (a[0],) + tuple(M.host_value(x) for x in a[1:])
            b = (b[0],) + tuple(M.host_value(x) for x in b[1:])
        if a[0] == "b":
            return ("b", a[1] + b[1], a[2] + b[2], a[3] + b[3], a[4] + b[4])
        ll = a[2] + b[2] if a[2] >= 0 and b[2] >= 0 else -1.0
        return ("m", a[1] + b[1], ll, a[3] + b[3])

    def _interval(self) -> float:
        v = _pget(self.getParams(), "timeInterval")
        return 3.0 if v is None else float(v)

    def _window_due(self) -> bool:
        """Whether the open window has lasted ``timeInterval`` seconds; under a process group every rank takes
        the same decision (the longest-open window of any rank), so the emitted windows line up."""
        age = time.perf_counter() - self._win_t0 if self._win_t0 is not None else 0.0
        if comm.is_distributed():
            age = float(comm.host_all_gather(torch.tensor([age], dtype=torch.float64)).max())
        return age >= self._interval()

    def _emit_window(self):
        s, self._win, self._win_t0 = self._win, None, None
        if s is not None:
            s = (s[0],) + tuple(M.host_value(x) for x in s[1:])     # device summaries: one read per window
        if s is None or s[-1] == 0:
            return
        self._acc = self._merge(self._acc, s)
        rows = [("window", self._metrics(s, self._labels).serialize()[0]),
                ("all", self._metrics(self._acc, self._labels).serialize()[0])]
        self._emit(MTable.from_rows(rows, _SCHEMA))

    def on_batch(self, port, mt):
        if mt.num_rows == 0 and not comm.is_distributed():
            return
        s = self._summary(mt)
        # a device summary's count is not read back per micro-batch: any non-empty micro-batch opens the window
        if s is not None and (mt.num_rows > 0 if isinstance(s[-1], torch.Tensor) else s[-1] != 0):
            if self._win_t0 is None:
                self._win_t0 = time.perf_counter()
            self._win = self._merge(self._win, s)
        if self._window_due():
            self._emit_window()

    def on_finish(self, port):
        self._emit_window()


class EvalBinaryClassStreamOp(_EvalStream):
    BINARY = True


class EvalMultiClassStreamOp(_EvalStream):
    pass
