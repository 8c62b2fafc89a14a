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
        """Binary summary straight from a ``DetailBlock`` (no detail strings): positive-class probability column,
        label match by distinct value, log-loss in row order — the values ``binary_summary`` computes from the
        strings (the strings are ``Double.toString`` of these same doubles, which parse back exactly)."""
        import numpy as np
        import torch
        keys = [str(x) for x in blk.labels]
        lab = lcol.values
        if isinstance(lab, torch.Tensor) and lab.dim() == 1:
            lab = lab.detach().cpu()
            uniq, inv = torch.unique(lab, return_inverse=True)
            ustr = [str(v) for v in uniq.tolist()]
            inv = inv.numpy()
            lnull = lcol.nulls.cpu().numpy() if lcol.nulls is not None else np.zeros(len(inv), bool)
        else:
            vals = lcol.to_list()
            ustr = sorted({str(v) for v in vals if v is not None})
            pos = {u: i for i, u in enumerate(ustr)}
            inv = np.asarray([pos[str(v)] if v is not None else 0 for v in vals], dtype=np.int64)
            lnull = np.asarray([v is None for v in vals], dtype=bool)
        ok = ~lnull if blk.nulls is None else (~lnull & ~blk.nulls)
        if self._labels is None:
            present = {ustr[i] for i in np.unique(inv[ok]).tolist()} if ok.any() else set()
            self._labels = M.build_label_index(set(keys) | present, True, _pget(p, "positiveLabelValueString"))
        la = self._labels
        if set(keys) != set(la):
            return None
        c0, c1 = keys.index(la[0]), keys.index(la[1])
        pr = blk.probs
        if not (np.all((pr >= 0.0) & (pr <= 1.0)) and np.all(np.abs(pr[:, c0] + pr[:, c1] - 1.0) < M.PROB_SUM_EPS)):
            return None
        code = np.array([0 if u == la[0] else (1 if u == la[1] else -1) for u in ustr], dtype=np.int64)
        rc = code[inv] if len(code) else np.zeros(0, np.int64)
        sel = ok & (rc >= 0)
        is_pos = rc[sel] == 0
        p0 = pr[sel, c0]
        pl = np.where(is_pos, p0, pr[sel, c1])
        terms = -np.log(np.clip(pl, M.LOG_LOSS_EPS, 1 - M.LOG_LOSS_EPS))
        ll = float(np.cumsum(terms)[-1]) if len(terms) else 0.0
        return ("b",) + M._binary_bins(p0, is_pos, ll, int(sel.sum()), torch.device("cpu"))

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
