"""Evaluation batch operators (reference ``A/operator/batch/evaluation/*``, ``BaseEvalClassBatchOp.java``):
each outputs ONE row ``Data`` = the metrics ``Params`` JSON; ``collectMetrics()`` returns the metric object."""
from __future__ import annotations

import numpy as np
import torch

from ...common.table import MTable
from ...common.types import TableSchema, Types
from ...models.evaluation import metrics as M

from ...parallel import comm
from ..base import BatchOperator

__all__ = ["EvalBinaryClassBatchOp", "EvalMultiClassBatchOp", "EvalRegressionBatchOp", "EvalClusterBatchOp"]

_SCHEMA = TableSchema(["Data"], [Types.STRING])


def _global_labels(vals):
    seen = set()
    for part in comm.all_gather_object(sorted({str(v) for v in vals if v is not None})):
        seen.update(part)
    return seen


def _pget(p, name):
    try:
        return p.get(name) if p.contains(name) else None
    except KeyError:
        return None


class _EvalBase(BatchOperator):
    METRICS = M.BaseMetrics

    def _out(self, metrics):
        self._metrics = metrics
        self.setOutputTable(MTable.from_rows([metrics.serialize()], _SCHEMA, replicated=True))
        return self

    def collectMetrics(self):
        rows = self.collect()
        return self.METRICS.fromRow(rows[0])

    def lazyCollectMetrics(self, *callbacks):
        def cb(rows):
            m = self.METRICS.fromRow(rows[0])
            for c in callbacks:
                c(m)
        return self.lazyCollect(cb)

    def lazyPrintMetrics(self, title=None):
        def cb(rows):
            if title:
                print(title)
            print(self.METRICS.fromRow(rows[0]))
        return self.lazyCollect(cb)


class _EvalClass(_EvalBase):
    BINARY = False

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        label_col = p.get("labelCol")
        detail_col = _pget(p, "predictionDetailCol")
        pred_col = _pget(p, "predictionCol")
        pos = _pget(p, "positiveLabelValueString")
        dev = self.env.device
        if detail_col:
            labels = mt.column_values(label_col)
            from ...common.detail import DetailBlock
            dvals = mt.col(detail_col).values
            blk = dvals if isinstance(dvals, DetailBlock) else None
            # the columnar and the string branch issue different collectives: every rank takes the same one (a
            # rank with no rows abstains)
            use_block = self.BINARY and (blk is not None or mt.num_rows == 0)
            if comm.is_distributed():
                use_block = bool(min(comm.all_gather_object(bool(use_block))))
            if use_block:
                # columnar detail (probabilities, not strings): label set and bins without per-row parsing
                label_set = set()
                keys = M.detail_block_keys(mt.col(label_col), blk) if blk is not None else set()
                for part in comm.all_gather_object(sorted(keys)):
                    label_set.update(part)
                arr = M.build_label_index(label_set, True, pos)
                fast = M.binary_summary_block(mt.col(label_col), blk, arr, dev)
                if fast is not None:
                    pb, nb, ll, n = fast
                    if n == 0:
                        raise ValueError("Please check the evaluation input! there is no effective row!")
                    return self._out(M.binary_metrics(pb, nb, arr, ll, n))
            details = mt.column_values(detail_col)
            keys = set()
            for l, d in zip(labels, details):
                if l is not None and d is not None:
                    keys.update(M.parse_detail(d).keys())
                    keys.add(str(l))
            label_set = set()
            for part in comm.all_gather_object(sorted(keys)):
                label_set.update(part)
            arr = M.build_label_index(label_set, self.BINARY, pos)
            if self.BINARY:
                pb, nb, ll, n = M.binary_summary(labels, details, arr, dev)
                if n == 0:
                    raise ValueError("Please check the evaluation input! there is no effective row!")
                return self._out(M.binary_metrics(pb, nb, arr, ll, n))
            mat, ll, n = M.multi_summary_from_detail(labels, details, arr, dev)
        elif pred_col:
            # integer / bool tensor columns: codes without a Python pass over the rows (every rank must take the
            # same branch: the label-set gather differs)
            fast_ok = M.multi_summary_pred_tensors if mt.num_rows else None
            use_fast = fast_ok is not None and all(
                isinstance(mt.col(c).values, torch.Tensor) and mt.col(c).values.dim() == 1 and
                not mt.col(c).values.is_floating_point() for c in (label_col, pred_col)) and \
                mt.col(label_col).values.dtype == mt.col(pred_col).values.dtype
            if comm.is_distributed():
                use_fast = bool(min(comm.all_gather_object(bool(use_fast))))
            fast = M.multi_summary_pred_tensors(mt.col(label_col), mt.col(pred_col), self.BINARY, pos, dev) \
                if use_fast else None
            if fast is not None:
                mat, ll, n, arr = fast
            else:
                labels = mt.column_values(label_col)
                preds = mt.column_values(pred_col)
                arr = M.build_label_index(_global_labels(labels) | _global_labels(preds), self.BINARY, pos)
                mat, ll, n = M.multi_summary_from_pred(labels, preds, arr, dev)
        else:
            raise ValueError("Error Input, must give either predictionCol or predictionDetailCol!")
        if n == 0:
            raise ValueError("Please check the evaluation input! there is no effective row!")
        return self._out(M.multi_metrics(mat, arr, ll, n))


class EvalBinaryClassBatchOp(_EvalClass):
    BINARY = True
    METRICS = M.BinaryClassMetrics


class EvalMultiClassBatchOp(_EvalClass):
    METRICS = M.MultiClassMetrics


class EvalRegressionBatchOp(_EvalBase):
    METRICS = M.RegressionMetrics

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        yc, pc = mt.col(self.getLabelCol()), mt.col(self.getPredictionCol())
        if all(isinstance(c.values, torch.Tensor) and c.values.dim() == 1 and not c.values.is_complex()
               for c in (yc, pc)):
            # tensor columns: the non-null pairs masked on the device, no Python pass over the rows
            ok = torch.ones(yc.values.shape, dtype=torch.bool, device=yc.values.device)
            for c in (yc, pc):
                if c.nulls is not None:
                    ok &= ~c.nulls.to(ok.device)
            s = M.regression_summary(yc.values[ok], pc.values.to(ok.device)[ok], self.env.device)
        else:
            y = mt.column_values(self.getLabelCol())
            pr = mt.column_values(self.getPredictionCol())
            keep = [(a, b) for a, b in zip(y, pr) if a is not None and b is not None]
            s = M.regression_summary([a for a, _ in keep], [b for _, b in keep], self.env.device)
        if s[-1] == 0:
            raise ValueError("Please check the evaluation input! there is no effective row!")
        return self._out(M.regression_metrics(s))


class EvalClusterBatchOp(_EvalBase):
    METRICS = M.ClusterMetrics

    def linkFrom(self, *inputs):
        from ...models.evaluation.cluster import cluster_metrics
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        return self._out(cluster_metrics(mt, self.getParams(), self.env))
