"""GLM and isotonic-regression batch operators.

Reference: ``A/operator/batch/regression/{GlmTrainBatchOp,GlmPredictBatchOp,GlmEvaluationBatchOp,
IsotonicRegTrainBatchOp,IsotonicRegPredictBatchOp}.java``.  ``GlmTrainBatchOp`` has two side outputs like the
reference: the residual table (features, label, weight, offset, pred, deviance/pearson/working/response
residuals) and the one-row JSON summary.
"""
from __future__ import annotations

import torch

from ...common.table import Column, MTable
from ...common.types import TableSchema, Types
from ...models.regression import glm as G
from ...models.regression.isotonic import (IsotonicRegressionConverter, IsotonicRegressionModelMapper,
                                           train_isotonic)
from ..base import BatchOperator, gather_table
from .utils import ModelMapBatchOp

__all__ = ["GlmTrainBatchOp", "GlmPredictBatchOp", "GlmEvaluationBatchOp", "IsotonicRegTrainBatchOp",
           "IsotonicRegPredictBatchOp"]


def _glm_data(op, mt):
    p = op.resolvedParams()

    def g(n):
        return p.get(n) if p.contains(n) else None
    return G.preprocess(mt, p.get("featureCols"), p.get("labelCol"), g("weightCol"), g("offsetCol"), op.env.device)


def _residual_table(d, model, fl, feature_cols) -> MTable:
    res = G.glm_residuals(d, model, fl)
    cols = [d.X[:, i] for i in range(d.X.shape[1])] + [d.y, d.w, d.off] + res
    names = list(feature_cols) + G.RESIDUAL_COLS
    return MTable(TableSchema(names, [Types.DOUBLE] * len(names)), [Column(c.detach().cpu()) for c in cols])


class GlmTrainBatchOp(BatchOperator):
    """IRLS generalized linear model; output = model table, side outputs = [residuals, summary]."""

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.resolvedParams()
        d = _glm_data(self, mt)
        fl = G.family_link_of(p)
        wls = G.train_glm(d, p)
        conv = G.GlmModelDataConverter()
        self.setOutputTable(MTable.from_rows(conv.save(conv.from_wls(wls, p)), conv.getModelSchema(),
                                             replicated=True))
        summary = G.glm_summary(d, wls, fl, float(p.get("regParam")), int(p.get("maxIter")),
                                float(p.get("epsilon")), bool(p.get("fitIntercept")))
        self.setSideOutputTables([_residual_table(d, wls, fl, p.get("featureCols")),
                                  MTable.from_rows([(summary,)], "summary string", replicated=True)])
        return self


class GlmPredictBatchOp(ModelMapBatchOp):
    MAPPER = G.GlmModelMapper


class GlmEvaluationBatchOp(BatchOperator):
    """Summary of a trained GLM on data (output = summary JSON, side output = residuals)."""

    def linkFrom(self, *inputs):
        if len(inputs) == 1 and isinstance(inputs[0], (list, tuple)):
            inputs = inputs[0]
        self.checkOpSize(2, inputs)
        model_op, data_op = inputs
        p = self.resolvedParams()
        m = G.GlmModelDataConverter().load(gather_table(model_op.getOutputTable()).rows())
        wls = G.WlsModel(m.coefficients, m.intercept, m.diagInvAtWA, m.fitIntercept, 0)
        d = _glm_data(self, data_op.getOutputTable())
        fl = G.family_link_of(p)
        summary = G.glm_summary(d, wls, fl, float(p.get("regParam")), int(p.get("maxIter")),
                                float(p.get("epsilon")), bool(p.get("fitIntercept")))
        self.setOutputTable(MTable.from_rows([(summary,)], "summary string", replicated=True))
        self.setSideOutputTables([_residual_table(d, wls, fl, p.get("featureCols"))])
        return self


class IsotonicRegTrainBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        m = train_isotonic(mt, self.resolvedParams())
        conv = IsotonicRegressionConverter()
        self.setOutputTable(MTable.from_rows(conv.save(m), conv.getModelSchema(), replicated=True))
        return self


class IsotonicRegPredictBatchOp(ModelMapBatchOp):
    MAPPER = IsotonicRegressionModelMapper
