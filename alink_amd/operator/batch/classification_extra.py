"""Batch operators of the non-linear classifiers (reference ``A/operator/batch/classification/*``)."""
from __future__ import annotations

from ...common.table import MTable
from ...models.classification.naive_bayes import (NaiveBayesTextModelDataConverter, NaiveBayesTextModelMapper,
                                                  train_naive_bayes_text)
from ..base import BatchOperator
from .utils import ModelMapBatchOp

__all__ = ["NaiveBayesTextTrainBatchOp", "NaiveBayesTextPredictBatchOp", "MultilayerPerceptronTrainBatchOp",
           "MultilayerPerceptronPredictBatchOp"]


class NaiveBayesTextTrainBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        m = train_naive_bayes_text(mt, p, self.env)
        conv = NaiveBayesTextModelDataConverter(mt.col_type(p.get("labelCol")))
        self.setOutputTable(MTable.from_rows(conv.save(m), conv.getModelSchema(), replicated=True))
        return self


class NaiveBayesTextPredictBatchOp(ModelMapBatchOp):
    MAPPER = NaiveBayesTextModelMapper


class MultilayerPerceptronTrainBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        from ...models.classification.mlp import MlpcModelDataConverter, train_mlp
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        meta, w, labels, lt = train_mlp(mt, self.getParams(), self.env)
        conv = MlpcModelDataConverter(lt)
        self.setOutputTable(MTable.from_rows(conv.save((meta, w, labels)), conv.getModelSchema(), replicated=True))
        return self


from ...models.classification.mlp import MlpcModelMapper  # noqa: E402


class MultilayerPerceptronPredictBatchOp(ModelMapBatchOp):
    MAPPER = MlpcModelMapper
