"""ALS batch operators (reference ``A/operator/batch/recommendation/{AlsTrain,AlsPredict,AlsTopKPredict}BatchOp``);
implementation in ``models/recommendation/als.py``."""
from __future__ import annotations

from ...common.table import MTable
from ...common.types import TableSchema, Types
from ...models.recommendation.als import AlsModelDataConverter, AlsModelMapper, als_topk, train_als
from ..base import BatchOperator
from .utils import ModelMapBatchOp

__all__ = ["AlsTrainBatchOp", "AlsPredictBatchOp", "AlsTopKPredictBatchOp"]


class AlsTrainBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        model = train_als(mt, p, self.env)
        conv = AlsModelDataConverter(p.get("userCol"), p.get("itemCol"))
        self.setOutputTable(MTable.from_rows(conv.save(model), conv.getModelSchema(), replicated=True))
        return self


class AlsPredictBatchOp(ModelMapBatchOp):
    MAPPER = AlsModelMapper


class AlsTopKPredictBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        if len(inputs) == 1 and isinstance(inputs[0], (list, tuple)):
            inputs = inputs[0]
        self.checkOpSize(2, inputs)
        model_op, data_op = inputs
        p = self.getParams()
        model = AlsModelDataConverter.load(model_op.getOutputTable().rows())
        data = data_op.getOutputTable()
        k = int(p.get("topK")) if p.contains("topK") and p.get("topK") is not None else 100
        users = data.column_values(p.get("userCol"))
        rows = als_topk(model, users, k, self.env.device)
        schema = TableSchema([p.get("userCol"), p.get("predictionCol")], [Types.LONG, Types.STRING])
        self.setOutputTable(MTable.from_rows(rows, schema, replicated=data.replicated))
        return self
