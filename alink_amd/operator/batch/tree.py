"""Tree batch operators: GBDT (classification / regression), random forest and decision tree.

Reference: ``A/operator/batch/classification/{Gbdt,RandomForest,DecisionTree}{Train,Predict}BatchOp.java``,
``A/operator/batch/regression/{GbdtReg,RandomForestReg,DecisionTreeReg}{Train,Predict}BatchOp.java`` ->
``A/operator/common/tree/{BaseGbdtTrainBatchOp,BaseRandomForestTrainBatchOp}.java``.  Training lives in
``models/tree`` (HIP histogram kernels in ``ops/csrc/tree_hist.hip``).
"""
from __future__ import annotations

from ...common.table import MTable
from ...models.tree.model import GbdtModelMapper, RandomForestModelMapper
from ...models.tree.train import IMPORTANCE_SCHEMA, train_forest, train_gbdt
from ..base import BatchOperator
from .modelinfo import WithTrainInfo
from .utils import ModelMapBatchOp

__all__ = ["GbdtTrainBatchOp", "GbdtRegTrainBatchOp", "GbdtPredictBatchOp", "GbdtRegPredictBatchOp",
           "RandomForestTrainBatchOp", "RandomForestRegTrainBatchOp", "RandomForestPredictBatchOp",
           "RandomForestRegPredictBatchOp", "DecisionTreeTrainBatchOp", "DecisionTreeRegTrainBatchOp",
           "DecisionTreePredictBatchOp", "DecisionTreeRegPredictBatchOp"]


class _TreeTrainInfo(WithTrainInfo):
    _train_info: dict = None

    def getTrainInfo(self):
        return self._train_info

    def createTrainInfo(self):
        return self._train_info


class BaseGbdtTrainBatchOp(BatchOperator, _TreeTrainInfo):
    """``algoType`` (the reference's public field, ``BaseGbdtTrainBatchOp.java:63-66``): 0 regression, 1 binary
    classification, 2 LambdaMART-NDCG, 3 LambdaMART-DCG, 4 GBRank — the ranking losses need ``groupCol``
    (query id).  Set it as ``op.algoType = 2`` or ``BaseGbdtTrainBatchOp(algoType=2)``."""
    ALGO_TYPE = 1

    def __init__(self, params=None, algoType=None, **kw):
        super().__init__(params, **kw)
        self.algoType = self.ALGO_TYPE if algoType is None else int(algoType)

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        algo = int(getattr(self, "algoType", self.ALGO_TYPE))
        if algo not in (0, 1, 2, 3, 4):
            raise ValueError(f"algoType must be 0..4, got {algo}")
        rows, conv, imp, info = train_gbdt(mt, self.getParams().clone(), self.env, algo)
        self._train_info = info
        self.setOutputTable(MTable.from_rows(rows, conv.getModelSchema(), replicated=True))
        self.setSideOutputTables([MTable.from_rows(imp, IMPORTANCE_SCHEMA, replicated=True)])
        return self


class GbdtTrainBatchOp(BaseGbdtTrainBatchOp):
    ALGO_TYPE = 1


class GbdtRegTrainBatchOp(BaseGbdtTrainBatchOp):
    ALGO_TYPE = 0


class BaseRandomForestTrainBatchOp(BatchOperator, _TreeTrainInfo):
    REGRESSION = False
    FORCED = {}

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams().clone()
        for k, v in self.FORCED.items():
            p.set(k, v)
        rows, conv, info = train_forest(mt, p, self.env, self.REGRESSION)
        self._train_info = info
        self.setOutputTable(MTable.from_rows(rows, conv.getModelSchema(), replicated=True))
        return self


class RandomForestTrainBatchOp(BaseRandomForestTrainBatchOp):
    pass


class RandomForestRegTrainBatchOp(BaseRandomForestTrainBatchOp):
    REGRESSION = True


class DecisionTreeTrainBatchOp(BaseRandomForestTrainBatchOp):
    FORCED = {"numTrees": 1, "featureSubsamplingRatio": 1.0, "subsamplingRatio": 1.0}


class DecisionTreeRegTrainBatchOp(BaseRandomForestTrainBatchOp):
    REGRESSION = True
    FORCED = {"numTrees": 1, "featureSubsamplingRatio": 1.0, "subsamplingRatio": 1.0}


class GbdtPredictBatchOp(ModelMapBatchOp):
    MAPPER = GbdtModelMapper


class GbdtRegPredictBatchOp(ModelMapBatchOp):
    MAPPER = GbdtModelMapper


class RandomForestPredictBatchOp(ModelMapBatchOp):
    MAPPER = RandomForestModelMapper


class RandomForestRegPredictBatchOp(ModelMapBatchOp):
    MAPPER = RandomForestModelMapper


class DecisionTreePredictBatchOp(ModelMapBatchOp):
    MAPPER = RandomForestModelMapper


class DecisionTreeRegPredictBatchOp(ModelMapBatchOp):
    MAPPER = RandomForestModelMapper
