"""Linear-family batch operators: LR, LinearSvm, LinearReg, Ridge, Lasso, Softmax, AFT survival.

Reference: ``A/operator/batch/classification/{LogisticRegression,LinearSvm,Softmax}{Train,Predict}BatchOp.java``,
``A/operator/batch/regression/{LinearReg,RidgeReg,LassoReg,AftSurvivalReg}{Train,Predict}BatchOp.java``;
training in ``models/linear/train.py``, optimizers in ``models/linear/optim.py``.
"""
from __future__ import annotations

from ...common.table import MTable
from ...models.linear.model import AFTModelMapper, LinearModelDataConverter, LinearModelMapper, SoftmaxModelMapper
from ...models.linear.train import train_aft, train_linear, train_softmax
from ..base import BatchOperator, format_rows
from .modelinfo import WithTrainInfo
from .utils import ModelMapBatchOp

__all__ = ["BaseLinearModelTrainBatchOp", "LogisticRegressionTrainBatchOp", "LogisticRegressionPredictBatchOp",
           "LinearSvmTrainBatchOp", "LinearSvmPredictBatchOp", "LinearRegTrainBatchOp", "LinearRegPredictBatchOp",
           "RidgeRegTrainBatchOp", "RidgeRegPredictBatchOp", "LassoRegTrainBatchOp", "LassoRegPredictBatchOp",
           "SoftmaxTrainBatchOp", "SoftmaxPredictBatchOp", "AftSurvivalRegTrainBatchOp",
           "AftSurvivalRegPredictBatchOp"]


class LinearTrainInfo:
    """Convergence summary of a linear train op: iterations and loss curve."""

    def __init__(self, info: dict):
        info = info or {}
        self.numIter = info.get("numIter")
        curve = info.get("lossCurve")
        self.lossCurve = [] if curve is None else [float(v) for v in curve]

    def __str__(self):
        return f"numIter: {self.numIter}, final loss: {self.lossCurve[-1] if self.lossCurve else None}"


class LinearModelSummary:
    """Model summary of a linear train op: model name, intercept flag and coefficients."""

    def __init__(self, model):
        self.modelName = model.modelName
        self.hasInterceptItem = model.hasInterceptItem
        self.coefVector = model.coefVector

    def __str__(self):
        return f"model: {self.modelName}, intercept: {self.hasInterceptItem}, coef: {self.coefVector}"


class _WithTrainInfo(WithTrainInfo):
    _train_info: dict = None

    def getTrainInfo(self):
        return self._train_info

    def createTrainInfo(self):
        return LinearTrainInfo(self._train_info)

    # model summary, lazy like the train info (the reference's WithModelInfoBatchOp protocol)
    def collectModelInfo(self):
        return LinearModelSummary(self._model)

    def lazyCollectModelInfo(self, *callbacks):
        cbs = list(callbacks[0]) if len(callbacks) == 1 and isinstance(callbacks[0], (list, tuple)) else callbacks
        self.lazyCollect(lambda _rows: [cb(self.collectModelInfo()) for cb in cbs])
        return self

    def lazyPrintModelInfo(self, title=None):
        def show(info):
            if self.env.rank == 0:
                if title is not None:
                    print(title)
                print(info)
        return self.lazyCollectModelInfo(show)


class BaseLinearModelTrainBatchOp(BatchOperator, _WithTrainInfo):
    _NO_AUTO_PARAMS = True
    MODEL_TYPE = "LR"
    MODEL_NAME = "Logistic Regression"

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        model, info = train_linear(mt, self.getParams(), self.MODEL_TYPE, self.MODEL_NAME, self.env)
        self._model, self._train_info = model, info
        conv = LinearModelDataConverter(model.labelType)
        self.setOutputTable(MTable.from_rows(conv.save(model), conv.getModelSchema(), replicated=True))
        return self


class LogisticRegressionTrainBatchOp(BaseLinearModelTrainBatchOp):
    _NO_AUTO_PARAMS = False
    MODEL_TYPE, MODEL_NAME = "LR", "Logistic Regression"


class LinearSvmTrainBatchOp(BaseLinearModelTrainBatchOp):
    _NO_AUTO_PARAMS = False
    MODEL_TYPE, MODEL_NAME = "SVM", "Linear SVM"


class LinearRegTrainBatchOp(BaseLinearModelTrainBatchOp):
    _NO_AUTO_PARAMS = False
    MODEL_TYPE, MODEL_NAME = "LinearReg", "Linear Regression"


class RidgeRegTrainBatchOp(BaseLinearModelTrainBatchOp):
    _NO_AUTO_PARAMS = False
    MODEL_TYPE, MODEL_NAME = "LinearReg", "Ridge Regression"


class LassoRegTrainBatchOp(BaseLinearModelTrainBatchOp):
    _NO_AUTO_PARAMS = False
    MODEL_TYPE, MODEL_NAME = "LinearReg", "LASSO"


class SoftmaxTrainBatchOp(BatchOperator, _WithTrainInfo):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        model, info = train_softmax(mt, self.getParams(), self.env)
        self._model, self._train_info = model, info
        conv = LinearModelDataConverter(model.labelType)
        self.setOutputTable(MTable.from_rows(conv.save(model), conv.getModelSchema(), replicated=True))
        return self


class AftSurvivalRegTrainBatchOp(BatchOperator, _WithTrainInfo):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        model, info = train_aft(mt, self.getParams(), self.env)
        self._model, self._train_info = model, info
        conv = LinearModelDataConverter(model.labelType)
        self.setOutputTable(MTable.from_rows(conv.save(model), conv.getModelSchema(), replicated=True))
        return self


class LogisticRegressionPredictBatchOp(ModelMapBatchOp):
    MAPPER = LinearModelMapper


class LinearSvmPredictBatchOp(ModelMapBatchOp):
    MAPPER = LinearModelMapper


class LinearRegPredictBatchOp(ModelMapBatchOp):
    MAPPER = LinearModelMapper


class RidgeRegPredictBatchOp(ModelMapBatchOp):
    MAPPER = LinearModelMapper


class LassoRegPredictBatchOp(ModelMapBatchOp):
    MAPPER = LinearModelMapper


class SoftmaxPredictBatchOp(ModelMapBatchOp):
    MAPPER = SoftmaxModelMapper


class AftSurvivalRegPredictBatchOp(ModelMapBatchOp):
    MAPPER = AFTModelMapper
