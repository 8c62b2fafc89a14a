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
from .utils import ModelMapBatchOp

__all__ = ["BaseLinearModelTrainBatchOp", "LogisticRegressionTrainBatchOp", "LogisticRegressionPredictBatchOp",
           "LinearSvmTrainBatchOp", "LinearSvmPredictBatchOp", "LinearRegTrainBatchOp", "LinearRegPredictBatchOp",
           "RidgeRegTrainBatchOp", "RidgeRegPredictBatchOp", "LassoRegTrainBatchOp", "LassoRegPredictBatchOp",
           "SoftmaxTrainBatchOp", "SoftmaxPredictBatchOp", "AftSurvivalRegTrainBatchOp",
           "AftSurvivalRegPredictBatchOp"]


class _WithTrainInfo:
    _train_info: dict = None

    def getTrainInfo(self):
        return self._train_info

    def lazyPrintTrainInfo(self, title=None):
        info = self._train_info or {}
        if title:
            print(title)
        curve = info.get("lossCurve")
        print(f"numIter: {info.get('numIter')}, final loss: {curve[-1] if curve is not None and len(curve) else None}")
        return self

    def lazyPrintModelInfo(self, title=None):
        if title:
            print(title)
        m = getattr(self, "_model", None)
        if m is not None:
            print(f"model: {m.modelName}, intercept: {m.hasInterceptItem}, coef: {m.coefVector}")
        return self


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
