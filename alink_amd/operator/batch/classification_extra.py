"""Batch operators of the non-linear classifiers (reference ``A/operator/batch/classification/*``)."""
from __future__ import annotations

from ...common.table import MTable
from ...models.classification.naive_bayes import (NaiveBayesTextModelDataConverter, NaiveBayesTextModelMapper,
                                                  train_naive_bayes_text)
from .modelinfo import FmModelInfoBatchOp, WithModelInfoBatchOp
from ..base import BatchOperator
from .utils import ModelMapBatchOp

__all__ = ["FmTrainBatchOp", "FmPredictBatchOp", "FmClassifierTrainBatchOp", "FmClassifierPredictBatchOp", "FmRegressorTrainBatchOp",
           "FmRegressorPredictBatchOp", "NaiveBayesTextTrainBatchOp", "NaiveBayesTextPredictBatchOp", "MultilayerPerceptronTrainBatchOp",
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


from ...models.recommendation import fm as _FM  # noqa: E402


class _FmTrainBatchOp(BatchOperator, WithModelInfoBatchOp):
    """``FmTrainBatchOp`` (task fixed by the subclass): device mini-batch AdaGrad + model averaging; model info via
    ``FmModelInfoBatchOp`` (``BaseFmTrainBatchOp.java:555``)."""
    TASK = "REGRESSION"
    _NO_AUTO_PARAMS = True

    def getModelInfoBatchOp(self):
        return FmModelInfoBatchOp(getattr(self, "_label_type", None)).linkFrom(self)

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        m, lt, info = _FM.train_fm(mt, self.resolvedParams(), self.TASK, self.env)
        self._label_type = lt
        self._train_info = info
        conv = _FM.FmModelDataConverter(lt)
        self.setOutputTable(MTable.from_rows(conv.save(m), conv.getModelSchema(), replicated=True))
        return self

    def getTrainInfo(self):
        return getattr(self, "_train_info", None)


class FmClassifierTrainBatchOp(_FmTrainBatchOp):
    _NO_AUTO_PARAMS = False
    TASK = "BINARY_CLASSIFICATION"


class FmRegressorTrainBatchOp(_FmTrainBatchOp):
    _NO_AUTO_PARAMS = False
    TASK = "REGRESSION"


class FmClassifierPredictBatchOp(ModelMapBatchOp):
    MAPPER = _FM.FmModelMapper


class FmRegressorPredictBatchOp(ModelMapBatchOp):
    MAPPER = _FM.FmModelMapper


_FM_TASKS = {"BINARY_CLASSIFICATION": "BINARY_CLASSIFICATION", "CLASSIFICATION": "BINARY_CLASSIFICATION",
             "REGRESSION": "REGRESSION"}


class FmTrainBatchOp(_FmTrainBatchOp):
    """The public generic FM trainer (``A/operator/common/fm/FmTrainBatchOp.java:17``): the task is a constructor
    argument / the ``task`` param (``ModelParamName.TASK``; "binary_classification" or "regression", case-insensitive
    as ``Task.valueOf(...toUpperCase())`` at ``BaseFmTrainBatchOp.java:99``).  Same trainer as the classifier /
    regressor ops, so the models are identical to theirs for the same task."""
    _NO_AUTO_PARAMS = True
    from ...params import op_params as _op_params
    from ...common.params import ParamInfo as _ParamInfo
    PARAMS = _op_params("FmRegressorTrainBatchOp") + [
        _ParamInfo("task", str, "FM task: binary_classification or regression (ModelParamName.TASK).", default=None)]
    del _op_params, _ParamInfo

    def __init__(self, params=None, task=None, **kwargs):
        if isinstance(params, str) and task is None:       # FmTrainBatchOp("regression")
            params, task = None, params
        super().__init__(params, **kwargs)
        if task is not None:
            self.getParams().set("task", task)

    @property
    def TASK(self):
        t = self.getParams().get("task") if self.getParams().contains("task") else None
        if t is None:
            raise ValueError("FmTrainBatchOp needs a task: binary_classification or regression")
        key = str(t).upper()
        if key not in _FM_TASKS:
            raise ValueError(f"unknown FM task {t!r}")
        return _FM_TASKS[key]


class FmPredictBatchOp(ModelMapBatchOp):
    """``A/operator/common/fm/FmPredictBatchOp.java:12``: a ModelMapBatchOp over ``FmModelMapper`` (the task comes
    from the model's meta, so one op serves both tasks)."""
    MAPPER = _FM.FmModelMapper
