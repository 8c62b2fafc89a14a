"""Model-information extraction ops (``A/common/lazy/ExtractModelInfoBatchOp.java``,
``WithModelInfoBatchOp.java``) and the FM model summary (``A/operator/common/fm/FmModelInfo{,BatchOp}.java``).

``ExtractModelInfoBatchOp`` passes its input model table through and turns the model rows into a summary object
(``createModelInfo``) that can be printed / collected lazily (fires with the next ``execute``/``collect``) or
eagerly (``collectModelInfo``).  A train op mixes in ``WithModelInfoBatchOp`` and names its extractor in
``getModelInfoBatchOp``; pipeline ``Trainer.enableLazyPrintModelInfo`` goes through the same hook.
"""
from __future__ import annotations

import json
from typing import Any, Callable, List

import numpy as np

from ..base import BatchOperator

__all__ = ["ExtractModelInfoBatchOp", "WithModelInfoBatchOp", "WithTrainInfo", "FmModelInfo", "FmModelInfoBatchOp"]


class ExtractModelInfoBatchOp(BatchOperator):
    _NO_AUTO_PARAMS = True

    def linkFrom(self, *inputs):
        op = self.checkAndGetFirst(inputs)
        self.setOutputTable(op.getOutputTable())
        return self

    def createModelInfo(self, rows: List[Any]):
        raise NotImplementedError

    def processModel(self) -> BatchOperator:
        return self

    def lazyPrintModelInfo(self, title=None):
        def show(info):
            if self.env.rank == 0:
                if title is not None:
                    print(title)
                print(info)
        return self.lazyCollectModelInfo(show)

    def lazyCollectModelInfo(self, *callbacks: Callable[[Any], None]):
        cbs = list(callbacks[0]) if len(callbacks) == 1 and isinstance(callbacks[0], (list, tuple)) else callbacks

        def fire(rows):
            info = self.createModelInfo(rows)
            for cb in cbs:
                cb(info)
        self.processModel().lazyCollect(fire)
        return self

    def collectModelInfo(self):
        return self.createModelInfo(self.processModel().collect())


class WithModelInfoBatchOp:
    """Mixin for train ops: ``getModelInfoBatchOp()`` returns an ``ExtractModelInfoBatchOp`` linked from self."""

    def getModelInfoBatchOp(self) -> ExtractModelInfoBatchOp:
        raise NotImplementedError

    def _info_op(self):
        return self.getModelInfoBatchOp().setMLEnvironmentId(self.getMLEnvironmentId())

    def lazyPrintModelInfo(self, title=None):
        self._info_op().lazyPrintModelInfo(title)
        return self

    def lazyCollectModelInfo(self, *callbacks):
        self._info_op().lazyCollectModelInfo(*callbacks)
        return self

    def collectModelInfo(self):
        return self._info_op().collectModelInfo()


class WithTrainInfo:
    """Train-information mixin for train ops (reference ``A/common/lazy/WithTrainInfo.java``): ``createTrainInfo``
    builds the summary object; ``collectTrainInfo`` returns it now, ``lazyCollectTrainInfo`` / ``lazyPrintTrainInfo``
    hand it to callbacks at the next execution (``execute`` / ``collect`` / ``print``), on rank 0 for prints."""

    def createTrainInfo(self):
        raise NotImplementedError

    def collectTrainInfo(self):
        return self.createTrainInfo()

    def lazyCollectTrainInfo(self, *callbacks: Callable[[Any], None]):
        cbs = list(callbacks[0]) if len(callbacks) == 1 and isinstance(callbacks[0], (list, tuple)) else callbacks

        def fire(_rows):
            info = self.createTrainInfo()
            for cb in cbs:
                cb(info)
        self.lazyCollect(fire)
        return self

    def lazyPrintTrainInfo(self, title=None):
        def show(info):
            if self.env.rank == 0:
                if title is not None:
                    print(title)
                print(info)
        return self.lazyCollectTrainInfo(show)


def _fmt8(x: float) -> str:
    return f"{float(x):.8f}"


class FmModelInfo:
    """Summary of an FM model: dim [bias?, linear?, k], task, vectorSize, factors, field positions, column names."""

    def __init__(self, rows, label_type=None):
        from ...models.recommendation.fm import FmModelDataConverter
        m = FmModelDataConverter(label_type).load(rows)
        self.dim = [int(v) for v in m.dim]
        self.task = str(getattr(m.task, "name", m.task))
        self.vectorSize = int(m.vectorSize)
        self.colNames = list(m.featureColNames) if m.featureColNames is not None else None
        self.filedPos = list(m.fieldPos) if m.fieldPos is not None else None
        self._model = m.fmModel

    def getDim(self):
        return self.dim

    def getTask(self):
        return self.task

    def getVectorSize(self):
        return self.vectorSize

    def getFactors(self):
        return np.asarray(self._model.factors)

    def getFiledPos(self):
        return self.filedPos

    def getColNames(self):
        return self.colNames

    def __str__(self):
        out = ["-" * 20 + " meta info " + "-" * 20]
        meta = {"vectorSize": str(self.vectorSize), "task": self.task, "dim": json.dumps(self.dim),
                "bias": str(float(self._model.bias))}
        if self.filedPos is not None:
            meta["filedPos"] = json.dumps(self.filedPos)
        out.append(" | ".join(f"{k}: {v}" for k, v in meta.items()))
        out.append("-" * 20 + " model info " + "-" * 20)
        k = self.dim[2]
        factors = np.asarray(self._model.factors)
        linear = np.asarray(self._model.linearItems) if self._model.linearItems is not None else None
        names = self.colNames if self.colNames is not None else [str(i) for i in range(len(factors))]
        show = min(len(names), 10)
        out.append(f"{'colName':>12} | {'linearItem':>12} | factor")
        for i in range(show):
            lin = _fmt8(linear[i]) if (self.dim[1] > 0 and linear is not None) else _fmt8(0.0)
            out.append(f"{names[i]:>12} | {lin:>12} | " + " ".join(_fmt8(f) for f in factors[i][:k]))
        if len(names) > 10:
            out.append(f"{'... ...':>12} | {'... ...':>12} | ... ...")
        return "\n".join(out)


class FmModelInfoBatchOp(ExtractModelInfoBatchOp):
    def __init__(self, label_type=None, params=None):
        super().__init__(params)
        self._label_type = label_type

    def createModelInfo(self, rows):
        return FmModelInfo(rows, self._label_type)
