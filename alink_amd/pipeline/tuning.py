"""Hyper-parameter tuning: ``ParamGrid``, ``GridSearchCV`` (k-fold), ``GridSearchTVSplit`` (train/validation
split), tuning evaluators and the JSON ``Report``.

Reference: ``A/pipeline/tuning/*`` — ``BaseTuning.java`` (``findBestTVSplit`` :92-173, ``findBestCV``
:175-237, ``kFoldCv`` :239-313, contiguous fold split of the shuffled data :340-404),
``PipelineCandidatesGrid.java`` (mixed-radix candidate decoding: the LAST grid item varies slowest),
``TuningEvaluator.java`` (metric lookup by name/alias, case-insensitive), ``Report.java`` (pretty JSON).

Every candidate is a full pipeline fit through the framework's batch engine, so each fit runs its BSP
supersteps on the rank's GPU with RCCL all-reduces; candidates are evaluated in sequence like the reference.
"""
from __future__ import annotations

import json
import re
from typing import Any, List, Optional, Sequence, Tuple

import numpy as np

from ..common.params import ParamInfo, Params, WithParams
from ..common.table import MTable
from ..parallel import comm
from .base import EstimatorBase, ModelBase, Pipeline, PipelineStageBase, TransformerBase

__all__ = ["ParamGrid", "PipelineCandidatesGrid", "Report", "TuningEvaluator", "BinaryClassificationTuningEvaluator",
           "MulticlassClassificationTuningEvaluator", "RegressionTuningEvaluator", "ClusterTuningEvaluator",
           "GridSearchCV", "GridSearchCVModel", "GridSearchTVSplit", "GridSearchTVSplitModel"]


def _camel(name: str) -> str:
    """``SUBSAMPLING_RATIO`` (PyAlink constant style) -> ``subsamplingRatio``; camelCase passes through."""
    if "_" in name or name.isupper():
        parts = name.lower().split("_")
        return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])
    return name


def _resolve_info(stage: PipelineStageBase, info) -> ParamInfo:
    if isinstance(info, ParamInfo):
        return info
    name = _camel(str(info))
    infos = stage._param_infos
    if name in infos:
        return infos[name]
    low = {k.lower(): v for k, v in infos.items()}
    if name.lower() in low:
        return low[name.lower()]
    for v in infos.values():
        if name in v.alias:
            return v
    raise KeyError(f"{type(stage).__name__} has no parameter {info}")


class ParamGrid:
    def __init__(self):
        self.items: List[Tuple[PipelineStageBase, ParamInfo, List[Any]]] = []

    def addGrid(self, stage: PipelineStageBase, info, values: Sequence[Any]):
        values = list(values)
        if not values:
            raise ValueError("The length of parameter should not be empty.")
        self.items.append((stage, _resolve_info(stage, info), values))
        return self

    def getItems(self):
        return list(self.items)


class PipelineCandidatesGrid:
    def __init__(self, estimator: EstimatorBase, grid: ParamGrid):
        self.pipeline = estimator if isinstance(estimator, Pipeline) else Pipeline(estimator)
        self.items = []
        for stage, info, vals in grid.getItems():
            idx = next((i for i, s in enumerate(self.pipeline.stages) if s is stage), None)
            if idx is None:
                raise ValueError(f"stage {type(stage).__name__} of the grid is not in the estimator")
            self.items.append((idx, info, vals))
        self.counts = [1]
        for _, _, vals in self.items:
            self.counts.append(self.counts[-1] * len(vals))

    def size(self) -> int:
        return self.counts[-1]

    def get(self, index: int) -> Tuple[Pipeline, List[Tuple[int, ParamInfo, Any]]]:
        plist = []
        for i in range(len(self.items) - 1, -1, -1):
            k, index = divmod(index, self.counts[i])
            idx, info, vals = self.items[i]
            plist.append((idx, info, vals[k]))
        stages = [s.clone() for s in self.pipeline.stages]
        for idx, info, v in plist:
            stages[idx].getParams().set(info, v)
        return Pipeline(stages), plist


class Report:
    def __init__(self, elements: List[Tuple[Pipeline, List[Tuple[int, ParamInfo, Any]], float]]):
        self.elements = elements

    def toPrettyJson(self) -> str:
        out = []
        for pipe, plist, metric in self.elements:
            params = [{"stage": type(pipe.get(idx)).__name__, "paramName": info.name,
                       "paramValue": v.name if hasattr(v, "name") else v} for idx, info, v in plist]
            out.append({"param": params, "metric": None if metric is None or np.isnan(metric) else metric})
        return json.dumps(out, indent=2)

    def __str__(self):
        return self.toPrettyJson()


def _norm(s: str) -> str:
    return re.sub(r"[^a-z0-9]", "", s.lower())


class TuningEvaluator(WithParams):
    """Evaluates a transformed BatchOperator to ONE metric, looked up by name case-insensitively."""
    EVAL_OP = None
    SMALLER_BETTER = ()
    LARGER_BETTER = None

    def evaluate(self, op) -> float:
        metrics = self.EVAL_OP(self.getParams()).linkFrom(op).collectMetrics()
        want = _norm(self.getMetricName())
        aliases = {"ks": "ks", "auc": "auc", "prc": "prc"}
        want = aliases.get(want, want)
        for k in metrics.getParams()._m:
            if _norm(k) == want:
                return float(metrics.getParams().get(k, float))
        raise RuntimeError(f"Can not find {self.getMetricName()}")

    def isLargerBetter(self) -> bool:
        w = _norm(self.getMetricName())
        if self.LARGER_BETTER is not None:
            return w in self.LARGER_BETTER
        return w not in self.SMALLER_BETTER


def _eval_ops():
    from ..operator.batch import evaluation as E
    return E


class BinaryClassificationTuningEvaluator(TuningEvaluator):
    EXTRA_PARAMS = [ParamInfo("metricName", str, "metric name", default="AUC")]

    @property
    def EVAL_OP(self):
        return _eval_ops().EvalBinaryClassBatchOp


class MulticlassClassificationTuningEvaluator(TuningEvaluator):
    EXTRA_PARAMS = [ParamInfo("metricName", str, "metric name", default="Accuracy")]

    @property
    def EVAL_OP(self):
        return _eval_ops().EvalMultiClassBatchOp


class RegressionTuningEvaluator(TuningEvaluator):
    EXTRA_PARAMS = [ParamInfo("metricName", str, "metric name", default="RMSE")]
    SMALLER_BETTER = ("mse", "rmse", "mae")

    @property
    def EVAL_OP(self):
        return _eval_ops().EvalRegressionBatchOp


class ClusterTuningEvaluator(TuningEvaluator):
    EXTRA_PARAMS = [ParamInfo("metricName", str, "metric name", default="CalinskiHarabaz")]
    LARGER_BETTER = ("ssb", "calinskiharabaz", "ch")

    @property
    def EVAL_OP(self):
        return _eval_ops().EvalClusterBatchOp


class BaseTuningModel(ModelBase):
    def __init__(self, transformer: TransformerBase = None, report: Report = None, params: Optional[Params] = None):
        if isinstance(transformer, Params):
            transformer, params = None, transformer
        super().__init__(params)
        self.transformer = transformer
        self.report = report

    def getReport(self) -> Report:
        return self.report

    def getBestPipelineModel(self):
        return self.transformer

    def transformBatch(self, input):
        return self.transformer.transform(input)

    def transformStream(self, input):
        return self.transformer.transform(input)


class GridSearchCVModel(BaseTuningModel):
    pass


class GridSearchTVSplitModel(BaseTuningModel):
    pass


def _shuffled_rows(input_op, seed: int) -> Tuple[list, Any]:
    """Global rows in a random order identical on every rank (``BaseTuning.shuffle``)."""
    from ..operator.base import gather_table
    full = gather_table(input_op.getOutputTable())
    rng = np.random.default_rng(seed)
    rows = full.rows()
    order = rng.permutation(len(rows))
    return [rows[i] for i in order], full.schema


def _source(rows, schema):
    from ..operator.batch.source import MemSourceBatchOp
    from ..operator.base import partition_bounds
    from ..common.mlenv import MLEnvironmentFactory
    env = MLEnvironmentFactory.getDefault()
    lo, hi = partition_bounds(len(rows), env)
    mt = MTable.from_rows(rows[lo:hi], schema)
    from ..operator.batch.source import TableSourceBatchOp
    return TableSourceBatchOp(mt)


class _BaseGridSearch(EstimatorBase):
    MODEL_CLS = None
    EXTRA_PARAMS = [ParamInfo("randomSeed", int, "seed of the data shuffle", default=0)]
    _NO_AUTO_PARAMS = False

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(params, **kw)
        self.estimator = None
        self.paramGrid = None
        self.tuningEvaluator = None

    def setEstimator(self, e):
        self.estimator = e
        return self

    def getEstimator(self):
        return self.estimator

    def setParamGrid(self, g: ParamGrid):
        self.paramGrid = g
        return self

    def getParamGrid(self):
        return self.paramGrid

    def setTuningEvaluator(self, ev: TuningEvaluator):
        self.tuningEvaluator = ev
        return self

    def fitBatch(self, input):
        cands = PipelineCandidatesGrid(self.estimator, self.paramGrid)
        best, report = self._find_best(input, cands)
        return self.MODEL_CLS(best.fit(input), report)

    def _better(self, a, b):
        return (a > b) if self.tuningEvaluator.isLargerBetter() else (a < b)


class GridSearchCV(_BaseGridSearch):
    """k-fold cross validation over the grid; best = best mean metric (``findBestCV``)."""

    def _find_best(self, input, cands):
        k = int(self.get("NumFolds"))
        if k <= 1:
            raise ValueError("numFolds could be greater than 1.")
        rows, schema = _shuffled_rows(input, int(self.get("randomSeed")))
        n = len(rows)
        bounds = [(i * n // k, (i + 1) * n // k) for i in range(k)]
        best, best_avg, elements = None, None, []
        for i in range(cands.size()):
            pipe, plist = cands.get(i)
            vals = []
            for lo, hi in bounds:
                train = rows[:lo] + rows[hi:]
                test = rows[lo:hi]
                try:
                    model = pipe.fit(_source(train, schema))
                    vals.append(self.tuningEvaluator.evaluate(model.transform(_source(test, schema))))
                except Exception as ex:  # noqa: BLE001 - a failing fold is skipped like the reference
                    if comm.get_rank() == 0:
                        print(f"kFoldCv err, k: {k}, metric: NaN, exception: {ex}")
            avg = float(np.mean(vals)) if vals else float("nan")
            elements.append((pipe, plist, avg))
            if np.isnan(avg):
                continue
            if best_avg is None or self._better(avg, best_avg):
                best, best_avg = pipe, avg
        if best is None:
            raise RuntimeError("Can not find a best model.")
        return best, Report(elements)


class GridSearchTVSplit(_BaseGridSearch):
    """Train on ``trainRatio`` of the shuffled data, validate on the rest (``findBestTVSplit``)."""

    def _find_best(self, input, cands):
        ratio = float(self.get("trainRatio"))
        rows, schema = _shuffled_rows(input, int(self.get("randomSeed")))
        cut = int(round(len(rows) * ratio))
        train, test = rows[:cut], rows[cut:]
        best_i, best_m, elements = -1, None, []
        for i in range(cands.size()):
            pipe, plist = cands.get(i)
            try:
                m = self.tuningEvaluator.evaluate(pipe.fit(_source(train, schema)).transform(_source(test, schema)))
            except Exception as ex:  # noqa: BLE001
                if comm.get_rank() == 0:
                    print(f"BestTVSplit, i: {i}, exception: {ex}")
                elements.append((pipe, plist, float("nan")))
                continue
            elements.append((pipe, plist, m))
            if best_i == -1 or self._better(m, best_m):
                best_i, best_m = i, m
        if best_i < 0:
            raise RuntimeError("Can not find a best model.")
        return cands.get(best_i)[0], Report(elements)


GridSearchCV.MODEL_CLS = GridSearchCVModel
GridSearchTVSplit.MODEL_CLS = GridSearchTVSplitModel
