"""Feature-engineering and statistics batch operators.

Reference: ``A/operator/batch/{dataproc,feature,statistics}/*`` — scalers/imputers (+ vector variants),
string indexers, one-hot, quantile discretizer, bucketizer, binarizer, feature hasher, DCT, summarizers,
correlation and chi-square tests.  Implementations live in ``models/feature`` and ``models/statistics``.
"""
from __future__ import annotations

from ...common.params import Params
from ...common.table import MTable
from ...common.types import TableSchema, Types
from ...models.feature import encoders as E
from ...models.feature import pca as PCA_
from ...models.feature import scalers as S
from ...models.statistics import summary as ST
from ..base import BatchOperator
from .utils import MapBatchOp, ModelMapBatchOp

__all__ = []


def _export(*names):
    __all__.extend(names)


class _FnTrainBatchOp(BatchOperator):
    """Train op whose model table is produced by ``train(mt, params, env)``."""

    def train(self, mt: MTable) -> MTable:
        raise NotImplementedError

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        self.setOutputTable(self.train(mt))
        return self


def _scaler_train(name, kind, vector=False):
    def train(self, mt):
        return (S.train_vector_scaler if vector else S.train_scaler)(kind, mt, self.getParams(), self.env)
    cls = type(name, (_FnTrainBatchOp,), {"train": train, "__module__": __name__})
    globals()[name] = cls
    _export(name)
    return cls


def _model_map(name, mapper):
    cls = type(name, (ModelMapBatchOp,), {"MAPPER": mapper, "__module__": __name__})
    globals()[name] = cls
    _export(name)
    return cls


def _map(name, mapper):
    cls = type(name, (MapBatchOp,), {"MAPPER": mapper, "__module__": __name__})
    globals()[name] = cls
    _export(name)
    return cls


for _k, _n in (("standard", "StandardScaler"), ("minmax", "MinMaxScaler"), ("maxabs", "MaxAbsScaler"),
               ("imputer", "Imputer")):
    _scaler_train(_n + "TrainBatchOp", _k)
    _scaler_train("Vector" + _n + "TrainBatchOp", _k, vector=True)

_model_map("StandardScalerPredictBatchOp", S.StandardScalerModelMapper)
_model_map("MinMaxScalerPredictBatchOp", S.MinMaxScalerModelMapper)
_model_map("MaxAbsScalerPredictBatchOp", S.MaxAbsScalerModelMapper)
_model_map("ImputerPredictBatchOp", S.ImputerModelMapper)
_model_map("VectorStandardScalerPredictBatchOp", S.VectorScalerModelMapper)
_model_map("VectorMinMaxScalerPredictBatchOp", S.VectorScalerModelMapper)
_model_map("VectorMaxAbsScalerPredictBatchOp", S.VectorScalerModelMapper)
_model_map("VectorImputerPredictBatchOp", S.VectorImputerModelMapper)


class StringIndexerTrainBatchOp(_FnTrainBatchOp):
    def train(self, mt):
        return E.train_string_indexer(mt, self.getParams())


class MultiStringIndexerTrainBatchOp(_FnTrainBatchOp):
    def train(self, mt):
        return E.train_multi_string_indexer(mt, self.getParams())


class OneHotTrainBatchOp(_FnTrainBatchOp):
    def train(self, mt):
        return E.train_one_hot(mt, self.getParams())


class QuantileDiscretizerTrainBatchOp(_FnTrainBatchOp):
    def train(self, mt):
        return E.train_quantile_discretizer(mt, self.getParams())


_export("StringIndexerTrainBatchOp", "MultiStringIndexerTrainBatchOp", "OneHotTrainBatchOp",
        "QuantileDiscretizerTrainBatchOp")
_model_map("StringIndexerPredictBatchOp", E.StringIndexerModelMapper)
_model_map("MultiStringIndexerPredictBatchOp", E.MultiStringIndexerModelMapper)
_model_map("IndexToStringPredictBatchOp", E.IndexToStringModelMapper)
_model_map("OneHotPredictBatchOp", E.OneHotModelMapper)
_model_map("QuantileDiscretizerPredictBatchOp", E.QuantileDiscretizerModelMapper)
_map("BucketizerBatchOp", E.BucketizerMapper)
_map("BinarizerBatchOp", E.BinarizerMapper)
_map("FeatureHasherBatchOp", E.FeatureHasherMapper)
_map("DCTBatchOp", E.DCTMapper)


# ---------------------------------------------------------------------------------------------------
# statistics
# ---------------------------------------------------------------------------------------------------
class SummarizerBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        cols = p.get("selectedCols") if p.contains("selectedCols") else None
        t = ST.table_summary(mt, cols, self.env.device)
        conv = ST.SummaryDataConverter()
        self.setOutputTable(MTable.from_rows(conv.save(t), conv.getModelSchema(), replicated=True))
        return self

    def collectSummary(self) -> ST.TableSummary:
        return ST.SummaryDataConverter().load(self.collect())

    def lazyCollectSummary(self, *callbacks):
        def cb(rows):
            s = ST.SummaryDataConverter().load(rows)
            for c in callbacks:
                c(s)
        return self.lazyCollect(cb)

    def lazyPrintSummary(self, title=None):
        def cb(s):
            if title:
                print(title)
            print(s)
        return self.lazyCollectSummary(cb)


class VectorSummarizerBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        vs = ST.vector_summary(mt, self.getParams().get("selectedCol"), self.env.device)
        conv = ST.VectorSummaryDataConverter()
        self.setOutputTable(MTable.from_rows(conv.save(vs), conv.getModelSchema(), replicated=True))
        return self

    def collectVectorSummary(self) -> ST.VectorSummary:
        return ST.VectorSummaryDataConverter().load(self.collect())

    def lazyPrintVectorSummary(self, title=None):
        def cb(rows):
            if title:
                print(title)
            print(ST.VectorSummaryDataConverter().load(rows))
        return self.lazyCollect(cb)


_CORR_SCHEMA = TableSchema(["model_id", "model_info"], [Types.LONG, Types.STRING])


def _corr_rows(res: ST.CorrelationResult):
    import json
    arr = res.getCorrelation()
    data = json.dumps({"colNames": res.colNames, "correlation": [[float(x) for x in r] for r in arr]})
    return [(0, data)]


def _corr_load(rows):
    import json
    import numpy as np
    d = json.loads(rows[0][1])
    return ST.CorrelationResult(np.asarray(d["correlation"]), d["colNames"])


class CorrelationBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        cols = p.get("selectedCols") if p.contains("selectedCols") and p.get("selectedCols") else \
            [n for n, t in zip(mt.schema.names, mt.schema.types) if t in (Types.DOUBLE, Types.FLOAT, Types.LONG,
                                                                         Types.INT, Types.SHORT, Types.BYTE)]
        method = str(getattr(p.get("method"), "name", p.get("method"))) if p.contains("method") else "PEARSON"
        res = ST.correlation(mt, cols, method, self.env.device)
        self.setOutputTable(MTable.from_rows(_corr_rows(res), _CORR_SCHEMA, replicated=True))
        return self

    def collectCorrelation(self) -> ST.CorrelationResult:
        return _corr_load(self.collect())

    def lazyPrintCorrelation(self, title=None):
        def cb(rows):
            if title:
                print(title)
            print(_corr_load(rows))
        return self.lazyCollect(cb)


class VectorCorrelationBatchOp(CorrelationBatchOp):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        method = str(getattr(p.get("method"), "name", p.get("method"))) if p.contains("method") else "PEARSON"
        res = ST.vector_correlation(mt, p.get("selectedCol"), method, self.env.device)
        self.setOutputTable(MTable.from_rows(_corr_rows(res), _CORR_SCHEMA, replicated=True))
        return self


_CHI_SCHEMA = TableSchema(["col", "chisquare_test"], [Types.STRING, Types.STRING])


def _chi_rows(results):
    from ...common.javafmt import gson_dumps
    return [(r.colName, gson_dumps(r)) for r in results]


class ChiSquareTestBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        cols = list(p.get("selectedCols"))
        label = mt.column_values(p.get("labelCol"))
        pairs = []
        for c in cols:
            d = {}
            for v, l in zip(mt.column_values(c), label):
                if v is None or l is None:
                    continue
                k = (str(v), str(l))
                d[k] = d.get(k, 0) + 1
            pairs.append(sorted(d.items()))
        res = ST.chi_square_test(pairs, cols)
        self.setOutputTable(MTable.from_rows(_chi_rows(res), _CHI_SCHEMA, replicated=True))
        return self

    def collectChiSquareTest(self):
        import json
        return [ST.ChiSquareTestResult(json.loads(r[1])["df"], json.loads(r[1])["p"], json.loads(r[1])["value"],
                                       col=r[0]) for r in self.collect()]


class VectorChiSquareTestBatchOp(ChiSquareTestBatchOp):
    def linkFrom(self, *inputs):
        from ...common.linalg import SparseVector, VectorUtil
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        label = mt.column_values(p.get("labelCol"))
        vecs = [VectorUtil.getVector(v) if v is not None else None for v in mt.column_values(p.get("selectedCol"))]
        d = max([v.size() for v in vecs if v is not None] + [0])
        from ...parallel import comm
        d = max(comm.all_gather_object(d))
        pairs = [dict() for _ in range(d)]
        for v, l in zip(vecs, label):
            if v is None or l is None:
                continue
            dense = v.toDenseVector().data if isinstance(v, SparseVector) else v.data
            for j in range(d):
                x = float(dense[j]) if j < len(dense) else 0.0
                k = (repr(x), str(l))
                pairs[j][k] = pairs[j].get(k, 0) + 1
        res = ST.chi_square_test([sorted(x.items()) for x in pairs], [str(j) for j in range(d)])
        self.setOutputTable(MTable.from_rows(_chi_rows(res), _CHI_SCHEMA, replicated=True))
        return self


_export("SummarizerBatchOp", "VectorSummarizerBatchOp", "CorrelationBatchOp", "VectorCorrelationBatchOp",
        "ChiSquareTestBatchOp", "VectorChiSquareTestBatchOp")


# ---------------------------------------------------------------------------------------------------
# PCA and chi-square feature selection
# ---------------------------------------------------------------------------------------------------
class PcaTrainBatchOp(_FnTrainBatchOp):
    def train(self, mt):
        from ...common.model.converter import SimpleModelDataConverter
        rows = PCA_.train_pca(mt, self.getParams(), self.env)
        return MTable.from_rows(rows, SimpleModelDataConverter().getModelSchema(), replicated=True)


_export("PcaTrainBatchOp")
_model_map("PcaPredictBatchOp", PCA_.PcaModelMapper)


def _chisq_select(results, p: Params):
    """``ChiSquareTest.selector``: rows (index, p-value) -> selected indices."""
    st = str(getattr(p.get("selectorType"), "name", p.get("selectorType"))).upper() \
        if p.contains("selectorType") and p.get("selectorType") is not None else "NUMTOPFEATURES"
    g = lambda k, d: p.get(k) if p.contains(k) and p.get(k) is not None else d  # noqa: E731
    rows = [(i, r.p) for i, r in enumerate(results)]
    n = len(rows)
    asc = sorted(rows, key=lambda t: (t[1], t[0]))
    if st == "NUMTOPFEATURES":
        sel = [i for i, _ in asc[:int(g("numTopFeatures", 50))]]
    elif st == "PERCENTILE":
        size = max(1, int(n * float(g("percentile", 0.1))))
        sel = [i for i, _ in asc[:size]]
    elif st == "FPR":
        sel = [i for i, pv in rows if pv < float(g("fpr", 0.05))]
    elif st == "FDR":
        fdr = float(g("fdr", 0.05))
        mx = 0
        for k, (_, pv) in enumerate(asc):
            if pv <= fdr * (k + 1) / n:
                mx = k
        sel = sorted(i for i, _ in asc[:mx + 1])
    elif st == "FWE":
        sel = [i for i, pv in rows if pv <= float(g("fwe", 0.05)) / n]
    else:
        raise ValueError(f"Selector Type not support. {st}")
    return sel


class ChiSqSelectorBatchOp(BatchOperator):
    """Chi-square feature selection over ``selectedCols`` (reference ``ChiSqSelectorBatchOp`` ->
    ``ChiSquareTestUtil.selector``); output = model table with the selected column indices (JSON int[])."""

    def linkFrom(self, *inputs):
        from ...common.model.converter import SimpleModelDataConverter
        inp = self.checkAndGetFirst(inputs)
        p = self.getParams()
        test = ChiSquareTestBatchOp(p.clone()).linkFrom(inp)
        import json as _json
        res = [ST.ChiSquareTestResult(_json.loads(r[1])["df"], _json.loads(r[1])["p"], _json.loads(r[1])["value"],
                                      col=r[0]) for r in test.collect()]
        sel = _chisq_select(res, p)
        rows = SimpleModelDataConverter.rows_from(Params(), [_json.dumps(sel, separators=(",", ":"))])
        self.setOutputTable(MTable.from_rows(rows, SimpleModelDataConverter().getModelSchema(), replicated=True))
        return self

    def collectResult(self):
        """As the reference (``ChiSqSelectorBatchOp.collectResult``): the first ``len(selected)`` names of
        ``selectedCols`` — the docs example output depends on it; ``selectedIndices()`` gives the indices."""
        cols = list(self.getParams().get("selectedCols"))
        return [cols[i] for i in range(len(self.selectedIndices()))]

    def selectedIndices(self):
        import json as _json
        return _json.loads(self.collect()[1][1])


class VectorChiSqSelectorBatchOp(ChiSqSelectorBatchOp):
    def linkFrom(self, *inputs):
        from ...common.model.converter import SimpleModelDataConverter
        import json as _json
        inp = self.checkAndGetFirst(inputs)
        p = self.getParams()
        test = VectorChiSquareTestBatchOp(p.clone()).linkFrom(inp)
        res = [ST.ChiSquareTestResult(_json.loads(r[1])["df"], _json.loads(r[1])["p"], _json.loads(r[1])["value"],
                                      col=r[0]) for r in test.collect()]
        sel = _chisq_select(res, p)
        rows = SimpleModelDataConverter.rows_from(Params(), [_json.dumps(sel, separators=(",", ":"))])
        self.setOutputTable(MTable.from_rows(rows, SimpleModelDataConverter().getModelSchema(), replicated=True))
        return self

    def collectResult(self):
        import json as _json
        return _json.loads(self.collect()[1][1])


_export("ChiSqSelectorBatchOp", "VectorChiSqSelectorBatchOp")
