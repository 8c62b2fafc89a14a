"""Evaluation ops vs the reference docs (docs/en/eval*.md script examples)."""
import json

import numpy as np
import pandas as pd
import pytest

from alink_amd import (BatchOperator, EvalBinaryClassBatchOp, EvalClusterBatchOp, EvalMultiClassBatchOp,
                       EvalRegressionBatchOp, EvalBinaryClassStreamOp, StreamOperator, CollectStreamOp)

DATA = [["prefix1", '{"prefix1": 0.9, "prefix0": 0.1}'], ["prefix1", '{"prefix1": 0.8, "prefix0": 0.2}'],
        ["prefix1", '{"prefix1": 0.7, "prefix0": 0.3}'], ["prefix0", '{"prefix1": 0.75, "prefix0": 0.25}'],
        ["prefix0", '{"prefix1": 0.6, "prefix0": 0.4}']]


def _in():
    df = pd.DataFrame({"label": [r[0] for r in DATA], "detailInput": [r[1] for r in DATA]})
    return BatchOperator.fromDataframe(df, schemaStr="label string, detailInput string"), df


def test_eval_binary_doc():
    op, _ = _in()
    m = EvalBinaryClassBatchOp().setLabelCol("label").setPredictionDetailCol("detailInput").linkFrom(op) \
        .collectMetrics()
    assert m.getAuc() == pytest.approx(0.8333333333333333, abs=1e-15)
    assert m.getKs() == pytest.approx(0.6666666666666666, abs=1e-15)
    assert m.getPrc() == pytest.approx(0.9027777777777777, abs=1e-15)
    assert m.getAccuracy() == pytest.approx(0.6)
    assert m.getMacroPrecision() == pytest.approx(0.3)
    assert m.getMicroRecall() == pytest.approx(0.6)
    assert m.getWeightedSensitivity() == pytest.approx(0.6)
    assert m.getLabelArray() == ["prefix1", "prefix0"]
    assert len(m.getThresholdArray()) == len(m.getPrecisionArray())


def test_eval_multi_doc():
    op, _ = _in()
    m = EvalMultiClassBatchOp().setLabelCol("label").setPredictionDetailCol("detailInput").linkFrom(op) \
        .collectMetrics()
    assert m.getAccuracy("prefix0") == pytest.approx(0.6)
    assert m.getRecall("prefix1") == pytest.approx(1.0)
    assert m.getMacroPrecision() == pytest.approx(0.3)
    assert m.getMicroRecall() == pytest.approx(0.6)
    assert m.getWeightedSensitivity() == pytest.approx(0.6)
    assert m.getConfusionMatrix().tolist() == [[3, 2], [0, 0]]


def test_eval_regression_doc():
    d = np.array([[0, 0], [8, 8], [1, 2], [9, 10], [3, 1], [10, 7]])
    op = BatchOperator.fromDataframe(pd.DataFrame({"pred": d[:, 0], "label": d[:, 1]}),
                                     schemaStr="pred int, label int")
    m = EvalRegressionBatchOp().setPredictionCol("pred").setLabelCol("label").linkFrom(op).collectMetrics()
    assert m.getCount() == 6.0 and m.getSse() == 15.0 and m.getSae() == 7.0
    assert m.getRmse() == pytest.approx(1.5811388300841898, abs=1e-15)
    assert m.getR2() == pytest.approx(0.8282442748091603, abs=1e-15)


def test_eval_cluster_doc():
    df = pd.DataFrame({"id": [0, 0, 0, 1, 1, 1],
                       "vec": ["0 0 0", "0.1,0.1,0.1", "0.2,0.2,0.2", "9 9 9", "9.1 9.1 9.1", "9.2 9.2 9.2"]})
    op = BatchOperator.fromDataframe(df, schemaStr="id int, vec string")
    m = EvalClusterBatchOp().setVectorCol("vec").setPredictionCol("id").linkFrom(op).collectMetrics()
    assert m.getCount() == 6 and m.getK() == 2
    assert m.getClusterArray() == ["0", "1"] and m.getCountArray() == [3.0, 3.0]
    assert m.getCompactness() == pytest.approx(0.11547005383792497, rel=1e-12)
    assert m.getDaviesBouldin() == pytest.approx(0.014814814814814791, rel=1e-10)
    assert m.getSeperation() == pytest.approx(15.588457268119896, rel=1e-12)
    assert m.getSsb() == pytest.approx(364.5, rel=1e-12)
    assert m.getSsw() == pytest.approx(0.12, rel=1e-9)
    assert m.getCalinskiHarabaz() == pytest.approx(12150.0, rel=1e-9)
    assert 0.9 < m.getSilhouetteCoefficient() <= 1.0


def test_eval_binary_stream_window_and_all():
    _, df = _in()
    box = []
    src = StreamOperator.fromDataframe(df, schemaStr="label string, detailInput string")
    EvalBinaryClassStreamOp().setLabelCol("label").setPredictionDetailCol("detailInput").linkFrom(src) \
        .link(CollectStreamOp(box))
    StreamOperator.execute()
    assert [r[0] for r in box] == ["window", "all"]
    auc = json.loads(json.loads(box[1][1])["AUC"])
    assert auc == pytest.approx(0.8333333333333333)


def test_eval_stream_processing_time_windows(monkeypatch):
    """Windows follow ``timeInterval`` (reference ``timeWindowAll``): 0 -> one window per micro-batch; the default
    3 s over a sub-second stream -> one window flushed at the end.  The final "all" row is the same either way."""
    monkeypatch.setenv("ALINK_STREAM_BATCH", "2")
    _, df = _in()
    out = {}
    for ti in (0, None):
        box = []
        src = StreamOperator.fromDataframe(df, schemaStr="label string, detailInput string")
        op = EvalBinaryClassStreamOp().setLabelCol("label").setPredictionDetailCol("detailInput")
        if ti is not None:
            op.setTimeInterval(ti)
        op.linkFrom(src).link(CollectStreamOp(box))
        StreamOperator.execute()
        out[ti] = box
    assert [r[0] for r in out[0]] == ["window", "all"] * 3            # 5 rows in micro-batches of 2
    assert [r[0] for r in out[None]] == ["window", "all"]
    assert out[0][-1][1] == out[None][-1][1] == out[None][0][1]
    win = [json.loads(r[1]) for r in out[0] if r[0] == "window"]
    assert [int(json.loads(w["TotalSamples"])) for w in win] == [2, 2, 1]


def test_binary_eval_on_columnar_detail_equals_string_detail():
    """EvalBinaryClassBatchOp / EvalBinaryClassStreamOp on a LinearModelMapper detail column (columnar
    DetailBlock: probabilities, no strings) give the same metrics as on the materialised JSON strings."""
    import numpy as np
    import pandas as pd
    from alink_amd import (BatchOperator, LogisticRegressionTrainBatchOp, LogisticRegressionPredictBatchOp,
                           EvalBinaryClassBatchOp)
    from alink_amd.common.detail import DetailBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.operator.batch.source import TableSourceBatchOp
    rng = np.random.default_rng(3)
    X = rng.normal(size=(3000, 4))
    y = (X @ np.array([1.0, -0.5, 0.3, 0.0]) + 0.5 * rng.normal(size=3000) > 0).astype(int)
    df = pd.DataFrame({f"x{i}": X[:, i] for i in range(4)})
    df["y"] = y
    src = BatchOperator.fromDataframe(df, schemaStr="x0 double, x1 double, x2 double, x3 double, y int")
    model = LogisticRegressionTrainBatchOp().setFeatureCols([f"x{i}" for i in range(4)]).setLabelCol("y") \
        .linkFrom(src)
    pred = LogisticRegressionPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d") \
        .linkFrom(model, src)
    mt = pred.getOutputTable()
    di = mt.schema.names.index("d")
    assert isinstance(mt.cols[di].values, DetailBlock)
    strs = MTable(mt.schema, [c if i != di else Column(c.to_list()) for i, c in enumerate(mt.cols)])
    a = EvalBinaryClassBatchOp().setLabelCol("y").setPredictionDetailCol("d").linkFrom(pred).collectMetrics()
    b = EvalBinaryClassBatchOp().setLabelCol("y").setPredictionDetailCol("d") \
        .linkFrom(TableSourceBatchOp(strs)).collectMetrics()
    for name in ("AUC", "LogLoss", "Accuracy", "PRC", "F1", "Precision"):
        assert getattr(a, "get" + name)() == getattr(b, "get" + name)(), name


def test_binary_metrics_from_bins_reference_values():
    """BinaryClassMetricsTest.saveAsParamsTest (reference operator/common/evaluation): positive bins at 0.7 / 0.8 /
    0.9, negative bins at 0.6 / 0.75, log loss 2.987 over 5 samples -> the doc's metric values."""
    from alink_amd.models.evaluation import metrics as M
    pos = np.zeros(M.DETAIL_BIN_NUMBER)
    neg = np.zeros(M.DETAIL_BIN_NUMBER)
    pos[[70000, 80000, 90000]] = 1
    neg[[60000, 75000]] = 1
    m = M.binary_metrics(pos, neg, ["0", "1"], 2.987, 5)
    expect = {"Prc": 0.9027777777777777, "MacroRecall": 0.5, "MacroSpecificity": 0.5, "Auc": 0.8333333333333333,
              "MacroAccuracy": 0.6, "MicroFalseNegativeRate": 0.4, "WeightedRecall": 0.6, "WeightedPrecision": 0.36,
              "MacroPrecision": 0.3, "MicroTruePositiveRate": 0.6, "MacroKappa": 0.0, "MicroSpecificity": 0.6,
              "MacroF1": 0.375, "WeightedKappa": 0.0, "WeightedTruePositiveRate": 0.6, "TotalSamples": 5,
              "MicroTrueNegativeRate": 0.6, "MicroSensitivity": 0.6, "WeightedAccuracy": 0.6,
              "Ks": 0.6666666666666666, "Accuracy": 0.6, "WeightedFalseNegativeRate": 0.4, "MicroF1": 0.6,
              "WeightedSpecificity": 0.4, "WeightedF1": 0.45, "MicroAccuracy": 0.6, "WeightedTrueNegativeRate": 0.4,
              "Kappa": 0.0, "MacroSensitivity": 0.5, "WeightedSensitivity": 0.6, "MicroRecall": 0.6,
              "MicroFalsePositiveRate": 0.4, "WeightedFalsePositiveRate": 0.6, "MicroPrecision": 0.6,
              "MacroTrueNegativeRate": 0.5, "MicroKappa": 0.2}
    for name, v in expect.items():
        assert getattr(m, "get" + name)() == pytest.approx(v, abs=0.01), name
    assert m.getLogLoss() == pytest.approx(2.987 / 5)


def _ref_cluster_metrics(X, cid, dist):
    """The reference ClusterEvaluationUtil / ClusterMetricsSummary formulas, written out in numpy."""
    ks = sorted(set(cid))
    if dist != "EUCLIDEAN":
        X = X / np.linalg.norm(X, axis=1, keepdims=True)

    def d(a, b):
        if dist == "COSINE":
            return 1.0 - a @ b / (np.linalg.norm(a) * np.linalg.norm(b))
        if dist == "CITYBLOCK":
            return np.abs(a - b).sum()
        return np.linalg.norm(a - b)
    mean = {k: X[cid == k].mean(0) for k in ks}
    cnt = {k: int((cid == k).sum()) for k in ks}
    dsum = {k: sum(d(mean[k], x) for x in X[cid == k]) for k in ks}
    d2 = {k: sum(d(mean[k], x) ** 2 for x in X[cid == k]) for k in ks}
    n2 = {k: float((X[cid == k] ** 2).sum()) for k in ks}
    gmean = sum(mean[k] * cnt[k] for k in ks) / len(X)
    ssb = sum(d(mean[k], gmean) ** 2 * cnt[k] for k in ks)
    ssw = sum(d2.values())
    comp = {k: dsum[k] / cnt[k] for k in ks}
    sil = 0.0
    for x, c in zip(X, cid):
        cur, nb = 0.0, np.inf
        for k in ks:
            if dist == "EUCLIDEAN":
                dis = cnt[k] * (x @ x) - 2 * cnt[k] * (x @ mean[k]) + n2[k]
                if k == c:
                    cur = dis / (cnt[k] - 1) if cnt[k] > 1 else 0.0
                else:
                    nb = min(nb, dis / cnt[k])
            else:
                dis = 1.0 - x @ mean[k]
                if k == c:
                    cur = dis * cnt[k] / (cnt[k] - 1) if cnt[k] > 1 else 0.0
                else:
                    nb = min(nb, dis)
        sil += 1 - cur / nb if cur < nb else nb / cur - 1
    return {"Ssb": ssb, "Ssw": ssw, "Compactness": sum(comp.values()) / len(ks),
            "SilhouetteCoefficient": sil / len(X)}


@pytest.mark.parametrize("dist", ["EUCLIDEAN", "COSINE", "CITYBLOCK"])
def test_eval_cluster_distance_types_match_reference_formulas(dist):
    from alink_amd import EvalClusterBatchOp
    rng = np.random.default_rng(4)
    X = np.abs(rng.normal(size=(60, 3))) + np.repeat(np.eye(3) * 3, 20, axis=0)
    cid = np.repeat(np.arange(3), 20)
    df = pd.DataFrame({"vec": [" ".join(map(str, r)) for r in X], "pred": cid})
    src = BatchOperator.fromDataframe(df, schemaStr="vec string, pred int")
    m = EvalClusterBatchOp().setVectorCol("vec").setPredictionCol("pred").setDistanceType(dist).linkFrom(src) \
        .collectMetrics()
    for name, v in _ref_cluster_metrics(X, cid, dist).items():
        assert getattr(m, "get" + name)() == pytest.approx(v, rel=1e-9, abs=1e-12), name


def test_multiclass_metrics_reference_values():
    """MultiClassMetricsTest.saveAsParamsTest (reference operator/common/evaluation)."""
    from alink_amd.models.evaluation import metrics as M
    m = M.multi_metrics(np.array([[0, 3, 1], [1, 1, 1], [2, 0, 4]], dtype=np.float64), ["0", "1", "2"], 0.4, 13)
    expect = {"MacroRecall": 0.3055555555555555, "MacroSpecificity": 0.6973544973544974,
              "MacroAccuracy": 0.5897435897435898, "MicroFalseNegativeRate": 0.6153846153846154,
              "WeightedRecall": 0.38461538461538464, "WeightedPrecision": 0.41025641025641024,
              "MacroPrecision": 0.3333333333333333, "MicroTruePositiveRate": 0.38461538461538464,
              "MacroKappa": 0.01753139066571909, "MicroSpecificity": 0.6923076923076923,
              "MacroF1": 0.31746031746031744, "WeightedKappa": 0.10234541577825165,
              "WeightedTruePositiveRate": 0.38461538461538464, "MicroTrueNegativeRate": 0.6923076923076923,
              "MicroSensitivity": 0.38461538461538464, "WeightedAccuracy": 0.6153846153846154,
              "Accuracy": 0.38461538461538464, "WeightedFalseNegativeRate": 0.6153846153846154,
              "MicroF1": 0.38461538461538464, "WeightedSpecificity": 0.7074481074481075,
              "WeightedF1": 0.39560439560439564, "MicroAccuracy": 0.5897435897435898,
              "WeightedTrueNegativeRate": 0.7074481074481075, "Kappa": 0.04587155963302759,
              "MacroSensitivity": 0.3055555555555555, "WeightedSensitivity": 0.38461538461538464,
              "MicroRecall": 0.38461538461538464, "MacroFalseNegativeRate": 0.6944444444444445,
              "MicroFalsePositiveRate": 0.3076923076923077, "WeightedFalsePositiveRate": 0.29255189255189257,
              "MicroPrecision": 0.38461538461538464, "MacroTrueNegativeRate": 0.6973544973544974,
              "MicroKappa": 0.0769230769230769}
    for name, v in expect.items():
        assert getattr(m, "get" + name)() == pytest.approx(v, rel=1e-9, abs=1e-12), name
    assert m.getLogLoss() == pytest.approx(0.4 / 13)


def test_regression_metrics_reference_values():
    """RegressionMetricsTest.saveAsParamsTest: sums (y, y^2, pred, pred^2, mae, sse, mape, total)."""
    from alink_amd.models.evaluation import metrics as M
    m = M.regression_metrics(np.array([1.6, 0.66, 2.8, 1.599, 1.2, 0.38, 7.08, 5]))
    for name, v in {"R2": -1.56, "Sse": 0.38, "Mape": 141.6, "Rmse": 0.27, "Mae": 0.24, "Ssr": 0.31}.items():
        assert getattr(m, "get" + name)() == pytest.approx(v, abs=0.01), name


def test_detail_json_label_with_percent():
    """Labels containing '%' survive the per-table detail template (it is %-formatted)."""
    from alink_amd.models.linear.model import _detail_json
    out = _detail_json(["50%", "a%s"], np.array([[0.25, 0.75], [1.0, 0.0]]))
    assert [json.loads(s) for s in out] == [{"50%": "0.25", "a%s": "0.75"}, {"50%": "1.0", "a%s": "0.0"}]


def test_multiclass_and_regression_eval_tensor_columns_equal_lists():
    """EvalMultiClass (prediction column) and EvalRegression on tensor columns (no per-row Python) give the
    metrics of the list columns: nulls in either column, labels seen only in predictions."""
    import torch
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    import alink_amd as A
    g = torch.Generator().manual_seed(0)
    n = 500
    lab = torch.randint(0, 4, (n,), generator=g)
    pred = torch.randint(0, 5, (n,), generator=g)
    ln = torch.rand(n, generator=g) < 0.05
    pn = torch.rand(n, generator=g) < 0.05
    to_list = lambda v, m: [None if m[i] else int(v[i]) for i in range(n)]  # noqa: E731
    s = TableSchema(["l", "p"], [Types.LONG, Types.LONG])
    outs = []
    for mt in (MTable(s, [Column(lab, ln), Column(pred, pn)]),
               MTable(s, [Column(to_list(lab, ln)), Column(to_list(pred, pn))])):
        outs.append(A.EvalMultiClassBatchOp().setLabelCol("l").setPredictionCol("p")
                    .linkFrom(TableSourceBatchOp(mt)).collect()[0][0])
    assert outs[0] == outs[1]
    y = torch.randn(n, generator=g, dtype=torch.float64)
    yp = y + 0.1 * torch.randn(n, generator=g, dtype=torch.float64)
    s = TableSchema(["l", "p"], [Types.DOUBLE, Types.DOUBLE])
    outs = []
    for mt in (MTable(s, [Column(y, ln), Column(yp)]),
               MTable(s, [Column([None if ln[i] else float(y[i]) for i in range(n)]), Column(yp.tolist())])):
        outs.append(A.EvalRegressionBatchOp().setLabelCol("l").setPredictionCol("p")
                    .linkFrom(TableSourceBatchOp(mt)).collect()[0][0])
    assert outs[0] == outs[1]
