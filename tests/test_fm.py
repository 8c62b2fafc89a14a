"""Factorization machine classifier / regressor: learns pairwise interactions, model round trip, stages,
multi-process model averaging (gloo).  Parity unpinned: the reference ships no FM doc outputs."""
import json

import numpy as np

from alink_amd import *  # noqa: F401,F403
from alink_amd.models.recommendation.fm import FmModelDataConverter
from alink_amd.common.types import Types


def _data(n=1500, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 6))
    return X


def test_fm_regressor_learns_interaction():
    X = _data()
    y = 2 * X[:, 0] * X[:, 1] + X[:, 3]
    src = MemSourceBatchOp([(" ".join(map(str, x)), float(t)) for x, t in zip(X.tolist(), y)], "vec string, y double")
    m = FmRegressor().setVectorCol("vec").setLabelCol("y").setNumEpochs(50).setLearnRate(0.1).setNumFactor(4) \
        .setPredictionCol("p").fit(src)
    out = m.transform(src).collect()
    rmse = np.sqrt(np.mean([(r[1] - r[2]) ** 2 for r in out]))
    assert rmse < 0.1 * y.std()


def test_fm_classifier_detail_and_model_format():
    X = _data(seed=1)
    logit = 3.0 * X[:, 0] * X[:, 1] - 2.0 * X[:, 2]
    y = np.where(logit > 0, "b", "a")
    src = MemSourceBatchOp([(float(a), float(b), float(c), str(t)) for (a, b, c), t in zip(X[:, :3].tolist(), y)],
                           "f0 double, f1 double, f2 double, label string")
    train = FmClassifierTrainBatchOp().setFeatureCols(["f0", "f1", "f2"]).setLabelCol("label") \
        .setNumEpochs(60).setLearnRate(0.1).setNumFactor(4)
    model = src.link(train)
    pred = FmClassifierPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d").linkFrom(model, src) \
        .collect()
    acc = np.mean([r[4] == r[3] for r in pred])
    assert acc > 0.9
    d = json.loads(pred[0][5])
    assert set(d) == {"a", "b"} and abs(float(d["a"]) + float(d["b"]) - 1) < 1e-12
    m = FmModelDataConverter(Types.STRING).load(model.collect())
    assert m.task == "BINARY_CLASSIFICATION" and m.labelValues[0] == "b" and m.dim == [1, 1, 4]
    assert len(m.fmModel.factors) == 3 and len(m.fmModel.factors[0]) == 4


def test_generic_fm_ops_equal_task_specific_ops():
    """FmTrainBatchOp(task) / FmPredictBatchOp (A/operator/common/fm/FmTrainBatchOp.java:17, FmPredictBatchOp.java:12)
    train the same model as the classifier / regressor ops and predict the same rows."""
    import pytest
    X = _data(400, seed=3)
    y = np.where(X[:, 0] * X[:, 1] > 0, "p", "n")
    yr = X[:, 0] * X[:, 1] + 0.5 * X[:, 2]
    src = MemSourceBatchOp([(" ".join(map(str, x)), str(a), float(b)) for x, a, b in zip(X.tolist(), y, yr)],
                           "vec string, label string, y double")
    for task, spec_cls, label in (("binary_classification", FmClassifierTrainBatchOp, "label"),
                                  ("REGRESSION", FmRegressorTrainBatchOp, "y")):
        def conf(op):
            return op.setVectorCol("vec").setLabelCol(label).setNumEpochs(5).setNumFactor(3).setLearnRate(0.05)
        a = src.link(conf(FmTrainBatchOp(task)))
        b = src.link(conf(spec_cls()))
        assert a.collect() == b.collect()
        pa = FmPredictBatchOp().setPredictionCol("p").linkFrom(a, src).collect()
        pb = (FmClassifierPredictBatchOp() if label == "label" else FmRegressorPredictBatchOp()) \
            .setPredictionCol("p").linkFrom(b, src).collect()
        assert pa == pb
    c = src.link(FmTrainBatchOp().setTask("regression").setVectorCol("vec").setLabelCol("y").setNumEpochs(5)
                 .setNumFactor(3).setLearnRate(0.05))
    assert c.collect() == src.link(FmRegressorTrainBatchOp().setVectorCol("vec").setLabelCol("y").setNumEpochs(5)
                                   .setNumFactor(3).setLearnRate(0.05)).collect()
    with pytest.raises(ValueError):
        src.link(FmTrainBatchOp().setVectorCol("vec").setLabelCol("y"))
