"""Multilayer perceptron classifier (reference ``MultilayerPerceptronClassifierTest.java``: iris, layers
[4, 5, 3], accuracy > 0.6; docs ``multilayerperceptronclassifier.md``).  Iris comes from scikit-learn's
bundled copy (the reference downloads it)."""
import json

import numpy as np
import pandas as pd
import pytest

from alink_amd import BatchOperator, MultilayerPerceptronClassifier, MultilayerPerceptronTrainBatchOp, \
    MultilayerPerceptronPredictBatchOp, MultilayerPerceptronPredictStreamOp, StreamOperator, CollectStreamOp
from alink_amd.common.jrandom import JavaRandom
from alink_amd.models.classification.mlp import weight_size


def _iris():
    from sklearn.datasets import load_iris
    d = load_iris()
    names = ["Iris-setosa", "Iris-versicolor", "Iris-virginica"]
    df = pd.DataFrame(d.data, columns=["sepal_length", "sepal_width", "petal_length", "petal_width"])
    df["category"] = [names[i] for i in d.target]
    return BatchOperator.fromDataframe(
        df, schemaStr="sepal_length double, sepal_width double, petal_length double, petal_width double, "
                      "category string"), df


FEATS = ["sepal_length", "sepal_width", "petal_length", "petal_width"]


def test_java_gaussian():
    r = JavaRandom(1)
    # java.util.Random(1).nextGaussian() x 2 (one polar draw: both values of the pair)
    got = [r.nextGaussian() for _ in range(2)]
    assert got == pytest.approx([1.561581040188955, -0.6081826070068602], abs=1e-15)


def test_mlpc_iris_accuracy():
    src, df = _iris()
    m = MultilayerPerceptronClassifier().setFeatureCols(FEATS).setLabelCol("category").setLayers([4, 5, 3]) \
        .setMaxIter(100).setPredictionCol("pred_label").setPredictionDetailCol("pred_detail").fit(src)
    out = m.transform(src).collectToDataframe()
    acc = (out["pred_label"].values == df["category"].values).mean()
    assert acc > 0.6
    det = json.loads(out["pred_detail"][0])
    assert set(det) == {"Iris-setosa", "Iris-versicolor", "Iris-virginica"}
    assert sum(det.values()) == pytest.approx(1.0)


def test_mlpc_model_format_and_stream():
    src, df = _iris()
    model = MultilayerPerceptronTrainBatchOp().setFeatureCols(FEATS).setLabelCol("category") \
        .setLayers([4, 5, 3]).setMaxIter(20).linkFrom(src)
    rows = model.collect()
    meta = json.loads(rows[0][1])
    assert json.loads(meta["layers"]) == [4, 5, 3]
    w = json.loads(rows[1][1])["data"]
    assert len(w) == weight_size([4, 5, 3]) == 43
    labels = sorted(r[2] for r in rows if r[2] is not None)
    assert labels == ["Iris-setosa", "Iris-versicolor", "Iris-virginica"]
    bp = MultilayerPerceptronPredictBatchOp().setPredictionCol("p").linkFrom(model, src).collectToDataframe()
    box = []
    MultilayerPerceptronPredictStreamOp(model).setPredictionCol("p").linkFrom(
        StreamOperator.fromDataframe(df, schemaStr="sepal_length double, sepal_width double, petal_length double, "
                                                   "petal_width double, category string")).link(CollectStreamOp(box))
    StreamOperator.execute()
    assert [r[-1] for r in box] == list(bp["p"])


def test_mlpc_vector_input_hidden_layers():
    rng = np.random.default_rng(0)
    X = rng.normal(size=(400, 6))
    y = ((X[:, 0] * X[:, 1] > 0) ^ (X[:, 2] > 0.5)).astype(int)
    df = pd.DataFrame({"vec": [" ".join(map(str, r)) for r in X], "label": y})
    src = BatchOperator.fromDataframe(df, schemaStr="vec string, label int")
    m = MultilayerPerceptronClassifier().setVectorCol("vec").setLabelCol("label").setLayers([6, 32, 2]) \
        .setMaxIter(300).setPredictionCol("p").fit(src)
    out = m.transform(src).collectToDataframe()
    assert (out["p"].values == y).mean() > 0.9
