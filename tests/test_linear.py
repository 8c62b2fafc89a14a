"""Linear family vs the reference's documented outputs (docs/en/*.md script examples)."""
import json

import numpy as np
import pandas as pd
import pytest

from alink_amd import (AftSurvivalRegression, BatchOperator, LinearRegression, LinearSvm, LogisticRegression,
                       Pipeline, PipelineModel, RidgeRegression, LassoRegression, Softmax, useLocalEnv,
                       LogisticRegressionTrainBatchOp, LogisticRegressionPredictBatchOp)

DATA = np.array([[2, 1, 1], [3, 2, 1], [4, 3, 2], [2, 4, 1], [2, 2, 1], [4, 3, 2], [1, 2, 1], [5, 3, 3]])


def _op(label_last=3):
    d = DATA.copy()
    d[7, 2] = label_last
    df = pd.DataFrame({"f0": d[:, 0], "f1": d[:, 1], "label": d[:, 2]})
    return BatchOperator.fromDataframe(df, schemaStr="f0 int, f1 int, label int")


def test_linear_regression_doc_example():
    b = _op()
    m = LinearRegression().setFeatureCols(["f0", "f1"]).setLabelCol("label").setPredictionCol("pred").fit(b)
    got = m.transform(b).collectToDataframe()["pred"].values
    ref = [1.000014, 1.538474, 2.076934, 1.138446, 1.046158, 2.076934, 0.553842, 2.569250]
    np.testing.assert_allclose(got, ref, atol=2e-6)


def test_ridge_regression_doc_example():
    b = _op()
    m = RidgeRegression().setFeatureCols(["f0", "f1"]).setLambda(0.1).setLabelCol("label") \
        .setPredictionCol("pred").fit(b)
    got = m.transform(b).collectToDataframe()["pred"].values
    ref = [0.830304, 1.377312, 1.924320, 1.159119, 0.939909, 1.924320, 0.502506, 2.361724]
    np.testing.assert_allclose(got, ref, atol=2e-6)


@pytest.mark.parametrize("stage", [LogisticRegression, LinearSvm])
def test_binary_classifiers_doc_example(stage):
    b = _op(label_last=2)
    m = stage().setFeatureCols(["f0", "f1"]).setLabelCol("label").setPredictionCol("pred").fit(b)
    got = m.transform(b).collectToDataframe()
    assert list(got["pred"]) == [1, 1, 2, 1, 1, 2, 1, 2]


def test_softmax_doc_example():
    b = _op()
    m = Softmax().setFeatureCols(["f0", "f1"]).setLabelCol("label").setPredictionCol("pred").fit(b)
    assert list(m.transform(b).collectToDataframe()["pred"]) == [1, 1, 2, 1, 1, 2, 1, 3]


def test_lr_detail_and_model_rows():
    b = _op(label_last=2)
    model = LogisticRegressionTrainBatchOp().setFeatureCols(["f0", "f1"]).setLabelCol("label").linkFrom(b)
    rows = model.collect()
    meta = json.loads(rows[0][1])
    assert meta["linearModelType"] == '"LR"' and meta["modelName"] == '"Logistic Regression"'
    assert meta["labelCol"] is None
    data = json.loads(rows[1][1])
    assert data["featureColNames"] == ["f0", "f1"] and data["featureColTypes"] == ["int", "int"]
    assert [r[2] for r in rows[2:]] == [2, 1]          # labels[0] = larger string = positive
    pred = LogisticRegressionPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d") \
        .linkFrom(model, b).collectToDataframe()
    det = json.loads(pred["d"][2])
    assert set(det) == {"1", "2"} and float(det["2"]) > 0.5


def test_aft_doc_example_bitwise():
    df = pd.DataFrame({"label": [1.218, 2.949, 3.627, 0.273, 4.199], "censor": [1.0, 0.0, 0.0, 1.0, 0.0],
                       "features": ["1.560,-0.605", "0.346,2.158", "1.380,0.231", "0.520,1.151", "0.795,-0.226"]})
    a = BatchOperator.fromDataframe(df, schemaStr="label double, censor double, features string")
    pm = Pipeline().add(AftSurvivalRegression().setVectorCol("features").setLabelCol("label")
                        .setCensorCol("censor").setPredictionCol("result")).fit(a)
    model_rows = pm.getTransformer(0).getModelData().rows()
    coef = json.loads(model_rows[1][1])["coefVector"]["data"]
    np.testing.assert_allclose(coef, [2.6373721387804276, -0.49591581739360013, 0.19847648151323818,
                                      1.5469720551612485], rtol=1e-12)
    meta = json.loads(model_rows[0][1])
    assert meta == {"hasInterceptItem": "true", "vectorCol": '"features"', "modelName": '"AFTSurvivalRegTrainBatchOp"',
                    "labelCol": None, "linearModelType": '"AFT"', "vectorSize": "3"}
    assert list(meta) == ["hasInterceptItem", "vectorCol", "modelName", "labelCol", "linearModelType", "vectorSize"]
    res = dict(zip(pm.transform(a).collectToDataframe()["label"], pm.transform(a).collectToDataframe()["result"]))
    ref = {0.273: 13.571097451777327, 1.218: 5.718263596902868, 3.627: 7.380610641992667,
           4.199: 9.009354073821902, 2.949: 18.067188679653064}
    for k, v in ref.items():
        assert abs(res[k] - v) < 1e-9 * v


@pytest.mark.parametrize("method", ["LBFGS", "GD", "Newton", "SGD", "OWLQN"])
def test_optimizers_agree_on_logistic_problem(method):
    rng = np.random.default_rng(0)
    X = rng.normal(size=(400, 3))
    w = np.array([1.5, -2.0, 0.5])
    y = (X @ w + 0.3 + 0.3 * rng.normal(size=400) > 0).astype(int)
    df = pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "c": X[:, 2], "y": y})
    b = BatchOperator.fromDataframe(df, schemaStr="a double, b double, c double, y int")
    st = LogisticRegression().setFeatureCols(["a", "b", "c"]).setLabelCol("y").setPredictionCol("p") \
        .setOptimMethod(method).setMaxIter(200 if method != "SGD" else 400)
    if method == "OWLQN":
        st.setL1(0.001)
    if method == "SGD":
        st.setLearningRate(1.0) if hasattr(st, "setLearningRate") else None
    m = st.fit(b)
    acc = (m.transform(b).collectToDataframe()["p"].values == y).mean()
    assert acc > 0.9, (method, acc)


def test_lasso_sparsity_and_pipeline_save_load(tmp_path):
    rng = np.random.default_rng(1)
    X = rng.normal(size=(200, 5))
    y = X[:, 0] * 3 + 0.01 * rng.normal(size=200)
    df = pd.DataFrame({f"x{i}": X[:, i] for i in range(5)})
    df["y"] = y
    b = BatchOperator.fromDataframe(df, schemaStr=", ".join(f"x{i} double" for i in range(5)) + ", y double")
    pm = Pipeline().add(LassoRegression().setFeatureCols([f"x{i}" for i in range(5)]).setLabelCol("y")
                        .setLambda(0.05).setPredictionCol("p")).fit(b)
    path = str(tmp_path / "m.csv")
    pm.save(path)
    pm2 = PipelineModel.load(path)
    p1 = pm.transform(b).collectToDataframe()["p"].values
    p2 = pm2.transform(b).collectToDataframe()["p"].values
    np.testing.assert_allclose(p1, p2)
    assert np.corrcoef(p1, y)[0, 1] > 0.99
