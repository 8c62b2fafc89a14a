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


def _legacy_rows(rows, chunk=9):
    """The reference's old 4-column layout (LinearModelData.loadOldFromatModel): id 0 = meta JSON (with the label
    values and the Flink label type name), ids 1.. = the ModelData JSON cut into pieces, two unused columns."""
    from alink_amd.common.params import Params
    meta = Params.fromJson(rows[0][1])
    labels = [r[2] for r in rows[2:]]
    meta.set("labelValues", labels)
    meta.set("labelTypeName", "INT")
    data = rows[1][1]
    pieces = [data[i:i + chunk] for i in range(0, len(data), chunk)]
    out = [(0, meta.toJson(), None, None)] + [(i + 1, p, None, None) for i, p in enumerate(pieces)]
    return out[::-1]                                   # row order must not matter (ids order the pieces)


def test_legacy_four_column_linear_model_predicts_like_three_column():
    """Legacy 4-column LR model (LinearModelDataConverter.java:77-85 -> LinearModelData.java:116-157) == its
    3-column equivalent in batch predict, LocalPredictor (detail included) and as the FTRL warm start."""
    from alink_amd import LogisticRegressionModel, FtrlTrainStreamOp, StreamOperator, CollectStreamOp
    from alink_amd.common.table import MTable
    from alink_amd.common.types import schema_str_to_schema
    from alink_amd.models.linear.model import LinearModelDataConverter
    from alink_amd.operator.batch.source import TableSourceBatchOp
    b = _op(label_last=2)
    model = LogisticRegressionTrainBatchOp().setFeatureCols(["f0", "f1"]).setLabelCol("label").linkFrom(b)
    rows = [tuple(r) for r in model.collect()]
    legacy = MTable.from_rows(_legacy_rows(rows), schema_str_to_schema(
        "model_id bigint, model_info string, label_value string, model_extra string"), replicated=True)
    m3 = LinearModelDataConverter().load(rows)
    m4 = LinearModelDataConverter().load(legacy.rows())
    assert m4.labelValues == [2, 1] and m4.coefVector.data.tolist() == m3.coefVector.data.tolist()
    assert m4.featureNames == ["f0", "f1"] and m4.linearModelType.name == "LR"
    p3 = LogisticRegressionPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d").linkFrom(model, b) \
        .collect()
    p4 = LogisticRegressionPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d") \
        .linkFrom(TableSourceBatchOp(legacy), b).collect()
    assert [tuple(r) for r in p4] == [tuple(r) for r in p3]
    lp = LogisticRegressionModel().setPredictionCol("p").setPredictionDetailCol("d").setModelData(legacy) \
        .getLocalPredictor("f0 int, f1 int, label int")
    assert [tuple(lp.map(r[:3])) for r in b.collect()] == [tuple(r) for r in p3]
    # FTRL warm start from either format: identical snapshots
    df = pd.DataFrame({"f0": DATA[:, 0], "f1": DATA[:, 1], "label": [1, 1, 2, 1, 1, 2, 1, 2]})
    snaps = {}
    for tag, init in (("three", model), ("four", TableSourceBatchOp(legacy))):
        got = []
        FtrlTrainStreamOp(init).setFeatureCols(["f0", "f1"]).setLabelCol("label").setTimeInterval(1e9) \
            .linkFrom(StreamOperator.fromDataframe(df, schemaStr="f0 int, f1 int, label int")) \
            .link(CollectStreamOp(got))
        StreamOperator.execute()
        snaps[tag] = [tuple(r) for r in got]
    assert snaps["three"] and snaps["four"] == snaps["three"]


def test_meta_label_values_without_aux_rows():
    """Label values carried only in the meta (LinearModelDataConverter.java:61-64) are recovered with the
    converter's label type."""
    from alink_amd.common.params import Params
    from alink_amd.common.types import Types
    from alink_amd.models.linear.model import LinearModelDataConverter
    b = _op(label_last=2)
    rows = [tuple(r) for r in LogisticRegressionTrainBatchOp().setFeatureCols(["f0", "f1"]).setLabelCol("label")
            .linkFrom(b).collect()]
    meta = Params.fromJson(rows[0][1])
    meta.set("labelValues", [2.0, 1.0])
    m = LinearModelDataConverter(Types.LONG).load([(rows[0][0], meta.toJson(), None), rows[1]])
    assert m.labelValues == [2, 1] and all(isinstance(v, int) for v in m.labelValues)


SOFTMAX_ROWS = [
    (0, '{"hasInterceptItem":"true","modelName":"\\"softmax\\"","labelType":"4","modelSchema":"\\"model_id bigint,'
        'model_info string,label_type int\\"","isNewFormat":"true"}', None),
    (1048576, '{"featureColNames":["f0","f1","f2"],"coefVector":{"data":[172.15928828045577,-18.99714734506609,'
              '-93.78617647691524,27.419236408736307,-825.863312143001,-47.67468533510818,97.56887933300092,'
              '87.33950982847793]}}', None),
    (2097152, None, None), (2147483647 * 1048576, None, 1), (2147483647 * 1048576 + 1, None, 2),
    (2147483647 * 1048576 + 2, None, 3)]


@pytest.mark.parametrize("reserved", [[], None])
def test_softmax_model_mapper_reference_rows(reserved):
    """SoftmaxModelMapperTest (reference operator/common/classification): 3-column model table with integer
    labels in the label_type column; (1, 7, 9) -> label 2, with and without reserved columns."""
    from alink_amd.common.params import Params
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.linear.model import SoftmaxModelMapper
    ms = TableSchema(["model_id", "model_info", "label_type"], [Types.LONG, Types.STRING, Types.INT])
    ds = TableSchema(["f0", "f1", "f2"], [Types.DOUBLE] * 3)
    p = Params().set("predictionCol", "pred")
    if reserved is not None:
        p.set("reservedCols", reserved)
    m = SoftmaxModelMapper(ms, ds, p)
    m.loadModel(SOFTMAX_ROWS)
    out = m.map((1.0, 7.0, 9.0))
    assert out[-1] == 2
    names = ["pred"] if reserved == [] else ["f0", "f1", "f2", "pred"]
    assert m.getOutputSchema() == TableSchema(names, [Types.DOUBLE] * (len(names) - 1) + [Types.INT])


def test_aft_model_mapper_reference_rows():
    """AFTRegressionMapperTest (reference operator/common/regression): a prediction column already in the input
    is overwritten in place; exp(x . coef) for "1.560 -0.605" = 5.71."""
    from alink_amd.common.params import Params
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.linear.model import AFTModelMapper
    rows = [(0, '{"hasInterceptItem":"true","vectorColName":"\\"features\\"","modelName":"\\"AFTSurvivalRegTrainBatchOp'
                '\\"","labelType":"8","modelSchema":"\\"model_id bigint,model_info string,label_type double\\"",'
                '"isNewFormat":"true","linearModelType":"\\"AFT\\"","vectorSize":"2"}', None),
            (1048576, '{"coefVector":{"data":[2.6380946835087933,-0.49631115827728234,0.19844422562555475,'
                      '1.5472345338855131]}}', None)]
    ms = TableSchema(["model_id", "model_info", "label_type"], [Types.LONG, Types.STRING, Types.DOUBLE])
    ds = TableSchema(["vector", "pred"], [Types.STRING, Types.DOUBLE])
    m = AFTModelMapper(ms, ds, Params().set("vectorCol", "vector").set("predictionCol", "pred"))
    m.loadModel(rows)
    assert float(m.map(("1.560 -0.605", None))[1]) == pytest.approx(5.71, abs=0.01)
    assert m.getOutputSchema() == ds


REG_ROWS = [("$3$0:1.0 1:7.0 2:9.0", "1.0 7.0 9.0", 1.0, 7.0, 9.0, 16.8),
            ("$3$0:1.0 1:3.0 2:3.0", "1.0 3.0 3.0", 1.0, 3.0, 3.0, 6.7),
            ("$3$0:1.0 1:2.0 2:4.0", "1.0 2.0 4.0", 1.0, 2.0, 4.0, 6.9),
            ("$3$0:1.0 1:3.0 2:4.0", "1.0 3.0 4.0", 1.0, 3.0, 4.0, 8.0)]


@pytest.mark.parametrize("name,expect", [
    ("LinearRegression", {16.8: (16.814789059973744, 16.814789059973744, 16.814788687904162),
                          6.7: (6.773942836224718, 6.773942836224718, 6.773943529327923)}),
    ("RidgeRegression", {16.8: (16.653595680699425, 16.653595680699425, 16.384437074591887),
                         6.7: (6.825267886078004, 6.825267886078004, 7.425378715755974)}),
    ("LassoRegression", {16.8: (16.784611802507232, 16.784611802507232, 16.78209421260283),
                         6.7: (6.7713287283076, 6.7713287283076, 6.826846826823054)})])
def test_regression_pipelines_reference_predictions(name, expect):
    """pipeline/regression/{Linear,Ridge,Lasso}RegressionTest: feature columns, dense vector and sparse vector
    (no mean centring for sparse input, hence the different regularised fit) give the reference's predictions."""
    import alink_amd as A
    from alink_amd.operator.batch.source import MemSourceBatchOp
    data = MemSourceBatchOp(REG_ROWS, ["svec", "vec", "f0", "f1", "f2", "label"])

    def mk():
        m = getattr(A, name)().setLabelCol("label")
        return m if name == "LinearRegression" else m.setLambda(0.01)
    pl = A.Pipeline().add(mk().setFeatureCols(["f0", "f1", "f2"]).setPredictionCol("p1")) \
        .add(mk().setVectorCol("vec").setPredictionCol("p2")).add(mk().setVectorCol("svec").setPredictionCol("p3"))
    got = {r[0]: tuple(r[1:]) for r in pl.fit(data).transform(data).select(["label", "p1", "p2", "p3"]).collect()}
    for label, e in expect.items():
        assert got[label] == pytest.approx(e, abs=1e-5), (label, got[label])


def test_linear_model_mapper_reference_rows():
    """LinearModelMapperTest: a new-format LR model table with an INT label column; prediction 1 for (1, 1, 0, 1),
    output schema ``pred INT`` with reservedCols [] and the input columns + ``pred`` otherwise."""
    from alink_amd.common.params import Params
    from alink_amd.common.types import schema_str_to_schema
    from alink_amd.models.linear.model import LinearModelMapper
    rows = [(0, '{"hasInterceptItem":"true","modelName":"\\"Logistic Regression\\"","labelType":"4",'
                '"modelSchema":"\\"model_id bigint,model_info string,label_type int\\"","isNewFormat":"true",'
                '"linearModelType":"\\"LR\\""}', None),
            (1048576, '{"featureColNames":["f0","f1","f2","f3"],"coefVector":{"data":[-9.634910228989458,'
                      '45.508924427487486,-22.06146649207175,-20.926964828123506,45.508924427487486]}}', None),
            (2147483647 * 1048576, None, 1), (2147483647 * 1048576 + 1, None, 0)]
    ms = schema_str_to_schema("model_id bigint, model_info string, label_type int")
    ds = schema_str_to_schema("f0 double, f1 double, f2 double, f3 double")
    m = LinearModelMapper(ms, ds, Params().set("predictionCol", "pred").set("reservedCols", []))
    m.loadModel(rows)
    assert tuple(m.map((1.0, 1.0, 0.0, 1.0))) == (1,)
    assert m.getOutputSchema().getFieldNames() == ["pred"] and str(m.getOutputSchema().getFieldTypes()[0]) == "INT"
    m = LinearModelMapper(ms, ds, Params().set("predictionCol", "pred"))
    m.loadModel(rows)
    assert tuple(m.map((1.0, 1.0, 0.0, 1.0)))[4] == 1
    assert m.getOutputSchema().getFieldNames() == ["f0", "f1", "f2", "f3", "pred"]


def test_linear_model_large_coefficients_native_parse():
    """A large coefficient vector is read by the C++ number parser (cut out of the model JSON), a vector with NaN
    by json.loads: both round-trip exactly through the model rows."""
    import numpy as np
    from alink_amd.common.linalg import DenseVector
    from alink_amd.common.types import Types
    from alink_amd.models.linear.model import LinearModelData, LinearModelDataConverter
    rng = np.random.default_rng(3)
    for special in (False, True):
        m = LinearModelData()
        m.modelName, m.linearModelType, m.hasInterceptItem = "Logistic Regression", "LR", True
        m.vectorColName, m.vectorSize, m.labelName = "vec", 150_000, "label"
        m.featureNames = m.featureTypes = m.coefVectors = None
        w = rng.normal(size=150_001) * 10.0 ** rng.integers(-20, 20, size=150_001)
        if special:
            w[7] = np.nan
        m.coefVector = DenseVector(w)
        m.labelValues = [0, 1]
        conv = LinearModelDataConverter(Types.INT)
        got = conv.load(conv.save(m))
        assert np.array_equal(got.coefVector.data, w, equal_nan=True)
        assert got.featureNames is None and got.vectorSize == 150_000
