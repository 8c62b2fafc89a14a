"""GLM (IRLS) and isotonic regression vs the reference docs (docs/en/glmtrainbatchop.md,
docs/en/isotonicregtrainbatchop.md) and closed-form / statsmodels-style checks."""
import json
import math

import numpy as np
import pytest

from alink_amd import *  # noqa: F401,F403

GLM_DATA = [[1.6094, 118.0, 69.0, 1.0, 2.0], [2.3026, 58.0, 35.0, 1.0, 2.0], [2.7081, 42.0, 26.0, 1.0, 2.0],
            [2.9957, 35.0, 21.0, 1.0, 2.0], [3.4012, 27.0, 18.0, 1.0, 2.0], [3.6889, 25.0, 16.0, 1.0, 2.0],
            [4.0943, 21.0, 13.0, 1.0, 2.0], [4.3820, 19.0, 12.0, 1.0, 2.0], [4.6052, 18.0, 12.0, 1.0, 2.0]]
GLM_SCHEMA = 'u double, lot1 double, lot2 double, offset double, weights double'
# docs/en/glmtrainbatchop.md "pred" column: the doc prints the linear predictor (log-link eta) of this model
DOC_ETA = [0.378525, 0.970639, 1.126458, 1.227753, 1.258898, 1.305654, 1.367991, 1.383571, 1.375774]


def _glm_train():
    src = MemSourceBatchOp([tuple(r) for r in GLM_DATA], GLM_SCHEMA)
    train = GlmTrainBatchOp().setFamily("gamma").setLink("Log").setRegParam(0.3).setMaxIter(5) \
        .setFeatureCols(["lot1", "lot2"]).setLabelCol("u")
    return src, src.link(train)


def test_glm_gamma_log_matches_doc():
    src, train = _glm_train()
    out = GlmPredictBatchOp().setPredictionCol("pred").setLinkPredResultCol("eta").linkFrom(train, src).collect()
    eta = [r[-1] for r in out]
    pred = [r[-2] for r in out]
    np.testing.assert_allclose(eta, DOC_ETA, atol=2e-6)
    np.testing.assert_allclose(pred, np.exp(eta), rtol=1e-12)
    summary = json.loads(train.getSideOutput(1).collect()[0][0])
    assert summary["rank"] == 3 and summary["degreeOfFreedom"] == 6
    res = train.getSideOutput(0)
    assert res.getColNames()[-4:] == ["residualdevianceResiduals", "pearsonResiduals", "workingResiduals",
                                      "responseResiduals"]
    ev = GlmEvaluationBatchOp().setFamily("gamma").setLink("Log").setRegParam(0.3).setMaxIter(5) \
        .setFeatureCols(["lot1", "lot2"]).setLabelCol("u").linkFrom(train, src).collect()
    assert json.loads(ev[0][0])["coefficients"] == summary["coefficients"]


def test_glm_gaussian_identity_is_ols():
    rng = np.random.default_rng(0)
    X = rng.normal(size=(200, 3))
    y = X @ np.array([1.0, -2.0, 0.5]) + 3.0 + 0.01 * rng.normal(size=200)
    rows = [tuple(x) + (float(t),) for x, t in zip(X.tolist(), y)]
    src = MemSourceBatchOp(rows, "a double, b double, c double, y double")
    m = GeneralizedLinearRegression().setFeatureCols(["a", "b", "c"]).setLabelCol("y") \
        .setPredictionCol("p").fit(src)
    pred = np.array([r[-1] for r in m.transform(src).collect()])
    A = np.c_[X, np.ones(200)]
    ols = A @ np.linalg.lstsq(A, y, rcond=None)[0]
    np.testing.assert_allclose(pred, ols, atol=1e-8)


@pytest.mark.parametrize("family,link", [("binomial", None), ("poisson", None), ("binomial", "probit"),
                                         ("poisson", "sqrt"), ("tweedie", None)])
def test_glm_families_converge(family, link):
    rng = np.random.default_rng(1)
    X = rng.normal(size=(400, 2))
    eta = X @ np.array([0.7, -0.4]) + 0.2
    if family == "binomial":
        y = (rng.random(400) < 1 / (1 + np.exp(-eta))).astype(float)
    else:
        y = rng.poisson(np.exp(eta)).astype(float)
    rows = [tuple(x) + (float(t),) for x, t in zip(X.tolist(), y)]
    src = MemSourceBatchOp(rows, "a double, b double, y double")
    op = GlmTrainBatchOp().setFamily(family).setFeatureCols(["a", "b"]).setLabelCol("y").setMaxIter(25)
    if link:
        op.setLink(link)
    if family == "tweedie":
        op.setVariancePower(1.5).setLink("log")
    model = src.link(op)
    s = json.loads(model.getSideOutput(1).collect()[0][0])
    assert all(math.isfinite(c) for c in s["coefficients"])
    if link is None and family != "tweedie":
        assert abs(s["coefficients"][0] - 0.7) < 0.35 and abs(s["coefficients"][1] + 0.4) < 0.35


ISO = [[0.35, 1], [0.6, 1], [0.55, 1], [0.5, 1], [0.18, 0], [0.1, 1], [0.8, 1], [0.45, 0], [0.4, 1], [0.7, 0],
       [0.02, 1], [0.3, 0], [0.27, 1], [0.2, 0], [0.9, 1]]


def test_isotonic_doc_model_and_predictions():
    src = MemSourceBatchOp([(float(l), float(f)) for f, l in ISO], "label double, feature double")
    model = IsotonicRegTrainBatchOp().setFeatureCol("feature").setLabelCol("label").linkFrom(src)
    rows = sorted(model.collect(), key=lambda r: r[0])
    assert json.loads(rows[1][1]) == [0.02, 0.3, 0.35, 0.45, 0.5, 0.7]
    assert json.loads(rows[2][1]) == [0.5, 0.5, 0.6666666865348816, 0.6666666865348816, 0.75, 0.75]
    pred = IsotonicRegPredictBatchOp().setPredictionCol("result").linkFrom(model, src).collect()
    doc = {0.9: 0.75, 0.7: 0.75, 0.35: 0.6666666865348816, 0.02: 0.5, 0.27: 0.5, 0.5: 0.75, 0.18: 0.5,
           0.45: 0.6666666865348816, 0.8: 0.75, 0.6: 0.75, 0.4: 0.6666666865348816, 0.3: 0.5, 0.55: 0.75,
           0.2: 0.5, 0.1: 0.5}
    for r in pred:
        assert r[2] == pytest.approx(doc[r[1]], abs=1e-12)
    m = IsotonicRegression().setFeatureCol("feature").setLabelCol("label").setPredictionCol("p").fit(src)
    assert len(m.transform(src).collect()) == 15


def test_isotonic_antitonic_and_vector_input():
    src = MemSourceBatchOp([(float(l), f"{f} 0.0") for f, l in ISO], "label double, vec string")
    model = IsotonicRegTrainBatchOp().setVectorCol("vec").setFeatureIndex(0).setLabelCol("label") \
        .setIsotonic(False).linkFrom(src)
    vals = json.loads(sorted(model.collect(), key=lambda r: r[0])[2][1])
    assert all(a >= b for a, b in zip(vals, vals[1:]))


ISO_META = ('{"vectorColName":%s,"modelName":"\\"IsotonicRegressionModel\\"","featureColName":%s,"featureIndex":"0",'
            '"modelSchema":"\\"model_id bigint,model_info string\\"","isNewFormat":"true"}')
ISO_ROWS = [(1048576, "[0.02,0.1,0.2,0.27,0.3,0.35,0.45,0.5,0.7,0.8,0.9]"),
            (2097152, "[0.0,0.3333333333333333,0.3333333333333333,0.5,0.5,0.6666666666666666,0.6666666666666666,"
                      "0.75,0.75,1.0,1.0]")]


@pytest.mark.parametrize("vector", [False, True])
def test_isotonic_mapper_reference_model_rows(vector):
    """IsotonicRegressionModelMapperTest: model meta with the old ``featureColName`` / ``vectorColName`` keys
    (aliases of featureCol / vectorCol); 0.35 -> 0.66, vector "0.81, 0.35" (index 0) -> 1.0.  (The reference
    declares the vector column DOUBLE and feeds a string; here it is a string column.)"""
    from alink_amd.common.params import Params
    from alink_amd.common.types import schema_str_to_schema
    from alink_amd.models.regression.isotonic import IsotonicRegressionModelMapper
    meta = ISO_META % (('"\\"vector\\""', "null") if vector else ("null", '"\\"feature\\""'))
    ms = schema_str_to_schema("model_id bigint, model_info string")
    ds = schema_str_to_schema("vector string" if vector else "feature double")
    m = IsotonicRegressionModelMapper(ms, ds, Params().set("predictionCol", "pred"))
    m.loadModel([(0, meta)] + ISO_ROWS)
    out = m.map(("0.81, 0.35",) if vector else (0.35,))
    assert float(out[1]) == pytest.approx(1.0 if vector else 0.66, abs=0.01)
    assert m.getOutputSchema().getFieldNames() == (["vector", "pred"] if vector else ["feature", "pred"])
