"""Naive Bayes text classifier vs the reference docs and NaiveBayesTextModelMapperTest fixture."""
import json

import numpy as np
import pandas as pd
import pytest

from alink_amd import *  # noqa: F401,F403
from alink_amd.common.table import MTable
from alink_amd.common.types import TableSchema, Types
from alink_amd.common.params import Params
from alink_amd.models.classification.naive_bayes import NaiveBayesTextModelMapper

DATA = [["$31$0:1.0 1:1.0 2:1.0 30:1.0", "1.0  1.0  1.0  1.0", "1"],
        ["$31$0:1.0 1:1.0 2:0.0 30:1.0", "1.0  1.0  0.0  1.0", "1"],
        ["$31$0:1.0 1:0.0 2:1.0 30:1.0", "1.0  0.0  1.0  1.0", "1"],
        ["$31$0:1.0 1:0.0 2:1.0 30:1.0", "1.0  0.0  1.0  1.0", "1"],
        ["$31$0:0.0 1:1.0 2:1.0 30:0.0", "0.0  1.0  1.0  0.0", "0"],
        ["$31$0:0.0 1:1.0 2:1.0 30:0.0", "0.0  1.0  1.0  0.0", "0"],
        ["$31$0:0.0 1:1.0 2:1.0 30:0.0", "0.0  1.0  1.0  0.0", "0"]]


@pytest.mark.parametrize("mtype", ["Multinomial", "Bernoulli"])
@pytest.mark.parametrize("col", ["sv", "dv"])
def test_naive_bayes_doc(mtype, col):
    df = pd.DataFrame(DATA, columns=["sv", "dv", "label"])
    b = BatchOperator.fromDataframe(df, schemaStr="sv string, dv string, label string")
    model = b.link(NaiveBayesTextTrainBatchOp().setVectorCol(col).setLabelCol("label").setModelType(mtype))
    out = NaiveBayesTextPredictBatchOp().setVectorCol(col).setReservedCols(["sv", "label"]) \
        .setPredictionCol("pred").setPredictionDetailCol("d").linkFrom(model, b).collect()
    assert [r[2] for r in out] == ["1", "1", "1", "1", "0", "0", "0"]
    for r in out:
        p = json.loads(r[3])
        assert abs(sum(p.values()) - 1.0) < 1e-12
    m = NaiveBayesTextClassifier().setVectorCol(col).setLabelCol("label").setPredictionCol("pred").fit(b)
    assert [r[3] for r in m.transform(b).collect()] == ["1", "1", "1", "1", "0", "0", "0"]


def test_reference_model_fixture():
    rows = [(0, '{"labelType":"4","modelType":"\\"BERNOULLI\\"","labelTypeName":"\\"INTEGER\\"",'
                '"isNewFormat":"true","vectorCol":"vec"}', None),
            (1048576, '{"piArray":[-0.6931471805599454,-0.6931471805599454],"theta":{"m":2,"n":4,"data":'
                      '[-2.3025850929940455,-0.10536051565782611,-0.10536051565782611,-0.6931471805599452,'
                      '-0.10536051565782611,-0.3566749439387322,-2.3025850929940455,-0.10536051565782611]}}', None),
            ((2 ** 31 - 1) * 1048576, None, 0), ((2 ** 31 - 1) * 1048576 + 1, None, 1)]
    ms = TableSchema(["model_id", "model_info", "label_type"], [Types.LONG, Types.STRING, Types.INT])
    ds = TableSchema(["vec"], [Types.STRING])
    mapper = NaiveBayesTextModelMapper(ms, ds, Params().set("vectorCol", "vec").set("predictionCol", "pred"))
    mapper.loadModel(rows)
    assert mapper.map(("1.0, 1.0, 0.0, 1.0",))[1] == 1
    assert mapper.getOutputSchema().names == ["vec", "pred"] and mapper.getOutputSchema().types[1] == Types.INT


@pytest.mark.parametrize("mtype", ["Multinomial", "Bernoulli"])
def test_vectorized_prediction_matches_detail_path(mtype):
    """Columnar prediction (CSR scores, argmax over the classes at once) gives the labels the per-row detail
    path picks; sparse indices beyond the model width are dropped as the dense path truncates."""
    rng = np.random.default_rng(1)
    rows = []
    for i in range(300):
        idx = sorted(rng.choice(12, 4, replace=False))
        vals = [1.0 if mtype == "Bernoulli" else float(rng.integers(1, 4)) for _ in idx]
        rows.append(["$12$" + " ".join(f"{a}:{b}" for a, b in zip(idx, vals)), ["a", "b", "c"][i % 3]])
    df = pd.DataFrame(rows, columns=["sv", "label"])
    b = BatchOperator.fromDataframe(df, schemaStr="sv string, label string")
    model = b.link(NaiveBayesTextTrainBatchOp().setVectorCol("sv").setLabelCol("label").setModelType(mtype))
    test = [[r[0].replace("$12$", "$20$") + (" 15:1.0" if mtype != "Bernoulli" else "")] for r in rows[:50]] + \
        [[r[0]] for r in rows[50:]]
    t = BatchOperator.fromDataframe(pd.DataFrame(test, columns=["sv"]), schemaStr="sv string")
    fast = NaiveBayesTextPredictBatchOp().setVectorCol("sv").setPredictionCol("p").linkFrom(model, t).collect()
    slow = NaiveBayesTextPredictBatchOp().setVectorCol("sv").setPredictionCol("p").setPredictionDetailCol("d") \
        .linkFrom(model, t).collect()
    assert [r[1] for r in fast] == [r[1] for r in slow]
    assert len({r[1] for r in fast}) > 1
