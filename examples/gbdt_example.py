#!/usr/bin/env python3
"""GBDT example (reference examples/.../GBDTExample.java): adult-census-shaped data (numeric + categorical
columns, binary label) -> GbdtClassifier (20 trees) -> predictions -> binary-classification metrics.

    python examples/gbdt_example.py [--device cuda:0] [--rows 20000]
"""
import numpy as np
import pandas as pd

from _common import args


def main():
    a = args(20000)
    from alink_amd import useLocalEnv, BatchOperator, GbdtClassifier, EvalBinaryClassBatchOp
    useLocalEnv(1, device=a.device)
    rng = np.random.default_rng(1)
    n = a.rows
    age = rng.integers(17, 90, n)
    hours = rng.integers(1, 99, n)
    edu = rng.integers(1, 16, n)
    gain = np.where(rng.random(n) < 0.1, rng.integers(1000, 99999, n), 0)
    work = rng.choice(["Private", "Self-emp", "Gov", "Never-worked"], n)
    rel = rng.choice(["Husband", "Wife", "Own-child", "Unmarried"], n)
    score = 0.04 * (age - 40) + 0.03 * (hours - 40) + 0.25 * (edu - 9) + (gain > 5000) * 2.0 \
        + (rel == "Husband") * 0.8 + rng.normal(size=n)
    label = np.where(score > 1.0, ">50K", "<=50K")
    df = pd.DataFrame({"age": age, "workclass": work, "education_num": edu, "relationship": rel,
                       "capital_gain": gain, "hours_per_week": hours, "label": label})
    schema = "age bigint, workclass string, education_num bigint, relationship string, capital_gain bigint, " \
             "hours_per_week bigint, label string"
    data = BatchOperator.fromDataframe(df, schemaStr=schema)
    train, test = data, data
    features = ["age", "workclass", "education_num", "relationship", "capital_gain", "hours_per_week"]
    gbdt = GbdtClassifier().setFeatureCols(features).setCategoricalCols(["workclass", "relationship"]) \
        .setLabelCol("label").setNumTrees(20).setPredictionCol("prediction_result") \
        .setPredictionDetailCol("prediction_detail")
    model = gbdt.fit(train)
    pred = model.transform(test)
    pred.select("label, prediction_result, prediction_detail").firstN(5).print()
    metrics = EvalBinaryClassBatchOp().setLabelCol("label").setPositiveLabelValueString(">50K") \
        .setPredictionDetailCol("prediction_detail").linkFrom(pred).collectMetrics()
    print("AUC:", metrics.getAuc(), "Accuracy:", metrics.getAccuracy())
    return metrics


if __name__ == "__main__":
    main()
