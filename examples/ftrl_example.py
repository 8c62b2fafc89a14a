#!/usr/bin/env python3
"""FTRL example (reference examples/.../FTRLExample.java): avazu-shaped click log -> feature pipeline
(StandardScaler on the numeric columns + FeatureHasher, 30000 hashed features) -> batch LR initial model ->
FTRL online training on a stream -> online predictions evaluated by EvalBinaryClassStreamOp.

    python examples/ftrl_example.py [--device cuda:0] [--rows 20000] [--mode SEQUENTIAL|SHARDED|HOGWILD]
"""
import os
import sys

import numpy as np

from _common import args


def main():
    mode = "SEQUENTIAL"
    if "--mode" in sys.argv:
        k = sys.argv.index("--mode")
        mode = sys.argv[k + 1]
        del sys.argv[k:k + 2]
    a = args(20000)
    from alink_amd import (useLocalEnv, CsvSourceBatchOp, CsvSourceStreamOp, Pipeline, StandardScaler, FeatureHasher,
                           LogisticRegressionTrainBatchOp, FtrlTrainStreamOp, FtrlPredictStreamOp, SplitStreamOp,
                           EvalBinaryClassStreamOp, CollectStreamOp, StreamOperator)
    useLocalEnv(1, device=a.device)
    rng = np.random.default_rng(3)
    path = os.path.join(a.workdir, "avazu_like.csv")
    cats = ["C1", "banner_pos", "site_category", "app_domain", "app_category", "device_type", "device_conn_type",
            "site_id", "site_domain", "device_id", "device_model"]
    nums = ["C14", "C15", "C16", "C17", "C18", "C19", "C20", "C21"]
    card = {c: int(rng.integers(3, 400)) for c in cats}
    eff = {c: rng.normal(size=card[c]) for c in cats}
    with open(path, "w") as f:
        f.write("id,click," + ",".join(cats + nums) + "\n")
        for i in range(a.rows):
            vals = {c: int(rng.integers(0, card[c]) ** 1) for c in cats}
            num = rng.normal(size=len(nums))
            logit = sum(eff[c][vals[c]] for c in cats) * 0.4 + 0.5 * num[0] - 1.5
            click = int(rng.random() < 1 / (1 + np.exp(-logit)))
            f.write(f"{i},{click}," + ",".join(f"{c}_{vals[c]}" for c in cats) + ","
                    + ",".join(f"{int(1000 + 100 * x)}" for x in num) + "\n")
    schema = "id string, click string, " + ", ".join(f"{c} string" for c in cats) + ", " + \
             ", ".join(f"{c} int" for c in nums)
    batch = CsvSourceBatchOp().setFilePath(path).setSchemaStr(schema).setIgnoreFirstLine(True)
    features = Pipeline().add(StandardScaler().setSelectedCols(nums)) \
        .add(FeatureHasher().setSelectedCols(cats + nums).setCategoricalCols(cats).setOutputCol("vec")
             .setNumFeatures(30000))
    fmodel = features.fit(batch)
    init = fmodel.transform(batch).link(LogisticRegressionTrainBatchOp().setVectorCol("vec").setLabelCol("click")
                                        .setWithIntercept(True).setMaxIter(10))
    stream = CsvSourceStreamOp().setFilePath(path).setSchemaStr(schema).setIgnoreFirstLine(True)
    split = SplitStreamOp().setFraction(0.5).linkFrom(stream)
    train = fmodel.transform(split)
    test = fmodel.transform(split.getSideOutput(0))
    model = FtrlTrainStreamOp(init).setVectorCol("vec").setLabelCol("click").setWithIntercept(True) \
        .setAlpha(0.1).setBeta(0.1).setL1(0.01).setL2(0.01).setTimeInterval(10).setVectorSize(30000) \
        .setUpdateMode(mode).linkFrom(train)
    pred = FtrlPredictStreamOp(init).setVectorCol("vec").setPredictionCol("pred").setReservedCols(["click"]) \
        .setPredictionDetailCol("details").linkFrom(model, test)
    evals = []
    EvalBinaryClassStreamOp().setLabelCol("click").setPredictionDetailCol("details").setTimeInterval(10) \
        .linkFrom(pred).link(CollectStreamOp(evals))
    StreamOperator.execute()
    import json
    print("stream evaluation windows:", len(evals))
    if evals:
        m = json.loads(evals[-1][1])
        print("final window: AUC", m.get("AUC"), "Accuracy", m.get("Accuracy"), "LogLoss", m.get("LogLoss"))
    return evals


if __name__ == "__main__":
    main()
