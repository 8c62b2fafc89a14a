#!/usr/bin/env python3
"""ALS example (reference examples/.../ALSExample.java): MovieLens-shaped ratings -> ALS (rank 10, 10
iterations, lambda 0.1) -> rating predictions (RMSE) and top-5 recommendations per user.

    python examples/als_example.py [--device cuda:0] [--rows 100000]
"""
import numpy as np
import pandas as pd

from _common import args


def main():
    a = args(100000)
    from alink_amd import (useLocalEnv, BatchOperator, AlsTrainBatchOp, AlsPredictBatchOp, AlsTopKPredictBatchOp,
                           EvalRegressionBatchOp)
    useLocalEnv(1, device=a.device)
    rng = np.random.default_rng(2)
    n_users, n_items, rank = 2000, 1000, 6
    U = rng.normal(size=(n_users, rank)) * 0.6
    V = rng.normal(size=(n_items, rank)) * 0.6
    u = rng.integers(0, n_users, a.rows)
    i = (n_items * rng.random(a.rows) ** 2).astype(np.int64)
    r = np.clip(np.round(3.0 + (U[u] * V[i]).sum(1) + rng.normal(scale=0.3, size=a.rows)), 1, 5)
    df = pd.DataFrame({"user_id": u, "item_id": i, "rating": r}).drop_duplicates(["user_id", "item_id"])
    data = BatchOperator.fromDataframe(df, schemaStr="user_id bigint, item_id bigint, rating double")
    als = AlsTrainBatchOp().setUserCol("user_id").setItemCol("item_id").setRateCol("rating").setNumIter(10) \
        .setRank(10).setLambda(0.1)
    model = als.linkFrom(data)
    pred = AlsPredictBatchOp().setUserCol("user_id").setItemCol("item_id").setPredictionCol("prediction_result") \
        .linkFrom(model, data)
    metrics = EvalRegressionBatchOp().setLabelCol("rating").setPredictionCol("prediction_result").linkFrom(pred) \
        .collectMetrics()
    print("RMSE:", metrics.getRmse())
    users = BatchOperator.fromDataframe(pd.DataFrame({"user_id": [0, 1, 2]}), schemaStr="user_id bigint")
    AlsTopKPredictBatchOp().setUserCol("user_id").setPredictionCol("top5").setTopK(5).linkFrom(model, users).print()
    return metrics


if __name__ == "__main__":
    main()
