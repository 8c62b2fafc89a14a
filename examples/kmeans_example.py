#!/usr/bin/env python3
"""KMeans example (reference examples/.../KMeansExample.java; BASELINE config 1): iris-shaped CSV ->
VectorAssembler -> KMeans(k=3, maxIter=100) -> predictions + cluster evaluation.

    python examples/kmeans_example.py [--device cuda:0]
"""
import os

import numpy as np

from _common import args


def main():
    a = args(150)
    from alink_amd import (useLocalEnv, CsvSourceBatchOp, VectorAssembler, KMeans, Pipeline, EvalClusterBatchOp)
    useLocalEnv(1, device=a.device)
    rng = np.random.default_rng(0)
    centers = np.array([[5.0, 3.4, 1.5, 0.2], [5.9, 2.8, 4.3, 1.3], [6.6, 3.0, 5.6, 2.0]])
    path = os.path.join(a.workdir, "iris_like.csv")
    with open(path, "w") as f:
        for i in range(a.rows):
            c = i % 3
            x = centers[c] + rng.normal(scale=0.25, size=4)
            f.write(",".join(f"{v:.1f}" for v in x) + f",Iris-{['setosa', 'versicolor', 'virginica'][c]}\n")
    data = CsvSourceBatchOp().setFilePath(path).setSchemaStr(
        "sepal_length double, sepal_width double, petal_length double, petal_width double, category string")
    va = VectorAssembler().setSelectedCols(["sepal_length", "sepal_width", "petal_length", "petal_width"]) \
        .setOutputCol("features")
    km = KMeans().setVectorCol("features").setK(3).setMaxIter(100).setPredictionCol("prediction_result") \
        .setPredictionDetailCol("prediction_detail")
    model = Pipeline().add(va).add(km).fit(data)
    pred = model.transform(data)
    pred.firstN(5).print()
    metrics = EvalClusterBatchOp().setVectorCol("features").setPredictionCol("prediction_result") \
        .setLabelCol("category").linkFrom(pred).collectMetrics()
    print("purity:", metrics.getPurity(), "NMI:", metrics.getNmi())
    return metrics


if __name__ == "__main__":
    main()
