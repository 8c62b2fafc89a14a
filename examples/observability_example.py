#!/usr/bin/env python3
"""Observability example: one KMeans + one logistic-regression job with the timeline tracer, the per-superstep
metrics and a DirectReader-served stream predictor (SURVEY §5.1 / §5.5 / §2.5 DirectReader).

    python examples/observability_example.py [--device cuda:0]

Writes ``<workdir>/trace_0.json`` (open in chrome://tracing or Perfetto: op / superstep / item / collective /
kernel spans; on a GPU also the device-time "gpu stream" track) and ``<workdir>/metrics_0.jsonl`` (one record per
superstep: wall time, rows/s, collective calls / bytes / time, the optimizer's loss).
"""
import json
import os

import numpy as np

from _common import args


def main():
    a = args(20000)
    from alink_amd import (useLocalEnv, BatchOperator, RandomVectorSourceBatchOp, KMeansTrainBatchOp,
                           KMeansPredictStreamOp, LogisticRegressionTrainBatchOp, StreamOperator)
    from alink_amd.common.directreader import DirectReaderPropertiesStore
    from alink_amd.operator.stream.source import TableSourceStreamOp
    from alink_amd.operator.stream.utils import CollectStreamOp
    from alink_amd.utils import metrics, trace
    import pandas as pd

    useLocalEnv(1, device=a.device)
    trace.reset()
    trace.enable(os.path.join(a.workdir, "trace_{rank}.json"))
    metrics.set_sink(os.path.join(a.workdir, "metrics_{rank}.jsonl"))

    src = RandomVectorSourceBatchOp().setNumRows(a.rows).setSize(16).setNumClusters(5).setOutputCol("vec")
    model = KMeansTrainBatchOp().setVectorCol("vec").setK(5).setMaxIter(10).linkFrom(src)

    rng = np.random.default_rng(0)
    X = rng.normal(size=(a.rows, 4))
    y = (X @ np.array([1.0, -1.0, 0.5, 2.0]) > 0).astype(int)
    df = pd.DataFrame({f"f{i}": X[:, i] for i in range(4)})
    df["y"] = y
    LogisticRegressionTrainBatchOp().setFeatureCols([f"f{i}" for i in range(4)]).setLabelCol("y").setMaxIter(15) \
        .linkFrom(BatchOperator.fromDataframe(df, schemaStr="f0 double, f1 double, f2 double, f3 double, y int"))

    # the stream predictor gets the batch model through DirectReader; the db policy stages it in a table
    DirectReaderPropertiesStore.setProperties({"direct.reader.policy": "db",
                                               "direct.reader.db.path": os.path.join(a.workdir, "bridge.sqlite")})
    box = []
    KMeansPredictStreamOp(model).setPredictionCol("pred").linkFrom(TableSourceStreamOp(src.getOutputTable())) \
        .link(CollectStreamOp(box))
    StreamOperator.execute()
    DirectReaderPropertiesStore.clear()

    path = trace.dump()
    trace.disable()
    metrics.set_sink(None)
    evs = [e for e in json.load(open(path))["traceEvents"] if e.get("ph") == "X"]
    cats = sorted({e["cat"] for e in evs})
    km = metrics.summary(job="KMeans")
    lr = [r for r in metrics.records("superstep") if str(r.get("job", "")).startswith("optim.")]
    print("trace:", path, "events:", len(evs), "categories:", cats)
    print("KMeans supersteps:", km["steps"], "rows/s: %.3g" % km.get("rows_per_s", 0.0))
    print("LR loss curve:", [round(r["loss"], 5) for r in lr][:5], "...")
    print("stream predictions:", len(box))
    return km


if __name__ == "__main__":
    main()
