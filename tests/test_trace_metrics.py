"""Tracing (Chrome-trace timeline + roctx) and structured per-superstep metrics."""
import json
import os

import numpy as np
import pytest

from test_distributed import _run


def _kmeans_small():
    from alink_amd import useLocalEnv, KMeansTrainBatchOp, RandomVectorSourceBatchOp
    useLocalEnv(1)
    src = RandomVectorSourceBatchOp().setNumRows(2000).setSize(8).setNumClusters(4).setOutputCol("vec")
    return KMeansTrainBatchOp().setVectorCol("vec").setK(4).setMaxIter(5).linkFrom(src)


def test_trace_spans_nest_and_dump(tmp_path):
    from alink_amd.utils import trace, metrics
    trace.reset()
    trace.enable()
    metrics.clear()
    try:
        _kmeans_small()
        path = trace.dump(str(tmp_path / "t_{rank}.json"))
    finally:
        trace.disable()
    with open(path) as f:
        doc = json.load(f)
    evs = [e for e in doc["traceEvents"] if e["ph"] == "X"]
    cats = {e["cat"] for e in evs}
    assert {"op", "superstep", "item"} <= cats
    ops = [e for e in evs if e["cat"] == "op"]
    assert any(e["name"] == "KMeansTrainBatchOp" for e in ops)
    train = next(e for e in ops if e["name"] == "KMeansTrainBatchOp")
    steps = [e for e in evs if e["cat"] == "superstep"]
    assert steps and all(train["ts"] <= s["ts"] and s["ts"] + s["dur"] <= train["ts"] + train["dur"] + 1.0
                         for s in steps)
    items = {e["name"] for e in evs if e["cat"] == "item"}
    assert "AllReduce(centroidAllReduce)" in items or any(n.startswith("AllReduce") for n in items)
    # metrics: one record per superstep with rows/s
    recs = metrics.records("superstep", job="KMeans")
    assert len(recs) == len(steps)
    assert all(r["rows"] == 2000 and r["rows_per_s"] > 0 for r in recs)


def test_tracing_off_records_nothing():
    from alink_amd.utils import trace
    trace.reset()
    trace.disable()
    _kmeans_small()
    assert trace.events() == []


def test_metrics_loss_curve_and_jsonl(tmp_path):
    from alink_amd import useLocalEnv, LogisticRegressionTrainBatchOp, BatchOperator
    from alink_amd.utils import metrics
    import pandas as pd
    useLocalEnv(1)
    rng = np.random.default_rng(0)
    X = rng.normal(size=(300, 3))
    y = (X @ np.array([1.0, -1.0, 0.5]) > 0).astype(int)
    df = pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "c": X[:, 2], "y": y})
    src = BatchOperator.fromDataframe(df, schemaStr="a double, b double, c double, y int")
    metrics.clear()
    metrics.set_sink(str(tmp_path / "m_{rank}.jsonl"))
    try:
        LogisticRegressionTrainBatchOp().setFeatureCols(["a", "b", "c"]).setLabelCol("y").setMaxIter(10) \
            .linkFrom(src)
    finally:
        metrics.set_sink(None)
    recs = [r for r in metrics.records("superstep") if str(r.get("job", "")).startswith("optim.")]
    assert recs and all("loss" in r for r in recs)
    losses = [r["loss"] for r in recs]
    assert losses[-1] <= losses[0]
    lines = (tmp_path / "m_0.jsonl").read_text().strip().splitlines()
    assert len(lines) >= len(recs)
    assert json.loads(lines[0])["kind"] == "superstep"
    s = metrics.summary(job=recs[0]["job"])
    assert s["steps"] == len(recs) and s["rows_per_s"] > 0


def test_trace_two_ranks_collectives_and_merge(tmp_path):
    from alink_amd.utils import trace
    outs = _run("trace", 2, tmp_path)
    paths = [o["trace"] for o in outs]
    merged = trace.merge(paths, str(tmp_path / "merged.json"))
    with open(merged) as f:
        evs = json.load(f)["traceEvents"]
    pids = {e["pid"] for e in evs if e["ph"] == "X"}
    assert pids == {0, 1}
    coll = [e for e in evs if e["ph"] == "X" and e["cat"] == "collective"]
    assert any(e["name"] == "all_reduce" and e["args"]["bytes"] > 0 for e in coll)
    for o in outs:
        assert o["steps"] and all(r["comm_calls"] >= 1 and r["comm_bytes"] > 0 for r in o["steps"])


@pytest.mark.gpu
def test_trace_kernel_device_track(tmp_path):
    """HIP kernel calls are spans on the host track AND timed on the gpu track from HIP events."""
    import torch
    from alink_amd.utils import trace
    from alink_amd.ops import kmeans as kops, _lib
    _lib.require()
    X = torch.randn(200000, 128, device="cuda").to(torch.bfloat16)
    C = torch.randn(16, 128, device="cuda", dtype=torch.float64)
    trace.reset()
    trace.enable()
    try:
        for _ in range(3):
            kops.assign_accumulate_hip(X, C)
        path = trace.dump(str(tmp_path / "g_{rank}.json"))
    finally:
        trace.disable()
    with open(path) as f:
        evs = json.load(f)["traceEvents"]
    host = [e for e in evs if e.get("cat") == "kernel"]
    gpu = [e for e in evs if e.get("cat") == "kernel.gpu"]
    name = f"kmeans_assign_accum_bf16_{kops.kernel_version(16)}"      # the production kernel for k = 16
    assert any(e["name"] == name for e in host)
    ks = [e for e in gpu if e["name"] == name]
    assert len(ks) == 3 and all(e["dur"] > 0 for e in ks)
    assert all(e["tid"] == "gpu" for e in gpu)
