#!/usr/bin/env python3
"""BASELINE config 5 end to end: the FTRL click-log StreamOp pipeline of the reference's FTRLExample
(``examples/src/main/java/com/alibaba/alink/FTRLExample.java:45-108``) on one MI355X:

    TableSourceStreamOp (synthetic click log, 20 categorical string fields + label, device-resident)
      -> FeatureHasherStreamOp (1e6 features, Guava murmur3 over "field=value" on the GPU)
      -> FtrlTrainStreamOp (warm start from a batch LR on the first rows; SHARDED or DATA_PARALLEL)
      -> FtrlPredictStreamOp (hot-swaps every model snapshot)  -> EvalBinaryClassStreamOp -> collect

Reports pipeline samples/s (wall of ``StreamOperator.execute`` over the streamed rows), the exclusive host time of
every operator (nested push calls subtracted), the final cumulative AUC / log-loss of the prequential evaluation,
and the snapshot-to-hot-swap latency (snapshot start in the train op -> the predict op serving it).  Run it under
``rocprofv3 --kernel-trace --stats`` to get the device-kernel share of the wall.

    python tools/ftrl_pipeline_bench.py [--rows 4000000] [--batch 65536] [--dim 1000000] [--mode SHARDED]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def click_table(n, fields, per_field, dev, seed=0):
    """n rows of ``fields`` categorical columns (zero-padded decimal value ids as packed UTF-8 on ``dev``, skewed:
    id = per_field * u^3) and an int label drawn from a hidden logistic model over the (field, value) pairs."""
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    g = torch.Generator(device=dev).manual_seed(seed)
    w_true = torch.randn((fields, per_field), generator=g, device=dev, dtype=torch.float64) * 0.6
    u = torch.rand((n, fields), generator=g, device=dev, dtype=torch.float64)
    ids = (per_field * u ** 3).long().clamp_max(per_field - 1)
    margin = w_true.gather(1, ids.T).sum(0) - 0.3
    y = (torch.rand(n, generator=g, device=dev, dtype=torch.float64) < torch.sigmoid(margin)).to(torch.int32)
    width = len(str(per_field - 1))
    pw = 10 ** torch.arange(width - 1, -1, -1, device=dev)
    offsets = torch.arange(n + 1, device=dev, dtype=torch.int64) * width
    cols = []
    for f in range(fields):
        digits = ((ids[:, f:f + 1] // pw) % 10 + 48).to(torch.uint8).reshape(-1).contiguous()
        cols.append(Column(StringBlock(digits, offsets.clone())))
    cols.append(Column(y))
    names = [f"C{f + 1}" for f in range(fields)] + ["label"]
    return MTable(TableSchema(names, [Types.STRING] * fields + [Types.INT]), cols)


class OpTimer:
    """Exclusive host time per operator of the synchronous push DAG (a child's on_batch runs inside its
    parent's _emit, so inclusive times nest; the child's time is subtracted from the parent's)."""

    def __init__(self):
        self.excl, self.calls, self._stack = {}, {}, []

    def wrap(self, op, name):
        orig = op.on_batch

        def timed(port, mt, _orig=orig, _name=name):
            t0 = time.perf_counter()
            self._stack.append(0.0)
            try:
                return _orig(port, mt)
            finally:
                child = self._stack.pop()
                dt = time.perf_counter() - t0
                self.excl[_name] = self.excl.get(_name, 0.0) + dt - child
                self.calls[_name] = self.calls.get(_name, 0) + 1
                if self._stack:
                    self._stack[-1] += dt
        op.on_batch = timed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000, help="streamed rows (after the warm-start rows)")
    ap.add_argument("--init-rows", type=int, default=50_000)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--dim", type=int, default=1_000_000)
    ap.add_argument("--fields", type=int, default=20)
    ap.add_argument("--per-field", type=int, default=100_000)
    ap.add_argument("--mode", default="SHARDED", help="SHARDED | DATA_PARALLEL | HOGWILD | SEQUENTIAL")
    ap.add_argument("--interval", type=int, default=1, help="FTRL snapshot interval (integer seconds, as the reference)")
    ap.add_argument("--async-reduce", action="store_true")
    a = ap.parse_args()
    os.environ["ALINK_STREAM_BATCH"] = str(a.batch)
    from alink_amd import (useLocalEnv, FeatureHasherBatchOp, LogisticRegressionTrainBatchOp, FtrlTrainStreamOp,
                           FtrlPredictStreamOp, EvalBinaryClassStreamOp, FeatureHasherStreamOp, StreamOperator,
                           CollectStreamOp)
    from alink_amd.operator.batch.source import TableSourceBatchOp
    from alink_amd.operator.stream.source import TableSourceStreamOp
    from alink_amd.ops import _lib
    env = useLocalEnv(1)
    dev = env.device
    gpu = dev.type == "cuda"
    if gpu:
        _lib.require()
    sync = (lambda: torch.cuda.synchronize(dev)) if gpu else (lambda: None)
    fields = [f"C{f + 1}" for f in range(a.fields)]
    t_gen = time.perf_counter()
    full = click_table(a.init_rows + a.rows, a.fields, a.per_field, dev)
    init_tab, stream_tab = full.slice(0, a.init_rows), full.slice(a.init_rows, a.init_rows + a.rows)
    sync()
    t_gen = time.perf_counter() - t_gen

    def hasher(cls):
        return cls().setSelectedCols(fields).setCategoricalCols(fields).setOutputCol("vec") \
            .setNumFeatures(a.dim).setReservedCols(["label"])
    t_init = time.perf_counter()
    init_vec = hasher(FeatureHasherBatchOp).linkFrom(TableSourceBatchOp(init_tab))
    init_model = LogisticRegressionTrainBatchOp().setVectorCol("vec").setLabelCol("label").setMaxIter(10) \
        .setWithIntercept(True).linkFrom(init_vec)
    init_model.getOutputTable()
    sync()
    t_init = time.perf_counter() - t_init

    src = TableSourceStreamOp(stream_tab)
    hashed = hasher(FeatureHasherStreamOp).linkFrom(src)
    train = FtrlTrainStreamOp(init_model).setVectorCol("vec").setLabelCol("label").setTimeInterval(a.interval) \
        .setAlpha(0.1).setBeta(0.1).setL1(0.01).setL2(0.01).setWithIntercept(True).setUpdateMode(a.mode)
    if a.async_reduce:
        train.set("asyncGradReduce", True)
    train.linkFrom(hashed)
    pred = FtrlPredictStreamOp(init_model).setVectorCol("vec").setPredictionCol("pred") \
        .setPredictionDetailCol("detail").setReservedCols(["label"]).linkFrom(train, hashed)
    ev = EvalBinaryClassStreamOp().setLabelCol("label").setPredictionDetailCol("detail").linkFrom(pred)
    box = []
    ev.link(CollectStreamOp(box))
    timer = OpTimer()
    for op, name in ((hashed, "FeatureHasherStreamOp"), (train, "FtrlTrainStreamOp"), (pred, "FtrlPredictStreamOp"),
                     (ev, "EvalBinaryClassStreamOp")):
        timer.wrap(op, name)
    sync()
    t0 = time.perf_counter()
    StreamOperator.execute()
    sync()
    wall = time.perf_counter() - t0
    last_all = [json.loads(r[1]) for r in box if r[0] == "all"][-1]
    lat = [train_ms for train_ms in
           ((pred.swap_log[s["bid"]] - s["t_begin"]) * 1e3 for s in train.snapshot_log if s["bid"] in pred.swap_log)]
    excl = {k: round(v, 4) for k, v in timer.excl.items()}
    accounted = sum(timer.excl.values())
    res = {"metric": "FTRL stream pipeline samples/s (source -> FeatureHasher -> FtrlTrain -> FtrlPredict -> "
                     "EvalBinaryClass)",
           "samples_per_s": a.rows / wall, "wall_s": wall, "rows": a.rows, "batch": a.batch, "dim": a.dim,
           "fields": a.fields, "mode": a.mode, "async_reduce": a.async_reduce, "device": str(dev),
           "micro_batches": -(-a.rows // a.batch),
           "op_exclusive_host_s": excl, "source_and_engine_s": round(wall - accounted, 4),
           "op_calls": timer.calls,
           "snapshots": len(train.snapshot_log), "hot_swaps": len(pred.swap_log),
           "snapshot_to_hot_swap_ms": {"n": len(lat), "mean": sum(lat) / len(lat) if lat else None,
                                       "max": max(lat) if lat else None, "first": lat[0] if lat else None},
           "final_all": {k: last_all.get(k) for k in ("AUC", "LogLoss", "Accuracy", "KS", "TotalSamples")},
           "datagen_s": t_gen, "warm_start_s": t_init,
           "data": "synthetic hashed click log (skewed categorical fields, hidden logistic model)"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
