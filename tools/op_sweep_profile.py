#!/usr/bin/env python3
"""Host hot-spot sweep: common batch ops on synthetic device tables at production-ish sizes, each run twice (the
first pays one-time costs), the second timed and cProfiled; prints the wall time and the top functions by own
time per op, so Python-level loops over rows / model entries stand out.

    python tools/op_sweep_profile.py [--rows 10000000] [--only kmeans_predict,...]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--only", default="")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    import alink_amd as A
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    env = A.useLocalEnv(1)
    dev = env.device
    n = a.rows
    g = torch.Generator(device=dev).manual_seed(0)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    # shared tables
    vec = A.RandomVectorSourceBatchOp().setNumRows(n).setSize(128).setNumClusters(100).setClusterStd(1.0) \
        .setCenterScale(4.0).setDtype("bf16").setSeed(7).setOutputCol("vec").getOutputTable()
    F = 20
    cols = [Column(torch.randn(n, generator=g, device=dev, dtype=torch.float64)) for _ in range(F)]
    y = (cols[0].values + 0.5 * cols[1].values > 0).to(torch.int32)
    names = [f"x{i}" for i in range(F)]
    dense = MTable(TableSchema(names + ["label"], [Types.DOUBLE] * F + [Types.INT]), cols + [Column(y)])
    cats = torch.randint(0, 1000, (n,), generator=g, device=dev)
    from alink_amd.common.strings import StringBlock
    vocab = StringBlock.from_list([f"cat_{i}" for i in range(1000)]).to(dev)
    catcol = MTable(TableSchema(["c"], [Types.STRING]), [Column(vocab.take(cats))])
    probs = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    lab = (torch.rand(n, generator=g, device=dev) < probs).to(torch.int32)
    sync()

    km_model = A.KMeansTrainBatchOp().setVectorCol("vec").setK(100).setMaxIter(3) \
        .linkFrom(TableSourceBatchOp(vec))
    lr_model = A.LogisticRegressionTrainBatchOp().setFeatureCols(names).setLabelCol("label").setMaxIter(5) \
        .linkFrom(TableSourceBatchOp(dense))
    si_model = A.StringIndexerTrainBatchOp().setSelectedCol("c").linkFrom(TableSourceBatchOp(catcol))
    oh_model = A.OneHotTrainBatchOp().setSelectedCols(["c"]).linkFrom(TableSourceBatchOp(catcol))
    qd_model = A.QuantileDiscretizerTrainBatchOp().setSelectedCols(names[:5]).setNumBuckets(16) \
        .linkFrom(TableSourceBatchOp(dense))

    det = MTable(TableSchema(["label", "p"], [Types.INT, Types.DOUBLE]), [Column(lab), Column(probs)])

    jobs = {
        "kmeans_predict": lambda: A.KMeansPredictBatchOp().setPredictionCol("pred").setReservedCols([])
        .linkFrom(km_model, TableSourceBatchOp(vec)).getOutputTable().col("pred").values,
        "lr_train": lambda: A.LogisticRegressionTrainBatchOp().setFeatureCols(names).setLabelCol("label")
        .setMaxIter(5).linkFrom(TableSourceBatchOp(dense)).getOutputTable(),
        "lr_predict": lambda: A.LogisticRegressionPredictBatchOp().setPredictionCol("p")
        .setPredictionDetailCol("d").setReservedCols([]).linkFrom(lr_model, TableSourceBatchOp(dense))
        .getOutputTable().col("p").values,
        "string_indexer_train": lambda: A.StringIndexerTrainBatchOp().setSelectedCol("c")
        .linkFrom(TableSourceBatchOp(catcol)).getOutputTable(),
        "string_indexer_predict": lambda: A.StringIndexerPredictBatchOp().setSelectedCol("c").setOutputCol("ci")
        .linkFrom(si_model, TableSourceBatchOp(catcol)).getOutputTable().col("ci").values,
        "onehot_predict": lambda: A.OneHotPredictBatchOp().setSelectedCols(["c"]).setOutputCols(["oh"])
        .linkFrom(oh_model, TableSourceBatchOp(catcol)).getOutputTable().col("oh").values,
        "quantile_predict": lambda: A.QuantileDiscretizerPredictBatchOp().setSelectedCols(names[:5])
        .linkFrom(qd_model, TableSourceBatchOp(dense)).getOutputTable(),
        "vector_assembler": lambda: A.VectorAssemblerBatchOp().setSelectedCols(names).setOutputCol("v")
        .setReservedCols([]).linkFrom(TableSourceBatchOp(dense)).getOutputTable().col("v").values,
        "eval_binary": lambda: A.EvalBinaryClassBatchOp().setLabelCol("label").setPredictionDetailCol("d")
        .linkFrom(A.LogisticRegressionPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d")
                  .setReservedCols(["label"]).linkFrom(lr_model, TableSourceBatchOp(dense))).collect(),
        "standard_scaler_train": lambda: A.StandardScalerTrainBatchOp().setSelectedCols(names)
        .linkFrom(TableSourceBatchOp(dense)).getOutputTable(),
    }
    only = [s for s in a.only.split(",") if s]
    for name, fn in jobs.items():
        if only and name not in only:
            continue
        try:
            fn()
            sync()
            pr = cProfile.Profile()
            t = time.perf_counter()
            pr.enable()
            fn()
            sync()
            pr.disable()
            wall = time.perf_counter() - t
        except Exception as e:          # keep sweeping; report the op
            print(f"== {name}: FAILED {type(e).__name__}: {e}", flush=True)
            continue
        sio = io.StringIO()
        pstats.Stats(pr, stream=sio).sort_stats("tottime").print_stats(a.top)
        lines = [ln for ln in sio.getvalue().splitlines() if ln.strip() and ("(" in ln or "ncalls" in ln)]
        print(f"== {name}: {wall:.3f} s for {n} rows ({n / wall:.3g} rows/s)", flush=True)
        for ln in lines[:a.top + 1]:
            print("   " + ln[:170], flush=True)


if __name__ == "__main__":
    main()
