#!/usr/bin/env python3
"""QuantileDiscretizer / Spearman at scale on one device (the P9 sample-sort call sites): ``--rows`` fp64 values in
one column, device-resident, ``QuantileDiscretizerTrainBatchOp`` with ``--buckets`` buckets and a two-column
Spearman ``CorrelationBatchOp``.  Prints one JSON line with the wall times.

    python tools/discretizer_bench.py --rows 100000000 --buckets 100
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--buckets", type=int, default=100)
    ap.add_argument("--spearman-rows", type=int, default=20_000_000)
    a = ap.parse_args()
    from alink_amd import useLocalEnv, QuantileDiscretizerTrainBatchOp, CorrelationBatchOp
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    env = useLocalEnv(1)
    dev = env.device
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(a.rows, generator=g, device=dev, dtype=torch.float64)
    src = TableSourceBatchOp(MTable(TableSchema(["x"], [Types.DOUBLE]), [Column(x)]))
    res = {"rows": a.rows, "buckets": a.buckets, "device": str(dev)}
    for rep in range(2):
        sync()
        t = time.perf_counter()
        m = QuantileDiscretizerTrainBatchOp().setSelectedCols(["x"]).setNumBuckets(a.buckets).linkFrom(src)
        rows = m.collect()
        sync()
        res[f"discretizer_s_{rep}"] = time.perf_counter() - t
    splits = json.loads(rows[1][1])["splitsArray"]
    res["n_splits"] = len(splits)
    res["median_split"] = splits[len(splits) // 2]
    n2 = min(a.spearman_rows, a.rows)
    y = x[:n2] * 0.5 + torch.randn(n2, generator=g, device=dev, dtype=torch.float64)
    src2 = TableSourceBatchOp(MTable(TableSchema(["x", "y"], [Types.DOUBLE, Types.DOUBLE]),
                                     [Column(x[:n2].clone()), Column(y)]))
    for rep in range(2):
        sync()
        t = time.perf_counter()
        c = CorrelationBatchOp().setSelectedCols(["x", "y"]).setMethod("SPEAMAN").linkFrom(src2) \
            .collectCorrelation().getCorrelation()
        sync()
        res[f"spearman_s_{rep}"] = time.perf_counter() - t
    res["spearman_rows"] = n2
    res["spearman_xy"] = float(c[0][1])
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
