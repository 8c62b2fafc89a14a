#!/usr/bin/env python3
"""Random forest with the default unbounded depth: per-level time (TreeBuilder.LEVEL_STATS: depth, nodes, split
candidates, wall s) and the tree time under maxMemoryInMB 64 (default) vs unbounded.

    python tools/rf_level_bench.py --rows 1000000 --features 100
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
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=100)
    ap.add_argument("--trees", type=int, default=1)
    a = ap.parse_args()
    from alink_amd import useLocalEnv, RandomForestTrainBatchOp
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.tree.engine import TreeBuilder
    from alink_amd.operator.batch.source import TableSourceBatchOp
    env = useLocalEnv(1)
    dev = env.device
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(a.rows, a.features, generator=g, device=dev, dtype=torch.float64)
    y = ((X[:, 0] + torch.sin(3 * X[:, 1]) + X[:, 2] * X[:, 3]
          + 0.5 * torch.randn(a.rows, generator=g, device=dev, dtype=torch.float64)) > 0).to(torch.int32)
    names = [f"f{i}" for i in range(a.features)]
    src = TableSourceBatchOp(MTable(TableSchema(names + ["label"], [Types.DOUBLE] * a.features + [Types.INT]),
                                    [Column(X[:, i].contiguous()) for i in range(a.features)] + [Column(y)]))
    out = {"rows": a.rows, "features": a.features, "trees": a.trees, "device": str(dev)}
    models = {}
    for mem in (64, 1 << 20):
        TreeBuilder.LEVEL_STATS.clear()
        t = time.perf_counter()
        m = RandomForestTrainBatchOp().setFeatureCols(names).setLabelCol("label").setNumTrees(a.trees) \
            .setMaxMemoryInMB(mem).linkFrom(src)
        models[mem] = m.collect()[1:]
        out[f"train_s_mem{mem}"] = time.perf_counter() - t
        out[f"levels_mem{mem}"] = [(d, n, c, round(s, 4)) for d, n, c, s in TreeBuilder.LEVEL_STATS]
    out["identical_trees"] = models[64] == models[1 << 20]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
