"""GBDT training throughput on a synthetic HIGGS-shaped table (n rows x F float features, binary label).

    python tools/gbdt_bench.py --rows 10000000 --features 28 --trees 20 --depth 6
    python tools/gbdt_bench.py --rows 100000000 --features 1000 --trees 20 --depth 8 --prebinned 1

Prints one JSON line: rows, features, trees, seconds, ms/tree, rows*trees/s, and per tree depth the mean host
wall time of a level (TreeBuilder.LEVEL_STATS).

``--prebinned 1`` (BASELINE config 3 at its full size on one GPU): the raw table would be 1e8 x 1000 fp32 = 400 GB,
more than one MI355X holds, so the rows are generated directly as the uint8 bin matrix the trainer keeps in HBM
(1e8 x 1000 = 100 GB, uniform bins 0..127, the label a noisy function of two features) and the binning stage
(``build_bins``, measured separately at the per-rank shape) is bypassed; everything from the gradient statistics
to the serialized model runs as in a normal job.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1000000)
    ap.add_argument("--features", type=int, default=28)
    ap.add_argument("--trees", type=int, default=20)
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--bins", type=int, default=128)
    ap.add_argument("--dtype", default="float64", choices=["float32", "float64"])
    ap.add_argument("--prebinned", type=int, default=0, help="1: generate the uint8 bin matrix directly")
    ap.add_argument("--ranks", type=int, default=8,
                    help="world size for the projected per-rank reduce-scatter traffic per level")
    a = ap.parse_args()
    from alink_amd import useLocalEnv, GbdtTrainBatchOp
    from alink_amd.common.table import MTable, Column
    from alink_amd.common.types import TableSchema, Types
    env = useLocalEnv(1)
    dev = env.device
    if a.prebinned:
        return prebinned(a, env)
    g = torch.Generator(device=dev).manual_seed(0)
    dt = getattr(torch, a.dtype)
    # one column tensor per feature (the MTable layout), generated on the device
    score = torch.zeros(a.rows, device=dev, dtype=torch.float32)
    cols = []
    for i in range(a.features):
        x = torch.randn(a.rows, generator=g, device=dev, dtype=torch.float32)
        score += x * (2.0 * i / max(1, a.features - 1) - 1.0)
        if i == 0:
            score += 0.5 * torch.sin(3 * x)
        cols.append(Column(x.to(dt)))
    y = ((score + 0.3 * torch.randn(a.rows, generator=g, device=dev)) > 0).to(torch.int32)
    del score
    names = [f"f{i}" for i in range(a.features)] + ["label"]
    cols.append(Column(y))
    ftype = Types.DOUBLE if a.dtype == "float64" else Types.FLOAT
    mt = MTable(TableSchema(names, [ftype] * a.features + [Types.INT]), cols)
    from alink_amd.operator.batch.source import TableSourceBatchOp
    src = TableSourceBatchOp(mt)
    op = GbdtTrainBatchOp().setFeatureCols(names[:-1]).setLabelCol("label").setNumTrees(a.trees) \
        .setMaxDepth(a.depth).setMaxBins(a.bins).setMinSamplesPerLeaf(100)
    from alink_amd.models.tree.engine import TreeBuilder
    TreeBuilder.HIST_BYTES.clear()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.time()
    op.linkFrom(src)
    op.getOutputTable()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.time() - t0
    info = op.getTrainInfo() if hasattr(op, "getTrainInfo") else {}
    B = (info or {}).get("bins", a.bins + 1)
    # bytes of the per-level histogram all-reduce at the deepest level (nodes/2 built slots x F x B x 3 fp32)
    hist_bytes = (2 ** (a.depth - 1)) // 2 * a.features * B * 3 * 4
    print(json.dumps({"rows": a.rows, "features": a.features, "trees": a.trees, "depth": a.depth,
                      "seconds": round(dt, 3), "ms_per_tree": round(1000 * dt / a.trees, 2),
                      "row_trees_per_s": a.rows * a.trees / dt, "device": str(dev), "feature_dtype": a.dtype,
                      "hist_allreduce_bytes_deepest_level": hist_bytes,
                      "bin_matrix_bytes": a.rows * a.features, "binning_s": (info or {}).get("binning_s"),
                      "trees_s": (info or {}).get("trees_s"),
                      "s_per_tree": ((info or {}).get("trees_s") or dt) / a.trees,
                      # histogram calls of the whole run (root + one per level per tree): the full-width bytes
                      # every rank reduce-scatters, and what one rank sends = (P-1)/P of it at P = --ranks
                      "hist_bytes_per_level_tree0": list(TreeBuilder.HIST_BYTES)[:a.depth],
                      "reduce_scatter_send_bytes_per_rank_per_tree": int(sum(TreeBuilder.HIST_BYTES) / a.trees
                                                                          * (a.ranks - 1) / a.ranks),
                      "projected_ranks": a.ranks}))


def prebinned(a, env):
    from alink_amd import GbdtTrainBatchOp
    from alink_amd.common.table import MTable, Column
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.tree import train as T
    from alink_amd.models.tree.data import BinnedData
    from alink_amd.models.tree.engine import TreeBuilder
    from alink_amd.operator.batch.source import TableSourceBatchOp
    dev = env.device
    n, F, nb = a.rows, a.features, a.bins
    t0 = time.time()
    g = torch.Generator(device=dev).manual_seed(0)
    bins = torch.empty((n, F), dtype=torch.uint8, device=dev)
    step = max(1, (1 << 33) // F)                      # 8 GiB of bins per generator call
    for lo in range(0, n, step):
        bins[lo:lo + step].random_(0, nb, generator=g)
    score = (bins[:, 0].float() - (nb - 1) / 2) + 0.5 * (bins[:, 1].float() - (nb - 1) / 2)
    y = ((score + 8.0 * torch.randn(n, generator=g, device=dev)) > 0).to(torch.int32)
    del score
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t_gen = time.time() - t0
    thr = np.arange(nb - 1, dtype=np.float64) + 0.5
    data = BinnedData(bins, nb + 1, [f"f{i}" for i in range(F)], [False] * F, [nb] * F, [thr] * F)
    names = [f"f{i}" for i in range(F)] + ["label"]
    zero = torch.zeros(1, dtype=torch.float32, device=dev).expand(n)   # schema-only feature columns (no memory)
    mt = MTable(TableSchema(names, [Types.FLOAT] * F + [Types.INT]), [Column(zero)] * F + [Column(y)])
    orig = T.build_bins
    T.build_bins = lambda *args, **kw: data
    TreeBuilder.LEVEL_STATS.clear()
    TreeBuilder.HIST_BYTES.clear()
    try:
        op = GbdtTrainBatchOp().setFeatureCols(names[:-1]).setLabelCol("label").setNumTrees(a.trees) \
            .setMaxDepth(a.depth).setMaxBins(nb).setMinSamplesPerLeaf(100)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t1 = time.time()
        op.linkFrom(TableSourceBatchOp(mt))
        op.getOutputTable()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        wall = time.time() - t1
    finally:
        T.build_bins = orig
    info = op.getTrainInfo() or {}
    levels = {}
    for d, nodes, cand, host_s in TreeBuilder.LEVEL_STATS:
        levels.setdefault(int(d), []).append(float(host_s))
    print(json.dumps({"rows": n, "features": F, "trees": a.trees, "depth": a.depth, "prebinned": True,
                      "bin_matrix_gb": n * F / 1e9, "datagen_s": round(t_gen, 2), "wall_s": round(wall, 3),
                      "trees_s": info.get("trees_s"), "s_per_tree": (info.get("trees_s") or wall) / a.trees,
                      "rows_per_s": n * a.trees / (info.get("trees_s") or wall),
                      "level_host_wall_ms_mean": {d: round(1e3 * float(np.mean(v)), 3) for d, v in sorted(levels.items())},
                      "hist_bytes_per_level_tree0": list(TreeBuilder.HIST_BYTES)[:a.depth],
                      "peak_mem_gb": (torch.cuda.max_memory_allocated(dev) / 1e9) if dev.type == "cuda" else None,
                      "device": str(dev)}), flush=True)


if __name__ == "__main__":
    main()
