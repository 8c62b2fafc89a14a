"""End-to-end effect of the split-K row products (ops/gemm.py) on 1 GPU: PCA, GLM (IRLS) and Newton linear
regression training on a dense fp64 table, with tn_matmul enabled vs disabled (plain library A^T B)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from alink_amd import useLocalEnv, PcaTrainBatchOp, GlmTrainBatchOp, LinearRegTrainBatchOp  # noqa: E402
from alink_amd.common.table import Column, MTable  # noqa: E402
from alink_amd.common.types import TableSchema, Types  # noqa: E402
from alink_amd.operator.batch.source import TableSourceBatchOp  # noqa: E402
from alink_amd.ops import gemm  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
    dev = sys.argv[2] if len(sys.argv) > 2 else "cuda:0"
    d = 64
    env = useLocalEnv(1, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(n, d, device=dev, dtype=torch.float64, generator=g)
    y = X @ torch.randn(d, device=dev, dtype=torch.float64, generator=g) + \
        0.1 * torch.randn(n, device=dev, dtype=torch.float64, generator=g)
    names = [f"f{i}" for i in range(d)]
    cols = [Column(X[:, i].contiguous()) for i in range(d)] + [Column(y)]
    mt = MTable(TableSchema(names + ["label"], [Types.DOUBLE] * (d + 1)), cols)
    src = TableSourceBatchOp(mt)

    def sync():
        if X.is_cuda:
            torch.cuda.synchronize()
    cases = {
        "PCA k=8": lambda: PcaTrainBatchOp().setSelectedCols(names).setK(8).linkFrom(src).collect(),
        "GLM gaussian": lambda: GlmTrainBatchOp().setFeatureCols(names).setLabelCol("label").linkFrom(src).collect(),
        "LinearReg Newton": lambda: LinearRegTrainBatchOp().setFeatureCols(names).setLabelCol("label")
        .setOptimMethod("Newton").setMaxIter(5).linkFrom(src).collect(),
    }
    for name, fn in cases.items():
        res = {}
        for mode in ("splitk", "plain"):
            gemm._MIN_ROWS = 4 * gemm.CHUNK if mode == "splitk" else 1 << 62
            fn()
            sync()
            t = time.perf_counter()
            fn()
            sync()
            res[mode] = time.perf_counter() - t
        print(f"{name} n={n} d={d} fp64: split-K {res['splitk'] * 1e3:.1f} ms  plain {res['plain'] * 1e3:.1f} ms  "
              f"({res['plain'] / res['splitk']:.1f}x)", flush=True)
    del env


if __name__ == "__main__":
    main()
