"""Diagnostics of KMeans convergence on the bench data: per-step max centroid shift + final cluster sizes."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from alink_amd import useLocalEnv, KMeansTrainBatchOp, RandomVectorSourceBatchOp
from alink_amd.operator.batch.source import TableSourceBatchOp

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--k", type=int, default=100)
ap.add_argument("--iters", type=int, default=100)
ap.add_argument("--init-steps", type=int, default=2)
ap.add_argument("--dtype", default="bf16")
a = ap.parse_args()
env = useLocalEnv(1)
src = RandomVectorSourceBatchOp().setNumRows(a.rows).setSize(128).setNumClusters(a.k) \
    .setClusterStd(1.0).setCenterScale(4.0).setDtype(a.dtype).setSeed(2024).setOutputCol("vec")
data = src.getOutputTable()
t = time.perf_counter()
op = KMeansTrainBatchOp().setVectorCol("vec").setK(a.k).setMaxIter(a.iters).setInitSteps(a.init_steps)
op.linkFrom(TableSourceBatchOp(data))
info = op.getTrainInfo()
hist = info["max_shift"]
print(json.dumps({"iterations": info["iterations"], "wall_s": time.perf_counter() - t,
                  "dtype": a.dtype, "shift_first10": hist[:10], "shift_last10": hist[-10:],
                  "shift_every10": hist[::10]}))
