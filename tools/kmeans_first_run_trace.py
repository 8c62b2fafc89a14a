#!/usr/bin/env python3
"""Host-side spans of the FIRST KMeans training in a process (the bench's timed run): which superstep items take
long on first use (lazy code-object loads of torch kernels, one-time setup), with cProfile of the slowest step.

    python tools/kmeans_first_run_trace.py [--rows 100000000]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    a = ap.parse_args()
    from alink_amd import useLocalEnv, KMeansTrainBatchOp, RandomVectorSourceBatchOp
    from alink_amd.operator.batch.source import TableSourceBatchOp
    useLocalEnv(1)
    data = RandomVectorSourceBatchOp().setNumRows(a.rows).setSize(128).setNumClusters(100).setClusterStd(1.0) \
        .setCenterScale(4.0).setDtype("bf16").setSeed(2024).setOutputCol("vec").getOutputTable()
    torch.cuda.synchronize()
    walls = []
    prof = cProfile.Profile()

    def on_step(step, q):
        torch.cuda.synchronize()
        walls.append((step, time.perf_counter()))
    op = KMeansTrainBatchOp().setVectorCol("vec").setK(100).setMaxIter(6).setEpsilon(-1.0)
    op._on_step = on_step
    t0 = time.perf_counter()
    prof.enable()
    op.linkFrom(TableSourceBatchOp(data))
    prof.disable()
    prev = t0
    for s, t in walls:
        print(f"step {s}: {1e3 * (t - prev):.1f} ms since previous mark")
        prev = t
    st = io.StringIO()
    pstats.Stats(prof, stream=st).sort_stats("tottime").print_stats(25)
    print(st.getvalue())


if __name__ == "__main__":
    main()
