#!/usr/bin/env python3
"""Host-side profile (cProfile) of one KMeans convergence run on the bench data (the bench's
convergence.reference run, after a first identical run has paid the one-time costs): where the wall time outside
the kernels goes.  Prints the top functions by cumulative and by own time.

    python tools/kmeans_host_profile.py [--rows 100000000] [--k 100]
"""
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
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    from alink_amd import useLocalEnv, RandomVectorSourceBatchOp, KMeansTrainBatchOp
    from alink_amd.operator.batch.source import TableSourceBatchOp
    env = useLocalEnv(1)
    dev = env.device
    src = RandomVectorSourceBatchOp().setNumRows(a.rows).setSize(128).setNumClusters(a.k) \
        .setClusterStd(1.0).setCenterScale(4.0).setDtype("bf16").setSeed(2024).setOutputCol("vec")
    data = src.getOutputTable()
    torch.cuda.synchronize(dev)

    def run():
        op = KMeansTrainBatchOp().setVectorCol("vec").setK(a.k).setMaxIter(100).setInitSteps(2)
        op.linkFrom(TableSourceBatchOp(data))
        return op
    run()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    run()
    torch.cuda.synchronize(dev)
    print(f"unprofiled wall {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
    pr = cProfile.Profile()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    pr.enable()
    run()
    torch.cuda.synchronize(dev)
    pr.disable()
    print(f"profiled wall {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
