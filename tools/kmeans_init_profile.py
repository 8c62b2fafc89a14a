#!/usr/bin/env python3
"""Where the KMeans k-means|| initialisation spends its time (bench data: 1e8 x 128 bf16, k = 100, initSteps 2,
the reference seeding rule).  Each helper of ``models/clustering/kmeans.py`` is wrapped with a device-synchronised
wall timer; ``other`` is the rest of ``kmeans_init`` (threshold sums, the oversampling draw, the candidate gather).
Then one full ``KMeansTrainBatchOp`` run to convergence, split into init / supersteps / the rest.

    python tools/kmeans_init_profile.py [--rows 100000000] [--k 100] [--reps 3]
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
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--init-steps", type=int, default=2)
    a = ap.parse_args()
    from alink_amd import useLocalEnv, RandomVectorSourceBatchOp, KMeansTrainBatchOp
    from alink_amd.models.clustering import kmeans as km
    from alink_amd.operator.batch.source import TableSourceBatchOp
    env = useLocalEnv(1)
    dev = env.device
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    src = RandomVectorSourceBatchOp().setNumRows(a.rows).setSize(128).setNumClusters(a.k) \
        .setClusterStd(1.0).setCenterScale(4.0).setDtype("bf16").setSeed(2024).setOutputCol("vec")
    data = src.getOutputTable()
    X = data.col("vec").values
    sync()
    acc = {}

    def wrap(name, fn):
        def w(*args, **kw):
            sync()
            t = time.perf_counter()
            r = fn(*args, **kw)
            sync()
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
            return r
        return w
    orig = {n: getattr(km, n) for n in ("_min_dist_to", "_nearest", "_local_kmeans", "_fetch_global_rows",
                                        "_global_count")}
    for n, f in orig.items():
        setattr(km, n, wrap(n, f))
    counts_orig = km.kops.nearest_counts_hip          # the candidate weights pass (one kernel, counts mode)
    km.kops.nearest_counts_hip = wrap("nearest_counts", counts_orig)
    res = {"rows": a.rows, "k": a.k, "initSteps": a.init_steps, "device": str(dev), "reps": []}
    for _ in range(a.reps):
        acc.clear()
        sync()
        t = time.perf_counter()
        C = km.kmeans_init(X, a.k, "K_MEANS_PARALLEL", a.init_steps, "EUCLIDEAN", seed=0)
        sync()
        tot = time.perf_counter() - t
        rep = {k: round(v * 1e3, 3) for k, v in acc.items()}
        rep["other"] = round((tot - sum(acc.values())) * 1e3, 3)
        rep["total_ms"] = round(tot * 1e3, 3)
        rep["k_out"] = int(C.shape[0])
        res["reps"].append(rep)
    for n, f in orig.items():
        setattr(km, n, f)
    km.kops.nearest_counts_hip = counts_orig
    # split of one full training run (the bench's convergence.reference run)
    marks = {}
    init_orig = km.kmeans_init

    def init_timed(*args, **kw):
        sync()
        marks["init0"] = time.perf_counter()
        r = init_orig(*args, **kw)
        sync()
        marks["init1"] = time.perf_counter()
        return r
    km.kmeans_init = init_timed
    sync()
    t = time.perf_counter()
    op = KMeansTrainBatchOp().setVectorCol("vec").setK(a.k).setMaxIter(100).setInitSteps(a.init_steps)
    op.linkFrom(TableSourceBatchOp(data))
    sync()
    wall = time.perf_counter() - t
    km.kmeans_init = init_orig
    st = op._queue.stats
    step_s = sum(s.get("wall_s", 0.0) for s in st) if st and "wall_s" in st[0] else None
    res["train"] = {"wall_ms": round(wall * 1e3, 3), "init_ms": round((marks["init1"] - marks["init0"]) * 1e3, 3),
                    "iterations": op.getTrainInfo()["iterations"],
                    "supersteps_ms": None if step_s is None else round(step_s * 1e3, 3),
                    "step_wall_ms": [round(s.get("wall_s", 0.0) * 1e3, 3) for s in st],
                    "stats_keys": sorted(st[0].keys()) if st else []}
    # a second identical run: one-time costs (workspaces, operand buffers) are paid by the first
    sync()
    t = time.perf_counter()
    op = KMeansTrainBatchOp().setVectorCol("vec").setK(a.k).setMaxIter(100).setInitSteps(a.init_steps)
    op.linkFrom(TableSourceBatchOp(data))
    sync()
    res["train2"] = {"wall_ms": round((time.perf_counter() - t) * 1e3, 3),
                     "step_wall_ms": [round(s.get("wall_s", 0.0) * 1e3, 3) for s in op._queue.stats]}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
