#!/usr/bin/env python3
"""Is the v10 kernel's time data dependent?  The kernel-bench data set (tools/kmeans_kernel_bench.py: centers x10,
unit noise) against the bench.py data set (RandomVectorSourceBatchOp: centers x4, unit noise, 100 components), each
with centroids near its true centers, plus the bench data with the bench's converged centroids' k (99 live) and
with the serpentine direction alternating.  Event-timed launches, median of --iters.

    python tools/kmeans_data_ab.py [--rows 100000000] [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, iters):
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return round(ts[len(ts) // 2], 4), round(ts[0], 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from alink_amd import useLocalEnv, RandomVectorSourceBatchOp
    from alink_amd.ops import kmeans as K
    useLocalEnv(1)
    dev = torch.device("cuda")
    n, d, k = a.rows, 128, 100
    # kernel-bench data
    X1 = torch.empty((n, d), dtype=torch.bfloat16, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    cen1 = torch.randn(k, d, device=dev, generator=g) * 10
    for s in range(0, n, 1 << 24):
        e = min(n, s + (1 << 24))
        lab = torch.randint(0, k, (e - s,), device=dev, generator=g)
        X1[s:e] = (cen1[lab] + torch.randn(e - s, d, device=dev, generator=g)).to(torch.bfloat16)
    C1 = (cen1 + 0.5 * torch.randn(k, d, device=dev, generator=g)).double()
    # bench data
    src = RandomVectorSourceBatchOp().setNumRows(n).setSize(d).setNumClusters(k).setClusterStd(1.0) \
        .setCenterScale(4.0).setDtype("bf16").setSeed(2024).setOutputCol("vec")
    X2 = src.getOutputTable().col("vec").values
    g2 = torch.Generator(device="cpu").manual_seed(2024)
    cen2 = (torch.randn(k, d, generator=g2, dtype=torch.float64) * 4.0).to(dev)
    C2 = cen2 + 0.5 * torch.randn(k, d, device=dev, dtype=torch.float64)
    res = {"rows": n, "X2_contiguous": X2.is_contiguous(), "X2_align": X2.data_ptr() % 4096,
           "X1_align": X1.data_ptr() % 4096}
    for rnd in range(2):
        for name, X, C in (("kbench_data", X1, C1), ("bench_data", X2, C2), ("bench_data_k99", X2, C2[:99]),
                           ("kbench_data_k99", X1, C1[:99])):
            res[f"{name}_r{rnd}"] = timeit(lambda: K.assign_accumulate_hip(X, C), a.iters)
        flip = [False]

        def alt():
            flip[0] = not flip[0]
            K.assign_accumulate_hip(X2, C2, reverse=flip[0])
        res[f"bench_data_serpentine_r{rnd}"] = timeit(alt, a.iters)
        X2c = X2.clone()
        res[f"bench_data_clone_r{rnd}"] = timeit(lambda: K.assign_accumulate_hip(X2c, C2), a.iters)
        del X2c
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
