"""Two-pass general HIP KMeans path (nearest + accumulate-by-index) vs the fused v7 kernel and vs torch, per
(d, k): ms per assign+accumulate call and rows/s.  Usage: python tools/kmeans_general_bench.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    from alink_amd.ops import kmeans as K
    res = []
    for d, k, n in [(64, 100, 100_000_000), (64, 500, 50_000_000), (128, 100, 100_000_000), (128, 256, 50_000_000),
                    (256, 100, 50_000_000), (256, 256, 50_000_000)]:
        g = torch.Generator(device="cuda").manual_seed(d + k)
        X = torch.randn(n, d, device="cuda", generator=g, dtype=torch.float32).to(torch.bfloat16)
        C = torch.randn(k, d, device="cuda", generator=g, dtype=torch.float64)
        t_gen = timeit(lambda: K.assign_accumulate_general_hip(X, C))
        idx, _ = K.nearest_hip(X, C)
        t_near = timeit(lambda: K.nearest_hip(X, C))
        t_acc = timeit(lambda: K.accumulate_by_index_hip(X, idx, k))
        r = {"d": d, "k": k, "rows": n, "general_ms": round(t_gen, 3), "nearest_ms": round(t_near, 3),
             "accum_ms": round(t_acc, 3), "general_rows_per_s": n / t_gen * 1e3,
             "x_GBps_per_pass": round(n * d * 2 / t_near / 1e6, 1)}
        if K.hip_supported(X, k):
            r["v7_ms"] = round(timeit(lambda: K.assign_accumulate_hip(X, C)), 3)
        m = 10_000_000
        r["torch_ms_per_1e7_rows"] = round(timeit(lambda: K.assign_accumulate_torch(X[:m], C), reps=2), 2)
        print(json.dumps(r), flush=True)
        res.append(r)
        del X, idx
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
