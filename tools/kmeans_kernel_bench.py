#!/usr/bin/env python3
"""Micro-benchmark of the fused KMeans assign+accumulate HIP kernel vs the PyTorch path.

python tools/kmeans_kernel_bench.py --rows 100000000 --k 100 --iters 10
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from alink_amd.ops import kmeans as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--torch", action="store_true", help="also time the PyTorch path")
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--load-only", action="store_true", help="time the LDS-DMA load pipeline alone")
    ap.add_argument("--compute-only", action="store_true", help="time the compute alone (no loads)")
    ap.add_argument("--var", type=int, default=0, help="v7 DMA variant (mode bits 4-5)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    n, d, k = a.rows, 128, a.k
    X = torch.empty((n, d), dtype=torch.bfloat16, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    centers = torch.randn(k, d, device=dev, generator=g) * 10
    B = 1 << 24
    for s in range(0, n, B):
        e = min(n, s + B)
        lab = torch.randint(0, k, (e - s,), device=dev, generator=g)
        X[s:e] = (centers[lab] + torch.randn(e - s, d, device=dev, generator=g)).to(torch.bfloat16)
    C = (centers + 0.5 * torch.randn(k, d, device=dev, generator=g)).double()
    def run(Xs):
        m = 2 if a.compute_only else 1 if a.load_only else 0
        return K.assign_accumulate_hip(Xs, C, grid=a.grid, mode=m | (a.var << 4))
    out = run(X)
    torch.cuda.synchronize()
    res = {"rows": n, "k": k, "load_only": a.load_only, "compute_only": a.compute_only, "var": a.var}
    if a.torch:
        ref0 = K.assign_accumulate_torch(X[:2_000_000], C)
        got0 = run(X[:2_000_000].contiguous())
        res["small_count_diff"] = float((got0[:, -1] - ref0[:, -1]).abs().sum().item())
    times = []
    for _ in range(a.iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = run(X)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t = sorted(times)[len(times) // 2]
    res.update({"hip_ms": t * 1e3, "hip_rows_per_s": n / t, "hip_GBps": n * d * 2 / t / 1e9,
                "hip_TFLOPs_eff": 4.0 * n * d * 128 / t / 1e12})
    if a.torch:
        ref = K.assign_accumulate_torch(X, C)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ref = K.assign_accumulate_torch(X, C)
        torch.cuda.synchronize()
        tt = time.perf_counter() - t0
        res.update({"torch_ms": tt * 1e3, "speedup_vs_torch": tt / t,
                    "count_diff": float((out[:, -1] - ref[:, -1]).abs().sum().item())})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
