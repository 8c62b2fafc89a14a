#!/usr/bin/env python3
"""Micro-benchmark of the fused KMeans assign+accumulate HIP kernels (v7 / v10) on one GPU.

One data set, several launch configurations in one process (data generation of 1e8 rows is the slow part):

python tools/kmeans_kernel_bench.py --rows 100000000 --k 100 --iters 10 \
    --configs v7:0,v10:0,v10:1,v10:2 --modes 0,1,2 --sub-rows 12500000

A config is ``kernel:flags`` (v7 flags = DMA variant bits 4-5, v10 flags = 1 non-temporal loads, 2 nine-slot
ring); modes are 0 full, 1 load pipeline only, 2 compute only.  ``--sub-rows`` also times the first R rows
(the per-rank shape of an 8-GPU job).  Prints one JSON line per (rows, config, mode).
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
    ap.add_argument("--sub-rows", type=str, default="", help="comma list of smaller row counts to time as well")
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--torch", action="store_true", help="also time the PyTorch path")
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--configs", type=str, default="v10:0")
    ap.add_argument("--modes", type=str, default="0")
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
    row_list = [n] + [int(r) for r in a.sub_rows.split(",") if r]
    ref_small = None
    ref_out = {}
    for rows in row_list:
        Xs = X[:rows]
        for cfg in a.configs.split(","):
            ver, flags = cfg.split(":")
            pool = None
            if "p" in flags:                   # "v10:1p0.1": work-stealing pool fraction (0 = static split)
                flags, pool = flags.split("p")
                K.V10_POOL = float(pool)
            alt = flags.endswith("a")          # "v10:1a": serpentine, the direction alternates every launch
            flags = flags.rstrip("a")
            pfd = "0"
            if "f" in flags:                   # "v10:1f4": L2 prefetch 4 tiles ahead (ALINK_KMEANS_V10_PFD)
                flags, pfd = flags.split("f")
            os.environ["ALINK_KMEANS_V10_PFD"] = pfd
            os.environ["ALINK_KMEANS_KERNEL"] = ver
            for m in [int(v) for v in a.modes.split(",")]:
                calls = [0]

                def run():
                    calls[0] += 1
                    return K.assign_accumulate_hip(Xs, C, grid=a.grid, mode=m | (int(flags) << 4),
                                                   reverse=alt and calls[0] % 2 == 1)
                out = run()
                torch.cuda.synchronize()
                res = {"rows": rows, "k": k, "kernel": K.kernel_version(k), "flags": int(flags), "mode": m,
                       "serpentine": alt, "pool": K.V10_POOL, "pfd": int(pfd)}
                if m == 0:
                    key = (rows, alt)
                    ref_out.setdefault(key, out.clone())
                    res["identical_to_first_config"] = bool(torch.equal(out.view(torch.int64),
                                                                        ref_out[key].view(torch.int64)))
                if m == 0 and rows == n:
                    if ref_small is None:
                        ref_small = K.assign_accumulate_torch(X[:2_000_000], C)
                    got0 = K.assign_accumulate_hip(X[:2_000_000], C, grid=a.grid, mode=int(flags) << 4)
                    res["small_count_diff_vs_torch"] = float((got0[:, -1] - ref_small[:, -1]).abs().sum().item())
                times = []
                for _ in range(a.iters):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    out = run()
                    torch.cuda.synchronize()
                    times.append(time.perf_counter() - t0)
                t = sorted(times)[len(times) // 2]
                res.update({"ms": round(t * 1e3, 4), "rows_per_s": rows / t, "TBps": rows * d * 2 / t / 1e12,
                            "min_ms": round(min(times) * 1e3, 4)})
                print(json.dumps(res), flush=True)
    os.environ.pop("ALINK_KMEANS_KERNEL", None)
    os.environ.pop("ALINK_KMEANS_V10_PFD", None)
    if a.torch:
        ref = K.assign_accumulate_torch(X, C)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ref = K.assign_accumulate_torch(X, C)
        torch.cuda.synchronize()
        print(json.dumps({"torch_ms": (time.perf_counter() - t0) * 1e3,
                          "count_diff": float((out[:, -1] - ref[:, -1]).abs().sum().item())}))


if __name__ == "__main__":
    main()
