#!/usr/bin/env python3
"""KMeans superstep kernels on fp32 input (1e7 x 128, k = 100, 1 GPU): the fp32 GEMM-assign + HIP accumulate path
vs the fp64 PyTorch path, and the centroid delta of one Lloyd update from each input precision (fp32 path, bf16
fused kernel) against fp64.  python tools/kmeans_fp32_bench.py [--rows 10000000]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from alink_amd.ops import kmeans as K  # noqa: E402


def timed(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return out, sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--k", type=int, default=100)
    a = ap.parse_args()
    n, d, k = a.rows, 128, a.k
    g = torch.Generator(device="cuda").manual_seed(0)
    centers = torch.randn(k, d, device="cuda", generator=g) * 6
    X = torch.empty((n, d), dtype=torch.float32, device="cuda")
    for s in range(0, n, 1 << 22):
        e = min(n, s + (1 << 22))
        lab = torch.randint(0, k, (e - s,), device="cuda", generator=g)
        X[s:e] = centers[lab] + torch.randn(e - s, d, device="cuda", generator=g)
    C = (centers + 0.3 * torch.randn(k, d, device="cuda", generator=g)).double()
    f32, t32 = timed(lambda: K.assign_accumulate_f32_hip(X, C))
    idx_only, t_assign = timed(lambda: K.assign_f32(X, C))
    X64 = X.double()
    ref, t64 = timed(lambda: K.assign_accumulate_torch(X64, C), iters=2)
    Xb = X.to(torch.bfloat16)
    bf, tb = timed(lambda: K.assign_accumulate_hip(Xb, C))

    def cent(buf):
        return buf[:, :d] / buf[:, d:].clamp_min(1)
    c_ref = cent(ref)
    res = {"rows": n, "d": d, "k": k,
           "fp32_path_ms": t32 * 1e3, "fp32_path_rows_per_s": n / t32, "fp32_assign_gemm_ms": t_assign * 1e3,
           "fp32_accumulate_ms": (t32 - t_assign) * 1e3, "fp32_bytes_GBps": n * d * 4 / t32 / 1e9,
           "fp64_torch_ms": t64 * 1e3, "bf16_fused_ms": tb * 1e3,
           "count_diff_fp32_vs_fp64": float((f32[:, d] - ref[:, d]).abs().sum()),
           "count_diff_bf16_vs_fp64": float((bf[:, d] - ref[:, d]).abs().sum()),
           "centroid_max_abs_delta_fp32": float((cent(f32) - c_ref).abs().max()),
           "centroid_max_abs_delta_bf16": float((cent(bf) - c_ref).abs().max()),
           "centroid_scale": float(c_ref.abs().max())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
