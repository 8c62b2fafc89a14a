#!/usr/bin/env python3
"""Per-workgroup timeline of the fused KMeans v10 kernel (diagnostic build ``variants/libalink_hip_timing.so``,
``tools/build_kmeans_variants.sh timing``): every workgroup stamps the 100 MHz wall clock at kernel entry, when its
first tile pair is published, at the end of its distance / accumulate loops, after the fold of the four wave-private
sums and at exit.  Prints, per row count and direction (forward / serpentine-reverse), the distribution over
workgroups of each phase and the kernel span (first entry -> last exit), so the per-launch fixed cost (ramp, fold,
straggler tail) can be read off directly.

    ALINK_HIP_LIB=variants/libalink_hip_timing.so python tools/kmeans_wg_timing.py --rows 12500000,100000000
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alink_amd.ops import kmeans as K  # noqa: E402


def _q(v):
    v = np.sort(np.asarray(v, dtype=np.float64))
    return {"min": round(float(v[0]), 2), "p50": round(float(v[len(v) // 2]), 2),
            "p90": round(float(v[int(len(v) * 0.9)]), 2), "max": round(float(v[-1]), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="12500000,100000000")
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    assert "timing" in os.environ.get("ALINK_HIP_LIB", ""), "run with ALINK_HIP_LIB=variants/libalink_hip_timing.so"
    dev = torch.device("cuda")
    rows = [int(r) for r in a.rows.split(",")]
    n, d, k = max(rows), 128, a.k
    X = torch.empty((n, d), dtype=torch.bfloat16, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    centers = torch.randn(k, d, device=dev, generator=g) * 4
    for s in range(0, n, 1 << 24):
        e = min(n, s + (1 << 24))
        lab = torch.randint(0, k, (e - s,), device=dev, generator=g)
        X[s:e] = (centers[lab] + torch.randn(e - s, d, device=dev, generator=g)).to(torch.bfloat16)
    C = (centers + 0.3 * torch.randn(k, d, device=dev, generator=g)).double()
    for r in rows:
        Xs = X[:r]
        for rev in (0, 1):
            mode = (K.V10_FLAGS << 4) | (rev << 5)
            stamps = torch.zeros(max(r, 8 * 1024 * 2), dtype=torch.int32, device=dev)
            for it in range(a.iters + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                K.assign_accumulate_hip(Xs, C, assign_out=stamps, mode=mode)
                torch.cuda.synchronize()
                wall = (time.perf_counter() - t0) * 1e3
            grid = K._GRID[("v10", r, None, X.device.index)]
            st = stamps[:16 * grid].view(torch.int64).view(grid, 8).cpu().numpy().astype(np.float64) * 0.01  # us
            t0 = st[:, 0].min()
            rel = st[:, :6] - t0
            res = {"rows": r, "rev": rev, "grid": grid, "wall_ms_last": round(wall, 4),
                   "span_us": round(float(rel[:, 5].max()), 2),
                   "entry_us": _q(rel[:, 0]),
                   "first_pair_us": _q(st[:, 1] - st[:, 0]),
                   "dist_loop_end_us": _q(rel[:, 2]),
                   "acc_loop_end_us": _q(rel[:, 3]),
                   "fold_us": _q(st[:, 4] - np.maximum(st[:, 2], st[:, 3])),
                   "slab_write_us": _q(st[:, 5] - st[:, 4]),
                   "exit_us": _q(rel[:, 5]),
                   "slowest_wgs": [int(i) for i in np.argsort(-rel[:, 5])[:8]]}
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
