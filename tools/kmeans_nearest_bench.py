#!/usr/bin/env python3
"""A/B of the k-means|| nearest-centroid kernel (csrc/kmeans_nearest.hip): rows per wave iteration (RG 1 / 2) and
persistent workgroups per CU, at the headline shape (1e8 x 128 bf16) for candidate counts 1 (the first cost pass),
~201 (initSteps = 2: the weights pass) and 401.  Every variant must give the same (idx, d2) as RG = 1.

    python tools/kmeans_nearest_bench.py [--rows 100000000] [--reps 5]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from alink_amd.ops import kmeans as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    X = (torch.randn(a.rows, 128, device=dev, generator=g) * 3).to(torch.bfloat16)
    floor_ms = X.numel() * 2 / 8e12 * 1e3
    print(json.dumps({"rows": a.rows, "bytes": X.numel() * 2, "hbm_floor_ms_at_8TBs": round(floor_ms, 3)}), flush=True)
    only_m = int(os.environ.get("NEAREST_ONLY_M", "0"))
    if only_m:        # one candidate count, default variant (profiler passes)
        C = X[torch.randint(0, a.rows, (only_m,), device=dev, generator=g)].double()
        for _ in range(a.reps):
            K.nearest_counts_hip(X, C)
        torch.cuda.synchronize()
        print(json.dumps({"m": only_m, "reps": a.reps}), flush=True)
        return
    if os.environ.get("RG_AB"):        # nearest kernel row groups per wave iteration at D = 128
        for m in (201, 256):
            C = X[torch.randint(0, a.rows, (m,), device=dev, generator=g)].double()
            ref = None
            for rg, gm, lag in ((2, 2, "0"), (3, 2, "0"), (2, 2, "1"), (3, 2, "1"), (4, 2, "1"), (2, 1, "1"),
                                (2, 2, "0"), (3, 2, "0"), (2, 2, "1"), (3, 2, "1"), (4, 2, "1"), (2, 1, "1")):
                K.NEAREST_RG, K.NEAREST_GRID = rg, gm
                os.environ["ALINK_KMEANS_NEAREST_LAG"] = lag
                cnt = K.nearest_counts_hip(X, C)
                idx = K.nearest_hip(X[:4_000_000], C)[0]
                torch.cuda.synchronize()
                ts = []
                for _ in range(a.reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    K.nearest_counts_hip(X, C)
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1))
                ts.sort()
                if ref is None:
                    ref = (cnt, idx)
                same = bool(torch.equal(cnt, ref[0]) and torch.equal(idx, ref[1]))
                print(json.dumps({"m": m, "rg": rg, "wg_per_cu": gm, "lag": lag,
                                  "counts_ms_median": round(ts[len(ts) // 2], 3),
                                  "ms_min": round(ts[0], 3), "identical_to_rg2": same}), flush=True)
        K.NEAREST_RG, K.NEAREST_GRID = 2, 2
        os.environ.pop("ALINK_KMEANS_NEAREST_LAG", None)
        return
    if os.environ.get("COUNTS_AB"):    # the k-means|| weights pass: exact vs packed (v_max3) argmax
        for m in (201, 256):
            C = X[torch.randint(0, a.rows, (m,), device=dev, generator=g)].double()
            res = {}
            for flag in ("0", "1", "0", "1"):
                os.environ["ALINK_KMEANS_COUNTS_PACKED"] = flag
                cnt = K.nearest_counts_hip(X, C)
                torch.cuda.synchronize()
                ts = []
                for _ in range(a.reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    K.nearest_counts_hip(X, C)
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1))
                ts.sort()
                res[flag] = cnt
                print(json.dumps({"m": m, "counts_packed": flag, "ms_median": round(ts[len(ts) // 2], 3),
                                  "ms_min": round(ts[0], 3)}), flush=True)
            moved = int((res["0"] - res["1"]).abs().sum()) // 2
            print(json.dumps({"m": m, "rows_moved_by_packing": moved, "rows": a.rows}), flush=True)
        return
    c = X[12345].double()
    for gm, var in ((4, 0), (4, 1), (4, 2), (4, 3), (2, 2), (6, 0), (8, 3)):
        K.COST1_GRID, K.COST1_VARIANT = gm, var
        K.cost1_hip(X, c)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            K.cost1_hip(X, c)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        print(json.dumps({"cost1_wg_per_cu": gm, "variant": var, "ms_median": round(ts[len(ts) // 2], 3), "ms_min": round(ts[0], 3),
                          "TBps": round((X.numel() * 2 + X.shape[0] * 8) / (ts[0] * 1e-3) / 1e12, 2)}), flush=True)
    K.COST1_GRID, K.COST1_VARIANT = 4, 1
    if os.environ.get("COST1_ONLY"):
        return
    for m in (1, 201, 256, 401):
        C = X[torch.randint(0, a.rows, (m,), device=dev, generator=g)].double()
        ref = None
        for rg, gm in ((1, 2), (2, 2), (1, 4), (2, 1)):
            K.NEAREST_RG, K.NEAREST_GRID = rg, gm
            out = K.nearest_hip(X, C)
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                K.nearest_hip(X, C)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            if ref is None:
                ref = out
                same = True
            else:
                same = bool(torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]))
            flops = 2.0 * a.rows * 128 * m
            print(json.dumps({"m": m, "rg": rg, "wg_per_cu": gm, "ms_median": round(ts[len(ts) // 2], 3),
                              "ms_min": round(ts[0], 3), "tflops": round(flops / (ts[0] * 1e-3) / 1e12, 1),
                              "identical_to_rg1": same}), flush=True)
            del out


if __name__ == "__main__":
    main()
