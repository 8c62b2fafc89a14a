#!/usr/bin/env python3
"""The k-means|| local step on its real shape (SURVEY §2.10 KMeans init: ~2k+1 weighted candidates of the 1e8-row
bench data, k = 100, d = 128): device time of the seeding kernel, the one-workgroup Lloyd kernel (per iteration
and to convergence) and the whole ``_local_kmeans`` with the kernels on / off (the torch device path).

    python tools/kmeans_local_bench.py [--n 201] [--k 100] [--d 128] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=201)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from alink_amd.models.clustering import kmeans as km
    from alink_amd.ops import kmeans as K
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    centers = torch.randn(a.k, a.d, generator=g, dtype=torch.float64) * 4
    lab = torch.randint(0, a.k, (a.n,), generator=g)
    X = (centers[lab] + torch.randn(a.n, a.d, generator=g, dtype=torch.float64)).to(torch.bfloat16).double().to(dev)
    w = torch.randint(1, 2_000_000, (a.n,), generator=g).to(torch.float64).to(dev)

    def timed(fn):
        out, ts = None, []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        return out, round(sorted(ts)[len(ts) // 2], 4)

    def ev(fn):
        ts = []
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e))
        return round(sorted(ts)[len(ts) // 2], 4)

    res = {"n": a.n, "k": a.k, "d": a.d}
    D = km.pairwise_distance(X, X, "EUCLIDEAN")
    res["pairwise_D_ms"] = ev(lambda: km.pairwise_distance(X, X, "EUCLIDEAN"))
    rng = np.random.default_rng(0)
    r0 = float(rng.random())
    U = torch.as_tensor(rng.random(a.k - 1), dtype=torch.float64, device=dev)
    chosen, mt = K.seed_ref_hip(D, w, U, a.k, idx0=-1, r0=r0)
    res["seed_kernel_ms"] = ev(lambda: K.seed_ref_hip(D, w, U, a.k, idx0=-1, r0=r0))
    sp = torch.zeros(20, dtype=torch.int64, device=dev)
    K.seed_ref_hip(D, w, U, a.k, idx0=-1, r0=r0, prof=sp)
    sp = sp.cpu().tolist()
    res["seed_phase_us"] = {"warmup+first": round((sp[1] - sp[0]) / 100, 2),
                            "pick": [round((sp[2 * j] - sp[2 * j - 1]) / 100, 2) for j in range(2, 9)],
                            "update": [round((sp[2 * j + 1] - sp[2 * j]) / 100, 2) for j in range(1, 9)]}
    C0 = X.index_select(0, chosen).contiguous()
    for it in (1, 2, 4):
        res[f"lloyd_kernel_{it}iter_ms"] = ev(lambda: K.local_lloyd_hip(X, w, a.k, C=C0.clone(), max_iter=it))
    prof = torch.zeros(50, dtype=torch.int64, device=dev)
    _, _, st, _ = K.local_lloyd_hip(X, w, a.k, C=C0.clone(), max_iter=30, prof=prof)
    res["lloyd_iters_to_stop"] = st.cpu().tolist()[:3]
    p = prof.cpu().tolist()
    it = int(res["lloyd_iters_to_stop"][0])
    res["lloyd_phase_us"] = {"setup": round((p[1] - p[0]) / 100, 2)}
    names = ["norms", "distance+assign", "member_counts", "offsets", "members+weights", "sums"]
    prev = p[1]
    for i in range(min(it, 8)):
        for j, nm in enumerate(names):
            v = p[2 + i * 6 + j]
            res["lloyd_phase_us"].setdefault(nm, []).append(round((v - prev) / 100, 2))
            prev = v
    res["lloyd_kernel_30iter_ms"] = ev(lambda: K.local_lloyd_hip(X, w, a.k, C=C0.clone(), max_iter=30))
    for flag in ("0", "1"):
        os.environ["ALINK_KMEANS_LOCAL_KERNEL"] = flag
        C, res[f"local_kmeans_wall_ms_kernel{flag}"] = timed(lambda: km._local_kmeans(X, w, a.k, "EUCLIDEAN", seed=0))
        res[f"_C{flag}"] = C
    c0, c1 = res.pop("_C0"), res.pop("_C1")
    res["max_abs_diff_kernel_vs_torch"] = float((c0 - c1).abs().max())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
