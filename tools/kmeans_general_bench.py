"""Two-pass general HIP KMeans path (nearest + accumulate-by-index) vs the fused v7 kernel and vs torch, per
(d, k): ms per assign+accumulate call and rows/s.  Usage: python tools/kmeans_general_bench.py
``--atomic``: the LDS-table accumulate shapes, fp64 table vs fp32 table, with errors vs an fp64 reference."""
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


def main_atomic():
    """Shapes that take the LDS-table accumulate kernel (weighted rows, d = 512, k > 256 at d = 64): the fp64
    table (default) vs the fp32 table (ALINK_KMEANS_ACC_F32=1, read once per process -> one child per arm)."""
    import subprocess
    for arm in ("f64", "f32"):
        env = dict(os.environ)
        if arm == "f32":
            env["ALINK_KMEANS_ACC_F32"] = "1"
        subprocess.run([sys.executable, os.path.abspath(__file__), "--atomic-child", arm], env=env, check=True)


def atomic_child(arm):
    from alink_amd.ops import kmeans as K
    for d, k, n, weighted in [(64, 100, 50_000_000, True), (128, 100, 50_000_000, True), (256, 256, 25_000_000, True),
                              (512, 100, 12_500_000, False), (64, 400, 50_000_000, False)]:
        g = torch.Generator(device="cuda").manual_seed(d + k)
        X = torch.randn(n, d, device="cuda", generator=g, dtype=torch.float32).to(torch.bfloat16)
        C = torch.randn(k, d, device="cuda", generator=g, dtype=torch.float64)
        w = torch.rand(n, device="cuda", generator=g, dtype=torch.float32) if weighted else None
        if d in (64, 128, 256):
            idx, _ = K.nearest_hip(X, C)
        else:                               # no nearest kernel for this width: a uniform random assignment
            idx = torch.randint(0, k, (n,), device="cuda", generator=g, dtype=torch.int32)
        t_acc = timeit(lambda: K.accumulate_by_index_hip(X, idx, k, w))
        got = K.accumulate_by_index_hip(X, idx, k, w)
        m = 2_000_000                       # fp64 reference on a prefix
        ref = torch.zeros((k, d + 1), dtype=torch.float64, device="cuda")
        xs = X[:m].double() * (w[:m].double()[:, None] if weighted else 1.0)
        ref[:, :d].index_add_(0, idx[:m].long(), xs)
        ref[:, d].index_add_(0, idx[:m].long(), w[:m].double() if weighted else torch.ones(m, dtype=torch.float64,
                                                                                               device="cuda"))
        part = K.accumulate_by_index_hip(X[:m], idx[:m].contiguous(), k, None if w is None else w[:m].contiguous())
        err = float(((part - ref).abs().max() / ref.abs().max()))
        print(json.dumps({"table": arm, "d": d, "k": k, "rows": n, "weighted": weighted, "accum_ms": round(t_acc, 3),
                          "x_GBps": round(n * d * 2 / t_acc / 1e6, 1), "max_rel_err_vs_fp64_2e6": err,
                          "checksum": float(got[:, d].sum())}), flush=True)
        del X, idx
        torch.cuda.empty_cache()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--atomic-child":
        atomic_child(sys.argv[2])
    elif len(sys.argv) > 1 and sys.argv[1] == "--atomic":
        main_atomic()
    else:
        main()
