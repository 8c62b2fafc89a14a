"""ALS top-K scoring throughput on 1 MI355X: fused HIP score+top-K kernel vs hipBLASLt GEMM + torch.topk.

    python tools/topk_bench.py [--users 16384] [--items 1000000] [--rank 64] [--k 100]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from alink_amd.ops import topk as T  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=16384)
    ap.add_argument("--items", type=int, default=1000000)
    ap.add_argument("--rank", type=int, default=64)
    ap.add_argument("--k", type=int, default=100)
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    Q = torch.rand(a.users, a.rank, device="cuda", generator=g)
    I = torch.rand(a.items, a.rank, device="cuda", generator=g)
    flop = 2.0 * a.users * a.items * a.rank
    res = {"users": a.users, "items": a.items, "rank": a.rank, "k": a.k}
    for name, uk in (("hip_fused", True), ("torch_gemm_topk", False)):
        def run():
            st = T.TopKState(a.users, a.k, "cuda")
            T.merge(st, Q, I, 0, use_kernel=uk)
            return T.finish(st)
        t = timed(run)
        res[name] = {"s": t, "pairs_per_s": a.users * a.items / t, "tflops": flop / t / 1e12}
        print(name, json.dumps(res[name]), flush=True)
    sa, sb = T.TopKState(512, a.k, "cuda"), T.TopKState(512, a.k, "cuda")
    T.merge(sa, Q[:512], I, 0, use_kernel=True)
    T.merge(sb, Q[:512], I, 0, use_kernel=False)
    a_v, b_v = T.finish(sa)[0], T.finish(sb)[0]
    res["max_abs_diff_first512"] = float((a_v - b_v).abs().max())
    res["speedup"] = res["torch_gemm_topk"]["s"] / res["hip_fused"]["s"]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
