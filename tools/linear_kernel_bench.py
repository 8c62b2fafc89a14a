"""Fused linear-gradient kernel (csrc/linear.hip) vs the torch two-pass form, and an LR training run.
Usage: python tools/linear_kernel_bench.py [n] [d]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    from alink_amd.models.linear import objfunc as O
    from alink_amd.ops import linear as lops
    n_req = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
    out = {}
    for d in ([int(sys.argv[2])] if len(sys.argv) > 2 else [8, 16, 32, 64, 128, 256, 512, 1024]):
        n = min(n_req, int(2.5e9 // (8 * d)))      # <= 2.5 GB of X per shape
        X = torch.randn(n, d, dtype=torch.float64, device="cuda")
        y = (torch.randint(0, 2, (n,), device="cuda") * 2 - 1).double()
        w = torch.ones(n, dtype=torch.float64, device="cuda")
        c = 0.1 * torch.randn(d, dtype=torch.float64, device="cuda")
        fn = O.LogLossFunc()
        t_hip = timeit(lambda: lops.linear_grad_hip(X, y, w, c, 0))
        t_torch = timeit(lambda: X.T @ (w * fn.derivative(X @ c, y)))
        gb = n * d * 8 / 1e9
        out[f"d{d}"] = {"n": n, "hip_ms": round(t_hip, 3), "torch_ms": round(t_torch, 3),
                        "hip_GBps": round(gb / t_hip * 1e3, 1), "torch_GBps": round(gb / t_torch * 1e3, 1)}
        del X
    print(json.dumps({"n_requested": n_req, "results": out}))


if __name__ == "__main__":
    main()
