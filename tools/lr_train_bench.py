"""Whole LogisticRegressionTrainBatchOp (L-BFGS, fp64, dense features) on the GPU: per-iteration time with the
K12 gradient + K14 line-search kernels, vs the same run with ALINK_DISABLE_K14=1 (torch GEMM line search).
Usage: python tools/lr_train_bench.py [rows] [dims]
       python tools/lr_train_bench.py --graphs [rows] [dims]   (two-loop as a HIP graph vs eager)"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(n, d, iters):
    from alink_amd import useLocalEnv
    from alink_amd.models.linear.objfunc import LabeledData, UnaryLossObjFunc, LogLossFunc
    from alink_amd.models.common.features import FeatureMatrix
    from alink_amd.models.linear.optim import optimize
    env = useLocalEnv(1, device="cuda:0")
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn(n, d, device="cuda", generator=g, dtype=torch.float64)
    wt = torch.randn(d, device="cuda", generator=g, dtype=torch.float64)
    y = torch.where(X @ wt + 0.5 * torch.randn(n, device="cuda", generator=g, dtype=torch.float64) > 0, 1.0, -1.0)
    data = LabeledData(FeatureMatrix(dense=X), y, torch.ones(n, device="cuda", dtype=torch.float64))
    obj = UnaryLossObjFunc(LogLossFunc(), 0.0, 0.0)
    from alink_amd.common.params import Params
    p = Params().set("maxIter", iters).set("epsilon", 1e-30)
    torch.cuda.synchronize()
    t = time.perf_counter()
    coef, curve = optimize(obj, data, d, p, env=env)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3, float(curve[-1]) if len(curve) else None


def main_graphs(n, d):
    """Per-iteration time with the two-loop replayed as a HIP graph (default) vs eager (ALINK_HIP_GRAPHS=0)."""
    from alink_amd.models.linear import optim
    out = {"rows": n, "dims": d}
    for flag in ("0", "1", "0", "1"):
        os.environ["ALINK_HIP_GRAPHS"] = flag
        ms, loss = run(n, d, 100)
        out.setdefault("ms_per_iter_graphs" if flag == "1" else "ms_per_iter_eager", []).append(round(ms, 3))
        out["final_loss_graphs" if flag == "1" else "final_loss_eager"] = loss
    out["graph_captures"], out["graph_replays"] = optim.GRAPH_STATS["captures"], optim.GRAPH_STATS["replays"]
    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--graphs":
        for n in ([int(sys.argv[2])] if len(sys.argv) > 2 else [100_000, 4_000_000]):
            main_graphs(n, int(sys.argv[3]) if len(sys.argv) > 3 else 28)
        return
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
    for d in ([int(sys.argv[2])] if len(sys.argv) > 2 else [28, 128, 512]):
        os.environ["ALINK_DISABLE_K14"] = "1"
        ms0, loss0 = run(n, d, 20)
        os.environ["ALINK_DISABLE_K14"] = "0"
        ms, loss = run(n, d, 20)
        print(json.dumps({"rows": n, "dims": d, "ms_per_lbfgs_iter": round(ms, 2),
                          "ms_per_lbfgs_iter_torch_search": round(ms0, 2), "final_loss": loss,
                          "final_loss_torch_search": loss0, "x_GB": n * d * 8 / 1e9}), flush=True)


if __name__ == "__main__":
    main()
