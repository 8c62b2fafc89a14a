#!/usr/bin/env python3
"""K8/K10 split search: the HIP tree_split_kernel vs the vectorised torch search on the same device histograms.

    python tools/split_bench.py --nodes 64 --features 1000 --bins 129
Prints one JSON line per criterion (ms per search for each path and the speedup)."""
import argparse
import json
import os
import sys
import time
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alink_amd.models.tree.engine import SplitConfig, TreeBuilder  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--features", type=int, default=1000)
    ap.add_argument("--bins", type=int, default=129)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    m, F, B = a.nodes, a.features, a.bins
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for kind, ncls in (("gbdt", 0), ("gini", 2), ("infogain", 2), ("mse", 0)):
        S = 4 if kind in ("gbdt", "mse") else ncls + 1
        cnt = torch.randint(0, 50, (m, F, B), device=dev, generator=g).double()
        if kind == "gbdt":
            gg = torch.randn(m, F, B, device=dev, generator=g, dtype=torch.float64) * cnt
            H = torch.stack([gg * gg, gg, 0.25 * cnt, cnt], -1)
        elif kind == "mse":
            y = torch.randn(m, F, B, device=dev, generator=g, dtype=torch.float64) * cnt
            H = torch.stack([cnt, y, y * y + cnt, cnt], -1)
        else:
            c0 = torch.floor(cnt * torch.rand(m, F, B, device=dev, generator=g, dtype=torch.float64))
            H = torch.stack([c0, cnt - c0, cnt], -1)
        H = H.float().double()
        is_cat = [f % 10 < 3 for f in range(F)]               # 30 % categorical features
        cfg = SplitConfig(kind=kind, max_depth=8, min_samples_per_leaf=5, n_classes=ncls)
        tb = TreeBuilder.__new__(TreeBuilder)          # only the search state: cfg, data flags, is_cat
        tb.cfg, tb.d, tb.is_cat = cfg, SimpleNamespace(is_cat=is_cat), torch.tensor(is_cat, device=dev)
        order = torch.arange(F, device=dev).expand(m, F).clone()
        ok = torch.ones((m, F), dtype=torch.bool, device=dev)
        res = {"criterion": kind, "nodes": m, "features": F, "bins": B, "S": S}
        outs = {}
        for name in ("hip", "torch"):
            r = (TreeBuilder._search(tb, H, order, ok) if name == "hip" else _torch_search(tb, H, order, ok))
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.iters):
                t0 = time.perf_counter()
                r = (TreeBuilder._search(tb, H, order, ok) if name == "hip" else _torch_search(tb, H, order, ok))
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            outs[name] = r
            res[name + "_ms"] = round(sorted(ts)[len(ts) // 2] * 1e3, 3)
        res["same_features"] = bool(torch.equal(outs["hip"][1], outs["torch"][1]))
        res["speedup"] = round(res["torch_ms"] / res["hip_ms"], 2)
        print(json.dumps(res), flush=True)


def _torch_search(tb, H, order, ok):
    """TreeBuilder._search with the GPU kernels hidden (the vectorised torch search on the device)."""
    from alink_amd.ops import tree as tops
    saved = tops.gpu_kernels_ok
    tops.gpu_kernels_ok = lambda: False
    try:
        return TreeBuilder._search(tb, H, order, ok)
    finally:
        tops.gpu_kernels_ok = saved


if __name__ == "__main__":
    main()
