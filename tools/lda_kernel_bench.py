#!/usr/bin/env python3
"""LDA kernels (csrc/lda.hip) on one GPU: the collapsed-Gibbs sweep (thread-per-token vs wave-cooperative) and the
online-VB E-step (HIP wave-per-document vs the torch loop on the device).

    python tools/lda_kernel_bench.py --tokens 2000000 --topics 100
Prints one JSON line per measurement."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from alink_amd.ops import lda as L  # noqa: E402


def timed(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=2_000_000)
    ap.add_argument("--topics", type=int, default=100)
    ap.add_argument("--docs", type=int, default=20000)
    ap.add_argument("--vocab", type=int, default=20000)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    T, K, D, V = a.tokens, a.topics, a.docs, a.vocab
    d_tok = torch.sort(torch.randint(0, D, (T,), device=dev, generator=g))[0]
    w_tok = torch.randint(0, V, (T,), device=dev, generator=g)
    z = torch.randint(0, K, (T,), device=dev, generator=g)
    nd = torch.bincount(d_tok * K + z, minlength=D * K).reshape(D, K).int()
    nw = torch.bincount(w_tok * K + z, minlength=V * K).reshape(V, K).int()
    nk = nw.sum(0).double()
    u = torch.rand(T, device=dev, generator=g, dtype=torch.float64)
    res = {"kernel": "gibbs", "tokens": T, "topics": K}
    for v in (0, 1):
        res[f"variant{v}_ms"] = round(timed(lambda: L.gibbs_sweep(d_tok, w_tok, z, nd, nw, nk, 0.5, 0.01, V, u,
                                                                    variant=v)), 3)
    res["speedup"] = round(res["variant0_ms"] / res["variant1_ms"], 2)
    res["tokens_per_s_wave"] = T / (res["variant1_ms"] * 1e-3)
    print(json.dumps(res), flush=True)

    from alink_amd.models.clustering import lda as M
    Dd = 20000
    lens = torch.randint(20, 200, (Dd,), device=dev, generator=g)
    doc = torch.repeat_interleave(torch.arange(Dd, device=dev), lens)
    word = torch.randint(0, V, (doc.numel(),), device=dev, generator=g)
    cts = torch.randint(1, 4, (doc.numel(),), device=dev, generator=g).double()
    lam = torch.rand((K, V), device=dev, generator=g, dtype=torch.float64) + 0.5
    ebT = torch.exp(M._dir_exp(lam)).T.contiguous()
    alpha = torch.full((K,), 1.0 / K, dtype=torch.float64, device=dev)
    g0 = torch.rand((Dd, K), device=dev, generator=g, dtype=torch.float64) + 0.5
    res = {"kernel": "online_vb_estep", "docs": Dd, "tokens": int(doc.numel()), "topics": K}
    res["hip_ms"] = round(timed(lambda: L.estep(doc, word, cts, Dd, ebT, alpha, g0), 3), 3)
    saved = L.kernel_supported
    L.kernel_supported = lambda d: False
    try:
        res["torch_ms"] = round(timed(lambda: M.e_step(doc, word, cts, Dd, ebT, alpha, g0), 3), 3)
    finally:
        L.kernel_supported = saved
    a1 = L.estep(doc, word, cts, Dd, ebT, alpha, g0)[0]
    L.kernel_supported = lambda d: False
    try:
        b1 = M.e_step(doc, word, cts, Dd, ebT, alpha, g0)[0]
    finally:
        L.kernel_supported = saved
    res["max_rel_diff_gamma"] = float(((a1 - b1).abs() / b1.abs().clamp(min=1e-12)).max())
    res["speedup"] = round(res["torch_ms"] / res["hip_ms"], 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
