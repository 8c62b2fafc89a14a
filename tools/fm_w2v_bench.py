#!/usr/bin/env python3
"""K18 FM and K20 Word2Vec kernels against the torch paths they replace (1 GPU).

FM (``csrc/fm.hip``): a micro-batch of CSR rows over a 1e6-coordinate model, rank-16 factors.
  * forward  -- ``ops.fm.fm_forward`` (wave per row: y and the X V row in one pass) vs the torch expression of
    ``models/recommendation/fm.fm_predict_raw`` (X w + 1/2 sum((X V)^2 - X^2 V^2), two SpMMs);
  * update   -- ``ops.fm.fm_coord_update`` (AdaGrad on the touched coordinates only, wave per coordinate
    segment, no atomics) vs the torch block of ``train_fm`` (index_add gradients + dense AdaGrad step).
  Both pairs must agree to 1e-9 relative; the time is per micro-batch (median of repeats).

Word2Vec (``csrc/w2v.hip``): skip-gram hierarchical softmax over synthetic Zipf documents.
  HIP Hogwild kernel (window enumeration on the device) vs the batched torch SGD (``word2vec._sgd``) over the
  same (centre, context) pairs; the two are different update schedules (Hogwild vs stale batches), so the line
  reports throughput in pairs/s for each and the final HS loss on a held-out pair sample for both.

    python tools/fm_w2v_bench.py [--rows 65536] [--nnz 20] [--k 16] [--vocab 100000] [--tokens 500000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def _median_ms(fn, reps=7):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    return float(np.median(ts))


def bench_fm(a, dev):
    from alink_amd.models.common.features import FeatureMatrix
    from alink_amd.models.recommendation import fm as fmm
    from alink_amd.ops import fm as fops
    g = torch.Generator(device="cpu").manual_seed(7)
    n, nnz, D, k = a.rows, a.nnz, a.dim, a.k
    # Zipf-ish coordinates (hashed click features): a few hot coordinates, a long tail
    col = (torch.rand(n * nnz, generator=g) ** 3 * D).long().clamp(max=D - 1)
    col = col.view(n, nnz).sort(1).values.reshape(-1)
    crow = torch.arange(0, n * nnz + 1, nnz, dtype=torch.int64)
    val = torch.rand(n * nnz, generator=g, dtype=torch.float64)
    fm = FeatureMatrix(crow=crow.to(dev), col=col.to(dev), val=val.to(dev), ncols=D)
    w = (torch.randn(D, generator=g, dtype=torch.float64) * 0.01).to(dev)
    V = (torch.randn(D, k, generator=g, dtype=torch.float64) * 0.01).to(dev)
    bias = 0.1

    def torch_fwd():
        y = torch.full((n,), bias, dtype=torch.float64, device=dev) + fm.mv(w)
        vx = fm.mm(V)
        v2x2 = fmm._sq(fm).mm(V * V)
        return y + 0.5 * (vx * vx - v2x2).sum(1), vx

    yk, vxk = fops.fm_forward(fm, w, V, bias)
    yt, vxt = torch_fwd()
    fwd_err = float(((yk - yt).abs() / yt.abs().clamp(min=1e-12)).max())
    t_k = _median_ms(lambda: fops.fm_forward(fm, w, V, bias))
    t_t = _median_ms(torch_fwd)
    print(json.dumps({"kernel": "fm_forward", "rows": n, "nnz_per_row": nnz, "coords": D, "k": k,
                      "hip_ms": round(t_k, 4), "torch_ms": round(t_t, 4), "speedup": round(t_t / t_k, 2),
                      "max_rel_diff": fwd_err}), flush=True)

    # ---- AdaGrad update on the touched coordinates ----
    yb = torch.rand(n, generator=g, dtype=torch.float64).round().to(dev)
    gvec = torch.sigmoid(yk) - yb
    sw = torch.ones(n, dtype=torch.float64, device=dev)
    lr, l1, l2, EPS = 0.01, 1e-4, 1e-4, fops.EPS

    def state():
        return (w.clone(), torch.zeros_like(w), V.clone(), torch.zeros_like(V), torch.zeros(D, dtype=torch.float64,
                                                                                            device=dev))

    def hip_upd(st):
        w1, sgw, V1, sgV, use = st
        fops.fm_coord_update(fm, gvec, vxk, sw, w1, sgw, V1, sgV, use, lr, l1, l2)
        return st

    def torch_upd(st):
        w1, sgw, V1, sgV, use = st
        rows, cols, vals = fm.row_ids(), fm.col, fm.val
        use.index_add_(0, cols, sw[rows])
        gr = gvec[rows]
        Vc = V1[cols]
        gv = (gr * vals)[:, None] * (vxk[rows] - vals[:, None] * Vc) + l2 * Vc
        G = torch.zeros_like(V1).index_add_(0, cols, gv)
        sgV.index_add_(0, cols, gv * gv)
        V1 = V1 - lr * G / torch.sqrt(sgV + EPS)
        gl = gr * vals + l1 * w1[cols]
        Gl = torch.zeros_like(w1).index_add_(0, cols, gl)
        sgw.index_add_(0, cols, gl * gl)
        w1 = w1 - lr * Gl / torch.sqrt(sgw + EPS)
        return w1, sgw, V1, sgV, use

    sk = hip_upd(state())
    stt = torch_upd(state())
    upd_err = max(float((sk[0] - stt[0]).abs().max()), float((sk[2] - stt[2]).abs().max()))
    st_k = [state() for _ in range(9)]
    st_t = [state() for _ in range(9)]
    t_k = _median_ms(lambda: hip_upd(st_k.pop()))
    t_t = _median_ms(lambda: torch_upd(st_t.pop()))
    print(json.dumps({"kernel": "fm_coord_update", "rows": n, "nnz_per_row": nnz, "coords": D, "k": k,
                      "touched_coords": int((sk[4] > 0).sum()), "hip_ms": round(t_k, 4), "torch_ms": round(t_t, 4),
                      "speedup": round(t_t / t_k, 2), "max_abs_diff": upd_err}), flush=True)


def bench_w2v(a, dev):
    from alink_amd.models.nlp import word2vec as w2m
    from alink_amd.ops import w2v as wops
    rng = np.random.default_rng(3)
    Vn, d, window = a.vocab, 100, 5
    ranks = np.arange(1, Vn + 1, dtype=np.float64)
    p = 1.0 / ranks
    p /= p.sum()
    toks = rng.choice(Vn, size=a.tokens, p=p).astype(np.int64)
    docs = [toks[i:i + 1000] for i in range(0, a.tokens, 1000)]
    counts = np.bincount(toks, minlength=Vn) + 1
    C, P, lens = w2m.huffman(counts)
    H = wops.HuffmanDevice(C, P, lens, dev)
    Ct, Pt, Lt = (torch.as_tensor(C, device=dev), torch.as_tensor(P, device=dev), torch.as_tensor(lens, device=dev))
    shr = [rng.integers(0, window, size=len(x)) for x in docs]
    # the same pairs for the torch path (shrinks drawn by _pairs with the same generator state)
    cen, ctx = w2m._pairs(docs, window, True, np.random.default_rng(11))
    npairs = int(cen.size)
    cen_t, ctx_t = torch.as_tensor(cen, device=dev), torch.as_tensor(ctx, device=dev)

    def fresh():
        g = torch.Generator().manual_seed(0)
        inp = ((torch.rand((Vn, d), generator=g, dtype=torch.float64) - 0.5) / d).to(dev, torch.float32)
        return inp, torch.zeros((Vn - 1, d), dtype=torch.float32, device=dev)

    inp_k, out_k = fresh()
    wops.sg_hs_train(docs[:4], shr[:4], window, H, inp_k, out_k, 0.025)       # warm-up (module load)
    inp_k, out_k = fresh()
    torch.cuda.synchronize()
    t = time.perf_counter()
    wops.sg_hs_train(docs, shr, window, H, inp_k, out_k, 0.025)
    torch.cuda.synchronize()
    t_k = time.perf_counter() - t
    inp_t, out_t = fresh()
    torch.cuda.synchronize()
    t = time.perf_counter()
    w2m._sgd(inp_t, out_t, Ct, Pt, Lt, cen_t, ctx_t, 0.025, batch=int(min(8192, max(16, 2 * Vn))))
    torch.cuda.synchronize()
    t_t = time.perf_counter() - t

    def hs_loss(inp, out):
        sel = torch.as_tensor(np.random.default_rng(5).integers(0, npairs, 20000), device=dev)
        c, x = cen_t[sel], ctx_t[sel]
        ar = torch.arange(Ct.shape[1], device=dev)
        mask = ar[None, :] < Lt[c][:, None]
        f = (out[Pt[c]] * inp[x][:, None, :]).sum(-1).double()
        code = Ct[c].double()
        ll = torch.nn.functional.logsigmoid(torch.where(code > 0, -f, f))
        return float(-(ll * mask).sum() / mask.sum())
    print(json.dumps({"kernel": "w2v_sg_hs", "vocab": Vn, "dim": d, "tokens": a.tokens, "window": window,
                      "pairs": npairs, "hip_s": round(t_k, 4), "torch_batched_s": round(t_t, 4),
                      "hip_pairs_per_s": npairs / t_k, "torch_pairs_per_s": npairs / t_t,
                      "speedup": round(t_t / t_k, 2), "hs_loss_init": hs_loss(*fresh()),
                      "hs_loss_hip": hs_loss(inp_k, out_k), "hs_loss_torch": hs_loss(inp_t, out_t)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--nnz", type=int, default=20)
    ap.add_argument("--dim", type=int, default=1_000_000)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--vocab", type=int, default=100_000)
    ap.add_argument("--tokens", type=int, default=500_000)
    a = ap.parse_args()
    from alink_amd.ops import _lib
    assert torch.cuda.is_available(), "needs a GPU"
    _lib.require()
    dev = torch.device("cuda:0")
    bench_fm(a, dev)
    bench_w2v(a, dev)


if __name__ == "__main__":
    main()
