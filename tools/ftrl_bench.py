#!/usr/bin/env python3
"""BASELINE config 5: FTRL streaming logistic regression on a 1e6-dim sparse click-log stream, 1 GPU.

Synthetic Avazu-like stream (no dataset access): each sample = intercept + ``--fields`` categorical fields
hashed into ``--dim`` coordinates (skewed: a few hot values per field), labels drawn from a hidden logistic
model.  Micro-batches of ``--batch`` samples go through the two GPU update paths of ``FtrlTrainStreamOp``:

* SHARDED — partial margins (``ftrl_partial_margin_kernel``) + per-coordinate replay in sample order
  (``ftrl_coord_update_kernel``), deterministic; at P ranks the margins are all-reduced;
* HOGWILD — one wave per sample with atomic n/z (``ftrl_hogwild_kernel``) + prox reconciliation.

Reports samples/s (timed over ``--batches`` micro-batches after warmup), prequential log-loss (each batch
scored before its update), the model-snapshot latency (device -> host + Alink linear-model table rows, 1e6
coefficients) and the GPU feature-hashing rate (Guava murmur3 over "field=value" strings).

    python tools/ftrl_bench.py [--dim 1000000] [--batch 65536] [--batches 40] [--fields 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def make_stream(dim, batch, nb, fields, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    per_field = (dim - 1) // fields
    w_true = torch.randn(dim, generator=g, device=dev, dtype=torch.float64) * 0.7
    out = []
    for _ in range(nb):
        u = torch.rand((batch, fields), generator=g, device=dev, dtype=torch.float64)
        local = (per_field * u ** 3).long().clamp_max(per_field - 1)           # skewed values per field
        idx = 1 + local + torch.arange(fields, device=dev) * per_field
        idx = torch.cat([torch.zeros((batch, 1), dtype=torch.long, device=dev), idx], 1)
        margin = w_true[idx].sum(1) - 0.5
        y = (torch.rand(batch, generator=g, device=dev, dtype=torch.float64) < torch.sigmoid(margin)).double()
        indptr = torch.arange(batch + 1, device=dev, dtype=torch.int64) * (fields + 1)
        out.append((indptr, idx.reshape(-1).to(torch.int32).contiguous(),
                    torch.ones(batch * (fields + 1), dtype=torch.float64, device=dev), y))
    return out


def logloss(margin, y):
    return float(torch.nn.functional.binary_cross_entropy_with_logits(margin, y))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--fields", type=int, default=20)
    ap.add_argument("--hash-strings", type=int, default=1_000_000)
    a = ap.parse_args()
    from alink_amd.ops import _lib
    from alink_amd.ops.ftrl import (ftrl_hogwild, ftrl_partial_margin_hip, ftrl_shard_update_hip, ftrl_dp_gradients,
                                    ftrl_dp_update)
    dev = torch.device("cuda")
    _lib.require()
    prm = (0.1, 1.0, 0.01, 0.01)   # alpha, beta, l1, l2 (FTRLExample: 0.1, 0.1, 0.01, 0.01 with beta 0.1)
    stream = make_stream(a.dim, a.batch, a.warmup + a.batches, a.fields, dev)
    res = {"config": {"dim": a.dim, "batch": a.batch, "batches": a.batches, "nnz_per_sample": a.fields + 1},
           "data": "synthetic hashed click stream (skewed categorical fields, hidden logistic model)"}
    for mode in ("SHARDED", "HOGWILD", "DATA_PARALLEL"):
        w = torch.zeros(a.dim, dtype=torch.float64, device=dev)
        n = torch.zeros_like(w)
        z = torch.zeros_like(w)
        losses = []
        t0 = None
        for b, (indptr, idx, val, y) in enumerate(stream):
            if b == a.warmup:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            if mode == "SHARDED":
                m = ftrl_partial_margin_hip(indptr, idx, val, w, 0, a.dim)
                losses.append(m)
                err = (torch.sigmoid(m) - y).contiguous()
                ftrl_shard_update_hip(indptr, idx, val, err, w, n, z, 0, a.dim, *prm)
            elif mode == "DATA_PARALLEL":
                gq, m = ftrl_dp_gradients(indptr, idx, val, y, w)     # P ranks: gq is all-reduced here
                losses.append(m)
                ftrl_dp_update(gq, w, n, z, *prm)
            else:
                losses.append(ftrl_partial_margin_hip(indptr, idx, val, w, 0, a.dim))
                ftrl_hogwild(indptr, idx, val, y, w, n, z, *prm)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ll = [logloss(m, s[3]) for m, s in zip(losses, stream)]
        res[mode] = {"samples_per_s": a.batch * a.batches / el, "ms_per_batch": el / a.batches * 1e3,
                     "prequential_logloss_first": ll[0], "prequential_logloss_last": ll[-1],
                     "scoring_included": mode != "SHARDED"}
        if mode == "SHARDED":
            w_sharded = w
    # model snapshot latency: device -> host + Alink linear model table rows
    from alink_amd.common.linalg import DenseVector
    from alink_amd.common.types import Types
    from alink_amd.models.linear.model import LinearModelData, LinearModelDataConverter
    torch.cuda.synchronize()
    t = time.perf_counter()
    wh = w_sharded.cpu().numpy()
    md = LinearModelData()
    md.coefVector = DenseVector(wh)
    md.hasInterceptItem = True
    md.modelName = "Logistic Regression"
    md.vectorColName = "vec"
    md.vectorSize = a.dim - 1
    md.labelValues = [1, 0]
    md.linearModelType = "LR"
    rows = LinearModelDataConverter(Types.INT).save(md)
    res["snapshot"] = {"ms": (time.perf_counter() - t) * 1e3, "rows": len(rows), "coefficients": a.dim}
    # GPU feature hashing of "field=value" strings
    from alink_amd.ops.feature import murmur3_index
    rng = np.random.default_rng(1)
    strs = [str(v) for v in rng.integers(0, 10 ** 7, size=a.hash_strings)]
    murmur3_index(strs[:1000], a.dim, prefix="C1=", device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    murmur3_index(strs, a.dim, prefix="C1=", device=dev)
    torch.cuda.synchronize()
    res["hash_strings_per_s"] = a.hash_strings / (time.perf_counter() - t)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
