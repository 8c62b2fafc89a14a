"""Clustering evaluation (reference ``A/operator/batch/evaluation/EvalClusterBatchOp.java``,
``A/operator/common/evaluation/{ClusterEvaluationUtil,ClusterMetricsSummary}.java``).

Per-cluster count / vector sum / squared-norm sum are segment sums on the device, merged by one all-reduce;
a second pass gives per-cluster distance sums and the silhouette (the reference's closed form using the
cluster sums, so it stays O(N k) instead of O(N^2)).  External indices (NMI, purity, RI, ARI) come from the
[prediction x label] contingency matrix.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from ...common.params import Params
from ...common.table import MTable
from ...parallel import comm
from ..common.features import extract_features
from .metrics import ClusterMetrics

__all__ = ["cluster_metrics", "contingency_params"]


def _pget(p, name):
    try:
        return p.get(name) if p.contains(name) else None
    except KeyError:
        return None


def contingency_params(mat: np.ndarray) -> dict:
    """NMI / purity / RI / ARI of a [pred][label] count matrix (``extractParamsFromConfusionMatrix``)."""
    m = np.asarray(mat, dtype=np.int64)
    actual, pred = m.sum(0), m.sum(1)
    total = int(m.sum())
    comb = lambda x: x * (x - 1) // 2  # noqa: E731
    ent = lambda f: 0.0 if f == 0 else (f / total) * math.log(f / total)  # noqa: E731
    ea = sum(ent(int(a)) for a in actual) / -math.log(2)
    ep = sum(ent(int(p)) for p in pred) / -math.log(2)
    tpfp = int(sum(comb(int(a)) for a in actual))
    tpfn = int(sum(comb(int(p)) for p in pred))
    mi, purity, tp = 0.0, 0.0, 0
    for i in range(m.shape[0]):
        purity += int(m[i].max()) if m.shape[1] else 0
        for j in range(m.shape[1]):
            v = int(m[i, j])
            if v:
                mi += v / total * math.log(total * v / pred[i] / actual[j])
            tp += comb(v)
    purity /= total
    mi /= math.log(2)
    fp, fn = tpfp - tp, tpfn - tp
    totc = comb(total)
    tn = totc - tp - fn - fp
    expected = tpfp * tpfn / totc
    mx = (tpfp + tpfn) / 2
    return {"NMI": 2.0 * mi / (ea + ep), "purity": purity, "ri": (tp + tn) / (tp + tn + fp + fn),
            "ari": (tp - expected) / (mx - expected)}


def cluster_metrics(mt: MTable, params: Params, env) -> ClusterMetrics:
    pred_col = params.get("predictionCol")
    label_col = _pget(params, "labelCol")
    vec_col = _pget(params, "vectorCol")
    dist = str(_pget(params, "distanceType") or "EUCLIDEAN")
    dist = getattr(dist, "name", dist).upper() if not isinstance(dist, str) else dist.upper()
    dev = env.device
    preds = mt.column_values(pred_col)
    out = Params()
    # global cluster id list (string order)
    ids = set()
    for part in comm.all_gather_object(sorted({str(p) for p in preds if p is not None})):
        ids.update(part)
    cids = sorted(ids)
    k = len(cids)
    index = {c: i for i, c in enumerate(cids)}
    if vec_col:
        rows = [i for i, p in enumerate(preds) if p is not None and mt.column_values(vec_col)[i] is not None] \
            if False else [i for i, p in enumerate(preds) if p is not None]
        sub = mt.take(rows)
        X = extract_features(sub, None, vec_col, dev).to_dense().double()
        cid = torch.tensor([index[str(preds[i])] for i in rows], dtype=torch.long, device=dev)
        if dist != "EUCLIDEAN":
            # reference getClusterStatistics: every non-Euclidean distance (COSINE, CITYBLOCK) sums unit vectors
            X = X / X.norm(dim=1, keepdim=True).clamp_min(1e-300)
        d = X.shape[1]
        d = max(comm.all_gather_object(int(d)))
        if X.shape[1] < d:
            X = torch.nn.functional.pad(X, (0, d - X.shape[1]))
        cnt = torch.zeros(k, dtype=torch.float64, device=dev).index_add_(0, cid, torch.ones_like(cid, dtype=torch.float64))
        s = torch.zeros((k, d), dtype=torch.float64, device=dev).index_add_(0, cid, X)
        n2 = torch.zeros(k, dtype=torch.float64, device=dev).index_add_(0, cid, (X * X).sum(1))
        buf = torch.cat([cnt, s.reshape(-1), n2])
        comm.all_reduce(buf, "sum")
        cnt, s, n2 = buf[:k], buf[k:k + k * d].reshape(k, d), buf[k + k * d:]
        mean = s / cnt.clamp_min(1.0)[:, None]

        def dfun(a, b):
            # ContinuousDistance.calc of the metric (CosineDistance divides by both norms; CITYBLOCK = ManHattan)
            if dist == "COSINE":
                cross = a.norm(dim=-1) * b.norm(dim=-1)
                dot = (a * b).sum(-1)
                return 1.0 - torch.where(cross > 0, dot / torch.where(cross > 0, cross, torch.ones_like(cross)),
                                         torch.zeros_like(dot))
            if dist == "CITYBLOCK":
                return (a - b).abs().sum(-1)
            return torch.sqrt(((a - b) ** 2).sum(-1).clamp_min(0.0))

        own = dfun(X, mean[cid])
        dsum = torch.zeros(k, dtype=torch.float64, device=dev).index_add_(0, cid, own)
        d2sum = torch.zeros(k, dtype=torch.float64, device=dev).index_add_(0, cid, own * own)
        # silhouette (closed form over cluster sums; the reference's non-Euclidean form uses 1 - x.mean)
        if dist != "EUCLIDEAN":
            dis = 1.0 - X @ mean.T                                         # [n, k]
            cur = torch.where(cnt[cid] > 1, dis.gather(1, cid[:, None])[:, 0] * cnt[cid] / (cnt[cid] - 1),
                              torch.zeros_like(own))
        else:
            xn = (X * X).sum(1, keepdim=True)
            dis = cnt[None, :] * xn - 2 * cnt[None, :] * (X @ mean.T) + n2[None, :]
            cur = torch.where(cnt[cid] > 1, dis.gather(1, cid[:, None])[:, 0] / (cnt[cid] - 1).clamp_min(1.0),
                              torch.zeros_like(own))
            dis = dis / cnt[None, :].clamp_min(1.0)
        dis = dis.scatter(1, cid[:, None], float("inf"))
        nb = dis.min(1).values if k > 1 else torch.full_like(own, float("inf"))
        sil = torch.where(cur < nb, 1 - cur / nb, nb / cur - 1)
        sil = torch.nan_to_num(sil, nan=0.0)
        buf2 = torch.cat([dsum, d2sum, sil.sum().reshape(1)])
        comm.all_reduce(buf2, "sum")
        dsum, d2sum, silsum = buf2[:k], buf2[k:2 * k], float(buf2[-1])
        total = float(cnt.sum())
        gmean = s.sum(0) / total
        cntn, meann = cnt.cpu().numpy(), mean
        ssb = float((dfun(mean, gmean[None, :]) ** 2 * cnt).sum())
        ssw = float(d2sum.sum())
        comp = (dsum / cnt.clamp_min(1.0))
        compactness = float(comp.sum()) / k
        sep = 0.0
        dbi = np.zeros(k)
        compn = comp.cpu().numpy()
        for i in range(k):
            for j in range(i + 1, k):
                dd = float(dfun(mean[i], mean[j]))
                sep += dd
                t = (compn[i] + compn[j]) / dd if dd != 0 else float("inf")
                dbi[i] = max(dbi[i], t)
                dbi[j] = max(dbi[j], t)
        out.set("SSB", ssb)
        out.set("SSW", ssw)
        out.set("compactness", compactness)
        out.set("k", k)
        out.set("count", int(total))
        out.set("seperation", 2 * sep / (k * k - k) if k > 1 else 0.0)
        out.set("daviesBouldin", float(dbi.sum() / k))
        out.set("calinskiHarabaz", ssb * (total - k) / ssw / (k - 1) if k > 1 and ssw > 0 else float("nan"))
        out.set("clusterArray", cids)
        out.set("countArray", [float(c) for c in cntn])
        out.set("silhouetteCoefficient", silsum / total)
    else:
        cnt = np.zeros(k)
        for p in preds:
            if p is not None:
                cnt[index[str(p)]] += 1
        t = torch.tensor(cnt, dtype=torch.float64)
        comm.all_reduce(t, "sum")
        out.set("count", int(t.sum()))
        out.set("k", k)
        out.set("clusterArray", cids)
        out.set("countArray", [float(c) for c in t.tolist()])
    if label_col:
        labels = mt.column_values(label_col)
        ls = set()
        for part in comm.all_gather_object(sorted({str(l) for l in labels if l is not None})):
            ls.update(part)
        lab_arr = sorted(ls, reverse=True)
        pred_arr = sorted(ids, reverse=True)
        li = {l: i for i, l in enumerate(lab_arr)}
        pi = {p: i for i, p in enumerate(pred_arr)}
        mat = torch.zeros((len(pred_arr), len(lab_arr)), dtype=torch.float64)
        for p, l in zip(preds, labels):
            if p is not None and l is not None:
                mat[pi[str(p)], li[str(l)]] += 1
        comm.all_reduce(mat, "sum")
        for key, v in contingency_params(mat.numpy().astype(np.int64)).items():
            out.set(key, v)
    return ClusterMetrics(out)
