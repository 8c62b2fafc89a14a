"""Bisecting k-means (reference ``A/operator/batch/clustering/BisectingKMeansTrainBatchOp.java``,
``A/operator/common/clustering/BisectingKMeansModel{Data,DataConverter,Mapper}.java``).

Semantics kept: clusters are nodes of a binary tree (root 1, children ``2i`` / ``2i + 1``); every bisecting
step splits the leaves with ``size > max(1, minDivisibleClusterSize)`` of largest cost (as many as needed to
reach ``k`` leaves), the two children start at ``c -/+ noise`` (``noise_j = 1e-4 |c| U[0,1)``, drawn with
``java.util.Random(0)``), and ``maxIter`` 2-means iterations move them (Euclidean: the half-space of the
middle plane ``x.(r - l) < (r + l)/2.(r - l)``; cosine: nearest child).  Cluster summaries hold ``size``,
``center`` and ``cost`` (``sum |x|^2 - n |c|^2``, or ``n - c.sum/|c|`` for cosine).  Prediction descends the
tree; leaves are numbered in BFS order and the detail vector turns tree distances into probabilities
(``KMeansUtil.getProbArrayFromDistanceArray``).

MI355X design: the samples stay on the device with an int64 tree-node id per row; an inner iteration is one
fused projection (``X @ V`` for all dividing clusters at once), a ``where`` and one one-hot GEMM for the
per-child segment sums, then one all-reduce of ``[#children, d + 2]`` statistics.
"""
from __future__ import annotations

import json
from typing import Dict, List

import numpy as np
import torch

from ...ops.gemm import tn_matmul
from ...common.javafmt import gson_dumps
from ...common.jrandom import JavaRandom
from ...common.linalg import DenseVector
from ...common.mapper import RichModelMapper
from ...common.model.converter import SimpleModelDataConverter
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import Types
from ...parallel import comm
from ..common.features import extract_features, global_vector_size

__all__ = ["train_bisecting_kmeans", "BisectingKMeansModelMapper"]


def _pget(p: Params, name, default=None):
    try:
        if p.contains(name):
            v = p.get(name)
            return default if v is None else v
    except KeyError:
        pass
    return default


class _Summary:
    __gson_fields__ = ("clusterId", "size", "center", "cost")

    def __init__(self, cid, size, center, cost):
        self.clusterId, self.size, self.center, self.cost = int(cid), int(size), center, float(cost)


def _summaries(X, node, ids: List[int], cosine: bool):
    """Global (size, center, cost) per tree node in ``ids``."""
    dev = X.device
    d = X.shape[1]
    m = len(ids)
    pos = torch.full((int(max(ids)) + 2,), -1, dtype=torch.long, device=dev) if ids else None
    stats = torch.zeros((m, d + 2), dtype=torch.float64, device=dev)
    if m:
        pos[torch.as_tensor(ids, device=dev)] = torch.arange(m, device=dev)
        nn = node.clamp(max=pos.numel() - 1)
        p = torch.where(node < pos.numel(), pos[nn], torch.full_like(node, -1))
        ok = p >= 0
        Xs, ps = X[ok], p[ok]
        norm2 = (Xs * Xs).sum(1)
        vec = Xs / torch.sqrt(norm2)[:, None] if cosine else Xs
        # segment sums as one [m, n] x [n, d + 2] GEMM (few segments: atomics would serialise)
        onehot = torch.nn.functional.one_hot(ps, m).to(X.dtype)
        stats += tn_matmul(onehot, torch.cat([vec, torch.ones_like(norm2)[:, None], norm2[:, None]], 1))
    comm.all_reduce(stats, "sum")
    out = {}
    S = stats.cpu().numpy()
    for i, cid in enumerate(ids):
        s, cnt, ss = S[i, :d], S[i, d], S[i, d + 1]
        c = s / cnt if cnt > 0 else np.zeros(d)
        if cosine and cnt > 0:
            c = c / np.sqrt(c @ c)
            cost = max(cnt - (c @ s) / np.sqrt(c @ c), 0.0)
        else:
            cost = max(ss - cnt * (c @ c), 0.0)
        out[cid] = (int(cnt), c, float(cost))
    return out


def train_bisecting_kmeans(mt: MTable, params: Params, env) -> List[tuple]:
    dev = env.device
    vcol = params.get("vectorCol")
    k = int(_pget(params, "k", 4))
    max_iter = int(_pget(params, "maxIter", 10))
    min_div = int(_pget(params, "minDivisibleClusterSize", 1))
    dist = str(getattr(_pget(params, "distanceType", "EUCLIDEAN"), "name", _pget(params, "distanceType",
                                                                                "EUCLIDEAN"))).upper()
    cosine = dist == "COSINE"
    fm = extract_features(mt, None, vcol, dev)
    d = global_vector_size(fm)
    if fm.is_sparse:
        fm.set_ncols(d)
    X = fm.to_dense().to(torch.float64)
    if X.shape[1] < d:
        X = torch.nn.functional.pad(X, (0, d - X.shape[1]))
    node = torch.ones(X.shape[0], dtype=torch.long, device=dev)
    summ: Dict[int, tuple] = _summaries(X, node, [1], cosine)
    rnd = JavaRandom(0)
    while True:
        ids = set(summ)
        leaves = [c for c in sorted(ids) if 2 * c not in ids and 2 * c + 1 not in ids]
        cand = [c for c in leaves if summ[c][0] > 1 and summ[c][0] > min_div]
        cand.sort(key=lambda c: -summ[c][2])          # stable: ties keep ascending id
        split = sorted(cand[:max(0, k - len(leaves))])
        if not split:
            break
        should_stop = len(split) + len(leaves) >= k
        centers = {}
        for c in split:
            ctr = summ[c][1]
            level = 1.0e-4 * np.sqrt(ctr @ ctr)
            noise = np.array([level * rnd.nextDouble() for _ in range(d)])
            centers[2 * c], centers[2 * c + 1] = ctr - noise, ctr + noise
        par = torch.as_tensor(split, device=dev)
        in_div = (node[:, None] == par[None, :])
        row_has = in_div.any(1)
        which = in_div.float().argmax(1)
        child = node.clone()
        for _ in range(max_iter):
            L = torch.as_tensor(np.stack([centers[2 * c] for c in split]), device=dev)
            R = torch.as_tensor(np.stack([centers[2 * c + 1] for c in split]), device=dev)
            if cosine:
                Xn = X / torch.sqrt((X * X).sum(1, keepdim=True))
                dl = 1.0 - (Xn @ (L / L.norm(dim=1, keepdim=True)).T)
                dr = 1.0 - (Xn @ (R / R.norm(dim=1, keepdim=True)).T)
                go_left = (dl < dr).gather(1, which[:, None])[:, 0]
            else:
                V = R - L
                mid = 0.5 * (R + L)
                length = (mid * V).sum(1)
                proj = X @ V.T
                go_left = (proj < length[None, :]).gather(1, which[:, None])[:, 0]
            child = torch.where(row_has, torch.where(go_left, 2 * node, 2 * node + 1), node)
            kids = [x for c in split for x in (2 * c, 2 * c + 1)]
            s = _summaries(X, child, kids, cosine)
            for cid in kids:
                if s[cid][0] > 0:
                    centers[cid] = s[cid][1]
        node = child
        kids = [x for c in split for x in (2 * c, 2 * c + 1)]
        summ.update(_summaries(X, node, kids, cosine))
        if should_stop:
            break
    meta = Params().set("distanceType", dist).set("k", k).set("vectorSize", d).set("vectorCol", vcol)
    data = [gson_dumps(_Summary(cid, summ[cid][0], DenseVector(summ[cid][1]), summ[cid][2]), java_map_order=False)
            for cid in sorted(summ)]
    return SimpleModelDataConverter.rows_from(meta, data)


class BisectingKMeansModelMapper(RichModelMapper):
    def predResultType(self):
        return Types.LONG

    def loadModel(self, rows):
        meta, data = SimpleModelDataConverter.split_rows(rows)
        self.d = int(meta.get("vectorSize"))
        self.cosine = str(getattr(meta.get("distanceType"), "name", meta.get("distanceType"))).upper() == "COSINE"
        self.vcol = meta.get("vectorCol")
        self.centers = {int(s["clusterId"]): np.asarray(s["center"]["data"]) for s in map(json.loads, data)}
        order, queue = [], [1]
        while queue:                       # BFS leaf numbering
            c = queue.pop(0)
            kids = [x for x in (2 * c, 2 * c + 1) if x in self.centers]
            if not kids:
                order.append(c)
            queue.extend(kids)
        self.leaf_ids = order
        self.leaf_index = {c: i for i, c in enumerate(order)}

    @staticmethod
    def _level(n):
        lv = 0
        while n > 1:
            n //= 2
            lv += 1
        return lv

    def _tree_dist(self, a, b):
        la, lb, dd = self._level(a), self._level(b), 0
        while la > lb:
            a //= 2
            la -= 1
            dd += 1
        while lb > la:
            b //= 2
            lb -= 1
            dd += 1
        while a != b:
            a //= 2
            b //= 2
            dd += 2
        return float(dd)

    def _leaf_of(self, x):
        c = 1
        while 2 * c in self.centers and 2 * c + 1 in self.centers:
            l, r = self.centers[2 * c], self.centers[2 * c + 1]
            if self.cosine:
                xn = x / np.sqrt(x @ x)
                left = (1 - xn @ (l / np.sqrt(l @ l))) < (1 - xn @ (r / np.sqrt(r @ r)))
            else:
                v, m = r - l, 0.5 * (r + l)
                left = x @ v < m @ v
            c = 2 * c if left else 2 * c + 1
        return c

    def _leaves_of(self, X: np.ndarray) -> np.ndarray:
        """``_leaf_of`` for every row at once: rows descend level by level, each internal node's rows split by
        one matrix-vector product (the row path's per-row dot to rounding)."""
        c = np.ones(X.shape[0], dtype=np.int64)
        while True:
            moved = False
            for node in np.unique(c).tolist():
                if not (2 * node in self.centers and 2 * node + 1 in self.centers):
                    continue
                rows = np.flatnonzero(c == node)
                x = X[rows]
                l, r = self.centers[2 * node], self.centers[2 * node + 1]
                if self.cosine:
                    xn = x / np.sqrt(np.einsum("ij,ij->i", x, x))[:, None]
                    left = (1 - xn @ (l / np.sqrt(l @ l))) < (1 - xn @ (r / np.sqrt(r @ r)))
                else:
                    v, m = r - l, 0.5 * (r + l)
                    left = x @ v < m @ v
                c[rows] = np.where(left, 2 * node, 2 * node + 1)
                moved = True
            if not moved:
                return c

    def _leaves_of_device(self, X: torch.Tensor) -> torch.Tensor:
        """``_leaves_of`` on the device (float64; the split products to rounding)."""
        c = torch.ones(X.shape[0], dtype=torch.int64, device=X.device)
        t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=X.device)  # noqa: E731
        while True:
            moved = False
            for node in torch.unique(c).tolist():
                if not (2 * node in self.centers and 2 * node + 1 in self.centers):
                    continue
                rows = torch.nonzero(c == node).reshape(-1)
                x = X[rows]
                l, r = self.centers[2 * node], self.centers[2 * node + 1]
                if self.cosine:
                    xn = x / torch.sqrt((x * x).sum(1, keepdim=True))
                    left = (1 - xn @ t(l / np.sqrt(l @ l))) < (1 - xn @ t(r / np.sqrt(r @ r)))
                else:
                    v, m = r - l, 0.5 * (r + l)
                    left = x @ t(v) < float(m @ v)
                c[rows] = torch.where(left, 2 * node, 2 * node + 1)
                moved = True
            if not moved:
                return c

    def _map_row_values(self, row):
        mt = MTable.from_rows([tuple(row)], self.dataSchema)
        return [c.to_list()[0] for c in self._map_columns(mt)]

    def _map_columns(self, mt):
        from ...common.linalg import VectorUtil
        vcol = self.params.get("vectorCol") if self.params.contains("vectorCol") and \
            self.params.get("vectorCol") else self.vcol
        from ..linear.model import _dev
        dev = _dev(mt) if not self.detail_col else torch.device("cpu")
        fm = extract_features(mt, None, vcol, dev)
        if fm.is_sparse:
            fm.set_ncols(self.d)
        X = fm.to_dense().double()
        if dev.type == "cuda":
            if X.shape[1] != self.d:
                raise RuntimeError(f"Dim of predict data not equal to vectorSize of training data: {self.d}")
            leaves = self._leaves_of_device(X)
            ids = torch.unique(leaves)
            idx = torch.tensor([self.leaf_index[int(i)] for i in ids.tolist()], dtype=torch.int64, device=dev)
            return [Column(idx[torch.searchsorted(ids, leaves)].cpu())]
        X = X.numpy()
        if X.shape[1] != self.d:
            raise RuntimeError(f"Dim of predict data not equal to vectorSize of training data: {self.d}")
        if not self.detail_col:
            leaves = self._leaves_of(X)
            ids = np.unique(leaves)
            idx = np.array([self.leaf_index[int(i)] for i in ids], dtype=np.int64)
            return [Column(torch.from_numpy(idx[np.searchsorted(ids, leaves)]))]
        preds, details = [], []
        nl = len(self.leaf_ids)
        for x in X:
            leaf = self._leaf_of(x)
            preds.append(self.leaf_index[leaf])
            if self.detail_col:
                dists = np.array([self._tree_dist(leaf, o) for o in self.leaf_ids])
                if nl > 1:
                    prob = np.full(nl, 1.0 / (nl - 1)) - dists / dists.sum() / (nl - 1)
                else:
                    prob = np.ones(1)
                details.append(VectorUtil.toString(DenseVector(prob)))
        cols = [Column.from_values(preds, Types.LONG)]
        if self.detail_col:
            cols.append(Column.from_values(details, Types.STRING))
        return cols
