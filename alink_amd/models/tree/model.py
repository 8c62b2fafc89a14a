"""Tree model objects, the tree model-table format and the tree predictors.

Reference: ``A/operator/common/tree/{Node,LabelCounter,TreeModelDataConverter}.java`` and
``predictors/{TreeModelMapper,GbdtModelMapper,RandomForestModelMapper}.java``.

Model table (``TreeModelDataConverter.serializeModel``): data strings are first the categorical
MultiStringIndexer model rows as JSON arrays, then every tree as BFS-ordered ``NodeSerializable`` JSON
(``{"node":{...},"id":i,"nextIds":[...]}``, Gson without nulls); the meta records
``stringIndexerModelPartition`` ``{f0,f1}`` and ``treePartition`` ``{"partitions":[{f0,f1},...]}``; labels go
to the ``label_value`` aux rows.

Prediction is vectorised: every tree is flattened into arrays (split feature, threshold, categorical child
map, children) and all rows descend level by level with tensor gathers; rows that meet a missing value on
their path take the reference's weighted descent over children (``TreeModelMapper.ProcessMissing``).
"""
from __future__ import annotations

import json
import math
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from ...common.javafmt import gson_dumps, java_str
from ...common.mapper import RichModelMapper
from ...common.model.converter import LabeledModelDataConverter
from ...common.params import Params
from ...common.types import Types

__all__ = ["LabelCounter", "Node", "TreeModelDataConverter", "TreeModel", "TreeModelMapper", "GbdtModelMapper",
           "RandomForestModelMapper", "serialize_tree", "deserialize_tree", "feature_importance"]


class LabelCounter:
    __gson_fields__ = ("weightSum", "numInst", "distributions")
    __gson_skip_nulls__ = True

    def __init__(self, weightSum=0.0, numInst=0, distributions=None):
        self.weightSum = float(weightSum)
        self.numInst = int(numInst)
        self.distributions = None if distributions is None else [float(x) for x in distributions]

    def norm_with_weight(self) -> "LabelCounter":
        if self.weightSum != 0.0 and self.distributions is not None:
            self.distributions = [x / self.weightSum for x in self.distributions]
        return self


class Node:
    __gson_fields__ = ("featureIndex", "gain", "counter", "categoricalSplit", "continuousSplit")
    __gson_skip_nulls__ = True

    def __init__(self, featureIndex=-1, gain=0.0, counter=None, categoricalSplit=None, continuousSplit=0.0):
        self.featureIndex = int(featureIndex)
        self.gain = float(gain)
        self.counter = counter
        self.categoricalSplit = categoricalSplit
        self.continuousSplit = float(continuousSplit)
        self.nextNodes: List["Node"] = []

    def isLeaf(self):
        return self.featureIndex == -1

    def make_leaf_prob(self):
        if self.counter is not None:
            self.counter.norm_with_weight()
        return self


class _NodeSerializable:
    __gson_fields__ = ("node", "id", "nextIds")
    __gson_skip_nulls__ = True

    def __init__(self, node, id_, next_ids=None):
        self.node = node
        self.id = id_
        self.nextIds = next_ids


class _Partition:
    __gson_fields__ = ("f0", "f1")

    def __init__(self, f0, f1):
        self.f0, self.f1 = int(f0), int(f1)


class _Partitions:
    __gson_fields__ = ("partitions",)

    def __init__(self, parts):
        self.partitions = parts


def serialize_tree(root: Node) -> List[str]:
    """BFS numbering exactly as ``TreeModelDataConverter.serializeTree`` (FIFO queue, ids on enqueue)."""
    out = []
    nid = 0
    queue = [_NodeSerializable(root, nid)]
    nid += 1
    head = 0
    while head < len(queue):
        ns = queue[head]
        head += 1
        if not ns.node.isLeaf():
            ids = []
            for ch in ns.node.nextNodes:
                ids.append(nid)
                queue.append(_NodeSerializable(ch, nid))
                nid += 1
            ns.nextIds = ids
        out.append(gson_dumps(ns, java_map_order=False))
    return out


def _node_from_json(d: dict) -> Node:
    c = d.get("counter")
    counter = None if c is None else LabelCounter(c.get("weightSum", 0.0), c.get("numInst", 0),
                                                  c.get("distributions"))
    return Node(d.get("featureIndex", -1), d.get("gain", 0.0), counter, d.get("categoricalSplit"),
                d.get("continuousSplit", 0.0))


def deserialize_tree(strings: Sequence[str]) -> Optional[Node]:
    objs = [json.loads(s) for s in strings]
    size = len(objs)
    nodes: List[Optional[Node]] = [None] * size
    nexts: List[Optional[list]] = [None] * size
    for o in objs:
        i = int(o["id"])
        if i < 0 or i >= size:
            raise RuntimeError(f"Model is broken. node index: {i}")
        nodes[i] = _node_from_json(o.get("node") or {})
        nexts[i] = o.get("nextIds")
    for i in range(size):
        if nexts[i]:
            nodes[i].nextNodes = [nodes[j] for j in nexts[i]]
    return nodes[0] if size else None


class TreeModel:
    def __init__(self, meta: Params, roots: List[Node], labels: Optional[List[Any]],
                 indexer_rows: Optional[List[Any]]):
        self.meta = meta
        self.roots = roots
        self.labels = labels
        self.indexer_rows = indexer_rows


class TreeModelDataConverter(LabeledModelDataConverter):
    def serializeModel(self, model: TreeModel):
        data: List[str] = []
        if model.indexer_rows:
            for r in model.indexer_rows:
                data.append(gson_dumps([r[0], r[1], r[2]], java_map_order=False))
        meta = model.meta
        meta.set("stringIndexerModelPartition", _Partition(0, len(data)))
        parts = []
        for root in model.roots:
            s = serialize_tree(root)
            parts.append(_Partition(len(data), len(data) + len(s)))
            data.extend(s)
        meta.set("treePartition", _Partitions(parts))
        return meta, data, model.labels

    def deserializeModel(self, meta, data, labels):
        sp = meta.get("stringIndexerModelPartition")
        f0, f1 = int(sp["f0"]), int(sp["f1"])
        indexer_rows = None
        if f1 != f0:
            indexer_rows = []
            for i in range(f0, f1):
                o = json.loads(data[i])
                indexer_rows.append((int(o[0]), o[1], o[2]))
        roots = [deserialize_tree(data[p["f0"]:p["f1"]]) for p in meta.get("treePartition")["partitions"]]
        return TreeModel(meta, roots, list(labels) if labels else [], indexer_rows)


def feature_importance(roots: Sequence[Node], feature_cols: Sequence[str]) -> List[tuple]:
    """Split counts per feature (``TreeModelDataConverter.FeatureImportanceReducer``), Java HashMap order."""
    counts: Dict[int, int] = {}
    for root in roots:
        stack = [root]
        while stack:
            nd = stack.pop()
            if nd.featureIndex >= 0:
                counts[nd.featureIndex] = counts.get(nd.featureIndex, 0) + 1
            stack.extend(nd.nextNodes)
    # HashMap<Integer,...> iterates small non-negative keys in ascending order
    return [(feature_cols[k], int(v)) for k, v in sorted(counts.items())]


# ---------------------------------------------------------------------------------------------------
# vectorised predictor
# ---------------------------------------------------------------------------------------------------
class _FlatForest:
    """All trees as flat arrays: feature (-1 leaf), threshold, categorical map row, first child, #children."""

    def __init__(self, roots: Sequence[Node], n_dist: int):
        feats, thr, catrow, first, nchild, dist, wsum = [], [], [], [], [], [], []
        cat_maps: List[List[int]] = []
        self.roots = []
        for root in roots:
            if root is None:
                continue
            base = len(feats)
            order = [root]
            head = 0
            while head < len(order):
                nd = order[head]
                head += 1
                order.extend(nd.nextNodes if not nd.isLeaf() else [])
            index = {id(nd): base + i for i, nd in enumerate(order)}
            self.roots.append(base)
            for nd in order:
                feats.append(nd.featureIndex)
                thr.append(nd.continuousSplit)
                if not nd.isLeaf() and nd.categoricalSplit is not None:
                    catrow.append(len(cat_maps))
                    cat_maps.append([int(x) for x in nd.categoricalSplit])
                else:
                    catrow.append(-1)
                if nd.isLeaf():
                    first.append(-1)
                    nchild.append(0)
                else:
                    first.append(index[id(nd.nextNodes[0])])
                    nchild.append(len(nd.nextNodes))
                    # children are contiguous in BFS order
                c = nd.counter
                d = (c.distributions if c is not None and c.distributions is not None else [])
                dist.append((list(d) + [0.0] * n_dist)[:n_dist])
                wsum.append(c.weightSum if c is not None else 0.0)
        self.feat = np.asarray(feats, dtype=np.int64)
        self.thr = np.asarray(thr, dtype=np.float64)
        self.catrow = np.asarray(catrow, dtype=np.int64)
        self.first = np.asarray(first, dtype=np.int64)
        self.nchild = np.asarray(nchild, dtype=np.int64)
        self.dist = np.asarray(dist, dtype=np.float64).reshape(len(feats), n_dist)
        self.wsum = np.asarray(wsum, dtype=np.float64)
        width = max([len(m) for m in cat_maps] + [1])
        self.cat = np.full((max(1, len(cat_maps)), width), -1, dtype=np.int64)
        for i, m in enumerate(cat_maps):
            self.cat[i, :len(m)] = m
        self.max_steps = len(feats) + 1


class TreeModelMapper(RichModelMapper):
    """Shared tree prediction (``TreeModelMapper.java``): categorical columns through the embedded string
    indexer (unseen -> missing), continuous columns as doubles, weighted descent on missing values."""

    model = None

    def loadModel(self, rows):
        from ...common.mapper import OutputColsHelper
        from ..linear.model import _recover_label
        ltype = self._label_type_from_rows(rows)
        conv = TreeModelDataConverter(ltype)
        self.model = conv.load(rows)
        self.model.labels = [_recover_label(v, ltype) for v in (self.model.labels or [])]
        meta = self.model.meta
        self.feature_cols = list(meta.get("featureCols"))
        cats = meta.get("categoricalCols") if meta.contains("categoricalCols") else None
        self.cat_cols = list(cats or [])
        self.cat_maps: Dict[str, Dict[str, int]] = {}
        if self.model.indexer_rows:
            for ci, tok, idx in self.model.indexer_rows:
                if ci >= 0:
                    self.cat_maps.setdefault(self.cat_cols[ci], {})[tok] = int(idx)
        self.labels = self.model.labels
        self._after_load()
        names = [self.pred_col] + ([self.detail_col] if self.detail_col else [])
        types = [self.predResultType()] + ([Types.STRING] if self.detail_col else [])
        reserved = self.params.get("reservedCols") if self.params.contains("reservedCols") else None
        self.helper = OutputColsHelper(self.dataSchema, names, types, reserved)

    def _label_type_from_rows(self, rows):
        schema = self.getModelSchema()
        if schema is not None and len(schema.names) >= 3:
            return schema.types[2]
        return Types.DOUBLE

    def _after_load(self):
        pass

    def _n_dist(self) -> int:
        r0 = self.model.roots[0] if self.model.roots else None
        if r0 is None or r0.counter is None or r0.counter.distributions is None:
            return 1
        return len(r0.counter.distributions)

    # -- feature matrix: X [n, F] float64 with NaN for missing; categorical as index (NaN if unseen) --
    def _features(self, mt) -> np.ndarray:
        n = mt.num_rows
        X = np.empty((n, len(self.feature_cols)), dtype=np.float64)
        for j, c in enumerate(self.feature_cols):
            vals = mt.column_values(c)
            if c in self.cat_cols:
                m = self.cat_maps.get(c, {})
                X[:, j] = [np.nan if v is None else m.get(java_str(v), np.nan) for v in vals]
            else:
                X[:, j] = [np.nan if v is None else float(v) for v in vals]
        return X

    def _accumulate(self, X: np.ndarray, flat: _FlatForest) -> (np.ndarray, np.ndarray):
        """Sum over trees of leaf distributions (x weight) and of the weights, per row."""
        n = X.shape[0]
        nd = flat.dist.shape[1]
        acc = np.zeros((n, nd), dtype=np.float64)
        wacc = np.zeros(n, dtype=np.float64)
        if n == 0 or len(flat.feat) == 0:
            return acc, wacc
        cat_nrows = flat.cat.shape[1]
        for root in flat.roots:
            node = np.full(n, root, dtype=np.int64)
            w = np.ones(n, dtype=np.float64)
            rows = np.arange(n)
            # (row, node, weight) triples; a missing value fans a triple out over all children
            for _ in range(flat.max_steps):
                f = flat.feat[node]
                leaf = f < 0
                if leaf.any():
                    r, nn_, ww = rows[leaf], node[leaf], w[leaf]
                    np.add.at(acc, r, flat.dist[nn_] * ww[:, None])
                    np.add.at(wacc, r, ww)
                    keep = ~leaf
                    rows, node, w, f = rows[keep], node[keep], w[keep], f[keep]
                if rows.size == 0:
                    break
                x = X[rows, f]
                cr = flat.catrow[node]
                child = np.where(x <= flat.thr[node], 0, 1)
                iscat = cr >= 0
                if iscat.any():
                    xi = np.where(np.isnan(x), -1, x).astype(np.int64)
                    ok = iscat & (xi >= 0) & (xi < cat_nrows)
                    cm = np.full(rows.size, -1, dtype=np.int64)
                    cm[ok] = flat.cat[cr[ok], xi[ok]]
                    child = np.where(iscat, cm, child)
                miss = np.isnan(x) | (child < 0)
                if miss.any():
                    mr, mn, mw = rows[miss], node[miss], w[miss]
                    fr, fnode, fw = [], [], []
                    for r_, n_, w_ in zip(mr, mn, mw):
                        k = flat.nchild[n_]
                        ch = flat.first[n_] + np.arange(k)
                        cw = flat.wsum[ch]
                        tot = cw.sum()
                        if tot == 0:
                            raise RuntimeError("Model is broken. Sum weight is zero.")
                        fr.extend([r_] * k)
                        fnode.extend(ch.tolist())
                        fw.extend((w_ * cw / tot).tolist())
                    keep = ~miss
                    rows = np.concatenate([rows[keep], np.asarray(fr, dtype=np.int64)])
                    node = np.concatenate([flat.first[node[keep]] + child[keep], np.asarray(fnode, dtype=np.int64)])
                    w = np.concatenate([w[keep], np.asarray(fw, dtype=np.float64)])
                else:
                    node = flat.first[node] + child
        return acc, wacc

    def _map_columns(self, mt):
        from ...common.table import Column
        X = self._features(mt)
        flat = getattr(self, "_flat", None)
        if flat is None:
            flat = self._flat = _FlatForest(self.model.roots, self._n_dist())
        acc, wacc = self._accumulate(X, flat)
        preds, details = self._finish(acc, wacc)
        cols = [Column.from_values(preds, self.helper.out_types[0])]
        if self.detail_col:
            cols.append(Column.from_values(details, Types.STRING))
        return cols

    def _map_row_values(self, row):
        from ...common.table import MTable
        mt = MTable.from_rows([tuple(row)], self.dataSchema)
        cols = self._map_columns(mt)
        return [c.to_list()[0] for c in cols]

    def _finish(self, acc, wacc):
        raise NotImplementedError


def _detail_json(d: Dict[str, float]) -> str:
    """Gson of a ``HashMap<String, Double>`` (Java HashMap iteration order)."""
    return gson_dumps(d, java_map_order=True)


class GbdtModelMapper(TreeModelMapper):
    """``GbdtModelMapper.java``: sum of leaf values; binary -> sigmoid, regression -> + gbdt.y.period."""

    def _after_load(self):
        meta = self.model.meta
        self.period = float(meta.get("gbdt.y.period")) if meta.contains("gbdt.y.period") else 0.0
        self.algo_type = int(meta.get("algoType")) if meta.contains("algoType") else 0

    def predResultType(self):
        if self.model is not None and self.algo_type == 1:
            return self._label_type_from_rows(None)
        return Types.DOUBLE

    def _finish(self, acc, wacc):
        s = acc[:, 0]
        if self.algo_type == 1:
            preds, details = [], []
            for v in s:
                p = 1.0 / (1.0 + math.exp(-v))
                preds.append(self.labels[1] if p >= 0.5 else self.labels[0])
                details.append(_detail_json({java_str(self.labels[0]): 1.0 - p, java_str(self.labels[1]): p}))
            return preds, details
        return [float(v) + self.period for v in s], [None] * len(s)


class RandomForestModelMapper(TreeModelMapper):
    """``RandomForestModelMapper.java``: average of leaf distributions; classification -> argmax label."""

    def _after_load(self):
        tt = self.model.meta.get("treeType") if self.model.meta.contains("treeType") else "AVG"
        self.regression = str(getattr(tt, "name", tt)).upper() == "MSE"

    def predResultType(self):
        if self.model is not None and not self.regression:
            return self._label_type_from_rows(None)
        return Types.DOUBLE

    def _finish(self, acc, wacc):
        norm = np.where(wacc[:, None] != 0, acc / np.where(wacc == 0, 1.0, wacc)[:, None], acc)
        if self.regression:
            return [float(v) for v in norm[:, 0]], [None] * len(norm)
        preds, details = [], []
        for row in norm:
            d, best, bi = {}, 0.0, -1
            for i, p in enumerate(row):
                d[java_str(self.labels[i])] = float(p)
                if best < p:
                    best, bi = p, i
            preds.append(self.labels[bi] if bi >= 0 else None)
            details.append(_detail_json(d))
        return preds, details
