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
    """BFS numbering exactly as ``TreeModelDataConverter.serializeTree`` (FIFO queue, ids on enqueue).  Every
    double of the tree is formatted in ONE host C++ ``Double.toString`` call and the node strings are assembled
    from them (``_serialize_tree_gson`` — the generic Gson walk — is the reference form and the fallback)."""
    fast = _serialize_tree_fast(root)
    return fast if fast is not None else _serialize_tree_gson(root)


def _serialize_tree_fast(root: Node) -> Optional[List[str]]:
    from ... import _native
    order = [root]
    head = 0
    while head < len(order):
        nd = order[head]
        head += 1
        if not nd.isLeaf():
            order.extend(nd.nextNodes)
    vals = []
    for nd in order:
        c = nd.counter
        vals.append(nd.gain)
        if c is not None:
            vals.append(c.weightSum)
            if c.distributions is not None:
                vals.extend(c.distributions)
        vals.append(nd.continuousSplit)
    arr = np.asarray(vals, dtype=np.float64)
    if not np.all(np.isfinite(arr)):
        return None
    body = _native.java_double_join(arr)
    if body is None:
        return None
    strs = body.split(",")
    out, k, nid = [], 0, 1
    for i, nd in enumerate(order):
        c = nd.counter
        parts = ['{"node":{"featureIndex":', str(int(nd.featureIndex)), ',"gain":', strs[k]]
        k += 1
        if c is not None:
            parts += [',"counter":{"weightSum":', strs[k], ',"numInst":', str(int(c.numInst))]
            k += 1
            if c.distributions is not None:
                nd_ = len(c.distributions)
                parts += [',"distributions":[', ",".join(strs[k:k + nd_]), "]"]
                k += nd_
            parts.append("}")
        if nd.categoricalSplit is not None:
            parts += [',"categoricalSplit":[', ",".join(str(int(x)) for x in nd.categoricalSplit), "]"]
        parts += [',"continuousSplit":', strs[k], '},"id":', str(i)]
        k += 1
        if not nd.isLeaf():
            ids = range(nid, nid + len(nd.nextNodes))
            nid += len(nd.nextNodes)
            parts += [',"nextIds":[', ",".join(str(x) for x in ids), "]"]
        parts.append("}")
        out.append("".join(parts))
    return out


def _serialize_tree_gson(root: Node) -> List[str]:
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
    # one JSON document per tree (a list of its node objects) instead of one parse per node
    objs = json.loads("[" + ",".join(strings) + "]") if strings else []
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
    """A tree ensemble.  A model read from a table keeps its trees as the node strings (``tree_strings``) and
    builds ``Node`` objects only when ``roots`` is first read; serving takes ``native_flat()`` instead — the flat
    arrays parsed in one C++ pass (``_native/csrc/tree_model.cpp``), no per-node Python objects."""

    def __init__(self, meta: Params, roots: Optional[List[Node]], labels: Optional[List[Any]],
                 indexer_rows: Optional[List[Any]], tree_strings: Optional[List[Sequence[str]]] = None):
        self.meta = meta
        self._roots = roots
        self.labels = labels
        self.indexer_rows = indexer_rows
        self._tree_strings = tree_strings
        self._native = None

    @property
    def roots(self) -> List[Optional[Node]]:
        if self._roots is None:
            self._roots = [deserialize_tree(s) for s in (self._tree_strings or [])]
        return self._roots

    @roots.setter
    def roots(self, v):
        self._roots = v
        self._tree_strings = None
        self._native = None

    def native_flat(self):
        """``(arrays, tree_lo)`` of ``_native.tree_flatten`` over the model's node strings, or None (model built in
        memory, library missing, or rows outside the serializer's form)."""
        if self._native is None:
            self._native = False
            if self._tree_strings is not None:
                from ... import _native
                sizes = [len(s) for s in self._tree_strings]
                lo = np.zeros(len(sizes) + 1, dtype=np.int64)
                np.cumsum(sizes, out=lo[1:])
                strings = [x for s in self._tree_strings for x in s]
                res = _native.tree_flatten(strings, lo)
                if res is not None:
                    self._native = (res, lo)
        return self._native or None


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
        trees = [data[p["f0"]:p["f1"]] for p in meta.get("treePartition")["partitions"]]
        return TreeModel(meta, None, list(labels) if labels else [], indexer_rows, tree_strings=trees)


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

    @classmethod
    def from_native(cls, nat: dict, tree_lo: np.ndarray, n_dist: int) -> "_FlatForest":
        """The same arrays from ``_native.tree_flatten`` (node i of tree t at tree_lo[t] + its BFS id — the order
        the constructor's BFS produces for a serialized tree)."""
        self = cls.__new__(cls)
        n = int(nat["feat"].shape[0])
        self.feat = nat["feat"].astype(np.int64)
        self.thr = nat["thr"]
        leaf = self.feat == -1
        self.first = np.where(leaf, -1, nat["first"]).astype(np.int64)
        self.nchild = np.where(leaf, 0, nat["nchild"]).astype(np.int64)
        d = nat["dist"]
        if d.shape[1] >= n_dist:
            self.dist = np.ascontiguousarray(d[:, :n_dist])
        else:
            self.dist = np.zeros((n, n_dist), dtype=np.float64)
            self.dist[:, :d.shape[1]] = d
        self.wsum = nat["wsum"]
        self.roots = [int(tree_lo[t]) for t in range(len(tree_lo) - 1) if tree_lo[t + 1] > tree_lo[t]]
        cl = nat["cat_len"].astype(np.int64)
        has = (~leaf) & (cl >= 0)
        self.catrow = np.full(n, -1, dtype=np.int64)
        idx = np.flatnonzero(has)
        self.catrow[idx] = np.arange(idx.size)
        lens = cl[idx]
        width = int(max(lens.max() if lens.size else 1, 1))
        self.cat = np.full((max(1, idx.size), width), -1, dtype=np.int64)
        if lens.sum():
            rows = np.repeat(np.arange(idx.size), lens)
            starts = nat["cat_off"][idx]
            pos = np.arange(int(lens.sum())) - np.repeat(np.cumsum(lens) - lens, lens)
            self.cat[rows, pos] = nat["cat"][np.repeat(starts, lens) + pos]
        self.max_steps = n + 1
        return self


class _DeviceForest:
    """``_FlatForest`` as the tables of ``ops/csrc/tree_predict.hip``: every feature the forest splits on gets a
    code slot; a continuous split stores the rank k of its threshold among that feature's sorted distinct
    thresholds (x <= thr  <=>  code(x) <= k, code(x) = #thresholds < x), a categorical split -(map row)-1."""

    def __init__(self, flat: "_FlatForest", cat_features: Sequence[int], cat_sizes: Sequence[int], device):
        internal = flat.feat >= 0
        used = np.unique(flat.feat[internal]).tolist()
        self.slot = {f: i for i, f in enumerate(used)}
        self.cat_features = set(int(f) for f in cat_features)
        ynode = np.zeros(len(flat.feat), dtype=np.int64)
        self.thresholds: Dict[int, np.ndarray] = {}
        widest = 0
        # every internal node at once (255k nodes x 1000 features took 0.11 s as a per-feature mask loop): continuous
        # nodes sorted by (feature, threshold); a threshold's rank is its dense index within its feature's distinct
        # values -- np.searchsorted(np.unique(thr of f), thr) -- NaN thresholds equal to each other, last
        is_cat = np.zeros(len(flat.feat), dtype=bool)
        if self.cat_features:
            is_cat = internal & np.isin(flat.feat, np.fromiter(self.cat_features, dtype=np.int64))
            ynode[is_cat] = -flat.catrow[is_cat] - 1
            for f in used:
                if f in self.cat_features:
                    widest = max(widest, int(cat_sizes[f]) if f < len(cat_sizes) else 0, flat.cat.shape[1])
        cidx = np.flatnonzero(internal & ~is_cat)
        if cidx.size:
            fz, tz = flat.feat[cidx], flat.thr[cidx]
            order = np.lexsort((tz, fz))
            fs, ts = fz[order], tz[order]
            new_f = np.ones(fs.size, dtype=bool)
            new_f[1:] = fs[1:] != fs[:-1]
            same_t = np.zeros(ts.size, dtype=bool)
            same_t[1:] = (ts[1:] == ts[:-1]) | (np.isnan(ts[1:]) & np.isnan(ts[:-1]))
            new_v = new_f | ~same_t
            dense = np.cumsum(new_v) - 1                       # global index of a distinct (feature, threshold)
            gstart = np.flatnonzero(new_f)                     # first sorted position of each feature
            glen = np.diff(np.append(gstart, fs.size))
            base = np.repeat(dense[gstart], glen)
            ynode[cidx[order]] = dense - base
            vals = ts[new_v]                                   # distinct thresholds, feature-major
            vstart = dense[gstart]
            vend = np.append(vstart[1:], vals.size)
            for f, a, b in zip(fs[gstart].tolist(), vstart.tolist(), vend.tolist()):
                self.thresholds[f] = vals[a:b]
                widest = max(widest, b - a + 1)
        # code width: uint8 while every code and the MISS sentinel (255) stay apart
        self.code_bytes = 1 if widest < 255 else (2 if widest < 65535 else 0)
        self.supported = self.code_bytes > 0 and len(flat.roots) > 0
        F = max(1, len(used))
        self.stride = ((F * max(1, self.code_bytes) + 15) // 16) * 16
        self.supported = self.supported and self.stride * 64 <= 160 * 1024
        lut = np.full(max(used) + 2 if used else 1, -1, dtype=np.int64)
        lut[np.asarray(used, dtype=np.int64)] = np.arange(len(used))
        node_slot = np.where(internal, lut[np.maximum(flat.feat, 0)], -1)
        nodes = np.stack([node_slot, ynode, np.where(internal, flat.first, 0), flat.nchild], 1).astype(np.int32)
        self.dev = device
        self.nodes = torch.from_numpy(np.ascontiguousarray(nodes)).to(device)
        self.dist = torch.from_numpy(np.ascontiguousarray(flat.dist)).to(device)
        self.nd = int(flat.dist.shape[1])
        self.wsum = torch.from_numpy(np.ascontiguousarray(flat.wsum)).to(device)
        self.cat = torch.from_numpy(np.ascontiguousarray(flat.cat.astype(np.int32))).to(device)
        self.roots = torch.tensor(flat.roots, dtype=torch.int32, device=device)
        # per continuous feature: thresholds padded with +inf into one [Fc, L] table for a batched searchsorted
        self.cont = [f for f in used if f not in self.cat_features]
        L = max([len(self.thresholds[f]) for f in self.cont] + [1])
        Tp = np.full((max(1, len(self.cont)), L), np.inf)
        for i, f in enumerate(self.cont):
            Tp[i, :len(self.thresholds[f])] = self.thresholds[f]
        self.T = torch.from_numpy(Tp).to(device)
        # the device code kernel's table: rows padded with +inf to a power of two W > every threshold count
        W = 1
        while W < L + 1:
            W *= 2
        Tw = np.full((max(1, len(self.cont)), W), np.inf)
        Tw[:, :L] = Tp
        self.TW, self.W = torch.from_numpy(Tw).to(device), W
        self.cont_slots = torch.tensor([self.slot[f] for f in self.cont] or [0], dtype=torch.int32, device=device)

    def codes(self, cols: Dict[int, torch.Tensor], cat_codes: Dict[int, torch.Tensor], n: int,
              row0: int = 0, use_kernel: Optional[bool] = None) -> torch.Tensor:
        """[n, stride] uint8 code rows (uint16 pairs when code_bytes is 2) of rows ``row0 .. row0+n-1`` from fp64
        continuous columns (NaN = missing) and int64 categorical indices (-1 = missing).  On the GPU the continuous
        codes come from ``alink_tree_codes`` (one pass, ops/csrc/tree_predict.hip); ``use_kernel=False`` is the
        torch searchsorted form (the tests' reference)."""
        from ...ops import _lib
        ct = torch.uint8 if self.code_bytes == 1 else torch.int16
        miss = 255 if self.code_bytes == 1 else -1              # 0xFFFF as int16
        if use_kernel is None:
            use_kernel = torch.device(self.dev).type == "cuda" and _lib.available() and \
                hasattr(_lib.require(), "alink_tree_codes")
        if use_kernel:
            L = _lib.require()
            out = torch.empty((n, self.stride // self.code_bytes), dtype=ct, device=self.dev)
            # column pointers go up from pinned memory without a host wait (a pageable copy would block until the
            # previous chunk's kernels finish)
            ptrs = torch.tensor([cols[f].data_ptr() for f in self.cont] or [0], dtype=torch.int64)
            if torch.device(self.dev).type == "cuda":
                ptrs = ptrs.pin_memory().to(self.dev, non_blocking=True)
            for f in self.cont:
                v = cols[f]
                if v.dtype != torch.float64 or not v.is_contiguous() or v.device != torch.device(self.dev) or \
                        v.numel() < row0 + n:
                    raise ValueError("tree codes need contiguous fp64 device columns covering the rows")
            rc = L.alink_tree_codes(ptrs.data_ptr(), len(self.cont), self.cont_slots.data_ptr(), self.TW.data_ptr(),
                                    self.W, int(row0), int(n), self.stride, self.code_bytes, out.data_ptr(),
                                    _lib.stream_ptr(self.dev))
            if rc != 0:
                raise RuntimeError(f"alink_tree_codes failed: {rc}")
            for f in self.slot:
                if f in self.cat_features:
                    v = cat_codes[f][row0:row0 + n]
                    out[:, self.slot[f]] = torch.where(v < 0, torch.full_like(v, miss), v).to(ct)
            return out
        cols = {f: v[row0:row0 + n] for f, v in cols.items()}
        cat_codes = {f: v[row0:row0 + n] for f, v in cat_codes.items()}
        out = torch.zeros((n, self.stride // self.code_bytes), dtype=ct, device=self.dev)
        if self.cont:
            X = torch.stack([cols[f] for f in self.cont])                                   # [Fc, n]
            c = torch.searchsorted(self.T, X.contiguous())
            c = torch.where(torch.isnan(X), torch.full_like(c, 65535), c)
            idx = torch.tensor([self.slot[f] for f in self.cont], device=self.dev)
            vals = torch.where(c >= 65535, torch.full_like(c, miss), c)
            out[:, idx] = vals.T.to(ct)
        for f in self.slot:
            if f in self.cat_features:
                v = cat_codes[f]
                out[:, self.slot[f]] = torch.where(v < 0, torch.full_like(v, miss), v).to(ct)
        return out


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
        nat = self.model.native_flat() if self.model._roots is None else None
        if nat is not None:
            res, lo = nat
            if len(lo) < 2 or lo[1] == lo[0] or res["dist_len"][0] < 0:
                return 1
            return int(res["dist_len"][0])
        r0 = self.model.roots[0] if self.model.roots else None
        if r0 is None or r0.counter is None or r0.counter.distributions is None:
            return 1
        return len(r0.counter.distributions)

    # -- feature columns, columnar: continuous -> fp64 (NaN = NULL), categorical -> indexer code (-1 = NULL/unseen) --
    def _cont_column(self, mt, c, device) -> torch.Tensor:
        col = mt.col(c)
        v = col.values
        if isinstance(v, torch.Tensor) and v.dim() == 1:
            x = v.to(device=device, dtype=torch.float64)
            if col.nulls is not None:
                x = torch.where(col.nulls.to(device), torch.full_like(x, float("nan")), x)
            return x
        vals = mt.column_values(c)
        return torch.tensor([np.nan if v is None else float(v) for v in vals], dtype=torch.float64, device=device)

    def _cat_column(self, mt, c, device) -> torch.Tensor:
        m = self.cat_maps.get(c, {})
        vals = mt.column_values(c)
        look = {v: m.get(java_str(v), -1) for v in set(vals) if v is not None}   # one indexer lookup per distinct
        look[None] = -1
        return torch.tensor([look[v] for v in vals], dtype=torch.int64, device=device)

    def _features(self, mt) -> np.ndarray:
        """X [n, F] float64 with NaN for missing; categorical as index (NaN if unseen) — the host walk's input."""
        n = mt.num_rows
        X = np.empty((n, len(self.feature_cols)), dtype=np.float64)
        for j, c in enumerate(self.feature_cols):
            if c in self.cat_cols:
                x = self._cat_column(mt, c, "cpu").numpy().astype(np.float64)
                X[:, j] = np.where(x < 0, np.nan, x)
            else:
                X[:, j] = self._cont_column(mt, c, "cpu").numpy()
        return X

    def _device(self, mt):
        for c in self.feature_cols:
            v = mt.col(c).values
            if isinstance(v, torch.Tensor) and v.is_cuda:
                return v.device
        env = getattr(self, "env", None)
        if env is None:
            from ...common.mlenv import MLEnvironmentFactory
            env = MLEnvironmentFactory.getDefault()
        env_dev = getattr(env, "device", None)
        return env_dev if env_dev is not None and torch.device(env_dev).type == "cuda" else None

    def _accumulate_device(self, mt, flat: "_FlatForest", dev):
        """(acc, wacc) on the GPU (``ops/csrc/tree_predict.hip``), or None when the forest does not fit the kernel
        (code width / stack) — the caller then takes the host walk."""
        from ...ops import _lib
        dfo = getattr(self, "_dforest", None)
        if dfo is None or dfo.dev != dev:
            sizes = [len(self.cat_maps.get(c, {})) if c in self.cat_cols else 0 for c in self.feature_cols]
            cat_idx = [j for j, c in enumerate(self.feature_cols) if c in self.cat_cols]
            dfo = self._dforest = _DeviceForest(flat, cat_idx, sizes, dev)
        if not dfo.supported:
            return None
        L = _lib.require()
        n = mt.num_rows
        cols = {f: self._cont_column(mt, self.feature_cols[f], dev) for f in dfo.cont}
        cats = {f: self._cat_column(mt, self.feature_cols[f], dev) for f in dfo.slot if f in dfo.cat_features}
        acc = torch.empty((n, dfo.nd), dtype=torch.float64, device=dev)
        wacc = torch.empty(n, dtype=torch.float64, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        # codes are built per chunk of rows (the batched searchsorted holds [features, rows] int64 temporaries)
        # the device code kernel needs only the [chunk, stride] code block (1 GiB of rows at a time); the torch form
        # holds [features, rows] int64 temporaries
        chunk = max(64, ((1 << 30) // dfo.stride) // 64 * 64) if hasattr(L, "alink_tree_codes") else \
            max(64, ((1 << 27) // max(1, len(dfo.slot))) // 64 * 64)
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            codes = dfo.codes(cols, cats, hi - lo, row0=lo)
            rc = L.alink_tree_predict(codes.data_ptr(), hi - lo, dfo.stride, dfo.code_bytes, dfo.nodes.data_ptr(),
                                      dfo.dist.data_ptr(), dfo.nd, dfo.wsum.data_ptr(), dfo.cat.data_ptr(),
                                      int(dfo.cat.shape[1]), dfo.roots.data_ptr(), int(dfo.roots.numel()),
                                      acc[lo:hi].data_ptr(), wacc[lo:hi].data_ptr(), err.data_ptr(),
                                      _lib.stream_ptr(dev))
            if rc != 0:
                raise RuntimeError(f"alink_tree_predict failed: {rc}")
        e = int(err.item())
        if e & 1:
            raise RuntimeError("Model is broken. Sum weight is zero.")
        if e & 2:
            return None
        return acc.cpu().numpy(), wacc.cpu().numpy()

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
                        fw.extend((w_ * (cw / tot)).tolist())       # ProcessMissing: weight * (w_i / sum)
                    keep = ~miss
                    rows = np.concatenate([rows[keep], np.asarray(fr, dtype=np.int64)])
                    node = np.concatenate([flat.first[node[keep]] + child[keep], np.asarray(fnode, dtype=np.int64)])
                    w = np.concatenate([w[keep], np.asarray(fw, dtype=np.float64)])
                else:
                    node = flat.first[node] + child
        return acc, wacc

    def _map_columns(self, mt):
        from ...common.table import Column
        flat = getattr(self, "_flat", None)
        if flat is None:
            nat = self.model.native_flat() if self.model._roots is None else None
            flat = self._flat = (_FlatForest.from_native(nat[0], nat[1], self._n_dist()) if nat is not None else
                                 _FlatForest(self.model.roots, self._n_dist()))
        res = None
        dev = self._device(mt) if mt.num_rows and len(flat.roots) else None
        if dev is not None:
            from ...ops import _lib
            if _lib.available() or not _lib.torch_fallback_allowed():
                res = self._accumulate_device(mt, flat, dev)
        if res is None:
            res = self._accumulate(self._features(mt), flat)
        preds, details = self._finish(*res)
        cols = [preds if isinstance(preds, Column) else Column.from_values(preds, self.helper.out_types[0])]
        if self.detail_col:
            cols.append(details if isinstance(details, Column) else Column.from_values(details, Types.STRING))
        return cols

    def _label_column(self, idx: np.ndarray) -> "Column":
        """Prediction column of label values ``labels[idx]`` (idx -1 -> NULL), built without a per-row loop."""
        from ...common.table import Column
        t = self.helper.out_types[0]
        bad = idx < 0
        labs = self.labels
        if labs and all(isinstance(l, (int, float)) and not isinstance(l, bool) for l in labs):
            arr = np.asarray(labs)[np.where(bad, 0, idx)]
            col = Column.from_values(arr, t)
            if bad.any():
                col = Column(col.values, torch.from_numpy(bad.copy()))
            return col
        lab = np.asarray(labs + [None], dtype=object)
        return Column.from_values(lab[np.where(bad, len(labs), idx)].tolist(), t)

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
        from ...common.detail import DetailBlock
        from ...common.table import Column
        s = acc[:, 0]
        if self.algo_type == 1:
            p = 1.0 / (1.0 + np.exp(-s))
            preds = self._label_column((p >= 0.5).astype(np.int64))
            det = Column(DetailBlock([java_str(self.labels[0]), java_str(self.labels[1])],
                                     np.stack([1.0 - p, p], 1), quoted=False))
            return preds, det
        return Column(torch.from_numpy(s + self.period)), [None] * len(s)


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
        from ...common.detail import DetailBlock
        from ...common.table import Column
        # LabelCounter.normWithWeight: divide by the weight sum unless it is zero
        norm = np.where(wacc[:, None] != 0, acc / np.where(wacc == 0, 1.0, wacc)[:, None], acc)
        if self.regression:
            return Column(torch.from_numpy(np.ascontiguousarray(norm[:, 0]))), [None] * len(norm)
        # argmax with the reference's strict "best < p" from best = 0: first maximum, none when nothing is > 0
        bi = np.argmax(norm, axis=1) if norm.shape[1] else np.zeros(len(norm), np.int64)
        bi = np.where(norm[np.arange(len(norm)), bi] > 0.0, bi, -1) if norm.shape[1] else bi - 1
        keys = [java_str(l) for l in self.labels]
        if len(set(keys)) == len(keys) and len(keys) == norm.shape[1]:
            det = Column(DetailBlock(keys, norm, quoted=False))
        else:
            det = [_detail_json({java_str(self.labels[i]): float(p) for i, p in enumerate(row)}) for row in norm]
        return self._label_column(bi.astype(np.int64)), det
