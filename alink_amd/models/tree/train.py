"""GBDT / random forest / decision tree training drivers on top of ``engine.TreeBuilder``.

Reference: ``A/operator/common/tree/BaseGbdtTrainBatchOp.java`` (params, depth from ``maxLeaves``
``:255-263``, label handling, model meta ``:265-300``, feature-importance side output ``:230-236``),
``parallelcart/ConstructLocalBin.java`` (gradients: least squares ``g = pred - (y - mean)``, ``h = 1``
``:105-131``; logistic ``g = p - y``, ``h = p(1-p)`` with float32 storage ``:170-205``; learning to rank
``algoType`` 2 LambdaMART-NDCG / 3 LambdaMART-DCG / 4 GBRank over ``groupCol`` queries ``:296-430``, see
``ops/csrc/gbdt_rank.hip``),
``parallelcart/Split.java`` (row / feature subsampling after every tree ``:100-160``) and
``BaseRandomForestTrainBatchOp.java`` (per-tree row sampling ``SampleData`` ``:470-503``, gain type per tree
for ``treeType`` AVG/PARTITION ``:420-460``, model meta = the op params).

Random-forest trees are independent: each one re-uses the device-resident bin matrix with its own row
sample, so the whole forest is trained without re-reading or re-binning the table.
"""
from __future__ import annotations

import math
import time
from typing import Any, List, Optional, Tuple

import numpy as np
import torch

from ...common.jrandom import JavaRandom
from ...common.params import Params
from ...common.table import MTable
from ...common.types import TableSchema, Types
from ...ops import elementwise as ew
from ...parallel import comm
from .data import build_bins, categorical_cols, distinct_labels, numeric_column
from .engine import SplitConfig, TreeBuilder
from .model import TreeModel, TreeModelDataConverter, feature_importance

__all__ = ["train_gbdt", "train_forest", "IMPORTANCE_SCHEMA"]

IMPORTANCE_SCHEMA = TableSchema(["feature", "importance"], [Types.STRING, Types.LONG])


def _pget(p: Params, name, default=None):
    try:
        if p.contains(name):
            v = p.get(name)
            return default if v is None else v
    except KeyError:
        pass
    return default


def _ename(v, default):
    if v is None:
        return default
    return str(getattr(v, "name", v)).upper()


def _label_indices(mt: MTable, label_col: str, labels: List[Any], device) -> torch.Tensor:
    from ...common.javafmt import java_str
    col = mt.col(label_col)
    if isinstance(col.values, torch.Tensor) and col.values.dim() == 1 and col.nulls is None and \
            all(isinstance(l, (int, float)) and not isinstance(l, bool) for l in labels):
        v = col.values.to(device=device, dtype=torch.float64)
        lab = torch.tensor([float(l) for l in labels], dtype=torch.float64, device=device)
        idx = torch.searchsorted(lab, v).clamp(max=len(labels) - 1)
        if not bool((lab[idx] == v).all()):
            raise RuntimeError("Can not find a label value in the label set")
        return idx
    pos = {java_str(l): i for i, l in enumerate(labels)}
    idx = []
    for v in mt.column_values(label_col):
        if v is None or java_str(v) not in pos:
            raise RuntimeError(f"Can not find {v}")
        idx.append(pos[java_str(v)])
    return torch.tensor(idx, dtype=torch.long, device=device)


def _weights(mt: MTable, params: Params, device) -> torch.Tensor:
    wc = _pget(params, "weightCol")
    if wc is None:
        return torch.ones(mt.num_rows, dtype=torch.float64, device=device)
    w, null = numeric_column(mt, wc, device)
    return torch.where(null, torch.zeros_like(w), w)


def _type_string(t) -> str:
    return t.sql if t.sql != "VARCHAR" else "VARCHAR"


# ---------------------------------------------------------------------------------------------------
# GBDT
# ---------------------------------------------------------------------------------------------------
def train_gbdt(mt: MTable, params: Params, env, algo_type: int) -> Tuple[List[tuple], TreeModelDataConverter,
                                                                         List[tuple], dict]:
    """Returns (model rows, converter, importance rows, train info)."""
    dev = env.device
    feature_cols = list(params.get("featureCols"))
    label_col = params.get("labelCol")
    cat = categorical_cols(mt.schema, feature_cols, _pget(params, "categoricalCols"))
    params.set("categoricalCols", cat)
    depth = int(_pget(params, "maxDepth", 6))
    max_leaves = int(_pget(params, "maxLeaves", 2 ** 31 - 1))
    if max_leaves > 0:
        depth_leaf = int(math.log(max_leaves + 0.01) / math.log(2.0)) + 1
        depth = min(depth, depth_leaf)
    num_trees = int(_pget(params, "numTrees", 100))
    max_bins = int(_pget(params, "maxBins", 128))
    lr = float(_pget(params, "learningRate", 0.3))
    sub_ratio = float(_pget(params, "subsamplingRatio", 1.0))
    feat_ratio = float(_pget(params, "featureSubsamplingRatio", 1.0))
    seed = int(_pget(params, "seed", 0))
    label_type = mt.col_type(label_col)
    labels = None
    offsets = group_sample_idx = None
    if algo_type >= 2:
        mt, offsets, group_sample_idx = _rank_groups(mt, params, dev)
        # InitialTrainningBuffer.java:221-224: the gain 2^min(label, 31) - 1, stored as float; no label centring
        yd, _ = numeric_column(mt, label_col, dev)
        y = (torch.pow(2.0, torch.clamp(yd, max=31.0)) - 1.0).to(torch.float32)
        period = 0.0
    elif algo_type == 1:
        labels = distinct_labels(mt, label_col)
        if len(labels) != 2:
            raise ValueError(f"Binary classification requires exactly 2 labels, found {len(labels)}")
        y = _label_indices(mt, label_col, labels, dev).to(torch.float32)
        period = 0.0
    else:
        yd, null = numeric_column(mt, label_col, dev)
        tot = torch.stack([yd.sum(), torch.tensor(float(yd.numel()), dtype=torch.float64, device=dev)])
        comm.all_reduce(tot, "sum")
        period = float(tot[0] / tot[1]) if float(tot[1]) > 0 else 0.0
        y = (yd - period).to(torch.float32)
    w = _weights(mt, params, dev).to(torch.float32)
    t_bin = time.perf_counter()
    data = build_bins(mt, feature_cols, cat, max_bins, dev, exact_midpoints=False, seed=seed)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t_bin = time.perf_counter() - t_bin
    t_trees = time.perf_counter()
    cfg = SplitConfig("gbdt", max_depth=depth, min_samples_per_leaf=int(_pget(params, "minSamplesPerLeaf", 100)),
                      min_info_gain=float(_pget(params, "minInfoGain", 0.0)),
                      min_sum_hessian_per_leaf=float(_pget(params, "minSumHessianPerLeaf", 0.0)),
                      learning_rate=lr)
    builder = TreeBuilder(data, cfg)
    n = mt.num_rows
    F = len(feature_cols)
    row_gen = _row_generator(dev, seed)
    feat_rng = np.random.default_rng(seed + 104729)       # identical on every rank
    pred = torch.zeros(n, dtype=torch.float32, device=dev)
    roots = []
    fmask = np.ones(F, dtype=bool)
    for t in range(num_trees):
        if sub_ratio < 1.0 and group_sample_idx is not None:
            # learning to rank samples whole queries (Split.java:142-153)
            ng = int(offsets.numel()) - 1
            sample = (torch.rand(ng, generator=row_gen, device=dev) < sub_ratio)[group_sample_idx]
        else:
            sample = (torch.rand(n, generator=row_gen, device=dev) < sub_ratio) if sub_ratio < 1.0 else \
                torch.ones(n, dtype=torch.bool, device=dev)
        if feat_ratio < 1.0:   # InitialTrainningBuffer / Split draw a feature subset for every tree
            fmask = feat_rng.random(F) < feat_ratio
        # K6: {g*g, g, h, 1} row records in one fused pass (logistic g/h in fp64, weights applied in fp32)
        if algo_type >= 2:
            # K6 ranking variant: per-query pair lambdas (ConstructLocalBin.java:296-430)
            stats = ew.gbdt_rank_stats(pred, y, w, offsets, algo_type)
        else:
            stats = ew.gbdt_grad_stats(pred, y, w, 1 if algo_type == 1 else 0)
        root, codes, leaves = builder.build(stats, sample, fmask)
        roots.append(root)
        # Split.java: predBuf = (float) (curPred + leftCounter.sum / leftCounter.weightSum)
        vals = torch.tensor([lf.counter.distributions[0] if lf.counter and lf.counter.distributions else 0.0
                             for lf in leaves] or [0.0], dtype=torch.float64, device=dev)
        if algo_type == 4:
            # GBRank keeps the running MEAN of the trees' outputs (Split.java:128-131, iterCount = t + 1)
            leaf = (-1 - codes.long()).clamp(min=0, max=vals.numel() - 1)
            inc = torch.where(codes < 0, vals[leaf], torch.zeros_like(vals[leaf]))
            pred = ((t * pred.double() + inc) / (t + 1)).to(torch.float32)
        else:
            pred = ew.gbdt_leaf_update(pred, codes.to(torch.int32), vals)
    meta = params.clone()
    meta.set("featureCols", feature_cols).set("labelCol", label_col).set("categoricalCols", cat)
    meta.set("numTrees", num_trees).set("maxDepth", depth).set("algoType", algo_type)
    lt = label_type if algo_type == 1 else Types.DOUBLE
    meta.set("labelTypeName", _type_string(lt))
    meta.set("gbdt.y.period", float(period))
    conv = TreeModelDataConverter(lt)
    model = TreeModel(meta, roots, labels, data.indexer_rows or None)
    rows = conv.save(model)
    imp = feature_importance(roots, feature_cols)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    info = {"numTrees": num_trees, "depth": depth, "bins": data.B, "binning_s": t_bin,
            "trees_s": time.perf_counter() - t_trees}
    return rows, conv, imp, info


def _rank_groups(mt: MTable, params: Params, dev):
    """Learning-to-rank layout (BaseGbdtTrainBatchOp.java:245-252, 431-446; InitialTrainningBuffer.java:157-235):
    the rows of one query (``groupCol``, read as an integer like the reference's ``intValue()``) on one rank
    (hash exchange), contiguous and in their input order.  Returns (the regrouped table, int64 [Q+1] query row
    offsets, each row's query index)."""
    from ...parallel.shuffle import hash_partition
    gcol = _pget(params, "groupCol")
    if gcol is None:
        raise ValueError("learning to rank (algoType 2-4) needs groupCol")
    mt = hash_partition(mt, [mt.schema.names.index(gcol)])
    gv, gnull = numeric_column(mt, gcol, dev)
    if bool(gnull.any()):
        raise ValueError(f"groupCol {gcol} has null values")
    gid = gv.to(torch.int64)                       # intValue(): truncation toward zero
    order = torch.sort(gid, stable=True).indices
    mt = mt.take(order)
    gid = gid[order]
    _, counts = torch.unique_consecutive(gid, return_counts=True)
    offsets = torch.zeros(counts.numel() + 1, dtype=torch.int64, device=gid.device)
    torch.cumsum(counts, 0, out=offsets[1:])
    qidx = torch.repeat_interleave(torch.arange(counts.numel(), device=gid.device), counts)
    return mt, offsets, qidx


# ---------------------------------------------------------------------------------------------------
# random forest / decision tree
# ---------------------------------------------------------------------------------------------------
def _tree_generator(dev, seed: int, tree: int, replicated_rows: bool) -> torch.Generator:
    """Row-sampling stream of one forest tree (Philox on the GPU).  Rows replicated on every rank (tree-parallel)
    use one stream per tree; partitioned rows add the rank so ranks draw distinct samples of their rows."""
    g = torch.Generator(device=dev)
    g.manual_seed((int(seed) * 1000003 + 7919 * int(tree) + (0 if replicated_rows else 104729 * comm.get_rank()))
                  & 0x7FFFFFFFFFFFFFFF)
    return g


def _row_generator(dev, seed: int) -> torch.Generator:
    """Per-rank device RNG for row subsampling (Philox on the GPU); rank-distinct streams."""
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed) * 1000003 + 7919 * comm.get_rank() + 17)
    return g


def _avg_gain(num_trees: int, tid: int) -> str:
    div, mod = num_trees // 3, num_trees % 3
    start_gini = div if mod < 1 else div + 1
    start_ratio = start_gini + div if mod < 2 else start_gini + div + 1
    return _interval_gain(start_gini, start_ratio, tid)


def _interval_gain(start_gini: int, start_ratio: int, tid: int) -> str:
    if tid < start_gini:
        return "infogain"
    if tid < start_ratio:
        return "gini"
    return "infogainratio"


def _gain_for_tree(tree_type: str, params: Params, num_trees: int, tid: int) -> str:
    if tree_type == "AVG":
        return _avg_gain(num_trees, tid)
    if tree_type == "PARTITION":
        a, b = str(_pget(params, "treePartition", "")).split(",")
        return _interval_gain(int(a), int(b), tid)
    return {"MSE": "mse", "GINI": "gini", "INFOGAIN": "infogain", "INFOGAINRATIO": "infogainratio"}[tree_type]


def train_forest(mt: MTable, params: Params, env, regression: bool) -> Tuple[List[tuple], TreeModelDataConverter,
                                                                             dict]:
    dev = env.device
    feature_cols = list(params.get("featureCols"))
    label_col = params.get("labelCol")
    tree_type = _ename(_pget(params, "treeType"), "AVG")
    if regression:
        tree_type = "MSE"
    params.set("treeType", tree_type)
    cat = categorical_cols(mt.schema, feature_cols, _pget(params, "categoricalCols"))
    params.set("categoricalCols", cat)
    params.set("featureTypes", [_type_string(mt.col_type(c)) for c in feature_cols])
    num_trees = int(_pget(params, "numTrees", 10))
    max_bins = int(_pget(params, "maxBins", 128))
    seed = int(_pget(params, "seed", 0))
    max_depth = int(_pget(params, "maxDepth", 2 ** 31 - 1))
    msl = int(_pget(params, "minSamplesPerLeaf", 2))
    F = len(feature_cols)
    ratio = float(_pget(params, "featureSubsamplingRatio", 0.2))
    nsub = int(_pget(params, "numSubsetFeatures", 2 ** 31 - 1))
    node_feats = max(1, min(int(ratio * F), min(F, nsub)))
    factor = float(_pget(params, "subsamplingRatio", 100000.0))
    n = mt.num_rows
    if factor > 1.0:
        total = float(sum(comm.all_gather_object(int(n))))
        factor = min(factor / total, 1.0) if total > 0 else 1.0
    label_type = mt.col_type(label_col)
    labels = None
    w = _weights(mt, params, dev)
    if regression:
        y, _ = numeric_column(mt, label_col, dev)
        lt = Types.DOUBLE
    else:
        labels = distinct_labels(mt, label_col)
        y = _label_indices(mt, label_col, labels, dev)
        lt = label_type
    params.set("labelTypeName", _type_string(lt))
    data = build_bins(mt, feature_cols, cat, max_bins, dev, exact_midpoints=True, seed=seed)
    hdt = torch.float32 if dev.type == "cuda" else torch.float64
    if regression:
        wy = (w * y)
        stats = torch.stack([w, wy, wy * wy, torch.ones_like(w)], dim=1).to(hdt)
    else:
        C = len(labels)
        stats = torch.zeros((n, C + 1), dtype=hdt, device=dev)
        stats[torch.arange(n, device=dev), y] = w.to(hdt)
        stats[:, C] = 1.0
    # P7 tree-parallel forest (createTreeMode "series", the reference default: SampleData tags rows per tree
    # and AvgPartition sends tree t to worker t % P, BaseRandomForestTrainBatchOp.java:219-262,446-503).  Here
    # the binned rows (uint8, F bytes/row) and their statistics are all-gathered once over RCCL, rank r grows
    # trees t = r (mod P) on its own GPU with no per-level collective, and the finished trees are gathered.
    # "parallel" keeps the data-parallel histogram all-reduce of every tree.
    ws = comm.get_world_size()
    series = str(_pget(params, "createTreeMode", "series")).lower() != "parallel" and ws > 1
    if series:
        data.bins = comm.all_gather_varlen(data.bins.contiguous())
        stats = comm.all_gather_varlen(stats.contiguous())
        n = data.bins.shape[0]
        mine = [t for t in range(num_trees) if t % ws == comm.get_rank()]
    else:
        mine = list(range(num_trees))
    grown = {}
    for t in mine:
        kind = _gain_for_tree(tree_type, params, num_trees, t)
        cfg = SplitConfig(kind, max_depth=max_depth, min_samples_per_leaf=msl,
                          n_classes=0 if regression else len(labels),
                          min_sample_ratio_per_child=float(_pget(params, "minSampleRatioPerChild", 0.0)),
                          min_info_gain=float(_pget(params, "minInfoGain", 0.0)),
                          max_leaves=int(_pget(params, "maxLeaves", 2 ** 31 - 1)),
                          node_feature_count=node_feats,
                          max_memory_bytes=int(_pget(params, "maxMemoryInMB", 64)) * (1 << 20))
        builder = TreeBuilder(data, cfg, local=series)
        # per-tree row sample drawn on the device from a (seed, tree)-keyed stream: the same tree gets the same
        # sample whichever rank grows it
        sample = (torch.rand(n, generator=_tree_generator(dev, seed, t, series), device=dev) < factor) \
            if factor < 1.0 else torch.ones(n, dtype=torch.bool, device=dev)
        # DecisionTree seeds java.util.Random with the same `seed` for every tree
        root, _, _ = builder.build(stats, sample, None, JavaRandom(seed))
        grown[t] = root
    if series:
        for part in comm.all_gather_object(grown):
            grown.update(part)
    roots = [grown[t] for t in range(num_trees)]
    meta = params.clone()
    conv = TreeModelDataConverter(lt)
    model = TreeModel(meta, roots, labels, data.indexer_rows or None)
    return conv.save(model), conv, {"numTrees": num_trees, "bins": data.B}
