"""Level-wise histogram tree builder shared by GBDT, random forests and decision trees.

Reference algorithms (behaviour, not structure):

* GBDT — ``parallelcart/{ConstructLocalBin,CalBestSplit,Split,UpdateTreeData,SaveModel}.java``: per level one
  ``[node][feature][bin](g^2, g, h, 1)`` histogram all-reduce, best split per node with
  ``gain = |GL^2/HL + GR^2/HR - G^2/H|`` (``CalBestSplit.java:178-218``), categorical bins ordered by ``g/h``
  (``:98-120``), child counters ``sum = -lr * G`` (``:296-297``), rows routed ``2id / 2id+1``.
* RF / decision tree — ``seriestree/{DecisionTree,ContinuousSplitter,CategoricalSplitter,FeatureSplitter}.java``
  and ``Criteria.java``: Gini / InfoGain / InfoGainRatio / MSE impurities, per-node feature bagging, C4.5
  multi-way categorical splits for the information-gain criteria, BFS node order.

MI355X design: the training rows never leave HBM.  Each level does ONE histogram launch over the uint8 bin
matrix (``ops/tree.py`` — LDS-privatised HIP kernel) for only the smaller children (the larger sibling is the
parent minus its siblings), ONE all-reduce of that histogram (RCCL), a fully vectorised split search over
``[nodes, features, bins]`` on the device, and ONE routing launch.  Only the chosen splits (a few numbers per
node) cross to the host to build the model objects.
"""
from __future__ import annotations

import collections
import time

import math
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np
import torch

from ...ops import tree as tops
from ...parallel import comm
from .data import BinnedData
from .model import LabelCounter, Node

__all__ = ["SplitConfig", "TreeBuilder", "EPS"]

EPS = 1e-15
NEG = float("-inf")


@dataclass
class SplitConfig:
    kind: str                              # gbdt | gini | infogain | infogainratio | mse
    max_depth: int                         # root has depth 1; nodes at depth >= max_depth are leaves
    min_samples_per_leaf: int = 1
    n_classes: int = 0
    min_sample_ratio_per_child: float = 0.0
    min_info_gain: float = 0.0
    max_leaves: int = 2 ** 31 - 1
    min_sum_hessian_per_leaf: float = 0.0
    learning_rate: float = 1.0
    node_feature_count: Optional[int] = None  # RF bagging: features tried per node (shuffled order)
    # device bytes the histograms of one pass may take (``maxMemoryInMB``, TreeObj.java:113,263-286): a level's
    # histogram builds and split searches run in node batches within it, and the level's histograms kept for the
    # next level's sibling subtraction move to host memory when they exceed it (None: unbounded)
    max_memory_bytes: Optional[int] = None

    @property
    def classification(self) -> bool:
        return self.kind in ("gini", "infogain", "infogainratio")

    @property
    def n_stats(self) -> int:
        return self.n_classes + 1 if self.classification else 4


# ---------------------------------------------------------------------------------------------------
# criteria on stacked statistics [..., S]
# ---------------------------------------------------------------------------------------------------
def _weight(cfg: SplitConfig, X: torch.Tensor) -> torch.Tensor:
    if cfg.classification:
        return X[..., :cfg.n_classes].sum(-1)
    if cfg.kind == "mse":
        return X[..., 0]
    return X[..., 2]  # gbdt: hessian


def _count(cfg: SplitConfig, X: torch.Tensor) -> torch.Tensor:
    return X[..., -1]


def _impurity(cfg: SplitConfig, X: torch.Tensor) -> torch.Tensor:
    w = _weight(cfg, X)
    safe = torch.where(w < EPS, torch.ones_like(w), w)
    if cfg.kind == "mse":
        mean = X[..., 1] / safe
        imp = X[..., 2] / safe - mean * mean
    else:
        p = X[..., :cfg.n_classes] / safe[..., None]
        if cfg.kind == "gini":
            imp = 1.0 - (p * p).sum(-1)
        else:
            lg = torch.where(p > 0, torch.log(torch.where(p > 0, p, torch.ones_like(p))) / math.log(2.0),
                             torch.zeros_like(p))
            imp = -(p * lg).sum(-1)
    return torch.where(w < EPS, torch.zeros_like(imp), imp)


def _binary_gain(cfg: SplitConfig, T: torch.Tensor, L: torch.Tensor, R: torch.Tensor) -> torch.Tensor:
    if cfg.kind == "gbdt":
        G, H = T[..., 1], T[..., 2]
        GL, HL = L[..., 1], L[..., 2]
        GR, HR = G - GL, H - HL
        ok = (HL != 0) & (HR != 0)
        sHL = torch.where(HL == 0, torch.ones_like(HL), HL)
        sHR = torch.where(HR == 0, torch.ones_like(HR), HR)
        sH = torch.where(H == 0, torch.ones_like(H), H)
        g = torch.abs(GL * GL / sHL + GR * GR / sHR - G * G / sH)
        return torch.where(ok, g, torch.zeros_like(g))
    wT = _weight(cfg, T)
    safe = torch.where(wT < EPS, torch.ones_like(wT), wT)
    pl, pr = _weight(cfg, L) / safe, _weight(cfg, R) / safe
    g = _impurity(cfg, T) - pl * _impurity(cfg, L) - pr * _impurity(cfg, R)
    if cfg.kind == "infogainratio":
        def lg2(p):
            return torch.where(p > 0, torch.log(torch.where(p > 0, p, torch.ones_like(p))) / math.log(2.0),
                               torch.zeros_like(p))
        iv = -(pl * lg2(pl) + pr * lg2(pr))
        g = torch.where(iv < EPS, torch.zeros_like(g), g / torch.where(iv < EPS, torch.ones_like(iv), iv))
    return torch.where(wT < EPS, torch.zeros_like(g), g)


# ---------------------------------------------------------------------------------------------------
@dataclass
class _Pending:
    node: Node
    depth: int
    total: np.ndarray          # [S] float64 node statistics (incl. missing)
    parent: int = -1           # index of the parent in the previous level
    splittable: bool = True
    order: Optional[list] = None  # RF: inherited (shuffled) feature order of this node's splitters


@dataclass
class _Split:
    feature: int
    gain: float
    route: np.ndarray          # [256] child index per bin
    n_children: int
    child_totals: np.ndarray   # [k, S]
    categorical: Optional[list]
    threshold: float


# GPU fixed-point histograms read the tree's node-grouped row order (tops.RowOrder) below the root; 0: a stable
# sort of the slot keys and a statistics gather per histogram call
ROW_ORDER = int(__import__("os").environ.get("ALINK_TREE_ROW_ORDER", "1"))


class TreeBuilder:
    """Grows trees over one ``BinnedData`` (rows stay on the device between trees)."""

    def __init__(self, data: BinnedData, cfg: SplitConfig, local: bool = False):
        self.d = data
        self.cfg = cfg
        self.local = local          # rows of ALL ranks are resident: no histogram / total all-reduce (P7)
        self.dev = data.bins.device
        self.F = len(data.feature_cols)
        self.B = data.B
        self.is_cat = torch.tensor(data.is_cat, dtype=torch.bool, device=self.dev)
        self.nbins = torch.tensor(data.nbins, dtype=torch.long, device=self.dev)
        self.hist_dtype = torch.float32 if data.bins.is_cuda else torch.float64
        # feature-parallel histograms (reference ConstructLocalBin / CalBestSplit split the feature space across
        # tasks): GBDT on continuous features over P > 1 ranks reduce-SCATTERS every histogram by feature block
        # (each rank receives 1/P of it instead of the full all-reduce), searches its block, and only the [m, F]
        # best gains / bins and the chosen feature's [B, S] row per node are exchanged afterwards
        ws = comm.get_world_size()
        # every criterion shards: GBDT (continuous and categorical) and the RF / decision-tree criteria of the
        # parallel (data-partitioned) mode; tree-parallel forests (local=True) hold all rows and never reduce
        self.fshard = (not local and ws > 1
                       and __import__("os").environ.get("ALINK_GBDT_FEATURE_SHARD", "1") == "1")
        # features per rank, padded to whole 32-feature groups (the histogram kernel's unit)
        self.Fb = -(-self.F // (ws * 32)) * 32 if self.fshard else self.F
        self._hist_sub = None          # (stats tensor, histogram columns, FmStats) of the tree being built
        self.f_lo = comm.get_rank() * self.Fb if self.fshard else 0
        # categorical flags of this rank's feature block (padding features: continuous, all-zero rows)
        cat_loc = torch.zeros(self.Fb, dtype=torch.bool, device=self.dev)
        n_loc = max(0, min(self.F, self.f_lo + self.Fb) - self.f_lo)
        if n_loc:
            cat_loc[:n_loc] = self.is_cat[self.f_lo:self.f_lo + n_loc]
        self.is_cat_local = cat_loc

    # -------------------------------------------------------------------------------------------
    def _hist_cols(self, S: int) -> List[int]:
        """Statistics the split search reads: GBDT needs (g, h, count) — the g^2 column only feeds node
        counters, which come from per-node row sums instead — so the kernel moves 3 floats, not 4."""
        return [1, 2, 3] if self.cfg.kind == "gbdt" else list(range(S))

    def _histograms(self, node_of_row, sample, slot_of_node: torch.Tensor, nslots: int, stats,
                    slot_nodes=None) -> torch.Tensor:
        """[nslots, F, B, S] histograms of the level nodes ``slot_nodes`` (slot s = node slot_nodes[s]; also
        given as the device map ``slot_of_node``)."""
        nn = slot_of_node.numel()
        act = sample & (node_of_row >= 0) & (node_of_row < nn)
        slot = torch.where(act, slot_of_node[node_of_row.clamp(0, max(nn - 1, 0)).long()].to(node_of_row.dtype),
                           torch.full_like(node_of_row, -1))
        cols = self._hist_cols(stats.shape[1])
        if self._hist_sub is None or self._hist_sub[0] is not stats:
            sub = stats if len(cols) == stats.shape[1] else stats[:, cols].contiguous()
            # the fixed-point kernel's quantised statistics are built once per tree, not once per level
            elig = tops.fm_eligible(self.d.bins, len(cols), self.B) or \
                (len(cols) == 3 and tops.fm_eligible(self.d.bins, 3, self.B, pack=True))
            prep = tops.FmStats(sub) if elig else None
            self._hist_sub = (stats, sub, prep)
        _, sub, prep = self._hist_sub
        TreeBuilder.HIST_BYTES.append(nslots * self.F * self.B * len(cols) * 4)
        tro = None
        if prep is not None and slot_nodes is not None and self._level_no > 0 and ROW_ORDER:
            # below the root: the tree's node-grouped row order, regrouped once per level (RowOrder)
            if self._tro is None:
                self._tro = tops.RowOrder(prep, sample & (node_of_row >= 0))
            self._tro.regroup(node_of_row, nn, self._level_no)
            tro = self._tro
        if self.fshard:
            H = self._histograms_sharded(slot, sub, nslots, prep, tro, slot_nodes)
        else:
            H = tops.histogram(self.d.bins, slot, sub, nslots, self.B, prep=prep, tro=tro, slot_nodes=slot_nodes)
            if not self.local:
                comm.all_reduce(H, "sum")
        if len(cols) != stats.shape[1]:
            full = torch.zeros(H.shape[:-1] + (stats.shape[1],), dtype=H.dtype, device=H.device)
            full[..., cols] = H
            H = full
        return H

    RS_BLOCKS = int(__import__("os").environ.get("ALINK_GBDT_RS_BLOCKS", "4"))
    # observability (bounded: long trainings and many jobs in one process must not grow them without limit)
    RS_BYTES = collections.deque(maxlen=4096)     # reduce-scatter input bytes (fp32) per histogram piece (latest)
    RS_CALLS = 0                                  # reduce-scattered histogram pieces (all time)
    HIST_BYTES = collections.deque(maxlen=4096)   # full-width fp32 histogram bytes per histogram call (latest)
    LEVEL_STATS = collections.deque(maxlen=4096)  # (depth, nodes, split candidates, host wall s) per grown level

    def _histograms_sharded(self, slot, sub, nslots: int, prep, tro=None, slot_nodes=None) -> torch.Tensor:
        """Feature-block reduce-scatter overlapped with the histogram build: every rank's
        block of Fb features is cut into G pieces; piece c of ALL ranks' blocks is built as one feature-major
        histogram ([P * piece, slots, B, S]) and its reduce-scatter is issued asynchronously (RCCL comm stream)
        while piece c+1 builds.  This rank keeps [slots, Fb, B, S] of its own block."""
        ws = comm.get_world_size()
        gpr = self.Fb // 32                                  # 32-feature groups per rank block
        G = max(1, min(self.RS_BLOCKS, gpr))
        ps = -(-gpr // G)                                    # groups per piece (last piece padded)
        pend, real = [], []
        pad = tops.PAD_GROUP                                 # a group index past every feature: zero rows
        for c in range(G):
            lo = c * ps
            if lo >= gpr:
                break
            fgs = [j * gpr + lo + t if lo + t < gpr else pad for j in range(ws) for t in range(ps)]
            Hc = tops.histogram_groups(self.d.bins, slot, sub, nslots, self.B, fgs, prep, tro, slot_nodes)
            TreeBuilder.RS_BYTES.append(int(Hc.numel() * 4))            # fp32-equivalent, as HIST_BYTES
            TreeBuilder.RS_CALLS += 1
            pend.append(comm.reduce_scatter_async(Hc, "sum"))
            real.append(min(ps, gpr - lo) * 32)
        parts = [p.wait()[:k] for p, k in zip(pend, real)]
        return torch.cat(parts).transpose(0, 1).contiguous()            # [slots, Fb, B, S]

    def _node_totals(self, node_of_row, sample, nnodes: int, stats) -> np.ndarray:
        """[nnodes, S] float64 per-node sums over the sampled rows (one pass over rows, then all-reduce)."""
        out = tops.node_sums(node_of_row, sample, stats, nnodes)
        if not self.local:
            comm.all_reduce(out, "sum")
        return out[:nnodes].cpu().numpy()

    # -------------------------------------------------------------------------------------------
    def _search(self, Hn: torch.Tensor, feat_order: torch.Tensor, feat_ok: torch.Tensor):
        """Best split per node.  Hn [m, F, B, S] (float64); feat_order [m, F] (scan order of features);
        feat_ok [m, F] allowed.  Returns per node (gain, feature, j, multi-way flag, accept, perm [m, F, B-1] or
        None = rebuild the chosen features' bin order on the host)."""
        gain, best_j, multi, perm = self._feature_best(Hn, self.is_cat)
        return self._choose(gain, best_j, multi, feat_order, feat_ok) + (perm,)

    def _choose(self, best_j_gain, best_j, multi, feat_order, feat_ok):
        """Per node, the first feature in ``feat_order`` with the largest admissible gain (the reference's scan
        order, ties included)."""
        cfg = self.cfg
        best_j_gain = torch.where(feat_ok, best_j_gain, torch.full_like(best_j_gain, NEG))
        ordered = torch.gather(best_j_gain, 1, feat_order)
        gbest, pos = ordered.max(dim=1)
        fbest = torch.gather(feat_order, 1, pos[:, None])[:, 0]
        jbest = torch.gather(best_j, 1, fbest[:, None])[:, 0]
        mbest = torch.gather(multi, 1, fbest[:, None])[:, 0]
        accept = gbest > (cfg.min_info_gain + 1e-6 if cfg.kind == "gbdt" else 0)
        return gbest, fbest, jbest, mbest, accept

    def _feature_best(self, Hn: torch.Tensor, is_cat: torch.Tensor):
        """Per (node, feature): best admissible gain [m, F] float64 (NEG: none), its position in the feature's
        bin order [m, F], the multi-way flag [m, F] and the bin order perm [m, F, B-1] (None when the GPU kernel
        searched: the chosen features' order is rebuilt on the host).  ``is_cat`` [F] are the flags of the
        features of ``Hn`` (all features, or one rank's block under feature sharding).

        Precision: the histograms are exact fixed-point sums rounded once to fp32 (``Hn`` holds those fp32
        values); every gain below — the K8 / K10 kernels and the torch scans alike — is computed in fp64 from
        them, so GPU and host differ only by the fp64 summation order of the prefix sums (relative 1e-16), not
        by fp32 rounding of the gains."""
        cfg = self.cfg
        m, F, B, S = Hn.shape
        anycat = bool(is_cat.any())
        gpu = Hn.is_cuda and tops.gpu_kernels_ok()
        if cfg.kind == "gbdt" and not anycat:
            g, j = self._feature_gains_gbdt(Hn)
            # perm is None exactly when the GPU kernels search, whatever this block's features are: under feature
            # sharding every rank must take the same branch (the perm rows travel in the owner all-reduce)
            return g, j, torch.zeros((m, F), dtype=torch.bool, device=Hn.device), \
                None if gpu else torch.arange(B - 1, device=Hn.device).expand(m, F, B - 1)
        if gpu:
            res = tops.tree_split(Hn, cfg.kind, is_cat, cfg.n_classes, cfg.min_samples_per_leaf,
                                  cfg.min_sum_hessian_per_leaf, cfg.min_sample_ratio_per_child, cfg.min_info_gain)
            if res is not None:           # None (no instantiation for this S): the torch scan below, on every rank
                best_j_gain, best_j = res
                multi = torch.zeros((m, F), dtype=torch.bool, device=Hn.device)
                if cfg.kind in ("infogain", "infogainratio") and anycat:
                    Hv = Hn[:, :, :B - 1, :]
                    mg = self._multiway_gain(Hv, Hn[:, :, B - 1, :], Hv.sum(2))
                    catf = is_cat[None, :].expand(m, F)
                    best_j_gain = torch.where(catf, mg, best_j_gain)
                    multi = catf.clone()
                return best_j_gain, best_j, multi, None
        Hv = Hn[:, :, :B - 1, :]
        Hmiss = Hn[:, :, B - 1, :]
        cnt = _count(cfg, Hv)
        # ordering key for categorical bins (continuous: identity)
        binpos = torch.arange(B - 1, device=Hn.device, dtype=Hn.dtype).expand(m, F, B - 1)
        if cfg.kind == "gbdt":
            g, h = Hv[..., 1], Hv[..., 2]
            key = torch.where(h < 1e-6, torch.full_like(g, -1.0), g / torch.where(h < 1e-6, torch.ones_like(h), h))
        elif cfg.kind == "mse":
            w = Hv[..., 0]
            key = torch.where(cnt > 0, Hv[..., 1] / torch.where(w == 0, torch.ones_like(w), w),
                              torch.full_like(w, float("inf")))
        else:
            w = _weight(cfg, Hv)
            key = torch.where(cnt > 0, Hv[..., 0] / torch.where(w == 0, torch.ones_like(w), w),
                              torch.full_like(w, float("inf")))
        iscat = is_cat[None, :, None].expand(m, F, B - 1)
        key = torch.where(iscat, key, binpos)
        key, perm = torch.sort(key, dim=2, stable=True)
        Hs = torch.gather(Hv, 2, perm[..., None].expand(m, F, B - 1, S))
        L = torch.cumsum(Hs, dim=2)
        Tv = L[:, :, -1, :]
        if cfg.kind == "gbdt":
            T = Tv + Hmiss
            R = T[:, :, None, :] - L
            gain = _binary_gain(cfg, T[:, :, None, :].expand_as(L), L, R)
            HT = T[..., 2][:, :, None]
            HL, HR = L[..., 2], T[..., 2][:, :, None] - L[..., 2]
            cT = _count(cfg, T)[:, :, None]
            cL = _count(cfg, L)
            ratio = HL / torch.where(HT < 1e-6, torch.ones_like(HT), HT)
            ok = (HT >= 1e-6) & (ratio >= 1e-7) & (ratio <= 1.0 - 1e-7)
            ok &= (cL >= cfg.min_samples_per_leaf) & (cT - cL >= cfg.min_samples_per_leaf)
            ok &= (HL >= cfg.min_sum_hessian_per_leaf) & (HR >= cfg.min_sum_hessian_per_leaf)
        else:
            R = Tv[:, :, None, :] - L
            gain = _binary_gain(cfg, Tv[:, :, None, :].expand_as(L), L, R)
            cM = _count(cfg, Hmiss)[:, :, None]
            cL, cR = _count(cfg, L), _count(cfg, R)
            cT = cL + cR
            ok = (cL > 0) & (cR > 0)
            ok &= (cfg.min_samples_per_leaf <= cL + cM) & (cfg.min_samples_per_leaf <= cR + cM)
            den = cT + cM
            den = torch.where(den == 0, torch.ones_like(den), den)
            ok &= (cfg.min_sample_ratio_per_child <= (cL + cM) / den)
            ok &= (cfg.min_sample_ratio_per_child <= (cR + cM) / den)
            # a categorical candidate is evaluated only right after a non-empty category joins the left side
            sorted_cnt = torch.gather(cnt, 2, perm)
            ok &= ~iscat | (sorted_cnt > 0)
            ok &= (gain > 0) & (gain >= cfg.min_info_gain)
        gain = torch.where(ok, gain, torch.full_like(gain, NEG))
        best_j_gain, best_j = gain.max(dim=2)       # first max along bins
        multi = torch.zeros((m, F), dtype=torch.bool, device=Hn.device)
        if cfg.kind in ("infogain", "infogainratio") and anycat:
            mg = self._multiway_gain(Hv, Hmiss, Tv)
            catf = is_cat[None, :].expand(m, F)
            best_j_gain = torch.where(catf, mg, best_j_gain)
            multi = catf.clone()
        return best_j_gain, best_j, multi, perm

    def _feature_gains_gbdt(self, Hn):
        """Per-(node, feature) best gain and bin of GBDT binary splits on continuous features: K8 on the GPU,
        the same scan in torch elsewhere.  Hn [m, Fx, B, S] -> (gain [m, Fx] float64, best_j [m, Fx])."""
        cfg = self.cfg
        m, Fx, B, S = Hn.shape
        if Hn.is_cuda and tops.gpu_kernels_ok():
            gain, best_j = tops.gbdt_split(Hn.to(torch.float32), cfg.min_samples_per_leaf,
                                           cfg.min_sum_hessian_per_leaf)
            return gain.to(torch.float64), best_j.to(torch.int64)
        Hv = Hn[:, :, :B - 1, :]
        Hmiss = Hn[:, :, B - 1, :]
        L = torch.cumsum(Hv, dim=2)
        T = L[:, :, -1, :] + Hmiss
        R = T[:, :, None, :] - L
        gain = _binary_gain(cfg, T[:, :, None, :].expand_as(L), L, R)
        HT = T[..., 2][:, :, None]
        HL, HR = L[..., 2], T[..., 2][:, :, None] - L[..., 2]
        cT = _count(cfg, T)[:, :, None]
        cL = _count(cfg, L)
        ratio = HL / torch.where(HT < 1e-6, torch.ones_like(HT), HT)
        ok = (HT >= 1e-6) & (ratio >= 1e-7) & (ratio <= 1.0 - 1e-7)
        ok &= (cL >= cfg.min_samples_per_leaf) & (cT - cL >= cfg.min_samples_per_leaf)
        ok &= (HL >= cfg.min_sum_hessian_per_leaf) & (HR >= cfg.min_sum_hessian_per_leaf)
        gain = torch.where(ok, gain, torch.full_like(gain, NEG))
        g, j = gain.max(dim=2)
        return g, j

    SHARDED_SEARCHES = 0

    def _search_sharded(self, Hn, feat_order, feat_ok):
        """Feature-sharded split search (reference ``CalBestSplit.java:122-153`` / ``TreeObj.java:321-390``: each
        task searches the features it owns): this rank scans its feature block — any criterion, categorical
        features included (their bin order is per (node, feature), so local to the owner) — the [m, Fb] best
        gains / positions / multi-way flags of all blocks are all-gathered (small), and every rank picks the same
        best feature per node in ``feat_order`` (identical tie-breaking to the replicated search).  Returns also
        the chosen features' [m, B, S] histogram rows, all-reduced from their owners."""
        m = Hn.shape[0]
        ws = comm.get_world_size()
        TreeBuilder.SHARDED_SEARCHES += 1
        g_loc, j_loc, multi_loc, perm_loc = self._feature_best(Hn, self.is_cat_local)   # [m, Fb]
        packed = torch.stack([g_loc.to(torch.float64), j_loc.to(torch.float64), multi_loc.to(torch.float64)], 0)
        allp = comm.all_gather_tensor(packed.contiguous().reshape(1, 3, m, self.Fb).to(comm.collective_device()))
        allp = allp.to(Hn.device).reshape(ws, 3, m, self.Fb).permute(1, 2, 0, 3).reshape(3, m, ws * self.Fb)
        gain, best_j = allp[0][:, :self.F], allp[1][:, :self.F].to(torch.int64)
        multi = allp[2][:, :self.F] > 0.5
        gbest, fbest, jbest, mbest, accept = self._choose(gain, best_j, multi, feat_order, feat_ok)
        # chosen feature's histogram row per node: owners contribute, everyone else adds zeros
        loc = fbest - self.f_lo
        mine = (loc >= 0) & (loc < self.Fb)
        B = Hn.shape[2]
        # the owner's bin order of the chosen feature travels with its row when the torch scan produced one (the
        # GPU kernels' order is rebuilt on the host from the row instead, like the replicated search)
        width = B * Hn.shape[3] + (B - 1 if perm_loc is not None else 0)
        rows = torch.zeros((m, width), dtype=torch.float64, device=Hn.device)
        if bool(mine.any()):
            idx = torch.nonzero(mine).reshape(-1)
            rows[idx, :B * Hn.shape[3]] = Hn[idx, loc[idx]].to(torch.float64).reshape(idx.numel(), -1)
            if perm_loc is not None:
                rows[idx, B * Hn.shape[3]:] = perm_loc[idx, loc[idx]].to(torch.float64)
        comm.all_reduce(rows, "sum")
        hist_rows = rows[:, :B * Hn.shape[3]].reshape((m,) + tuple(Hn.shape[2:]))
        perm_rows = rows[:, B * Hn.shape[3]:].to(torch.int64) if perm_loc is not None else None
        return gbest, fbest, jbest, mbest, accept, hist_rows, perm_rows

    def _multiway_gain(self, Hv, Hmiss, Tv):
        """C4.5 split on every non-empty category (``CategoricalSplitter.bestSplitInfo``)."""
        cfg = self.cfg
        cnt = _count(cfg, Hv)
        w = _weight(cfg, Hv)
        nonempty = (cnt > 0) & (w != 0)
        wT = _weight(cfg, Tv)
        safe = torch.where(wT < EPS, torch.ones_like(wT), wT)
        p = w / safe[..., None]
        g = _impurity(cfg, Tv) - (torch.where(nonempty, p * _impurity(cfg, Hv), torch.zeros_like(p))).sum(-1)
        if cfg.kind == "infogainratio":
            lg = torch.where(p > 0, torch.log(torch.where(p > 0, p, torch.ones_like(p))) / math.log(2.0),
                             torch.zeros_like(p))
            iv = -(torch.where(nonempty, p * lg, torch.zeros_like(p))).sum(-1)
            g = torch.where(iv < EPS, torch.zeros_like(g), g / torch.where(iv < EPS, torch.ones_like(iv), iv))
        cM = _count(cfg, Hmiss)
        cT = cnt.sum(-1)
        bad = nonempty & ((cfg.min_samples_per_leaf > cnt + cM[..., None])
                          | (cfg.min_sample_ratio_per_child > (cnt + cM[..., None])
                             / torch.where(cT + cM == 0, torch.ones_like(cT), cT + cM)[..., None]))
        nchild = nonempty.sum(-1)
        ok = (~bad.any(-1)) & (nchild >= 2) & (wT >= EPS) & (g > 0) & (g >= cfg.min_info_gain)
        return torch.where(ok, g, torch.full_like(g, NEG))

    # -------------------------------------------------------------------------------------------
    def _materialise(self, Hn_np_feat: np.ndarray, f: int, j: int, multi: bool, perm_row: np.ndarray,
                     gain: float) -> _Split:
        """Host-side split description from the chosen feature's [B, S] histogram row."""
        cfg, B = self.cfg, self.B
        h = Hn_np_feat                      # [B, S]
        cnt = h[:, -1]
        nb = self.d.nbins[f]
        route = np.zeros(256, dtype=np.int64)
        categorical, threshold = None, 0.0
        if multi:
            cats = [c for c in range(nb) if cnt[c] > 0 and self._w_np(h[c]) != 0]
            k = len(cats)
            child = {c: i for i, c in enumerate(cats)}
            categorical = [child.get(c, -1) for c in range(nb)]
            totals = np.stack([h[c] for c in cats])
            big = int(np.argmax(totals[:, -1]))
            for b in range(256):
                route[b] = child.get(b, big)
        else:
            k = 2
            if self.d.is_cat[f]:
                left = set(int(x) for x in perm_row[:j + 1])
                if cfg.kind == "gbdt":
                    categorical = [0 if c in left else 1 for c in range(nb)]
                else:
                    categorical = [(-1 if cnt[c] <= 0 else (0 if c in left else 1)) for c in range(nb)]
                inl = np.array([b in left for b in range(B - 1)])
            else:
                inl = np.arange(B - 1) <= j
                vals = self.d.bin_values[f] if self.d.bin_values else None
                if cfg.kind != "gbdt" and vals is not None:
                    nz = np.nonzero(cnt[:B - 1] > 0)[0]
                    nxt = nz[nz > j]
                    hi = vals[nxt[0]] if nxt.size else vals[min(j + 1, len(vals) - 1)]
                    threshold = float((vals[j] + hi) / 2.0)
                else:
                    threshold = float(self.d.thresholds[f][j]) if j < len(self.d.thresholds[f]) else float("inf")
            lt = h[:B - 1][inl].sum(0)
            rt = h[:B - 1][~inl].sum(0)
            totals = np.stack([lt, rt])
            route[:B - 1] = np.where(inl, 0, 1)
            route[B - 1:] = 1
        # missing bin (and bins no training row used): GBDT right; otherwise the heavier child
        miss = h[B - 1]
        if cfg.kind == "gbdt":
            mchild = 1 if not multi else int(np.argmax(totals[:, -1]))
        else:
            mchild = int(np.argmax(totals[:, -1]))
            if not multi and self.d.is_cat[f]:
                for c in range(nb):
                    if cnt[c] <= 0:
                        route[c] = mchild
        route[B - 1] = mchild
        totals = totals.copy()
        totals[mchild] += miss
        return _Split(f, gain, route, k, totals, categorical, threshold)

    def _w_np(self, x):
        cfg = self.cfg
        if cfg.classification:
            return float(x[:cfg.n_classes].sum())
        return float(x[0] if cfg.kind == "mse" else x[2])

    # -------------------------------------------------------------------------------------------
    def _counter(self, total: np.ndarray) -> LabelCounter:
        cfg = self.cfg
        if cfg.kind == "gbdt":
            return LabelCounter(total[2], int(round(total[3])), [-total[1] * cfg.learning_rate, total[0]])
        if cfg.kind == "mse":
            return LabelCounter(total[0], int(round(total[3])), [total[1], total[2]])
        return LabelCounter(float(total[:cfg.n_classes].sum()), int(round(total[-1])),
                            [float(x) for x in total[:cfg.n_classes]])

    def _node_splittable(self, p: _Pending) -> bool:
        cfg = self.cfg
        if p.depth >= cfg.max_depth:
            return False
        if cfg.kind != "gbdt" and p.total[-1] <= cfg.min_samples_per_leaf:
            return False
        return p.total[-1] > 0

    def _node_batch(self, nl: int, S: int) -> Tuple[int, bool]:
        """(nodes per histogram pass / split search, park the level's histograms on the host) under
        ``cfg.max_memory_bytes`` — the reference's loop buffer (TreeObj.determineLoopNode: as many node
        histograms as fit maxMemoryInMB, at least one)."""
        budget = self.cfg.max_memory_bytes
        if budget is None:
            return max(1, nl), False
        per = self.Fb * self.B * S * (4 if self.dev.type == "cuda" else 8)
        return max(1, int(budget // max(1, per))), nl * per > budget

    def _search_batch(self, level, cand, Hn, fmask, bagging) -> dict:
        """Best splits of the candidate nodes ``cand`` (level indices) from their histograms ``Hn`` [m, F, B, S]
        (device): {level index: _Split} for the accepted ones."""
        cfg, F, B, dev = self.cfg, self.F, self.B, self.dev
        Hn = Hn.to(torch.float32).to(torch.float64)
        m = len(cand)
        order = torch.arange(F, device=dev).expand(m, F).clone()
        ok = fmask[None, :].expand(m, F).clone()
        if bagging:
            # the batch's scan orders and admitted features in one host->device copy each
            k = cfg.node_feature_count or F
            ord_np = np.stack([np.asarray(level[i].order, dtype=np.int64) for i in cand])
            ok_np = np.zeros((m, F), dtype=bool)
            np.put_along_axis(ok_np, ord_np[:, :k], True, axis=1)
            order = torch.from_numpy(ord_np).to(dev)
            ok = torch.from_numpy(ok_np).to(dev)
        if self.fshard:
            gbest, fbest, jbest, mbest, accept, rows_t, prow = self._search_sharded(Hn, order, ok)
            rows_host = rows_t.cpu().numpy()                                     # [m, B, S]
            perm = None if prow is None else prow[:, None, :].expand(m, F, B - 1)
        else:
            gbest, fbest, jbest, mbest, accept, perm = self._search(Hn, order, ok)
            rows_host = Hn[torch.arange(m, device=dev), fbest].cpu().numpy()      # [m, B, S]
        if perm is None:                     # GPU / sharded search: rebuild the chosen features' order
            fb_np = fbest.cpu().numpy()
            perm_host = np.stack([tops.split_order_key(rows_host[r_], cfg.kind, cfg.n_classes,
                                                       bool(self.d.is_cat[int(fb_np[r_])]))
                                  for r_ in range(m)]) if m else np.zeros((0, B - 1), np.int64)
        else:
            perm_host = perm[torch.arange(m, device=dev), fbest].cpu().numpy()    # [m, B-1]
        acc = accept.cpu().numpy()
        fb, jb, mb, gb = (fbest.cpu().numpy(), jbest.cpu().numpy(), mbest.cpu().numpy(), gbest.cpu().numpy())
        out = {}
        # binary threshold splits of continuous features: every accepted node of the batch at once
        vec = acc.astype(bool) & ~mb.astype(bool) & ~np.asarray(self.d.is_cat, dtype=bool)[fb]
        out.update(self._materialise_cont(rows_host, fb, jb, gb, [i for r_, i in enumerate(cand) if vec[r_]],
                                          np.nonzero(vec)[0]))
        for r_, i in enumerate(cand):
            if acc[r_] and not vec[r_]:
                out[i] = self._materialise(rows_host[r_], int(fb[r_]), int(jb[r_]), bool(mb[r_]), perm_host[r_],
                                           float(gb[r_]))
        return out

    def _materialise_cont(self, rows_host, fb, jb, gb, ids, rsel) -> dict:
        """``_materialise`` of binary threshold splits on continuous features for many nodes in numpy: left =
        bins <= j; the missing bin goes right (GBDT) or to the heavier child; the threshold is the training
        threshold (GBDT) or the midpoint to the next used bin value (the other criteria); child totals as
        sequential row sums (the same order as one node at a time)."""
        if len(ids) == 0:
            return {}
        cfg, B = self.cfg, self.B
        h = rows_host[rsel]                                   # [m, B, S]
        j = jb[rsel].astype(np.int64)
        b = np.arange(B - 1)
        inl = b[None, :] <= j[:, None]                        # [m, B-1]
        hv = h[:, :B - 1]
        lt = np.cumsum(np.where(inl[..., None], hv, 0.0), axis=1)[:, -1]
        rt = np.cumsum(np.where(inl[..., None], 0.0, hv), axis=1)[:, -1]
        miss = h[:, B - 1]
        if cfg.kind == "gbdt":
            mchild = np.ones(len(ids), dtype=np.int64)
        else:
            mchild = (rt[:, -1] > lt[:, -1]).astype(np.int64)     # np.argmax of the two counts (ties -> 0)
        lt = lt + np.where(mchild[:, None] == 0, miss, 0.0)
        rt = rt + np.where(mchild[:, None] == 1, miss, 0.0)
        route = np.ones((len(ids), 256), dtype=np.int64)
        route[:, :B - 1] = np.where(inl, 0, 1)
        route[:, B - 1] = mchild
        vals_all = self.d.bin_values if (cfg.kind != "gbdt" and self.d.bin_values) else None
        if vals_all is not None:
            used = (hv[:, :, -1] > 0) & ~inl                  # used bins right of the split
            has = used.any(1)
            nxt = np.argmax(used, 1)
        out = {}
        thr = self.d.thresholds
        for k, i in enumerate(ids):
            f, jj = int(fb[rsel[k]]), int(j[k])
            vals = vals_all[f] if vals_all is not None else None
            if vals is not None:
                hi = vals[nxt[k]] if has[k] else vals[min(jj + 1, len(vals) - 1)]
                t = float((vals[jj] + hi) / 2.0)
            else:
                t = float(thr[f][jj]) if jj < len(thr[f]) else float("inf")
            out[i] = _Split(f, float(gb[rsel[k]]), route[k], 2, np.stack([lt[k], rt[k]]), None, t)
        return out

    def _derive_batched(self, derive: dict, hist: dict, dev) -> None:
        """Sibling subtraction for every derived node of a level in a few launches: the parents' histograms
        stacked, minus the k-th built sibling of every node in round k (the same fp32 subtraction order as one
        node at a time, so bitwise the same histograms)."""
        if not derive:
            return
        bigs = list(derive)
        H = torch.stack([self._prev_hist[derive[b][0]].to(dev) for b in bigs])
        for k in range(max(len(derive[b][1]) for b in bigs)):
            rows = [r for r, b in enumerate(bigs) if len(derive[b][1]) > k]
            sib = torch.stack([hist[derive[bigs[r]][1][k]] for r in rows])
            if len(rows) == len(bigs):
                H -= sib
            else:
                ri = torch.as_tensor(rows, dtype=torch.long, device=dev)
                H[ri] = H[ri] - sib
        for r, b in enumerate(bigs):
            hist[b] = H[r]

    def _level_parked(self, level, node_of_row, sample, stats, build_ids, derive, mbatch, fmask, bagging):
        """A level whose histograms exceed the memory budget, one node batch at a time: the batch's built
        histograms, its derived ones (parent parked on the host from the previous level, minus the siblings
        built in the same batch: batches are whole sibling groups), the split search, and the park of the
        accepted nodes' histograms (the next level's parents) to the host in ONE copy.  Returns (splits, parked
        histograms {level index: host tensor})."""
        dev, nl = self.dev, len(level)
        built = set(build_ids)
        # whole sibling groups (contiguous in BFS order), packed up to mbatch histograms per batch
        groups, cur = [], []
        for i in range(nl):
            if cur and level[i].parent != level[cur[-1]].parent:
                groups.append(cur)
                cur = []
            cur.append(i)
        if cur:
            groups.append(cur)
        batches, cur, cnt = [], [], 0
        for gr in groups:
            k = sum(1 for i in gr if i in built or i in derive)
            if cur and cnt + k > mbatch:
                batches.append(cur)
                cur, cnt = [], 0
            cur.extend(gr)
            cnt += k
        if cur:
            batches.append(cur)
        splits, parked = {}, {}
        for batch in batches:
            bids = [i for i in batch if i in built]
            hb = {}
            if bids:
                som = torch.full((nl,), -1, dtype=torch.int32)
                for s_, i in enumerate(bids):
                    som[i] = s_
                H = self._histograms(node_of_row, sample, som.to(dev), len(bids), stats, bids)
                for s_, i in enumerate(bids):
                    hb[i] = H[s_]
            self._derive_batched({b: derive[b] for b in batch if b in derive}, hb, dev)
            cand = [i for i in batch if level[i].splittable]
            if cand:
                got = self._search_batch(level, cand, torch.stack([hb[i] for i in cand]), fmask, bagging)
                splits.update(got)
                keep = [i for i in cand if i in got]
                if keep:
                    Hk = torch.stack([hb[i] for i in keep]).cpu()
                    for s_, i in enumerate(keep):
                        parked[i] = Hk[s_]
            del hb
        return splits, parked

    def build(self, stats: torch.Tensor, sample: torch.Tensor, feature_mask: Optional[np.ndarray] = None,
              rng=None) -> Tuple[Node, torch.Tensor, List[Node]]:
        """Grow one tree.  ``stats`` [n, S] per-row statistics, ``sample`` [n] rows that count.
        ``rng`` (a ``JavaRandom``) enables RF per-node feature bagging.
        Returns (root, leaf code per row (-1-k for leaf k; rows outside the tree keep their code), leaves)."""
        cfg, F, B = self.cfg, self.F, self.B
        n = self.d.bins.shape[0]
        dev = self.dev
        stats = stats.to(self.hist_dtype if stats.is_cuda else torch.float64).contiguous()
        node_of_row = torch.zeros(n, dtype=torch.int32, device=dev)
        if cfg.kind != "gbdt":
            node_of_row = torch.where(sample, node_of_row, torch.full_like(node_of_row, -(1 << 30)))
        fmask = torch.ones(F, dtype=torch.bool, device=dev) if feature_mask is None else \
            torch.as_tensor(feature_mask, dtype=torch.bool, device=dev)
        leaves: List[Node] = []
        # root statistics from a 1-slot histogram
        self._tro, self._level_no = None, 0
        Hroot = self._histograms(node_of_row, sample, torch.zeros(1, dtype=torch.int32, device=dev), 1, stats, [0])
        root_total = self._node_totals(node_of_row, sample, 1, stats)[0]
        root = Node(counter=self._counter(root_total))
        bagging = cfg.kind != "gbdt" and rng is not None
        level = [_Pending(root, 1, root_total, order=list(range(F)))]
        level_hist = {0: Hroot[0]}
        while level:
            nl = len(level)
            t_level = time.perf_counter()
            self._level_no += 1
            for p in level:
                p.splittable = self._node_splittable(p)
            if bagging:
                # every polled node shuffles its inherited splitter order (DecisionTree.bagging), in BFS order:
                # the whole level in one host C++ call (the same java.util.Random draws, node after node)
                orders = rng.shuffle_rows(np.asarray([p.order for p in level], dtype=np.int32))
                for p, o in zip(level, orders):
                    p.order = o
            # which nodes need a histogram built vs derived from the parent
            build_ids, derive = [], {}
            parked = None
            if all(k in level_hist for k in range(nl)):
                pass
            else:
                groups = {}
                for i, p in enumerate(level):
                    groups.setdefault(p.parent, []).append(i)
                for par, ids in groups.items():
                    need = [i for i in ids if level[i].splittable]
                    if not need:
                        continue
                    big = max(ids, key=lambda i: (level[i].total[-1], -i))
                    if big in need and len(ids) >= 2 and par in self._prev_hist:
                        derive[big] = (par, [i for i in ids if i != big])
                        build_ids.extend(i for i in ids if i != big)
                    else:
                        build_ids.extend(need)
                build_ids = sorted(set(build_ids))
                # memory bound: one histogram pass holds at most `mbatch` nodes; a level whose histograms exceed
                # the budget runs batch by batch (build, derive, search) and parks only its accepted nodes'
                # histograms (the next level's parents) in host memory
                mbatch, park = self._node_batch(nl, stats.shape[1])
                if park:
                    parked, level_hist = self._level_parked(level, node_of_row, sample, stats, build_ids, derive,
                                                            mbatch, fmask, bagging)
                else:
                    for c0 in range(0, len(build_ids), mbatch):
                        chunk = build_ids[c0:c0 + mbatch]
                        som = torch.full((nl,), -1, dtype=torch.int32)
                        for s, i in enumerate(chunk):
                            som[i] = s
                        H = self._histograms(node_of_row, sample, som.to(dev), len(chunk), stats, chunk)
                        for s, i in enumerate(chunk):
                            level_hist[i] = H[s]
                        del H
                    self._derive_batched(derive, level_hist, dev)
            cand_all = [i for i in range(nl) if level[i].splittable]
            if parked is not None:
                splits = parked
            else:
                splits = {}
                mbatch = self._node_batch(nl, stats.shape[1])[0]
                for c0 in range(0, len(cand_all), mbatch):
                    cand = cand_all[c0:c0 + mbatch]
                    Hn = torch.stack([level_hist[i] for i in cand]).to(dev)
                    splits.update(self._search_batch(level, cand, Hn, fmask, bagging))
            # finalize nodes in BFS order; children form the next level
            nxt: List[_Pending] = []
            feat = np.full(nl, -1, dtype=np.int32)
            base = np.zeros(nl, dtype=np.int32)
            route = np.zeros((nl, 256), dtype=np.int16)
            for i, p in enumerate(level):
                sp = splits.get(i)
                if sp is not None and cfg.kind != "gbdt":
                    queue_size = (nl - i - 1) + len(nxt)
                    if queue_size + sp.n_children >= cfg.max_leaves:
                        sp = None
                if sp is None:
                    code = len(leaves)
                    leaves.append(p.node)
                    feat[i] = -1
                    base[i] = -1 - code
                    continue
                nd = p.node
                nd.featureIndex = sp.feature
                if cfg.kind != "gbdt":
                    nd.gain = sp.gain
                if sp.categorical is not None:
                    nd.categoricalSplit = [int(x) for x in sp.categorical]
                else:
                    nd.continuousSplit = sp.threshold
                feat[i] = sp.feature
                base[i] = len(nxt)
                route[i] = sp.route
                for c in range(sp.n_children):
                    child = Node(counter=self._counter(sp.child_totals[c]))
                    nd.nextNodes.append(child)
                    nxt.append(_Pending(child, p.depth + 1, sp.child_totals[c], parent=i, order=p.order))
            node_of_row = tops.route(self.d.bins, node_of_row, torch.as_tensor(feat, device=dev),
                                     torch.as_tensor(base, device=dev), torch.as_tensor(route, device=dev))
            if nxt:
                # exact child statistics (all S columns, missing rows where they were routed)
                tot = self._node_totals(node_of_row, sample, len(nxt), stats)
                for c, q in enumerate(nxt):
                    q.total = tot[c]
                    q.node.counter = self._counter(tot[c])
            self._prev_hist = level_hist
            level_hist = {}
            TreeBuilder.LEVEL_STATS.append((level[0].depth if level else 0, nl, len(cand_all),
                                            time.perf_counter() - t_level))
            level = nxt
        self._prev_hist = {}
        self._hist_sub = None
        self._tro = None
        # leaf probabilities (split nodes keep raw counters)
        for lf in leaves:
            lf.make_leaf_prob()
        if cfg.kind == "gbdt" and root.featureIndex >= 0:
            root.counter = LabelCounter(0.0, 0, [0.0, 0.0])
        return root, node_of_row, leaves

    _prev_hist: dict = {}
    _tro = None
    _level_no = 0
