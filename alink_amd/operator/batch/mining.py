"""Association rules, sequential patterns, outlier selection and LSH similarity batch ops.

Reference: ``A/operator/batch/associationrule/{FpGrowthBatchOp,PrefixSpanBatchOp}.java`` (output = patterns,
side output 0 = rules), ``A/operator/batch/outlier/SosBatchOp.java``,
``A/operator/batch/similarity/{ApproxVectorSimilarityJoinLSHBatchOp,ApproxVectorSimilarityTopNLSHBatchOp}.java``.
"""
from __future__ import annotations

import numpy as np
import torch

from ...common.linalg import VectorUtil
from ...common.table import Column, MTable
from ...common.types import TableSchema, Types
from ...models.associationrule import mining as M
from ...models.outlier.sos import sos_scores
from ...models.similarity import lsh as L
from ...parallel import comm
from ..base import BatchOperator, gather_table, partition_bounds

__all__ = ["FpGrowthBatchOp", "PrefixSpanBatchOp", "SosBatchOp", "ApproxVectorSimilarityJoinLSHBatchOp",
           "ApproxVectorSimilarityTopNLSHBatchOp"]

ITEM_SEP, ELEMENT_SEP, RULE_SEP = ",", ";", "=>"


def _own_block(rows, schema, env, replicated_in):
    mt = MTable.from_rows(rows, schema)
    if comm.get_world_size() > 1 and not replicated_in:
        lo, hi = partition_bounds(mt.num_rows, env)
        mt = mt.slice(lo, hi)
    return mt


class FpGrowthBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.resolvedParams()
        items = mt.col(p.get("itemsCol")).to_list()
        tx = [s.split(ITEM_SEP) if s is not None and s.strip() else [] for s in items]
        names, pats, n, _ = M.fp_growth(tx, int(p.get("minSupportCount")), float(p.get("minSupportPercent")),
                                        int(p.get("maxPatternLength")))
        order = sorted(pats, key=lambda t: (len(t), t))
        prow = [(ITEM_SEP.join(names[i] for i in pat), int(pats[pat]), len(pat)) for pat in order]
        rules = M.association_rules(pats, n, float(p.get("minConfidence")), float(p.get("minLift")),
                                    int(p.get("maxConsequentLength")))
        rules.sort(key=lambda r: (len(r[0]) + len(r[1]), r[0], r[1]))
        rrow = [(ITEM_SEP.join(names[i] for i in a) + RULE_SEP + ITEM_SEP.join(names[i] for i in c), len(a) + len(c),
                 float(lift), float(sup), float(conf), int(cnt)) for a, c, cnt, lift, sup, conf in rules]
        rep = mt.replicated
        self.setOutputTable(_own_block(prow, "itemset string, supportcount bigint, itemcount bigint", self.env, rep))
        self.setSideOutputTables([_own_block(
            rrow, "rule string, itemcount bigint, lift double, support_percent double, confidence_percent double, "
                  "transaction_count bigint", self.env, rep)])
        return self


def _encode_seq(names, elements) -> str:
    return ELEMENT_SEP.join(ITEM_SEP.join(names[i] for i in el) for el in elements)


class PrefixSpanBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.resolvedParams()
        seqs = []
        for s in mt.col(p.get("itemsCol")).to_list():
            if s is None or not s.strip():
                seqs.append([])
                continue
            seqs.append([el.strip().split(ITEM_SEP) for el in s.split(ELEMENT_SEP)])
        names, pats, n = M.prefix_span(seqs, int(p.get("minSupportCount")), float(p.get("minSupportPercent")),
                                       int(p.get("maxPatternLength")))
        order = sorted(pats, key=lambda t: (sum(len(e) for e in t), t))
        prow = [(_encode_seq(names, pat), int(pats[pat]), sum(len(e) for e in pat)) for pat in order]
        rules = M.sequence_rules(pats, n, float(p.get("minConfidence")))
        rules.sort(key=lambda r: (len(r[0]) + 1, r[0], r[1]))
        rrow = [(_encode_seq(names, a) + RULE_SEP + _encode_seq(names, c), len(a) + len(c), float(sup), float(conf),
                 int(cnt)) for a, c, cnt, sup, conf in rules]
        rep = mt.replicated
        self.setOutputTable(_own_block(prow, "itemset string, supportcount bigint, itemcount bigint", self.env, rep))
        self.setSideOutputTables([_own_block(
            rrow, "rule string, chain_length bigint, support double, confidence double, transaction_count bigint",
            self.env, rep)])
        return self


def _dense_block(values, device) -> torch.Tensor:
    vecs = [VectorUtil.getVector(v) for v in values]
    d = max((v.size() for v in vecs), default=0)
    X = np.zeros((len(vecs), d))
    for i, v in enumerate(vecs):
        X[i] = v.toDense().getData()[:d] if v.size() == d else np.pad(v.toDense().getData(), (0, d - v.size()))
    return torch.as_tensor(X, device=device)


class SosBatchOp(BatchOperator):
    """Outlier probability per row; the n x n affinity work is split by row blocks across ranks and the
    per-column log-products are all-reduced."""

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.resolvedParams()
        full = gather_table(mt)
        X = _dense_block(full.col(p.get("vectorCol")).to_list(), self.env.device)
        scores = sos_scores(X, float(p.get("perplexity")))
        lo, hi = (0, full.num_rows) if mt.replicated or comm.get_world_size() == 1 else \
            partition_bounds(full.num_rows, self.env)
        own = full.slice(lo, hi) if (lo, hi) != (0, full.num_rows) else full
        out = own.with_columns([p.get("predictionCol")], [Types.DOUBLE], [Column(scores[lo:hi].cpu())])
        # each rank keeps its own row block of the gathered table: a partitioned output (collect gathers it)
        out.replicated = bool(mt.replicated or comm.get_world_size() == 1)
        self.setOutputTable(out)
        return self


def _lsh_args(p):
    dt = p.get("distanceType")
    return (getattr(dt, "name", str(dt)), int(p.get("seed")), int(p.get("numProjectionsPerTable")),
            int(p.get("numHashTables")), float(p.get("projectionWidth")))


class ApproxVectorSimilarityJoinLSHBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        self.checkOpSize(2, inputs)
        p = self.resolvedParams()
        left, right = gather_table(inputs[0].getOutputTable()), gather_table(inputs[1].getOutputTable())
        lid, rid = p.get("leftIdCol"), p.get("rightIdCol")
        res = L.approx_similarity_join(left.col(p.get("leftCol")).to_list(), right.col(p.get("rightCol")).to_list(),
                                       *_lsh_args(p), float(p.get("distanceThreshold")), self.env.device)
        lids, rids = left.col(lid).to_list(), right.col(rid).to_list()
        ln, rn = (lid + "_left", rid + "_right") if lid.lower() == rid.lower() else (lid, rid)
        dcol = p.get("outputCol") if p.contains("outputCol") and p.get("outputCol") else "distance"
        schema = TableSchema([ln, rn, dcol], [left.col_type(lid), right.col_type(rid), Types.DOUBLE])
        rows = [(lids[a], rids[b], d) for a, b, d in res]
        self.setOutputTable(_own_block(rows, schema, self.env, False))
        return self


class ApproxVectorSimilarityTopNLSHBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        self.checkOpSize(2, inputs)
        p = self.resolvedParams()
        left, right = gather_table(inputs[0].getOutputTable()), gather_table(inputs[1].getOutputTable())
        lid, rid = p.get("leftIdCol"), p.get("rightIdCol")
        lv = left.col(p.get("leftCol")).to_list()
        res = L.approx_nearest_neighbors(right.col(p.get("rightCol")).to_list(), lv, *_lsh_args(p),
                                         int(p.get("topN")), self.env.device, lsh_basis_vecs=lv)
        lids, rids = left.col(lid).to_list(), right.col(rid).to_list()
        ln, rn = (lid + "_left", rid + "_right") if lid.lower() == rid.lower() else (lid, rid)
        dcol = p.get("outputCol") if p.contains("outputCol") and p.get("outputCol") else "distance"
        schema = TableSchema([rn, ln, dcol, "rank"], [right.col_type(rid), left.col_type(lid), Types.DOUBLE,
                                                     Types.LONG])
        rows = [(rids[q], lids[d], dist, rank) for q, d, dist, rank in res]
        self.setOutputTable(_own_block(rows, schema, self.env, False))
        return self
