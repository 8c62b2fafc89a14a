"""Isotonic regression: parallel pool-adjacent-violators (PAV).

Reference: ``A/operator/batch/regression/IsotonicRegTrainBatchOp.java`` (``partitionByRange`` + per-partition
``PoolAdjacentViolators`` :167-181 + a final merge of all partitions' blocks :115-162, blocks stored as
``(float labelSum, double start, double end, float weight)`` in ``isotonicReg/LinkedData.java:28-32``),
``IsotonicRegressionModelMapper.java`` (binary search + linear interpolation), ``IsotonicRegressionConverter``.

Rows are range-partitioned by feature with the distributed sample sort (``parallel/sort.py``), every rank pools
its sorted range, the (small) block lists are all-gathered in range order and pooled once more — the same
two-level scheme as the reference, without funnelling the data through one task.  Label sums and weights are
kept in float32 exactly like the reference's LinkedData, so model values match it bit for bit.
"""
from __future__ import annotations

import bisect
import json
from typing import List, Tuple

import numpy as np
import torch

from ...common.javafmt import gson_dumps
from ...common.linalg import VectorUtil
from ...common.mapper import ModelMapper, OutputColsHelper
from ...common.model import SimpleModelDataConverter
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import Types
from ...parallel import comm
from ...parallel.sort import sample_sort

__all__ = ["train_isotonic", "IsotonicRegressionModelData", "IsotonicRegressionConverter",
           "IsotonicRegressionModelMapper", "pav_blocks"]

Block = Tuple[np.float32, float, float, np.float32]


def pav_blocks(blocks: List[Block]) -> List[Block]:
    """``updateLinkedData``: merge adjacent blocks while mean(prev) >= mean(cur) (float32 sums)."""
    out: List[Block] = []
    for b in blocks:
        out.append(b)
        while len(out) >= 2:
            pl, ps, pe, pw = out[-2]
            cl, cs, ce, cw = out[-1]
            if float(pl) / float(pw) >= float(cl) / float(cw):
                out[-2:] = [(np.float32(cl + pl), ps, ce, np.float32(pw + cw))]
            else:
                break
    return out


class IsotonicRegressionModelData:
    def __init__(self):
        self.boundaries: List[float] = []
        self.values: List[float] = []
        self.meta = Params()


def train_isotonic(mt: MTable, p: Params) -> IsotonicRegressionModelData:
    label_col = p.get("labelCol")
    feature_col = p.get("featureCol") if p.contains("featureCol") else None
    vector_col = p.get("vectorCol") if p.contains("vectorCol") else None
    weight_col = p.get("weightCol") if p.contains("weightCol") else None
    isotonic = bool(p.get("isotonic")) if p.contains("isotonic") else True
    index = int(p.get("featureIndex")) if p.contains("featureIndex") else 0
    if (vector_col is None) == (feature_col is None):
        raise ValueError("Either featureColName or vectorColName is required!")
    lab = np.asarray([float(x) for x in mt.col(label_col).to_list()], dtype=np.float64)
    lab = lab if isotonic else -lab
    if vector_col is None:
        feat = np.asarray([float(x) for x in mt.col(feature_col).to_list()], dtype=np.float64)
    else:
        feat = np.asarray([VectorUtil.getVector(v).get(index) for v in mt.col(vector_col).to_list()],
                          dtype=np.float64)
    w = (np.ones_like(lab) if weight_col is None else
         np.asarray([float(x) for x in mt.col(weight_col).to_list()], dtype=np.float64))
    if (w < 0).any():
        raise ValueError("Weights must be non-negative!")
    keep = w > 0
    f, (lv, wv) = sample_sort(torch.from_numpy(feat[keep]), [torch.from_numpy(lab[keep]),
                                                              torch.from_numpy(w[keep])],
                              secondary=torch.from_numpy(lab[keep]))
    f, lv, wv = f.numpy(), lv.numpy(), wv.numpy()
    local = pav_blocks([(np.float32(l * ww), float(x), float(x), np.float32(ww)) for x, l, ww in zip(f, lv, wv)])
    parts = [b for b in comm.all_gather_object(local) if b]
    parts.sort(key=lambda bl: bl[0][1])
    merged = pav_blocks([b for part in parts for b in part])
    m = IsotonicRegressionModelData()
    # BuildModel walks the merged list with ``while (hasNext()) {use current; advance();}``
    # (IsotonicRegTrainBatchOp.java:134-152), which never emits the LAST block; the documented model
    # (docs/en/isotonicregtrainbatchop.md) shows exactly that, so it is reproduced (a single block is kept).
    emit = merged[:-1] if len(merged) > 1 else merged
    for l, s, e, ww in emit:
        q = np.float32(l) / np.float32(ww)
        val = float(q) if isotonic else float(-q)
        m.boundaries.append(s)
        m.values.append(val)
        if s != e:
            m.boundaries.append(e)
            m.values.append(val)
    m.meta.set("featureCol", feature_col)
    m.meta.set("vectorCol", vector_col)
    m.meta.set("featureIndex", index)
    return m


class IsotonicRegressionConverter(SimpleModelDataConverter):
    def serializeModel(self, m: IsotonicRegressionModelData):
        return m.meta, [gson_dumps([float(x) for x in m.boundaries]), gson_dumps([float(x) for x in m.values])]

    def deserializeModel(self, meta: Params, data: List[str]) -> IsotonicRegressionModelData:
        m = IsotonicRegressionModelData()
        m.boundaries = [float(x) for x in json.loads(data[0])]
        m.values = [float(x) for x in json.loads(data[1])]
        m.meta = meta
        return m


def _meta_first(meta: Params, *names):
    for n in names:
        if meta.contains(n):
            v = meta.get(n)
            if v is not None:
                return v
    return None


class IsotonicRegressionModelMapper(ModelMapper):
    """Binary search of the feature in the boundaries, linear interpolation between neighbours."""

    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        p = self.params
        self.helper = OutputColsHelper(dataSchema, [p.get("predictionCol")], [Types.DOUBLE],
                                       p.get("reservedCols") if p.contains("reservedCols") else None)

    def loadModel(self, modelRows):
        self.m = IsotonicRegressionConverter().load(modelRows)
        meta = self.m.meta
        # ParamInfo aliases of the reference meta (vectorColName / featureColName in older models)
        self.vector_col = _meta_first(meta, "vectorCol", "vectorColName", "tensorColName", "vecColName")
        self.feature_col = _meta_first(meta, "featureCol", "featureColName")
        self.index = int(meta.get("featureIndex")) if meta.contains("featureIndex") else 0
        self.b = np.asarray(self.m.boundaries, dtype=np.float64)
        self.v = np.asarray(self.m.values, dtype=np.float64)

    def _predict(self, x: float) -> float:
        b, v = self.b, self.v
        i = bisect.bisect_left(b, x)
        if i < len(b) and b[i] == x:
            return float(v[i])
        if i == 0:
            return float(v[0])
        if i == len(b):
            return float(v[-1])
        return float((x - b[i - 1]) / (b[i] - b[i - 1]) * (v[i] - v[i - 1]) + v[i - 1])

    def _map_columns(self, mt: MTable):
        col = self.vector_col or self.feature_col
        c = mt.col(col)
        if not self.vector_col and isinstance(c.values, torch.Tensor) and c.values.dim() == 1 and len(self.b):
            # the whole column through searchsorted (bisect_left's index; NaN goes left as bisect sends it)
            # separate elementwise tensor ops (no fused multiply-add): the scalar formula's rounding
            x = c.values.detach().to(torch.float64)
            b = torch.as_tensor(self.b, device=x.device)
            v = torch.as_tensor(self.v, device=x.device)
            i = torch.searchsorted(b, x, side="left")
            i = torch.where(torch.isnan(x), torch.zeros_like(i), i)
            ic = i.clamp(max=len(b) - 1)
            lo = (i - 1).clamp(min=0)
            mid = (x - b[lo]) / (b[ic] - b[lo]) * (v[ic] - v[lo]) + v[lo]
            out = torch.where(i == 0, v[0], torch.where(i == len(b), v[-1], mid))
            out = torch.where((i < len(b)) & (b[ic] == x), v[ic], out)
            nm = c.nulls.to(x.device) if c.nulls is not None else None
            if nm is not None:
                out = torch.where(nm, torch.zeros_like(out), out)
            return [Column(out, nm)]
        vals = c.to_list()
        out = []
        for x in vals:
            if x is None:
                out.append(None)
                continue
            f = VectorUtil.getVector(x).get(self.index) if self.vector_col else float(x)
            out.append(self._predict(f))
        return [Column.from_values(out, Types.DOUBLE)]
