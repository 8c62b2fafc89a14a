"""Factorization machines (classification / regression): device mini-batch AdaGrad + per-superstep model
averaging.

Reference: ``A/operator/common/fm/BaseFmTrainBatchOp.java`` (data transform :313-404, label ordering
:287-304, ``FmDataFormat`` init with ``Random(2020)`` :499-547, losses :443-494),
``A/operator/common/optim/FmOptimizer.java`` (``UpdateLocalModel`` per-sample AdaGrad :302-441, usage-weighted
model averaging ``UpdateGlobalModel`` :262-297, loss / AUC / accuracy :154-257, termination :98-149,
``calcY`` :487-531), ``FmModelDataConverter.java``, ``FmModelMapper.java``.

MI355X-first: the reference visits ``batchSize`` randomly drawn samples one at a time per superstep.  Here the
drawn samples are processed in micro-batches on the rank's device — ``X V`` / ``X^2 V^2`` as one sparse
(CSR gather + segment-sum) or dense GEMM, the per-occurrence gradients scattered with ``index_add_`` into the
gradient and squared-gradient accumulators, then one AdaGrad step for the touched coordinates.  The
superstep ends like the reference's: factors, linear items and AdaGrad state weighted by per-feature usage
are summed in ONE all-reduce and divided by the usage totals.
"""
from __future__ import annotations

import json
import math
from typing import Any, List, Optional

import numpy as np
import torch

from ...common.javafmt import gson_dumps, java_hashmap_order, java_str
from ...common.jrandom import JavaRandom
from ...common.mapper import RichModelMapper
from ...common.model import LabeledModelDataConverter
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import Types
from ...models.common.features import FeatureMatrix, extract_features
from ...ops import fm as fops
from ...parallel import comm

__all__ = ["FmModelData", "FmModelDataConverter", "FmModelMapper", "train_fm", "fm_predict_raw"]

EPS = 1.0e-8


class FmDataFormat:
    __gson_fields__ = ("linearItems", "factors", "bias", "dim")

    def __init__(self, linearItems=None, factors=None, bias=0.0, dim=None):
        self.linearItems = linearItems
        self.factors = factors
        self.bias = bias
        self.dim = dim


class FmModelData:
    def __init__(self):
        self.fmModel: FmDataFormat = None
        self.vectorColName = None
        self.featureColNames = None
        self.labelColName = None
        self.task = "REGRESSION"
        self.vectorSize = 0
        self.labelValues: List[Any] = []
        self.dim = [1, 1, 10]
        self.fieldPos = None


class FmModelDataConverter(LabeledModelDataConverter):
    """Meta (vectorColName, labelColName, task, vectorSize, featureColNames, labelValues, dim, filedPos) +
    ONE JSON ``FmDataFormat`` string + label aux rows (``FmModelDataConverter.java:38-53``)."""

    def serializeModel(self, m: FmModelData):
        meta = Params()
        meta.set("vectorColName", m.vectorColName)
        meta.set("labelColName", m.labelColName)
        meta.set("task", m.task)
        meta.set("vectorSize", int(m.vectorSize))
        meta.set("featureColNames", m.featureColNames)
        meta.set("labelValues", list(m.labelValues))
        meta.set("dim", list(m.dim))
        meta.set("filedPos", m.fieldPos)
        return meta, [gson_dumps(m.fmModel)], list(m.labelValues)

    def deserializeModel(self, meta: Params, data: List[str], labels: List[Any]) -> FmModelData:
        m = FmModelData()

        def g(n, d=None):
            return meta.get(n) if meta.contains(n) else d
        m.vectorColName = g("vectorColName")
        m.labelColName = g("labelColName")
        m.task = g("task", "REGRESSION")
        m.vectorSize = int(g("vectorSize", 0) or 0)
        m.featureColNames = g("featureColNames")
        m.dim = [int(x) for x in g("dim", [1, 1, 10])]
        m.fieldPos = g("filedPos")
        vals = g("labelValues")
        m.labelValues = list(labels) if labels else (list(vals) if vals else [])
        d = json.loads(data[0])
        m.fmModel = FmDataFormat(d.get("linearItems"), d.get("factors"), float(d.get("bias", 0.0)), d.get("dim"))
        return m


def _init_model(vec_size: int, dim, stdev: float) -> FmDataFormat:
    """``FmDataFormat(vecSize, dim, initStdev).reset``: ``Random(2020)`` Gaussians, linear items first."""
    rnd = JavaRandom(2020)
    lin = [rnd.nextGaussian() * stdev for _ in range(vec_size)] if dim[1] > 0 else None
    fac = ([[rnd.nextGaussian() * stdev for _ in range(dim[2])] for _ in range(vec_size)] if dim[2] > 0 else None)
    return FmDataFormat(lin, fac, 0.0, list(dim))


def _sq(fm: FeatureMatrix) -> FeatureMatrix:
    if fm.dense is not None:
        return FeatureMatrix(fm.dense * fm.dense)
    return FeatureMatrix(crow=fm.crow, col=fm.col, val=fm.val * fm.val, ncols=fm.ncols)


def fm_predict_raw(fm: FeatureMatrix, w: Optional[torch.Tensor], V: Optional[torch.Tensor], bias: float,
                   dim) -> (torch.Tensor, Optional[torch.Tensor]):
    """``FmOptimizer.calcY`` for a block of rows: y = b + X w + 1/2 sum_f ((X V)_f^2 - (X^2 V^2)_f)."""
    n = fm.nrows
    dev = fm.device
    if dim[2] > 0 and V is not None and fops.kernel_supported(fm, V.shape[1]):
        return fops.fm_forward(fm, w if dim[1] > 0 else None, V.contiguous(), float(bias) if dim[0] > 0 else 0.0)
    y = torch.full((n,), float(bias) if dim[0] > 0 else 0.0, dtype=torch.float64, device=dev)
    vx = None
    if dim[1] > 0 and w is not None:
        y = y + fm.mv(w)
    if dim[2] > 0 and V is not None:
        vx = fm.mm(V)
        v2x2 = _sq(fm).mm(V * V)
        y = y + 0.5 * (vx * vx - v2x2).sum(1)
    return y, vx


def _dldy(task: str, ytrue: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    if task == "REGRESSION":
        return 2.0 * (y - ytrue)
    return torch.sigmoid(y) - ytrue


def _loss(task: str, ytrue: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    if task == "REGRESSION":
        return (ytrue - y) ** 2
    p = torch.sigmoid(y)
    return torch.where(ytrue > 0.5, -torch.log(p), -torch.log(1.0 - p))


def _auc(y: torch.Tensor, lab: torch.Tensor) -> float:
    order = torch.argsort(y, stable=True)
    pos = lab[order] > 0.5
    ranks = torch.arange(1, y.shape[0] + 1, dtype=torch.float64, device=y.device)
    m = int(pos.sum())
    n = y.shape[0] - m
    if m == 0 or n == 0:
        return 0.0
    return float((ranks[pos].sum() - 0.5 * m * (m + 1.0)) / (m * float(n)))


def _order_labels(labels: List[Any]) -> List[Any]:
    """``BaseFmTrainBatchOp.orderLabels``: the label whose string is larger goes first (positive)."""
    if len(labels) != 2:
        raise ValueError("labels count should be 2 in 2 classification algo.")
    a, b = labels
    return [b, a] if java_str(b) > java_str(a) else [a, b]


def train_fm(mt: MTable, p: Params, task: str, env, micro_batch: int = 512):
    """Returns (FmModelData, label type, train info)."""
    dev = env.device
    label_col = p.get("labelCol")
    vector_col = p.get("vectorCol") if p.contains("vectorCol") else None
    feature_cols = p.get("featureCols") if p.contains("featureCols") else None
    weight_col = p.get("weightCol") if p.contains("weightCol") else None
    if feature_cols is None and vector_col is None:
        feature_cols = [n for n, t in zip(mt.schema.names, mt.schema.types)
                        if n != label_col and t in (Types.DOUBLE, Types.FLOAT, Types.LONG, Types.INT)]
    dim = [1 if p.get("withIntercept") else 0, 1 if p.get("hasLinearItem") else 0, int(p.get("numFactor"))]
    fm = extract_features(mt, feature_cols, vector_col, dev)
    vec_size = max(comm.all_gather_object(int(fm.ncols)))
    fm.set_ncols(vec_size)
    raw = mt.col(label_col).to_list()
    label_type = Types.DOUBLE if task == "REGRESSION" else mt.col_type(label_col)
    if task == "REGRESSION":
        labels = [0.0]
        y = torch.tensor([float(v) for v in raw], dtype=torch.float64, device=dev)
    else:
        distinct = set()
        for part in comm.all_gather_object(list(set(raw))):
            distinct.update(part)
        labels = _order_labels(sorted(distinct, key=java_str))
        y = torch.tensor([1.0 if v == labels[0] else 0.0 for v in raw], dtype=torch.float64, device=dev)
    sw = (torch.ones(fm.nrows, dtype=torch.float64, device=dev) if weight_col is None else
          torch.tensor([float(v) for v in mt.col(weight_col).to_list()], dtype=torch.float64, device=dev))
    init = _init_model(vec_size, dim, float(p.get("initStdev")))
    w = torch.tensor(init.linearItems, dtype=torch.float64, device=dev) if dim[1] > 0 else None
    V = torch.tensor(init.factors, dtype=torch.float64, device=dev).reshape(vec_size, dim[2]) if dim[2] > 0 else None
    bias = torch.zeros((), dtype=torch.float64, device=dev)
    sg_w = torch.zeros_like(w) if w is not None else None
    sg_V = torch.zeros_like(V) if V is not None else None
    sg_b = torch.zeros((), dtype=torch.float64, device=dev)
    lam = [float(p.get("lambda_0")), float(p.get("lambda_1")), float(p.get("lambda_2"))]
    lr = float(p.get("learnRate"))
    epochs = int(p.get("numEpochs"))
    bsz = int(p.get("minibatchSize"))
    eps_stop = float(p.get("epsilon"))
    n0 = comm.broadcast_object(fm.nrows, 0)
    num_batches = epochs if (bsz == -1 or bsz > n0) else (n0 // bsz + 1) * epochs
    n_local = fm.nrows
    per_step = n_local if bsz == -1 else min(bsz, n_local) if n_local else 0
    gen = torch.Generator(device="cpu").manual_seed(2020 + comm.get_rank())
    old_loss = None
    curve = []
    step = 0
    while True:
        step += 1
        use = torch.zeros(vec_size, dtype=torch.float64, device=dev)
        if per_step:
            draw = torch.randint(0, n_local, (per_step,), generator=gen).to(dev)
            for s in range(0, per_step, micro_batch):
                idx = draw[s:s + micro_batch]
                xb = fm.take(idx)
                yb, vx = fm_predict_raw(xb, w, V, float(bias), dim)
                g = _dldy(task, y[idx], yb)
                if dim[0] > 0:
                    gb = g + lam[0] * bias
                    sg_b = sg_b + (gb * gb).sum()
                    bias = bias - lr * gb.sum() / torch.sqrt(sg_b + EPS)
                if dim[2] > 0 and fops.kernel_supported(xb, dim[2]):
                    # K18: AdaGrad on the touched coordinates only, one wave per coordinate segment
                    fops.fm_coord_update(xb, g, vx, sw[idx], w if dim[1] > 0 else None,
                                         sg_w if dim[1] > 0 else None, V, sg_V, use, lr, lam[1], lam[2])
                    continue
                if xb.dense is not None:
                    rows = torch.arange(xb.nrows, device=dev).repeat_interleave(vec_size)
                    cols = torch.arange(vec_size, device=dev).repeat(xb.nrows)
                    vals = xb.dense.reshape(-1)
                else:
                    rows, cols, vals = xb.row_ids(), xb.col, xb.val
                use.index_add_(0, cols, sw[idx][rows])
                gr = g[rows]
                if dim[2] > 0:
                    Vc = V[cols]
                    gv = (gr * vals)[:, None] * (vx[rows] - vals[:, None] * Vc) + lam[2] * Vc
                    G = torch.zeros_like(V).index_add_(0, cols, gv)
                    sg_V.index_add_(0, cols, gv * gv)
                    V = V - lr * G / torch.sqrt(sg_V + EPS)
                if dim[1] > 0:
                    gl = gr * vals + lam[1] * w[cols]
                    Gl = torch.zeros_like(w).index_add_(0, cols, gl)
                    sg_w.index_add_(0, cols, gl * gl)
                    w = w - lr * Gl / torch.sqrt(sg_w + EPS)
        # ---- model averaging (UpdateGlobalModel): one all-reduce of usage-weighted state ----
        parts = [use]
        if dim[2] > 0:
            parts += [(V * use[:, None]).reshape(-1), (sg_V * use[:, None]).reshape(-1)]
        if dim[1] > 0:
            parts += [w * use, sg_w * use]
        parts.append(torch.stack([bias, sg_b]))
        buf = torch.cat(parts)
        comm.all_reduce(buf, "sum")
        tot = buf[:vec_size]
        off = vec_size
        has = tot > 0
        den = torch.where(has, tot, torch.ones_like(tot))
        if dim[2] > 0:
            k = dim[2]
            nv = buf[off:off + vec_size * k].reshape(vec_size, k) / den[:, None]
            ns = buf[off + vec_size * k:off + 2 * vec_size * k].reshape(vec_size, k) / den[:, None]
            V = torch.where(has[:, None], nv, V)
            sg_V = torch.where(has[:, None], ns, sg_V)
            off += 2 * vec_size * k
        if dim[1] > 0:
            nw = buf[off:off + vec_size] / den
            ns = buf[off + vec_size:off + 2 * vec_size] / den
            w = torch.where(has, nw, w)
            sg_w = torch.where(has, ns, sg_w)
            off += 2 * vec_size
        if dim[0] > 0:
            ws = comm.get_world_size()
            bias = buf[off] / ws
            sg_b = buf[off + 1] / ws
        # ---- loss / evaluation (CalcLossAndEvaluation) ----
        yall, _ = fm_predict_raw(fm, w, V, float(bias), dim)
        lsum = float(_loss(task, y, yall).sum()) if n_local else 0.0
        if task == "REGRESSION":
            diff = yall - y
            m2, m3 = float(diff.abs().sum()), float((diff * diff).sum())
        else:
            m2 = _auc(yall, y) if n_local else 0.0
            m3 = float((((yall > 0) & (y > 0.5)) | ((yall < 0) & (y < 0.5))).sum())
        stats = torch.tensor([lsum, float(n_local), m2, m3], dtype=torch.float64)
        comm.all_reduce(stats, "sum")
        loss = float(stats[0] / max(stats[1], 1.0))
        curve.append(loss)
        if step >= num_batches:
            break
        if old_loss is not None and old_loss != 0 and abs(old_loss - loss) / old_loss < eps_stop:
            break
        old_loss = loss
    m = FmModelData()
    m.fmModel = FmDataFormat(w.cpu().tolist() if w is not None else None,
                             V.cpu().tolist() if V is not None else None, float(bias), list(dim))
    m.vectorColName = vector_col
    m.featureColNames = list(feature_cols) if feature_cols else None
    m.labelColName = label_col
    m.task = task
    m.vectorSize = vec_size
    m.labelValues = labels
    m.dim = dim
    return m, label_type, {"lossCurve": curve, "numSteps": step}


class FmModelMapper(RichModelMapper):
    """Batched FM scoring; binary detail = ``{label1: 1-p, label0: p}`` in Java HashMap order."""

    def __init__(self, modelSchema, dataSchema, params=None):
        self._label_type = modelSchema.types[2] if len(modelSchema.types) > 2 else Types.DOUBLE
        super().__init__(modelSchema, dataSchema, params)

    def predResultType(self):
        return self._label_type

    def loadModel(self, modelRows):
        self.m = FmModelDataConverter(self._label_type).load(modelRows)
        f = self.m.fmModel
        self.w = torch.tensor(f.linearItems, dtype=torch.float64) if f.linearItems is not None else None
        self.V = torch.tensor(f.factors, dtype=torch.float64) if f.factors is not None else None
        p = self.params
        vc = p.get("vectorCol") if p.contains("vectorCol") else None
        self.vector_col = vc or self.m.vectorColName
        self.feature_cols = None if vc else self.m.featureColNames

    def _map_columns(self, mt: MTable):
        fm = extract_features(mt, self.feature_cols, self.vector_col if not self.feature_cols else None,
                              torch.device("cpu"), vector_size=self.m.vectorSize)
        fm.set_ncols(max(fm.ncols, self.m.vectorSize))
        w = self.w
        V = self.V
        d = fm.ncols
        if w is not None and w.shape[0] < d:
            w = torch.nn.functional.pad(w, (0, d - w.shape[0]))
        if V is not None and V.shape[0] < d:
            V = torch.nn.functional.pad(V, (0, 0, 0, d - V.shape[0]))
        y, _ = fm_predict_raw(fm, w, V, self.m.fmModel.bias, self.m.dim)
        if self.m.task == "REGRESSION":
            pred = Column(y)
            det = ['{"label":%f}' % v for v in y.tolist()]   # FmModelMapper.java:92 String.format %f if self.detail_col else None
        else:
            pr = torch.sigmoid(y).tolist()
            l0, l1 = self.m.labelValues[0], self.m.labelValues[1]
            pred = Column.from_values([l1 if v <= 0.5 else l0 for v in pr], self._label_type)
            det = None
            if self.detail_col:
                keys = java_hashmap_order([java_str(l1), java_str(l0)])
                det = []
                for v in pr:
                    vals = {java_str(l1): java_str(1 - v), java_str(l0): java_str(v)}
                    det.append(gson_dumps({k: vals[k] for k in keys}, java_map_order=False))
        return [pred] + ([Column.from_values(det, Types.STRING)] if self.detail_col else [])
