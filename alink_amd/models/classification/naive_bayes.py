"""Naive Bayes for text / count vectors (multinomial, Bernoulli).

Reference: ``A/operator/batch/classification/NaiveBayesTextTrainBatchOp.java`` (per-label weighted feature
sums, ``pi = log(n_l + s) - log(N + L s)``, multinomial ``theta = log(f + s) - log(sum f + D s)``, Bernoulli
``theta = log(f + s) - log(n_l + 2 s)``) and ``A/operator/common/classification/NaiveBayesText{ModelMapper,
ModelDataConverter}.java`` (``pi + theta x`` (+ Bernoulli ``phi`` / ``log(1-e^theta)`` terms), detail =
softmax of the log scores).

Device path: the per-label sums are one ``Y^T X`` product (one-hot(label) * weight against the dense or CSR
sample matrix) followed by a single all-reduce; prediction is one ``X theta^T`` GEMM per micro-batch.
"""
from __future__ import annotations

import json
import math
from typing import Any, List

import numpy as np
import torch

from ...common.javafmt import gson_dumps, java_str
from ...common.linalg import DenseMatrix
from ...common.mapper import OutputColsHelper, RichModelMapper
from ...common.model.converter import LabeledModelDataConverter
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import Types
from ...parallel import comm
from ..common.features import FeatureMatrix, extract_features, global_vector_size
from ..linear.model import _dev, _recover_label, label_column


def _recount_crow(crow: torch.Tensor, keep: torch.Tensor) -> torch.Tensor:
    """CSR row pointers after dropping the entries where ``keep`` is False."""
    c = torch.zeros(keep.numel() + 1, dtype=torch.int64, device=keep.device)
    torch.cumsum(keep.to(torch.int64), 0, out=c[1:])
    return c[crow.to(torch.int64)]

__all__ = ["train_naive_bayes_text", "NaiveBayesTextModelDataConverter", "NaiveBayesTextModelMapper"]


def _pget(p: Params, name, default=None):
    try:
        if p.contains(name):
            v = p.get(name)
            return default if v is None else v
    except KeyError:
        pass
    return default


class _ProbInfo:
    __gson_fields__ = ("piArray", "theta")

    def __init__(self, pi, theta):
        self.piArray = [float(x) for x in pi]
        self.theta = theta


class NaiveBayesTextModelDataConverter(LabeledModelDataConverter):
    def serializeModel(self, m):
        meta = Params().set("modelType", m["modelType"]).set("vectorCol", m["vectorCol"])
        return meta, [gson_dumps(_ProbInfo(m["pi"], DenseMatrix(m["theta"])), java_map_order=False)], m["labels"]

    def deserializeModel(self, meta, data, labels):
        d = json.loads(data[0])
        th = d["theta"]
        theta = np.asarray(th["data"], dtype=np.float64).reshape(int(th["n"]), int(th["m"])).T
        mt = str(getattr(meta.get("modelType"), "name", meta.get("modelType")))
        mt = "Bernoulli" if mt.upper() == "BERNOULLI" else "Multinomial"
        return {"pi": np.asarray(d["piArray"], dtype=np.float64), "theta": theta, "labels": list(labels),
                "modelType": mt, "vectorCol": meta.get("vectorCol") if meta.contains("vectorCol") else None}


def train_naive_bayes_text(mt: MTable, params: Params, env):
    dev = env.device
    label_col = params.get("labelCol")
    vec_col = params.get("vectorCol")
    smoothing = float(_pget(params, "smoothing", 1.0))
    model_type = str(getattr(_pget(params, "modelType", "Multinomial"), "name", _pget(params, "modelType",
                                                                                       "Multinomial")))
    model_type = "Bernoulli" if model_type.upper() == "BERNOULLI" else "Multinomial"
    wcol = _pget(params, "weightCol")
    fm = extract_features(mt, None, vec_col, dev)
    d = global_vector_size(fm)
    fm.set_ncols(d) if fm.is_sparse else None
    labels_local = mt.column_values(label_col)
    keys = sorted({java_str(v) for part in comm.all_gather_object(sorted({java_str(v) for v in labels_local}))
                   for v in part})
    first = {}
    for v in labels_local:
        first.setdefault(java_str(v), v)
    reps = {}
    for part in comm.all_gather_object(first):
        for k, v in part.items():
            reps.setdefault(k, v)
    L = len(keys)
    pos = {k: i for i, k in enumerate(keys)}
    y = torch.tensor([pos[java_str(v)] for v in labels_local], dtype=torch.long, device=dev)
    w = torch.ones(len(labels_local), dtype=torch.float64, device=dev) if wcol is None else \
        torch.tensor([float(x) for x in mt.column_values(wcol)], dtype=torch.float64, device=dev)
    Y = torch.zeros((len(labels_local), L), dtype=torch.float64, device=dev)
    if len(labels_local):
        Y[torch.arange(len(labels_local), device=dev), y] = w
    feat = fm.rmm(Y, d).T.contiguous() if len(labels_local) else torch.zeros((L, d), dtype=torch.float64,
                                                                                device=dev)
    wsum = Y.sum(0)
    buf = torch.cat([feat.reshape(-1), wsum])
    comm.all_reduce(buf, "sum")
    feat, wsum = buf[:L * d].reshape(L, d).cpu().numpy(), buf[L * d:].cpu().numpy()
    ndocs = wsum.sum()
    pi_log = math.log(ndocs + L * smoothing)
    pi = np.log(wsum + smoothing) - pi_log
    if model_type == "Multinomial":
        theta_log = np.log(feat.sum(1) + d * smoothing)
    else:
        theta_log = np.log(wsum + 2.0 * smoothing)
    theta = np.log(feat + smoothing) - theta_log[:, None]
    return {"pi": pi, "theta": theta, "labels": [reps[k] for k in keys], "modelType": model_type,
            "vectorCol": vec_col}


class NaiveBayesTextModelMapper(RichModelMapper):
    model = None

    def loadModel(self, rows):
        from ..linear.model import LinearModelDataConverter
        lt = LinearModelDataConverter.extractLabelType(self.modelSchema)
        self.model = NaiveBayesTextModelDataConverter(lt).load(rows)
        self.model["labels"] = [_recover_label(v, lt) for v in self.model["labels"]]
        self.lt = lt
        th = self.model["theta"]
        if self.model["modelType"] == "Bernoulli":
            tmp = np.log(1.0 - np.exp(th))
            self.phi = tmp.sum(1)
            self.minmat = th - tmp
        names = [self.pred_col] + ([self.detail_col] if self.detail_col else [])
        types = [lt or Types.STRING] + ([Types.STRING] if self.detail_col else [])
        self.helper = OutputColsHelper(self.dataSchema, names, types, self.params.get("reservedCols")
                                       if self.params.contains("reservedCols") else None)

    def _scores(self, mt):
        vec_col = self.params.get("vectorCol") if self.params.contains("vectorCol") else self.model["vectorCol"]
        dev = _dev(mt)
        fm = extract_features(mt, None, vec_col, dev)
        th = self.model["theta"]
        d = th.shape[1]
        if fm.is_sparse and self.model["modelType"] != "Bernoulli":
            # X @ theta^T straight from the CSR rows (indices >= d dropped, as the dense path truncates)
            fm.set_ncols(d)
            if fm.val.numel() and int(fm.col.max()) >= d:
                keep = fm.col < d
                fm = FeatureMatrix(crow=_recount_crow(fm.crow, keep), col=fm.col[keep], val=fm.val[keep], ncols=d)
            T = torch.as_tensor(th.T, dtype=torch.float64, device=dev)
            S = fm.to(dev).mm(T) if fm.val.dtype == torch.float64 else \
                FeatureMatrix(crow=fm.crow, col=fm.col, val=fm.val.double(), ncols=d).mm(T)
            return (S + torch.as_tensor(self.model["pi"], dtype=torch.float64, device=dev)[None, :]).cpu().numpy()
        if fm.is_sparse:
            fm.set_ncols(d)
        X = fm.to_dense().double().cpu().numpy()
        if X.shape[1] < d:
            X = np.pad(X, ((0, 0), (0, d - X.shape[1])))
        X = X[:, :d]
        if self.model["modelType"] == "Bernoulli":
            if not np.isin(X, (0.0, 1.0)).all():
                raise ValueError("Bernoulli naive Bayes requires 0 or 1 feature values.")
            return X @ self.minmat.T + self.model["pi"][None, :] + self.phi[None, :]
        return X @ th.T + self.model["pi"][None, :]

    def _map_row_values(self, row):
        mt = MTable.from_rows([tuple(row)], self.dataSchema)
        return [c.to_list()[0] for c in self._map_columns(mt)]

    def _map_columns(self, mt):
        S = self._scores(mt)
        labels = self.model["labels"]
        if not self.detail_col and len(S):
            # first strict maximum over the classes (NaN never wins; a row of -inf / NaN predicts null)
            Sf = np.where(np.isnan(S), -np.inf, S)
            idx = Sf.argmax(1)
            ok = Sf[np.arange(len(Sf)), idx] > -np.inf
            t = self.helper.out_types[0]
            if ok.all():
                return [label_column(labels, idx, t)]
            lab = np.empty(len(labels), dtype=object)
            lab[:] = labels
            preds = lab[idx]
            preds[~ok] = None
            return [Column.from_values(preds.tolist(), t)]
        preds, details = [], []
        for s in S:
            best, res = float("-inf"), None
            for i, v in enumerate(s):
                if best < v:
                    best, res = v, labels[i]
            preds.append(res)
            if self.detail_col:
                m = s.max()
                lse = m + math.log(np.exp(s - m).sum())
                details.append(gson_dumps({java_str(labels[i]): float(math.exp(s[i] - lse)) for i in range(len(s))}))
        cols = [Column.from_values(preds, self.helper.out_types[0])]
        if self.detail_col:
            cols.append(Column.from_values(details, Types.STRING))
        return cols
