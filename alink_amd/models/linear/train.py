"""Training drivers of the linear family: binary/regression (LR, SVM, LinearReg, Ridge, Lasso, SVR,
Perceptron), multinomial softmax and AFT survival regression.

Reference: ``A/operator/common/linear/BaseLinearModelTrainBatchOp.java:68-790`` (label ordering, feature
transform, standardization statistics, optimize, model build), ``A/operator/batch/classification/
SoftmaxTrainBatchOp.java`` and ``A/operator/batch/regression/AftSurvivalRegTrainBatchOp.java``.

SPMD flow (every rank holds one row partition, device-resident):
  distinct labels -> all-gather -> ordered label list (identical on all ranks)
  features -> FeatureMatrix on the device; global column moments by one all-reduce
  standardize/prefix intercept in place -> BSP optimizer (optim.py) -> coefficient de-standardization
  -> model rows (replicated table).
"""
from __future__ import annotations

import functools
from typing import Any, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...common.linalg import DenseVector
from ...common.params import Params
from ...common.table import MTable
from ...common.types import Types, is_numeric
from ...parallel import comm
from ..common.features import FeatureMatrix, column_stats, extract_features, global_vector_size
from .model import (LinearModelData, LinearModelDataConverter, LinearModelType, linear_feature_type_name)
from .objfunc import (AftRegObjFunc, LabeledData, LogLossFunc, PerceptronLossFunc, SmoothHingeLossFunc,
                      SoftmaxObjFunc, SquareLossFunc, SvrLossFunc, UnaryLossObjFunc)
from .optim import optimize

__all__ = ["train_linear", "train_softmax", "train_aft", "distinct_labels", "order_binary_labels",
           "java_compare", "resolve_feature_cols"]


def _pget(p: Params, name: str, default=None):
    try:
        if p.contains(name):
            v = p.get(name)
            return default if v is None else v
    except KeyError:
        pass
    return default


def java_compare(a, b) -> int:
    """Natural ordering of two label values (Comparable semantics: numbers numerically, else strings)."""
    if isinstance(a, (int, float, np.number)) and isinstance(b, (int, float, np.number)):
        return (a > b) - (a < b)
    sa, sb = str(a), str(b)
    return (sa > sb) - (sa < sb)


def _int_label_tensor(col):
    """The label column as an integer / bool tensor (no nulls), or None (other types take the per-value path)."""
    v = col.values
    if isinstance(v, torch.Tensor) and v.dim() == 1 and not v.is_floating_point() and not v.is_complex() and \
            (col.nulls is None or not bool(col.nulls.any())):
        return v
    return None


def distinct_labels(mt: MTable, label_col: str) -> List[Any]:
    """Global distinct label values (first-seen order across ranks)."""
    col = mt.col(label_col)
    t = _int_label_tensor(col)
    if t is not None and t.numel():
        # first-seen order of the distinct values from one unique + first-index pass (what the loop below yields)
        uq, inv = torch.unique(t, return_inverse=True)
        first = torch.full((uq.numel(),), t.numel(), dtype=torch.int64, device=t.device)
        first.scatter_reduce_(0, inv, torch.arange(t.numel(), device=t.device), reduce="amin")
        vals = uq[torch.argsort(first)].tolist()
        local = [bool(x) for x in vals] if t.dtype == torch.bool else [int(x) for x in vals]
    else:
        local = []
        seen = set()
        for v in col.to_list():
            if v is not None and v not in seen:
                seen.add(v)
                local.append(v)
    out, seen = [], set()
    for part in comm.all_gather_object(local):
        for v in part:
            if v not in seen:
                seen.add(v)
                out.append(v)
    return out


def order_binary_labels(labels: Sequence[Any]) -> List[Any]:
    """Two labels; the one with the larger ``toString()`` becomes labels[0] (the positive class,
    ``BaseLinearModelTrainBatchOp.orderLabels``)."""
    labels = list(labels)
    if len(labels) != 2:
        raise ValueError("labels count should be 2 in 2 classification algo.")
    s0, s1 = str(labels[0]), str(labels[1])
    pos = s1 if s1 > s0 else s0
    if str(labels[1]) == pos:
        labels[0], labels[1] = labels[1], labels[0]
    return labels


def resolve_feature_cols(mt: MTable, params: Params, exclude: Sequence[str]) -> Optional[List[str]]:
    fc = _pget(params, "featureCols")
    vc = _pget(params, "vectorCol")
    if not fc and not vc:
        fc = [n for n, t in zip(mt.schema.names, mt.schema.types) if is_numeric(t) and n not in exclude]
        params.set("featureCols", fc)
    return list(fc) if fc else None


def _weights(mt: MTable, weight_col: Optional[str], dev) -> torch.Tensor:
    if weight_col:
        c = mt.col(weight_col)
        v = c.values if isinstance(c.values, torch.Tensor) else torch.tensor([float(x) for x in c.values])
        return v.to(device=dev, dtype=torch.float64)
    return torch.ones(mt.num_rows, dtype=torch.float64, device=dev)


def _feature_types(mt: MTable, fc: Optional[List[str]]) -> Optional[List[str]]:
    if fc is None:
        return None
    return [linear_feature_type_name(mt.col_type(c)) for c in fc]


def _mean_std(X: FeatureMatrix, d: int, standardization: bool):
    dev = X.device
    if not standardization:
        return None, None
    st = column_stats(X, d)
    if X.is_sparse:
        mean = torch.zeros(d, dtype=torch.float64, device=dev)
        std = st["maxAbs"].clone()
    else:
        mean, std = st["mean"].clone(), st["std"].clone()
    zero = std == 0
    std[zero] = 1.0
    mean[zero] = 0.0
    return mean, std


def _is_global_sparse(X: FeatureMatrix) -> bool:
    return any(comm.all_gather_object(bool(X.is_sparse)))


def train_linear(mt: MTable, params: Params, model_type: str, model_name: str, env) -> Tuple[LinearModelData, dict]:
    """Binary classification / regression linear model (``BaseLinearModelTrainBatchOp.linkFrom``)."""
    params = params.clone()
    dev = env.device
    label_col = params.get("labelCol")
    # parameter transforms of getIsRegProc
    is_reg = model_type in ("LinearReg", "SVR")
    l1 = float(_pget(params, "l1", 0.0))
    l2 = float(_pget(params, "l2", 0.0))
    if model_name == "Ridge Regression":
        lam = float(params.get("lambda"))
        if not lam > 0:
            raise ValueError(f"lambda must be positive number or zero! lambda is : {lam}")
        l2, l1 = lam, 0.0
    elif model_name == "LASSO":
        lam = float(params.get("lambda"))
        if lam < 0:
            raise ValueError("lambda must be positive number or zero!")
        l1, l2 = lam, 0.0
    elif model_type == "SVR":
        tau, c = float(params.get("tau")), float(params.get("C"))
        if tau < 0:
            raise ValueError("Parameter tau must be positive number or zero!")
        if c <= 0:
            raise ValueError("Parameter C must be positive number!")
        l1, l2 = 0.0, 1.0 / c
    fc = resolve_feature_cols(mt, params, [label_col])
    vc = _pget(params, "vectorCol") or None
    weight_col = _pget(params, "weightCol")
    with_intercept = bool(_pget(params, "withIntercept", True))
    standardization = bool(_pget(params, "standardization", True))
    label_type = Types.DOUBLE if is_reg else mt.col_type(label_col)
    labels = None
    lcol = mt.col(label_col)
    lt = lcol.values if isinstance(lcol.values, torch.Tensor) and lcol.values.dim() == 1 and \
        (lcol.nulls is None or not bool(lcol.nulls.any())) else None
    if is_reg:
        y = lt.to(device=dev, dtype=torch.float64) if lt is not None and not lt.is_complex() else \
            torch.tensor([float(v) for v in lcol.to_list()], dtype=torch.float64, device=dev)
    else:
        labels = order_binary_labels(distinct_labels(mt, label_col))
        it = _int_label_tensor(lcol)
        if it is not None and isinstance(labels[0], (int, bool)):
            # integer labels: str(v) == str(labels[0]) <=> v == labels[0]
            y = torch.where(it.to(dev) == int(labels[0]), 1.0, -1.0).to(torch.float64)
        else:
            pos = str(labels[0])
            y = torch.tensor([1.0 if str(v) == pos else -1.0 for v in lcol.to_list()], dtype=torch.float64,
                             device=dev)
    X = extract_features(mt, fc, vc, dev)
    d = global_vector_size(X) if vc else len(fc)
    X.set_ncols(d)
    mean, std = _mean_std(X, d, standardization)
    Xs = X
    if standardization:
        Xs = X.standardize(mean, std, center=with_intercept)
    if with_intercept:
        Xs = Xs.prefix_one()
    data = LabeledData(Xs, y, _weights(mt, weight_col, dev))
    loss = {"LR": LogLossFunc(), "SVM": SmoothHingeLossFunc(), "LinearReg": SquareLossFunc(),
            "Perceptron": PerceptronLossFunc(),
            "SVR": SvrLossFunc(float(_pget(params, "tau", 0.1)))}[model_type]
    obj = UnaryLossObjFunc(loss, l1, l2)
    dim = d + (1 if with_intercept else 0)
    hist: list = []
    opt_params = params.clone()
    coef, curve = optimize(obj, data, dim, opt_params, env=env, history=hist)
    coef = coef.copy()
    if standardization:
        mu, sd = mean.cpu().numpy(), std.cpu().numpy()
        if with_intercept:
            s = float(np.sum(coef[1:] * mu / sd))
            coef[1:] = coef[1:] / sd
            coef[0] -= s
        else:
            coef = coef / sd
    m = LinearModelData()
    m.modelName = model_name
    m.linearModelType = LinearModelType[model_type]
    m.hasInterceptItem = with_intercept
    m.vectorColName = vc
    m.vectorSize = d
    m.labelName = None  # LinearModelData(labelType, meta, ...) never copies labelCol: always null
    m.labelValues = labels
    m.labelType = label_type
    m.featureNames = fc
    m.featureTypes = _feature_types(mt, fc)
    m.coefVector = DenseVector(coef)
    m.lossCurve = curve
    return m, {"lossCurve": curve, "history": hist, "numIter": len(curve)}


def _sorted_labels(labels: List[Any]) -> List[Any]:
    return sorted(labels, key=functools.cmp_to_key(java_compare))


def train_softmax(mt: MTable, params: Params, env) -> Tuple[LinearModelData, dict]:
    """Multinomial LR (``SoftmaxTrainBatchOp.java``): labels sorted naturally, class index = position."""
    params = params.clone()
    dev = env.device
    label_col = params.get("labelCol")
    fc = resolve_feature_cols(mt, params, [label_col])
    vc = _pget(params, "vectorCol") or None
    weight_col = _pget(params, "weightCol")
    with_intercept = bool(_pget(params, "withIntercept", True))
    standardization = bool(_pget(params, "standardization", True))
    labels = _sorted_labels(distinct_labels(mt, label_col))
    K = len(labels)
    if K < 2:
        raise ValueError("softmax needs at least 2 label values")
    idx = {v: i for i, v in enumerate(labels)}
    y = torch.tensor([float(idx[v]) for v in mt.col(label_col).to_list()], dtype=torch.float64, device=dev)
    X = extract_features(mt, fc, vc, dev)
    d = global_vector_size(X) if vc else len(fc)
    X.set_ncols(d)
    mean, std = _mean_std(X, d, standardization)
    Xs = X.standardize(mean, std, center=with_intercept) if standardization else X
    if with_intercept:
        Xs = Xs.prefix_one()
    m_dim = d + (1 if with_intercept else 0)
    obj = SoftmaxObjFunc(K, float(_pget(params, "l1", 0.0)), float(_pget(params, "l2", 0.0)))
    data = LabeledData(Xs, y, _weights(mt, weight_col, dev))
    hist: list = []
    coef, curve = optimize(obj, data, (K - 1) * m_dim, params, env=env, history=hist)
    coef = coef.copy()
    if standardization:
        mu, sd = mean.cpu().numpy(), std.cpu().numpy()
        W = coef.reshape(K - 1, m_dim)
        if with_intercept:
            for k in range(K - 1):
                s = float(np.sum(W[k, 1:] * mu / sd))
                W[k, 1:] = W[k, 1:] / sd
                W[k, 0] -= s
        else:
            W /= sd[None, :]
        coef = W.reshape(-1)
    m = LinearModelData()
    m.modelName = "softmax"
    m.linearModelType = None
    m.hasInterceptItem = with_intercept
    m.vectorColName = vc
    m.vectorSize = d
    m.labelName = None  # LinearModelData(labelType, meta, ...) never copies labelCol: always null
    m.labelValues = labels
    m.labelType = mt.col_type(label_col)
    m.featureNames = fc
    m.featureTypes = _feature_types(mt, fc)
    m.coefVector = DenseVector(coef)
    m.coefVectors = None
    m.lossCurve = curve
    return m, {"lossCurve": curve, "history": hist, "numIter": len(curve)}


def train_aft(mt: MTable, params: Params, env) -> Tuple[LinearModelData, dict]:
    """AFT survival regression (``AftSurvivalRegTrainBatchOp.java``): label = log(time), censor as the
    sample-weight slot, features scaled by their std (no centering), last coefficient = log(sigma)."""
    params = params.clone()
    dev = env.device
    label_col = params.get("labelCol")
    censor_col = params.get("censorCol")
    fc = resolve_feature_cols(mt, params, [label_col, censor_col])
    vc = _pget(params, "vectorCol") or None
    with_intercept = bool(_pget(params, "withIntercept", True))
    times = torch.tensor([float(v) for v in mt.col(label_col).to_list()], dtype=torch.float64)
    if len(times) and bool((times <= 0).any()):
        raise ValueError("Survival Time must be greater than 0!")
    cens = torch.tensor([float(v) for v in mt.col(censor_col).to_list()], dtype=torch.float64)
    if len(cens) and bool(((cens != 0.0) & (cens != 1.0)).any()):
        raise ValueError("Censor must be 1.0 or 0.0!")
    X = extract_features(mt, fc, vc, dev)
    d = global_vector_size(X) if vc else len(fc)
    X.set_ncols(d)
    std = column_stats(X, d)["std"]
    safe = torch.where(std > 0, std, torch.ones_like(std))
    if X.is_sparse:
        keep = std[X.col] > 0
        Xs = FeatureMatrix(crow=X.crow, col=X.col, val=torch.where(keep, X.val / safe[X.col],
                                                                   torch.zeros_like(X.val)), ncols=d)
    else:
        Xs = FeatureMatrix(torch.where(std[None, :] > 0, X.dense / safe[None, :], torch.zeros_like(X.dense)))
    if with_intercept:
        Xs = Xs.prefix_one()
    data = LabeledData(Xs, torch.log(times).to(dev), cens.to(dev))
    obj = AftRegObjFunc(float(_pget(params, "l1", 0.0)), float(_pget(params, "l2", 0.0)))
    dim = d + (1 if with_intercept else 0) + 1
    hist: list = []
    coef, curve = optimize(obj, data, dim, params, env=env, history=hist)
    sd = std.cpu().numpy()
    out = coef.copy()
    size = len(coef) - 1
    if with_intercept:
        for i in range(1, size):
            out[i] = coef[i] / sd[i - 1] if sd[i - 1] > 0 else 0.0
        out[size] = np.exp(coef[size])
    else:
        for i in range(size):
            out[i] = coef[i] / sd[i] if sd[i] > 0 else 0.0
    m = LinearModelData()
    m.modelName = "AFTSurvivalRegTrainBatchOp"
    m.linearModelType = LinearModelType["AFT"]
    m.hasInterceptItem = with_intercept
    m.vectorColName = vc
    # buildLinearModelData compares the enum with a String there, so the AFT slot is never subtracted:
    # the stored vectorSize is coef.size - intercept (docs/en/aftsurvivalregression.md shows 3 for 2 features)
    m.vectorSize = dim - (1 if with_intercept else 0)
    m.labelName = None  # LinearModelData(labelType, meta, ...) never copies labelCol: always null
    m.labelValues = None
    m.labelType = Types.DOUBLE
    m.featureNames = fc
    m.featureTypes = _feature_types(mt, fc)
    m.coefVector = DenseVector(out)
    m.lossCurve = curve
    return m, {"lossCurve": curve, "history": hist, "numIter": len(curve)}
