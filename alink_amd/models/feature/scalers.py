"""Scalers and imputers (column and vector variants).

Reference: ``A/operator/common/dataproc/{StandardScaler,MinMaxScaler,MaxAbsScaler,Imputer}{ModelDataConverter,
ModelMapper}.java``, ``ScalerUtil.java`` and ``A/operator/common/dataproc/vector/Vector*``.

Training = one distributed ``TableSummary`` (device reductions + all-reduce).  Prediction is a fused
elementwise transform over the whole partition (``(x - mean) / std`` etc. on ``[n, cols]`` tensors), falling
back to Python only for non-tensor (object) columns.
"""
from __future__ import annotations

import json
from typing import List, Optional

import numpy as np
import torch

from ...common.javafmt import gson_dumps
from ...common.linalg import DenseVector, SparseVector, VectorUtil
from ...common.mapper import ModelMapper, OutputColsHelper
from ...common.model.converter import RichModelDataConverter, SimpleModelDataConverter
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import AlinkType, TableSchema, Types
from ...ops import elementwise as ew
from ..common.features import extract_features
from ..statistics.summary import TableSummary, table_summary, vector_summary

__all__ = ["ScalerModelData", "ScalerConverter", "StandardScalerModelMapper", "MinMaxScalerModelMapper",
           "MaxAbsScalerModelMapper", "ImputerModelMapper", "VectorScalerModelMapper", "VectorImputerModelMapper",
           "train_scaler", "train_vector_scaler"]


def _pget(p, name, default=None):
    try:
        return p.get(name) if p.contains(name) and p.get(name) is not None else default
    except KeyError:
        return default


class ScalerModelData:
    def __init__(self, kind: str, meta: Params, arrays: List[np.ndarray], cols: Optional[List[str]],
                 col_types: Optional[List[AlinkType]] = None):
        self.kind, self.meta, self.arrays, self.cols, self.col_types = kind, meta, arrays, cols, col_types


class ScalerConverter(RichModelDataConverter):
    """meta Params + JSON double arrays; selected columns ride along as extra (empty) model columns so the
    predict side can recover their names/types (``ImputerModelDataConverter.extractSelectedColNames``)."""

    def __init__(self, cols: Optional[List[str]] = None, types: Optional[List[AlinkType]] = None):
        self.cols = cols or []
        self.types = types or []

    def additionalColNames(self):
        return list(self.cols)

    def additionalColTypes(self):
        return list(self.types)

    def serializeModel(self, m: ScalerModelData):
        # exactly the reference converters' meta (Standard: withMean/withStd; MinMax: selectedCols/min/max;
        # MaxAbs: selectedCols; Imputer: strategy/selectedCols[/fillValue]) and data rows (JSON double arrays)
        data = [gson_dumps([float(x) for x in a]) if a is not None else "null" for a in m.arrays]
        return m.meta.clone(), data, []

    def deserializeModel(self, meta, data, aux):
        arrays = [None if d == "null" else np.asarray(json.loads(d), dtype=np.float64) for d in data]
        return ScalerModelData(infer_scaler_kind(meta), meta, arrays, None)


def infer_scaler_kind(meta: Params) -> str:
    """The model kind from the reference's meta keys (models written before round 4 also carry scalerKind)."""
    if meta.contains("scalerKind"):
        return str(meta.get("scalerKind"))
    if meta.contains("strategy"):
        return "imputer"
    if meta.contains("withMean") or meta.contains("withStd"):
        return "standard"
    if meta.contains("min") and meta.contains("max"):
        return "minmax"
    return "maxabs"


def train_scaler(kind: str, mt: MTable, params: Params, env) -> MTable:
    cols = list(_pget(params, "selectedCols") or [n for n, t in zip(mt.schema.names, mt.schema.types)
                                                      if t in (Types.DOUBLE, Types.FLOAT, Types.LONG, Types.INT,
                                                               Types.SHORT, Types.BYTE, Types.DECIMAL)])
    t = table_summary(mt, cols, env.device)
    meta = Params()
    if kind == "standard":
        with_mean = bool(_pget(params, "withMean", True))
        with_std = bool(_pget(params, "withStd", True))
        means = np.array([t.mean(c) if with_mean else 0.0 for c in cols])
        stds = np.array([t.standardDeviation(c) if with_std else 1.0 for c in cols])
        meta.set("withMean", with_mean).set("withStd", with_std)
        arrays = [means, stds]
    elif kind == "minmax":
        meta.set("selectedCols", cols).set("min", float(_pget(params, "min", 0.0))).set(
            "max", float(_pget(params, "max", 1.0)))
        arrays = [np.array([t.min(c) for c in cols]), np.array([t.max(c) for c in cols])]
    elif kind == "maxabs":
        meta.set("selectedCols", cols)
        arrays = [np.array([max(abs(t.min(c)), abs(t.max(c))) for c in cols])]
    elif kind == "imputer":
        strategy = str(getattr(_pget(params, "strategy", "MEAN"), "name", _pget(params, "strategy", "MEAN"))).upper()
        meta.set("strategy", strategy).set("selectedCols", cols)
        if strategy == "MIN":
            arrays = [np.array([t.min(c) for c in cols])]
        elif strategy == "MAX":
            arrays = [np.array([t.max(c) for c in cols])]
        elif strategy == "MEAN":
            arrays = [np.array([t.mean(c) for c in cols])]
        else:
            meta.set("fillValue", str(_pget(params, "fillValue")))
            arrays = [None]
    else:
        raise ValueError(kind)
    types = [mt.col_type(c) for c in cols]
    conv = ScalerConverter(cols, types)
    return MTable.from_rows(conv.save(ScalerModelData(kind, meta, arrays, cols)), conv.getModelSchema(),
                            replicated=True)


def _col_tensor(mt: MTable, name: str, dev):
    c = mt.col(name)
    if isinstance(c.values, torch.Tensor) and c.values.dim() == 1:
        v = c.values.to(device=dev, dtype=torch.float64)
        nulls = c.nulls.to(dev) if c.nulls is not None else torch.zeros(v.shape[0], dtype=torch.bool, device=dev)
        return v, nulls | torch.isnan(v)
    lst = c.to_list()
    v = torch.tensor([float(x) if x is not None else float("nan") for x in lst], dtype=torch.float64, device=dev)
    return torch.nan_to_num(v, nan=0.0), torch.tensor([x is None for x in lst], dtype=torch.bool, device=dev)


def _dev(mt):
    for c in mt.cols:
        if isinstance(c.values, torch.Tensor):
            return c.values.device
    return torch.device("cpu")


class _ColumnScalerMapper(ModelMapper):
    """Shared structure: model schema carries the selected columns; output cols default to them."""
    OUT_DOUBLE = True

    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        self.cols = list(modelSchema.names[2:])
        self.col_types = list(modelSchema.types[2:])
        out = _pget(self.params, "outputCols") or self.cols
        types = [Types.DOUBLE] * len(out) if self.OUT_DOUBLE else list(self.col_types)
        self.helper = OutputColsHelper(dataSchema, list(out), types, _pget(self.params, "reservedCols"))

    def loadModel(self, modelRows):
        self.model: ScalerModelData = ScalerConverter(self.cols, self.col_types).load(modelRows)

    def _transform(self, j, v, nulls):
        raise NotImplementedError

    def _map_columns(self, mt):
        dev = _dev(mt)
        out = []
        for j, c in enumerate(self.cols):
            v, nulls = _col_tensor(mt, c, dev)
            r = self._transform(j, v, nulls)
            out.append(Column(r.cpu() if not v.is_cuda else r, nulls.cpu() if bool(nulls.any()) else None))
        return out


class StandardScalerModelMapper(_ColumnScalerMapper):
    def _transform(self, j, v, nulls):
        mean, std = float(self.model.arrays[0][j]), float(self.model.arrays[1][j])
        if v.is_cuda:   # K27 fused transform (one pass, bit-identical)
            return ew.col_transform(v, "standard", [mean], [std])
        return (v - mean) / std if std > 0 else torch.zeros_like(v)


class MinMaxScalerModelMapper(_ColumnScalerMapper):
    def _transform(self, j, v, nulls):
        lo, hi = float(self.model.meta.get("min")), float(self.model.meta.get("max"))
        emin, emax = float(self.model.arrays[0][j]), float(self.model.arrays[1][j])
        if v.is_cuda:
            return ew.col_transform(v, "minmax", [emin], [emax], lo, hi)
        if emin != emax:
            return (v - emin) / (emax - emin) * (hi - lo) + lo
        return torch.full_like(v, 0.5 * (hi + lo))


class MaxAbsScalerModelMapper(_ColumnScalerMapper):
    def _transform(self, j, v, nulls):
        m = float(self.model.arrays[0][j])
        if v.is_cuda:
            return ew.col_transform(v, "maxabs", [m])
        return v if m == 0 else v / m


class ImputerModelMapper(_ColumnScalerMapper):
    """Null -> statistic / fill value, keeping the column type (``ImputerModelMapper.map``)."""
    OUT_DOUBLE = False

    def _map_columns(self, mt):
        out = []
        vals = self.model.arrays[0] if self.model.arrays else None
        fill = self.model.meta.get("fillValue") if self.model.meta.contains("fillValue") else None
        for j, c in enumerate(self.cols):
            t = self.col_types[j]
            if vals is not None:
                f = float(vals[j])
                rep = int(f) if t in (Types.LONG, Types.INT, Types.SHORT, Types.BYTE) else f
            elif t == Types.STRING:
                rep = "" if fill == "str_type_empty" else fill
            elif t == Types.BOOLEAN:
                if fill in ("true", "1"):
                    rep = True
                elif fill in ("false", "0"):
                    rep = False
                else:
                    raise ValueError("Missing value filling policy not correct!")
            elif t in (Types.LONG, Types.INT, Types.SHORT, Types.BYTE):
                rep = int(fill)
            else:
                rep = float(fill)
            col = mt.col(c)
            v = col.values
            if isinstance(v, torch.Tensor) and v.dim() == 1 and t != Types.STRING and \
                    getattr(t, "torch_dtype", None) is not None:
                # a tensor column stays a tensor: nulls (and NaN in a float column) take the statistic
                bad = col.nulls.to(v.device) if col.nulls is not None else torch.zeros(v.shape, dtype=torch.bool,
                                                                                         device=v.device)
                if v.is_floating_point():
                    bad = bad | torch.isnan(v)
                r = torch.where(bad, torch.tensor(rep, dtype=v.dtype, device=v.device), v)
                out.append(Column(r.to(t.torch_dtype)))
                continue
            out.append(Column.from_values([rep if (x is None or (isinstance(x, float) and x != x)) else x
                                           for x in col.to_list()], t))
        return out


# ---------------------------------------------------------------------------------------------------
# vector variants
# ---------------------------------------------------------------------------------------------------
def train_vector_scaler(kind: str, mt: MTable, params: Params, env) -> MTable:
    vc = params.get("selectedCol")
    vs = vector_summary(mt, vc, env.device)
    n = vs.vectorSize()
    meta = Params().set("selectedCol", vc)
    if kind == "standard":
        wm, ws = bool(_pget(params, "withMean", True)), bool(_pget(params, "withStd", True))
        mean = vs._sum / max(vs.count, 1) if wm else np.zeros(n)
        var = np.maximum(0.0, (vs._s2 - vs._sum ** 2 / max(vs.count, 1)) / max(vs.count - 1, 1))
        std = np.sqrt(var) if ws else np.ones(n)
        meta.set("withMean", wm).set("withStd", ws)
        arrays = [mean, std]
    elif kind == "minmax":
        meta.set("min", float(_pget(params, "min", 0.0))).set("max", float(_pget(params, "max", 1.0)))
        arrays = [vs._mn, vs._mx]
    elif kind == "maxabs":
        arrays = [np.maximum(np.abs(vs._mn), np.abs(vs._mx))]
    elif kind == "imputer":
        strategy = str(getattr(_pget(params, "strategy", "MEAN"), "name", _pget(params, "strategy", "MEAN"))).upper()
        meta.set("strategy", strategy)
        if strategy == "MIN":
            arrays = [vs._mn]
        elif strategy == "MAX":
            arrays = [vs._mx]
        elif strategy == "MEAN":
            arrays = [vs._sum / max(vs.count, 1)]
        else:
            meta.set("fillValue", str(_pget(params, "fillValue")))
            arrays = [None]
    else:
        raise ValueError(kind)
    conv = ScalerConverter()
    return MTable.from_rows(conv.save(ScalerModelData(kind, meta, arrays, None)), conv.getModelSchema(),
                            replicated=True)


class VectorScalerModelMapper(ModelMapper):
    """Vector standard / min-max / max-abs scaling, batched on the device for dense vector blocks."""

    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        self.vc = _pget(self.params, "selectedCol")
        self.out = _pget(self.params, "outputCol") or self.vc
        self.helper = OutputColsHelper(dataSchema, [self.out], [Types.VECTOR], _pget(self.params, "reservedCols"))

    def loadModel(self, modelRows):
        self.model = ScalerConverter().load(modelRows)
        if self.vc is None:
            self.vc = self.model.meta.get("selectedCol")
            self.out = _pget(self.params, "outputCol") or self.vc
            self.helper = OutputColsHelper(self.dataSchema, [self.out], [Types.VECTOR],
                                           _pget(self.params, "reservedCols"))

    def _scale(self, X: torch.Tensor) -> torch.Tensor:
        m = self.model
        a = [torch.as_tensor(x, dtype=torch.float64, device=X.device) if x is not None else None for x in m.arrays]
        d = X.shape[1]
        if X.is_cuda and m.kind in ("standard", "minmax", "maxabs"):   # K27: one fused pass over the block
            if m.kind == "minmax":
                return ew.col_transform(X, "minmax", a[0][:d], a[1][:d], float(m.meta.get("min")),
                                        float(m.meta.get("max")))
            return ew.col_transform(X, m.kind, a[0][:d], a[1][:d] if m.kind == "standard" else None)
        if m.kind == "standard":
            mean, std = a[0][:d], a[1][:d]
            return torch.where(std > 0, (X - mean) / torch.where(std > 0, std, torch.ones_like(std)),
                               torch.zeros_like(X))
        if m.kind == "minmax":
            lo, hi = float(m.meta.get("min")), float(m.meta.get("max"))
            emin, emax = a[0][:d], a[1][:d]
            rng = emax - emin
            return torch.where(rng != 0, (X - emin) / torch.where(rng != 0, rng, torch.ones_like(rng)) * (hi - lo) + lo,
                               torch.full_like(X, 0.5 * (hi + lo)))
        if m.kind == "maxabs":
            mx = a[0][:d]
            return torch.where(mx == 0, X, X / torch.where(mx == 0, torch.ones_like(mx), mx))
        raise ValueError(m.kind)

    def _map_columns(self, mt):
        c = mt.col(self.vc)
        if isinstance(c.values, torch.Tensor) and c.values.dim() == 2:
            X = c.values
            return [Column(self._scale(X if X.is_cuda and X.dtype == torch.float32 else X.double()))]
        out = []
        for v in c.to_list():
            if v is None:
                out.append(None)
                continue
            vec = VectorUtil.getVector(v)
            if isinstance(vec, SparseVector) and self.model.kind == "maxabs":
                mx = self.model.arrays[0]
                vals = np.array([x / mx[i] if i < len(mx) and mx[i] != 0 else x
                                 for i, x in zip(vec.indices, vec.values)])
                out.append(SparseVector(vec.size(), vec.indices, vals))
                continue
            dense = vec.toDenseVector().data if isinstance(vec, SparseVector) else vec.data
            r = self._scale(torch.as_tensor(dense, dtype=torch.float64)[None, :])[0].numpy()
            out.append(DenseVector(r))
        return [Column(out)]


class VectorImputerModelMapper(VectorScalerModelMapper):
    def _map_columns(self, mt):
        m = self.model
        vals = m.arrays[0] if m.arrays else None
        fill = float(m.meta.get("fillValue")) if vals is None else None
        out = []
        for v in mt.col(self.vc).to_list():
            if v is None:
                out.append(None)
                continue
            vec = VectorUtil.getVector(v)
            if isinstance(vec, SparseVector):
                nv = vec.values.copy()
                for k, i in enumerate(vec.indices):
                    if nv[k] != nv[k]:
                        nv[k] = fill if vals is None else vals[i]
                out.append(SparseVector(vec.size(), vec.indices, nv))
            else:
                a = vec.data.copy()
                nan = np.isnan(a)
                a[nan] = fill if vals is None else np.asarray(vals)[:len(a)][nan]
                out.append(DenseVector(a))
        return [Column(out)]
