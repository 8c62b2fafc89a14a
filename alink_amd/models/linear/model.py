"""Linear model data, its table format and the prediction mappers.

Reference: ``A/operator/common/linear/{LinearModelData,LinearModelDataConverter,LinearModelMapper,
SoftmaxModelMapper}.java``, ``A/operator/common/regression/AFTModelMapper.java``.

Model table = ``LabeledModelDataConverter`` layout: meta row (modelName, hasInterceptItem, linearModelType,
[vectorCol, vectorSize], labelCol), one data row with the Gson JSON of ``ModelData``
(``featureColNames``, ``featureColTypes``, ``coefVector``, ``coefVectors``; nulls written) and the label
values as auxiliary rows in the ``label_value`` column.  Also loaded: label values carried in the meta
(``labelValues``, ``LinearModelDataConverter.java:61-64``), and the legacy 4-column format still written by
PAI online learning (``LinearModelDataConverter.java:77-85`` -> ``LinearModelData.loadOldFromatModel``
``:116-157``): meta JSON at id 0, the data JSON split over ids 1.., labels recovered from the meta
``labelValues`` typed by ``labelTypeName``.

Prediction is batched: the partition's features become one FeatureMatrix and margins are a single GEMV
(GEMM for softmax) on the device; detail strings are formatted on the host.
"""
from __future__ import annotations

import json
import math
from typing import Any, List, Optional, Sequence

import numpy as np
import torch

from ...common.javafmt import gson_dumps, java_double_str, java_hashmap_order
from ...common.detail import DetailBlock
from ...common.linalg import DenseVector
from ...common.mapper import RichModelMapper
from ...common.model.converter import LabeledModelDataConverter
from ...common.params import ParamInfo, Params
from ...common.table import Column, MTable
from ...common.types import AlinkType, TableSchema, Types
from ...params import get_enum
from ..common.features import FeatureMatrix, extract_features

__all__ = ["LinearModelType", "LinearModelData", "LinearModelDataConverter", "LinearModelMapper",
           "SoftmaxModelMapper", "AFTModelMapper", "MODEL_NAME", "HAS_INTERCEPT_ITEM", "LINEAR_MODEL_TYPE",
           "VECTOR_COL", "VECTOR_SIZE", "LABEL_COL", "linear_feature_type_name"]

LinearModelType = get_enum("LinearModelType")

# ModelParamName.java
MODEL_NAME = ParamInfo("modelName", str, "model name")
HAS_INTERCEPT_ITEM = ParamInfo("hasInterceptItem", bool, "has intercept", default=True)
LINEAR_MODEL_TYPE = ParamInfo("linearModelType", LinearModelType, "linear model type")
VECTOR_COL = ParamInfo("vectorCol", str, "vector column")
VECTOR_SIZE = ParamInfo("vectorSize", int, "vector size")
LABEL_COL = ParamInfo("labelCol", str, "label column")
NUM_CLASSES = ParamInfo("numClasses", int, "number of classes")
LABEL_VALUES = "labelValues"                                      # ModelParamName.LABEL_VALUES (Object[])
LABEL_TYPE_NAME = ParamInfo("labelTypeName", str, "label type name", alias=("labelType",))
IS_OLD_FORMAT = ParamInfo("isOldFormat", bool, "legacy 4-column model")

_TYPE_NAMES = {Types.DOUBLE: "double", Types.FLOAT: "float", Types.LONG: "long", Types.INT: "int",
               Types.SHORT: "short", Types.BOOLEAN: "bool", Types.BYTE: "byte", Types.DECIMAL: "double"}


def linear_feature_type_name(t: AlinkType) -> str:
    if t not in _TYPE_NAMES:
        raise ValueError(f"linear algorithm only support numerical data type. type is : {t}")
    return _TYPE_NAMES[t]


class _ModelDataJson:
    __gson_fields__ = ("featureColNames", "featureColTypes", "coefVector", "coefVectors")

    def __init__(self, names=None, types=None, coef=None, coefs=None):
        self.featureColNames, self.featureColTypes = names, types
        self.coefVector, self.coefVectors = coef, coefs


class LinearModelData:
    def __init__(self):
        self.featureNames: Optional[List[str]] = None
        self.featureTypes: Optional[List[str]] = None
        self.vectorColName: Optional[str] = None
        self.coefVector: Optional[DenseVector] = None
        self.coefVectors: Optional[List[DenseVector]] = None
        self.vectorSize: int = 0
        self.modelName: Optional[str] = None
        self.labelName: Optional[str] = None
        self.labelValues: Optional[List[Any]] = None
        self.linearModelType = None
        self.hasInterceptItem: bool = True
        self.lossCurve: Optional[np.ndarray] = None
        self.labelType: Optional[AlinkType] = None


class LinearModelDataConverter(LabeledModelDataConverter):
    def __init__(self, label_type: Optional[AlinkType] = None):
        super().__init__(label_type)

    @staticmethod
    def extractLabelType(model_schema: TableSchema) -> Optional[AlinkType]:
        return model_schema.types[2] if len(model_schema.types) > 2 else None

    def serializeModel(self, m: LinearModelData):
        meta = Params()
        meta.set(MODEL_NAME, m.modelName)
        meta.set(HAS_INTERCEPT_ITEM, bool(m.hasInterceptItem))
        meta.set(LINEAR_MODEL_TYPE, m.linearModelType)
        if m.vectorColName is not None:
            meta.set(VECTOR_COL, m.vectorColName)
            meta.set(VECTOR_SIZE, int(m.vectorSize))
        meta.set(LABEL_COL, m.labelName)
        data = gson_dumps(_ModelDataJson(m.featureNames, m.featureTypes, m.coefVector, m.coefVectors))
        return meta, [data], (list(m.labelValues) if m.labelValues is not None else None)

    def deserializeModel(self, meta: Params, data: List[str], labels: List[Any]) -> LinearModelData:
        m = LinearModelData()
        m.modelName = meta.get(MODEL_NAME)
        m.linearModelType = meta.get(LINEAR_MODEL_TYPE) if meta.contains(LINEAR_MODEL_TYPE) else None
        m.hasInterceptItem = meta.get(HAS_INTERCEPT_ITEM) if meta.contains(HAS_INTERCEPT_ITEM) else True
        m.vectorSize = meta.get(VECTOR_SIZE) if meta.contains(VECTOR_SIZE) else 0
        m.vectorColName = meta.get(VECTOR_COL) if meta.contains(VECTOR_COL) else None
        m.labelName = meta.get(LABEL_COL) if meta.contains(LABEL_COL) else None
        m.labelType = self.labelType
        m.labelValues = None
        if meta.contains(LABEL_VALUES):
            raw = meta.get(LABEL_VALUES)
            if isinstance(raw, str):
                raw = json.loads(raw)
            m.labelValues = [_recover_label(v, m.labelType) for v in raw] if raw is not None else None
        if labels:
            # the auxiliary label rows win (the reference overrides the meta values with them; an EMPTY aux
            # list keeps the meta values here instead of erasing them)
            m.labelValues = list(labels)
        if len(data) != 1:
            raise RuntimeError("Not valid model.")
        d, coef = _split_coef_json(data[0])
        m.featureNames = d.get("featureColNames")
        m.featureTypes = d.get("featureColTypes")
        cv = d.get("coefVector")
        if coef is not None:
            m.coefVector = DenseVector(coef)
        else:
            m.coefVector = DenseVector(np.asarray(cv["data"], dtype=np.float64)) if cv else None
        if m.modelName == "softmax" and m.coefVector is not None:
            w = m.coefVector.data
            K = len(m.labelValues)
            mm = len(w) // (K - 1)
            m.coefVectors = [DenseVector(w[k * mm:(k + 1) * mm].copy()) for k in range(K - 1)]
        return m

    def load(self, rows):
        rows = [tuple(r) for r in rows]
        if rows and len(rows[0]) == 4:         # old format model, still used in PAI online learning
            return self._load_old_format(rows)
        return super().load(rows)

    def _load_old_format(self, rows) -> LinearModelData:
        """``LinearModelData.loadOldFromatModel``: rows (id, string, *, *); id 0 = meta JSON, ids 1..m-1 = the
        data JSON in pieces, concatenated in id order up to the first missing id."""
        from ...common.types import type_from_str
        m = len(rows)
        meta_str, pieces = "", [None] * m
        for r in rows:
            idx = int(r[0])
            if idx == 0:
                meta_str = r[1]
            elif 1 <= idx <= m:
                pieces[idx - 1] = r[1]
        buf = []
        for p in pieces:
            if p is None:
                break
            buf.append(p)
        meta = Params.fromJson(meta_str)
        meta.set(IS_OLD_FORMAT, True)
        # recoverLabelsFromOldFormatModel: the label type is the meta's Flink type string
        label_type = type_from_str(meta.get(LABEL_TYPE_NAME)) if meta.contains(LABEL_TYPE_NAME) else self.labelType
        conv = LinearModelDataConverter(label_type)
        return conv.deserializeModel(meta, ["".join(buf)], [])


_COEF_KEY = '"coefVector":{"data":['


def _split_coef_json(s: str):
    """(model JSON dict, coefficients or None): a large coefficient array is cut out of the string and parsed by the
    C++ number reader (``_native.parse_double_csv``; ~10x json.loads for 1e6 values), the rest by json.loads.
    Small models, special values (NaN / Infinity) or another layout take plain json.loads."""
    i = s.find(_COEF_KEY) if len(s) > 100_000 else -1
    if i >= 0:
        a = i + len(_COEF_KEY)
        b = s.find("]", a)
        if b > a:
            from ... import _native
            coef = _native.parse_double_csv(s[a:b])
            if coef is not None:
                return json.loads(s[:a] + s[b:]), coef
    return json.loads(s), None


def _recover_label(v, t: Optional[AlinkType]):
    if v is None or t is None:
        return v
    if t in (Types.LONG, Types.INT, Types.SHORT, Types.BYTE):
        return int(float(v)) if isinstance(v, str) else int(v)
    if t in (Types.DOUBLE, Types.FLOAT, Types.DECIMAL):
        return float(v)
    if t == Types.BOOLEAN:
        return v if isinstance(v, bool) else str(v).lower() == "true"
    return str(v) if t == Types.STRING else v


class _LinearMapperBase(RichModelMapper):
    """Shared feature handling (``FeatureLabelUtil.getFeatureVector``)."""
    model: Optional[LinearModelData] = None

    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        p = self.params
        self.vector_col = p.get("vectorCol") if p.contains("vectorCol") and p.get("vectorCol") else None
        self.model: Optional[LinearModelData] = None

    def predResultType(self):
        if self.model is not None and self.model.labelType is not None and not self._is_regression():
            return self.model.labelType
        return Types.DOUBLE if self._is_regression() else (self.modelSchema.types[2]
                                                           if len(self.modelSchema.types) > 2 else Types.STRING)

    def _is_regression(self) -> bool:
        return False

    def loadModel(self, modelRows):
        conv = LinearModelDataConverter(LinearModelDataConverter.extractLabelType(self.modelSchema))
        self.model = conv.load(modelRows)
        if self.model.labelType is None:
            self.model.labelType = conv.labelType
        if self.model.labelValues is not None:
            self.model.labelValues = [_recover_label(v, self.model.labelType) for v in self.model.labelValues]
        if self.vector_col is None and self.model.featureNames is None:
            self.vector_col = self.model.vectorColName
        # rebuild helper with the resolved prediction type
        from ...common.mapper import OutputColsHelper
        names = [self.pred_col] + ([self.detail_col] if self.detail_col else [])
        types = [self.predResultType()] + ([Types.STRING] if self.detail_col else [])
        reserved = self.params.get("reservedCols") if self.params.contains("reservedCols") else None
        self.helper = OutputColsHelper(self.dataSchema, names, types, reserved)

    def swapCoef(self, w) -> None:
        """Hot swap of the coefficient vector of a loaded model (online learning snapshots with unchanged
        meta and labels)."""
        self.model.coefVector = DenseVector(np.asarray(w, dtype=np.float64))
        self._coef_cache = None

    def _coef(self, dev) -> torch.Tensor:
        """The coefficient vector on ``dev``, cached until the model changes (no per-batch H2D copy of a
        1e6-dim vector in a serving loop)."""
        cv = self.model.coefVector
        c = getattr(self, "_coef_cache", None)
        if c is None or c[0] is not cv or c[1].device != dev:
            c = (cv, torch.as_tensor(cv.data, dtype=torch.float64, device=dev))
            self._coef_cache = c
        return c[1]

    def _features(self, mt: MTable) -> FeatureMatrix:
        m = self.model
        fm = extract_features(mt, m.featureNames if self.vector_col is None else None, self.vector_col,
                              torch.device("cpu") if not _on_gpu(mt) else _dev(mt))
        if fm.is_sparse and m.vectorSize:   # SparseVector.setSize(vectorSize); dense vectors keep their size
            fm.set_ncols(m.vectorSize)
        return fm.prefix_one() if m.hasInterceptItem else fm

    def _map_row_values(self, row):
        mt = MTable.from_rows([tuple(row)], self.dataSchema)
        cols = self._map_columns(mt)
        return [c.to_list()[0] for c in cols]


def _on_gpu(mt: MTable) -> bool:
    return any(isinstance(c.values, torch.Tensor) and c.values.is_cuda for c in mt.cols)


def _dev(mt: MTable):
    for c in mt.cols:
        if isinstance(c.values, torch.Tensor) and c.values.is_cuda:
            return c.values.device
    return torch.device("cpu")


def label_column(labels: Sequence[Any], idx, t) -> Column:
    """``[labels[i] for i in idx]`` as a column of type ``t`` without a per-row list: a tensor gather for numeric
    labels, a ``StringBlock`` take for string labels (a list of python values otherwise)."""
    idx = np.asarray(idx, dtype=np.int64)
    it = torch.from_numpy(idx)
    if t.torch_dtype is not None and t.py in (int, float) and labels and \
            all(isinstance(v, (int, float)) and not isinstance(v, bool) for v in labels):
        return Column(torch.tensor(list(labels), dtype=t.torch_dtype)[it])
    if t == Types.STRING and labels and all(isinstance(v, str) for v in labels):
        from ...common.strings import StringBlock
        return Column(StringBlock.from_list(list(labels)).take(it))
    lab = np.empty(len(labels), dtype=object)
    lab[:] = list(labels)
    return Column.from_values(lab[idx].tolist(), t)


def _detail_json(labels: Sequence[Any], probs: np.ndarray, quoted: bool = True) -> List[str]:
    """HashMap<String,String> of label -> Double.toString(prob), Gson-serialised in Java HashMap order
    (``quoted`` False: HashMap<String,Double>, the same digits as JSON numbers — the tree mappers' detail).
    Batched: every probability is formatted by the C++ Double.toString twin in one call and the rows are
    assembled from one per-table template (the keys and their order are the same on every row)."""
    from ... import _native
    keys = [str(l) for l in labels]
    order = java_hashmap_order(keys)
    probs = np.asarray(probs, dtype=np.float64)
    cols = [keys.index(k) for k in order]
    body = _native.java_double_join(np.ascontiguousarray(probs[:, cols]).reshape(-1)) if probs.size else ""
    if body is None:
        if not quoted:
            return [gson_dumps({k: float(row[keys.index(k)]) for k in order}, java_map_order=True) for row in probs]
        return [gson_dumps({k: java_double_str(float(row[keys.index(k)])) for k in order}, java_map_order=True)
                for row in probs]
    strs = body.split(",") if probs.size else []
    K = len(order)
    val = ':"%s"' if quoted else ':%s'
    tmpl = "{" + ",".join(gson_dumps(k).replace("%", "%%") + val for k in order) + "}"
    return [tmpl % tuple(strs[i * K:(i + 1) * K]) for i in range(probs.shape[0])]


class LinearModelMapper(_LinearMapperBase):
    """LR / SVM / Perceptron -> label (margin >= 0 -> labelValues[0]); LinearReg / SVR -> margin."""

    def _is_regression(self):
        t = self.model.linearModelType if self.model is not None else None
        return t is not None and t.name in ("LinearReg", "SVR")

    def _map_columns(self, mt):
        m = self.model
        fm = self._features(mt)
        coef = self._coef(fm.device)
        if mt.num_rows and fm.device.type == "cuda":
            dev_cols = self._map_columns_device(fm.mv(coef))
            if dev_cols is not None:
                return dev_cols
        dot = fm.mv(coef).cpu().numpy() if mt.num_rows else np.zeros(0)
        tname = m.linearModelType.name
        out = []
        if tname in ("LinearReg", "SVR"):
            out.append(Column(torch.from_numpy(dot.copy())))
        else:
            lv = m.labelValues
            t = self.helper.out_types[0]
            if t.torch_dtype is not None and all(isinstance(x, (int, float)) and not isinstance(x, bool) for x in lv):
                preds = torch.where(torch.from_numpy(dot >= 0), torch.tensor(lv[0], dtype=t.torch_dtype),
                                    torch.tensor(lv[1], dtype=t.torch_dtype))
                out.append(Column(preds))
            else:
                out.append(label_column(lv, np.where(dot >= 0, 0, 1), t))
        if self.detail_col:
            if tname in ("LR", "SVM"):
                prob = 1.0 - 1.0 / (1.0 + np.exp(dot))
                # columnar detail: strings are formatted only if a consumer reads them (common/detail.py)
                out.append(Column(DetailBlock(m.labelValues, np.stack([prob, 1 - prob], 1))))
            else:
                out.append(Column([None] * mt.num_rows))
        return out


    def _map_columns_device(self, dot: torch.Tensor):
        """GPU scoring without a host round trip: margins, labels and the detail block stay device tensors (a
        scoring -> evaluation stream reads them there).  None when the labels are not numeric (host path)."""
        m = self.model
        tname = m.linearModelType.name
        if tname in ("LinearReg", "SVR"):
            out = [Column(dot)]
        else:
            lv = m.labelValues
            t = self.helper.out_types[0]
            if t.torch_dtype is None or not all(isinstance(x, (int, float)) and not isinstance(x, bool) for x in lv):
                return None
            # filled on the device from Python scalars: no per-batch host -> device copies of the label values
            out = [Column(torch.full(dot.shape, lv[1], dtype=t.torch_dtype, device=dot.device)
                          .masked_fill_(dot >= 0, lv[0]))]
        if self.detail_col:
            if tname in ("LR", "SVM"):
                prob = 1.0 - 1.0 / (1.0 + torch.exp(dot))
                out.append(Column(DetailBlock(m.labelValues, torch.stack([prob, 1 - prob], 1), trusted=True)))
            else:
                out.append(Column([None] * int(dot.shape[0])))
        return out


class SoftmaxModelMapper(_LinearMapperBase):
    def _map_columns(self, mt):
        m = self.model
        fm = self._features(mt)
        W = torch.as_tensor(np.stack([c.data for c in m.coefVectors]), dtype=torch.float64, device=fm.device)
        eta = fm.mm(W.T).cpu().numpy() if mt.num_rows else np.zeros((0, W.shape[0]))
        K = len(m.labelValues)
        out = []
        if self.detail_col:
            e = np.exp(eta)
            s = 1.0 + e.sum(1, keepdims=True)
            probs = np.concatenate([e, np.ones((e.shape[0], 1))], 1) / s
            idx = probs.argmax(1)
            out.append(label_column(m.labelValues, idx, self.helper.out_types[0]))
            out.append(Column(_detail_json(m.labelValues, probs)))
        else:
            # predictResult: argmax over k < K-1 of eta with a 0.0 floor -> pivot class K-1
            best = np.full(eta.shape[0], K - 1)
            bval = np.zeros(eta.shape[0])
            for k in range(K - 1):
                better = eta[:, k] > bval
                best[better] = k
                bval[better] = eta[better, k]
            out.append(label_column(m.labelValues, best, self.helper.out_types[0]))
        return out


class AFTModelMapper(_LinearMapperBase):
    def _is_regression(self):
        return True

    def predResultType(self):
        return Types.DOUBLE

    def _map_columns(self, mt):
        m = self.model
        fm = self._features(mt)
        coef = torch.as_tensor(m.coefVector.data, dtype=torch.float64, device=fm.device)
        dot = np.exp(fm.mv(coef).cpu().numpy()) if mt.num_rows else np.zeros(0)
        dot = np.where(np.isinf(dot), np.finfo(np.float64).max, dot)
        out = [Column(torch.from_numpy(dot.copy()))]
        if self.detail_col:
            q = self.params.get("quantileProbabilities") if self.params.contains("quantileProbabilities") else \
                [0.01, 0.05, 0.1, 0.25, 0.5, 0.75, 0.9, 0.95, 0.99]
            scale = m.coefVector.data[-1]
            fac = np.exp(np.log(-np.log(1 - np.asarray(q, dtype=np.float64))) * scale)
            out.append(Column([DenseVector(v * fac).toString() for v in dot]))
        return out
