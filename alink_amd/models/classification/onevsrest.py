"""One-vs-rest reduction of multiclass classification to binary classifiers.

Reference: ``A/pipeline/classification/OneVsRest.java`` (labels sorted, class i trained on label==labels[i]
-> 1.0 else 0.0 :48-113, model = concatTables([meta, union of per-class models tagged ``ovr_id``, labels])
:120-156, ``TableUtil.concatTables`` layout ``table_id, t0_*, t1_*, t2_*``) and
``A/operator/common/classification/OneVsRestModelMapper.java`` (per-class positive score, argmax, detail =
scores normalised to sum 1 :164-220).  Unlike the reference (LR / LinearSvm / GBDT only) any binary
classifier whose model mapper emits a prediction-detail JSON works.
"""
from __future__ import annotations

import json
from typing import Any, List

import numpy as np

from ...common.javafmt import gson_dumps, java_hashmap_order, java_str
from ...common.mapper import ModelMapper, OutputColsHelper
from ...common.params import Params
from ...common.table import Column, MTable, Row
from ...common.types import TableSchema, Types, type_from_str

__all__ = ["OneVsRestModelMapper", "build_ovr_model_table", "JDBC_TYPE", "FLINK_TYPE_NAME"]

JDBC_TYPE = {"STRING": 12, "VARCHAR": 12, "BOOLEAN": 16, "BYTE": -6, "SHORT": 5, "INT": 4, "LONG": -5,
             "BIGINT": -5, "FLOAT": 6, "DOUBLE": 8, "DECIMAL": 3, "DATE": 91, "TIME": 92, "TIMESTAMP": 93}
_JDBC_BACK = {12: Types.STRING, 16: Types.BOOLEAN, 4: Types.INT, -5: Types.LONG, 6: Types.FLOAT, 8: Types.DOUBLE}
FLINK_TYPE_NAME = {"STRING": "VARCHAR", "LONG": "BIGINT", "INT": "INT", "DOUBLE": "DOUBLE", "FLOAT": "FLOAT",
                   "BOOLEAN": "BOOLEAN"}


def _tname(t) -> str:
    return getattr(t, "name", str(t)).upper()


def build_ovr_model_table(models: List[MTable], labels: List[Any], label_type, bin_cls_class: str,
                          bin_params: Params, num_classes: int) -> MTable:
    ms = models[0].schema
    meta = Params()
    meta.set("numClasses", int(num_classes))
    meta.set("binClsClassName", bin_cls_class)
    meta.set("binClsParams", bin_params.toJson())
    meta.set("labelTypeName", FLINK_TYPE_NAME.get(_tname(label_type), _tname(label_type)))
    meta.set("modelColNames", list(ms.names))
    meta.set("modelColTypes", [JDBC_TYPE.get(_tname(t), 12) for t in ms.types])
    meta.set("labels", gson_dumps(list(labels), java_map_order=False))
    names = ["table_id", "t0_meta", "t1_ovr_id"] + [f"t1_{n}" for n in ms.names] + [f"t2_{labels_col()}"]
    types = [Types.LONG, Types.STRING, Types.LONG] + list(ms.types) + [label_type]
    width = len(names)
    rows = []
    r = [None] * width
    r[0], r[1] = 0, meta.toJson()
    rows.append(Row(r))
    for i, m in enumerate(models):
        for mr in m.rows():
            r = [None] * width
            r[0], r[2] = 1, i
            r[3:3 + len(mr)] = list(mr)
            rows.append(Row(r))
    for lab in labels:
        r = [None] * width
        r[0], r[-1] = 2, lab
        rows.append(Row(r))
    return MTable.from_rows(rows, TableSchema(names, types), replicated=True)


def labels_col():
    return "label"


class OneVsRestModelMapper(ModelMapper):
    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        p = self.params
        self.label_type = modelSchema.types[-1]
        self.detail_col = p.get("predictionDetailCol") if p.contains("predictionDetailCol") else None
        names = [p.get("predictionCol")] + ([self.detail_col] if self.detail_col else [])
        types = [self.label_type] + ([Types.STRING] if self.detail_col else [])
        self.helper = OutputColsHelper(dataSchema, names, types,
                                       p.get("reservedCols") if p.contains("reservedCols") else None)

    def loadModel(self, modelRows):
        from ...pipeline.base import stage_class_from_java
        meta = None
        for r in modelRows:
            if r[1] is not None:
                meta = Params.fromJson(r[1])
                break
        n = int(meta.get("numClasses"))
        labels = json.loads(meta.get("labels"))
        tn = meta.get("labelTypeName").upper()
        if tn in ("BIGINT", "LONG", "INT", "INTEGER"):
            labels = [int(v) for v in labels]
        elif tn in ("DOUBLE", "FLOAT"):
            labels = [float(v) for v in labels]
        self.labels = labels
        col_names = list(meta.get("modelColNames"))
        col_types = [_JDBC_BACK.get(int(t), Types.STRING) for t in meta.get("modelColTypes")]
        ms = TableSchema(col_names, col_types)
        stage_cls = stage_class_from_java(meta.get("binClsClassName"))
        model_stage = stage_cls(Params.fromJson(meta.get("binClsParams")))
        model_cls = model_stage.MODEL if not isinstance(model_stage.MODEL, str) else None
        if model_cls is None:
            from ...pipeline.base import STAGE_REGISTRY
            model_cls = STAGE_REGISTRY[model_stage.MODEL]
        bin_params = self.params.clone()
        bin_params.set("reservedCols", [])
        bin_params.set("predictionCol", "pred_result")
        bin_params.set("predictionDetailCol", "pred_detail")
        self.predictors = []
        w = len(col_names)
        for i in range(n):
            rows = [tuple(r[3:3 + w]) for r in modelRows if r[2] is not None and int(r[2]) == i]
            mp = model_cls.MAPPER(ms, self.dataSchema, bin_params)
            mp.loadModel(rows)
            mp.open()
            self.predictors.append(mp)

    def _score(self, mp, mt: MTable) -> np.ndarray:
        out = mp.map_table(mt)
        det = out.col("pred_detail").to_list()
        s = []
        for d in det:
            m = json.loads(d)
            v = m.get("1.0", m.get("1"))
            s.append(float(v) if v is not None else 0.0)
        return np.asarray(s)

    def _map_columns(self, mt: MTable):
        S = np.stack([self._score(mp, mt) for mp in self.predictors], 1) if mt.num_rows else \
            np.zeros((0, len(self.predictors)))
        idx = S.argmax(1) if S.shape[0] else np.zeros(0, dtype=int)
        preds = [self.labels[i] for i in idx]
        outs = [Column.from_values(preds, self.label_type)]
        if self.detail_col:
            keys = java_hashmap_order([java_str(l) for l in self.labels])
            det = []
            for row in S:
                tot = row.sum()
                vals = {java_str(l): float(row[j] / tot) for j, l in enumerate(self.labels)}
                det.append(gson_dumps({k: vals[k] for k in keys}, java_map_order=False))
            outs.append(Column.from_values(det, Types.STRING))
        return outs
