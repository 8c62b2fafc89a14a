"""Model-table checkpoint format.

Every model is a table ``(model_id BIGINT, model_info VARCHAR[, aux cols...])`` — reference
``A/common/model/ModelConverterUtils.java:13-329``:

* ``model_id = 1048576 * stringIndex + sliceIndex``;
* ``stringIndex 0`` holds the meta ``Params`` JSON, ``1..n`` the data strings, ``Integer.MAX_VALUE``
  auxiliary rows (e.g. label values);
* strings are cut into 32 K-char slices; loading sorts by ``model_id`` and re-joins slices.

``SimpleModelDataConverter`` (2 cols), ``LabeledModelDataConverter`` (3rd col ``label_value``) and
``RichModelDataConverter`` (extra aux columns) mirror the reference base classes.
"""
from __future__ import annotations

from typing import Any, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from ..params import Params
from ..table import LazyRows, MTable, Row
from ..types import AlinkType, TableSchema, Types

__all__ = ["SEGMENT_SIZE", "MAX_NUM_SLICES", "get_model_id", "get_string_index", "append_meta_rows",
           "append_data_rows", "append_aux_rows", "extract_meta_and_data", "extract_aux_data",
           "ModelDataConverter", "SimpleModelDataConverter", "LabeledModelDataConverter",
           "RichModelDataConverter", "AUX_STRING_INDEX"]

SEGMENT_SIZE = 32 * 1024
MAX_NUM_SLICES = 1024 * 1024
AUX_STRING_INDEX = 2147483647


def get_model_id(string_index: int, slice_index: int) -> int:
    return MAX_NUM_SLICES * string_index + slice_index


def get_string_index(model_id: int) -> int:
    return int(model_id // MAX_NUM_SLICES)


def _slices(s: str) -> List[str]:
    if s is None or len(s) == 0:
        return []
    return [s[i:i + SEGMENT_SIZE] for i in range(0, len(s), SEGMENT_SIZE)]


def _row(n_fields: int, mid: int, s: Optional[str]) -> Row:
    r = [None] * n_fields
    r[0] = mid
    r[1] = s
    return Row(r)


def append_meta_rows(meta: Optional[Params], out: List[Row], n_fields: int):
    if meta is not None:
        for i, seg in enumerate(_slices(meta.toJson())):
            out.append(_row(n_fields, get_model_id(0, i), seg))


def append_data_rows(data: Optional[Iterable[str]], out: List[Row], n_fields: int):
    if data is None:
        return
    pad = (None,) * (n_fields - 2)
    for idx, s in enumerate(data):
        if s and len(s) <= SEGMENT_SIZE:         # the common case: one segment, no slicing / helper calls
            out.append(Row((MAX_NUM_SLICES * (idx + 1), s) + pad))
            continue
        for i, seg in enumerate(_slices(s)):
            out.append(_row(n_fields, get_model_id(idx + 1, i), seg))


def append_aux_rows(aux: Optional[Iterable[Any]], out: List[Row], n_fields: int):
    if aux is None:
        return
    n_add = n_fields - 2
    for i, d in enumerate(aux):
        r = [None] * n_fields
        r[0] = get_model_id(AUX_STRING_INDEX, i)
        if isinstance(d, (tuple, list, Row)):
            for j in range(n_add):
                r[2 + j] = d[j]
        else:
            r[2] = d
        out.append(Row(r))


def _ordered(rows: Sequence[Sequence[Any]]):
    return sorted(rows, key=lambda r: int(r[0]))


def _lazy_order(rows: LazyRows):
    """(stable sort order by model_id, string index per sorted row) of a columnar model table, or None."""
    ids = rows.int_column(0) if rows.width >= 2 else None
    if ids is None:
        return None
    order = np.argsort(ids, kind="stable")
    return order, ids[order] // MAX_NUM_SLICES


def _extract_meta_and_data_lazy(rows: LazyRows):
    got = _lazy_order(rows)
    if got is None:
        return None
    order, sid = got
    info = rows.column(1)
    meta_idx = order[sid == 0]
    sel = (sid != 0) & (sid != AUX_STRING_INDEX)
    idx, ks = order[sel], sid[sel]
    keep = [k for k, i in enumerate(idx.tolist()) if info[i] is not None]
    if len(keep) != idx.size:
        idx, ks = idx[keep], ks[keep]
    il = idx.tolist()
    if ks.size <= 1 or bool(np.all(ks[1:] != ks[:-1])):
        data = [info[i] for i in il]                         # one slice per string: no joins
    else:
        cut = [0] + (np.flatnonzero(ks[1:] != ks[:-1]) + 1).tolist() + [ks.size]
        data = ["".join(info[i] for i in il[a:b]) for a, b in zip(cut[:-1], cut[1:])]
    meta_segs = [info[i] for i in meta_idx.tolist() if info[i] is not None]
    meta = Params.fromJson("".join(meta_segs)) if meta_segs else Params()
    return meta, data


def extract_meta_and_data(rows: Sequence[Sequence[Any]]) -> Tuple[Params, List[str]]:
    if isinstance(rows, LazyRows):
        got = _extract_meta_and_data_lazy(rows)
        if got is not None:
            return got
    rows = _ordered(rows)
    meta_segs: List[str] = []
    data: List[str] = []
    cur_id, cur = None, []
    for r in rows:
        sid = get_string_index(int(r[0]))
        if sid == AUX_STRING_INDEX or r[1] is None:
            continue
        if sid == 0:
            meta_segs.append(r[1])
            continue
        if cur_id is not None and sid != cur_id:
            data.append("".join(cur))
            cur = []
        cur_id = sid
        cur.append(r[1])
    if cur:
        data.append("".join(cur))
    meta = Params.fromJson("".join(meta_segs)) if meta_segs else Params()
    return meta, data


def extract_aux_data(rows: Sequence[Sequence[Any]], is_label: bool) -> List[Any]:
    if isinstance(rows, LazyRows):
        got = _lazy_order(rows)
        if got is not None:
            order, sid = got
            idx = order[sid == AUX_STRING_INDEX].tolist()
            if is_label:
                col = rows.column(2)
                return [col[i] for i in idx]
            cols = [rows.column(j) for j in range(2, rows.width)]
            return [Row(tuple(c[i] for c in cols)) for i in idx]
    out = []
    for r in _ordered(rows):
        if get_string_index(int(r[0])) == AUX_STRING_INDEX:
            out.append(r[2] if is_label else Row(tuple(r[2:])))
    return out


class ModelDataConverter:
    """save(model) -> rows;  load(rows) -> model;  getModelSchema()."""

    def getModelSchema(self) -> TableSchema:
        raise NotImplementedError

    def save(self, model) -> List[Row]:
        raise NotImplementedError

    def load(self, rows: Sequence[Sequence[Any]]):
        raise NotImplementedError

    # convenience
    def save_table(self, model) -> MTable:
        return MTable.from_rows(self.save(model), self.getModelSchema(), replicated=True)


class SimpleModelDataConverter(ModelDataConverter):
    def serializeModel(self, model) -> Tuple[Params, Iterable[str]]:
        raise NotImplementedError

    def deserializeModel(self, meta: Params, data: List[str]):
        raise NotImplementedError

    def getModelSchema(self):
        return TableSchema(["model_id", "model_info"], [Types.LONG, Types.STRING])

    @staticmethod
    def rows_from(meta: Params, data: Iterable[str]) -> List[Row]:
        """Model rows of the default ``(model_id, model_info)`` schema from a meta + data strings."""
        out: List[Row] = []
        append_meta_rows(meta, out, 2)
        append_data_rows(data, out, 2)
        return out

    @staticmethod
    def split_rows(rows) -> Tuple[Params, List[str]]:
        return extract_meta_and_data(rows)

    def save(self, model):
        meta, data = self.serializeModel(model)
        out: List[Row] = []
        append_meta_rows(meta, out, 2)
        append_data_rows(data, out, 2)
        return out

    def load(self, rows):
        meta, data = extract_meta_and_data(rows)
        return self.deserializeModel(meta, data)


class LabeledModelDataConverter(ModelDataConverter):
    def __init__(self, label_type: Optional[AlinkType] = None):
        self.labelType = label_type

    def serializeModel(self, model) -> Tuple[Params, Iterable[str], Iterable[Any]]:
        raise NotImplementedError

    def deserializeModel(self, meta: Params, data: List[str], labels: List[Any]):
        raise NotImplementedError

    def getModelSchema(self):
        if self.labelType is None:
            raise ValueError("label type is null.")
        return TableSchema(["model_id", "model_info", "label_value"], [Types.LONG, Types.STRING, self.labelType])

    def save(self, model):
        meta, data, labels = self.serializeModel(model)
        out: List[Row] = []
        append_meta_rows(meta, out, 3)
        append_data_rows(data, out, 3)
        append_aux_rows(labels, out, 3)
        return out

    def load(self, rows):
        meta, data = extract_meta_and_data(rows)
        labels = extract_aux_data(rows, True)
        return self.deserializeModel(meta, data, labels)


class RichModelDataConverter(ModelDataConverter):
    def additionalColNames(self) -> List[str]:
        raise NotImplementedError

    def additionalColTypes(self) -> List[AlinkType]:
        raise NotImplementedError

    def serializeModel(self, model) -> Tuple[Params, Iterable[str], Iterable[Sequence[Any]]]:
        raise NotImplementedError

    def deserializeModel(self, meta: Params, data: List[str], aux: List[Row]):
        raise NotImplementedError

    def getModelSchema(self):
        return TableSchema(["model_id", "model_info"] + list(self.additionalColNames()),
                           [Types.LONG, Types.STRING] + list(self.additionalColTypes()))

    def save(self, model):
        meta, data, aux = self.serializeModel(model)
        n = 2 + len(self.additionalColNames())
        out: List[Row] = []
        append_meta_rows(meta, out, n)
        append_data_rows(data, out, n)
        append_aux_rows(aux, out, n)
        return out

    def load(self, rows):
        meta, data = extract_meta_and_data(rows)
        return self.deserializeModel(meta, data, extract_aux_data(rows, False))
