"""Mapper layer: row/column transforms with declared output schema.

Reference: ``A/common/mapper/{Mapper,ModelMapper,RichModelMapper,SISOMapper,MISOMapper,FlatMapper}.java`` and
``A/common/utils/OutputColsHelper.java``.  Every mapper here has two equivalent paths:

* ``map(row)`` — row-at-a-time, used by ``LocalPredictor`` (serving);
* ``map_table(mtable)`` — columnar/batched, used by ``MapBatchOp`` / ``ModelMapBatchOp`` and the stream
  micro-batch engine; hot mappers override ``_map_columns`` with tensor / HIP implementations.

A subclass implements either ``_map_row_values`` (row) or ``_map_columns`` (batch); the base class derives
the other one.
"""
from __future__ import annotations

from typing import Any, List, Optional, Sequence, Tuple

from .params import Params
from .table import Column, MTable, Row
from .types import AlinkType, TableSchema, Types

__all__ = ["OutputColsHelper", "Mapper", "ModelMapper", "SISOMapper", "MISOMapper", "FlatMapper",
           "RichModelMapper", "find_col_index", "find_col_indices"]


def find_col_index(names: Sequence[str], name: str, required: bool = True) -> int:
    names = list(names)
    if name in names:
        return names.index(name)
    low = [n.lower() for n in names]
    if name is not None and name.lower() in low:
        return low.index(name.lower())
    if required:
        raise ValueError(f"Can not find column: {name}, all columns: {names}")
    return -1


def find_col_indices(names, sel) -> List[int]:
    return [find_col_index(names, s) for s in sel]


class OutputColsHelper:
    """Result schema = reserved input columns + output columns (an output column that shares its name
    with an input column replaces it in place)."""

    def __init__(self, input_schema: TableSchema, output_names: Sequence[str], output_types: Sequence[AlinkType],
                 reserved_names: Optional[Sequence[str]] = None):
        if isinstance(output_names, str):
            output_names = [output_names]
            output_types = [output_types] if isinstance(output_types, AlinkType) else list(output_types)
        self.in_names = list(input_schema.names)
        self.in_types = list(input_schema.types)
        self.out_names = list(output_names)
        self.out_types = list(output_types)
        keep = set(self.in_names if reserved_names is None else reserved_names)
        self.out_pos = [-1] * len(self.out_names)
        self.reserved_idx: List[int] = []
        self.reserved_pos: List[int] = []
        idx = 0
        for i, n in enumerate(self.in_names):
            if n in self.out_names:
                self.out_pos[self.out_names.index(n)] = idx
                idx += 1
                continue
            if n in keep:
                self.reserved_idx.append(i)
                self.reserved_pos.append(idx)
                idx += 1
        for k in range(len(self.out_pos)):
            if self.out_pos[k] == -1:
                self.out_pos[k] = idx
                idx += 1
        self.n_result = idx

    def getReservedColumns(self):
        return [self.in_names[i] for i in self.reserved_idx]

    def getResultSchema(self) -> TableSchema:
        names = [None] * self.n_result
        types = [None] * self.n_result
        for i, p in zip(self.reserved_idx, self.reserved_pos):
            names[p], types[p] = self.in_names[i], self.in_types[i]
        for k, p in enumerate(self.out_pos):
            names[p], types[p] = self.out_names[k], self.out_types[k]
        return TableSchema(names, types)

    def getResultRow(self, inp: Sequence[Any], out: Sequence[Any]) -> Row:
        res = [None] * self.n_result
        for i, p in zip(self.reserved_idx, self.reserved_pos):
            res[p] = inp[i]
        for k, p in enumerate(self.out_pos):
            res[p] = out[k]
        return Row(res)

    def result_table(self, inp: MTable, out_cols: List[Column]) -> MTable:
        cols: List[Optional[Column]] = [None] * self.n_result
        for i, p in zip(self.reserved_idx, self.reserved_pos):
            cols[p] = inp.cols[i]
        for k, p in enumerate(self.out_pos):
            c = out_cols[k]
            cols[p] = c if isinstance(c, Column) else Column.from_values(c, self.out_types[k])
        return MTable(self.getResultSchema(), cols, inp.replicated)


class Mapper:
    """Row/column transformer bound to an input schema and Params."""

    def __init__(self, dataSchema: TableSchema, params: Optional[Params] = None):
        self.dataSchema = dataSchema
        self.params = params.clone() if params is not None else Params()

    def getDataSchema(self) -> TableSchema:
        return self.dataSchema

    # subclasses must define the output helper (or override getOutputSchema + map_table)
    helper: OutputColsHelper = None

    def getOutputSchema(self) -> TableSchema:
        return self.helper.getResultSchema()

    def open(self):
        pass

    def close(self):
        pass

    # --- row path ---
    def map(self, row: Sequence[Any]) -> Row:
        outs = self._map_row_values(row)
        return self.helper.getResultRow(row, outs)

    def _map_row_values(self, row: Sequence[Any]) -> Sequence[Any]:
        mt = MTable.from_rows([tuple(row)], self.dataSchema)
        cols = self._map_columns(mt)
        return [c.to_list()[0] if isinstance(c, Column) else list(c)[0] for c in cols]

    # --- batch path ---
    def map_table(self, mt: MTable) -> MTable:
        return self.helper.result_table(mt, self._map_columns(mt))

    def _map_columns(self, mt: MTable) -> List[Column]:
        if type(self)._map_row_values is Mapper._map_row_values:
            raise NotImplementedError(f"{type(self).__name__} must implement _map_row_values or _map_columns")
        outs = [self._map_row_values(r) for r in mt.rows()]
        n_out = len(self.helper.out_names)
        return [Column.from_values([o[k] for o in outs], self.helper.out_types[k]) for k in range(n_out)]


class ModelMapper(Mapper):
    def __init__(self, modelSchema: TableSchema, dataSchema: TableSchema, params: Optional[Params] = None):
        super().__init__(dataSchema, params)
        self.modelSchema = modelSchema

    def getModelSchema(self):
        return self.modelSchema

    def loadModel(self, modelRows: List[Row]):
        raise NotImplementedError


class SISOMapper(Mapper):
    """Single input column -> single output column (``selectedCol``/``outputCol``/``reservedCols``)."""

    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        p = self.params
        self.selected = p.get("selectedCol") if p.contains("selectedCol") else None
        if self.selected is None and p.contains("selectedCols"):
            self.selected = p.get("selectedCols")[0]
        out = p.get("outputCol") if p.contains("outputCol") else None
        if not out:
            out = self.selected
        reserved = p.get("reservedCols") if p.contains("reservedCols") else None
        self.col_idx = find_col_index(dataSchema.names, self.selected)
        self.helper = OutputColsHelper(dataSchema, [out], [self.outputType()], reserved)

    def outputType(self) -> AlinkType:
        return Types.STRING

    def mapColumn(self, v):
        raise NotImplementedError

    def _map_row_values(self, row):
        return [self.mapColumn(row[self.col_idx])]


class MISOMapper(Mapper):
    """Multiple input columns -> single output column."""

    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        p = self.params
        self.selected = p.get("selectedCols")
        self.col_idx = find_col_indices(dataSchema.names, self.selected)
        reserved = p.get("reservedCols") if p.contains("reservedCols") else None
        self.helper = OutputColsHelper(dataSchema, [p.get("outputCol")], [self.outputType()], reserved)

    def outputType(self) -> AlinkType:
        return Types.STRING

    def mapColumns(self, vals):
        raise NotImplementedError

    def _map_row_values(self, row):
        return [self.mapColumns([row[i] for i in self.col_idx])]


class FlatMapper:
    """Row -> zero or more rows."""

    def __init__(self, dataSchema: TableSchema, params: Optional[Params] = None):
        self.dataSchema = dataSchema
        self.params = params.clone() if params is not None else Params()

    def getOutputSchema(self) -> TableSchema:
        raise NotImplementedError

    def flatMap(self, row) -> List[Row]:
        raise NotImplementedError

    def flat_map_table(self, mt: MTable) -> MTable:
        out = []
        for r in mt.rows():
            out.extend(self.flatMap(r))
        return MTable.from_rows(out, self.getOutputSchema(), mt.replicated)


class RichModelMapper(ModelMapper):
    """Prediction column + optional prediction-detail column (reference ``RichModelMapper.java:24-97``)."""

    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        p = self.params
        self.pred_col = p.get("predictionCol")
        self.detail_col = p.get("predictionDetailCol") if p.contains("predictionDetailCol") else None
        reserved = p.get("reservedCols") if p.contains("reservedCols") else None
        names = [self.pred_col] + ([self.detail_col] if self.detail_col else [])
        types = [self.predResultType()] + ([Types.STRING] if self.detail_col else [])
        self.helper = OutputColsHelper(dataSchema, names, types, reserved)

    def predResultType(self) -> AlinkType:
        return Types.STRING

    def predictResult(self, row):
        raise NotImplementedError

    def predictResultDetail(self, row) -> Tuple[Any, Optional[str]]:
        return self.predictResult(row), None

    def _map_row_values(self, row):
        if self.detail_col:
            return list(self.predictResultDetail(row))
        return [self.predictResult(row)]
