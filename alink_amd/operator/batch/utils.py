"""Generic mapper-driven batch ops: ``MapBatchOp``, ``ModelMapBatchOp``, ``FlatMapBatchOp``, UDF/UDTF, Print.

Reference: ``A/operator/batch/utils/MapBatchOp.java:30-42``, ``ModelMapBatchOp.java:34-54`` (model rows as a
broadcast variable), ``FlatMapBatchOp``, ``UDFBatchOp``/``UDTFBatchOp``, ``PrintBatchOp``.
Model broadcast = gather of the (small) model table to every rank; the mapper then runs on the rank's
partition in batched (columnar) form.
"""
from __future__ import annotations

from typing import Callable, List, Optional

from ...common.mapper import FlatMapper, Mapper, ModelMapper, OutputColsHelper
from ...common.params import ParamInfo, Params
from ...common.table import Column, MTable
from ...common.types import AlinkType, TableSchema, Types, type_from_str
from ..base import BatchOperator, gather_table

__all__ = ["MapBatchOp", "ModelMapBatchOp", "FlatMapBatchOp", "UDFBatchOp", "UDTFBatchOp", "PrintBatchOp",
           "load_model_mapper"]


class MapBatchOp(BatchOperator):
    MAPPER: Callable[..., Mapper] = None

    def __init__(self, params: Optional[Params] = None, mapper: Callable[..., Mapper] = None, **kw):
        super().__init__(params, **kw)
        if mapper is not None:
            self.MAPPER = mapper

    def linkFrom(self, *inputs):
        inp = self.checkAndGetFirst(inputs)
        mt = inp.getOutputTable()
        mapper = self.MAPPER(mt.schema, self.getParams())
        mapper.open()
        self.setOutputTable(mapper.map_table(mt))
        mapper.close()
        return self


def load_model_mapper(mapper_cls, model, data_schema: TableSchema, params: Params) -> ModelMapper:
    """Build and open a ``ModelMapper`` from a model table (broadcast source), a ``ModelSource`` or a
    ``DataBridge`` (``common/directreader.py``)."""
    from ...common.directreader import model_source_of
    src = model_source_of(model)
    mapper = mapper_cls(src.getSchema(), data_schema, params)
    mapper.loadModel(src.getModelRows())
    mapper.open()
    return mapper


class ModelMapBatchOp(BatchOperator):
    MAPPER: Callable[..., ModelMapper] = None

    def __init__(self, params: Optional[Params] = None, mapper: Callable[..., ModelMapper] = None, **kw):
        super().__init__(params, **kw)
        if mapper is not None:
            self.MAPPER = mapper

    def linkFrom(self, *inputs):
        if len(inputs) == 1 and isinstance(inputs[0], (list, tuple)):
            inputs = inputs[0]
        self.checkOpSize(2, inputs)
        model_op, data_op = inputs
        data = data_op.getOutputTable()
        mapper = load_model_mapper(self.MAPPER, model_op.getOutputTable(), data.schema, self.getParams())
        mapper.env = self.env                           # device-aware mappers (tree predict) read the op's env
        self.setOutputTable(mapper.map_table(data))
        mapper.close()
        return self


class FlatMapBatchOp(BatchOperator):
    MAPPER: Callable[..., FlatMapper] = None

    def __init__(self, params: Optional[Params] = None, mapper=None, **kw):
        super().__init__(params, **kw)
        if mapper is not None:
            self.MAPPER = mapper

    def linkFrom(self, *inputs):
        inp = self.checkAndGetFirst(inputs)
        mt = inp.getOutputTable()
        mapper = self.MAPPER(mt.schema, self.getParams())
        self.setOutputTable(mapper.flat_map_table(mt))
        return self


_FUNC = ParamInfo("func", object, "python callable")
_RESULT_TYPE = ParamInfo("resultType", str, "result type of the udf", default="DOUBLE")


class _UDFMapper(Mapper):
    def __init__(self, dataSchema, params, func, result_type):
        super().__init__(dataSchema, params)
        self.func = func
        sel = self.params.get("selectedCols")
        self.idx = [dataSchema.names.index(c) for c in sel]
        reserved = self.params.get("reservedCols") if self.params.contains("reservedCols") else None
        self.helper = OutputColsHelper(dataSchema, [self.params.get("outputCol")], [result_type], reserved)

    def _map_row_values(self, row):
        f = self.func
        f = getattr(f, "eval", f)
        return [f(*[row[i] for i in self.idx])]


class UDFBatchOp(BatchOperator):
    EXTRA_PARAMS = [_RESULT_TYPE]

    def setFunc(self, f):
        self._func = f
        return self

    def getFunc(self):
        return getattr(self, "_func", None)

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        f = self.getFunc()
        rt = getattr(f, "result_type", None) or self.getParams().get(_RESULT_TYPE)
        rt = type_from_str(rt) if isinstance(rt, str) else rt
        self.setOutputTable(_UDFMapper(mt.schema, self.getParams(), f, rt).map_table(mt))
        return self


class UDTFBatchOp(BatchOperator):
    EXTRA_PARAMS = [ParamInfo("resultTypes", [str], "result types", default=None)]

    def setFunc(self, f):
        self._func = f
        return self

    def getFunc(self):
        return getattr(self, "_func", None)

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        sel = p.get("selectedCols")
        outs = p.get("outputCols")
        reserved = p.get("reservedCols") if p.contains("reservedCols") else None
        f = self.getFunc()
        from ..common.sql.udf import TableFunction
        if not isinstance(f, TableFunction):       # a TableFunction collects its rows; plain callables return them
            f = getattr(f, "eval", f)
        idx = [mt.schema.names.index(c) for c in sel]
        rts = getattr(self.getFunc(), "result_types", None) or p.get(self._param_infos["resultTypes"])
        rows_out = []
        keep = [i for i, n in enumerate(mt.schema.names) if (reserved is None or n in reserved) and n not in outs]
        for r in mt.rows():
            for o in f(*[r[i] for i in idx]) or []:
                o = o if isinstance(o, (list, tuple)) else (o,)
                rows_out.append(tuple(r[i] for i in keep) + tuple(o))
        if rts is None:
            first = rows_out[0][len(keep):] if rows_out else [None] * len(outs)
            from ...common.table import infer_type
            types = [infer_type(v) if v is not None else Types.STRING for v in first]
        else:
            types = [type_from_str(t) for t in rts]
        schema = TableSchema([mt.schema.names[i] for i in keep] + list(outs),
                             [mt.schema.types[i] for i in keep] + types)
        self.setOutputTable(MTable.from_rows(rows_out, schema))
        return self


class PrintBatchOp(BatchOperator):
    PARAMS = ()

    def linkFrom(self, *inputs):
        inp = self.checkAndGetFirst(inputs)
        self.setOutputTable(inp.getOutputTable())
        inp.print()
        return self
