"""Format-conversion pipeline stages and the SQL ``Select`` stage.

Reference: ``A/pipeline/dataproc/format/*`` (``BaseFormatTrans`` = ``MapTransformer`` over
``FormatTransMapper`` with fixed from/to formats), ``A/pipeline/dataproc/{CsvToColumns,JsonToColumns,
KvToColumns}.java`` and ``A/pipeline/sql/Select.java``.
"""
from typing import Optional

from ..common.params import ParamInfo, Params
from ..models.dataproc import format as F
from ..operator.batch.format import FORMATS
from .base import MapTransformer, TransformerBase, register_stage

__all__ = ["BaseFormatTrans", "CsvToColumns", "JsonToColumns", "KvToColumns", "Select"]


class BaseFormatTrans(MapTransformer):
    MAPPER = F.FormatTransMapper
    EXTRA_PARAMS = [ParamInfo("fromFormat", str, "the format type of trans from", default=None),
                    ParamInfo("toFormat", str, "the format type of trans to", default=None)]
    FROM: Optional[str] = None
    TO: Optional[str] = None

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(params, **kw)
        if self.FROM is not None:
            self.getParams().set("fromFormat", self.FROM)
            self.getParams().set("toFormat", self.TO)


class CsvToColumns(MapTransformer):
    MAPPER = F.CsvToColumnsMapper


class JsonToColumns(MapTransformer):
    MAPPER = F.JsonToColumnsMapper


class KvToColumns(MapTransformer):
    MAPPER = F.KvToColumnsMapper


class Select(TransformerBase):
    """``Select(clause)`` — SQL projection as a pipeline stage (batch and stream)."""

    def __init__(self, clause=None, params: Optional[Params] = None, **kw):
        if isinstance(clause, Params):
            clause, params = None, clause
        super().__init__(params, **kw)
        if clause is not None:
            self.setClause(clause)

    def transformBatch(self, input):
        from ..operator.batch.sql import SelectBatchOp
        return SelectBatchOp(self.getClause()).linkFrom(input)

    def transformStream(self, input):
        from ..operator.stream.sql import SelectStreamOp
        return SelectStreamOp(self.getClause()).linkFrom(input)


for _f in FORMATS:
    for _t in FORMATS:
        if _f == _t or _t == "Columns" and _f in ("Csv", "Json", "Kv", "Vector"):
            continue
        _n = f"{_f}To{_t}"
        _cls = type(_n, (BaseFormatTrans,), {"FROM": _f.upper(), "TO": _t.upper(), "__module__": __name__})
        register_stage(_cls)
        globals()[_n] = _cls
        __all__.append(_n)
