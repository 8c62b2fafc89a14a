"""Format-conversion batch ops: ``XToYBatchOp`` for X, Y in {Columns, Csv, Json, Kv, Vector}, ``XToTriple``,
``TripleToX``, the schema-driven ``CsvToColumns``/``JsonToColumns``/``KvToColumns`` and ``JsonValue``.

Reference: ``A/operator/batch/dataproc/format/*`` (``BaseFormatTransBatchOp`` = ``MapBatchOp`` over
``FormatTransMapper`` with fixed ``fromFormat``/``toFormat``; ``AnyToTripleBatchOp`` = ``FlatMapBatchOp`` over
``AnyToTripleFlatMapper``; ``TripleToAnyBatchOp.java`` groups triples by row and writes each group) and
``A/operator/batch/dataproc/{CsvToColumns,JsonToColumns,KvToColumns,JsonValue}BatchOp.java``.
Row-local conversions run on each rank's partition; ``TripleToAny`` gathers the triples, groups them once and
keeps this rank's block of the grouped rows (like the SQL global ops).
"""
from __future__ import annotations

from typing import Optional

from ...common.params import ParamInfo, Params
from ...common.table import MTable
from ...common.types import TableSchema
from ...models.dataproc import format as F
from ...parallel import comm
from ..base import BatchOperator, gather_table, partition_bounds
from .utils import FlatMapBatchOp, MapBatchOp

FORMATS = ["Columns", "Csv", "Json", "Kv", "Vector"]

__all__ = ["BaseFormatTransBatchOp", "AnyToTripleBatchOp", "TripleToAnyBatchOp", "CsvToColumnsBatchOp",
           "JsonToColumnsBatchOp", "KvToColumnsBatchOp", "JsonValueBatchOp"]


def _all_format_params():
    """Every column / schema param of the concrete X-to-Y ops: the generic ops (BaseFormatTrans, AnyToTriple,
    TripleToAny) take any source and target format, so they accept all of them."""
    from ...params import op_params
    seen = {}
    for f in FORMATS + ["Triple"]:
        for t in FORMATS + ["Triple"]:
            for p in op_params(f"{f}To{t}BatchOp"):
                seen.setdefault(p.name, p)
    return list(seen.values())


def format_ctor_args(args):
    """The reference's format-op constructors take the FormatType(s) first: ``BaseFormatTransBatchOp(from, to,
    params)``, ``AnyToTripleBatchOp(from, params)``, ``TripleToAnyBatchOp(to, params)``.  -> (format names,
    params)."""
    fmts, params = [], None
    for a in args:
        if a is None or isinstance(a, Params):
            params = a
        else:
            fmts.append(str(getattr(a, "name", a)).upper())
    return fmts, params


class BaseFormatTransBatchOp(MapBatchOp):
    """Generic ``fromFormat`` -> ``toFormat`` conversion (``BaseFormatTransBatchOp.java``)."""
    MAPPER = F.FormatTransMapper
    EXTRA_PARAMS = [ParamInfo("fromFormat", str, "the format type of trans from", default=None),
                    ParamInfo("toFormat", str, "the format type of trans to", default=None)] + _all_format_params()
    FROM: Optional[str] = None
    TO: Optional[str] = None

    def __init__(self, *args, **kw):
        fmts, params = format_ctor_args(args)
        super().__init__(params, **kw)
        if self.FROM is not None:
            self.getParams().set("fromFormat", self.FROM)
            self.getParams().set("toFormat", self.TO)
        if len(fmts) == 2:
            self.getParams().set("fromFormat", fmts[0]).set("toFormat", fmts[1])


class AnyToTripleBatchOp(FlatMapBatchOp):
    """Row -> (reserved cols, key, value) rows (``AnyToTripleBatchOp.java``)."""
    MAPPER = F.AnyToTripleFlatMapper
    EXTRA_PARAMS = BaseFormatTransBatchOp.EXTRA_PARAMS
    FROM: Optional[str] = None

    def __init__(self, *args, **kw):
        fmts, params = format_ctor_args(args)
        super().__init__(params, **kw)
        if self.FROM is not None:
            self.getParams().set("fromFormat", self.FROM)
        if fmts:
            self.getParams().set("fromFormat", fmts[0])


class TripleToAnyBatchOp(BatchOperator):
    """Group ``(tripleRowCol, tripleColCol, tripleValCol)`` by row and write each group (``TripleToAnyBatchOp.java``)."""
    EXTRA_PARAMS = BaseFormatTransBatchOp.EXTRA_PARAMS
    TO: Optional[str] = None

    def __init__(self, *args, **kw):
        fmts, params = format_ctor_args(args)
        super().__init__(params, **kw)
        if self.TO is not None:
            self.getParams().set("toFormat", self.TO)
        if fmts:
            self.getParams().set("toFormat", fmts[0])

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        rc, cc, vc = p.get("tripleRowCol"), p.get("tripleColCol"), p.get("tripleValCol")
        full = mt if (mt.replicated or comm.get_world_size() == 1) else gather_table(mt)
        sel = full.select([rc, cc, vc])
        names, types, rows = F.triple_to_any_rows(sel.rows(), p)
        schema = TableSchema([rc] + list(names), [full.col_type(rc)] + list(types))
        out = MTable.from_rows(rows, schema)
        if not mt.replicated and comm.get_world_size() > 1:
            lo, hi = partition_bounds(out.num_rows, self.env)
            out = out.slice(lo, hi)
            out.replicated = False
        else:
            out.replicated = mt.replicated
        self.setOutputTable(out)
        return self


class CsvToColumnsBatchOp(MapBatchOp):
    """CSV string column -> typed columns by ``schemaStr`` (``StringToColumnsMappers.CsvToColumnsMapper``)."""
    MAPPER = F.CsvToColumnsMapper
    EXTRA_PARAMS = [ParamInfo("selectedCol", str, "Name of the selected column", default=None),
                    ParamInfo("fieldDelimiter", str, "Field delimiter", default=None)]


class JsonToColumnsBatchOp(MapBatchOp):
    MAPPER = F.JsonToColumnsMapper
    EXTRA_PARAMS = [ParamInfo("selectedCol", str, "Name of the selected column", default=None)]


class KvToColumnsBatchOp(MapBatchOp):
    MAPPER = F.KvToColumnsMapper
    EXTRA_PARAMS = [ParamInfo("selectedCol", str, "Name of the selected column", default=None),
                    ParamInfo("colDelimiter", str, "Delimiter between key-value pairs", default=None),
                    ParamInfo("valDelimiter", str, "Delimiter between key and value", default=None)]


class JsonValueBatchOp(MapBatchOp):
    """``jsonPath`` extraction into string columns (``JsonValueBatchOp`` / ``JsonPathMapper.java``)."""
    MAPPER = F.JsonPathMapper


def _make(name, base, attrs):
    cls = type(name, (base,), dict(attrs, __module__=__name__,
                                   __doc__=f"{name}: " + ", ".join(f"{k}={v}" for k, v in attrs.items())))
    globals()[name] = cls
    __all__.append(name)
    return cls


for _f in FORMATS:
    for _t in FORMATS:
        if _f == _t or (_f, _t) in (("Csv", "Columns"), ("Json", "Columns"), ("Kv", "Columns"), ("Vector", "Columns")):
            continue
        _make(f"{_f}To{_t}BatchOp", BaseFormatTransBatchOp, {"FROM": _f.upper(), "TO": _t.upper()})
    _make(f"{_f}ToTripleBatchOp", AnyToTripleBatchOp, {"FROM": _f.upper()})
    _make(f"TripleTo{_f}BatchOp", TripleToAnyBatchOp, {"TO": _f.upper()})
