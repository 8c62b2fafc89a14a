"""Stream twins of the row-local transforms: format conversion (``XToYStreamOp``, ``XToTripleStreamOp``),
``CsvToColumns``/``JsonToColumns``/``KvToColumns``/``JsonValue``, the vector mapper family, UDF/UDTF and
``VectorSerialize``.

Reference: ``A/operator/stream/dataproc/format/*``, ``A/operator/stream/dataproc/{CsvToColumns,JsonToColumns,
KvToColumns,JsonValue}StreamOp.java``, ``A/operator/stream/dataproc/vector/*StreamOp.java`` and
``A/operator/stream/utils/{UDF,UDTF,VectorSerialize}StreamOp.java`` — each is a ``MapStreamOp`` /
``FlatMapStreamOp`` around the same mapper as its batch twin; here every micro-batch is mapped columnar.
"""
from __future__ import annotations

from typing import Optional

from ...common.mapper import FlatMapper
from ...common.params import ParamInfo, Params
from ...common.table import MTable, Row, infer_type
from ...common.types import TableSchema, Types, type_from_str
from ...models.dataproc import format as F
from ...models.dataproc import vector as V
from ..batch.format import FORMATS, BaseFormatTransBatchOp, format_ctor_args
from ..batch.utils import _UDFMapper
from .base import FlatMapStreamOp, MapStreamOp, StreamOperator, _register_upstream_sources

__all__ = ["BaseFormatTransStreamOp", "AnyToTripleStreamOp", "CsvToColumnsStreamOp", "JsonToColumnsStreamOp",
           "KvToColumnsStreamOp", "JsonValueStreamOp", "UDFStreamOp", "UDTFStreamOp", "VectorSerializeStreamOp"]


class BaseFormatTransStreamOp(MapStreamOp):
    MAPPER = F.FormatTransMapper
    EXTRA_PARAMS = list(BaseFormatTransBatchOp.EXTRA_PARAMS)      # fromFormat / toFormat + every format's columns
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


class AnyToTripleStreamOp(FlatMapStreamOp):
    MAPPER = F.AnyToTripleFlatMapper
    EXTRA_PARAMS = BaseFormatTransStreamOp.EXTRA_PARAMS
    FROM: Optional[str] = None

    def __init__(self, *args, **kw):
        fmts, params = format_ctor_args(args)
        super().__init__(params, **kw)
        if self.FROM is not None:
            self.getParams().set("fromFormat", self.FROM)
        if fmts:
            self.getParams().set("fromFormat", fmts[0])


class CsvToColumnsStreamOp(MapStreamOp):
    MAPPER = F.CsvToColumnsMapper
    EXTRA_PARAMS = [ParamInfo("selectedCol", str, "Name of the selected column", default=None),
                    ParamInfo("fieldDelimiter", str, "Field delimiter", default=None)]


class JsonToColumnsStreamOp(MapStreamOp):
    MAPPER = F.JsonToColumnsMapper
    EXTRA_PARAMS = [ParamInfo("selectedCol", str, "Name of the selected column", default=None)]


class KvToColumnsStreamOp(MapStreamOp):
    MAPPER = F.KvToColumnsMapper
    EXTRA_PARAMS = [ParamInfo("selectedCol", str, "Name of the selected column", default=None),
                    ParamInfo("colDelimiter", str, "Delimiter between key-value pairs", default=None),
                    ParamInfo("valDelimiter", str, "Delimiter between key and value", default=None)]


class JsonValueStreamOp(MapStreamOp):
    MAPPER = F.JsonPathMapper


class VectorSerializeStreamOp(MapStreamOp):
    PARAMS = ()
    MAPPER = V.VectorSerializeMapper


class UDFStreamOp(MapStreamOp):
    """Python scalar function over ``selectedCols`` into ``outputCol`` on every micro-batch."""
    _ALINK_NAME = "UDFBatchOp"
    EXTRA_PARAMS = [ParamInfo("resultType", str, "result type of the udf", default="DOUBLE")]

    def setFunc(self, f):
        self._func = f
        return self

    def getFunc(self):
        return getattr(self, "_func", None)

    def linkFrom(self, *inputs):
        (inp,) = self._connect(*inputs)
        f = self.getFunc()
        rt = getattr(f, "result_type", None) or self.getParams().get(self._param_infos["resultType"])
        rt = type_from_str(rt) if isinstance(rt, str) else rt
        self._mapper = _UDFMapper(inp.getSchema(), self.getParams(), f, rt)
        self._schema = self._mapper.getOutputSchema()
        _register_upstream_sources(inp)
        return self


class _UDTFMapper(FlatMapper):
    def __init__(self, dataSchema, params, func, result_types):
        super().__init__(dataSchema, params)
        p = self.params
        from ..common.sql.udf import TableFunction
        self.func = func if isinstance(func, TableFunction) else getattr(func, "eval", func)
        self.idx = [dataSchema.names.index(c) for c in p.get("selectedCols")]
        self.outs = list(p.get("outputCols"))
        reserved = p.get("reservedCols") if p.contains("reservedCols") else None
        self.keep = [i for i, n in enumerate(dataSchema.names)
                     if (reserved is None or n in reserved) and n not in self.outs]
        self.types = [type_from_str(t) for t in result_types] if result_types else None

    def getOutputSchema(self):
        types = self.types or [Types.STRING] * len(self.outs)
        return TableSchema([self.dataSchema.names[i] for i in self.keep] + self.outs,
                           [self.dataSchema.types[i] for i in self.keep] + list(types))

    def flatMap(self, row):
        out = []
        for o in self.func(*[row[i] for i in self.idx]) or []:
            o = o if isinstance(o, (list, tuple)) else (o,)
            out.append(Row(tuple(row[i] for i in self.keep) + tuple(o)))
        return out


class UDTFStreamOp(FlatMapStreamOp):
    _ALINK_NAME = "UDTFBatchOp"
    EXTRA_PARAMS = [ParamInfo("resultTypes", [str], "result types", default=None)]

    def setFunc(self, f):
        self._func = f
        return self

    def getFunc(self):
        return getattr(self, "_func", None)

    def linkFrom(self, *inputs):
        (inp,) = self._connect(*inputs)
        f = self.getFunc()
        rts = getattr(f, "result_types", None) or self.getParams().get(self._param_infos["resultTypes"])
        self._mapper = _UDTFMapper(inp.getSchema(), self.getParams(), f, rts)
        self._schema = self._mapper.getOutputSchema()
        _register_upstream_sources(inp)
        return self


def _make(name, base, attrs):
    cls = type(name, (base,), dict(attrs, __module__=__name__, __doc__=f"{name} (stream twin of the batch op)."))
    globals()[name] = cls
    __all__.append(name)
    return cls


for _f in FORMATS:
    for _t in FORMATS:
        if _f == _t or (_f, _t) in (("Csv", "Columns"), ("Json", "Columns"), ("Kv", "Columns")):
            continue
        _make(f"{_f}To{_t}StreamOp", BaseFormatTransStreamOp, {"FROM": _f.upper(), "TO": _t.upper()})
    _make(f"{_f}ToTripleStreamOp", AnyToTripleStreamOp, {"FROM": _f.upper()})

# VectorToColumnsStreamOp: both flavours, like the batch op (vector: selectedCol + outputCols; format: vectorCol +
# schemaStr)
from ..batch.dataproc import VectorToColumnsBatchOp as _V2CB  # noqa: E402
VectorToColumnsStreamOp = type("VectorToColumnsStreamOp", (MapStreamOp,), dict(  # noqa: F811
    MAPPER=V.VectorToColumnsMapper, EXTRA_PARAMS=list(_V2CB.EXTRA_PARAMS), __module__=__name__,
    __doc__="VectorToColumnsStreamOp (stream twin of the batch op)."))

for _n, _m in {"VectorAssemblerStreamOp": V.VectorAssemblerMapper,
               "VectorElementwiseProductStreamOp": V.VectorElementwiseProductMapper,
               "VectorInteractionStreamOp": V.VectorInteractionMapper,
               "VectorNormalizeStreamOp": V.VectorNormalizeMapper,
               "VectorPolynomialExpandStreamOp": V.VectorPolynomialExpandMapper,
               "VectorSizeHintStreamOp": V.VectorSizeHintMapper,
               "VectorSliceStreamOp": V.VectorSliceMapper}.items():
    _make(_n, MapStreamOp, {"MAPPER": _m})
