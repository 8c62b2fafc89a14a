"""IO operator / DB registry: the reference's ``@IoOpAnnotation`` / ``@DBAnnotation`` + ``AnnotationUtils``
(``A/common/io/annotations/AnnotationUtils.java:80-110``) and the ``of(params)`` factories of the source / sink
bases (``A/operator/batch/source/BaseSourceBatchOp.java:30-42`` and the sink / stream twins).

Operators register under ``(ioName, IOType)``; a source or sink can then be re-created from nothing but its
Params (``ioName`` + ``ioType`` + its own parameters) — how a saved pipeline or a remote job spec names its IO.
``@io_op`` is the annotation; ``register_builtin()`` applies it to the built-in sources / sinks (the same names
the reference uses: csv, text, libsvm, memory, db, print, ...).  DB classes register with ``@db_class`` and a
``DBSource*`` / ``DBSink*`` is chosen when the Params describe a DB (``ioName`` is a registered DB name).
"""
from __future__ import annotations

import enum
from typing import Dict, Optional, Tuple, Type

from .params import ParamInfo, Params

__all__ = ["IOType", "io_op", "db_class", "AnnotationUtils", "IO_TYPE", "IO_NAME", "register_builtin"]


class IOType(enum.Enum):
    SourceBatch = "SourceBatch"
    SinkBatch = "SinkBatch"
    SourceStream = "SourceStream"
    SinkStream = "SinkStream"


IO_TYPE = ParamInfo("ioType", str, "io type", default=None)
IO_NAME = ParamInfo("ioName", str, "io name", default=None)

_IO_OPS: Dict[Tuple[str, IOType], Tuple[type, bool]] = {}
_DBS: Dict[str, Tuple[type, bool]] = {}


def io_op(name: str, io_type: IOType, has_timestamp: bool = False):
    """Class decorator: register an IO operator under (name, io_type) and stamp ioName / ioType."""
    def deco(cls):
        prev = _IO_OPS.get((name, io_type))
        if prev is not None and prev[0] is not cls:
            raise ValueError(f"Multiple IO Operator class with same name {name} and IOType: {io_type}: "
                             f"{prev[0].__name__} and {cls.__name__}")
        _IO_OPS[(name, io_type)] = (cls, has_timestamp)
        cls.IO_NAME = name
        cls.IO_TYPE = io_type
        return cls
    return deco


def db_class(name: str, has_timestamp: bool = False):
    def deco(cls):
        _DBS[name] = (cls, has_timestamp)
        cls.DB_NAME = name
        return cls
    return deco


def _io_type(v) -> Optional[IOType]:
    if v is None:
        return None
    if isinstance(v, IOType):
        return v
    return IOType(str(getattr(v, "name", v)))


class AnnotationUtils:
    @staticmethod
    def annotatedName(cls) -> Optional[str]:
        return getattr(cls, "IO_NAME", None) or getattr(cls, "DB_NAME", None)

    @staticmethod
    def annotatedIoType(cls) -> Optional[IOType]:
        return getattr(cls, "IO_TYPE", None)

    @staticmethod
    def isDB(params: Params) -> bool:
        return params.contains("ioName") and params.get(IO_NAME) in _DBS

    @staticmethod
    def isDbHasTimestamp(name: str) -> bool:
        return _DBS[name][1]

    @staticmethod
    def isIoOpHasTimestamp(name: str, io_type: IOType) -> bool:
        return _IO_OPS[(name, _io_type(io_type))][1]

    @staticmethod
    def allDBAndOpNames():
        return sorted(set(_DBS) | {n for n, _ in _IO_OPS})

    @staticmethod
    def createDB(name: str, params: Params):
        if name not in _DBS:
            raise ValueError(f"DB class with name {name} not found")
        return _DBS[name][0](params=params)

    @staticmethod
    def createOp(name: str, io_type, params: Params):
        key = (name, _io_type(io_type))
        if key not in _IO_OPS:
            raise ValueError(f"IO Operator class with name {name} and IOType {io_type} not found")
        op = _IO_OPS[key][0](params=params.clone())
        op.getParams().set(IO_NAME, name).set(IO_TYPE, key[1].value)
        return op

    @staticmethod
    def of(params: Params, io_type: IOType):
        """``Base{Source,Sink}{Batch,Stream}Op.of(params)``: DB-backed op when ioName names a DB, else the
        registered IO operator."""
        io_type = _io_type(io_type)
        if not (params.contains("ioType") and _io_type(params.get(IO_TYPE)) == io_type and params.contains("ioName")):
            raise RuntimeError("Parameter Error.")
        name = params.get(IO_NAME)
        if name in _DBS:
            db = AnnotationUtils.createDB(name, params)
            cls = _IO_OPS[("db", io_type)][0]
            op = cls(db, params=params.clone())
            op.getParams().set(IO_NAME, "db").set(IO_TYPE, io_type.value)
            return op
        return AnnotationUtils.createOp(name, io_type, params)


def register_builtin():
    """Apply ``@io_op`` / ``@db_class`` to the built-in IO classes (names as in the reference)."""
    from ..operator.batch import db as bdb, sink as bsink, source as bsrc, utils as butils
    from ..operator.common.io import db as iodb
    from ..operator.stream import db as sdb, sink as ssink, source as ssrc, utils as sutils
    S, K, SS, KS = IOType.SourceBatch, IOType.SinkBatch, IOType.SourceStream, IOType.SinkStream
    table = [
        ("csv", S, bsrc.CsvSourceBatchOp), ("text", S, bsrc.TextSourceBatchOp),
        ("libsvm", S, bsrc.LibSvmSourceBatchOp), ("memory", S, bsrc.MemSourceBatchOp),
        ("db", S, bdb.DBSourceBatchOp), ("my_sql_batch_source", S, bdb.MySqlSourceBatchOp),
        ("csv", K, bsink.CsvSinkBatchOp), ("text", K, bsink.TextSinkBatchOp), ("libsvm", K, bsink.LibSvmSinkBatchOp),
        ("db", K, bdb.DBSinkBatchOp), ("my_sql_batch_sink", K, bdb.MySqlSinkBatchOp),
        ("print", K, butils.PrintBatchOp),
        ("csv", SS, ssrc.CsvSourceStreamOp), ("text", SS, ssrc.TextSourceStreamOp),
        ("libsvm", SS, ssrc.LibSvmSourceStreamOp), ("memory", SS, ssrc.MemSourceStreamOp),
        ("db", SS, sdb.DBSourceStreamOp), ("my_sql_stream_source", SS, sdb.MySqlSourceStreamOp),
        ("csv", KS, ssink.CsvSinkStreamOp), ("text", KS, ssink.TextSinkStreamOp),
        ("libsvm", KS, ssink.LibSvmSinkStreamOp), ("db", KS, sdb.DBSinkStreamOp),
        ("my_sql_stream_sink", KS, sdb.MySqlSinkStreamOp), ("print", KS, sutils.PrintStreamOp),
    ]
    for name, t, cls in table:
        if (name, t) not in _IO_OPS:
            io_op(name, t)(cls)
    for name, cls in (("sqlite", iodb.SqliteDB), ("derby", iodb.SqliteDB), ("mysql", iodb.MySqlDB)):
        if name not in _DBS:
            db_class(name)(cls)
