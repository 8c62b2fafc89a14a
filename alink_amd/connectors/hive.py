"""Hive batch source / sink and stream source.

Reference: ``connectors/connector-hive/.../{HiveDB,HiveBatchSource,HiveSourceBatchOp,HiveSinkBatchOp,
HiveSourceStreamOp}.java`` (``hiveConfDir``, ``hiveVersion``, ``dbName``, ``partition(s)``).

A ``hiveConfDir`` of the form ``file:///warehouse`` selects a local warehouse (one embedded SQLite catalogue per
database under that directory, partitions stored as ``__partition`` values); any other value needs ``pyhive``
(not installed in this image) and fails with a clear error.
"""
from __future__ import annotations

import os
from typing import Optional

from ..common.params import ParamInfo, Params
from ..common.table import Column, MTable
from ..common.types import Types
from ..operator.base import BatchOperator
from ..operator.batch.db import read_db_table, write_db_table
from ..operator.common.io.db import SqliteDB
from ..operator.stream.db import DBSourceStreamOp

__all__ = ["HiveDB", "HiveSourceBatchOp", "HiveSinkBatchOp", "HiveSourceStreamOp"]

_DB_PARAMS = [ParamInfo("hiveConfDir", str, "hive conf dir (file:///warehouse for the local warehouse)",
                        optional=False),
              ParamInfo("hiveVersion", str, "hive version", default="2.3.4"),
              ParamInfo("dbName", str, "database", default="default")]


class HiveDB(SqliteDB):
    NAME = "hive"

    def __init__(self, hiveConfDir: Optional[str] = None, hiveVersion: str = "2.3.4", dbName: str = "default",
                 params: Optional[Params] = None):
        p = params.clone() if params is not None else Params()
        if hiveConfDir is not None:
            p.set("hiveConfDir", hiveConfDir)
        p.set("hiveVersion", p.get("hiveVersion") if p.contains("hiveVersion") else hiveVersion)
        p.set("dbName", p.get("dbName") if p.contains("dbName") else dbName)
        conf = p.get("hiveConfDir")
        if not conf.startswith("file://"):
            try:
                import pyhive  # type: ignore  # noqa: F401
            except ImportError as e:
                raise RuntimeError("Hive access needs pyhive (not installed); use hiveConfDir=file:///dir for the "
                                   "local warehouse") from e
            raise RuntimeError("remote Hive metastores are not supported in this build")
        root = conf[len("file://"):]
        os.makedirs(root, exist_ok=True)
        super().__init__(os.path.join(root, f"{p.get('dbName')}.db"), p)


def _with_partition(mt: MTable, spec: Optional[str]) -> MTable:
    if not spec:
        return mt
    return mt.with_columns(["__partition"], [Types.STRING], [Column.from_values([spec] * mt.num_rows, Types.STRING)])


class HiveSourceBatchOp(BatchOperator):
    PARAMS = _DB_PARAMS + [ParamInfo("inputTableName", str, "table", optional=False),
                           ParamInfo("partitions", str, "partitions to read, '/'-separated specs", default=None)]

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(params, **kw)
        self._loaded = False

    def getOutputTable(self):
        if not self._loaded:
            self._loaded = True
            db = HiveDB(params=self.getParams())
            mt = read_db_table(db, self.getInputTableName(), None, self.env)
            parts = self.getPartitions()
            if "__partition" in mt.schema.names:
                if parts:
                    keep = set(parts.split("/")) if "/" in parts else {parts}
                    idx = [i for i, v in enumerate(mt.col("__partition").to_list()) if v in keep]
                    mt = mt.take(idx)
                mt = mt.select([n for n in mt.schema.names if n != "__partition"])
            self.setOutputTable(mt)
        return super().getOutputTable()

    def linkFrom(self, *inputs):
        raise RuntimeError("Source operator does not support linkFrom()")


class HiveSinkBatchOp(BatchOperator):
    PARAMS = _DB_PARAMS + [ParamInfo("outputTableName", str, "table", optional=False),
                           ParamInfo("partition", str, "static partition spec, e.g. ds=20200101", default=None),
                           ParamInfo("overwriteSink", bool, "drop an existing table first", default=False)]

    def linkFrom(self, *inputs):
        inp = self.checkAndGetFirst(inputs)
        db = HiveDB(params=self.getParams())
        write_db_table(db, self.getOutputTableName(), _with_partition(inp.getOutputTable(), self.getPartition()),
                       bool(self.getOverwriteSink()))
        self.setOutputTable(inp.getOutputTable())
        return self


class HiveSourceStreamOp(DBSourceStreamOp):
    PARAMS = _DB_PARAMS + [ParamInfo("inputTableName", str, "table", optional=False),
                           ParamInfo("schemaStr", str, "schema", default=None)]

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(None, None, params)
        for k, v in kw.items():
            self.set(k, v)

    def _db(self):
        return HiveDB(params=self.getParams())
