"""DB / MySQL batch sources and sinks (reference ``A/operator/batch/source/{DBSourceBatchOp,MySqlSourceBatchOp}``,
``A/operator/batch/sink/{DBSinkBatchOp,MySqlSinkBatchOp}.java``).  Sources read on rank 0 and scatter blocks;
sinks gather and write on rank 0."""
from __future__ import annotations

from typing import Optional

from ...common.params import ParamInfo, Params
from ...common.table import MTable
from ...common.types import schema_str_to_schema
from ...parallel import comm
from ..base import BatchOperator, gather_table, partition_bounds
from ..common.io.db import BaseDB, MySqlDB

__all__ = ["DBSourceBatchOp", "DBSinkBatchOp", "MySqlSourceBatchOp", "MySqlSinkBatchOp", "read_db_table",
           "write_db_table"]

_TABLE = ParamInfo("inputTableName", str, "input table name", default=None)
_OUT = ParamInfo("outputTableName", str, "output table name", default=None)
_OVERWRITE = ParamInfo("overwriteSink", bool, "drop an existing table first", default=False)


def read_db_table(db: BaseDB, name: str, schema_str: Optional[str], env) -> MTable:
    schema = schema_str_to_schema(schema_str) if schema_str else None
    if comm.get_world_size() == 1:
        return db.read(name, schema)
    full = comm.broadcast_object(db.read(name, schema).rows() if comm.get_rank() == 0 else None, 0)
    sch = comm.broadcast_object(schema or (db.getTableSchema(name) if comm.get_rank() == 0 else None), 0)
    lo, hi = partition_bounds(len(full), env)
    return MTable.from_rows(full[lo:hi], sch)


def write_db_table(db: BaseDB, name: str, mt: MTable, overwrite: bool = False, upsert_keys=None):
    full = gather_table(mt)
    if comm.get_rank() == 0:
        db.write(name, full, overwrite, upsert_keys)
    comm.barrier()


class DBSourceBatchOp(BatchOperator):
    EXTRA_PARAMS = [_TABLE, ParamInfo("schemaStr", str, "schema", default=None)]

    def __init__(self, db: BaseDB = None, tableName: Optional[str] = None, params: Optional[Params] = None):
        super().__init__(params)
        self.db = db
        if tableName is not None:
            self.setInputTableName(tableName)
        self._loaded = False

    def _db(self) -> BaseDB:
        return self.db

    def getOutputTable(self):
        if not self._loaded:
            self._loaded = True
            self.setOutputTable(read_db_table(self._db(), self.getInputTableName(), self.getSchemaStr(), self.env))
        return super().getOutputTable()

    def linkFrom(self, *inputs):
        raise RuntimeError("Source operator does not support linkFrom()")


class DBSinkBatchOp(BatchOperator):
    EXTRA_PARAMS = [_OUT, _OVERWRITE]

    def __init__(self, db: BaseDB = None, tableName: Optional[str] = None, params: Optional[Params] = None):
        super().__init__(params)
        self.db = db
        if tableName is not None:
            self.setOutputTableName(tableName)

    def _db(self) -> BaseDB:
        return self.db

    def linkFrom(self, *inputs):
        inp = self.checkAndGetFirst(inputs)
        write_db_table(self._db(), self.getOutputTableName(), inp.getOutputTable(), bool(self.getOverwriteSink()))
        self.setOutputTable(inp.getOutputTable())
        return self


class MySqlSourceBatchOp(DBSourceBatchOp):
    _NO_AUTO_PARAMS = False
    EXTRA_PARAMS = []

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(None, None, params)
        for k, v in kw.items():
            self.set(k, v)

    def _db(self):
        return MySqlDB(params=self.getParams())


class MySqlSinkBatchOp(DBSinkBatchOp):
    _NO_AUTO_PARAMS = False
    EXTRA_PARAMS = [_OVERWRITE]

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(None, None, params)
        for k, v in kw.items():
            self.set(k, v)

    def _db(self):
        return MySqlDB(params=self.getParams())
