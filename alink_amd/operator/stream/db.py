"""DB / MySQL stream sources and sinks and the JDBC retract (upsert) sink.

Reference: ``A/operator/stream/source/{DBSourceStreamOp,MySqlSourceStreamOp}.java``,
``A/operator/stream/sink/{DBSinkStreamOp,MySqlSinkStreamOp,JdbcRetractSinkStreamOp}.java`` and
``JDBCUpserOutputFormat.java``.  Sinks write every micro-batch as it arrives (one ``executemany`` per batch);
the retract sink upserts on its primary-key columns.
"""
from __future__ import annotations

from typing import Iterator, Optional, Sequence

from ...common.params import ParamInfo, Params
from ...common.table import MTable
from ...parallel import comm
from ..batch.db import read_db_table
from ..common.io.db import BaseDB, MySqlDB
from .base import StreamSourceOp
from .source import _batch_rows
from .utils import StreamSinkOp

__all__ = ["DBSourceStreamOp", "DBSinkStreamOp", "MySqlSourceStreamOp", "MySqlSinkStreamOp",
           "JdbcRetractSinkStreamOp"]


class DBSourceStreamOp(StreamSourceOp):
    EXTRA_PARAMS = [ParamInfo("inputTableName", str, "input table name", default=None),
                    ParamInfo("schemaStr", str, "schema", default=None)]

    def __init__(self, db: BaseDB = None, tableName: Optional[str] = None, params: Optional[Params] = None):
        super().__init__(params)
        self.db = db
        if tableName is not None:
            self.setInputTableName(tableName)
        self._mt = None

    def _db(self):
        return self.db

    def getSchema(self):
        if self._mt is None:
            self._mt = read_db_table(self._db(), self.getInputTableName(), self.getSchemaStr(), self.env)
            self._schema = self._mt.schema
        return self._schema

    def batches(self) -> Iterator[MTable]:
        self.getSchema()
        bs = max(1, _batch_rows())
        for s in range(0, self._mt.num_rows, bs):
            yield self._mt.slice(s, min(self._mt.num_rows, s + bs))


class MySqlSourceStreamOp(DBSourceStreamOp):
    _NO_AUTO_PARAMS = False
    EXTRA_PARAMS = []

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(None, None, params)
        for k, v in kw.items():
            self.set(k, v)

    def _db(self):
        return MySqlDB(params=self.getParams())


class DBSinkStreamOp(StreamSinkOp):
    EXTRA_PARAMS = [ParamInfo("outputTableName", str, "output table name", default=None)]
    KEYS: Optional[Sequence[str]] = None

    def __init__(self, db: BaseDB = None, tableName: Optional[str] = None, params: Optional[Params] = None):
        super().__init__(params)
        self.db = db
        if tableName is not None:
            self.setOutputTableName(tableName)
        self._created = False

    def _db(self):
        return self.db

    def _keys(self):
        return None

    def on_batch(self, port, mt: MTable):
        parts = comm.all_gather_object(mt.rows()) if comm.get_world_size() > 1 else [mt.rows()]
        if comm.get_rank() == 0:
            rows = [r for p in parts for r in p]
            self._db().write(self.getOutputTableName(), MTable.from_rows(rows, self._schema), False, self._keys())


class MySqlSinkStreamOp(DBSinkStreamOp):
    _NO_AUTO_PARAMS = False
    EXTRA_PARAMS = []

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(None, None, params)
        for k, v in kw.items():
            self.set(k, v)

    def _db(self):
        return MySqlDB(params=self.getParams())


class JdbcRetractSinkStreamOp(DBSinkStreamOp):
    """Upsert sink: rows with the same ``primaryKeys`` replace the stored one (the retract stream's latest
    value wins, ``JDBCUpserOutputFormat``)."""
    EXTRA_PARAMS = [ParamInfo("outputTableName", str, "output table name", default=None),
                    ParamInfo("primaryKeys", [str], "primary key columns", default=None)]

    def __init__(self, db: BaseDB = None, tableName: Optional[str] = None, primaryKeys=None,
                 params: Optional[Params] = None):
        super().__init__(db, tableName, params)
        if primaryKeys is not None:
            self.setPrimaryKeys(list(primaryKeys))

    def _keys(self):
        return self.getPrimaryKeys()
