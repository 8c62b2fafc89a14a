"""Database access for DB / MySQL sources and sinks.

Reference: ``A/common/io/{BaseDB,JdbcDB,MySqlDB,DerbyDB}.java`` (list/create/drop/has table, read a table as a
batch table, write rows), ``A/operator/common/io/jdbc/JDBCUpserOutputFormat.java`` (upsert / retract sink) and
``JdbcTypeConverter.java`` (Flink type <-> SQL type).

``SqliteDB`` is the embedded, file-backed engine of this build (the reference's embedded one is Derby); it is
always available.  ``MySqlDB`` speaks MySQL through ``pymysql`` / ``mysql.connector`` when one is importable and
raises a clear error otherwise (no network drivers ship in this image).  Rows are moved as whole batches
(``executemany``), and only rank 0 writes in multi-process runs after gathering.
"""
from __future__ import annotations

import sqlite3
from typing import Any, List, Optional, Sequence

from ....common.params import Params
from ....common.table import MTable
from ....common.types import TableSchema, Types

__all__ = ["BaseDB", "SqliteDB", "DerbyDB", "MySqlDB", "JdbcDB", "sql_type", "alink_type"]

_TO_SQL = {"STRING": "VARCHAR(65535)", "DOUBLE": "DOUBLE", "FLOAT": "FLOAT", "LONG": "BIGINT", "INT": "INTEGER",
           "BOOLEAN": "BOOLEAN", "SHORT": "SMALLINT", "BYTE": "TINYINT", "DECIMAL": "DECIMAL",
           "VECTOR": "VARCHAR(65535)", "DENSE_VECTOR": "VARCHAR(65535)", "SPARSE_VECTOR": "VARCHAR(65535)"}


def sql_type(t) -> str:
    return _TO_SQL.get(getattr(t, "name", str(t)).upper(), "VARCHAR(65535)")


def alink_type(decl: str):
    d = (decl or "").upper()
    if "BIGINT" in d or "LONG" in d:
        return Types.LONG
    if "INT" in d:
        return Types.INT
    if "DOUBLE" in d or "REAL" in d or "FLOA" in d or "DEC" in d or "NUM" in d:
        return Types.DOUBLE
    if "BOOL" in d:
        return Types.BOOLEAN
    return Types.STRING


def _cell(v):
    from ....common.linalg import Vector, VectorUtil
    if isinstance(v, Vector):
        return VectorUtil.toString(v)
    if hasattr(v, "item"):
        return v.item()
    return v


class BaseDB:
    """Abstract table store: the operations the reference's ``BaseDB`` exposes."""
    NAME = "db"

    def __init__(self, params: Optional[Params] = None):
        self.params = params.clone() if params is not None else Params()

    def getParams(self) -> Params:
        return self.params

    # -- connection --
    def connect(self):
        raise NotImplementedError

    def _q(self, name: str) -> str:
        return '"' + name.replace('"', '""') + '"'

    def execute(self, sql: str, args: Sequence[Any] = ()):
        con = self.connect()
        try:
            cur = con.cursor()
            cur.execute(sql, tuple(args))
            rows = cur.fetchall() if cur.description else []
            con.commit()
            return rows
        finally:
            con.close()

    # -- catalogue --
    def listTableNames(self) -> List[str]:
        raise NotImplementedError

    def hasTable(self, name: str) -> bool:
        return name in self.listTableNames()

    def createTable(self, name: str, schema: TableSchema, primary_keys: Optional[Sequence[str]] = None):
        cols = ", ".join(f"{self._q(n)} {sql_type(t)}" for n, t in zip(schema.names, schema.types))
        if primary_keys:
            cols += ", PRIMARY KEY (" + ", ".join(self._q(k) for k in primary_keys) + ")"
        self.execute(f"CREATE TABLE {self._q(name)} ({cols})")

    def dropTable(self, name: str):
        self.execute(f"DROP TABLE IF EXISTS {self._q(name)}")

    def getTableSchema(self, name: str) -> TableSchema:
        raise NotImplementedError

    # -- data --
    def read(self, name: str, schema: Optional[TableSchema] = None) -> MTable:
        schema = schema or self.getTableSchema(name)
        cols = ", ".join(self._q(n) for n in schema.names)
        rows = self.execute(f"SELECT {cols} FROM {self._q(name)}")
        return MTable.from_rows([tuple(r) for r in rows], schema)

    def write(self, name: str, mt: MTable, overwrite: bool = False, upsert_keys: Optional[Sequence[str]] = None):
        if overwrite and self.hasTable(name):
            self.dropTable(name)
        if not self.hasTable(name):
            self.createTable(name, mt.schema, upsert_keys)
        cols = ", ".join(self._q(n) for n in mt.schema.names)
        ph = ", ".join([self.PLACEHOLDER] * len(mt.schema.names))
        verb = self.UPSERT_VERB if upsert_keys else "INSERT INTO"
        con = self.connect()
        try:
            con.cursor().executemany(f"{verb} {self._q(name)} ({cols}) VALUES ({ph})",
                                     [tuple(_cell(v) for v in r) for r in mt.rows()])
            con.commit()
        finally:
            con.close()

    def delete(self, name: str, keys: Sequence[str], rows: List[Sequence[Any]]):
        if not rows:
            return
        cond = " AND ".join(f"{self._q(k)} = {self.PLACEHOLDER}" for k in keys)
        con = self.connect()
        try:
            con.cursor().executemany(f"DELETE FROM {self._q(name)} WHERE {cond}", [tuple(_cell(v) for v in r)
                                                                               for r in rows])
            con.commit()
        finally:
            con.close()

    PLACEHOLDER = "?"
    UPSERT_VERB = "INSERT OR REPLACE INTO"


class SqliteDB(BaseDB):
    """Embedded file-backed DB (``dbName`` = file path, ``:memory:`` not shared across ops)."""
    NAME = "sqlite"

    def __init__(self, dbName: Optional[str] = None, params: Optional[Params] = None):
        super().__init__(params)
        if dbName is not None:
            self.params.set("dbName", dbName)

    def connect(self):
        return sqlite3.connect(self.params.get("dbName"))

    def listTableNames(self) -> List[str]:
        return [r[0] for r in self.execute("SELECT name FROM sqlite_master WHERE type='table' ORDER BY name")]

    def getTableSchema(self, name: str) -> TableSchema:
        info = self.execute(f"PRAGMA table_info({self._q(name)})")
        if not info:
            raise ValueError(f"table {name} not found")
        return TableSchema([r[1] for r in info], [alink_type(r[2]) for r in info])


DerbyDB = SqliteDB
JdbcDB = SqliteDB


class MySqlDB(BaseDB):
    NAME = "mysql"
    PLACEHOLDER = "%s"
    UPSERT_VERB = "REPLACE INTO"

    def __init__(self, dbName=None, ip=None, port=None, username=None, password=None,
                 params: Optional[Params] = None):
        super().__init__(params)
        for k, v in (("dbName", dbName), ("ip", ip), ("port", port), ("username", username), ("password", password)):
            if v is not None:
                self.params.set(k, v)

    def _q(self, name: str) -> str:
        return "`" + name.replace("`", "``") + "`"

    def connect(self):
        p = self.params
        kw = dict(host=p.get("ip"), port=int(p.get("port")), user=p.get("username"), password=p.get("password"),
                  database=p.get("dbName"))
        try:
            import pymysql  # type: ignore
            return pymysql.connect(**kw)
        except ImportError:
            pass
        try:
            import mysql.connector  # type: ignore
            return mysql.connector.connect(**kw)
        except ImportError as e:
            raise RuntimeError("MySQL access needs pymysql or mysql-connector-python, neither is installed") from e

    def listTableNames(self) -> List[str]:
        return [r[0] for r in self.execute("SHOW TABLES")]

    def getTableSchema(self, name: str) -> TableSchema:
        info = self.execute(f"DESCRIBE {self._q(name)}")
        return TableSchema([r[0] for r in info], [alink_type(r[1]) for r in info])
