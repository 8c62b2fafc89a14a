"""Column types and table schemas.

Type names follow Flink's ``TypeStringUtils`` spelling used in Alink schema strings
(``"f0 int, f1 bigint, f2 string"``; reference ``A/operator/common/io/csv/CsvUtil.java:30-88``) plus
Alink's vector pseudo-types ``VEC_TYPES_VECTOR / _DENSE_VECTOR / _SPARSE_VECTOR``
(``A/common/VectorTypes.java``).
"""
from __future__ import annotations

from typing import List, Sequence

import torch

__all__ = ["AlinkType", "Types", "TableSchema", "schema_str_to_schema", "schema_to_schema_str",
           "type_from_str", "torch_dtype_of", "is_numeric", "AlinkTypes"]


class AlinkType:
    __slots__ = ("name", "sql", "py", "torch_dtype")

    def __init__(self, name, sql, py, torch_dtype=None):
        self.name, self.sql, self.py, self.torch_dtype = name, sql, py, torch_dtype

    def __repr__(self):
        return self.sql

    def __eq__(self, o):
        return isinstance(o, AlinkType) and o.name == self.name

    def __hash__(self):
        return hash(self.name)


class Types:
    STRING = AlinkType("STRING", "VARCHAR", str)
    BOOLEAN = AlinkType("BOOLEAN", "BOOLEAN", bool, torch.bool)
    BYTE = AlinkType("BYTE", "TINYINT", int, torch.int8)
    SHORT = AlinkType("SHORT", "SMALLINT", int, torch.int16)
    INT = AlinkType("INT", "INT", int, torch.int32)
    LONG = AlinkType("LONG", "BIGINT", int, torch.int64)
    FLOAT = AlinkType("FLOAT", "FLOAT", float, torch.float32)
    DOUBLE = AlinkType("DOUBLE", "DOUBLE", float, torch.float64)
    DECIMAL = AlinkType("DECIMAL", "DECIMAL", float, torch.float64)
    DATE = AlinkType("DATE", "DATE", object)
    TIME = AlinkType("TIME", "TIME", object)
    TIMESTAMP = AlinkType("TIMESTAMP", "TIMESTAMP", object)
    VARBINARY = AlinkType("VARBINARY", "VARBINARY", bytes)
    VECTOR = AlinkType("VECTOR", "VEC_TYPES_VECTOR", object)
    DENSE_VECTOR = AlinkType("DENSE_VECTOR", "VEC_TYPES_DENSE_VECTOR", object)
    SPARSE_VECTOR = AlinkType("SPARSE_VECTOR", "VEC_TYPES_SPARSE_VECTOR", object)
    # tensor-valued column (e.g. fixed-size bf16 feature block)
    OBJECT = AlinkType("OBJECT", "RAW", object)


AlinkTypes = Types

_READ = {
    "VARCHAR": Types.STRING, "STRING": Types.STRING, "CHAR": Types.STRING,
    "BOOLEAN": Types.BOOLEAN, "BOOL": Types.BOOLEAN,
    "TINYINT": Types.BYTE, "BYTE": Types.BYTE,
    "SMALLINT": Types.SHORT, "SHORT": Types.SHORT,
    "INT": Types.INT, "INTEGER": Types.INT,
    "BIGINT": Types.LONG, "LONG": Types.LONG,
    "FLOAT": Types.FLOAT, "REAL": Types.FLOAT,
    "DOUBLE": Types.DOUBLE, "DECIMAL": Types.DECIMAL,
    "DATE": Types.DATE, "TIME": Types.TIME, "TIMESTAMP": Types.TIMESTAMP,
    "VARBINARY": Types.VARBINARY, "BYTES": Types.VARBINARY,
    "VEC_TYPES_VECTOR": Types.VECTOR, "VEC_TYPES_DENSE_VECTOR": Types.DENSE_VECTOR,
    "VEC_TYPES_SPARSE_VECTOR": Types.SPARSE_VECTOR, "VECTOR": Types.VECTOR,
    "DENSE_VECTOR": Types.DENSE_VECTOR, "SPARSE_VECTOR": Types.SPARSE_VECTOR, "RAW": Types.OBJECT,
}

NUMERIC = {Types.BYTE, Types.SHORT, Types.INT, Types.LONG, Types.FLOAT, Types.DOUBLE, Types.DECIMAL}
VECTORS = {Types.VECTOR, Types.DENSE_VECTOR, Types.SPARSE_VECTOR}


def type_from_str(s: str) -> AlinkType:
    t = _READ.get(s.strip().upper())
    if t is None:
        raise ValueError(f"Unsupported type: {s}")
    return t


def is_numeric(t: AlinkType) -> bool:
    return t in NUMERIC


def is_vector(t: AlinkType) -> bool:
    return t in VECTORS


def torch_dtype_of(t: AlinkType):
    return t.torch_dtype


class TableSchema:
    def __init__(self, names: Sequence[str], types: Sequence[AlinkType]):
        names = list(names)
        types = list(types)
        if len(names) != len(types):
            raise ValueError("names and types length mismatch")
        self.names: List[str] = names
        self.types: List[AlinkType] = types

    def getFieldNames(self):
        return list(self.names)

    def getFieldTypes(self):
        return list(self.types)

    def getFieldCount(self):
        return len(self.names)

    def index(self, name: str) -> int:
        return self.names.index(name)

    def type_of(self, name: str) -> AlinkType:
        return self.types[self.names.index(name)]

    def __eq__(self, o):
        return isinstance(o, TableSchema) and o.names == self.names and o.types == self.types

    def __repr__(self):
        return "root\n" + "\n".join(f" |-- {n}: {t.sql}" for n, t in zip(self.names, self.types))

    def to_str(self):
        return schema_to_schema_str(self)


def schema_str_to_schema(s: str) -> TableSchema:
    names, types = [], []
    for field in s.split(","):
        kv = field.strip().split()
        names.append(kv[0])
        types.append(type_from_str(kv[1]))
    return TableSchema(names, types)


def schema_to_schema_str(schema: TableSchema) -> str:
    return ",".join(f"{n} {t.sql}" for n, t in zip(schema.names, schema.types))
