"""DirectReader / DataBridge / ModelSource: how a model (or any batch result) reaches code that runs outside the
batch dataflow — stream predictors, FTRL warm start, local serving.

Reference:
* ``A/common/io/directreader/DirectReader.java:61-76`` (``collect`` -> ``DataBridge``), ``:78-106``
  (``directRead`` with a filter), ``:144-190`` (policy from ``direct_reader.properties`` in the CWD / on the
  classpath, then ``-Ddirect.reader.*`` system properties, then ``DirectReaderPropertiesStore``);
  ``MemoryDataBridgeGenerator.java:6-12`` (policy ``memory``: rows collected eagerly),
  ``DbDataBridgeGenerator`` (policy ``db``: rows written to a DB table, read back on demand), ``dummy``;
  generators discovered by Java SPI (``META-INF/services/...DataBridgeGenerator``).
* ``A/common/mapper/{BroadcastVariableModelSource.java:11-26, RowsModelSource.java,
  DataBridgeModelSource.java:14-29}`` — where a ``ModelMapper`` gets its rows.

Here the SPMD runtime needs no broadcast variables: a model table is a row-partitioned ``MTable`` on every rank,
and the *broadcast* source gathers it once (tensor/object all-gather) — the reference's broadcast variable.
Policies are registered with :func:`register_data_bridge` (the SPI analogue; extra plugin modules are imported
from ``ALINK_DATA_BRIDGE_PLUGINS``), and the policy is resolved exactly in the reference's order:
``direct_reader.properties`` (CWD) < environment ``ALINK_DIRECT_READER_*`` (the ``-Ddirect.reader.*``
analogue) < :class:`DirectReaderPropertiesStore`.
"""
from __future__ import annotations

import importlib
import os
import uuid
from typing import Any, Callable, Dict, List, Optional

from .table import MTable, Row
from .types import TableSchema

__all__ = ["DataBridge", "MemoryDataBridge", "DbDataBridge", "DummyDataBridge", "DataBridgeGenerator",
           "register_data_bridge", "DirectReader", "DirectReaderPropertiesStore", "ModelSource",
           "BroadcastModelSource", "RowsModelSource", "DataBridgeModelSource", "POLICY_KEY"]

POLICY_KEY = "direct.reader.policy"
_PROPS_FILE = "direct_reader.properties"


# ---------------------------------------------------------------------------------------------------------
# data bridges
# ---------------------------------------------------------------------------------------------------------
class DataBridge:
    """A materialised batch result readable from anywhere in this process (``DataBridge.java``)."""

    def getSchema(self) -> TableSchema:
        raise NotImplementedError

    def read(self, filter: Optional[Callable[[Row], bool]] = None) -> List[Row]:
        raise NotImplementedError

    def readTable(self) -> MTable:
        return MTable.from_rows([tuple(r) for r in self.read()], self.getSchema())


class MemoryDataBridge(DataBridge):
    """Policy ``memory``: the rows, collected eagerly (every rank holds the full table)."""

    def __init__(self, rows: List[Row], schema: TableSchema):
        self._rows, self._schema = list(rows), schema

    def getSchema(self):
        return self._schema

    def read(self, filter=None):
        return [r for r in self._rows if filter is None or filter(r)]


class DbDataBridge(DataBridge):
    """Policy ``db``: rows written once to a table of an embedded DB (``direct.reader.db.path``, default a file
    under the system temp dir), read back on every :meth:`read` — for models too large to keep twice."""

    def __init__(self, db, table: str, schema: TableSchema):
        self.db, self.table, self._schema = db, table, schema

    def getSchema(self):
        return self._schema

    def read(self, filter=None):
        rows = self.db.read(self.table, self._schema).rows()
        return [r for r in rows if filter is None or filter(r)]


class DummyDataBridge(DataBridge):
    """Policy ``dummy``: reads nothing (the reference's placeholder for plans that never read back)."""

    def __init__(self, schema: TableSchema):
        self._schema = schema

    def getSchema(self):
        return self._schema

    def read(self, filter=None):
        return []


class DataBridgeGenerator:
    """Builds a :class:`DataBridge` from a batch operator under one policy (``DataBridgeGenerator.java``)."""

    def generate(self, op, props: Dict[str, str]) -> DataBridge:
        raise NotImplementedError


_GENERATORS: Dict[str, Callable[[], DataBridgeGenerator]] = {}


def register_data_bridge(name: str):
    """Class decorator registering a generator under a policy name (the Java SPI analogue)."""
    def deco(cls):
        _GENERATORS[name.lower()] = cls
        return cls
    return deco


def _full_table(op) -> MTable:
    from ..operator.base import gather_table
    return gather_table(op.getOutputTable())


@register_data_bridge("memory")
class MemoryDataBridgeGenerator(DataBridgeGenerator):
    def generate(self, op, props):
        mt = _full_table(op)
        return MemoryDataBridge(mt.rows(), mt.schema)


@register_data_bridge("db")
class DbDataBridgeGenerator(DataBridgeGenerator):
    def generate(self, op, props):
        import tempfile
        from ..operator.common.io.db import SqliteDB
        from ..parallel import comm
        mt = _full_table(op)
        path = props.get("direct.reader.db.path") or os.path.join(tempfile.gettempdir(),
                                                                   f"alink_direct_reader_{os.getpid()}.sqlite")
        table = "bridge_" + uuid.uuid4().hex[:12] + f"_r{comm.get_rank()}"
        db = SqliteDB(path)
        db.write(table, mt, overwrite=True)
        return DbDataBridge(db, table, mt.schema)


@register_data_bridge("dummy")
class DummyDataBridgeGenerator(DataBridgeGenerator):
    def generate(self, op, props):
        return DummyDataBridge(op.getOutputTable().schema)


# ---------------------------------------------------------------------------------------------------------
# policy resolution
# ---------------------------------------------------------------------------------------------------------
class DirectReaderPropertiesStore:
    """Programmatic overrides (highest priority), as ``DirectReaderPropertiesStore`` in the reference."""
    _props: Dict[str, str] = {}

    @classmethod
    def setProperties(cls, props: Dict[str, str]):
        cls._props = {str(k): str(v) for k, v in props.items()}

    @classmethod
    def getProperties(cls) -> Dict[str, str]:
        return dict(cls._props)

    @classmethod
    def clear(cls):
        cls._props = {}


def _read_properties_file(path: str) -> Dict[str, str]:
    out: Dict[str, str] = {}
    if not os.path.exists(path):
        return out
    with open(path, encoding="utf-8") as f:
        for line in f:
            line = line.strip()
            if not line or line[0] in "#!":
                continue
            for sep in ("=", ":"):
                if sep in line:
                    k, v = line.split(sep, 1)
                    out[k.strip()] = v.strip()
                    break
    return out


def _load_plugins():
    for mod in filter(None, os.environ.get("ALINK_DATA_BRIDGE_PLUGINS", "").split(",")):
        importlib.import_module(mod.strip())


class DirectReader:
    """``collect(op)`` materialises a batch operator as a :class:`DataBridge` under the configured policy;
    ``directRead(bridge)`` returns its rows."""

    @staticmethod
    def readProperties() -> Dict[str, str]:
        props = _read_properties_file(os.path.join(os.getcwd(), _PROPS_FILE))
        for k, v in os.environ.items():        # ALINK_DIRECT_READER_POLICY -> direct.reader.policy
            if k.startswith("ALINK_DIRECT_READER_"):
                props["direct.reader." + k[len("ALINK_DIRECT_READER_"):].lower().replace("_", ".")] = v
        props.update(DirectReaderPropertiesStore.getProperties())
        return props

    @staticmethod
    def policy() -> str:
        return DirectReader.readProperties().get(POLICY_KEY, "memory").lower()

    @staticmethod
    def collect(op) -> DataBridge:
        props = DirectReader.readProperties()
        name = props.get(POLICY_KEY, "memory").lower()
        if name not in _GENERATORS:
            _load_plugins()
        if name not in _GENERATORS:
            raise ValueError(f"unknown direct reader policy {name!r}; registered: {sorted(_GENERATORS)}")
        return _GENERATORS[name]().generate(op, props)

    @staticmethod
    def directRead(bridge: DataBridge, filter: Optional[Callable[[Row], bool]] = None) -> List[Row]:
        return bridge.read(filter)


# ---------------------------------------------------------------------------------------------------------
# model sources
# ---------------------------------------------------------------------------------------------------------
class ModelSource:
    """Where a ``ModelMapper`` gets its model rows (``ModelSource.java``)."""

    def getModelRows(self) -> List[Row]:
        raise NotImplementedError

    def getSchema(self) -> TableSchema:
        raise NotImplementedError


class BroadcastModelSource(ModelSource):
    """The model table of the dataflow, gathered from every rank (``BroadcastVariableModelSource``)."""

    def __init__(self, model_table: MTable):
        self._mt = model_table
        self._full: Optional[MTable] = None

    def _get(self) -> MTable:
        if self._full is None:
            from ..operator.base import gather_table
            self._full = gather_table(self._mt)
        return self._full

    def getModelRows(self):
        return self._get().lazy_rows()

    def getSchema(self):
        return self._mt.schema


class RowsModelSource(ModelSource):
    """Rows already in memory (``RowsModelSource``: local serving)."""

    def __init__(self, rows: List[Row], schema: TableSchema):
        self._rows, self._schema = list(rows), schema

    def getModelRows(self):
        return list(self._rows)

    def getSchema(self):
        return self._schema


class DataBridgeModelSource(ModelSource):
    """Rows read through a :class:`DataBridge` (``DataBridgeModelSource.java:14-29``: stream predictors)."""

    def __init__(self, bridge: DataBridge):
        self.bridge = bridge

    def getModelRows(self):
        return DirectReader.directRead(self.bridge)

    def getSchema(self):
        return self.bridge.getSchema()


def model_source_of(obj: Any) -> ModelSource:
    """Normalise a model table / operator / bridge / source to a :class:`ModelSource`."""
    if isinstance(obj, ModelSource):
        return obj
    if isinstance(obj, DataBridge):
        return DataBridgeModelSource(obj)
    if isinstance(obj, MTable):
        return BroadcastModelSource(obj)
    if hasattr(obj, "getOutputTable"):
        return BroadcastModelSource(obj.getOutputTable())
    raise TypeError(f"cannot build a model source from {type(obj).__name__}")
