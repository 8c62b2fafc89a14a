"""Kafka stream source and sink.

Reference: ``connectors/connector-kafka-base/.../BaseKafkaSourceStreamOp.java`` (output schema
``(message_key, message, topic, topic_partition, partition_offset)``; startup modes EARLIEST / LATEST /
GROUP_OFFSETS / TIMESTAMP), ``BaseKafkaSinkStreamOp`` (rows serialised as CSV or JSON, ``dataFormat``,
``fieldDelimiter``), ``KafkaSourceParams`` / ``KafkaSinkParams`` and the 0.10 / 0.11 variants.

Transport: ``bootstrapServers`` of the form ``file:///dir`` selects the built-in log broker (one append-only
JSON-lines file per topic partition under ``dir`` — used by the tests and for single-host pipelines); any
other value goes through ``kafka-python`` (``import kafka``) when it is installed and fails with a clear error
otherwise (no Kafka client ships in this image).
"""
from __future__ import annotations

import glob
import json
import os
import re
import time
from typing import Iterator, List, Optional

from ..common.javafmt import gson_dumps, java_str
from ..common.params import ParamInfo, Params
from ..common.table import MTable
from ..common.types import TableSchema, Types
from ..operator.common.io.csv import CsvFormatter
from ..operator.stream.base import StreamSourceOp
from ..operator.stream.utils import StreamSinkOp

__all__ = ["KafkaSourceStreamOp", "KafkaSinkStreamOp", "Kafka010SourceStreamOp", "Kafka010SinkStreamOp",
           "Kafka011SourceStreamOp", "Kafka011SinkStreamOp", "LocalLogBroker"]

SOURCE_SCHEMA = TableSchema(["message_key", "message", "topic", "topic_partition", "partition_offset"],
                            [Types.STRING, Types.STRING, Types.STRING, Types.INT, Types.LONG])


class LocalLogBroker:
    """File-backed topic log: ``<dir>/<topic>/partition-<p>.jsonl``; each line ``{"k","v","ts"}``."""

    def __init__(self, root: str):
        self.root = root[len("file://"):] if root.startswith("file://") else root

    def send(self, topic: str, key: Optional[str], value: str, partition: int = 0):
        d = os.path.join(self.root, topic)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"partition-{partition}.jsonl"), "a", encoding="utf-8") as f:
            f.write(json.dumps({"k": key, "v": value, "ts": time.time()}) + "\n")

    def topics(self) -> List[str]:
        return sorted(os.path.basename(p) for p in glob.glob(os.path.join(self.root, "*")) if os.path.isdir(p))

    def read(self, topic: str, start_ts: Optional[float] = None, latest: bool = False):
        for fn in sorted(glob.glob(os.path.join(self.root, topic, "partition-*.jsonl"))):
            part = int(re.findall(r"partition-(\d+)", fn)[0])
            with open(fn, encoding="utf-8") as f:
                lines = f.readlines()
            if latest:
                continue
            for off, line in enumerate(lines):
                m = json.loads(line)
                if start_ts is not None and m["ts"] < start_ts:
                    continue
                yield m["k"], m["v"], topic, part, off


def _client(servers: str):
    if servers and servers.startswith("file://"):
        return LocalLogBroker(servers)
    try:
        import kafka  # type: ignore  # noqa: F401
    except ImportError as e:
        raise RuntimeError("Kafka access needs the kafka-python client (not installed); use a file:// "
                           "bootstrapServers for the built-in log broker") from e
    return None


_SRC_PARAMS = [ParamInfo("bootstrapServers", str, "kafka bootstrap servers", optional=False),
               ParamInfo("groupId", str, "consumer group id", default=None),
               ParamInfo("startupMode", str, "EARLIEST / LATEST / GROUP_OFFSETS / TIMESTAMP", default="GROUP_OFFSETS"),
               ParamInfo("topic", str, "topic", default=None),
               ParamInfo("topicPattern", str, "topic regex", default=None),
               ParamInfo("startTime", str, "start time (yyyy-MM-dd HH:mm:ss) for TIMESTAMP mode", default=None),
               ParamInfo("properties", str, "extra client properties", default=None)]
_SINK_PARAMS = [ParamInfo("bootstrapServers", str, "kafka bootstrap servers", optional=False),
                ParamInfo("topic", str, "topic", optional=False),
                ParamInfo("dataFormat", str, "CSV or JSON", default="JSON"),
                ParamInfo("fieldDelimiter", str, "CSV field delimiter", default=","),
                ParamInfo("properties", str, "extra client properties", default=None)]


class KafkaSourceStreamOp(StreamSourceOp):
    PARAMS = _SRC_PARAMS

    def getSchema(self):
        return SOURCE_SCHEMA

    def batches(self) -> Iterator[MTable]:
        self._schema = SOURCE_SCHEMA
        cl = _client(self.getBootstrapServers())
        if cl is None:
            yield from self._kafka_python_batches()
            return
        topics = [self.getTopic()] if self.getTopic() else [t for t in cl.topics()
                                                            if re.fullmatch(self.getTopicPattern() or ".*", t)]
        mode = str(getattr(self.getStartupMode(), "name", self.getStartupMode())).upper()
        start = None
        if mode == "TIMESTAMP" and self.getStartTime():
            start = time.mktime(time.strptime(self.getStartTime(), "%Y-%m-%d %H:%M:%S"))
        rows = []
        for t in topics:
            rows.extend(cl.read(t, start, latest=(mode == "LATEST")))
        bs = 1024
        for s in range(0, len(rows), bs):
            yield MTable.from_rows(rows[s:s + bs], SOURCE_SCHEMA)

    def _kafka_python_batches(self):  # pragma: no cover - needs a broker
        from kafka import KafkaConsumer  # type: ignore
        mode = str(getattr(self.getStartupMode(), "name", self.getStartupMode())).upper()
        c = KafkaConsumer(self.getTopic(), bootstrap_servers=self.getBootstrapServers(), group_id=self.getGroupId(),
                          auto_offset_reset="earliest" if mode == "EARLIEST" else "latest",
                          consumer_timeout_ms=10000)
        buf = []
        for m in c:
            buf.append((None if m.key is None else m.key.decode(), m.value.decode(), m.topic, m.partition, m.offset))
            if len(buf) >= 1024:
                yield MTable.from_rows(buf, SOURCE_SCHEMA)
                buf = []
        if buf:
            yield MTable.from_rows(buf, SOURCE_SCHEMA)


class KafkaSinkStreamOp(StreamSinkOp):
    PARAMS = _SINK_PARAMS

    def on_batch(self, port, mt: MTable):
        fmt = str(self.getDataFormat()).upper()
        names = mt.schema.names
        if fmt == "CSV":
            f = CsvFormatter(mt.schema.types, self.getFieldDelimiter(), '"')
            msgs = [f.format(r) for r in mt.rows()]
        else:
            msgs = [gson_dumps({n: (java_str(v) if not isinstance(v, (int, float, str, bool)) or isinstance(v, bool)
                                    else v) for n, v in zip(names, r) if v is not None}, java_map_order=False)
                    for r in mt.rows()]
        cl = _client(self.getBootstrapServers())
        if cl is None:  # pragma: no cover - needs a broker
            from kafka import KafkaProducer  # type: ignore
            pr = KafkaProducer(bootstrap_servers=self.getBootstrapServers())
            for m in msgs:
                pr.send(self.getTopic(), m.encode())
            pr.flush()
            return
        for m in msgs:
            cl.send(self.getTopic(), None, m)


class Kafka010SourceStreamOp(KafkaSourceStreamOp):
    PARAMS = _SRC_PARAMS


class Kafka011SourceStreamOp(KafkaSourceStreamOp):
    PARAMS = _SRC_PARAMS


class Kafka010SinkStreamOp(KafkaSinkStreamOp):
    PARAMS = _SINK_PARAMS


class Kafka011SinkStreamOp(KafkaSinkStreamOp):
    PARAMS = _SINK_PARAMS
