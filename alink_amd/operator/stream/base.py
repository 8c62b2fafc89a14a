"""Micro-batch streaming engine: ``StreamOperator`` and the generic Map/ModelMap/FlatMap stream ops.

Reference: ``A/operator/stream/StreamOperator.java:37-389`` (Flink ``DataStream<Row>`` wrapper; ``link``,
``print``, ``execute``) and ``A/operator/stream/utils/{MapStreamOp,ModelMapStreamOp,FlatMapStreamOp}.java``.

Design: Flink's record-at-a-time dataflow becomes a *push-based DAG of micro-batches*.
Each operator receives ``MTable`` micro-batches on an input port and emits micro-batches to its
subscribers; ``StreamOperator.execute()`` drives every source of the environment to exhaustion, interleaving
sources round-robin (a deterministic stand-in for Flink's asynchronous arrival order).  Model streams
(FTRL snapshots) are just another input port, so predictors hot-swap models between micro-batches.
Micro-batches keep tensors on the rank's device, so the per-batch math runs on the GPU.
"""
from __future__ import annotations

import sys
from typing import Callable, Dict, Iterator, List, Optional

from ...common.mapper import FlatMapper, Mapper, ModelMapper
from ...common.mlenv import MLEnvironmentFactory
from ...common.params import ParamInfo, Params
from ...common.table import MTable, Row
from ...common.types import TableSchema
from ..base import AlgoOperator, format_rows, format_title, _fmt_val

__all__ = ["StreamOperator", "StreamSourceOp", "MapStreamOp", "ModelMapStreamOp", "FlatMapStreamOp",
           "StreamEngine"]


class StreamEngine:
    """Per-environment registry of stream sources and sinks."""

    def __init__(self):
        self.sources: List["StreamSourceOp"] = []
        self.sinks: List["StreamOperator"] = []

    def register_source(self, src):
        if src not in self.sources:
            self.sources.append(src)

    def register_sink(self, op):
        if op not in self.sinks:
            self.sinks.append(op)

    # ---- checkpointing (StreamOperator.setCheckPointConf) ----
    def _dag(self) -> List["StreamOperator"]:
        """Every operator reachable from the sources, in a deterministic BFS order (the checkpoint key)."""
        seen, order, queue = set(), [], list(self.sources)
        while queue:
            op = queue.pop(0)
            if id(op) in seen:
                continue
            seen.add(id(op))
            order.append(op)
            queue.extend(sub for sub, _ in op._subscribers)
        return order

    def _fingerprint(self) -> str:
        """Identity of the stream job a checkpoint belongs to: operator classes + params along the DAG order."""
        import hashlib
        h = hashlib.sha1()
        for op in self._dag():
            h.update(type(op).__name__.encode())
            try:
                h.update(op.getParams().toJson().encode())
            except Exception:       # pragma: no cover - params that do not serialise still pin the class
                pass
        return h.hexdigest()

    def _ckpt_files(self, conf):
        """This rank's checkpoint files as {round: path}."""
        import os
        import re
        from ...parallel import comm
        os.makedirs(conf["dir"], exist_ok=True)
        pat = re.compile(rf"stream_ckpt_rank{comm.get_rank()}_round(\d+)\.pt$")
        out = {}
        for f in os.listdir(conf["dir"]):
            m = pat.match(f)
            if m:
                out[int(m.group(1))] = os.path.join(conf["dir"], f)
        return out

    def _save(self, conf, consumed, rnd, fp):
        """Write this rank's state at micro-batch round ``rnd`` atomically and keep the last two rounds (so the
        ranks can always agree on a round every rank has completely written, see ``_restore``)."""
        import os
        import torch
        from ...parallel import comm
        state = {"round": int(rnd), "fingerprint": fp, "consumed": [int(c) for c in consumed],
                 "ops": {i: op._state_dict() for i, op in enumerate(self._dag()) if op._state_dict() is not None}}
        path = os.path.join(conf["dir"], f"stream_ckpt_rank{comm.get_rank()}_round{int(rnd)}.pt")
        torch.save(state, path + ".tmp")
        os.replace(path + ".tmp", path)          # atomic: a crash mid-write keeps the previous checkpoints
        files = self._ckpt_files(conf)
        for r in sorted(files)[:-2]:
            os.remove(files[r])

    def _restore(self, conf, fp):
        """Agree on the newest round every rank holds (MIN all-reduce of each rank's newest round), load it, and
        return (consumed counts, round) — or None when some rank has no checkpoint (fresh start everywhere)."""
        import torch
        from ...parallel import comm
        files = self._ckpt_files(conf)
        latest = torch.tensor([max(files) if files else -1], dtype=torch.int64)
        if comm.get_world_size() > 1:
            comm.all_reduce(latest, "min")
        rnd = int(latest.item())
        if rnd < 0:
            return None
        if rnd not in files:
            raise RuntimeError(f"stream checkpoint round {rnd} missing on rank {comm.get_rank()} ({conf['dir']})")
        state = torch.load(files[rnd], weights_only=True)
        if state.get("fingerprint") != fp:
            raise RuntimeError(f"stream checkpoint in {conf['dir']} was written by a different stream job "
                               "(operator DAG / params differ); remove it or use another directory")
        dag = self._dag()
        for i, st in state["ops"].items():
            dag[int(i)]._load_state_dict(st)
        return state["consumed"], rnd

    def run(self, checkpoint=None):
        """Drive every source to exhaustion, one micro-batch per source per round.

        On a multi-rank job the rounds are a LOCKSTEP protocol: every round ends with one MAX all-reduce of (any
        source still live, checkpoint due), a rank whose sources ended keeps emitting empty micro-batches until
        every rank's have, and with a checkpoint conf a checkpoint is written by all ranks at the same round — a
        consistent cut (the reference's Flink checkpoint barrier, ``StreamOperator.java:216-239``)."""
        import time
        import torch
        from ...parallel import comm
        srcs = [s for s in self.sources if s._subscribers]
        its = [(s, s.batches()) for s in srcs]
        consumed = [0] * len(its)
        # under a process group every rank runs the same number of rounds (an ended source emits empty
        # micro-batches until every rank's sources have ended), so operators whose on_batch issues collectives
        # (evaluation windows, DB sinks, FTRL) stay in step even when the ranks' streams differ in length
        lockstep = comm.get_world_size() > 1
        fp = self._fingerprint() if checkpoint is not None else None
        rnd = 0
        if checkpoint is not None:
            got = self._restore(checkpoint, fp)
            if got is not None:                  # replay: skip what the checkpoint already covers
                done, rnd = got
                for k, ((src, it), n) in enumerate(zip(its, done)):
                    for _ in range(n):
                        next(it, None)
                    consumed[k] = n
        last = time.time()
        ended = set()
        while True:
            live = False
            for k, (src, it) in enumerate(its):
                mt = None
                if k not in ended:
                    try:
                        mt = next(it)
                    except StopIteration:
                        ended.add(k)
                        if not lockstep:
                            src._finish()
                if mt is not None:
                    src._emit(mt)
                    consumed[k] += 1
                    live = True
                elif lockstep:
                    src._emit(MTable.empty(src.getSchema()))
            rnd += 1
            due = checkpoint is not None and (
                (checkpoint.get("every_batches") is not None and rnd % checkpoint["every_batches"] == 0)
                or (time.time() - last) >= checkpoint["interval_s"])
            if lockstep:
                flags = comm.all_reduce(torch.tensor([int(live), int(due)], dtype=torch.int64), "max")
                live, due = bool(flags[0]), bool(flags[1])
            if not live:
                break
            if due:
                self._save(checkpoint, consumed, rnd, fp)
                last = time.time()
        if lockstep:
            for src, _ in its:
                src._finish()
        for s in self.sinks:
            s._close()
        if checkpoint is not None and checkpoint.get("clear_on_finish", True):
            import os
            for f in self._ckpt_files(checkpoint).values():
                os.remove(f)
        self.sources.clear()
        self.sinks.clear()


def _engine(env) -> StreamEngine:
    e = getattr(env, "_stream_engine", None)
    if e is None:
        e = StreamEngine()
        env._stream_engine = e
    return e


class StreamOperator(AlgoOperator):
    """A node of the micro-batch DAG.  Subclasses implement ``on_batch(port, mt)`` (and optionally
    ``on_finish(port)``) and call ``self._emit(mt)``; ``linkFrom`` wires ports and sets the output schema."""

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(params, **kw)
        self._subscribers: List[tuple] = []  # (op, port)
        self._schema: Optional[TableSchema] = None
        self._n_inputs = 0
        self._finished_ports = set()
        self._side: List["StreamOperator"] = []

    # ---- wiring ----
    def link(self, nxt: "StreamOperator"):
        nxt.linkFrom(self)
        return nxt

    linkTo = link

    def linkFrom(self, *inputs):
        raise NotImplementedError

    def _connect(self, *inputs: "StreamOperator"):
        if len(inputs) == 1 and isinstance(inputs[0], (list, tuple)):
            inputs = inputs[0]
        self._n_inputs = len(inputs)
        self._upstreams = list(inputs)
        for port, inp in enumerate(inputs):
            inp._subscribers.append((self, port))
            _register_upstream_sources(inp)
        return inputs

    def getSchema(self) -> TableSchema:
        return self._schema

    def getColNames(self):
        return list(self._schema.names)

    def getColTypes(self):
        return list(self._schema.types)

    def getOutputTable(self):
        raise RuntimeError("stream operators have no materialised output table; use print/collect sinks")

    # ---- data flow ----
    # row-local operators (mappers, predictors, SQL select / where) map an empty micro-batch to an empty one of their
    # output schema without running: the lockstep rounds of a multi-rank job feed every operator empty batches
    # after its rank's stream ended, and a mapper need not handle zero rows.  Operators that issue collectives per
    # batch (evaluation windows, FTRL, DB sinks) keep receiving them.
    EMPTY_PASSTHROUGH = False

    def _emit(self, mt: MTable):
        for op, port in self._subscribers:
            if op.EMPTY_PASSTHROUGH and mt.num_rows == 0 and op._schema is not None:
                op._emit(MTable.empty(op._schema))
            else:
                op.on_batch(port, mt)

    def on_batch(self, port: int, mt: MTable):
        raise NotImplementedError

    def on_finish(self, port: int):
        pass

    def _finish(self, port: int = 0):
        self._finished_ports.add(port)
        self.on_finish(port)
        if len(self._finished_ports) >= max(1, self._n_inputs):
            for op, p in self._subscribers:
                op._finish(p)
            for s in self._side:
                for op, p in s._subscribers:
                    op._finish(p)

    def _close(self):
        pass

    def getSideOutput(self, i: int) -> "StreamOperator":
        return self._side[i]

    # ---- sinks / execution ----
    def print(self, key: Optional[str] = None, refreshInterval: int = 0, maxLimit: int = 100):
        from .utils import PrintStreamOp
        self.link(PrintStreamOp().setMLEnvironmentId(self.getMLEnvironmentId()))
        return self

    def collect_to(self, box: List[Row]):
        from .utils import CollectStreamOp
        self.link(CollectStreamOp(box).setMLEnvironmentId(self.getMLEnvironmentId()))
        return self

    @staticmethod
    def execute(env=None):
        env = env or MLEnvironmentFactory.getDefault()
        _engine(env).run(getattr(env, "stream_checkpoint", None))

    @staticmethod
    def setCheckPointConf(interval_s: float = 1800.0, directory: Optional[str] = None,
                          every_batches: Optional[int] = None, env=None):
        """Reference ``StreamOperator.setCheckPointConf`` (``StreamOperator.java:216-239``: a checkpoint every
        30 min, exactly-once).  Here a checkpoint is a consistent cut at a micro-batch boundary: how many
        micro-batches every source has delivered plus the state of every stateful operator (``_state_dict``),
        written atomically to ``directory`` (default ``$ALINK_CKPT_DIR`` or ``./alink_stream_ckpt``) every
        ``interval_s`` seconds (or ``every_batches`` micro-batches).  Re-running the same program restores the
        operator state and skips the delivered micro-batches: exactly-once for operator state, at-least-once
        for external sinks (batches after the checkpoint are emitted again).  A completed run deletes it."""
        import os
        env = env or MLEnvironmentFactory.getDefault()
        env.stream_checkpoint = {"interval_s": float(interval_s), "every_batches": every_batches,
                                 "dir": directory or os.environ.get("ALINK_CKPT_DIR", "alink_stream_ckpt")}

    # operators with state override these (tensors / numbers / lists / dicts only: loaded with weights_only)
    def _state_dict(self):
        return None

    def _load_state_dict(self, state):
        pass

    def select(self, fields):
        from .sql import SelectStreamOp
        if isinstance(fields, (list, tuple)):
            fields = ",".join(fields)
        return self.link(SelectStreamOp().setClause(fields))

    def where(self, predicate: str):
        from .sql import WhereStreamOp
        return self.link(WhereStreamOp().setClause(predicate))

    filter = where

    def alias(self, fields):
        from .sql import AsStreamOp
        if isinstance(fields, (list, tuple)):
            fields = ",".join(fields)
        return self.link(AsStreamOp().setClause(fields))

    def unionAll(self, other):
        from .sql import UnionAllStreamOp
        return UnionAllStreamOp().linkFrom(self, other)

    @staticmethod
    def fromDataframe(df, schemaStr: Optional[str] = None):
        from .source import MemSourceStreamOp
        return MemSourceStreamOp.fromDataframe(df, schemaStr)

    def sample(self, ratio: float):
        from .dataproc import SampleStreamOp
        return self.link(SampleStreamOp().setRatio(ratio))


class StreamSourceOp(StreamOperator):
    """Base of stream sources: ``batches()`` yields micro-batches for this rank."""

    @staticmethod
    def of(params):
        """Re-create the registered stream source named by ``params`` (ioName / ioType)."""
        from ...common.io_registry import AnnotationUtils, IOType
        return AnnotationUtils.of(params, IOType.SourceStream)
    _NO_AUTO_PARAMS = False
    BATCH_SIZE = 1024

    def linkFrom(self, *inputs):
        raise RuntimeError("Source operator does not support linkFrom()")

    def batches(self) -> Iterator[MTable]:
        raise NotImplementedError

    def _emit(self, mt):
        super()._emit(mt)

    def link(self, nxt):
        _engine(self.env).register_source(self)
        return super().link(nxt)

    def _ensure_registered(self):
        _engine(self.env).register_source(self)


class MapStreamOp(StreamOperator):
    MAPPER: Callable[..., Mapper] = None
    EMPTY_PASSTHROUGH = True

    def __init__(self, params: Optional[Params] = None, mapper=None, **kw):
        super().__init__(params, **kw)
        if mapper is not None:
            self.MAPPER = mapper

    def linkFrom(self, *inputs):
        (inp,) = self._connect(*inputs)
        self._mapper = self.MAPPER(inp.getSchema(), self.getParams())
        self._mapper.open()
        self._schema = self._mapper.getOutputSchema()
        _register_upstream_sources(inp)
        return self

    def on_batch(self, port, mt):
        self._emit(self._mapper.map_table(mt))


class ModelMapStreamOp(StreamOperator):
    """Stream predict with a static model (reference ``ModelMapStreamOp.java:39-56``)."""
    MAPPER: Callable[..., ModelMapper] = None
    EMPTY_PASSTHROUGH = True

    def __init__(self, model=None, params: Optional[Params] = None, mapper=None, **kw):
        if isinstance(model, Params):
            model, params = None, model
        super().__init__(params, **kw)
        self._model_op = model
        if mapper is not None:
            self.MAPPER = mapper

    def linkFrom(self, *inputs):
        (inp,) = self._connect(*inputs)
        from ..batch.utils import load_model_mapper
        from ...common.directreader import DataBridgeModelSource, DirectReader
        # the batch model reaches the stream through DirectReader under the configured policy
        # (reference ModelMapStreamOp.java:39-56 -> DataBridgeModelSource)
        self._bridge = DirectReader.collect(self._model_op)
        self._mapper = load_model_mapper(self.MAPPER, DataBridgeModelSource(self._bridge), inp.getSchema(),
                                         self.getParams())
        self._schema = self._mapper.getOutputSchema()
        _register_upstream_sources(inp)
        return self

    def on_batch(self, port, mt):
        self._emit(self._mapper.map_table(mt))


class FlatMapStreamOp(StreamOperator):
    MAPPER: Callable[..., FlatMapper] = None
    EMPTY_PASSTHROUGH = True

    def __init__(self, params: Optional[Params] = None, mapper=None, **kw):
        super().__init__(params, **kw)
        if mapper is not None:
            self.MAPPER = mapper

    def linkFrom(self, *inputs):
        (inp,) = self._connect(*inputs)
        self._mapper = self.MAPPER(inp.getSchema(), self.getParams())
        self._schema = self._mapper.getOutputSchema()
        _register_upstream_sources(inp)
        return self

    def on_batch(self, port, mt):
        self._emit(self._mapper.flat_map_table(mt))


def _register_upstream_sources(op: StreamOperator, seen=None):
    """Make sure every source feeding ``op`` is registered with the engine."""
    seen = seen if seen is not None else set()
    if id(op) in seen:
        return
    seen.add(id(op))
    if isinstance(op, StreamSourceOp):
        op._ensure_registered()
    for up in getattr(op, "_upstreams", []):
        _register_upstream_sources(up, seen)
