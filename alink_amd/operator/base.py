"""Operator framework: ``AlgoOperator`` / ``BatchOperator``.

Reference: ``A/operator/AlgoOperator.java:24-271`` and ``A/operator/batch/BatchOperator.java:52-604``
(``link/linkTo/linkFrom``, SQL sugar, ``collect/print/lazyPrint/lazyCollect/execute``, side outputs).

Execution model: ``linkFrom`` executes immediately on this rank's partition (eager SPMD: every rank runs
the same program on its own block of rows; collectives inside algorithms keep ranks in lock step).
Observable laziness is preserved: ``lazyPrint``/``lazyCollect`` fire at the next trigger
(``print``/``collect``/``execute``) in registration order, exactly like the reference's
``triggerLazyEvaluation`` (``BatchOperator.java:527-547``).
"""
from __future__ import annotations

import sys
from typing import Any, Callable, List, Optional, Sequence

from ..common.mlenv import MLEnvironment, MLEnvironmentFactory
from ..common.params import ParamInfo, Params, WithParams
from ..common.table import MTable, Row
from ..common.types import TableSchema
from ..parallel import comm
from ..utils import trace as _trace

__all__ = ["AlgoOperator", "BatchOperator", "gather_table", "gather_rows", "partition_rows", "format_rows",
           "register_op"]

OP_REGISTRY = {}


def register_op(cls):
    OP_REGISTRY[cls.__name__] = cls
    return cls


def partition_bounds(n: int, env: MLEnvironment):
    """Contiguous block [lo, hi) of n global rows owned by this rank."""
    ws, r = env.world_size, env.rank
    base, rem = divmod(n, ws)
    lo = r * base + min(r, rem)
    hi = lo + base + (1 if r < rem else 0)
    return lo, hi


def partition_rows(rows: Sequence[Any], env: MLEnvironment) -> List[Any]:
    lo, hi = partition_bounds(len(rows), env)
    return list(rows[lo:hi])


def gather_table(mt: MTable, env: Optional[MLEnvironment] = None) -> MTable:
    """Full table on every rank (partitions concatenated in rank order = global row order)."""
    if mt is None:
        return None
    if mt.replicated or comm.get_world_size() == 1:
        return mt
    out = _gather_columnar(mt)
    out.replicated = True
    return out


def _col_kind(c) -> tuple:
    """Wire form of a column for the columnar gather: ('tensor', dtype, trailing shape), ('sparse',),
    ('string',) or ('object',)."""
    import torch
    from ..common.linalg.block import SparseBlock
    from ..common.strings import StringBlock
    v = c.values
    if isinstance(v, torch.Tensor):
        return ("tensor", str(v.dtype), tuple(v.shape[1:]))
    if isinstance(v, SparseBlock):
        return ("sparse",)
    if isinstance(v, StringBlock) or (isinstance(v, list) and all(x is None or isinstance(x, str) for x in v)):
        return ("string",)
    return ("object",)


def _gather_columnar(mt: MTable) -> MTable:
    """Partitions concatenated in rank order, one column at a time in its native form: tensor columns (numeric,
    dense-vector blocks) and their null masks by a variable-length tensor all-gather (RCCL / gloo), sparse
    blocks as (row lengths, col, val), string columns as packed UTF-8 (lengths, -1 = NULL, + bytes); only
    columns of arbitrary Python objects are pickled.  Replaces a pickled all-gather of whole tables."""
    import torch
    from ..common.linalg.block import SparseBlock
    from ..common.strings import StringBlock
    from ..common.table import Column
    kinds = [_col_kind(c) for c in mt.cols]
    allk = comm.all_gather_object(kinds)
    cdev = comm.collective_device()
    cols = []
    for i, c in enumerate(mt.cols):
        ks = {k[i] for k in allk}
        kind = next(iter(ks)) if len(ks) == 1 else ("object",)
        v = c.values
        if kind[0] == "tensor":
            vals = comm.all_gather_varlen(v.to(cdev)).cpu()
            nulls = None
            flags = comm.all_gather_object(c.nulls is not None)
            if any(flags):
                m = c.nulls if c.nulls is not None else torch.zeros(v.shape[0], dtype=torch.bool)
                nulls = comm.all_gather_varlen(m.to(torch.uint8).to(cdev)).cpu().to(torch.bool)
            cols.append(Column(vals, nulls))
        elif kind[0] == "sparse":
            ln = (v.crow[1:] - v.crow[:-1]).to(cdev)
            rl = comm.all_gather_varlen(ln).cpu()
            col = comm.all_gather_varlen(v.col.to(cdev)).cpu()
            val = comm.all_gather_varlen(v.val.to(cdev)).cpu()
            size = max(comm.all_gather_object(int(v.size)))
            crow = torch.zeros(rl.numel() + 1, dtype=torch.int64)
            torch.cumsum(rl, 0, out=crow[1:])
            nulls = None
            if any(comm.all_gather_object(c.nulls is not None)):
                m = c.nulls if c.nulls is not None else torch.zeros(len(v), dtype=torch.bool)
                nulls = comm.all_gather_varlen(m.to(torch.uint8).to(cdev)).cpu().to(torch.bool)
            cols.append(Column(SparseBlock(crow, col, val, size, getattr(v, "dense_ratio", None)), nulls))
        elif kind[0] == "string":
            blk = v if isinstance(v, StringBlock) else StringBlock.from_list(c.to_list())
            ln = torch.where(blk.null_mask(), torch.full_like(blk.lengths(), -1), blk.lengths())
            rl = comm.all_gather_varlen(ln.to(cdev)).cpu()
            data = comm.all_gather_varlen(blk.data.to(cdev)).cpu()
            nulls = rl < 0
            cols.append(Column(StringBlock.from_parts(rl.clamp(min=0), data, nulls if bool(nulls.any()) else None)))
        else:
            parts = comm.all_gather_object(c.to_list())
            cols.append(Column([x for p in parts for x in p]))
    return MTable(mt.schema, cols, True)


def gather_rows(mt: MTable) -> List[Row]:
    return gather_table(mt).rows()


def _fmt_val(v):
    if isinstance(v, float):
        return "%.4f" % v
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def format_title(names):
    return "|".join(names) + "\n" + "|".join("-" * (len(n) if n is not None else 4) for n in names)


def format_rows(names, rows) -> str:
    lines = [format_title(names)]
    for r in rows:
        lines.append("|".join(_fmt_val(v) for v in r))
    return "\n".join(lines)


def _traced_link(fn, opname):
    """``linkFrom`` as an ``op`` span of the timeline (``utils.trace``; one attribute check when tracing is off)."""
    import functools

    @functools.wraps(fn)
    def linkFrom(self, *inputs):
        if any(isinstance(t, MTable) for t in inputs):     # a model table (PipelineModel.getModelData()) as input
            inputs = tuple(BatchOperator.fromTable(t) if isinstance(t, MTable) else t for t in inputs)
        if not _trace.enabled():
            return fn(self, *inputs)
        with _trace.span(opname, "op"):
            return fn(self, *inputs)
    linkFrom._alink_traced = True
    return linkFrom


class AlgoOperator(WithParams):
    _NO_AUTO_PARAMS = True
    PARAMS = [ParamInfo("MLEnvironmentId", int, "ID of ML environment.", default=0)]

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        lf = cls.__dict__.get("linkFrom")
        if lf is not None and not getattr(lf, "_alink_traced", False):
            cls.linkFrom = _traced_link(lf, cls.__name__)

    def __init__(self, params: Optional[Params] = None, **kwargs):
        super().__init__(params, **kwargs)
        self._output: Optional[MTable] = None
        self._side_outputs: List[MTable] = []

    # ---- env ----
    def getMLEnvironmentId(self) -> int:
        return self.getParams().get(AlgoOperator.PARAMS[0])

    def setMLEnvironmentId(self, i: int):
        self.getParams().set(AlgoOperator.PARAMS[0], i)
        return self

    @property
    def env(self) -> MLEnvironment:
        return MLEnvironmentFactory.get(self.getMLEnvironmentId())

    # ---- output ----
    def setOutputTable(self, mt: MTable):
        self._output = mt
        return self

    def getOutputTable(self) -> MTable:
        if self._output is None:
            raise RuntimeError(f"There is no output. Please call current BatchOperator's 'link' or related "
                               f"method firstly, or this BatchOperator has no output. ({type(self).__name__})")
        return self._output

    def setSideOutputTables(self, tables: List[MTable]):
        self._side_outputs = list(tables)
        return self

    def getSideOutputTables(self):
        return self._side_outputs

    def getSchema(self) -> TableSchema:
        return self.getOutputTable().schema

    def getColNames(self):
        return self.getOutputTable().getColNames()

    def getColTypes(self):
        return self.getOutputTable().getColTypes()

    @staticmethod
    def checkAndGetFirst(inputs):
        if len(inputs) == 1 and isinstance(inputs[0], (list, tuple)):
            inputs = inputs[0]
        if len(inputs) != 1:
            raise ValueError("Only support one input.")
        return inputs[0]

    def checkOpSize(self, size, inputs):
        if len(inputs) != size:
            raise ValueError(f"The size of operators should be equal to {size}, current: {len(inputs)}")


class BatchOperator(AlgoOperator):
    """Batch operator: wraps this rank's partition of a table."""

    # ---- linking ----
    def link(self, nxt: "BatchOperator"):
        nxt.linkFrom(self)
        return nxt

    linkTo = link

    def linkFrom(self, *inputs: "BatchOperator"):
        raise NotImplementedError(f"{type(self).__name__}.linkFrom")

    def getSideOutput(self, idx: int) -> "BatchOperator":
        if not self._side_outputs:
            raise RuntimeError("There is no side output.")
        if idx < 0 or idx >= len(self._side_outputs):
            raise RuntimeError("There is no  side output.")
        from .batch.source import TableSourceBatchOp
        return TableSourceBatchOp(self._side_outputs[idx]).setMLEnvironmentId(self.getMLEnvironmentId())

    def getSideOutputCount(self) -> int:
        return len(self._side_outputs)

    @staticmethod
    def fromTable(table: MTable) -> "BatchOperator":
        """A batch operator over an existing table (reference ``BatchOperator.fromTable``)."""
        from .batch.source import TableSourceBatchOp
        return TableSourceBatchOp(table)

    # ---- execution / observation ----
    @classmethod
    def execute(cls, env: Optional[MLEnvironment] = None):
        env = env or MLEnvironmentFactory.getDefault()
        cls._trigger(env)

    @staticmethod
    def _trigger(env: MLEnvironment):
        lm = env.lazy
        try:
            sinks = lm.getLazySinks()
            for op, lazy in sinks:
                rows = gather_rows(op.getOutputTable())
                lazy.addValue((op, rows))
        finally:
            lm.clearVirtualSinks()

    def collect(self) -> List[Row]:
        lazy = self.env.lazy.genLazySink(self)
        self._trigger(self.env)
        return lazy.getLatestValue()[1]

    def collectToDataframe(self):
        import pandas as pd
        rows = self.collect()
        return pd.DataFrame([list(r) for r in rows], columns=self.getColNames())

    def collectToMTable(self) -> MTable:
        return gather_table(self.getOutputTable())

    def count(self) -> int:
        n = self.getOutputTable().num_rows
        if self.getOutputTable().replicated:
            return n
        return sum(comm.all_gather_object(n))

    def print(self, n: int = -1, title: Optional[str] = None):
        self.lazyPrint(n, title)
        self._trigger(self.env)
        return self

    def lazyPrint(self, n: int = -1, title: Optional[str] = None):
        op = self.firstN(n) if n is not None and n > 0 else self
        lazy = self.env.lazy.genLazySink(op)
        env = self.env

        def cb(d):
            o, rows = d
            if env.rank == 0:
                if title is not None:
                    print(title)
                print(format_rows(o.getColNames(), rows))
                sys.stdout.flush()
        lazy.addCallback(cb)
        return self

    def lazyCollect(self, *callbacks: Callable[[List[Row]], None]):
        lazy = self.env.lazy.genLazySink(self)
        for cb in callbacks:
            lazy.addCallback(lambda d, cb=cb: cb(d[1]))
        return self

    def lazyPrintStatistics(self, title=None):
        from .batch.feature import SummarizerBatchOp
        s = SummarizerBatchOp().setMLEnvironmentId(self.getMLEnvironmentId())
        self.link(s)
        s.lazyPrintSummary(title)
        return self

    def collectStatistics(self):
        from .batch.feature import SummarizerBatchOp
        s = SummarizerBatchOp().setMLEnvironmentId(self.getMLEnvironmentId())
        self.link(s)
        return s.collectSummary()

    # ---- sugar that links well-known ops ----
    def firstN(self, n: int):
        from .batch.dataproc import FirstNBatchOp
        return self.link(FirstNBatchOp().setSize(n).setMLEnvironmentId(self.getMLEnvironmentId()))

    def sample(self, ratio: float, withReplacement: bool = False):
        from .batch.dataproc import SampleBatchOp
        return self.link(SampleBatchOp().setRatio(ratio).setWithReplacement(withReplacement)
                         .setMLEnvironmentId(self.getMLEnvironmentId()))

    def sampleWithSize(self, numSamples: int, withReplacement: bool = False):
        from .batch.dataproc import SampleWithSizeBatchOp
        return self.link(SampleWithSizeBatchOp().setSize(numSamples).setWithReplacement(withReplacement)
                         .setMLEnvironmentId(self.getMLEnvironmentId()))

    def select(self, fields):
        from .batch.sql import SelectBatchOp
        if isinstance(fields, (list, tuple)):
            fields = ",".join(fields)
        return self.link(SelectBatchOp().setClause(fields).setMLEnvironmentId(self.getMLEnvironmentId()))

    def alias(self, fields):
        from .batch.sql import AsBatchOp
        if isinstance(fields, (list, tuple)):
            fields = ",".join(fields)
        return self.link(AsBatchOp().setClause(fields).setMLEnvironmentId(self.getMLEnvironmentId()))

    as_ = alias

    def where(self, predicate: str):
        from .batch.sql import WhereBatchOp
        return self.link(WhereBatchOp().setClause(predicate).setMLEnvironmentId(self.getMLEnvironmentId()))

    def filter(self, predicate: str):
        from .batch.sql import FilterBatchOp
        return self.link(FilterBatchOp().setClause(predicate).setMLEnvironmentId(self.getMLEnvironmentId()))

    def distinct(self):
        from .batch.sql import DistinctBatchOp
        return self.link(DistinctBatchOp().setMLEnvironmentId(self.getMLEnvironmentId()))

    def orderBy(self, field: str, limit: int = -1, fetch: int = -1, offset: int = -1, isAscending: bool = True):
        from .batch.sql import OrderByBatchOp
        op = OrderByBatchOp().setClause(field).setOrder("asc" if isAscending else "desc")
        if limit is not None and limit >= 0:
            op.setLimit(limit)
        if fetch is not None and fetch >= 0:
            op.setFetch(fetch)
        if offset is not None and offset >= 0:
            op.setOffset(offset)
        return self.link(op.setMLEnvironmentId(self.getMLEnvironmentId()))

    def groupBy(self, by: str, select: str):
        from .batch.sql import GroupByBatchOp
        return self.link(GroupByBatchOp().setGroupByPredicate(by).setSelectClause(select)
                         .setMLEnvironmentId(self.getMLEnvironmentId()))

    def _join(self, kind, right, cond, select):
        from .batch import sql
        cls = {"inner": sql.JoinBatchOp, "left": sql.LeftOuterJoinBatchOp, "right": sql.RightOuterJoinBatchOp,
               "full": sql.FullOuterJoinBatchOp}[kind]
        op = cls().setJoinPredicate(cond).setSelectClause(select).setMLEnvironmentId(self.getMLEnvironmentId())
        return op.linkFrom(self, right)

    def join(self, right, joinPredicate: str, selectClause: str = "*"):
        return self._join("inner", right, joinPredicate, selectClause)

    def leftOuterJoin(self, right, joinPredicate: str, selectClause: str = "*"):
        return self._join("left", right, joinPredicate, selectClause)

    def rightOuterJoin(self, right, joinPredicate: str, selectClause: str = "*"):
        return self._join("right", right, joinPredicate, selectClause)

    def fullOuterJoin(self, right, joinPredicate: str, selectClause: str = "*"):
        return self._join("full", right, joinPredicate, selectClause)

    def _setop(self, cls_name, other):
        from .batch import sql
        return getattr(sql, cls_name)().setMLEnvironmentId(self.getMLEnvironmentId()).linkFrom(self, other)

    def union(self, other):
        return self._setop("UnionBatchOp", other)

    def unionAll(self, other):
        return self._setop("UnionAllBatchOp", other)

    def intersect(self, other):
        return self._setop("IntersectBatchOp", other)

    def intersectAll(self, other):
        return self._setop("IntersectAllBatchOp", other)

    def minus(self, other):
        return self._setop("MinusBatchOp", other)

    def minusAll(self, other):
        return self._setop("MinusAllBatchOp", other)

    def udf(self, selectedColName, outputColName, func, reservedColNames=None):
        from .batch.utils import UDFBatchOp
        op = UDFBatchOp().setSelectedCols([selectedColName]).setOutputCol(outputColName).setFunc(func)
        if reservedColNames is not None:
            op.setReservedCols(reservedColNames)
        return self.link(op.setMLEnvironmentId(self.getMLEnvironmentId()))

    def udtf(self, selectedColName, outputColNames, func, reservedColNames=None):
        from .batch.utils import UDTFBatchOp
        op = UDTFBatchOp().setSelectedCols([selectedColName]).setOutputCols(outputColNames).setFunc(func)
        if reservedColNames is not None:
            op.setReservedCols(reservedColNames)
        return self.link(op.setMLEnvironmentId(self.getMLEnvironmentId()))

    def registerTableName(self, name: str):
        self.env.tables[name] = self
        return self

    @staticmethod
    def sqlQuery(query: str):
        from .batch.sql import sql_query
        return sql_query(query)

    @staticmethod
    def fromDataframe(df, schemaStr: Optional[str] = None):
        from .batch.source import MemSourceBatchOp
        return MemSourceBatchOp.fromDataframe(df, schemaStr)

    def __repr__(self):
        return f"{type(self).__name__}({self.getParams()})"
