"""SQL-sugar batch operators (reference ``A/operator/batch/sql/*``, ``BatchSqlOperators.java``).

Row-local operators (select/as/where/filter) run on each rank's partition.  Global ones follow the
reference's plans (``BatchSqlOperators.java:51-388`` -> Flink SQL: repartition, then evaluate per partition):

* distinct, set operations: hash-partition by all columns, evaluate locally;
* groupBy on plain columns: hash-partition by the group keys; equi-joins: hash-partition both sides by the
  join keys (``parallel/shuffle.py``: murmur3 key hash, one all-to-all per column);
* orderBy: range partition on sampled splitters of the sort key (rank r holds the r-th key range, so the
  ranks' partitions concatenated are the global order), local sort; offset/limit/fetch by global position;
* anything else (non-equi joins, expression group keys): gather, evaluate once, keep this rank's block.
"""
from __future__ import annotations

import re

from ...common.table import MTable
from ...parallel import comm
from ..base import BatchOperator, gather_table, partition_bounds
from ..common.sql import engine as E

__all__ = ["SelectBatchOp", "AsBatchOp", "WhereBatchOp", "FilterBatchOp", "DistinctBatchOp", "OrderByBatchOp",
           "GroupByBatchOp", "JoinBatchOp", "LeftOuterJoinBatchOp", "RightOuterJoinBatchOp", "FullOuterJoinBatchOp",
           "UnionBatchOp", "UnionAllBatchOp", "IntersectBatchOp", "IntersectAllBatchOp", "MinusBatchOp",
           "MinusAllBatchOp", "sql_query", "registerFunction"]


def _local_ok(tables):
    return all(t.replicated for t in tables) or comm.get_world_size() == 1


def _copartitioned(fn, parts, *tables_and_keys):
    """Hash-partition every (table, key columns) input, evaluate ``fn`` on this rank's co-partitions."""
    from ...parallel.shuffle import hash_partition
    tabs = [hash_partition(t, k) for t, k in tables_and_keys]
    out = fn(*tabs)
    out.replicated = False
    return out


def _order_by_distributed(env, mt, clause, order, lim, off, fet):
    """Range-partitioned sort: sampled splitters (all-gathered), rows to their key range, local sort."""
    import bisect
    import numpy as np
    from ...parallel.shuffle import exchange
    ws, me = comm.get_world_size(), comm.get_rank()
    keyf = E.order_key_fn(mt, clause, order)
    rows = mt.rows()
    step = max(1, len(rows) // 64)
    sample = [tuple(r) for r in rows[::step]]
    allsmp = [r for part in comm.all_gather_object(sample) for r in part]
    allsmp.sort(key=keyf)
    spl = [keyf(allsmp[int(round(q))]) for q in np.linspace(0, len(allsmp) - 1, ws + 1)[1:-1]] if allsmp else []
    dest = np.asarray([bisect.bisect_right(spl, keyf(r)) for r in rows], dtype=np.int64)
    part = exchange(mt, dest)
    part = E.sql_order_by(part, clause, order)
    # offset / fetch / limit by global position
    sizes = comm.all_gather_object(int(part.num_rows))
    start = sum(sizes[:me])
    lo, hi = 0, sum(sizes)
    if off is not None and off > 0:
        lo = off
    if fet is not None and fet >= 0:
        hi = min(hi, lo + fet)
    if lim is not None and lim >= 0:
        hi = min(hi, lo + lim)
    a, b = max(lo - start, 0), max(min(hi - start, part.num_rows), 0)
    out = part.slice(a, max(a, b))
    out.replicated = False
    return out


def _global(env, fn, *tables):
    if all(t.replicated for t in tables) or comm.get_world_size() == 1:
        out = fn(*tables)
        out.replicated = all(t.replicated for t in tables)
        return out
    full = fn(*[gather_table(t) for t in tables])
    lo, hi = partition_bounds(full.num_rows, env)
    out = full.slice(lo, hi)
    out.replicated = False
    return out


class SelectBatchOp(BatchOperator):
    def __init__(self, clause=None, params=None, **kw):
        super().__init__(params, **kw)
        if clause is not None:
            self.setClause(clause)

    def linkFrom(self, *inputs):
        self.setOutputTable(E.sql_select(self.checkAndGetFirst(inputs).getOutputTable(), self.getClause()))
        return self


class AsBatchOp(SelectBatchOp):
    def linkFrom(self, *inputs):
        self.setOutputTable(E.sql_as(self.checkAndGetFirst(inputs).getOutputTable(), self.getClause()))
        return self


class WhereBatchOp(SelectBatchOp):
    def linkFrom(self, *inputs):
        self.setOutputTable(E.sql_where(self.checkAndGetFirst(inputs).getOutputTable(), self.getClause()))
        return self


class FilterBatchOp(WhereBatchOp):
    pass


class DistinctBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        if _local_ok([mt]):
            self.setOutputTable(_global(self.env, E.sql_distinct, mt))
        else:
            self.setOutputTable(_copartitioned(E.sql_distinct, None, (mt, list(range(len(mt.schema.names))))))
        return self


class OrderByBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        lim = p.get(self._param_infos["limit"]) if p.contains("limit") else None
        off = p.get(self._param_infos["offset"]) if p.contains("offset") else None
        fet = p.get(self._param_infos["fetch"]) if p.contains("fetch") else None
        if _local_ok([mt]):
            self.setOutputTable(_global(self.env, lambda t: E.sql_order_by(t, self.getClause(), self.getOrder(),
                                                                           lim, off, fet), mt))
        else:
            self.setOutputTable(_order_by_distributed(self.env, mt, self.getClause(), self.getOrder(), lim, off,
                                                      fet))
        return self


class GroupByBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        fn = (lambda t: E.sql_group_by(t, self.getGroupByPredicate(), self.getSelectClause()))
        keys = None if _local_ok([mt]) else E.group_key_cols(mt.schema, self.getGroupByPredicate())
        if keys:
            self.setOutputTable(_copartitioned(fn, None, (mt, keys)))
        else:
            self.setOutputTable(_global(self.env, fn, mt))
        return self


class _JoinBase(BatchOperator):
    HOW = "inner"

    def linkFrom(self, *inputs):
        if len(inputs) == 1 and isinstance(inputs[0], (list, tuple)):
            inputs = inputs[0]
        self.checkOpSize(2, inputs)
        a, b = inputs[0].getOutputTable(), inputs[1].getOutputTable()
        how = self.HOW
        if how == "inner" and self.getParams().contains("type"):
            t = self.getParams().get(self._param_infos["type"])
            how = {"JOIN": "inner", "LEFTOUTERJOIN": "left", "RIGHTOUTERJOIN": "right",
                   "FULLOUTERJOIN": "full"}.get(str(getattr(t, "name", t)).upper(), "inner")
        fn = (lambda x, y: E.sql_join(x, y, self.getJoinPredicate(), self.getSelectClause(), how))
        if not _local_ok([a, b]):
            kl, kr = E.join_keys(a.schema, b.schema, self.getJoinPredicate())
            if kl:
                self.setOutputTable(_copartitioned(fn, None, (a, kl), (b, kr)))
                return self
        self.setOutputTable(_global(self.env, fn, a, b))
        return self


class JoinBatchOp(_JoinBase):
    HOW = "inner"


class LeftOuterJoinBatchOp(_JoinBase):
    HOW = "left"


class RightOuterJoinBatchOp(_JoinBase):
    HOW = "right"


class FullOuterJoinBatchOp(_JoinBase):
    HOW = "full"


class _SetOp(BatchOperator):
    FN = None
    ALL = False
    LOCAL = False

    def linkFrom(self, *inputs):
        if len(inputs) == 1 and isinstance(inputs[0], (list, tuple)):
            inputs = inputs[0]
        tabs = [i.getOutputTable() for i in inputs]
        fn = type(self).FN
        if self.LOCAL and not any(t.replicated for t in tabs):
            out = tabs[0]
            for t in tabs[1:]:
                out = fn(out, t, self.ALL)
            self.setOutputTable(out)
            return self
        out = None
        for t in tabs:
            if out is None:
                out = t
            elif _local_ok([out, t]):
                out = _global(self.env, lambda x, y: fn(x, y, self.ALL), out, t)
            else:
                allc = list(range(len(t.schema.names)))
                out = _copartitioned(lambda x, y: fn(x, y, self.ALL), None, (out, allc), (t, allc))
        self.setOutputTable(out)
        return self


class UnionAllBatchOp(_SetOp):
    FN = staticmethod(E.sql_union)
    ALL = True
    LOCAL = True


class UnionBatchOp(_SetOp):
    FN = staticmethod(E.sql_union)


class IntersectBatchOp(_SetOp):
    FN = staticmethod(E.sql_intersect)


class IntersectAllBatchOp(_SetOp):
    FN = staticmethod(E.sql_intersect)
    ALL = True


class MinusBatchOp(_SetOp):
    FN = staticmethod(E.sql_minus)


class MinusAllBatchOp(_SetOp):
    FN = staticmethod(E.sql_minus)
    ALL = True


def registerFunction(name, fn):
    from ..common.sql.udf import register_function
    register_function(name, fn)


def sql_query(query: str, env=None):
    """``BatchOperator.sqlQuery`` over tables registered with ``registerTableName``: SELECT [DISTINCT] with
    joins (inner/left/right/full/cross, comma joins), subqueries in FROM and in expressions, WHERE, GROUP BY,
    HAVING, UNION/INTERSECT/EXCEPT [ALL], ORDER BY, LIMIT/OFFSET (``operator/common/sql/query.py``)."""
    from ...common.mlenv import MLEnvironmentFactory
    from ..common.sql.query import execute_query
    from .source import TableSourceBatchOp
    env = env or MLEnvironmentFactory.getDefault()
    text = query.strip().rstrip(";")
    used = [op.getOutputTable() for name, op in env.tables.items()
            if re.search(r"(?<![\w`])" + re.escape(name) + r"(?![\w`])", text, re.I)]
    names = [name for name, op in env.tables.items()
             if re.search(r"(?<![\w`])" + re.escape(name) + r"(?![\w`])", text, re.I)]
    # every rank evaluates the query over the gathered tables, then keeps its slice (as the other global ops)
    return TableSourceBatchOp(_global(env, lambda *ts: execute_query(text, dict(zip(names, ts))), *used))
