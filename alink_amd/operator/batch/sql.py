"""SQL-sugar batch operators (reference ``A/operator/batch/sql/*``, ``BatchSqlOperators.java``).

Row-local operators (select/as/where/filter) run on each rank's partition; global ones (distinct, orderBy,
groupBy, joins, set operations) gather their inputs, evaluate once and keep this rank's block of the result.
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
        self.setOutputTable(_global(self.env, E.sql_distinct, mt))
        return self


class OrderByBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        p = self.getParams()
        lim = p.get(self._param_infos["limit"]) if p.contains("limit") else None
        off = p.get(self._param_infos["offset"]) if p.contains("offset") else None
        fet = p.get(self._param_infos["fetch"]) if p.contains("fetch") else None
        self.setOutputTable(_global(self.env, lambda t: E.sql_order_by(t, self.getClause(), self.getOrder(), lim,
                                                                       off, fet), mt))
        return self


class GroupByBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        self.setOutputTable(_global(self.env, lambda t: E.sql_group_by(t, self.getGroupByPredicate(),
                                                                       self.getSelectClause()), mt))
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
        self.setOutputTable(_global(self.env, lambda x, y: E.sql_join(x, y, self.getJoinPredicate(),
                                                                      self.getSelectClause(), how), a, b))
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
            out = t if out is None else _global(self.env, lambda x, y: fn(x, y, self.ALL), out, t)
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


_Q = re.compile(r"^\s*select\s+(?P<sel>.*?)\s+from\s+(?P<tab>[\w`]+)(?:\s+(?:as\s+)?(?P<al>\w+))?"
                r"(?:\s+where\s+(?P<where>.*?))?(?:\s+group\s+by\s+(?P<gb>.*?))?"
                r"(?:\s+order\s+by\s+(?P<ob>.*?))?(?:\s+limit\s+(?P<lim>\d+))?\s*$", re.I | re.S)


def sql_query(query: str, env=None):
    """``BatchOperator.sqlQuery``: single-table SELECT [WHERE] [GROUP BY] [ORDER BY] [LIMIT] over tables
    registered with ``registerTableName``."""
    from ...common.mlenv import MLEnvironmentFactory
    from .source import TableSourceBatchOp
    env = env or MLEnvironmentFactory.getDefault()
    m = _Q.match(query)
    if not m:
        raise ValueError(f"unsupported query: {query}")
    tab = m.group("tab").strip("`")
    op = env.tables[tab]
    mt = op.getOutputTable()
    if m.group("where"):
        mt = E.sql_where(mt, m.group("where"))
    if m.group("gb"):
        mt = _global(env, lambda t: E.sql_group_by(t, m.group("gb"), m.group("sel")), mt)
    else:
        mt = E.sql_select(mt, m.group("sel"))
    if m.group("ob"):
        mt = _global(env, lambda t: E.sql_order_by(t, m.group("ob"),
                                                   limit=int(m.group("lim")) if m.group("lim") else None), mt)
    return TableSourceBatchOp(mt)
