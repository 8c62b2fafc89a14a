"""Stream SQL operators (reference ``A/operator/stream/sql/*`` + ``StreamSqlOperators.java:46-94``):
select / as / where / filter run per micro-batch; unionAll merges two streams."""
from __future__ import annotations

from typing import Optional

from ...common.params import Params
from ..common.sql import engine as E
from .base import StreamOperator

__all__ = ["SelectStreamOp", "AsStreamOp", "WhereStreamOp", "FilterStreamOp", "UnionAllStreamOp"]


class _RowLocal(StreamOperator):
    FN = None

    def __init__(self, clause=None, params: Optional[Params] = None, **kw):
        if isinstance(clause, Params):
            clause, params = None, clause
        super().__init__(params, **kw)
        if clause is not None:
            self.setClause(clause)

    def linkFrom(self, *inputs):
        (inp,) = self._connect(*inputs)
        from ...common.table import MTable
        self._schema = type(self).FN(MTable.empty(inp.getSchema()), self.getClause()).schema
        return self

    def on_batch(self, port, mt):
        self._emit(type(self).FN(mt, self.getClause()))


class SelectStreamOp(_RowLocal):
    FN = staticmethod(E.sql_select)


class AsStreamOp(_RowLocal):
    FN = staticmethod(E.sql_as)


class WhereStreamOp(_RowLocal):
    FN = staticmethod(E.sql_where)


class FilterStreamOp(WhereStreamOp):
    pass


class UnionAllStreamOp(StreamOperator):
    def linkFrom(self, *inputs):
        ins = self._connect(*inputs)
        self._schema = ins[0].getSchema()
        return self

    def on_batch(self, port, mt):
        from ...common.table import MTable
        self._emit(MTable(self._schema, mt.cols, mt.replicated))
