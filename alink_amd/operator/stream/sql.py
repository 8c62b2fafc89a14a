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
    EMPTY_PASSTHROUGH = True

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


# ---------------------------------------------------------------------------------------------------
# windowed group-by (StreamSqlOperators.windowGroupBy: GROUP BY TUMBLE/HOP/SESSION(proctime, ...), keys)
# ---------------------------------------------------------------------------------------------------
import math as _math  # noqa: E402
import time as _time  # noqa: E402

from ...common.params import ParamInfo  # noqa: E402
from ...common.table import Column as _Column, MTable as _MTable  # noqa: E402

_UNIT_S = {"SECOND": 1, "MINUTE": 60, "HOUR": 3600, "DAY": 86400, "MONTH": 2592000, "YEAR": 31536000}


class WindowGroupByStreamOp(StreamOperator):
    """Aggregates rows per time window and ``groupByClause`` key; emits each window when it closes (or at
    end of stream).  Time is the micro-batch arrival time (Flink ``proctime``) unless ``timeCol`` names an
    event-time column in seconds."""
    EXTRA_PARAMS = [ParamInfo("timeCol", str, "event-time column (seconds); processing time if null",
                              default=None)]

    def __init__(self, params: Optional[Params] = None, **kw):
        super().__init__(params, **kw)
        self._pending = []          # (t, row)
        self._watermark = -_math.inf

    def _unit(self):
        u = self.getIntervalUnit()
        return _UNIT_S[getattr(u, "name", str(u)).upper()]

    def _kind(self):
        w = self.getWindowType()
        return getattr(w, "name", str(w)).upper()

    def linkFrom(self, *inputs):
        (inp,) = self._connect(*inputs)
        self._in_schema = inp.getSchema()
        self._schema = self._windowed(_MTable.empty(self._in_schema), 0.0, 0.0).schema
        return self

    def _windowed(self, rows_mt, start: float, end: float):
        """The aggregate of one window plus its ``window_start`` / ``window_end`` TIMESTAMP columns (the
        reference's ``CAST(TUMBLE_START(...) AS TIMESTAMP(3))`` pair, WindowGroupByStreamOp.java:80-82)."""
        import datetime as _dt
        from ...common.types import Types as _T
        agg = self._aggregate(rows_mt)
        n = agg.num_rows
        ts = [_dt.datetime.fromtimestamp(round(start, 3)), _dt.datetime.fromtimestamp(round(end, 3))]
        return agg.with_columns(["window_start", "window_end"], [_T.TIMESTAMP, _T.TIMESTAMP],
                                [_Column.from_values([v] * n, _T.TIMESTAMP) for v in ts])

    def _aggregate(self, mt):
        by = self.getGroupByClause()
        if by and by.strip():
            return E.sql_group_by(mt, by, self.getSelectClause())
        from ...common.types import Types as _T
        k = mt.with_columns(["__w"], [_T.INT], [_Column.from_values([0] * mt.num_rows, _T.INT)])
        return E.sql_group_by(k, "__w", self.getSelectClause())

    def _windows(self, t):
        L = float(self.getWindowLength() or 0) * self._unit()
        kind = self._kind()
        if kind == "HOP":
            S = float(self.getSlidingLength()) * self._unit()
            first = _math.floor((t - L) / S) + 1
            return [(k * S, k * S + L) for k in range(first, _math.floor(t / S) + 1)]
        return [(_math.floor(t / L) * L, _math.floor(t / L) * L + L)]

    def _flush(self, final=False):
        if not self._pending:
            return
        kind = self._kind()
        if kind == "SESSION":
            gap = float(self.getSessionGap()) * self._unit()
            self._pending.sort(key=lambda x: x[0])
            sessions, cur = [], [self._pending[0]]
            for t, r in self._pending[1:]:
                if t - cur[-1][0] > gap:
                    sessions.append(cur)
                    cur = []
                cur.append((t, r))
            keep = []
            if not final and cur and self._watermark - cur[-1][0] <= gap:
                keep = cur
            else:
                sessions.append(cur)
            for s in sessions:
                self._emit(self._windowed(_MTable.from_rows([r for _, r in s], self._in_schema), s[0][0],
                                          s[-1][0] + gap))
            self._pending = keep
            return
        buckets = {}
        for t, r in self._pending:
            for w in self._windows(t):
                buckets.setdefault(w, []).append((t, r))
        remaining = {}
        for w in sorted(buckets):
            if final or w[1] <= self._watermark:
                self._emit(self._windowed(_MTable.from_rows([r for _, r in buckets[w]], self._in_schema), w[0], w[1]))
            else:
                for item in buckets[w]:
                    remaining[id(item[1])] = item
        self._pending = list(remaining.values())

    def on_batch(self, port, mt):
        tc = self.getTimeCol()
        if tc:
            ts = [float(x) for x in mt.col(tc).to_list()]
        else:
            now = _time.time()
            ts = [now] * mt.num_rows
        rows = mt.rows()
        self._pending.extend(zip(ts, rows))
        if ts:
            self._watermark = max(self._watermark, max(ts))
        self._flush(False)

    def on_finish(self, port):
        self._flush(True)


__all__.append("WindowGroupByStreamOp")
