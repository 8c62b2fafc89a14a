"""SQL query planner/executor behind ``BatchOperator.sqlQuery`` (reference: the Flink ``TableEnvironment.sqlQuery``
that ``BatchOperator.sqlQuery`` forwards to, ``A/operator/batch/BatchOperator.java`` + ``A/common/MLEnvironment.java``
table registry).

Grammar (case-insensitive keywords)::

    query   := core ((UNION | INTERSECT | EXCEPT | MINUS) [ALL] core)* [ORDER BY keys] [LIMIT n] [OFFSET m]
    core    := SELECT [DISTINCT] items FROM from (join)* [WHERE e] [GROUP BY e, ...] [HAVING e]
             | '(' query ')'
    from    := name [[AS] alias] | '(' query ')' [AS] alias
    join    := [INNER | CROSS | LEFT [OUTER] | RIGHT [OUTER] | FULL [OUTER]] JOIN from [ON e] | ',' from

Expressions are the shared engine of ``expr.py`` (arithmetic, CASE, CAST, LIKE, IN, BETWEEN, functions,
aggregates) with ``alias.column`` qualification; ``alias.*`` expands one side; an uncorrelated subquery inside
an expression (``x IN (SELECT ...)``, ``(SELECT MAX(y) FROM t)``) is evaluated first and inlined as literals.
Joins hash on the equality conjuncts of ``ON``.  Registered tables that are partitioned over ranks are
gathered first, so every rank computes the same result (the operator API — JoinBatchOp, GroupByBatchOp, ... —
is the distributed path: hash/range shuffles in ``operator/batch/sql.py``).
"""
from __future__ import annotations

import re
from collections import OrderedDict
from typing import Any, Callable, Dict, List, Optional, Tuple

from ....common.table import MTable, Row
from ....common.types import TableSchema
from .engine import _key, _names_for, _out_type, _resolver, _split_and, sql_distinct, sql_intersect, sql_minus, \
    sql_union
from .expr import _TOKEN, Expr, SelectItem, compile_expr, parse_expr, parse_select_list, split_top_level

__all__ = ["execute_query", "parse_query"]

_CLAUSE_END = {"FROM", "WHERE", "GROUP", "HAVING", "ORDER", "LIMIT", "OFFSET", "UNION", "INTERSECT", "EXCEPT",
               "MINUS", "JOIN", "INNER", "LEFT", "RIGHT", "FULL", "CROSS", "ON"}
_SETOPS = {"UNION", "INTERSECT", "EXCEPT", "MINUS"}


class _Tok:
    __slots__ = ("kind", "val", "up", "start", "end")

    def __init__(self, kind, val, start, end):
        self.kind, self.val, self.start, self.end = kind, val, start, end
        self.up = val.upper() if kind == "id" else val


def _lex(text: str) -> List[_Tok]:
    out, pos = [], 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise ValueError(f"SQL syntax error near: {text[pos:pos + 20]!r}")
        kind = m.lastgroup
        if kind != "ws":
            val = m.group(kind)
            if kind in ("bq", "dq"):
                kind, val = "qid", val[1:-1]
            out.append(_Tok(kind, val, m.start(), m.end()))
        pos = m.end()
    return out


# ------------------------------------------------------------------------------------------------ AST
class FromItem:
    def __init__(self, table: Optional[str], sub: Optional["Query"], alias: Optional[str]):
        self.table, self.sub, self.alias = table, sub, alias


class Core:
    def __init__(self):
        self.distinct = False
        self.items = ""
        self.sources: List[FromItem] = []
        self.joins: List[Tuple[str, str]] = []      # (how, on-text) for sources[1:]
        self.where = self.group = self.having = None


class SetOp:
    def __init__(self, op: str, all_: bool, left, right):
        self.op, self.all, self.left, self.right = op, all_, left, right


class Query:
    def __init__(self, body, order: Optional[str], limit: Optional[int], offset: Optional[int]):
        self.body, self.order, self.limit, self.offset = body, order, limit, offset


class _P:
    def __init__(self, text: str):
        self.text = text
        self.t = _lex(text)
        self.i = 0

    def peek(self, k=0) -> Optional[_Tok]:
        j = self.i + k
        return self.t[j] if j < len(self.t) else None

    def kw(self, *words) -> bool:
        tk = self.peek()
        return tk is not None and tk.kind == "id" and tk.up in words

    def take_kw(self, *words) -> bool:
        if self.kw(*words):
            self.i += 1
            return True
        return False

    def expect_kw(self, word):
        if not self.take_kw(word):
            tk = self.peek()
            raise ValueError(f"SQL: expected {word} near {tk.val if tk else 'end of query'!r}")

    def op(self, v) -> bool:
        tk = self.peek()
        return tk is not None and tk.kind == "op" and tk.val == v

    def span_until(self, stops, allow_comma=True) -> str:
        """Source text from here to the next top-level stop keyword / ')' / (optionally) ','."""
        depth, j = 0, self.i
        while j < len(self.t):
            tk = self.t[j]
            if tk.kind == "op" and tk.val == "(":
                depth += 1
            elif tk.kind == "op" and tk.val == ")":
                if depth == 0:
                    break
                depth -= 1
            elif depth == 0 and tk.kind == "id" and tk.up in stops:
                break
            elif depth == 0 and not allow_comma and tk.kind == "op" and tk.val == ",":
                break
            j += 1
        if j == self.i:
            raise ValueError("SQL: empty clause near " + (self.t[j].val if j < len(self.t) else "end"))
        s = self.text[self.t[self.i].start:self.t[j - 1].end]
        self.i = j
        return s

    # query := body [ORDER BY] [LIMIT] [OFFSET]
    def query(self) -> Query:
        body = self.setexpr()
        order = limit = offset = None
        if self.take_kw("ORDER"):
            self.expect_kw("BY")
            order = self.span_until(_CLAUSE_END)
        if self.take_kw("LIMIT"):
            limit = int(self.t[self.i].val)
            self.i += 1
        if self.take_kw("OFFSET"):
            offset = int(self.t[self.i].val)
            self.i += 1
            self.take_kw("ROWS", "ROW")
        if self.take_kw("FETCH"):
            self.take_kw("FIRST", "NEXT")
            limit = int(self.t[self.i].val)
            self.i += 1
            self.take_kw("ROWS", "ROW")
            self.take_kw("ONLY")
        return Query(body, order, limit, offset)

    def setexpr(self):
        left = self.core()
        while self.kw(*_SETOPS):
            op = self.t[self.i].up
            self.i += 1
            all_ = self.take_kw("ALL")
            self.take_kw("DISTINCT")
            left = SetOp("MINUS" if op == "EXCEPT" else op, all_, left, self.core())
        return left

    def core(self):
        if self.op("("):
            self.i += 1
            q = self.query()
            self._close()
            return q
        self.expect_kw("SELECT")
        c = Core()
        c.distinct = self.take_kw("DISTINCT")
        self.take_kw("ALL")
        c.items = self.span_until({"FROM"})
        self.expect_kw("FROM")
        c.sources.append(self.from_item())
        while True:
            if self.op(","):
                self.i += 1
                c.sources.append(self.from_item())
                c.joins.append(("cross", None))
                continue
            how = None
            if self.take_kw("JOIN"):
                how = "inner"
            elif self.kw("INNER", "CROSS", "LEFT", "RIGHT", "FULL"):
                w = self.t[self.i].up
                self.i += 1
                self.take_kw("OUTER")
                self.expect_kw("JOIN")
                how = {"INNER": "inner", "CROSS": "cross", "LEFT": "left", "RIGHT": "right", "FULL": "full"}[w]
            if how is None:
                break
            c.sources.append(self.from_item())
            on = None
            if self.take_kw("ON"):
                on = self.span_until(_CLAUSE_END)
            elif how != "cross":
                raise ValueError("SQL: JOIN needs an ON condition")
            c.joins.append((how, on))
        if self.take_kw("WHERE"):
            c.where = self.span_until(_CLAUSE_END)
        if self.take_kw("GROUP"):
            self.expect_kw("BY")
            c.group = self.span_until(_CLAUSE_END)
        if self.take_kw("HAVING"):
            c.having = self.span_until(_CLAUSE_END)
        return c

    def _close(self):
        if not self.op(")"):
            raise ValueError("SQL: missing ')'")
        self.i += 1

    def from_item(self) -> FromItem:
        if self.op("("):
            self.i += 1
            q = self.query()
            self._close()
            self.take_kw("AS")
            alias = self._alias()
            return FromItem(None, q, alias)
        tk = self.peek()
        if tk is None or tk.kind not in ("id", "qid"):
            raise ValueError("SQL: expected a table name")
        self.i += 1
        self.take_kw("AS")
        return FromItem(tk.val, None, self._alias() or tk.val)

    def _alias(self) -> Optional[str]:
        tk = self.peek()
        if tk is not None and (tk.kind == "qid" or (tk.kind == "id" and tk.up not in _CLAUSE_END | {"WHERE"})):
            self.i += 1
            return tk.val
        return None


def parse_query(text: str) -> Query:
    p = _P(text.strip().rstrip(";"))
    q = p.query()
    if p.peek() is not None:
        raise ValueError(f"SQL: unexpected {p.peek().val!r} in {text!r}")
    return q


# ------------------------------------------------------------------------------------------------ execution
class _Rel:
    """Rows + column names + qualifier map ``alias -> (offset, names)``."""

    def __init__(self, rows: List[tuple], schema: TableSchema, qual: Dict[str, Tuple[int, List[str]]]):
        self.rows, self.schema, self.qual = rows, schema, qual

    def resolver(self):
        return _resolver(self.schema.names, self.qual)


def _literal(v) -> str:
    if v is None:
        return "NULL"
    if isinstance(v, bool):
        return "TRUE" if v else "FALSE"
    if isinstance(v, (int, float)):
        return repr(v)
    return "'" + str(v).replace("'", "''") + "'"


_SUB = re.compile(r"\(\s*select\b", re.I)


def _inline_subqueries(text: str, run: Callable[[str], MTable]) -> str:
    """Replace every ``(SELECT ...)`` inside an expression by the literal list of its (single-column) result."""
    while True:
        m = _SUB.search(text)
        if not m:
            return text
        depth, j, q = 0, m.start(), None
        while j < len(text):
            ch = text[j]
            if q:
                if ch == q:
                    q = None
            elif ch in "'`\"":
                q = ch
            elif ch == "(":
                depth += 1
            elif ch == ")":
                depth -= 1
                if depth == 0:
                    break
            j += 1
        inner = text[m.start() + 1:j]
        res = run(inner)
        if len(res.schema.names) != 1:
            raise ValueError("SQL: a subquery used as a value must return one column")
        vals = [r[0] for r in res.rows()]
        text = text[:m.start()] + "(" + (", ".join(_literal(v) for v in vals) if vals else "NULL") + ")" + text[j + 1:]


class Executor:
    def __init__(self, tables: Dict[str, MTable]):
        self.tables = tables

    def run_text(self, text: str) -> MTable:
        return self.run(parse_query(text))

    def run(self, q) -> MTable:
        if isinstance(q, Query):
            if isinstance(q.body, Core) and q.order:
                mt = self._core(q.body, q.order)       # keys may name source columns that are not selected
            else:
                mt = self.run(q.body)
                if q.order:
                    mt = self._order(mt, q.order)
            if q.offset:
                mt = mt.take(list(range(min(q.offset, mt.num_rows), mt.num_rows)))
            if q.limit is not None:
                mt = mt.take(list(range(min(q.limit, mt.num_rows))))
            return mt
        if isinstance(q, SetOp):
            a, b = self.run(q.left), self.run(q.right)
            if len(a.schema.names) != len(b.schema.names):
                raise ValueError("SQL: set operation inputs have different column counts")
            fn = {"UNION": sql_union, "INTERSECT": sql_intersect, "MINUS": sql_minus}[q.op]
            return fn(a, b, q.all)
        return self._core(q)

    def _expr(self, text: str) -> Expr:
        return parse_expr(_inline_subqueries(text, self.run_text))

    def _source(self, fi: FromItem) -> _Rel:
        if fi.sub is not None:
            mt = self.run(fi.sub)
        else:
            key = fi.table if fi.table in self.tables else \
                next((k for k in self.tables if k.lower() == fi.table.lower()), None)
            if key is None:
                raise ValueError(f"SQL: table {fi.table!r} is not registered (registerTableName)")
            mt = self.tables[key]
        names = list(mt.schema.names)
        qual = {fi.alias: (0, names)} if fi.alias else {}
        return _Rel([tuple(r) for r in mt.rows()], mt.schema, qual)

    def _join(self, left: _Rel, right: _Rel, how: str, on: Optional[str]) -> _Rel:
        nl = len(left.schema.names)
        names = list(left.schema.names) + list(right.schema.names)
        schema = TableSchema(names, list(left.schema.types) + list(right.schema.types))
        qual = dict(left.qual)
        for a, (off, sub) in right.qual.items():
            qual[a] = (off + nl, sub)
        rel = _Rel([], schema, qual)
        resolve = rel.resolver()
        pred = self._expr(on) if on else None
        pf = compile_expr(pred, resolve) if pred is not None else (lambda r, g=None: True)
        eq_l, eq_r = [], []
        if pred is not None:
            for c in _split_and(pred):
                if c.kind == "cmp" and c.args[0] == "=" and c.args[1].kind == "col" and c.args[2].kind == "col":
                    i, j = resolve(c.args[1].args[0]), resolve(c.args[2].args[0])
                    if i < nl <= j:
                        eq_l.append(i)
                        eq_r.append(j - nl)
                    elif j < nl <= i:
                        eq_l.append(j)
                        eq_r.append(i - nl)
        rrows = right.rows
        null_l, null_r = (None,) * nl, (None,) * len(right.schema.names)
        matched = [False] * len(rrows)
        index = None
        if eq_l:
            index = {}
            for j, r in enumerate(rrows):
                k = tuple(_key(r[x]) for x in eq_r)
                if None not in k:
                    index.setdefault(k, []).append(j)
        out = []
        for l in left.rows:
            cands = index.get(tuple(_key(l[x]) for x in eq_l), ()) if index is not None else range(len(rrows))
            hit = False
            for j in cands:
                row = l + rrows[j]
                if pf(row) is True:
                    out.append(row)
                    matched[j] = hit = True
            if not hit and how in ("left", "full"):
                out.append(l + null_r)
        if how in ("right", "full"):
            out.extend(null_l + r for j, r in enumerate(rrows) if not matched[j])
        rel.rows = out
        return rel

    def _items(self, text: str, rel: _Rel) -> List[SelectItem]:
        items = []
        for part in split_top_level(text):
            m = re.match(r"^\s*`?(\w+)`?\s*\.\s*\*\s*$", part)
            if m and m.group(1) in rel.qual:
                off, sub = rel.qual[m.group(1)]
                items.extend(SelectItem(Expr("col", f"{m.group(1)}.{c}"), c, c) for c in sub)
            elif part.strip() == "*":
                items.extend(SelectItem(Expr("col", f"#{i}"), n, n) for i, n in enumerate(rel.schema.names))
            else:
                items.extend(parse_select_list(_inline_subqueries(part, self.run_text)))
        return items

    def _core(self, c: Core, order: Optional[str] = None) -> MTable:
        rel = self._source(c.sources[0])
        for fi, (how, on) in zip(c.sources[1:], c.joins):
            rel = self._join(rel, self._source(fi), how, on)
        base = rel.resolver()

        def resolve(n: str) -> int:
            return int(n[1:]) if n.startswith("#") and n[1:].isdigit() else base(n)
        if c.where:
            f = compile_expr(self._expr(c.where), resolve)
            rel.rows = [r for r in rel.rows if f(r) is True]
        items = self._items(c.items, rel)
        fns = [compile_expr(it.expr, resolve) for it in items]
        grouped = c.group is not None or c.having is not None or any(it.expr.has_agg() for it in items)
        if grouped:
            groups: "OrderedDict[tuple, List[tuple]]" = OrderedDict()
            if c.group:
                kfs = [compile_expr(self._expr(p), resolve) for p in split_top_level(c.group)]
                for r in rel.rows:
                    groups.setdefault(tuple(_key(f(r)) for f in kfs), []).append(r)
            else:
                groups[()] = rel.rows        # global aggregate: one row even over no input
            hf = compile_expr(self._expr(c.having), resolve) if c.having else None
            out, ctx = [], []
            for g in groups.values():
                first = g[0] if g else (None,) * len(rel.schema.names)
                if hf is not None and hf(first, g) is not True:
                    continue
                out.append(Row(tuple(f(first, g) for f in fns)))
                ctx.append((first, g))
        else:
            out = [Row(tuple(f(r) for f in fns)) for r in rel.rows]
            ctx = [(r, None) for r in rel.rows]
        names = _names_for(items)
        if order:
            out = self._sort_core(out, ctx, names, order, resolve)
        types = [_out_type(it.expr, rel.schema, [o[j] for o in out[:100]], resolve) for j, it in enumerate(items)]
        mt = MTable.from_rows(out, TableSchema(names, types))
        return sql_distinct(mt) if c.distinct else mt

    def _sort_core(self, out, ctx, names, clause, resolve):
        """ORDER BY of a single SELECT: ordinals and output aliases read the result row, anything else is
        evaluated on the source row (or group) that produced it."""
        lower = [n.lower() for n in names]
        keys = []
        for part in split_top_level(clause):
            toks = part.split()
            asc = True
            if len(toks) > 1 and toks[-1].lower() in ("asc", "desc"):
                asc = toks[-1].lower() == "asc"
                part = " ".join(toks[:-1])
            t = part.strip().strip("`")
            if t.isdigit():
                keys.append(([o[int(t) - 1] for o in out], asc))
            elif "." not in t and t.lower() in lower and lower.count(t.lower()) == 1:
                j = lower.index(t.lower())
                keys.append(([o[j] for o in out], asc))
            else:
                f = compile_expr(self._expr(part), resolve)
                keys.append(([f(r, g) for r, g in ctx], asc))
        idx = list(range(len(out)))
        for vals, asc in reversed(keys):
            idx.sort(key=lambda i: (vals[i] is not None, vals[i] if vals[i] is not None else 0), reverse=not asc)
        return [out[i] for i in idx]

    def _order(self, mt: MTable, clause: str) -> MTable:
        resolve = _resolver(mt.schema.names)
        rows = mt.rows()
        idx = list(range(len(rows)))
        keys = []
        for part in split_top_level(clause):
            toks = part.split()
            asc = True
            if len(toks) > 1 and toks[-1].lower() in ("asc", "desc"):
                asc = toks[-1].lower() == "asc"
                part = " ".join(toks[:-1])
            if part.strip().isdigit():          # ORDER BY <ordinal>
                pos = int(part) - 1
                keys.append(((lambda p: lambda r, g=None: r[p])(pos), asc))
            else:
                keys.append((compile_expr(self._expr(part), resolve), asc))
        for f, asc in reversed(keys):
            vals = [f(r) for r in rows]
            # NULLs first ascending, last descending (Flink)
            idx.sort(key=lambda i: (vals[i] is not None, vals[i] if vals[i] is not None else 0), reverse=not asc)
        return mt.take(idx)


def execute_query(text: str, tables: Dict[str, MTable]) -> MTable:
    return Executor(tables).run_text(text)
