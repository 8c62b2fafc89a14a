"""Columnar (vectorised) evaluation of SQL expressions over tensor columns.

The row evaluator (``expr.compile_expr``) walks one Python ``Row`` at a time; for the common projection and
filter shapes -- arithmetic, comparisons, three-valued AND/OR/NOT, IS [NOT] NULL, BETWEEN, IN over literals,
CASE WHEN, casts and elementwise math functions over numeric / boolean columns -- ``evaluate`` evaluates
the whole column at once with torch ops, on the device where the columns live (a GPU-resident table is
filtered and projected without leaving HBM).  Values follow the row evaluator's semantics: integers stay int64
(SQL integer division truncates toward zero and yields NULL on a zero divisor, ``%`` is ``fmod``), anything
touching a float is fp64, comparisons / logic produce booleans, NULL propagates through a mask.  Any other node
(strings, vectors, aggregates, UDFs, ...) raises ``Unsupported`` and the caller falls back to the row path.

Reference: ``A/operator/common/sql/BatchSqlOperators.java:51-388`` (Flink SQL evaluates these as generated code
over rows).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch

from ....common.table import MTable
from .expr import Expr

__all__ = ["Unsupported", "evaluate", "try_evaluate"]


class Unsupported(Exception):
    pass


V = Tuple[torch.Tensor, Optional[torch.Tensor]]          # values, null mask (None = no NULLs)


def _or_null(a: Optional[torch.Tensor], b: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if a is None:
        return b
    if b is None:
        return a
    return a | b


def _norm(t: torch.Tensor) -> torch.Tensor:
    if t.dtype == torch.bool:
        return t
    if t.dtype.is_floating_point:
        return t.to(torch.float64)
    return t.to(torch.int64)


def _is_int(t: torch.Tensor) -> bool:
    return not t.dtype.is_floating_point and t.dtype != torch.bool


def _lit(v, n: int, dev) -> V:
    if isinstance(v, bool):
        return torch.full((n,), v, dtype=torch.bool, device=dev), None
    if isinstance(v, int):
        return torch.full((n,), v, dtype=torch.int64, device=dev), None
    if isinstance(v, float):
        return torch.full((n,), v, dtype=torch.float64, device=dev), None
    if v is None:
        return torch.zeros(n, dtype=torch.int64, device=dev), torch.ones(n, dtype=torch.bool, device=dev)
    raise Unsupported(f"literal {v!r}")


def _num(x: V) -> V:
    if x[0].dtype == torch.bool:
        raise Unsupported("arithmetic on booleans")
    return x


def _arith(op: str, a: V, b: V) -> V:
    a, b = _num(a), _num(b)
    x, y = a[0], b[0]
    nulls = _or_null(a[1], b[1])
    ints = _is_int(x) and _is_int(y)
    if not ints:
        x, y = x.to(torch.float64), y.to(torch.float64)
    if op == "+":
        return x + y, nulls
    if op == "-":
        return x - y, nulls
    if op == "*":
        return x * y, nulls
    if op == "/":
        if ints:
            zero = y == 0
            q = torch.div(x, torch.where(zero, torch.ones_like(y), y), rounding_mode="trunc")
            return q, _or_null(nulls, zero)
        # a / 0: +-inf for a != 0, NaN for 0 (the row evaluator's rule; IEEE gives the same)
        return x / y, nulls
    if op == "%":
        if ints:
            zero = y == 0
            r = torch.fmod(x, torch.where(zero, torch.ones_like(y), y))
            if bool(zero.any()):
                raise Unsupported("integer modulo by zero")      # the row path raises; keep its behaviour
            return r, nulls
        return torch.fmod(x, y), nulls
    raise Unsupported(op)


def _compare(op: str, a: V, b: V) -> V:
    x, y = a[0], b[0]
    if (x.dtype == torch.bool) != (y.dtype == torch.bool):
        raise Unsupported("bool vs number comparison")
    if x.dtype != y.dtype and x.dtype != torch.bool:
        x, y = x.to(torch.float64), y.to(torch.float64)
    nulls = _or_null(a[1], b[1])
    f = {"=": torch.eq, "<>": torch.ne, "!=": torch.ne, "<": torch.lt, "<=": torch.le, ">": torch.gt,
         ">=": torch.ge}.get(op)
    if f is None:
        raise Unsupported(op)
    return f(x, y), nulls


def _bool(x: V) -> V:
    if x[0].dtype != torch.bool:
        raise Unsupported("non-boolean in logic")
    return x


def _and(a: V, b: V) -> V:
    a, b = _bool(a), _bool(b)
    an = a[1] if a[1] is not None else torch.zeros_like(a[0])
    bn = b[1] if b[1] is not None else torch.zeros_like(b[0])
    af = ~a[0] & ~an            # definitely false
    bf = ~b[0] & ~bn
    false = af | bf
    null = ~false & (an | bn)
    return ~false & ~null, (null if bool(null.any()) else None)


def _or(a: V, b: V) -> V:
    a, b = _bool(a), _bool(b)
    an = a[1] if a[1] is not None else torch.zeros_like(a[0])
    bn = b[1] if b[1] is not None else torch.zeros_like(b[0])
    true = (a[0] & ~an) | (b[0] & ~bn)
    null = ~true & (an | bn)
    return true, (null if bool(null.any()) else None)


_FN: dict = {
    "ABS": lambda x: torch.abs(x),
    "SQRT": lambda x: torch.sqrt(x.to(torch.float64)),
    "EXP": lambda x: torch.exp(x.to(torch.float64)),
    "LN": lambda x: torch.log(x.to(torch.float64)),
    "LOG10": lambda x: torch.log10(x.to(torch.float64)),
    "LOG2": lambda x: torch.log2(x.to(torch.float64)),
    "SIN": lambda x: torch.sin(x.to(torch.float64)),
    "COS": lambda x: torch.cos(x.to(torch.float64)),
    "TAN": lambda x: torch.tan(x.to(torch.float64)),
    "FLOOR": lambda x: torch.floor(x).to(torch.int64) if x.dtype.is_floating_point else x,
    "CEIL": lambda x: torch.ceil(x).to(torch.int64) if x.dtype.is_floating_point else x,
    "CEILING": lambda x: torch.ceil(x).to(torch.int64) if x.dtype.is_floating_point else x,
    "SIGN": lambda x: torch.sign(x).to(torch.int64),
}


def _cast(x: V, t: str) -> V:
    t = t.upper()
    v = x[0]
    if t in ("DOUBLE", "FLOAT", "REAL", "DECIMAL"):
        return v.to(torch.float64), x[1]
    if t in ("INT", "INTEGER", "BIGINT", "LONG", "SMALLINT", "TINYINT"):
        return (torch.trunc(v).to(torch.int64) if v.dtype.is_floating_point else v.to(torch.int64)), x[1]
    if t == "BOOLEAN":
        return v != 0 if v.dtype != torch.bool else v, x[1]
    raise Unsupported(f"cast to {t}")


def evaluate(e: Expr, mt: MTable, resolve: Callable[[str], int]) -> V:
    """(values, null mask) of ``e`` over every row of ``mt``; raises ``Unsupported`` for non-columnar nodes."""
    n = mt.num_rows
    dev = next((c.values.device for c in mt.cols if isinstance(c.values, torch.Tensor)), torch.device("cpu"))

    def ev(x: Expr) -> V:
        k = x.kind
        if k == "lit":
            return _lit(x.args[0], n, dev)
        if k == "col":
            c = mt.cols[resolve(x.args[0])]
            if not isinstance(c.values, torch.Tensor) or c.values.dim() != 1:
                raise Unsupported("non-tensor column")
            return _norm(c.values.to(dev)), (c.nulls.to(dev) if c.nulls is not None else None)
        if k == "neg":
            a = _num(ev(x.args[0]))
            return -a[0], a[1]
        if k == "bin":
            return _arith(x.args[0], ev(x.args[1]), ev(x.args[2]))
        if k == "cmp":
            return _compare(x.args[0], ev(x.args[1]), ev(x.args[2]))
        if k == "and":
            return _and(ev(x.args[0]), ev(x.args[1]))
        if k == "or":
            return _or(ev(x.args[0]), ev(x.args[1]))
        if k == "not":
            a = _bool(ev(x.args[0]))
            return ~a[0], a[1]
        if k == "isnull":
            a = ev(x.args[0])
            isn = a[1] if a[1] is not None else torch.zeros(n, dtype=torch.bool, device=dev)
            return (isn != x.args[1]), None
        if k == "between":
            a, lo, hi = (ev(y) for y in x.args[:3])
            inside = _compare(">=", a, lo)[0] & _compare("<=", a, hi)[0]
            return (inside != x.args[3]), _or_null(_or_null(a[1], lo[1]), hi[1])
        if k == "in":
            a = ev(x.args[0])
            if any(y.kind != "lit" or y.args[0] is None for y in x.args[1]):
                raise Unsupported("IN over non-literals")
            hit = torch.zeros(n, dtype=torch.bool, device=dev)
            for y in x.args[1]:
                hit |= _compare("=", a, _lit(y.args[0], n, dev))[0]
            return (hit != x.args[2]), a[1]
        if k == "case":
            if x.args[0] is not None:
                raise Unsupported("simple CASE")
            out = ev(x.args[2])
            for c, v in reversed(x.args[1]):
                cv, cn = _bool(ev(c))
                take = cv & (~cn if cn is not None else torch.ones_like(cv))
                vv = ev(v)
                if vv[0].dtype != out[0].dtype:
                    if vv[0].dtype == torch.bool or out[0].dtype == torch.bool:
                        raise Unsupported("mixed CASE types")
                    vv, out = (vv[0].to(torch.float64), vv[1]), (out[0].to(torch.float64), out[1])
                vals = torch.where(take, vv[0], out[0])
                on = out[1] if out[1] is not None else torch.zeros(n, dtype=torch.bool, device=dev)
                vn = vv[1] if vv[1] is not None else torch.zeros(n, dtype=torch.bool, device=dev)
                nulls = torch.where(take, vn, on)
                out = (vals, nulls if bool(nulls.any()) else None)
            return out
        if k == "cast":
            return _cast(ev(x.args[0]), x.args[1])
        if k == "fn":
            f = _FN.get(x.args[0])
            if f is None or len(x.args[1]) != 1:
                raise Unsupported(f"function {x.args[0]}")
            a = _num(ev(x.args[1][0]))
            return f(a[0]), a[1]
        raise Unsupported(k)

    return ev(e)


def try_evaluate(e: Expr, mt: MTable, resolve) -> Optional[V]:
    try:
        return evaluate(e, mt, resolve)
    except Unsupported:
        return None
