"""A small SQL expression engine for the SQL-sugar operators.

The reference implements ``select/where/groupBy/join/...`` by registering a temp table and running Flink SQL
(``A/operator/common/sql/BatchSqlOperators.java:51-388``) plus scalar UDFs
(``A/operator/common/sql/functions/{MathFunctions,StringFunctions}.java``).  Here expressions are parsed
once (recursive descent) and compiled to Python closures evaluated per row with SQL three-valued NULL
semantics.  Supported: arithmetic, ``||``, comparisons, AND/OR/NOT, IS [NOT] NULL, [NOT] LIKE,
[NOT] IN, [NOT] BETWEEN, CASE WHEN, CAST(x AS t), scalar functions, and the aggregates COUNT/SUM/AVG/MIN/MAX/
VAR_SAMP/VAR_POP/STDDEV_SAMP/STDDEV_POP (optionally DISTINCT) for GROUP BY.
"""
from __future__ import annotations

import math
import re
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

__all__ = ["parse_expr", "split_top_level", "compile_expr", "SelectItem", "parse_select_list", "Expr",
           "AGGREGATES"]

_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<num>\d+\.\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|\d+(?:[eE][-+]?\d+)?)
  | (?P<str>'(?:[^']|'')*')
  | (?P<bq>`[^`]+`)
  | (?P<dq>"[^"]+")
  | (?P<op><>|!=|<=|>=|\|\||[-+*/%=<>(),.])
  | (?P<id>[A-Za-z_][A-Za-z_0-9]*)
""", re.X)

KEYWORDS = {"AND", "OR", "NOT", "IS", "NULL", "LIKE", "IN", "BETWEEN", "CASE", "WHEN", "THEN", "ELSE", "END",
            "CAST", "AS", "TRUE", "FALSE", "DISTINCT"}
AGGREGATES = {"COUNT", "SUM", "AVG", "MIN", "MAX", "VAR_SAMP", "VAR_POP", "STDDEV_SAMP", "STDDEV_POP", "STDDEV",
              "VARIANCE"}


def tokenize(s: str) -> List[Tuple[str, str]]:
    out = []
    pos = 0
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise ValueError(f"SQL syntax error near: {s[pos:pos + 20]!r}")
        pos = m.end()
        kind = m.lastgroup
        val = m.group(kind)
        if kind == "ws":
            continue
        if kind == "bq":
            out.append(("id", val[1:-1]))
        elif kind == "dq":
            out.append(("id", val[1:-1]))
        elif kind == "id" and val.upper() in KEYWORDS:
            out.append(("kw", val.upper()))
        else:
            out.append((kind, val))
    return out


def split_top_level(s: str, sep: str = ",") -> List[str]:
    parts, depth, cur, q = [], 0, [], None
    for ch in s:
        if q:
            cur.append(ch)
            if ch == q:
                q = None
            continue
        if ch in ("'", "`", '"'):
            q = ch
        elif ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == sep and depth == 0:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    if cur or parts:
        parts.append("".join(cur))
    return [p.strip() for p in parts]


class Expr:
    """AST node: (kind, payload...)."""
    __slots__ = ("kind", "args")

    def __init__(self, kind, *args):
        self.kind, self.args = kind, args

    def __repr__(self):
        return f"{self.kind}{self.args}"

    def columns(self) -> List[str]:
        out = []
        if self.kind == "col":
            out.append(self.args[0])
        for a in self.args:
            if isinstance(a, Expr):
                out.extend(a.columns())
            elif isinstance(a, (list, tuple)):
                for x in a:
                    if isinstance(x, Expr):
                        out.extend(x.columns())
                    elif isinstance(x, tuple):
                        for y in x:
                            if isinstance(y, Expr):
                                out.extend(y.columns())
        return out

    def has_agg(self) -> bool:
        if self.kind == "agg":
            return True
        for a in self.args:
            if isinstance(a, Expr) and a.has_agg():
                return True
            if isinstance(a, (list, tuple)):
                for x in a:
                    if isinstance(x, Expr) and x.has_agg():
                        return True
                    if isinstance(x, tuple) and any(isinstance(y, Expr) and y.has_agg() for y in x):
                        return True
        return False


class _Parser:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else ("eof", None)

    def take(self):
        tok = self.peek()
        self.i += 1
        return tok

    def accept(self, kind, val=None):
        k, v = self.peek()
        if k == kind and (val is None or v == val):
            self.i += 1
            return True
        return False

    def expect(self, kind, val=None):
        if not self.accept(kind, val):
            raise ValueError(f"SQL: expected {val or kind}, got {self.peek()}")

    def parse(self):
        e = self.expr()
        return e

    def expr(self):
        return self.or_()

    def or_(self):
        e = self.and_()
        while self.accept("kw", "OR"):
            e = Expr("or", e, self.and_())
        return e

    def and_(self):
        e = self.not_()
        while self.accept("kw", "AND"):
            e = Expr("and", e, self.not_())
        return e

    def not_(self):
        if self.accept("kw", "NOT"):
            return Expr("not", self.not_())
        return self.cmp()

    def cmp(self):
        e = self.add()
        k, v = self.peek()
        if k == "op" and v in ("=", "<>", "!=", "<", "<=", ">", ">="):
            self.take()
            return Expr("cmp", v, e, self.add())
        if self.accept("kw", "IS"):
            neg = self.accept("kw", "NOT")
            self.expect("kw", "NULL")
            return Expr("isnull", e, neg)
        neg = False
        if self.peek() == ("kw", "NOT") and self.peek(1)[1] in ("LIKE", "IN", "BETWEEN"):
            self.take()
            neg = True
        if self.accept("kw", "LIKE"):
            return Expr("like", e, self.add(), neg)
        if self.accept("kw", "IN"):
            self.expect("op", "(")
            items = [self.expr()]
            while self.accept("op", ","):
                items.append(self.expr())
            self.expect("op", ")")
            return Expr("in", e, items, neg)
        if self.accept("kw", "BETWEEN"):
            lo = self.add()
            self.expect("kw", "AND")
            hi = self.add()
            return Expr("between", e, lo, hi, neg)
        return e

    def add(self):
        e = self.mul()
        while True:
            k, v = self.peek()
            if k == "op" and v in ("+", "-", "||"):
                self.take()
                e = Expr("bin", v, e, self.mul())
            else:
                return e

    def mul(self):
        e = self.unary()
        while True:
            k, v = self.peek()
            if k == "op" and v in ("*", "/", "%"):
                self.take()
                e = Expr("bin", v, e, self.unary())
            else:
                return e

    def unary(self):
        if self.accept("op", "-"):
            return Expr("neg", self.unary())
        if self.accept("op", "+"):
            return self.unary()
        return self.primary()

    def primary(self):
        k, v = self.take()
        if k == "num":
            return Expr("lit", float(v) if any(c in v for c in ".eE") else int(v))
        if k == "str":
            return Expr("lit", v[1:-1].replace("''", "'"))
        if k == "kw":
            if v == "NULL":
                return Expr("lit", None)
            if v == "TRUE":
                return Expr("lit", True)
            if v == "FALSE":
                return Expr("lit", False)
            if v == "CASE":
                return self.case()
            if v == "CAST":
                self.expect("op", "(")
                e = self.expr()
                self.expect("kw", "AS")
                _, t = self.take()
                while self.accept("op", "("):
                    while not self.accept("op", ")"):
                        self.take()
                self.expect("op", ")")
                return Expr("cast", e, t.upper())
        if k == "op" and v == "(":
            e = self.expr()
            self.expect("op", ")")
            return e
        if k == "op" and v == "*":
            return Expr("star")
        if k == "id":
            if self.accept("op", "("):
                name = v.upper()
                distinct = self.accept("kw", "DISTINCT")
                args = []
                if not self.accept("op", ")"):
                    if self.peek() == ("op", "*"):
                        self.take()
                        args.append(Expr("star"))
                    else:
                        args.append(self.expr())
                    while self.accept("op", ","):
                        args.append(self.expr())
                    self.expect("op", ")")
                if name in AGGREGATES:
                    return Expr("agg", name, args, distinct)
                return Expr("fn", name, args)
            name = v
            while self.accept("op", "."):  # qualified t.col -> keep last + qualifier
                _, v2 = self.take()
                name = name + "." + v2
            return Expr("col", name)
        raise ValueError(f"SQL: unexpected token {v!r}")

    def case(self):
        operand = None
        if self.peek() != ("kw", "WHEN"):
            operand = self.expr()
        whens = []
        while self.accept("kw", "WHEN"):
            c = self.expr()
            self.expect("kw", "THEN")
            whens.append((c, self.expr()))
        els = Expr("lit", None)
        if self.accept("kw", "ELSE"):
            els = self.expr()
        self.expect("kw", "END")
        return Expr("case", operand, whens, els)


def parse_expr(s: str) -> Expr:
    p = _Parser(tokenize(s))
    e = p.parse()
    if p.peek()[0] != "eof":
        raise ValueError(f"SQL: trailing tokens in {s!r}: {p.t[p.i:]}")
    return e


class SelectItem:
    def __init__(self, expr: Expr, alias: Optional[str], text: str):
        self.expr, self.alias, self.text = expr, alias, text


def parse_select_list(s: str) -> List[SelectItem]:
    items = []
    for part in split_top_level(s):
        toks = tokenize(part)
        alias = None
        # trailing "AS alias" or "expr alias"
        if len(toks) >= 3 and toks[-2] == ("kw", "AS") and toks[-1][0] == "id":
            alias = toks[-1][1]
            toks = toks[:-2]
        elif len(toks) >= 2 and toks[-1][0] == "id" and toks[-2][0] in ("id", "op", "num", "str") \
                and not (toks[-2] == ("op", ".")) and toks[-2] != ("op", "("):
            if toks[-2][0] == "op" and toks[-2][1] in (")",):
                alias = toks[-1][1]
                toks = toks[:-1]
            elif toks[-2][0] in ("id", "num", "str"):
                alias = toks[-1][1]
                toks = toks[:-1]
        p = _Parser(toks)
        e = p.parse()
        items.append(SelectItem(e, alias, part))
    return items


# ---------------------------------------------------------------------------------------------------
# evaluation
# ---------------------------------------------------------------------------------------------------
def _like_to_regex(pat: str):
    out = []
    for ch in pat:
        if ch == "%":
            out.append(".*")
        elif ch == "_":
            out.append(".")
        else:
            out.append(re.escape(ch))
    return re.compile("^" + "".join(out) + "$", re.S)


def _num(a):
    return a


def _arith(op, a, b):
    if a is None or b is None:
        return None
    if op == "+":
        if isinstance(a, str) or isinstance(b, str):
            return str(a) + str(b)
        return a + b
    if op == "-":
        return a - b
    if op == "*":
        return a * b
    if op == "/":
        if isinstance(a, int) and isinstance(b, int) and not isinstance(a, bool):
            if b == 0:
                return None
            q = abs(a) // abs(b)
            return q if (a >= 0) == (b >= 0) else -q
        return a / b if b != 0 else (math.copysign(math.inf, a) if a != 0 else math.nan)
    if op == "%":
        return math.fmod(a, b) if isinstance(a, float) or isinstance(b, float) else int(math.fmod(a, b))
    if op == "||":
        return str(a) + str(b)
    raise ValueError(op)


def _compare(op, a, b):
    if a is None or b is None:
        return None
    if op == "=":
        return a == b
    if op in ("<>", "!="):
        return a != b
    if op == "<":
        return a < b
    if op == "<=":
        return a <= b
    if op == ">":
        return a > b
    return a >= b


def _cast(v, t):
    if v is None:
        return None
    t = t.upper()
    if t in ("DOUBLE", "FLOAT", "REAL", "DECIMAL"):
        return float(v)
    if t in ("INT", "INTEGER", "BIGINT", "LONG", "SMALLINT", "TINYINT"):
        return int(float(v)) if isinstance(v, str) else int(v)
    if t in ("VARCHAR", "STRING", "CHAR"):
        if isinstance(v, float):
            from ....common.javafmt import java_double_str
            return java_double_str(v)
        if isinstance(v, bool):
            return "true" if v else "false"
        return str(v)
    if t == "BOOLEAN":
        return v.lower() == "true" if isinstance(v, str) else bool(v)
    return v


def _nullsafe(fn):
    def f(*a):
        if any(x is None for x in a):
            return None
        return fn(*a)
    return f


FUNCTIONS: Dict[str, Callable] = {
    "ABS": _nullsafe(abs), "SQRT": _nullsafe(math.sqrt), "LN": _nullsafe(math.log),
    "LOG10": _nullsafe(math.log10), "LOG2": _nullsafe(math.log2), "EXP": _nullsafe(math.exp),
    "POWER": _nullsafe(lambda a, b: float(a) ** b), "POW": _nullsafe(lambda a, b: float(a) ** b),
    "FLOOR": _nullsafe(lambda a: math.floor(a)), "CEIL": _nullsafe(lambda a: math.ceil(a)),
    "CEILING": _nullsafe(lambda a: math.ceil(a)),
    "ROUND": _nullsafe(lambda a, n=0: round(a, int(n)) if n else float(round(a)) if isinstance(a, float) else a),
    "SIN": _nullsafe(math.sin), "COS": _nullsafe(math.cos), "TAN": _nullsafe(math.tan),
    "ASIN": _nullsafe(math.asin), "ACOS": _nullsafe(math.acos), "ATAN": _nullsafe(math.atan),
    "SIGN": _nullsafe(lambda a: (a > 0) - (a < 0)), "MOD": _nullsafe(lambda a, b: a % b),
    "UPPER": _nullsafe(lambda s: s.upper()), "LOWER": _nullsafe(lambda s: s.lower()),
    "CHAR_LENGTH": _nullsafe(len), "CHARACTER_LENGTH": _nullsafe(len), "LENGTH": _nullsafe(len),
    "TRIM": _nullsafe(lambda s: s.strip()), "LTRIM": _nullsafe(lambda s: s.lstrip()),
    "RTRIM": _nullsafe(lambda s: s.rstrip()),
    "CONCAT": lambda *a: None if any(x is None for x in a) else "".join(str(x) for x in a),
    "CONCAT_WS": lambda sep, *a: None if sep is None else sep.join(str(x) for x in a if x is not None),
    "SUBSTRING": _nullsafe(lambda s, p, n=None: s[int(p) - 1:] if n is None else s[int(p) - 1:int(p) - 1 + int(n)]),
    "SUBSTR": _nullsafe(lambda s, p, n=None: s[int(p) - 1:] if n is None else s[int(p) - 1:int(p) - 1 + int(n)]),
    "REPLACE": _nullsafe(lambda s, a, b: s.replace(a, b)),
    "POSITION": _nullsafe(lambda a, s: s.find(a) + 1),
    "REGEXP_REPLACE": _nullsafe(lambda s, p, r: re.sub(p, r, s)),
    "REGEXP_EXTRACT": _nullsafe(lambda s, p, g=0: (lambda m: m.group(int(g)) if m else None)(re.search(p, s))),
    "COALESCE": lambda *a: next((x for x in a if x is not None), None),
    "IF": lambda c, a, b: a if c else b,
    "NULLIF": lambda a, b: None if a == b else a,
    "GREATEST": _nullsafe(lambda *a: max(a)), "LEAST": _nullsafe(lambda *a: min(a)),
    "RAND": lambda *a: __import__("random").random(),
    "PI": lambda: math.pi, "E": lambda: math.e,
    "TO_BASE64": _nullsafe(lambda s: __import__("base64").b64encode(s.encode()).decode()),
    "FROM_BASE64": _nullsafe(lambda s: __import__("base64").b64decode(s.encode()).decode()),
    "MD5": _nullsafe(lambda s: __import__("hashlib").md5(s.encode()).hexdigest()),
    "HASH_CODE": _nullsafe(lambda s: __import__("alink_amd.common.javafmt", fromlist=["x"]).java_string_hash(s)),
}


def _pad(s, n, pad, left):
    """Flink LPAD / RPAD: NULL for a negative length or an empty pad; truncation when ``n`` <= len(s)."""
    n = int(n)
    if n < 0 or not pad:
        return None
    if n <= len(s):
        return s[:n]
    fill = (pad * (n // len(pad) + 1))[:n - len(s)]
    return fill + s if left else s + fill


def _sha(bits):
    import hashlib
    algo = {1: hashlib.sha1, 224: hashlib.sha224, 256: hashlib.sha256, 384: hashlib.sha384, 512: hashlib.sha512}
    return lambda s: algo[bits](s.encode("utf-8")).hexdigest()


def _sha2(s, bits):
    b = int(bits)
    if b == 0:
        b = 256
    if b not in (224, 256, 384, 512):
        return None
    return _sha(b)(s)


def _log(a, b=None):
    # LOG(x) = ln x; LOG(base, x) = ln x / ln base (reference MathFunctions.LOG / LOG_WITH_BASE)
    return math.log(a) if b is None else math.log(b) / math.log(a)


# the reference's registered scalar functions (common/sql/functions MathFunctions, StringFunctions) and the Flink
# built-ins they complete
FUNCTIONS.update({
    "LOG": _nullsafe(_log), "SINH": _nullsafe(math.sinh), "COSH": _nullsafe(math.cosh), "TANH": _nullsafe(math.tanh),
    "COT": _nullsafe(lambda a: 1.0 / math.tan(a)), "ATAN2": _nullsafe(math.atan2),
    "DEGREES": _nullsafe(math.degrees), "RADIANS": _nullsafe(math.radians),
    "TRUNCATE": _nullsafe(lambda a, n=0: math.trunc(a * 10 ** int(n)) / 10 ** int(n) if int(n) else
                          (math.trunc(a) if isinstance(a, int) else float(math.trunc(a)))),
    "BIN": _nullsafe(lambda v: format(int(v) & 0xFFFFFFFFFFFFFFFF, "b")),       # Long.toBinaryString
    "HEX": _nullsafe(lambda v: v.encode("utf-8").hex().upper() if isinstance(v, str)
                     else format(int(v) & 0xFFFFFFFFFFFFFFFF, "x")),                 # Long.toHexString / bytes
    "LPAD": _nullsafe(lambda s, n, p: _pad(s, n, p, True)),
    "RPAD": _nullsafe(lambda s, n, p: _pad(s, n, p, False)),
    "SHA1": _nullsafe(_sha(1)), "SHA224": _nullsafe(_sha(224)), "SHA256": _nullsafe(_sha(256)),
    "SHA384": _nullsafe(_sha(384)), "SHA512": _nullsafe(_sha(512)), "SHA2": _nullsafe(_sha2),
    "UUID": lambda: str(__import__("uuid").uuid4()),
    "INITCAP": _nullsafe(lambda s: re.sub(r"[A-Za-z0-9]+", lambda m: m.group(0)[0].upper() + m.group(0)[1:].lower(), s)),
    "REPEAT": _nullsafe(lambda s, n: s * max(0, int(n))),
})


def _agg(name, vals, distinct):
    vals = [v for v in vals if v is not None]
    if distinct:
        seen = []
        for v in vals:
            if v not in seen:
                seen.append(v)
        vals = seen
    if name == "COUNT":
        return len(vals)
    if not vals:
        return None
    if name == "SUM":
        return sum(vals)
    if name == "AVG":
        s = sum(vals) / len(vals)
        return s if not all(isinstance(v, int) for v in vals) else s
    if name == "MIN":
        return min(vals)
    if name == "MAX":
        return max(vals)
    n = len(vals)
    mean = sum(vals) / n
    ss = sum((v - mean) ** 2 for v in vals)
    if name in ("VAR_SAMP", "VARIANCE"):
        return ss / (n - 1) if n > 1 else None
    if name == "VAR_POP":
        return ss / n
    if name in ("STDDEV_SAMP", "STDDEV"):
        return math.sqrt(ss / (n - 1)) if n > 1 else None
    if name == "STDDEV_POP":
        return math.sqrt(ss / n)
    raise ValueError(name)


def compile_expr(e: Expr, resolve: Callable[[str], int]) -> Callable:
    """Compile to ``f(row, group_rows=None)``; ``resolve(name) -> column index``."""
    k = e.kind
    if k == "lit":
        v = e.args[0]
        return lambda r, g=None: v
    if k == "col":
        i = resolve(e.args[0])
        return lambda r, g=None: r[i]
    if k == "star":
        return lambda r, g=None: 1
    if k == "neg":
        f = compile_expr(e.args[0], resolve)
        return lambda r, g=None: (lambda x: None if x is None else -x)(f(r, g))
    if k == "bin":
        op = e.args[0]
        a, b = compile_expr(e.args[1], resolve), compile_expr(e.args[2], resolve)
        return lambda r, g=None: _arith(op, a(r, g), b(r, g))
    if k == "cmp":
        op = e.args[0]
        a, b = compile_expr(e.args[1], resolve), compile_expr(e.args[2], resolve)
        return lambda r, g=None: _compare(op, a(r, g), b(r, g))
    if k == "and":
        a, b = compile_expr(e.args[0], resolve), compile_expr(e.args[1], resolve)

        def f_and(r, g=None):
            x = a(r, g)
            if x is False:
                return False
            y = b(r, g)
            if y is False:
                return False
            if x is None or y is None:
                return None
            return True
        return f_and
    if k == "or":
        a, b = compile_expr(e.args[0], resolve), compile_expr(e.args[1], resolve)

        def f_or(r, g=None):
            x = a(r, g)
            if x is True:
                return True
            y = b(r, g)
            if y is True:
                return True
            if x is None or y is None:
                return None
            return False
        return f_or
    if k == "not":
        a = compile_expr(e.args[0], resolve)
        return lambda r, g=None: (lambda x: None if x is None else not x)(a(r, g))
    if k == "isnull":
        a = compile_expr(e.args[0], resolve)
        neg = e.args[1]
        return lambda r, g=None: (a(r, g) is None) != neg
    if k == "like":
        a, p = compile_expr(e.args[0], resolve), compile_expr(e.args[1], resolve)
        neg = e.args[2]
        cache = {}

        def f_like(r, g=None):
            x, pat = a(r, g), p(r, g)
            if x is None or pat is None:
                return None
            rx = cache.get(pat) or cache.setdefault(pat, _like_to_regex(pat))
            return bool(rx.match(x)) != neg
        return f_like
    if k == "in":
        a = compile_expr(e.args[0], resolve)
        items = [compile_expr(x, resolve) for x in e.args[1]]
        neg = e.args[2]

        def f_in(r, g=None):
            x = a(r, g)
            if x is None:
                return None
            return (x in [f(r, g) for f in items]) != neg
        return f_in
    if k == "between":
        a, lo, hi = (compile_expr(x, resolve) for x in e.args[:3])
        neg = e.args[3]

        def f_bt(r, g=None):
            x, l, h = a(r, g), lo(r, g), hi(r, g)
            if x is None or l is None or h is None:
                return None
            return (l <= x <= h) != neg
        return f_bt
    if k == "case":
        operand = compile_expr(e.args[0], resolve) if e.args[0] is not None else None
        whens = [(compile_expr(c, resolve), compile_expr(v, resolve)) for c, v in e.args[1]]
        els = compile_expr(e.args[2], resolve)

        def f_case(r, g=None):
            ov = operand(r, g) if operand else None
            for c, v in whens:
                cv = c(r, g)
                if (operand is not None and cv == ov) or (operand is None and cv is True):
                    return v(r, g)
            return els(r, g)
        return f_case
    if k == "cast":
        a = compile_expr(e.args[0], resolve)
        t = e.args[1]
        return lambda r, g=None: _cast(a(r, g), t)
    if k == "fn":
        name = e.args[0]
        fn = FUNCTIONS.get(name)
        if fn is None:
            from .udf import get_registered_function
            fn = get_registered_function(name)
        args = [compile_expr(x, resolve) for x in e.args[1]]
        return lambda r, g=None: fn(*[f(r, g) for f in args])
    if k == "agg":
        name, args, distinct = e.args
        star = len(args) == 1 and args[0].kind == "star"
        af = compile_expr(args[0], resolve) if args and not star else (lambda r, g=None: 1)

        def f_agg(r, g=None):
            rows = g if g is not None else [r]
            return _agg(name, [af(x) for x in rows], distinct)
        return f_agg
    raise ValueError(f"cannot compile {e}")
