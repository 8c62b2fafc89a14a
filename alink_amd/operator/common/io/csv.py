"""CSV parsing / formatting with Alink semantics.

Reference: ``A/operator/common/io/csv/CsvParser.java`` (quote handling only for string columns,
doubled quote = literal quote, empty / blank token -> NULL for non-string columns) and
``CsvFormatter.java``.  Bulk parsing goes through the native C++ runtime (``alink_amd._native``) when it
is built; this module is the reference implementation and fallback.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

from ....common.javafmt import java_double_str
from ....common.linalg import Vector, VectorUtil
from ....common.types import AlinkType, Types

__all__ = ["CsvParser", "CsvFormatter", "parse_token"]


def parse_token(tok: str, t: AlinkType):
    if t == Types.STRING:
        return tok
    if not tok.strip():
        return None
    s = tok.strip()
    if t in (Types.DOUBLE, Types.FLOAT, Types.DECIMAL):
        return float(s)
    if t in (Types.LONG, Types.INT, Types.SHORT, Types.BYTE):
        return int(s)
    if t == Types.BOOLEAN:
        ls = s.lower()
        if ls in ("true", "1"):
            return True
        if ls in ("false", "0"):
            return False
        raise ValueError(s)
    if t in (Types.VECTOR, Types.DENSE_VECTOR, Types.SPARSE_VECTOR):
        return VectorUtil.parse(s)
    return s


class CsvParser:
    def __init__(self, types: Sequence[AlinkType], field_delim: str = ",", quote_char: Optional[str] = '"'):
        self.types = list(types)
        self.delim = field_delim
        self.quote = quote_char if quote_char else None
        self.is_str = [t == Types.STRING for t in self.types]

    def _next_delim(self, line: str, start: int, is_str: bool) -> int:
        n = len(line)
        if start >= n:
            return -1
        if self.quote is None or not is_str or line[start] != self.quote:
            return line.find(self.delim, start)
        pos = start + 1
        escaped = False
        while pos < n:
            c = line[pos]
            if c == self.quote:
                if not escaped:
                    if pos + 1 < n and line[pos + 1] == self.quote:
                        escaped = True
                    else:
                        break
                else:
                    escaped = False
            pos += 1
        if pos >= n:
            return -1
        return line.find(self.delim, pos + 1)

    def parse(self, line: str) -> Tuple[bool, List]:
        out = [None] * len(self.types)
        if not line:
            return False, out
        start, ok, n = 0, True, len(line)
        for i, t in enumerate(self.types):
            if start > n:
                ok = False
                break
            d = self._next_delim(line, start, self.is_str[i])
            if d < 0:
                d = n
            tok = line[start:d]
            if tok:
                if self.is_str[i]:
                    if self.quote is not None and tok[0] == self.quote:
                        content = tok[1:-1] if tok.endswith(self.quote) and len(tok) > 1 else tok[1:]
                        out[i] = content.replace(self.quote * 2, self.quote)
                    else:
                        out[i] = tok
                else:
                    try:
                        out[i] = parse_token(tok, t)
                    except ValueError:
                        ok = False
            start = d + len(self.delim)
        return ok, out


class CsvFormatter:
    def __init__(self, types: Sequence[AlinkType], field_delim: str = ",", quote_char: Optional[str] = '"'):
        self.types = list(types)
        self.delim = field_delim
        self.quote = quote_char if quote_char else None

    def _fmt(self, v, t):
        if v is None:
            return ""
        if isinstance(v, Vector):
            v = VectorUtil.toString(v)
        if t == Types.STRING:
            s = str(v)
            if self.quote is not None and (not s or self.delim in s or self.quote in s):
                return self.quote + s.replace(self.quote, self.quote * 2) + self.quote
            return s
        if isinstance(v, bool):
            return "true" if v else "false"
        if isinstance(v, float):
            return java_double_str(v)
        return str(v)

    def format(self, row) -> str:
        return self.delim.join(self._fmt(v, t) for v, t in zip(row, self.types))
