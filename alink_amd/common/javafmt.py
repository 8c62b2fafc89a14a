"""JVM-compatible text formatting.

Alink's persisted artefacts (Params JSON, model tables, vector strings) are produced by the JVM:
``Double.toString``, Gson with ``serializeNulls().disableHtmlEscaping().serializeSpecialFloatingPointValues()``
(reference ``core/src/main/java/org/apache/flink/ml/api/misc/param/Params.java:19-27``) and ``HashMap``
iteration order.  To read *and write* byte-compatible models we reproduce those three behaviours here.
"""
from __future__ import annotations

import math
import re
from typing import Any, Dict, Iterable, List

__all__ = [
    "java_double_str", "java_float_str", "gson_dumps", "java_str", "java_string_hash", "java_hashmap_order",
]


def _digits_exp(x: float):
    """Shortest round-trip decimal digits and decimal exponent of |x| (x finite, != 0).

    Returns (digits, e) with value = 0.digits * 10**e.
    """
    r = repr(abs(x))
    if "e" in r or "E" in r:
        mant, ex = r.lower().split("e")
        ex = int(ex)
    else:
        mant, ex = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    # position of decimal point relative to start of ip+fp
    point = len(ip) + ex
    # strip leading zeros accounted for
    lead = len(ip + fp) - len((ip + fp).lstrip("0"))
    point -= lead
    digits = digits.rstrip("0")
    if not digits:
        digits = "0"
    return digits, point


def java_double_str(x: float) -> str:
    """Reproduce ``java.lang.Double.toString(double)``.

    * |x| in [1e-3, 1e7): plain decimal with at least one fractional digit ("3.0", "0.001").
    * otherwise computerized scientific notation ("1.0E-4", "1.234E10").
    """
    if x is None:
        return "null"
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    sign = "-" if x < 0 else ""
    digits, point = _digits_exp(x)
    ax = abs(x)
    if 1e-3 <= ax < 1e7:
        if point <= 0:
            s = "0." + "0" * (-point) + digits
        elif point >= len(digits):
            s = digits + "0" * (point - len(digits)) + ".0"
        else:
            s = digits[:point] + "." + digits[point:]
        return sign + s
    # scientific: d.dddEn
    exp = point - 1
    mant = digits[0] + "." + (digits[1:] if len(digits) > 1 else "0")
    return f"{sign}{mant}E{exp}"


def java_float_str(x: float) -> str:
    """``java.lang.Float.toString`` (shortest float32 repr, same layout rules)."""
    import numpy as np
    f = np.float32(x)
    if np.isnan(f):
        return "NaN"
    if np.isinf(f):
        return "Infinity" if f > 0 else "-Infinity"
    if f == 0:
        return "-0.0" if np.signbit(f) else "0.0"
    r = np.format_float_positional(f, unique=True, trim="-")
    # reuse the double path on the shortest float digits
    return java_double_str(float(r)) if abs(float(r)) >= 1e-3 and abs(float(r)) < 1e7 else \
        java_double_str(float(np.format_float_scientific(f, unique=True)))


_NEEDS_ESCAPE = re.compile('["\\\\\x00-\x1f\u2028\u2029]')


def _gson_escape(s: str) -> str:
    if _NEEDS_ESCAPE.search(s) is None:          # the common case: nothing to escape
        return '"' + s + '"'
    out: List[str] = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "\b":
            out.append("\\b")
        elif ch == "\f":
            out.append("\\f")
        elif o < 0x20 or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def gson_dumps(v: Any, java_map_order: bool = True) -> str:
    """Serialize a Python value the way Gson serialises the corresponding Java value.

    * ``float`` -> ``Double.toString``; ``int`` -> decimal; ``bool`` -> true/false; ``None`` -> null.
    * ``dict`` -> JSON object, keys in Java ``HashMap`` order when ``java_map_order`` (Params maps are
      ``HashMap<String,String>``); objects that declare ``__gson_fields__`` keep that field order
      (Gson serialises POJO fields in declaration order).
    * enums (objects with ``.name``) -> their quoted name.
    """
    import enum
    import numpy as np
    if v is None:
        return "null"
    if isinstance(v, bool) or isinstance(v, np.bool_):
        return "true" if v else "false"
    if isinstance(v, enum.Enum):
        return _gson_escape(v.name)
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, (float, np.floating)):
        return java_double_str(float(v))
    if isinstance(v, str):
        return _gson_escape(v)
    if hasattr(v, "__gson_fields__"):
        # POJO fields in declaration order; null fields are written as null (what the reference's model
        # tables show, e.g. docs/en/aftsurvivalregression.md) unless the class sets __gson_skip_nulls__
        keep_nulls = not getattr(v, "__gson_skip_nulls__", False)
        parts = []
        for f in v.__gson_fields__:
            fv = getattr(v, f, None)
            if fv is None and not keep_nulls:
                continue
            parts.append(_gson_escape(f) + ":" + gson_dumps(fv, java_map_order))
        return "{" + ",".join(parts) + "}"
    if isinstance(v, dict):
        keys = java_hashmap_order(list(v.keys())) if java_map_order else list(v.keys())
        return "{" + ",".join(_gson_escape(str(k)) + ":" + gson_dumps(v[k], java_map_order) for k in keys) + "}"
    if isinstance(v, np.ndarray) and v.dtype.kind == "f" and v.ndim == 1 and v.size >= 64:
        # large float vectors (model coefficients): the host C++ formatter, same digits and layout
        from .. import _native
        body = _native.java_double_join(v)
        if body is not None:
            return "[" + body + "]"
    if isinstance(v, (list, tuple)) and len(v) >= 64 and all(type(e) is float for e in v):
        # long Python float lists (metric curves) through the same C++ formatter
        return gson_dumps(np.asarray(v, dtype=np.float64), java_map_order)
    if isinstance(v, (list, tuple)) or (hasattr(v, "tolist") and not isinstance(v, str)):
        seq = v.tolist() if hasattr(v, "tolist") else v
        return "[" + ",".join(gson_dumps(e, java_map_order) for e in seq) + "]"
    raise TypeError(f"cannot gson-serialize {type(v)}")


def java_string_hash(s: str) -> int:
    """``java.lang.String.hashCode`` over UTF-16 code units, as a signed 32-bit int."""
    h = 0
    data = s.encode("utf-16-le")
    for i in range(0, len(data), 2):
        cu = data[i] | (data[i + 1] << 8)
        h = (31 * h + cu) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def _spread(h: int) -> int:
    h &= 0xFFFFFFFF
    return (h ^ (h >> 16)) & 0xFFFFFFFF


def java_hashmap_order(keys: Iterable[str]) -> List[str]:
    """Iteration order of a ``java.util.HashMap`` filled by ``put`` in the given order.

    Capacity starts at 16 and doubles whenever size exceeds 0.75*capacity; resizing keeps the
    relative order inside each bucket, so the final order is (bucket index, insertion order).
    """
    keys = list(dict.fromkeys(keys))  # de-duplicate, keep first insertion position
    cap = 16
    while len(keys) > cap * 0.75:
        cap *= 2
    indexed = [(_spread(java_string_hash(k)) & (cap - 1), i, k) for i, k in enumerate(keys)]
    indexed.sort(key=lambda t: (t[0], t[1]))
    return [k for _, _, k in indexed]


def java_str(v) -> str:
    """``String.valueOf(obj)`` of a Java-typed cell: booleans lower-case, doubles via ``Double.toString``,
    vectors in Alink's string format."""
    import numpy as np
    if v is None:
        return "null"
    if isinstance(v, (bool, np.bool_)):
        return "true" if v else "false"
    if isinstance(v, (float, np.floating)):
        return java_double_str(float(v))
    if hasattr(v, "toString") and not isinstance(v, str):
        return v.toString()
    return str(v)
