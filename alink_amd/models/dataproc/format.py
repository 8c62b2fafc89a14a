"""Format conversion between Columns / CSV / JSON / KV / Vector / Triple, JSON path extraction and the
string-to-columns parsers.

Reference behaviour (``A/operator/common/dataproc/format/*``, ``StringToColumnsMappers.java``,
``StringParsers.java``, ``A/common/utils/JsonPathMapper.java``):

* a *reader* turns one input row into a ``key -> string`` map (``FormatReader.read``; ``ColumnsReader``
  uses ``toString`` of each non-null cell, ``VectorReader`` the index (or schema name) of each entry);
* a *writer* turns the map into the output cells (``ColumnsWriter`` parses each value with the column
  type, ``CsvWriter`` quotes values containing the delimiter/quote, ``KvWriter``/``JsonWriter`` iterate
  the map, ``VectorWriter`` builds a sparse vector from integer keys or a dense string in schema order);
* the map is a ``java.util.HashMap`` in the reference, so KV/JSON outputs follow HashMap iteration order —
  reproduced with ``java_hashmap_order`` so the strings are byte-identical to the reference's.
* ``AnyToTriple`` flattens a row into ``(reserved..., key, value)`` rows; ``TripleToAny`` groups triples
  by row id and writes each group with a writer (``TripleToAnyBatchOp.java``).

These are host (string) transforms — the reference runs them as Flink ``MapFunction``s; here they run
per micro-batch on the CPU side of the DAG, columnar where the input allows it.
"""
from __future__ import annotations

import functools
import json
import re
from typing import Any, Dict, List, Optional, Sequence, Tuple

from ...common.javafmt import gson_dumps, java_double_str, java_hashmap_order, java_str
from ...common.linalg import DenseVector, SparseVector, VectorUtil
from ...common.mapper import FlatMapper, Mapper, OutputColsHelper, find_col_index, find_col_indices
from ...common.params import Params
from ...common.table import Column, Row
from ...common.types import TableSchema, Types, schema_str_to_schema
from ...operator.common.io.csv import CsvParser, parse_token

__all__ = ["FormatTransMapper", "AnyToTripleFlatMapper", "triple_to_any_rows", "CsvToColumnsMapper",
           "JsonToColumnsMapper", "KvToColumnsMapper", "JsonPathMapper", "lenient_json_loads", "json_path_read",
           "init_format_reader", "init_format_writer"]


def _enum_name(v) -> str:
    return v.name if hasattr(v, "name") else str(v).upper()


def _p(params: Params, name: str, default=None):
    return params.get(name) if params.contains(name) else default


# ---------------------------------------------------------------------------------------------------
# lenient JSON (json-smart / Gson-lenient style: unquoted keys & values, single quotes)
# ---------------------------------------------------------------------------------------------------
class _LenientJson:
    _STOP = set(",:}]")

    def __init__(self, s: str):
        self.s = s
        self.i = 0

    def _ws(self):
        s, n = self.s, len(self.s)
        while self.i < n and s[self.i] in " \t\r\n":
            self.i += 1

    def value(self):
        self._ws()
        if self.i >= len(self.s):
            raise ValueError("unexpected end of json")
        c = self.s[self.i]
        if c == "{":
            return self._obj()
        if c == "[":
            return self._arr()
        if c in "\"'":
            return self._quoted()
        return self._bare()

    def _quoted(self):
        q = self.s[self.i]
        self.i += 1
        out = []
        while self.i < len(self.s):
            c = self.s[self.i]
            if c == "\\" and self.i + 1 < len(self.s):
                nxt = self.s[self.i + 1]
                if nxt == "u":
                    out.append(chr(int(self.s[self.i + 2:self.i + 6], 16)))
                    self.i += 6
                    continue
                out.append({"n": "\n", "t": "\t", "r": "\r", "b": "\b", "f": "\f"}.get(nxt, nxt))
                self.i += 2
                continue
            if c == q:
                self.i += 1
                return "".join(out)
            out.append(c)
            self.i += 1
        raise ValueError("unterminated string")

    def _bare(self):
        st = self.i
        while self.i < len(self.s) and self.s[self.i] not in self._STOP:
            self.i += 1
        tok = self.s[st:self.i].strip()
        if tok == "null":
            return None
        if tok == "true":
            return True
        if tok == "false":
            return False
        if re.fullmatch(r"-?\d+", tok):
            return int(tok)
        if re.fullmatch(r"-?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?", tok):
            return float(tok)
        return tok

    def _obj(self):
        self.i += 1
        out: Dict[str, Any] = {}
        self._ws()
        if self.i < len(self.s) and self.s[self.i] == "}":
            self.i += 1
            return out
        while True:
            self._ws()
            k = self._quoted() if self.s[self.i] in "\"'" else str(self._bare())
            self._ws()
            if self.i >= len(self.s) or self.s[self.i] not in ":=":
                raise ValueError("expected ':' in json object")
            self.i += 1
            out[k] = self.value()
            self._ws()
            if self.i >= len(self.s):
                raise ValueError("unterminated object")
            if self.s[self.i] == ",":
                self.i += 1
                continue
            if self.s[self.i] == "}":
                self.i += 1
                return out
            raise ValueError("bad json object")

    def _arr(self):
        self.i += 1
        out: List[Any] = []
        self._ws()
        if self.i < len(self.s) and self.s[self.i] == "]":
            self.i += 1
            return out
        while True:
            out.append(self.value())
            self._ws()
            if self.s[self.i] == ",":
                self.i += 1
                continue
            if self.s[self.i] == "]":
                self.i += 1
                return out
            raise ValueError("bad json array")


def lenient_json_loads(s: str):
    try:
        return json.loads(s)
    except (ValueError, TypeError):
        p = _LenientJson(s)
        v = p.value()
        return v


_PATH_TOK = re.compile(r"\.\.|\.\*|\.([^.\[\]]+)|\[\s*\*\s*\]|\[\s*(-?\d+)\s*\]|\[\s*['\"]([^'\"]+)['\"]\s*\]")


@functools.lru_cache(maxsize=256)
def _json_path_tokens(path: str):
    """A json path split once into (kind, arg) steps: ("*", None) wildcard, ("i", int) index, ("k", str) key."""
    path = path.strip()
    if not path.startswith("$"):
        path = "$." + path
    toks = []
    pos = 1
    while pos < len(path):
        m = _PATH_TOK.match(path, pos)
        if m is None:
            raise ValueError(f"bad json path {path}")
        tok = m.group(0)
        pos = m.end()
        if tok == "..":
            raise ValueError("deep scan '..' is not supported")
        if tok in (".*",) or tok.replace(" ", "") == "[*]":
            toks.append(("*", None))
        elif m.group(2) is not None:
            toks.append(("i", int(m.group(2))))
        else:
            toks.append(("k", m.group(1) if m.group(1) is not None else m.group(3)))
    return path, tuple(toks)


def json_path_read(doc, path: str):
    """Subset of Jayway JsonPath used by Alink docs: ``$``, ``.name``, ``['name']``, ``[i]``, ``[*]``, ``.*``.
    A wildcard makes the result a list.  Missing keys raise ``KeyError`` (``PathNotFoundException``)."""
    path, toks = _json_path_tokens(path)
    cur = [doc]
    multi = False
    for kind, arg in toks:
        nxt = []
        if kind == "*":
            multi = True
            for c in cur:
                if isinstance(c, dict):
                    nxt.extend(c.values())
                elif isinstance(c, list):
                    nxt.extend(c)
        elif kind == "i":
            for c in cur:
                if not isinstance(c, list):
                    raise KeyError(path)
                nxt.append(c[arg])
        else:
            for c in cur:
                if isinstance(c, dict) and arg in c:
                    nxt.append(c[arg])
                elif not multi:
                    raise KeyError(f"No results for path: {path}")
        cur = nxt
    return cur if multi else cur[0]


def _gson_of(v) -> str:
    """``gson.toJson`` of a json-smart value (JSONObject is a HashMap -> HashMap key order)."""
    return gson_dumps(v, java_map_order=True)


def _java_to_string(v) -> str:
    """``Object.toString`` of a Gson-parsed value (numbers are Doubles, objects LinkedTreeMaps)."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return java_double_str(float(v))
    if isinstance(v, dict):
        return "{" + ", ".join(f"{k}={_java_to_string(x)}" for k, x in v.items()) + "}"
    if isinstance(v, list):
        return "[" + ", ".join(_java_to_string(x) for x in v) + "]"
    if v is None:
        return "null"
    return str(v)


# ---------------------------------------------------------------------------------------------------
# field parsing (Flink FieldParser semantics for the target column type)
# ---------------------------------------------------------------------------------------------------
def parse_field(token: Optional[str], t) -> Tuple[bool, Any]:
    if t == Types.STRING:
        return True, token
    if token is None or not str(token).strip():
        return False, None
    try:
        if t in (Types.LONG, Types.INT, Types.SHORT, Types.BYTE):
            s = str(token).strip()
            if not re.fullmatch(r"[-+]?\d+", s):
                return False, None
            return True, int(s)
        return True, parse_token(str(token), t)
    except (ValueError, TypeError):
        return False, None


# ---------------------------------------------------------------------------------------------------
# readers
# ---------------------------------------------------------------------------------------------------
class _Reader:
    def read(self, row) -> Tuple[bool, Dict[str, Optional[str]]]:
        raise NotImplementedError


class ColumnsReader(_Reader):
    def __init__(self, idx: List[int], names: List[str]):
        self.idx, self.names = idx, names

    def read(self, row):
        out = {}
        for i, n in zip(self.idx, self.names):
            v = row[i]
            if v is not None:
                out[n] = java_str(v)
        return True, out


class CsvReader(_Reader):
    def __init__(self, col: int, schema: TableSchema, delim: str, quote: Optional[str]):
        self.col = col
        self.names = list(schema.names)
        self.parser = CsvParser(schema.types, delim, quote)

    def read(self, row):
        line = row[self.col]
        if line is None:
            return False, {}
        ok, vals = self.parser.parse(line)
        return ok, {n: (java_str(v) if v is not None else None) for n, v in zip(self.names, vals)}


class JsonReader(_Reader):
    def __init__(self, col: int):
        self.col = col

    def read(self, row):
        line = row[self.col]
        if line is None:
            return False, {}
        try:
            m = lenient_json_loads(line)
        except ValueError:
            return False, {}
        if not isinstance(m, dict):
            return False, {}
        return True, {str(k): _java_to_string(v) for k, v in m.items()}


class KvReader(_Reader):
    def __init__(self, col: int, col_delim: str, val_delim: str):
        self.col, self.cd, self.vd = col, col_delim, val_delim

    def read(self, row):
        line = row[self.col]
        out = {}
        if line is None:
            return False, out
        for f in re.split(self.cd, line) if len(self.cd) > 1 else line.split(self.cd):
            if not f.strip():
                return False, out
            kv = re.split(self.vd, f) if len(self.vd) > 1 else f.split(self.vd)
            if len(kv) != 2:
                return False, out
            out[kv[0]] = kv[1]
        return True, out


class VectorReader(_Reader):
    def __init__(self, col: int, names: Optional[List[str]]):
        self.col, self.names = col, names

    def read(self, row):
        v = VectorUtil.getVector(row[self.col])
        out = {}
        if v is None:
            return False, out
        if isinstance(v, SparseVector):
            for i, x in zip(v.getIndices().tolist(), v.getValues().tolist()):
                if self.names is None:
                    out[str(i)] = java_double_str(x)
                elif i < len(self.names):
                    out[self.names[i]] = java_double_str(x)
        else:
            data = v.getData().tolist()
            for i, x in enumerate(data):
                if self.names is None:
                    out[str(i)] = java_double_str(x)
                elif i < len(self.names):
                    out[self.names[i]] = java_double_str(x)
        return True, out


# ---------------------------------------------------------------------------------------------------
# writers
# ---------------------------------------------------------------------------------------------------
class _Writer:
    names: List[str]
    types: list

    def write(self, m: Dict[str, Optional[str]]) -> Tuple[bool, List[Any]]:
        raise NotImplementedError


def _hash_items(m: Dict[str, Any]):
    return [(k, m[k]) for k in java_hashmap_order(list(m.keys()))]


class ColumnsWriter(_Writer):
    def __init__(self, schema: TableSchema):
        self.names, self.types = list(schema.names), list(schema.types)
        self.pos = {n: i for i, n in enumerate(self.names)}

    def write(self, m):
        out = [None] * len(self.names)
        for k, v in m.items():
            i = self.pos.get(k)
            if i is None:
                continue
            ok, pv = parse_field(v, self.types[i])
            if not ok:
                return False, out
            out[i] = pv
        return True, out


class CsvWriter(_Writer):
    def __init__(self, out_col: str, schema: TableSchema, delim: str, quote: Optional[str]):
        self.cols = list(schema.names)
        self.delim, self.quote = delim, quote
        self.names, self.types = [out_col], [Types.STRING]

    def write(self, m):
        parts = []
        for c in self.cols:
            v = m.get(c)
            if v is None:
                parts.append("")
            elif self.quote and (not v or self.delim in v or self.quote in v):
                parts.append(self.quote + v.replace(self.quote, self.quote * 3) + self.quote)
            else:
                parts.append(v)
        return True, [self.delim.join(parts)]


class JsonWriter(_Writer):
    def __init__(self, out_col: str):
        self.names, self.types = [out_col], [Types.STRING]

    def write(self, m):
        # Gson without serializeNulls drops null map values (JsonConverter.java:117)
        return True, [gson_dumps({k: v for k, v in m.items() if v is not None}, java_map_order=True)]


class KvWriter(_Writer):
    def __init__(self, out_col: str, col_delim: str, val_delim: str):
        self.names, self.types = [out_col], [Types.STRING]
        self.cd, self.vd = col_delim, val_delim

    def write(self, m):
        return True, [self.cd.join(f"{k}{self.vd}{java_str(v)}" for k, v in _hash_items(m))]


class VectorWriter(_Writer):
    def __init__(self, out_col: str, size: int, from_names: Optional[List[str]]):
        self.names, self.types = [out_col], [Types.STRING]
        self.size = int(size) if size is not None else -1
        self.from_names = from_names

    def write(self, m):
        if self.from_names is None:
            try:
                items = _hash_items(m)
                idx = [int(k) for k, _ in items]
                vals = [float(v) for _, v in items]
            except (TypeError, ValueError):
                return False, [None]
            return True, [VectorUtil.toString(SparseVector(self.size, idx, vals))]
        n = len(self.from_names)
        prefix = ""
        if self.size > n:
            prefix = f"${self.size}$"
        elif 0 < self.size < n:
            n = self.size
        return True, [prefix + " ".join(java_str(m.get(c)) for c in self.from_names[:n])]


# ---------------------------------------------------------------------------------------------------
# factory (FormatTransMapper.initFormatReader / initFormatWriter)
# ---------------------------------------------------------------------------------------------------
def init_format_reader(schema: TableSchema, params: Params) -> Tuple[_Reader, Optional[List[str]]]:
    f = _enum_name(params.get("fromFormat"))
    names = list(schema.names)
    if f == "KV":
        return KvReader(find_col_index(names, params.get("kvCol")), _p(params, "kvColDelimiter", ","),
                        _p(params, "kvValDelimiter", ":")), None
    if f == "CSV":
        sch = schema_str_to_schema(params.get("schemaStr"))
        return CsvReader(find_col_index(names, params.get("csvCol")), sch, _p(params, "csvFieldDelimiter", ","),
                         _p(params, "quoteChar", '"')), list(sch.names)
    if f == "VECTOR":
        ss = _p(params, "schemaStr")
        vn = list(schema_str_to_schema(ss).names) if ss else None
        return VectorReader(find_col_index(names, params.get("vectorCol")), vn), None
    if f == "JSON":
        return JsonReader(find_col_index(names, params.get("jsonCol"))), None
    if f == "COLUMNS":
        sel = _p(params, "selectedCols") or names
        return ColumnsReader(find_col_indices(names, sel), list(sel)), list(sel)
    raise ValueError(f"Can not translate this type : {f}")


def init_format_writer(params: Params, from_names: Optional[List[str]]) -> _Writer:
    t = _enum_name(params.get("toFormat"))
    if t == "COLUMNS":
        return ColumnsWriter(schema_str_to_schema(params.get("schemaStr")))
    if t == "JSON":
        return JsonWriter(params.get("jsonCol"))
    if t == "KV":
        return KvWriter(params.get("kvCol"), _p(params, "kvColDelimiter", ","), _p(params, "kvValDelimiter", ":"))
    if t == "CSV":
        return CsvWriter(params.get("csvCol"), schema_str_to_schema(params.get("schemaStr")),
                         _p(params, "csvFieldDelimiter", ","), _p(params, "quoteChar", '"'))
    if t == "VECTOR":
        return VectorWriter(params.get("vectorCol"), _p(params, "vectorSize", -1), from_names)
    raise ValueError(f"Can not translate to this type : {t}")


def _handle_error(params: Params) -> bool:
    return _enum_name(_p(params, "handleInvalid", "ERROR")) == "ERROR"


# ---------------------------------------------------------------------------------------------------
# columnar fast paths: numeric conversions done over whole columns (C++ formatting / parsing) with output
# identical to the reader -> map -> writer row path; any input outside the exact conditions returns None and
# the caller takes the row path (which also owns every error / handleInvalid case)
# ---------------------------------------------------------------------------------------------------
_SAFE_SEP = set("0123456789.-+eEINaityf")          # separators that could occur inside Double.toString


def _native():
    try:
        from ... import _native as N
    except Exception:   # pragma: no cover - library import failure: row path
        return None
    return N if N.lib is not None else None


def _double_matrix(mt, names: Sequence[str]):
    """(n, k) float64 numpy of DOUBLE columns without nulls, or None."""
    import numpy as np
    import torch
    cols = []
    for nm in names:
        i = find_col_index(mt.schema.names, nm)
        c = mt.cols[i]
        if mt.schema.types[i] != Types.DOUBLE or not isinstance(c.values, torch.Tensor) or c.values.dim() != 1:
            return None
        if c.nulls is not None and bool(c.nulls.any()):
            return None
        cols.append(c.values)
    if not cols:
        return None
    return np.ascontiguousarray(torch.stack(cols, 1).to("cpu", torch.float64).numpy())


def _packed_strings(col):
    """(uint8 bytes, int64 offsets [n+1]) of a string column without nulls — a host view of a ``StringBlock``, or
    one pack of a list of str — or None."""
    import numpy as np
    from ...common.strings import StringBlock
    v = col.values
    if isinstance(v, StringBlock):
        if v.nulls is not None:
            return None
        return v.data.cpu().numpy(), v.offsets.cpu().numpy()
    if not isinstance(v, list) or not all(isinstance(s, str) for s in v):
        return None
    N = _native()
    buf, off = N._pack_utf8(v)
    return np.frombuffer(buf, dtype=np.uint8), off


def _string_block(data, off, prefix: str = ""):
    """``StringBlock`` over packed ASCII rows, with ``prefix`` prepended to every row."""
    import numpy as np
    import torch
    from ...common.strings import StringBlock
    if prefix:
        pb = np.frombuffer(prefix.encode("ascii"), dtype=np.uint8)
        n, lp = off.size - 1, pb.size
        lens = np.diff(off)
        noff = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens + lp, out=noff[1:])
        out = np.empty(int(noff[-1]), dtype=np.uint8)
        for j in range(lp):
            out[noff[:-1] + j] = pb[j]
        row = np.repeat(np.arange(n, dtype=np.int64), lens)
        out[np.arange(data.size, dtype=np.int64) + lp * (row + 1)] = data
        data, off = out, noff
    return StringBlock(torch.from_numpy(np.array(data, dtype=np.uint8)), torch.from_numpy(off))


_CSV_CODES = {Types.DOUBLE: 1, Types.FLOAT: 1, Types.LONG: 2, Types.INT: 2, Types.SHORT: 2, Types.BYTE: 2,
              Types.BOOLEAN: 3, Types.STRING: 0}
_INT_RANGE = {Types.INT: 31, Types.SHORT: 15, Types.BYTE: 7}


def csv_columns_fast(col, types, delim: str, quote: Optional[str]):
    """Typed columns of a column of non-empty CSV lines through the C++ parser (the CSV source's bulk path), or
    None when a line is null / empty / unparsable, a type has no native code or an integer leaves its Java range."""
    import numpy as np
    import torch
    from ...common.table import Column
    N = _native()
    if N is None or len(delim) != 1 or (quote is not None and len(quote) > 1):
        return None
    if any(t not in _CSV_CODES for t in types):
        return None
    packed = _packed_strings(col) if isinstance(col, Column) else _packed_strings(Column(list(col)))
    if packed is None or (packed[1].size > 1 and not np.diff(packed[1]).all()):
        return None
    try:
        res = N.parse_csv_packed(packed[0], packed[1], [_CSV_CODES[t] for t in types], delim, quote or "")
    except RuntimeError:
        return None
    if res is None:
        return None
    out = []
    for t, (vals, nulls) in zip(types, res):
        if isinstance(vals, list):
            out.append(Column(vals))
            continue
        if t in _INT_RANGE:
            b = 1 << _INT_RANGE[t]
            if vals.size and (int(vals.min()) < -b or int(vals.max()) >= b):
                return None
        nm = torch.from_numpy(np.ascontiguousarray(nulls)) if nulls is not None and nulls.any() else None
        out.append(Column(torch.from_numpy(vals).to(t.torch_dtype), nm))
    return out


def _w_vector(m: "FormatTransMapper", get, names):
    w = m.writer
    n, prefix = len(w.from_names), ""
    if w.size > n:
        prefix = f"${w.size}$"
    elif 0 < w.size < n:
        n = w.size
    if list(names) != list(w.from_names):
        return None
    X = get(w.from_names[:n])
    N = _native()
    if X is None or N is None:
        return None
    from ...common.table import Column
    r = N.java_double_rows_packed(X, " ")
    return None if r is None else [Column(_string_block(r[0], r[1], prefix))]


def _w_csv(m: "FormatTransMapper", get, names):
    w = m.writer
    if (len(w.delim) != 1 or w.delim in _SAFE_SEP or (w.quote and (len(w.quote) != 1 or w.quote in _SAFE_SEP))
            or not set(w.cols) <= set(names)):
        return None
    X = get(w.cols)
    N = _native()
    if X is None or N is None:
        return None
    from ...common.table import Column
    r = N.java_double_rows_packed(X, w.delim)
    return None if r is None else [Column(_string_block(r[0], r[1]))]


def _cols_getter(mt):
    return lambda names: _double_matrix(mt, names)


def _cols_to_vector(m: "FormatTransMapper", mt):
    return _w_vector(m, _cols_getter(mt), m.reader.names)


def _cols_to_csv(m: "FormatTransMapper", mt):
    return _w_csv(m, _cols_getter(mt), m.reader.names)


def _vector_to_cols(m: "FormatTransMapper", mt):
    import numpy as np
    import torch
    from ...common.table import Column
    vn, w = m.reader.names, m.writer
    if vn is None or len(set(vn)) != len(vn) or any(t != Types.DOUBLE for t in w.types):
        return None
    c = mt.cols[m.reader.col]
    if isinstance(c.values, torch.Tensor) and c.values.dim() == 2:
        if c.nulls is not None and bool(c.nulls.any()):
            return None
        V, d = c.values.to(torch.float64), int(c.values.shape[1])
    else:
        N = _native()
        packed = _packed_strings(c) if N is not None else None
        if packed is None:
            return None
        P = N.parse_dense_vectors_packed(packed[0], packed[1], len(vn))
        if P is None:
            return None
        V, d = torch.from_numpy(P), len(vn)
    pos = {nm: i for i, nm in enumerate(vn)}
    out = []
    for nm in w.names:
        i = pos.get(nm)
        if i is None or i >= d:
            out.append(Column(torch.zeros(V.shape[0], dtype=torch.float64, device=V.device)))
        else:
            out.append(Column(V[:, i].contiguous()))
    return out


def _csv_to_cols(m: "FormatTransMapper", mt):
    r, w = m.reader, m.writer
    if r.names != w.names or [*r.parser.types] != [*w.types]:
        return None
    cols = csv_columns_fast(mt.cols[r.col], w.types, r.parser.delim, r.parser.quote)
    # an empty typed field is a null map value that ColumnsWriter fails to parse: the row path owns that case
    if cols is None or any(c.nulls is not None for c in cols):
        return None
    return cols


def kv_columns_fast(col, names, types, cd: str, vd: str, need_all: bool, allow_dup: bool):
    """DOUBLE columns of a column of plain KV lines through the C++ parser: (columns with NULL where a key is
    absent) or None -- another column type, a multi-character delimiter (the row path splits on a regex then),
    a line outside the plain form, a key given twice (unless ``allow_dup``: the last one wins, as a HashMap put),
    or a line missing a key when ``need_all``."""
    import torch
    from ...common.table import Column
    N = _native()
    if N is None or len(cd) != 1 or len(vd) != 1 or any(t != Types.DOUBLE for t in types):
        return None
    packed = _packed_strings(col)
    if packed is None:
        return None
    r = N.parse_kv_packed(packed[0], packed[1], names, cd, vd)
    if r is None:
        return None
    vals, found, dup = r
    if (not allow_dup and dup.any()) or (need_all and not found.all()):
        return None
    out = []
    for j in range(len(names)):
        miss = ~found[:, j]
        out.append(Column(torch.from_numpy(vals[:, j].copy()), torch.from_numpy(miss) if miss.any() else None))
    return out


_PLAIN_KEY = re.compile(r"[A-Za-z_][A-Za-z0-9_]*")


def json_columns_fast(col, names, types, need_all: bool):
    """DOUBLE columns of a column of flat JSON objects with numeric members through the C++ reader (NULL where a
    key is absent), or None: another column type, a key that is a JSON path rather than a plain name, a line
    outside that form, or a line missing a key when ``need_all``."""
    import torch
    from ...common.table import Column
    N = _native()
    if N is None or any(t != Types.DOUBLE for t in types) or not all(_PLAIN_KEY.fullmatch(n) for n in names):
        return None
    packed = _packed_strings(col)
    if packed is None:
        return None
    r = N.parse_json_flat_packed(packed[0], packed[1], names)
    if r is None:
        return None
    vals, found = r
    if need_all and not found.all():
        return None
    out = []
    for j in range(len(names)):
        miss = ~found[:, j]
        out.append(Column(torch.from_numpy(vals[:, j].copy()), torch.from_numpy(miss) if miss.any() else None))
    return out


def _json_to_cols(m: "FormatTransMapper", mt):
    return json_columns_fast(mt.cols[m.reader.col], m.writer.names, m.writer.types, need_all=False)


def _w_kv(m: "FormatTransMapper", get, names):
    """KV over DOUBLE values without nulls: the HashMap key order of the row path (the same for every row when
    no value is null), one C++ formatting pass into a StringBlock."""
    w, names = m.writer, list(names)
    if (len(w.cd) != 1 or w.cd in _SAFE_SEP or any(w.cd in k or w.vd in k for k in names)
            or len(set(names)) != len(names) or not all(k.isascii() for k in names) or not w.vd.isascii()):
        return None
    order = [k for k, _ in _hash_items({k: "" for k in names})]
    X = get(order)
    N = _native()
    if X is None or N is None:
        return None
    from ...common.table import Column
    r = N.java_double_rows_fmt(X, [k + w.vd for k in order], [""] * len(order), w.cd)
    return None if r is None else [Column(_string_block(r[0], r[1]))]


def _w_json(m: "FormatTransMapper", get, names):
    """JSON over DOUBLE values without nulls with plain key names: {"k":"v",...} (the map holds the values'
    strings) in the row path's HashMap order."""
    import json as _json
    names = list(names)
    if not all(_PLAIN_KEY.fullmatch(k) for k in names) or len(set(names)) != len(names):
        return None
    order = list(_json.loads(gson_dumps({k: "0" for k in names}, java_map_order=True)).keys())
    X = get(order)
    N = _native()
    if X is None or N is None:
        return None
    from ...common.table import Column
    r = N.java_double_rows_fmt(X, ['"' + k + '":"' for k in order], ['"'] * len(order), ",", "{", "}")
    return None if r is None else [Column(_string_block(r[0], r[1]))]


def _cols_to_kv(m: "FormatTransMapper", mt):
    return _w_kv(m, _cols_getter(mt), m.reader.names)


def _cols_to_json(m: "FormatTransMapper", mt):
    return _w_json(m, _cols_getter(mt), m.reader.names)


def _csv_getter(m: "FormatTransMapper", mt):
    """The CSV reader's DOUBLE fields parsed once (C++), as a getter of [n, k] matrices; None unless every field
    is DOUBLE and present (an empty field is a null map value: the row path)."""
    import numpy as np
    r = m.reader
    if any(t != Types.DOUBLE for t in r.parser.types):
        return None
    cols = csv_columns_fast(mt.cols[r.col], r.parser.types, r.parser.delim, r.parser.quote)
    if cols is None or any(c.nulls is not None for c in cols):
        return None
    arr = {nm: c.values.numpy() for nm, c in zip(r.names, cols)}
    return lambda names: np.ascontiguousarray(np.stack([arr[nm] for nm in names], 1)) if names else None


def _vector_getter(m: "FormatTransMapper", mt):
    """(names, getter) of the VECTOR reader over dense vectors that all have exactly the reader's width (the map
    then holds every name: the schema names, or "0" .. "d-1" without a schema), or None."""
    import numpy as np
    import torch
    r = m.reader
    c = mt.cols[r.col]
    if isinstance(c.values, torch.Tensor) and c.values.dim() == 2:
        if c.nulls is not None and bool(c.nulls.any()):
            return None
        V = c.values.to("cpu", torch.float64).numpy()
        d = V.shape[1]
    else:
        N = _native()
        packed = _packed_strings(c) if N is not None else None
        if packed is None or packed[1].size < 2:
            return None
        d = len(r.names) if r.names is not None else None
        if d is None:
            # width from the first row, then every row must match it
            first = bytes(packed[0][packed[1][0]:packed[1][1]]).decode("ascii", "replace")
            d = len([t for t in first.replace(",", " ").split(" ") if t])
        res = N.parse_dense_vectors_packed(packed[0], packed[1], d, with_counts=True) if d else None
        if res is None:
            return None
        V, cnt = res
        if not (cnt == d).all():
            return None
    names = list(r.names) if r.names is not None else [str(i) for i in range(d)]
    if len(names) != d or len(set(names)) != d:
        return None
    pos = {nm: i for i, nm in enumerate(names)}
    return names, (lambda ns: np.ascontiguousarray(V[:, [pos[nm] for nm in ns]]) if ns else None)


def _vector_to(writer):
    def fn(m: "FormatTransMapper", mt):
        g = _vector_getter(m, mt)
        return None if g is None else writer(m, g[1], g[0])
    return fn


def _csv_to(writer):
    def fn(m: "FormatTransMapper", mt):
        get = _csv_getter(m, mt)
        return None if get is None else writer(m, get, m.reader.names)
    return fn


def _kv_to_cols(m: "FormatTransMapper", mt):
    r, w = m.reader, m.writer
    return kv_columns_fast(mt.cols[r.col], w.names, w.types, r.cd, r.vd, need_all=False, allow_dup=True)


_COLUMNAR = {("COLUMNS", "VECTOR"): _cols_to_vector, ("COLUMNS", "CSV"): _cols_to_csv,
             ("VECTOR", "COLUMNS"): _vector_to_cols, ("CSV", "COLUMNS"): _csv_to_cols,
             ("KV", "COLUMNS"): _kv_to_cols, ("JSON", "COLUMNS"): _json_to_cols,
             ("COLUMNS", "KV"): _cols_to_kv, ("COLUMNS", "JSON"): _cols_to_json,
             ("CSV", "VECTOR"): _csv_to(_w_vector), ("CSV", "CSV"): _csv_to(_w_csv), ("CSV", "KV"): _csv_to(_w_kv),
             ("CSV", "JSON"): _csv_to(_w_json),
             ("VECTOR", "CSV"): _vector_to(_w_csv), ("VECTOR", "KV"): _vector_to(_w_kv),
             ("VECTOR", "JSON"): _vector_to(_w_json)}


class FormatTransMapper(Mapper):
    """``FormatTransMapper.java`` — ``fromFormat``/``toFormat`` params pick the reader and the writer."""

    def __init__(self, dataSchema: TableSchema, params: Optional[Params] = None):
        super().__init__(dataSchema, params)
        self.reader, from_names = init_format_reader(dataSchema, self.params)
        self.writer = init_format_writer(self.params, from_names)
        self.err = _handle_error(self.params)
        self.vec_to_cols = (_enum_name(self.params.get("fromFormat")) == "VECTOR"
                            and _enum_name(self.params.get("toFormat")) == "COLUMNS")
        self.helper = OutputColsHelper(dataSchema, self.writer.names, self.writer.types,
                                       _p(self.params, "reservedCols"))
        self._fast = _COLUMNAR.get((_enum_name(self.params.get("fromFormat")),
                                    _enum_name(self.params.get("toFormat"))))

    def _map_columns(self, mt):
        if self._fast is not None and mt.num_rows > 0:
            cols = self._fast(self, mt)
            if cols is not None:
                return cols
        return super()._map_columns(mt)

    def _map_row_values(self, row):
        ok, m = self.reader.read(row)
        if not ok and self.err:
            raise RuntimeError(f"Fail to read: {list(row)}")
        ok, out = self.writer.write(m)
        if not ok and self.err:
            raise RuntimeError(f"Fail to write: {gson_dumps(m)}")
        if self.vec_to_cols:
            out = [0.0 if v is None else v for v in out]
        return out


class AnyToTripleFlatMapper(FlatMapper):
    """``AnyToTripleFlatMapper.java`` — one output row per (key, value) of the read map."""

    def __init__(self, dataSchema: TableSchema, params: Optional[Params] = None):
        super().__init__(dataSchema, params)
        sch = schema_str_to_schema(self.params.get("tripleColValSchemaStr"))
        self.kt, self.vt = sch.types[0], sch.types[1]
        self.reader, _ = init_format_reader(dataSchema, self.params)
        self.err = _handle_error(self.params)
        self.helper = OutputColsHelper(dataSchema, list(sch.names), list(sch.types), _p(self.params, "reservedCols"))

    def getOutputSchema(self):
        return self.helper.getResultSchema()

    def flatMap(self, row) -> List[Row]:
        ok, m = self.reader.read(row)
        out = []
        if not ok:
            if self.err:
                raise RuntimeError(f"Fail to read: {list(row)}")
            return out
        for k, v in _hash_items(m):
            if v is None or not str(v).strip():
                continue
            ok1, pk = parse_field(k, self.kt)
            ok2, pv = parse_field(v, self.vt)
            if ok1 and ok2:
                out.append(self.helper.getResultRow(row, [pk, pv]))
            elif self.err:
                raise RuntimeError(f"Fail to write: {gson_dumps(m)}")
        return out


def triple_to_any_rows(rows: Sequence[Sequence[Any]], params: Params) -> Tuple[List[str], list, List[Row]]:
    """Group ``(row, col, val)`` triples by row id and write each group (``TripleToAnyBatchOp.ToAny``).
    Returns output names/types (excluding the row column) and the output rows ``(rowId, cells...)``."""
    writer = init_format_writer(params, None)
    err = _handle_error(params)
    groups: Dict[Any, Dict[str, str]] = {}
    for r, c, v in rows:
        groups.setdefault(r, {})[java_str(c)] = java_str(v)
    out = []
    for r in sorted(groups, key=lambda x: (x is None, x)):
        ok, cells = writer.write(groups[r])
        if not ok:
            if err:
                raise RuntimeError(f"Fail to convert: {gson_dumps(groups[r])}")
            continue
        out.append(Row((r,) + tuple(cells)))
    return writer.names, writer.types, out


# ---------------------------------------------------------------------------------------------------
# StringToColumnsMappers (CsvToColumns / JsonToColumns / KvToColumns with schemaStr)
# ---------------------------------------------------------------------------------------------------
class _StringToColumns(Mapper):
    COL_PARAMS: Tuple[str, ...] = ()

    def __init__(self, dataSchema: TableSchema, params: Optional[Params] = None):
        super().__init__(dataSchema, params)
        col = None
        for name in self.COL_PARAMS + ("selectedCol",):
            col = col or _p(self.params, name)
        self.idx = find_col_index(dataSchema.names, col)
        sch = schema_str_to_schema(self.params.get("schemaStr"))
        self.names, self.types = list(sch.names), list(sch.types)
        self.err = _handle_error(self.params)
        self.helper = OutputColsHelper(dataSchema, self.names, self.types, _p(self.params, "reservedCols"))

    def parse(self, text: str) -> Tuple[bool, List[Any]]:
        raise NotImplementedError

    def _map_row_values(self, row):
        text = row[self.idx]
        ok, vals = self.parse(text) if text is not None else (False, [None] * len(self.names))
        if not ok and self.err:
            raise RuntimeError(f'Fail to parse "{text}"')
        return vals


class CsvToColumnsMapper(_StringToColumns):
    COL_PARAMS = ("csvCol",)

    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        delim = _p(self.params, "csvFieldDelimiter") or _p(self.params, "fieldDelimiter") or ","
        self.parser = CsvParser(self.types, delim, _p(self.params, "quoteChar", '"'))

    def _map_columns(self, mt):
        if mt.num_rows > 0:
            cols = csv_columns_fast(mt.cols[self.idx], self.types, self.parser.delim, self.parser.quote)
            if cols is not None:
                return cols
        return super()._map_columns(mt)

    def parse(self, text):
        return self.parser.parse(text)


class JsonToColumnsMapper(_StringToColumns):
    COL_PARAMS = ("jsonCol",)

    def _map_columns(self, mt):
        if mt.num_rows > 0:
            cols = json_columns_fast(mt.cols[self.idx], self.names, self.types, need_all=self.err)
            if cols is not None:
                return cols
        return super()._map_columns(mt)

    def parse(self, text):
        try:
            doc = lenient_json_loads(text)
        except ValueError:
            return False, [None] * len(self.names)
        out, ok = [], True
        for n, t in zip(self.names, self.types):
            try:
                o = json_path_read(doc, "$." + n)
            except (KeyError, IndexError, ValueError):
                o = None
            if o is None:
                ok = False
                out.append(None)
                continue
            s = o if isinstance(o, str) else _gson_of(o)
            good, v = parse_field(s, t)
            ok = ok and good
            out.append(v)
        return ok, out


class KvToColumnsMapper(_StringToColumns):
    COL_PARAMS = ("kvCol",)

    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        self.cd = _p(self.params, "kvColDelimiter") or _p(self.params, "colDelimiter") or ","
        self.vd = _p(self.params, "kvValDelimiter") or _p(self.params, "valDelimiter") or ":"
        self.pos = {n: i for i, n in enumerate(self.names)}

    def _map_columns(self, mt):
        if mt.num_rows > 0:
            # lines missing a key fail this parser (ERROR mode raises: the row path owns that), else NULL cells
            cols = kv_columns_fast(mt.cols[self.idx], self.names, self.types, self.cd, self.vd, need_all=self.err,
                                   allow_dup=False)
            if cols is not None:
                return cols
        return super()._map_columns(mt)

    def parse(self, text):
        out = [None] * len(self.names)
        ok, cnt = True, 0
        for f in text.split(self.cd):
            if not f.strip():
                ok = False
                continue
            kv = f.split(self.vd)
            if len(kv) < 2:
                ok = False
                continue
            i = self.pos.get(kv[0])
            if i is None:
                continue
            good, v = parse_field(kv[1], self.types[i])
            ok = ok and good
            out[i] = v
            cnt += 1
        if cnt < len(self.names):
            ok = False
        return ok, out


class JsonPathMapper(Mapper):
    """``JsonValueBatchOp`` — ``jsonPath[i]`` of the selected column into ``outputCols[i]`` (strings)."""

    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        self.idx = find_col_index(dataSchema.names, self.params.get("selectedCol"))
        self.outs = [c.strip() for c in self.params.get("outputCols")]
        self.paths = list(self.params.get("jsonPath"))
        if len(self.paths) != len(self.outs):
            raise ValueError(f"jsonPath and outputColName mismatch: {len(self.paths)} vs {len(self.outs)}")
        self.skip = bool(_p(self.params, "skipFailed", False))
        self.helper = OutputColsHelper(dataSchema, self.outs, [Types.STRING] * len(self.outs),
                                       _p(self.params, "reservedCols"))

    def _map_row_values(self, row):
        text = row[self.idx]
        if text is None or not str(text).strip():
            if self.skip:
                return [None] * len(self.paths)
            raise RuntimeError("empty json string")
        res = []
        try:
            doc = lenient_json_loads(text)
        except ValueError as e:
            if not self.skip:
                raise RuntimeError(f"Fail to getVector json path: {e}")
            return [None] * len(self.paths)
        for p in self.paths:
            try:
                o = json_path_read(doc, p)
                res.append(o if isinstance(o, str) else _gson_of(o))
            except (KeyError, IndexError, ValueError) as e:
                if not self.skip:
                    raise RuntimeError(f"Fail to getVector json path: {e}")
                res.append(None)
        return res

    def _map_columns(self, mt):
        """Plain key paths (``$.a.b``) read over the whole column in one loop: no row tuples, no per-row path
        walk set-up; the row path's values, NULLs and errors."""
        try:
            keys = [_json_path_tokens(p)[1] for p in self.paths]
        except ValueError:
            return super()._map_columns(mt)
        if not all(toks and all(k == "k" for k, _ in toks) for toks in keys):
            return super()._map_columns(mt)
        keys = [tuple(a for _, a in toks) for toks in keys]
        if mt.num_rows and all(len(ks) == 1 for ks in keys):
            out = self._top_members_native(mt, [ks[0] for ks in keys])
            if out is not None:
                return out
        texts = mt.cols[self.idx].to_list()
        n = len(texts)
        outs = [[None] * n for _ in keys]
        skip = self.skip
        for i, text in enumerate(texts):
            if text is None or not str(text).strip():
                if skip:
                    continue
                raise RuntimeError("empty json string")
            try:
                doc = lenient_json_loads(text)
            except ValueError as e:
                if not skip:
                    raise RuntimeError(f"Fail to getVector json path: {e}")
                continue
            for j, ks in enumerate(keys):
                o = doc
                for k in ks:
                    if isinstance(o, dict) and k in o:
                        o = o[k]
                    else:
                        if not skip:
                            raise RuntimeError(f"Fail to getVector json path: 'No results for path: "
                                               f"{_json_path_tokens(self.paths[j])[0]}'")
                        o = None
                        break
                else:
                    outs[j][i] = o if isinstance(o, str) else _gson_of(o)
        return [Column(o) for o in outs]

    def _top_members_native(self, mt, keys):
        """Top-level members through the C++ scanner (``_native.json_top_values``): plain strings, integer
        literals and booleans are copied as bytes, other numbers formatted by the C++ Double.toString, and only
        documents holding something else (objects, arrays, null, escapes, a missing member without skipFailed,
        a malformed document) go through ``_map_row_values``; the columns come back as ``StringBlock``s."""
        import numpy as np
        import torch
        from ... import _native as N
        from ...common.strings import StringBlock
        v = mt.cols[self.idx].values
        n = mt.num_rows
        if isinstance(v, StringBlock):
            data, off = v.data.cpu().numpy(), v.offsets.cpu().numpy()
            nm = v.nulls.cpu().numpy() if v.nulls is not None else np.zeros(n, dtype=bool)
        elif isinstance(v, list) and all(x is None or isinstance(x, str) for x in v):
            b, off = N._pack_utf8(["" if x is None else x for x in v])
            data = np.frombuffer(b, dtype=np.uint8)
            nm = np.fromiter((x is None for x in v), dtype=bool, count=n)
        else:
            return None
        r = N.json_top_values(data, off, keys)
        if r is None:
            return None
        span, kind, num, ok = r
        py = ~ok | nm | (kind == 2).any(1)
        if not self.skip:
            py |= (kind == 0).any(1)
        py_rows = np.flatnonzero(py)
        py_vals = []
        for i in py_rows.tolist():
            text = None if nm[i] else bytes(data[off[i]:off[i + 1]]).decode("utf-8")
            row = [None] * (self.idx + 1)
            row[self.idx] = text
            py_vals.append(self._map_row_values(row))
        fast = ~py
        cols = []
        for j in range(len(keys)):
            kj = kind[:, j]
            lens = np.where(fast & ((kj == 1) | (kj == 3) | (kj == 5)), span[:, j, 1] - span[:, j, 0], 0)
            src = span[:, j, 0].copy()
            nulls = fast & (kj == 0)
            parts = [data]
            base = data.size
            f = np.flatnonzero(fast & (kj == 4))
            if f.size:
                fb, fo = N.java_double_rows_packed(num[f, j].reshape(-1, 1), " ")
                lens[f] = fo[1:] - fo[:-1]
                src[f] = base + fo[:-1]
                parts.append(np.asarray(fb, dtype=np.uint8))
                base += int(fo[-1])
            if py_rows.size:
                strs = [pv[j] for pv in py_vals]
                pb, po = N._pack_utf8(["" if x is None else x for x in strs])
                lens[py_rows] = po[1:] - po[:-1]
                src[py_rows] = base + po[:-1]
                nulls[py_rows] = np.fromiter((x is None for x in strs), dtype=bool, count=len(strs))
                parts.append(np.frombuffer(pb, dtype=np.uint8))
            allb = np.concatenate(parts) if len(parts) > 1 else data
            o = np.zeros(n + 1, dtype=np.int64)
            np.cumsum(lens, out=o[1:])
            idx = np.repeat(src - o[:-1], lens) + np.arange(int(o[-1]), dtype=np.int64)
            cols.append(Column(StringBlock(torch.from_numpy(allb[idx]), torch.from_numpy(o),
                                           torch.from_numpy(nulls) if nulls.any() else None)))
        return cols
