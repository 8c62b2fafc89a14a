"""ctypes binding of the host C++ runtime (``csrc/runtime.cpp`` -> ``libalink_native.so``).

Provides bulk CSV parsing, Guava-compatible murmur3 (UTF-16) hashing and dense vector-string parsing.
Every function has a pure-Python fallback in its caller; ``lib`` is ``None`` when the library is not built.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import numpy as np

__all__ = ["lib", "parse_csv_lines", "murmur3_utf16", "murmur3_bytes", "murmur3_utf8", "parse_dense_vectors", "ftrl_update_csr",
           "ftrl_partial_margin", "ftrl_shard_update", "parse_binary_detail", "java_double_join",
           "java_double_rows", "java_double_rows_packed", "parse_csv_packed",
           "parse_dense_vectors_packed", "parse_kv_packed", "parse_json_flat_packed", "java_double_rows_fmt", "sample_thresholds", "gbdt_rank_grad",
           "tree_flatten", "java_float_rows", "java_float_rows_packed", "parse_double_csv",
           "java_float_kv_rows", "join_packed_columns", "parse_csv_spans",
           "json_top_values"]

# ALINK_NATIVE_LIB points at another build of the same sources (e.g. the AddressSanitizer build of
# tools/asan_host.py)
_PATH = os.environ.get("ALINK_NATIVE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                           "libalink_native.so")
lib = None
if os.path.exists(_PATH):
    try:
        lib = ctypes.CDLL(_PATH)
        lib.alink_csv_parse.restype = ctypes.c_int
        lib.alink_csv_parse_spans.restype = ctypes.c_int
        lib.alink_murmur3_utf16_batch.restype = None
        if hasattr(lib, "alink_murmur3_bytes_batch"):
            lib.alink_murmur3_bytes_batch.restype = None
            lib.alink_murmur3_utf8_batch.restype = None
        lib.alink_parse_dense_vectors.restype = ctypes.c_int
        lib.alink_ftrl_update_csr.restype = ctypes.c_int
        lib.alink_ftrl_partial_margin.restype = ctypes.c_int
        lib.alink_ftrl_shard_update.restype = ctypes.c_int
        lib.alink_parse_binary_detail.restype = ctypes.c_int64
        if hasattr(lib, "alink_java_double_join"):
            lib.alink_java_double_join.restype = ctypes.c_int64
        if hasattr(lib, "alink_java_double_rows"):
            lib.alink_java_double_rows.restype = ctypes.c_int64
        if hasattr(lib, "alink_java_float_rows"):
            lib.alink_java_float_rows.restype = ctypes.c_int64
        if hasattr(lib, "alink_java_float_kv_rows"):
            lib.alink_java_float_kv_rows.restype = ctypes.c_int64
        if hasattr(lib, "alink_json_top_values"):
            lib.alink_json_top_values.restype = None
        if hasattr(lib, "alink_join_packed_columns"):
            lib.alink_join_packed_columns.restype = None
        if hasattr(lib, "alink_java_double_rows_fmt"):
            lib.alink_java_double_rows_fmt.restype = ctypes.c_int64
        if hasattr(lib, "alink_sample_thresholds"):
            lib.alink_sample_thresholds.restype = ctypes.c_int64
        if hasattr(lib, "alink_binary_bins"):
            lib.alink_binary_bins.restype = None
        if hasattr(lib, "alink_kv_parse"):
            lib.alink_kv_parse.restype = ctypes.c_int64
        if hasattr(lib, "alink_json_flat_parse"):
            lib.alink_json_flat_parse.restype = ctypes.c_int64
        if hasattr(lib, "alink_gbdt_rank_grad_host"):
            lib.alink_gbdt_rank_grad_host.restype = ctypes.c_int
        if hasattr(lib, "alink_tree_flatten"):
            lib.alink_tree_scan.restype = ctypes.c_int64
            lib.alink_tree_flatten.restype = ctypes.c_int64
    except OSError:
        lib = None


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _pack_utf8(strings: Sequence[str]):
    """(bytes, int64 offsets[n+1]) of UTF-8 strings laid back to back: one join + encode when the text is ASCII
    (offsets from the character lengths), per-string encodes otherwise."""
    n = len(strings)
    off = np.zeros(n + 1, dtype=np.int64)
    text = "".join(strings)
    if text.isascii():
        if n:
            np.cumsum(np.fromiter(map(len, strings), dtype=np.int64, count=n), out=off[1:])
        return text.encode("ascii"), off
    enc = [x.encode("utf-8") for x in strings]
    if n:
        np.cumsum(np.fromiter(map(len, enc), dtype=np.int64, count=n), out=off[1:])
    return b"".join(enc), off


def parse_csv_lines(lines: Sequence[str], codes: List[int], delim: str, quote: str, skip_blank: bool):
    """Returns per column (values, nulls): numpy arrays for numeric, python lists for strings; or None."""
    if lib is None:
        return None
    if not skip_blank:
        lines = list(lines)
    else:
        lines = [l for l in lines if l]
    buf, off = _pack_utf8(lines)
    try:
        return parse_csv_packed(np.frombuffer(buf, dtype=np.uint8), off, codes, delim, quote)
    except _CsvLineError as e:
        raise RuntimeError(f'Fail to parse line "{lines[e.line]}"') from None


class _CsvLineError(RuntimeError):
    def __init__(self, line: int):
        super().__init__(f"Fail to parse line {line}")
        self.line = line


def parse_csv_packed(data: np.ndarray, off: np.ndarray, codes: List[int], delim: str, quote: str):
    """``parse_csv_lines`` over lines already packed as UTF-8 bytes (``data`` uint8, ``off`` int64 [n+1], e.g. a
    host ``StringBlock``); raises ``RuntimeError`` (with ``.line``) on the first line it cannot parse."""
    off = np.ascontiguousarray(off, dtype=np.int64)
    return parse_csv_spans(data, off[:-1], off[1:], codes, delim, quote)


def parse_csv_spans(data: np.ndarray, starts: np.ndarray, ends: np.ndarray, codes: List[int], delim: str,
                    quote: str, blocks: bool = False):
    """Lines ``data[starts[i]:ends[i]]`` of one buffer (a file read whole, row delimiters left between the spans)
    parsed in C++.  Per column (values, nulls): numpy arrays for numeric columns; for string columns a python
    list, or with ``blocks`` a (bytes, offsets [n+1], nulls) triple -- the ``StringBlock`` layout -- when no
    field of the column holds an escaped quote."""
    if lib is None:
        return None
    data = np.ascontiguousarray(data, dtype=np.uint8) if data.size else np.zeros(1, np.uint8)
    starts = np.ascontiguousarray(starts, dtype=np.int64)
    ends = np.ascontiguousarray(ends, dtype=np.int64)
    n = starts.size
    ncol = len(codes)
    nums, nulls, soffs, sescs = [], [], [], []
    num_ptrs = (ctypes.c_void_p * ncol)()
    null_ptrs = (ctypes.c_void_p * ncol)()
    soff_ptrs = (ctypes.c_void_p * ncol)()
    sesc_ptrs = (ctypes.c_void_p * ncol)()
    for c, t in enumerate(codes):
        a = np.empty(n, dtype=np.float64 if t == 1 else np.int64) if t != 0 else np.zeros(1, dtype=np.int64)
        if t != 0:
            a.fill(0)
        nl = np.empty(max(n, 1), dtype=np.uint8)
        so = np.empty(2 * max(n, 1), dtype=np.int64) if t == 0 else np.zeros(2, dtype=np.int64)
        se = np.empty(max(n, 1), dtype=np.uint8) if t == 0 else np.zeros(1, dtype=np.uint8)
        nums.append(a), nulls.append(nl), soffs.append(so), sescs.append(se)
        num_ptrs[c] = a.ctypes.data
        null_ptrs[c] = nl.ctypes.data
        soff_ptrs[c] = so.ctypes.data
        sesc_ptrs[c] = se.ctypes.data
    ct = np.asarray(codes, dtype=np.int32)
    q = ord(quote) if quote else -1
    rc = lib.alink_csv_parse_spans(_ptr(data), _ptr(starts), _ptr(ends), ctypes.c_int64(n), ctypes.c_int(ncol),
                                   _ptr(ct), ctypes.c_char(delim.encode()), ctypes.c_int(q), num_ptrs, null_ptrs,
                                   soff_ptrs, sesc_ptrs)
    if rc != 0:
        raise _CsvLineError(-1 - rc)
    out = []
    raw = None
    for c, t in enumerate(codes):
        nl = nulls[c][:n].astype(bool)
        if t == 0:
            so = soffs[c][:2 * n].reshape(n, 2)
            if blocks and not sescs[c][:n].any():
                lens = np.where(so[:, 0] < 0, 0, so[:, 1] - so[:, 0])
                o = np.zeros(n + 1, dtype=np.int64)
                np.cumsum(lens, out=o[1:])
                src = np.repeat(so[:, 0] - o[:-1], lens) + np.arange(int(o[-1]), dtype=np.int64)
                out.append(((data[src], o, so[:, 0] < 0), None))
                continue
            raw = data.tobytes() if raw is None else raw
            vals = []
            for i in range(n):
                a, b = so[i, 0], so[i, 1]
                if a < 0:
                    vals.append(None)
                else:
                    s = raw[a:b].decode("utf-8")
                    if sescs[c][i]:
                        s = s.replace(quote * 2, quote)
                    vals.append(s)
            out.append((vals, None))
        elif t == 3:
            out.append((nums[c].astype(bool), nl))
        else:
            out.append((nums[c], nl))
    return out


def murmur3_utf16(strings: Sequence[str], seed: int = 0) -> Optional[np.ndarray]:
    if lib is None:
        return None
    units = [np.frombuffer(s.encode("utf-16-le"), dtype=np.uint16) for s in strings]
    off = np.zeros(len(units) + 1, dtype=np.int64)
    if units:
        np.cumsum([len(u) for u in units], out=off[1:])
    chars = np.concatenate(units) if units else np.zeros(1, dtype=np.uint16)
    out = np.zeros(len(units), dtype=np.int32)
    lib.alink_murmur3_utf16_batch(_ptr(chars), _ptr(off), ctypes.c_int64(len(units)), ctypes.c_uint32(seed),
                                  _ptr(out))
    return out


def murmur3_bytes(data: np.ndarray, off: np.ndarray, seed: int = 0) -> Optional[np.ndarray]:
    """MurmurHash3_x86_32 of packed byte strings (uint8 ``data``, int64 ``off[n+1]``) -> int32 [n]."""
    if lib is None or not hasattr(lib, "alink_murmur3_bytes_batch"):
        return None
    data = np.ascontiguousarray(data, dtype=np.uint8) if data.size else np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.int64)
    out = np.zeros(off.size - 1, dtype=np.int32)
    lib.alink_murmur3_bytes_batch(_ptr(data), _ptr(off), ctypes.c_int64(out.size), ctypes.c_uint32(seed), _ptr(out))
    return out


def murmur3_utf8(data: np.ndarray, off: np.ndarray, prefix: str = "", seed: int = 0) -> Optional[np.ndarray]:
    """Guava ``hashUnencodedChars(prefix + s)`` of packed UTF-8 strings -> int32 [n]."""
    if lib is None or not hasattr(lib, "alink_murmur3_utf8_batch"):
        return None
    data = np.ascontiguousarray(data, dtype=np.uint8) if data.size else np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.int64)
    pu = np.frombuffer(prefix.encode("utf-16-le"), dtype=np.uint16).copy() if prefix else np.zeros(1, np.uint16)
    out = np.zeros(off.size - 1, dtype=np.int32)
    lib.alink_murmur3_utf8_batch(_ptr(data), _ptr(off), ctypes.c_int64(out.size), _ptr(pu),
                                 ctypes.c_int(len(prefix.encode("utf-16-le")) // 2), ctypes.c_uint32(seed), _ptr(out))
    return out


def java_double_join(x) -> Optional[str]:
    """``",".join(java_double_str(v) for v in x)`` for a float array, in C++ (or None without the library)."""
    if lib is None or getattr(lib, "alink_java_double_join", None) is None:
        return None
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    buf = np.empty(26 * max(a.size, 1) + 16, dtype=np.uint8)     # no zero fill
    n = lib.alink_java_double_join(_ptr(a), ctypes.c_int64(a.size), _ptr(buf))
    return buf[:n].tobytes().decode("ascii")


def java_double_rows_packed(x, sep: str = " "):
    """(uint8 bytes, int64 offsets [n+1]) of one string per row of a 2-D float array,
    ``sep.join(java_double_str(v) for v in row)`` formatted in C++ (OpenMP row blocks) and left packed, the layout
    of a ``StringBlock``; None without the library."""
    if lib is None or getattr(lib, "alink_java_double_rows", None) is None:
        return None
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    if a.ndim != 2:
        raise ValueError("java_double_rows needs a 2-D array")
    n, k = a.shape
    buf = np.empty(26 * max(a.size, 1) + 16, dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.int64)
    total = lib.alink_java_double_rows(_ptr(a), ctypes.c_int64(n), ctypes.c_int64(k), ctypes.c_char(sep.encode()),
                                       _ptr(buf), _ptr(off[1:]))
    return buf[:total], off


def java_float_rows_packed(x, sep: str = " "):
    """``java_double_rows_packed`` for a float32 array in ``java.lang.Float.toString`` form
    (``common/javafmt.java_float_str`` per value); None without the library."""
    if lib is None or getattr(lib, "alink_java_float_rows", None) is None:
        return None
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    if a.ndim != 2:
        raise ValueError("java_float_rows needs a 2-D array")
    n, k = a.shape
    buf = np.empty(26 * max(a.size, 1) + 16, dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.int64)
    total = lib.alink_java_float_rows(_ptr(a), ctypes.c_int64(n), ctypes.c_int64(k), ctypes.c_char(sep.encode()),
                                      _ptr(buf), _ptr(off[1:]))
    return buf[:total], off


def java_float_rows(x, sep: str = " ") -> Optional[List[str]]:
    """One string per row of a float32 2-D array, values in ``Float.toString`` form joined by ``sep``; None without
    the library."""
    r = java_float_rows_packed(x, sep)
    if r is None:
        return None
    data, off = r
    text = data.tobytes().decode("ascii")
    o = off.tolist()
    return [text[o[i]:o[i + 1]] for i in range(len(o) - 1)]


def java_float_kv_rows(keys, vals, kvsep: str = ":", sep: str = ",") -> Optional[List[str]]:
    """One string per row of ``key kvsep Float.toString(value)`` pairs joined by ``sep`` (int64 keys [n, k], float32
    values [n, k]), formatted in C++; None without the library."""
    if lib is None or getattr(lib, "alink_java_float_kv_rows", None) is None:
        return None
    ka = np.ascontiguousarray(np.asarray(keys, dtype=np.int64))
    va = np.ascontiguousarray(np.asarray(vals, dtype=np.float32))
    if ka.shape != va.shape or ka.ndim != 2:
        raise ValueError("java_float_kv_rows needs two 2-D arrays of one shape")
    n, k = ka.shape
    buf = np.empty(48 * max(ka.size, 1) + 16, dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.int64)
    total = lib.alink_java_float_kv_rows(_ptr(ka), _ptr(va), ctypes.c_int64(n), ctypes.c_int64(k),
                                         ctypes.c_char(kvsep.encode()), ctypes.c_char(sep.encode()), _ptr(buf),
                                         _ptr(off[1:]))
    text = buf[:total].tobytes().decode("ascii")
    o = off.tolist()
    return [text[o[i]:o[i + 1]] for i in range(n)]


def join_packed_columns(cols, delim: str, rowdelim: str) -> Optional[np.ndarray]:
    """uint8 bytes of the lines ``col0 + delim + ... + col{k-1} + rowdelim`` over k packed columns, each a
    (uint8 bytes, int64 offsets [n+1]) pair, assembled in C++; None without the library."""
    if lib is None or getattr(lib, "alink_join_packed_columns", None) is None or not cols:
        return None
    n = int(cols[0][1].size) - 1
    datas = [np.ascontiguousarray(c[0], dtype=np.uint8) if c[0].size else np.zeros(1, np.uint8) for c in cols]
    offs = [np.ascontiguousarray(c[1], dtype=np.int64) for c in cols]
    d, rd = delim.encode("utf-8"), rowdelim.encode("utf-8")
    lens = sum(o[1:] - o[:-1] for o in offs) + (len(cols) - 1) * len(d) + len(rd)
    row_off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=row_off[1:])
    out = np.empty(max(int(row_off[-1]), 1), dtype=np.uint8)
    dp = (ctypes.c_void_p * len(cols))(*[a.ctypes.data for a in datas])
    op = (ctypes.c_void_p * len(cols))(*[o.ctypes.data for o in offs])
    lib.alink_join_packed_columns(ctypes.c_int64(len(cols)), dp, op, ctypes.c_int64(n), ctypes.c_char_p(d),
                                  ctypes.c_int64(len(d)), ctypes.c_char_p(rd), ctypes.c_int64(len(rd)),
                                  _ptr(row_off), _ptr(out))
    return out[:int(row_off[-1])]


def java_double_rows_fmt(x, pre: Sequence[str], post: Sequence[str], sep: str, ropen: str = "", rclose: str = ""):
    """(uint8 bytes, int64 offsets [n+1]) of rows ``ropen + sep.join(pre[j] + Double.toString(x[i, j]) + post[j])
    + rclose`` (ASCII decorations), formatted in C++; None without the library."""
    if lib is None or getattr(lib, "alink_java_double_rows_fmt", None) is None:
        return None
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    n, k = a.shape
    pb, poff = _pack_utf8(list(pre))
    qb, qoff = _pack_utf8(list(post))
    pa = np.frombuffer(pb, dtype=np.uint8) if pb else np.zeros(1, np.uint8)
    qa = np.frombuffer(qb, dtype=np.uint8) if qb else np.zeros(1, np.uint8)
    ro, rc = ropen.encode("ascii"), rclose.encode("ascii")
    per_row = len(ro) + len(rc) + max(k - 1, 0) + int(poff[-1]) + int(qoff[-1]) + 26 * k
    buf = np.empty(per_row * max(n, 1) + 16, dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.int64)
    total = lib.alink_java_double_rows_fmt(_ptr(a), ctypes.c_int64(n), ctypes.c_int64(k), _ptr(pa), _ptr(poff),
                                           _ptr(qa), _ptr(qoff), ctypes.c_char(sep.encode()), ctypes.c_char_p(ro),
                                           ctypes.c_int64(len(ro)), ctypes.c_char_p(rc), ctypes.c_int64(len(rc)),
                                           _ptr(buf), _ptr(off[1:]))
    return buf[:total], off


def java_double_rows(x, sep: str = " ") -> Optional[List[str]]:
    """One string per row of a 2-D float array: ``sep.join(java_double_str(v) for v in row)`` (Alink's dense
    vector string), formatted in C++; None without the library."""
    r = java_double_rows_packed(x, sep)
    if r is None:
        return None
    data, off = r
    text = data.tobytes().decode("ascii")
    o = off.tolist()
    return [text[o[i]:o[i + 1]] for i in range(len(o) - 1)]


def sample_thresholds(thr, step: float, err: float) -> Optional[np.ndarray]:
    """Kept indices of the curve-threshold sampling (index 0, then each threshold at least ``step`` below the
    last kept one or within ``err`` of 0.5) as int64, scanned in C++; None without the library."""
    if lib is None or getattr(lib, "alink_sample_thresholds", None) is None:
        return None
    a = np.ascontiguousarray(np.asarray(thr, dtype=np.float64))
    keep = np.empty(max(a.size, 1), dtype=np.int64)
    m = lib.alink_sample_thresholds(_ptr(a), ctypes.c_int64(a.size), ctypes.c_double(step), ctypes.c_double(err),
                                    _ptr(keep))
    return keep[:m]


def gbdt_rank_grad(pred: np.ndarray, gain: np.ndarray, offsets: np.ndarray, disc: np.ndarray, algo: int):
    """(g, h) float32 of the GBDT learning-to-rank losses (algo 2 LambdaMART-NDCG, 3 LambdaMART-DCG, 4 GBRank)
    over contiguous queries ``offsets`` (int64 [Q+1]) — the reference's pair loop in C++ (``csrc/gbdt_rank.cpp``,
    the host twin of ``ops/csrc/gbdt_rank.hip``); None without the library."""
    if lib is None or getattr(lib, "alink_gbdt_rank_grad_host", None) is None:
        return None
    p = np.ascontiguousarray(pred, dtype=np.float32)
    y = np.ascontiguousarray(gain, dtype=np.float32)
    off = np.ascontiguousarray(offsets, dtype=np.int64)
    d = np.ascontiguousarray(disc, dtype=np.float32)
    g = np.zeros(p.size, dtype=np.float32)
    h = np.zeros(p.size, dtype=np.float32)
    rc = lib.alink_gbdt_rank_grad_host(_ptr(p), _ptr(y), _ptr(off), ctypes.c_int64(off.size - 1), _ptr(d),
                                       ctypes.c_int(algo), _ptr(g), _ptr(h))
    if rc != 0:
        raise RuntimeError(f"alink_gbdt_rank_grad_host failed: {rc}")
    return g, h


def binary_bins(probs: np.ndarray, c0: int, c1: int, code: np.ndarray, ok: Optional[np.ndarray], B: int,
                eps: float):
    """(bins int64 [2B]: positive then negative half, log loss, kept rows) of a binary detail block in one C++
    pass (``alink_binary_bins``); None without the library."""
    if lib is None or getattr(lib, "alink_binary_bins", None) is None:
        return None
    pr = np.ascontiguousarray(probs, dtype=np.float64)
    cd = np.ascontiguousarray(code, dtype=np.int64)
    okb = None if ok is None else np.ascontiguousarray(ok, dtype=np.uint8)
    bins = np.zeros(2 * B, dtype=np.int64)
    out2 = np.zeros(2, dtype=np.float64)
    lib.alink_binary_bins(_ptr(pr), ctypes.c_int64(pr.shape[0]), ctypes.c_int(pr.shape[1]), ctypes.c_int(c0),
                          ctypes.c_int(c1), _ptr(cd), None if okb is None else _ptr(okb), ctypes.c_int(B),
                          ctypes.c_double(eps), _ptr(bins), _ptr(out2))
    return bins, float(out2[0]), int(out2[1])


def parse_binary_detail(strings: Sequence[str], key0: str, key1: str):
    """(p0, p1) float64 arrays: the probabilities of labels ``key0`` / ``key1`` in two-entry detail JSON strings,
    or None (library missing, or a string outside the plain two-entry form: the caller parses it as JSON)."""
    if lib is None or getattr(lib, "alink_parse_binary_detail", None) is None:
        return None
    try:
        buf, off = _pack_utf8(strings)
    except TypeError:
        return None
    n = len(strings)
    k0, k1 = key0.encode("utf-8"), key1.encode("utf-8")
    p0 = np.zeros(n, dtype=np.float64)
    p1 = np.zeros(n, dtype=np.float64)
    bad = lib.alink_parse_binary_detail(ctypes.c_char_p(buf), _ptr(off), ctypes.c_int64(n), ctypes.c_char_p(k0),
                                        ctypes.c_int(len(k0)), ctypes.c_char_p(k1), ctypes.c_int(len(k1)), _ptr(p0),
                                        _ptr(p1))
    return None if bad != 0 else (p0, p1)


def parse_dense_vectors(strings: Sequence[str], d: int) -> Optional[np.ndarray]:
    if lib is None:
        return None
    buf, off = _pack_utf8(strings)
    return parse_dense_vectors_packed(np.frombuffer(buf, dtype=np.uint8), off, d)


def parse_dense_vectors_packed(data: np.ndarray, off: np.ndarray, d: int, with_counts: bool = False):
    """[n, d] float64 of packed dense-vector strings (plain decimal tokens split by ' ' / ','; shorter rows are
    zero-padded), or None (library missing, or a row with another token or more than ``d`` values).
    ``with_counts``: also the int64 [n] number of values of every row."""
    if lib is None:
        return None
    data = np.ascontiguousarray(data, dtype=np.uint8) if data.size else np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.int64)
    n = off.size - 1
    out = np.zeros((n, d), dtype=np.float64)
    cnt = np.zeros(max(n, 1), dtype=np.int64) if with_counts else None
    rc = lib.alink_parse_dense_vectors(_ptr(data), _ptr(off), ctypes.c_int64(n), ctypes.c_int64(d), _ptr(out),
                                       None if cnt is None else _ptr(cnt))
    if rc != 0:
        return None
    return (out, cnt[:n]) if with_counts else out


def parse_double_csv(text: str) -> Optional[np.ndarray]:
    """float64 [n] of a comma-separated list of plain decimal numbers (the inside of a JSON number array, e.g. a
    serialized coefficient vector), parsed in C++ over up to 64 comma-aligned chunks in parallel; None when the
    library is missing or a token is not a plain decimal (NaN / Infinity / anything else: the caller's JSON path)."""
    if lib is None:
        return None
    try:
        b = text.encode("ascii")
    except UnicodeEncodeError:
        return None
    n = len(b)
    if n == 0 or not b.strip():
        return np.zeros(0, dtype=np.float64)
    nch = min(64, max(1, n // 65536))
    cuts = [0]
    for c in range(1, nch):
        p = b.find(b",", c * n // nch)
        if p >= 0 and p + 1 > cuts[-1]:
            cuts.append(p + 1)
    cuts.append(n)
    per = [b.count(b",", cuts[i], cuts[i + 1]) + 1 for i in range(len(cuts) - 1)]
    res = parse_dense_vectors_packed(np.frombuffer(b, dtype=np.uint8), np.asarray(cuts, dtype=np.int64), max(per),
                                     with_counts=True)
    if res is None:
        return None
    out, cnt = res
    total = b.count(b",") + 1
    if int(cnt.sum()) != total:                 # an empty token (",,") or a stray separator: not a plain list
        return None
    return np.concatenate([out[i, :int(cnt[i])] for i in range(out.shape[0])])


def parse_kv_packed(data: np.ndarray, off: np.ndarray, keys: Sequence[str], cd: str, vd: str):
    """(values float64 [n, k], found bool [n, k], dup bool [n]) of packed KV lines for the schema ``keys``
    (single-character delimiters), or None: library missing, or a line outside the plain form (the caller parses
    the batch on its general path)."""
    if lib is None or getattr(lib, "alink_kv_parse", None) is None or len(cd) != 1 or len(vd) != 1:
        return None
    data = np.ascontiguousarray(data, dtype=np.uint8) if data.size else np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.int64)
    n, k = off.size - 1, len(keys)
    kb, koff = _pack_utf8(list(keys))
    kb = np.frombuffer(kb, dtype=np.uint8) if kb else np.zeros(1, np.uint8)
    out = np.empty((n, max(k, 1)), dtype=np.float64)
    found = np.empty((n, max(k, 1)), dtype=np.uint8)
    flags = np.empty(max(n, 1), dtype=np.uint8)
    bad = lib.alink_kv_parse(_ptr(data), _ptr(off), ctypes.c_int64(n), ctypes.c_char(cd.encode()),
                             ctypes.c_char(vd.encode()), _ptr(kb), _ptr(koff), ctypes.c_int64(k), _ptr(out),
                             _ptr(found), _ptr(flags))
    if bad:
        return None
    return out[:, :k], found[:, :k].astype(bool), (flags[:n] & 2).astype(bool)


def parse_json_flat_packed(data: np.ndarray, off: np.ndarray, keys: Sequence[str]):
    """(values float64 [n, k], found bool [n, k]) of packed flat JSON objects with numeric members for the schema
    ``keys``, or None (library missing, or a line outside that form: the caller parses with the JSON reader)."""
    if lib is None or getattr(lib, "alink_json_flat_parse", None) is None:
        return None
    data = np.ascontiguousarray(data, dtype=np.uint8) if data.size else np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.int64)
    n, k = off.size - 1, len(keys)
    kb, koff = _pack_utf8(list(keys))
    kb = np.frombuffer(kb, dtype=np.uint8) if kb else np.zeros(1, np.uint8)
    out = np.empty((n, max(k, 1)), dtype=np.float64)
    found = np.empty((n, max(k, 1)), dtype=np.uint8)
    flags = np.empty(max(n, 1), dtype=np.uint8)
    bad = lib.alink_json_flat_parse(_ptr(data), _ptr(off), ctypes.c_int64(n), _ptr(kb), _ptr(koff),
                                    ctypes.c_int64(k), _ptr(out), _ptr(found), _ptr(flags))
    if bad:
        return None
    return out[:, :k], found[:, :k].astype(bool)


def ftrl_update_csr(indptr, indices, values, label, w, n, z, alpha, beta, l1, l2, scale=1.0) -> bool:
    """Sequential FTRL-proximal over CSR rows (in place on ``w, n, z``); False when the library is missing."""
    if lib is None:
        return False
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    values = np.ascontiguousarray(values, dtype=np.float64)
    label = np.ascontiguousarray(label, dtype=np.float64)
    for a in (w, n, z):
        assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    rc = lib.alink_ftrl_update_csr(_ptr(indptr), _ptr(indices), _ptr(values), _ptr(label),
                                   ctypes.c_int64(len(indptr) - 1), _ptr(w), _ptr(n), _ptr(z),
                                   ctypes.c_int64(len(w)), ctypes.c_double(alpha), ctypes.c_double(beta),
                                   ctypes.c_double(l1), ctypes.c_double(l2), ctypes.c_double(scale))
    if rc != 0:
        raise ValueError("feature index out of range in FTRL update")
    return True


def _csr(indptr, indices, values):
    return (np.ascontiguousarray(indptr, dtype=np.int64), np.ascontiguousarray(indices, dtype=np.int32),
            np.ascontiguousarray(values, dtype=np.float64))


def ftrl_partial_margin(indptr, indices, values, w, lo, hi) -> np.ndarray:
    """Per-row margin restricted to coordinates [lo, hi) (``w`` is that shard)."""
    indptr, indices, values = _csr(indptr, indices, values)
    nrows = len(indptr) - 1
    out = np.zeros(nrows, dtype=np.float64)
    if lib is None:
        for r in range(nrows):
            s, e = indptr[r], indptr[r + 1]
            ii = indices[s:e].astype(np.int64)
            m = (ii >= lo) & (ii < hi)
            out[r] = float(np.dot(values[s:e][m], w[ii[m] - lo]))
        return out
    w = np.ascontiguousarray(w, dtype=np.float64)
    lib.alink_ftrl_partial_margin(_ptr(indptr), _ptr(indices), _ptr(values), ctypes.c_int64(nrows), _ptr(w),
                                  ctypes.c_int64(lo), ctypes.c_int64(hi), _ptr(out))
    return out


def ftrl_shard_update(indptr, indices, values, err, w, n, z, lo, hi, alpha, beta, l1, l2) -> None:
    """In-place FTRL on the owned shard [lo, hi) with per-row ``err = p - y`` fixed for the micro-batch."""
    indptr, indices, values = _csr(indptr, indices, values)
    err = np.ascontiguousarray(err, dtype=np.float64)
    for a in (w, n, z):
        assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    if lib is None:
        for r in range(len(indptr) - 1):
            for k in range(indptr[r], indptr[r + 1]):
                i = int(indices[k]) - lo
                if i < 0 or i >= hi - lo:
                    continue
                g = err[r] * values[k]
                nn = n[i] + g * g
                sigma = (np.sqrt(nn) - np.sqrt(n[i])) / alpha
                z[i] += g - sigma * w[i]
                n[i] = nn
                w[i] = 0.0 if abs(z[i]) <= l1 else (np.sign(z[i]) * l1 - z[i]) / (beta + np.sqrt(n[i]) / alpha + l2)
        return
    lib.alink_ftrl_shard_update(_ptr(indptr), _ptr(indices), _ptr(values), _ptr(err),
                                ctypes.c_int64(len(indptr) - 1), _ptr(w), _ptr(n), _ptr(z), ctypes.c_int64(lo),
                                ctypes.c_int64(hi), ctypes.c_double(alpha), ctypes.c_double(beta),
                                ctypes.c_double(l1), ctypes.c_double(l2))


def tree_flatten(strings: Sequence[str], tree_lo: Sequence[int]):
    """Tree-model node strings (``TreeModelDataConverter`` rows; tree t = strings[tree_lo[t]:tree_lo[t+1]]) parsed
    straight into flat arrays by ``csrc/tree_model.cpp``: dict of feat / thr / first / nchild / wsum / dist
    [n, max_dist] / dist_len / cat_len / cat_off / cat (int32 values), or None (library missing, or a row outside
    the serializer's form -- the caller takes the generic JSON path)."""
    if lib is None or getattr(lib, "alink_tree_flatten", None) is None:
        return None
    data, off = _pack_utf8(strings)
    buf = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, np.uint8)
    n = len(strings)
    lo = np.ascontiguousarray(tree_lo, dtype=np.int64)
    nd, ncat = 4, 1024          # first guess (GBDT leaves hold 1 value, classifiers one per label)
    md, ct = ctypes.c_int64(0), ctypes.c_int64(0)
    for _ in range(2):
        out = {"feat": np.empty(n, np.int32), "thr": np.empty(n, np.float64), "first": np.empty(n, np.int32),
               "nchild": np.empty(n, np.int32), "wsum": np.empty(n, np.float64),
               "dist": np.empty((n, nd), np.float64), "dist_len": np.empty(n, np.int32),
               "cat_len": np.empty(n, np.int32), "cat_off": np.empty(n, np.int64), "cat": np.empty(ncat, np.int32)}
        rc = lib.alink_tree_flatten(_ptr(buf), _ptr(off), ctypes.c_int64(n), _ptr(lo), ctypes.c_int64(len(lo) - 1),
                                    ctypes.c_int64(nd), _ptr(out["feat"]), _ptr(out["thr"]), _ptr(out["first"]),
                                    _ptr(out["nchild"]), _ptr(out["wsum"]), _ptr(out["dist"]),
                                    _ptr(out["dist_len"]), _ptr(out["cat_len"]), _ptr(out["cat_off"]),
                                    _ptr(out["cat"]), ctypes.c_int64(ncat), ctypes.byref(md), ctypes.byref(ct))
        if rc != -2:
            break
        nd, ncat = max(1, int(md.value)), max(1, int(ct.value))
    if rc != 0:
        return None
    out["dist"] = out["dist"][:, :max(1, int(md.value))]
    out["max_dist"] = int(md.value)
    return out


def json_top_values(data: np.ndarray, off: np.ndarray, keys: Sequence[str]):
    """Top-level members ``keys`` of packed JSON objects scanned in C++: (span int64 [n, k, 2] absolute byte
    offsets, kind uint8 [n, k], num float64 [n, k], row_ok bool [n]) -- kinds as ``alink_json_top_values``
    documents; None without the library."""
    if lib is None or getattr(lib, "alink_json_top_values", None) is None:
        return None
    data = np.ascontiguousarray(data, dtype=np.uint8) if data.size else np.zeros(1, np.uint8)
    off = np.ascontiguousarray(off, dtype=np.int64)
    n, k = off.size - 1, len(keys)
    kb, koff = _pack_utf8(list(keys))
    kb = np.frombuffer(kb, dtype=np.uint8) if kb else np.zeros(1, np.uint8)
    span = np.zeros((max(n, 1), k, 2), dtype=np.int64)
    kind = np.zeros((max(n, 1), k), dtype=np.uint8)
    num = np.zeros((max(n, 1), k), dtype=np.float64)
    ok = np.zeros(max(n, 1), dtype=np.uint8)
    lib.alink_json_top_values(_ptr(data), _ptr(off), ctypes.c_int64(n), _ptr(kb), _ptr(koff), ctypes.c_int64(k),
                              _ptr(span), _ptr(kind), _ptr(num), _ptr(ok))
    return span[:n], kind[:n], num[:n], ok[:n].astype(bool)
