"""Categorical / discretisation encoders: StringIndexer, MultiStringIndexer, IndexToString, OneHotEncoder,
QuantileDiscretizer, Bucketizer, Binarizer, FeatureHasher, DCT.

Reference: ``A/operator/common/dataproc/{StringIndexer*,MultiStringIndexer*,IndexToStringModelMapper,
StringIndexerUtil}.java``, ``A/operator/common/feature/{OneHotModelMapper,QuantileDiscretizerModelMapper,
BucketizerMapper,BinarizerMapper,FeatureHasherMapper,DCTMapper}.java``, ``A/operator/batch/feature/
QuantileDiscretizerTrainBatchOp.java`` (QIndex: ``round(q * (n-1) * k)``).

Token dictionaries are built from per-rank counts merged with one all-gather; numeric bucketing is a
vectorised ``searchsorted`` over the whole column (device tensors when available); FeatureHasher uses the
native Guava-compatible murmur3 (``_native.murmur3_utf16``) over all cells at once.
"""
from __future__ import annotations

import json
import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...common.javafmt import java_str
from ...common.linalg import DenseVector, SparseVector, VectorUtil
from ...common.mapper import Mapper, ModelMapper, OutputColsHelper, SISOMapper
from ...common.params import Params
from ...common.table import Column, MTable, Row
from ...common.types import TableSchema, Types, is_numeric
from ...parallel import comm

__all__ = ["train_string_indexer", "StringIndexerModelMapper", "train_multi_string_indexer",
           "MultiStringIndexerModelMapper", "IndexToStringModelMapper", "train_one_hot", "OneHotModelMapper",
           "train_quantile_discretizer", "QuantileDiscretizerModelMapper", "BucketizerMapper", "BinarizerMapper",
           "FeatureHasherMapper", "DCTMapper", "murmur3_index", "STRING_INDEXER_SCHEMA", "MULTI_INDEXER_SCHEMA"]

STRING_INDEXER_SCHEMA = TableSchema(["token", "token_index"], [Types.STRING, Types.LONG])
MULTI_INDEXER_SCHEMA = TableSchema(["column_index", "token", "token_index"], [Types.LONG, Types.STRING, Types.LONG])


def _pget(p, name, default=None):
    try:
        return p.get(name) if p.contains(name) and p.get(name) is not None else default
    except KeyError:
        return default


def _ename(v, default):
    if v is None:
        return default
    return getattr(v, "name", str(v)).upper()


# ---------------------------------------------------------------------------------------------------
# token dictionaries
# ---------------------------------------------------------------------------------------------------
def _column_token_counts(col) -> Dict[str, int]:
    """Token (``String.valueOf``) -> count of one column without a per-cell Python loop: numeric / boolean tensor
    columns count distinct values with ``torch.unique`` (formatting each distinct value once), string columns
    go through ``collections.Counter`` (C) over the values."""
    from collections import Counter
    v = col.values
    enc = _block_codes(col)
    if enc is not None:        # packed strings: counts of the distinct tokens from one device encoding
        _, words, _, cnt = enc
        return {w: int(c) for w, c in zip(words, cnt.tolist()) if c > 0}
    if isinstance(v, torch.Tensor) and v.dim() == 1:
        x = v if col.nulls is None else v[~col.nulls.to(v.device)]
        if x.numel() == 0:
            return {}
        x = x.detach().cpu()
        out: Dict[str, int] = {}
        if x.dtype.is_floating_point:
            # torch.unique merges -0.0 into 0.0 (and splits NaNs): String.valueOf keeps "-0.0" apart, NaN as one
            negz = (x == 0) & torch.signbit(x)
            nz = int(negz.sum())
            if nz:
                out["-0.0"] = nz
                x = x[~negz]
        uniq, cnt = torch.unique(x, return_counts=True)
        for u, c in zip(uniq.tolist(), cnt.tolist()):
            k = java_str(u)
            out[k] = out.get(k, 0) + int(c)
        return out
    vals = col.to_list()
    if all(x is None or isinstance(x, str) for x in vals):
        cnt = Counter(vals)
        cnt.pop(None, None)
        return dict(cnt)
    cnt = Counter(java_str(x) for x in vals if x is not None)
    return dict(cnt)


def _block_codes(col):
    """Device dictionary encoding of a packed string column (``ops/strings.unique_ids``): (ids int64 [n] on the
    column's device, distinct strings [u] -- "" for an id shared only by empty strings and nulls, None for an id of
    nulls only --, null mask bool [n] or None, per-id count of non-null rows int64 [u]), or None for another column
    type or a hash collision (the caller's per-value path)."""
    from ...common.strings import StringBlock
    v = col.values
    if not isinstance(v, StringBlock) or len(v) == 0:
        return None
    from ...ops.strings import unique_ids
    enc = unique_ids(v)
    if enc is None:
        return None
    ids, rep = enc
    nm = v.nulls
    if col.nulls is not None:
        cn = col.nulls.to(ids.device)
        nm = cn if nm is None else (nm.to(ids.device) | cn)
    u = int(rep.numel())
    live = ids if nm is None else ids[~nm]
    cnt = torch.bincount(live, minlength=u).cpu().numpy()
    words = v.take(rep).to_list()
    words = [("" if (w is None and cnt[i] > 0) else w) for i, w in enumerate(words)]
    return ids, words, nm, cnt


def _global_token_counts(mt: MTable, cols: Sequence[str]) -> List[Dict[str, int]]:
    local = [_column_token_counts(mt.col(c)) for c in cols]
    merged = [dict() for _ in cols]
    for part in comm.all_gather_object(local):
        for i, d in enumerate(part):
            for k, v in d.items():
                merged[i][k] = merged[i].get(k, 0) + v
    return merged


def _order_tokens(counts: Dict[str, int], order: str, seed: int = 0) -> List[str]:
    toks = list(counts)
    if order == "RANDOM":
        rng = np.random.default_rng(seed)
        toks = sorted(toks)
        rng.shuffle(toks)
        return toks
    if order == "FREQUENCY_ASC":
        return sorted(toks, key=lambda t: (counts[t], t))
    if order == "FREQUENCY_DESC":
        return sorted(toks, key=lambda t: (-counts[t], t))
    if order == "ALPHABET_ASC":
        return sorted(toks)
    if order == "ALPHABET_DESC":
        return sorted(toks, reverse=True)
    raise ValueError(f"unknown stringOrderType {order}")


def train_string_indexer(mt: MTable, params: Params) -> MTable:
    col = params.get("selectedCol")
    extra = list(_pget(params, "selectedCols") or [])
    order = _ename(_pget(params, "stringOrderType"), "RANDOM")
    counts = _global_token_counts(mt, [col] + extra)
    merged: Dict[str, int] = {}
    for d in counts:
        for k, v in d.items():
            merged[k] = merged.get(k, 0) + v
    toks = _order_tokens(merged, order)
    return MTable.from_rows([(t, i) for i, t in enumerate(toks)], STRING_INDEXER_SCHEMA, replicated=True)


class _SISOModelMapper(ModelMapper):
    """One input column -> one output column, model-based (``SISOModelMapper``)."""

    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        p = self.params
        self.selected = _pget(p, "selectedCol")
        out = _pget(p, "outputCol") or self.selected
        from ...common.mapper import find_col_index
        self.col_idx = find_col_index(dataSchema.names, self.selected)
        self.helper = OutputColsHelper(dataSchema, [out], [self.outputType()], _pget(p, "reservedCols"))

    def outputType(self):
        return Types.STRING

    def mapColumn(self, v):
        raise NotImplementedError

    def _map_row_values(self, row):
        return [self.mapColumn(row[self.col_idx])]


class StringIndexerModelMapper(_SISOModelMapper):
    """token -> index; unseen: KEEP -> max+1, SKIP -> null, ERROR -> raise."""

    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        self.invalid = _ename(_pget(self.params, "handleInvalid"), "KEEP")

    def outputType(self):
        return Types.LONG

    def loadModel(self, rows):
        self.map_ = {str(r[0]): int(r[1]) for r in rows}
        self.default = max(self.map_.values(), default=-1) + 1

    def mapColumn(self, v):
        key = None if v is None else java_str(v)
        if key in self.map_:
            return self.map_[key]
        if self.invalid == "KEEP":
            return self.default
        if self.invalid == "SKIP":
            return None
        raise RuntimeError(f"Unseen token: {key}")

    def _map_columns(self, mt):
        """A packed string column maps through its device dictionary encoding: every DISTINCT token is looked up
        once (mapColumn's rules, nulls included) and the rows gather their id's result on the device."""
        col = mt.col(self.selected)
        enc = _block_codes(col)
        if enc is None:
            return super()._map_columns(mt)
        ids, words, nm, cnt = enc
        u = len(words)
        lut = np.zeros(u + 1, dtype=np.int64)
        lut_null = np.zeros(u + 1, dtype=bool)
        for i, w in enumerate(words + [None]):          # slot u: the null rows
            if i < u and cnt[i] == 0:
                continue                                # an id of null rows only: they use slot u
            r = self.mapColumn(w)
            if r is None:
                lut_null[i] = True
            else:
                lut[i] = r
        dev = ids.device
        if nm is not None:
            if bool(nm.any()):
                self.mapColumn(None)                    # ERROR on a null raises as the row path does
            ids = torch.where(nm, torch.full_like(ids, u), ids)
        out = torch.from_numpy(lut).to(dev)[ids]
        null = torch.from_numpy(lut_null).to(dev)[ids]
        return [Column(out.cpu(), null.cpu() if bool(null.any()) else None)]


class IndexToStringModelMapper(_SISOModelMapper):
    def outputType(self):
        return Types.STRING

    def loadModel(self, rows):
        self.map_ = {int(r[1]): r[0] for r in rows}

    def mapColumn(self, v):
        return None if v is None else self.map_.get(int(v))

    def _map_columns(self, mt):
        """An integer tensor column: each DISTINCT index looked up once, the rows take their string from a
        packed block of the results (unknown index -> NULL, as ``map_.get``)."""
        from ...common.strings import StringBlock
        col = mt.cols[self.col_idx]
        v = col.values
        if not (isinstance(v, torch.Tensor) and v.dim() == 1 and not v.is_floating_point() and v.dtype != torch.bool
                and mt.num_rows):
            return super()._map_columns(mt)
        uniq, inv = torch.unique(v.cpu(), return_inverse=True)
        words = [self.map_.get(int(u)) for u in uniq.tolist()]
        if not all(w is None or isinstance(w, str) for w in words):
            return super()._map_columns(mt)
        blk = StringBlock.from_list(words).take(inv)
        nm = blk.nulls
        if col.nulls is not None:
            cn = col.nulls.cpu()
            nm = cn if nm is None else (nm.cpu() | cn)
        if nm is not None and bool(nm.any()):
            keep = ~nm
            lens = (blk.offsets[1:] - blk.offsets[:-1]) * keep
            data = blk.data[torch.repeat_interleave(keep, blk.offsets[1:] - blk.offsets[:-1])]
            off = torch.zeros(len(lens) + 1, dtype=torch.int64)
            torch.cumsum(lens, 0, out=off[1:])
            blk = StringBlock(data, off, nm)
        return [Column(blk)]


def train_multi_string_indexer(mt: MTable, params: Params, meta_extra: Optional[Params] = None) -> MTable:
    cols = list(params.get("selectedCols"))
    order = _ename(_pget(params, "stringOrderType"), "RANDOM")
    counts = _global_token_counts(mt, cols)
    meta = Params().set("selectedCols", cols)
    if meta_extra is not None:
        meta.merge(meta_extra)
    rows = [(-1, meta.toJson(), None)]
    for i, d in enumerate(counts):
        for j, t in enumerate(_order_tokens(d, order)):
            rows.append((i, t, j))
    return MTable.from_rows(rows, MULTI_INDEXER_SCHEMA, replicated=True)


def _load_multi(rows):
    meta, maps = Params(), {}
    for r in rows:
        ci = int(r[0])
        if ci < 0:
            meta = Params.fromJson(r[1])
        else:
            maps.setdefault(ci, {})[r[1]] = int(r[2])
    return meta, maps


class MultiStringIndexerModelMapper(ModelMapper):
    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        self.invalid = _ename(_pget(self.params, "handleInvalid"), "KEEP")

    def loadModel(self, rows):
        self.meta, maps = _load_multi(rows)
        train_cols = list(self.meta.get("selectedCols"))
        self.cols = list(_pget(self.params, "selectedCols") or train_cols)
        self.maps = [maps.get(train_cols.index(c), {}) for c in self.cols]
        out = _pget(self.params, "outputCols") or self.cols
        self.helper = OutputColsHelper(self.dataSchema, list(out), [Types.LONG] * len(out),
                                       _pget(self.params, "reservedCols"))

    def _map_row_values(self, row):
        out = []
        for c, m in zip(self.cols, self.maps):
            v = row[self.dataSchema.names.index(c)]
            key = None if v is None else java_str(v)
            if key in m:
                out.append(m[key])
            elif self.invalid == "KEEP":
                out.append(len(m))
            elif self.invalid == "SKIP":
                out.append(None)
            else:
                raise RuntimeError(f"Unseen token: {key}")
        return out

    def _index_one(self, m, v):
        key = None if v is None else java_str(v)
        if key in m:
            return m[key]
        if self.invalid == "KEEP":
            return len(m)
        if self.invalid == "SKIP":
            return None
        raise RuntimeError(f"Unseen token: {key}")

    def _map_columns(self, mt):
        """Packed string columns through their device dictionary encodings: each DISTINCT token (and NULL, when
        present) looked up once with the row path's rules, the rows gather their id's index."""
        encs = [_block_codes(mt.col(c)) for c in self.cols]
        if any(e is None for e in encs):
            return super()._map_columns(mt)
        out = []
        for m, (ids, words, nm, cnt) in zip(self.maps, encs):
            u = len(words)
            lut = np.zeros(u + 1, dtype=np.int64)
            lut_null = np.zeros(u + 1, dtype=bool)
            has_null = nm is not None and bool(nm.any())
            for i, w in enumerate(words + [None]):
                if (i < u and cnt[i] == 0) or (i == u and not has_null):
                    continue
                r = self._index_one(m, w)
                if r is None:
                    lut_null[i] = True
                else:
                    lut[i] = r
            if has_null:
                ids = torch.where(nm, torch.full_like(ids, u), ids)
            dev = ids.device
            o = torch.from_numpy(lut).to(dev)[ids]
            null = torch.from_numpy(lut_null).to(dev)[ids]
            out.append(Column(o.cpu(), null.cpu() if bool(null.any()) else None))
        return out


# ---------------------------------------------------------------------------------------------------
# discretizer output encoding (QuantileDiscretizerModelMapper.setResultRow)
# ---------------------------------------------------------------------------------------------------
class _EncodeSpec:
    def __init__(self, params: Params, data_schema: TableSchema, default_encode: str, cols: Optional[List[str]]):
        self.encode = _ename(_pget(params, "encode"), default_encode)
        self.invalid = _ename(_pget(params, "handleInvalid"), "KEEP")
        self.drop_last = bool(_pget(params, "dropLast", True))
        self.cols = list(_pget(params, "selectedCols") or cols or [])
        out = _pget(params, "outputCols")
        if out is None and _pget(params, "outputCol") is not None:
            out = [params.get("outputCol")]
        reserved = _pget(params, "reservedCols")
        if self.encode == "INDEX":
            out = list(out or self.cols)
            self.helper = OutputColsHelper(data_schema, out, [Types.LONG] * len(out), reserved)
        elif self.encode == "VECTOR":
            out = list(out or self.cols)
            self.helper = OutputColsHelper(data_schema, out, [Types.SPARSE_VECTOR] * len(out), reserved)
        elif self.encode == "ASSEMBLED_VECTOR":
            if not out or len(out) != 1:
                raise ValueError("When encode is ASSEMBLED_VECTOR, outputCols must be given and the length must be 1!")
            self.helper = OutputColsHelper(data_schema, list(out), [Types.SPARSE_VECTOR], reserved)
        else:
            raise ValueError(f"Not support encode: {self.encode}")
        self.vector_size: List[int] = []
        self.drop_index: List[Optional[int]] = []

    def assembled_size(self):
        s = sum(self.vector_size)
        return s - len(self.vector_size) if self.drop_last else s

    def _size_index(self, i, idx):
        vs = self.vector_size[i]
        if self.drop_last:
            d = self.drop_index[i]
            if idx == d:
                return vs - 1, None
            return vs - 1, (idx - 1 if d is not None and idx > d else idx)
        return vs, idx

    def columns(self, idx: np.ndarray, valid: np.ndarray) -> List[Column]:
        """idx [n, cols] int64 bucket indices; valid False -> null (SKIP)."""
        n, k = idx.shape
        if self.encode == "INDEX":
            # columnar: int64 values (0 under a null, as Column.from_values fills) + a null mask when any is null
            out = []
            for j in range(k):
                ok = valid[:, j]
                v = np.where(ok, idx[:, j], 0).astype(np.int64)
                out.append(Column(torch.from_numpy(v), None if ok.all() else torch.from_numpy(~ok)))
            return out
        if self.encode == "VECTOR":
            out = []
            for j in range(k):
                col = []
                for r in range(n):
                    if not valid[r, j]:
                        col.append(None)
                        continue
                    size, ii = self._size_index(j, int(idx[r, j]))
                    col.append(SparseVector(size) if ii is None else SparseVector(size, [ii], [1.0]))
                out.append(Column(col))
            return out
        # ASSEMBLED_VECTOR: global index = column offset + (drop-last adjusted) bucket, on the env's device
        from ...ops.feature import csr_assemble
        total = self.assembled_size()
        gidx = np.zeros((k, n), dtype=np.int64)
        keep = np.zeros((k, n), dtype=bool)
        start = 0
        for j in range(k):
            b = idx[:, j]
            vs = self.vector_size[j]
            if self.drop_last:
                d = self.drop_index[j]
                size = vs - 1
                keep[j] = b != d if d is not None else True
                gidx[j] = start + (np.where(b > d, b - 1, b) if d is not None else b)
            else:
                size = vs
                keep[j] = True
                gidx[j] = start + b
            start += size
        row_ok = valid.all(1)
        keep &= row_ok[None, :]
        dev = feature_device()
        blk = csr_assemble(torch.from_numpy(gidx).to(dev), None, torch.from_numpy(keep).to(dev), total)
        return [Column(blk, None if row_ok.all() else torch.from_numpy(~row_ok))]


# ---------------------------------------------------------------------------------------------------
# OneHot
# ---------------------------------------------------------------------------------------------------
def train_one_hot(mt: MTable, params: Params) -> MTable:
    cols = list(params.get("selectedCols"))
    p = params.clone()
    p.set("stringOrderType", "ALPHABET_ASC") if not p.contains("stringOrderType") else None
    thr = _pget(params, "discreteThresholds")
    thr_arr = _pget(params, "discreteThresholdsArray")
    enable_else = thr is not None or thr_arr is not None
    counts = _global_token_counts(mt, cols)
    meta = Params().set("selectedCols", cols).set("enableElse", bool(enable_else))
    rows = [(-1, meta.toJson(), None)]
    for i, d in enumerate(counts):
        limit = (thr_arr[i] if thr_arr is not None else thr) if enable_else else None
        toks = sorted(t for t in d if limit is None or d[t] >= limit)
        for j, t in enumerate(toks):
            rows.append((i, t, j))
    return MTable.from_rows(rows, MULTI_INDEXER_SCHEMA, replicated=True)


class OneHotModelMapper(ModelMapper):
    """Token -> one-hot index with the reference's invalid/else strategies
    (``OneHotModelMapper.InvalidStrategy``): KEEP reserves the last slot(s), enableElse adds an 'else' slot."""

    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)

    def loadModel(self, rows):
        self.meta, maps = _load_multi(rows)
        train_cols = list(self.meta.get("selectedCols"))
        self.spec = _EncodeSpec(self.params, self.dataSchema, "ASSEMBLED_VECTOR", train_cols)
        self.cols = self.spec.cols
        self.maps = [maps.get(train_cols.index(c), {}) for c in self.cols]
        self.enable_else = bool(self.meta.get("enableElse")) if self.meta.contains("enableElse") else False
        self.helper = self.spec.helper
        for m in self.maps:
            max_idx = len(set(m.values())) - 1
            add = {("KEEP", True): 3, ("SKIP", True): 2, ("ERROR", True): 2,
                   ("KEEP", False): 2, ("SKIP", False): 1, ("ERROR", False): 1}[(self.spec.invalid, self.enable_else)]
            self.spec.vector_size.append(max_idx + add)
            self.spec.drop_index.append(0 if self.spec.drop_last else None)

    def _map_columns(self, mt):
        """Token lookup per distinct value (pandas factorize: one dict probe per unique token, then a vectorised
        gather), invalid/else strategies on whole arrays; the assembled vector is built on the env's device by
        the CSR assembler (``ops/csrc/feature.hip``)."""
        import pandas as pd
        n, k = mt.num_rows, len(self.cols)
        idx = np.zeros((n, k), dtype=np.int64)
        valid = np.ones((n, k), dtype=bool)
        inv, ee = self.spec.invalid, self.enable_else
        for j, (c, m) in enumerate(zip(self.cols, self.maps)):
            vs = self.spec.vector_size[j]
            enc = _block_codes(mt.col(c))
            if enc is not None:         # packed strings: the device dictionary encoding, no Python list of rows
                ids, uniq, nm, _ = enc
                codes = ids.cpu().numpy()
                if nm is not None:
                    codes = np.where(nm.cpu().numpy(), -1, codes)
            else:
                vals = mt.col(c).to_list()
                codes, uniq = pd.factorize(pd.Series(vals, dtype=object), use_na_sentinel=True)
            look = np.asarray([m.get(java_str(u), -1) if u is not None else -1 for u in uniq], dtype=np.int64)
            got = np.where(codes >= 0, look[np.maximum(codes, 0)] if look.size else -1, -1)
            is_null = codes < 0
            unseen = (got < 0) & ~is_null
            idx[:, j] = np.maximum(got, 0)
            if ee and inv == "KEEP":
                idx[is_null, j] = vs - 2
                idx[unseen, j] = vs - 1
            elif ee:
                if is_null.any():
                    if inv != "SKIP":
                        raise RuntimeError("Input is null!")
                    valid[is_null, j] = False
                idx[unseen, j] = vs - 1
            elif inv == "KEEP":
                idx[is_null | unseen, j] = vs - 1
            elif inv == "SKIP":
                valid[is_null | unseen, j] = False
            elif (is_null | unseen).any():
                i0 = int(np.nonzero(is_null | unseen)[0][0])
                bad = None if codes[i0] < 0 else uniq[int(codes[i0])]
                raise RuntimeError(f"Unseen token: {bad}")
        return self.spec.columns(idx, valid)


# ---------------------------------------------------------------------------------------------------
# numeric bucketing
# ---------------------------------------------------------------------------------------------------
QUANTILE_SCHEMA = TableSchema(["model_id", "model_info"], [Types.LONG, Types.STRING])


def _round(x: float, mode: str) -> int:
    if mode == "CEIL":
        return int(math.ceil(x))
    if mode == "FLOOR":
        return int(math.floor(x))
    return int(math.floor(x + 0.5))


def train_quantile_discretizer(mt: MTable, params: Params) -> MTable:
    """Exact distributed quantiles (reference ``QuantileDiscretizerTrainBatchOp.java:181``, ``SortUtilsNext.pSort``):
    each column's non-missing values stay on their rank as a device tensor; the split values are the order
    statistics at global positions round(q * (n-1) * j) (``QIndex.genIndex``), de-duplicated, found by
    ``parallel/sort.global_order_statistics`` — a device sort on one rank, the distributed sample sort plus a
    count prefix on several; no rank ever holds another rank's values."""
    from ...parallel.sort import global_order_statistics
    from ..tree.data import numeric_column
    from ...common.model.converter import SimpleModelDataConverter, append_meta_rows, append_data_rows
    cols = list(params.get("selectedCols"))
    nb = _pget(params, "numBuckets")
    nba = _pget(params, "numBucketsArray")
    nums = list(nba) if nba is not None else [int(nb if nb is not None else 2)] * len(cols)
    mode = _ename(_pget(params, "roundMode"), "ROUND")
    left_open = bool(_pget(params, "leftOpen", True))
    borders = {}
    dev = _device_of(mt)
    for c, q in zip(cols, nums):
        x, null = numeric_column(mt, c, dev)
        x = x[~(null | torch.isnan(x))]
        n, vals = global_order_statistics(
            x, lambda n: [min(n - 1, _round(1.0 / q * (n - 1.0) * j, mode)) for j in range(1, q)] if n else [])
        splits = sorted(set(float(v) for v in vals)) if n else []
        ctype = "LONG" if mt.col_type(c) in (Types.LONG, Types.INT, Types.SHORT, Types.BYTE) else "DOUBLE"
        borders[c] = {"featureName": c, "splitsArray": splits, "isLeftOpen": left_open, "colType": ctype}
    meta = Params().set("selectedCols", cols).set("leftOpen", left_open)
    rows = []
    append_meta_rows(meta, rows, 2)
    append_data_rows([json.dumps(borders[c], separators=(",", ":")) for c in cols], rows, 2)
    return MTable.from_rows(rows, QUANTILE_SCHEMA, replicated=True)


def _device_of(mt: MTable):
    for c in mt.cols:
        if isinstance(c.values, torch.Tensor) and c.values.is_cuda:
            return c.values.device
    return torch.device("cpu")


class _Bucketing:
    """bounds [-inf, s_0, ..., s_{m-1}, +inf]; bucket = searchsorted (left-open: (a, b])."""

    def __init__(self, splits: Sequence[float], left_open: bool):
        self.bounds = np.concatenate([[-np.inf], np.asarray(sorted(splits), dtype=np.float64), [np.inf]])
        self.left_open = left_open
        self.nbins = len(splits) + 1
        self.null_index = self.nbins

    def find(self, v: np.ndarray, null: np.ndarray) -> np.ndarray:
        side = "left" if self.left_open else "right"
        hit = np.searchsorted(self.bounds, v, side=side) - 1
        hit = np.clip(hit, 0, self.nbins - 1)
        return np.where(null, self.null_index, hit)


def _column_array(mt: MTable, c: str):
    col = mt.col(c)
    if isinstance(col.values, torch.Tensor) and col.values.dim() == 1:
        v = col.values.detach().cpu().double().numpy()
        null = col.nulls.cpu().numpy() if col.nulls is not None else np.zeros(len(v), dtype=bool)
        return v, null | np.isnan(v)
    lst = col.to_list()
    v = np.array([float(x) if x is not None else np.nan for x in lst], dtype=np.float64)
    return np.nan_to_num(v), np.array([x is None for x in lst], dtype=bool) | np.isnan(v)


class _BucketMapperMixin:
    def _setup(self, buckets: List[_Bucketing]):
        self.buckets = buckets
        for b in buckets:
            keep = self.spec.invalid == "KEEP"
            self.spec.vector_size.append(b.nbins + 1 if keep else b.nbins)
            self.spec.drop_index.append(b.nbins - 1 if self.spec.drop_last else None)
        self.helper = self.spec.helper

    def _map_columns(self, mt):
        n, k = mt.num_rows, len(self.spec.cols)
        if self.spec.encode == "INDEX" and all(isinstance(mt.col(c).values, torch.Tensor) and
                                               mt.col(c).values.dim() == 1 for c in self.spec.cols):
            return self._index_columns_device(mt)
        idx = np.zeros((n, k), dtype=np.int64)
        valid = np.ones((n, k), dtype=bool)
        for j, c in enumerate(self.spec.cols):
            v, null = _column_array(mt, c)
            idx[:, j] = self.buckets[j].find(v, null)
            if null.any():
                if self.spec.invalid == "SKIP":
                    valid[null, j] = False
                elif self.spec.invalid == "ERROR":
                    raise RuntimeError("Unseen token: null")
        return self.spec.columns(idx, valid)


    def _index_columns_device(self, mt):
        """INDEX output of tensor columns where they live: ``torch.searchsorted`` over the bucket bounds (the
        side ``_Bucketing.find`` uses), nulls / NaN to the null bucket or, under SKIP, to a null cell."""
        out = []
        for j, c in enumerate(self.spec.cols):
            col = mt.col(c)
            v = col.values.to(torch.float64)
            null = torch.isnan(v)
            if col.nulls is not None:
                null = null | col.nulls.to(v.device)
            b = self.buckets[j]
            bt = torch.as_tensor(b.bounds, dtype=torch.float64, device=v.device)
            hit = (torch.searchsorted(bt, v, right=not b.left_open) - 1).clamp_(0, b.nbins - 1)
            hit = torch.where(null, torch.full_like(hit, b.null_index), hit)
            any_null = bool(null.any())
            if any_null and self.spec.invalid == "ERROR":
                raise RuntimeError("Unseen token: null")
            if any_null and self.spec.invalid == "SKIP":
                out.append(Column(torch.where(null, torch.zeros_like(hit), hit), null))
            else:
                out.append(Column(hit))
        return out


class QuantileDiscretizerModelMapper(_BucketMapperMixin, ModelMapper):
    def loadModel(self, rows):
        from ...common.model.converter import extract_meta_and_data
        meta, data = extract_meta_and_data(rows)
        borders = {d["featureName"]: d for d in (json.loads(s) for s in data)}
        train_cols = list(meta.get("selectedCols"))
        self.spec = _EncodeSpec(self.params, self.dataSchema, "INDEX", train_cols)
        self._setup([_Bucketing(borders[c]["splitsArray"], borders[c]["isLeftOpen"]) for c in self.spec.cols])


class BucketizerMapper(_BucketMapperMixin, Mapper):
    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        self.spec = _EncodeSpec(self.params, dataSchema, "INDEX", None)
        cuts = self.params.get("cutsArray")
        if len(cuts) != len(self.spec.cols):
            raise ValueError("The lengths of selectedCols and cusArray are not equal!")
        self._setup([_Bucketing(c, bool(_pget(self.params, "leftOpen", True))) for c in cuts])


class BinarizerMapper(SISOMapper):
    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        self.thr = float(_pget(self.params, "threshold", 0.0))
        t = dataSchema.types[self.col_idx]
        self.is_num = is_numeric(t)
        self.helper = OutputColsHelper(dataSchema, [self.helper.out_names[0]],
                                       [Types.DOUBLE if self.is_num else t], _pget(self.params, "reservedCols"))

    def mapColumn(self, v):
        if v is None:
            return None
        if self.is_num:
            return 1.0 if float(v) > self.thr else 0.0
        vec = VectorUtil.getVector(v)
        if isinstance(vec, SparseVector):
            keep = [i for i, x in zip(vec.indices, vec.values) if x > self.thr]
            return SparseVector(vec.size(), keep, [1.0] * len(keep))
        return DenseVector((vec.data > self.thr).astype(np.float64))

    def _map_columns(self, mt):
        col = mt.col(self.selected)
        if self.is_num and isinstance(col.values, torch.Tensor):
            r = (col.values.double() > self.thr).double()
            return [Column(r, col.nulls)]
        return [Column.from_values([self.mapColumn(v) for v in col.to_list()], self.helper.out_types[0])]


def murmur3_index(strings: Sequence[str], num_features: int) -> np.ndarray:
    """``floorMod(abs(murmur3_32(0).hashUnencodedChars(s)), numFeatures)`` for every string."""
    from ... import _native
    h = _native.murmur3_utf16(list(strings))
    if h is None:
        h = np.array([_murmur3_py(s) for s in strings], dtype=np.int64)
    h = np.abs(h.astype(np.int64))
    h = np.where(h == 2 ** 31, -(2 ** 31), h)   # Math.abs(Integer.MIN_VALUE) stays negative
    return np.mod(h, num_features)


def _murmur3_py(s: str) -> int:
    def rotl(x, r):
        return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF
    u = np.frombuffer(s.encode("utf-16-le"), dtype=np.uint16).astype(np.uint32)
    h1 = 0
    i = 1
    n = len(u)
    while i < n:
        k1 = int(u[i - 1]) | (int(u[i]) << 16)
        k1 = (k1 * 0xcc9e2d51) & 0xFFFFFFFF
        k1 = rotl(k1, 15)
        k1 = (k1 * 0x1b873593) & 0xFFFFFFFF
        h1 ^= k1
        h1 = rotl(h1, 13)
        h1 = (h1 * 5 + 0xe6546b64) & 0xFFFFFFFF
        i += 2
    if n & 1:
        k1 = int(u[n - 1])
        k1 = (k1 * 0xcc9e2d51) & 0xFFFFFFFF
        k1 = rotl(k1, 15)
        k1 = (k1 * 0x1b873593) & 0xFFFFFFFF
        h1 ^= k1
    h1 ^= (2 * n) & 0xFFFFFFFF
    h1 ^= h1 >> 16
    h1 = (h1 * 0x85ebca6b) & 0xFFFFFFFF
    h1 ^= h1 >> 13
    h1 = (h1 * 0xc2b2ae35) & 0xFFFFFFFF
    h1 ^= h1 >> 16
    return h1 - (1 << 32) if h1 >= (1 << 31) else h1


class FeatureHasherMapper(Mapper):
    """Numeric columns contribute their value at hash(colName); categorical ones 1.0 at hash("col=val")."""

    def __init__(self, dataSchema, params=None):
        super().__init__(dataSchema, params)
        sel = list(self.params.get("selectedCols"))
        cat = _pget(self.params, "categoricalCols")
        if cat is None:
            cat = [c for c in sel if not is_numeric(dataSchema.types[dataSchema.names.index(c)])]
        self.cat = [c for c in sel if c in cat]
        self.num = [c for c in sel if c not in self.cat]
        self.nf = int(_pget(self.params, "numFeatures", 262144))
        self.helper = OutputColsHelper(dataSchema, [self.params.get("outputCol")], [Types.VECTOR],
                                       _pget(self.params, "reservedCols"))
        self.num_index = murmur3_index(self.num, self.nf) if self.num else np.zeros(0, dtype=np.int64)

    def _map_columns(self, mt):
        """Columnar: one [m, n] entry matrix (numeric: fixed index hash(colName), value; categorical:
        hash("col=val"), 1.0), hashed and assembled into a row-sorted CSR ``SparseBlock`` on the env's device
        (``ops/csrc/feature.hip`` on a GPU) — no per-row Python objects."""
        from ...ops.feature import csr_assemble, murmur3_index
        from ...common.strings import StringBlock
        dev = feature_device()
        n = mt.num_rows
        m = len(self.num) + len(self.cat)
        if dev.type == "cuda" and not self.num and n:
            blocks = [mt.col(c).values for c in self.cat]
            if all(isinstance(b, StringBlock) and b.device == dev for b in blocks):
                # every field hashed in one launch straight into the [m, n] entry matrix
                from ...ops.strings import murmur3_multi_index
                r = murmur3_multi_index(blocks, [c + "=" for c in self.cat], self.nf)
                if r is not None:
                    return [Column(csr_assemble(r[0], None, r[1], self.nf))]
        idx = torch.zeros((m, n), dtype=torch.int64, device=dev)
        val = torch.ones((m, n), dtype=torch.float64, device=dev)
        valid = torch.zeros((m, n), dtype=torch.bool, device=dev)
        for j, c in enumerate(self.num):
            v, null = _column_array(mt, c)
            idx[j] = int(self.num_index[j])
            val[j] = torch.from_numpy(v).to(dev)
            valid[j] = torch.from_numpy(~null).to(dev)
        for j, c in enumerate(self.cat, start=len(self.num)):
            colv = mt.col(c).values
            if isinstance(colv, StringBlock):
                # packed UTF-8 column: hashed where it lives, no per-row Python strings
                blk = colv.to(dev)
                idx[j] = murmur3_index(blk, self.nf, prefix=c + "=", device=dev).to(dev)
                valid[j] = ~blk.null_mask()
                continue
            vals = mt.col(c).to_list()
            present = np.asarray([v is not None for v in vals], dtype=bool)
            if present.any():
                keys = [java_str(v) for v in vals if v is not None]
                pos = torch.from_numpy(np.nonzero(present)[0]).to(dev)
                idx[j, pos] = murmur3_index(keys, self.nf, prefix=c + "=", device=dev).to(dev)
                valid[j, pos] = True
        return [Column(csr_assemble(idx, val, valid, self.nf))]


def feature_device() -> torch.device:
    """Device of the default environment when it is a GPU with the HIP library, else the host."""
    from ...common.mlenv import MLEnvironmentFactory
    from ...ops import _lib
    dev = MLEnvironmentFactory.getDefault().device
    if dev.type == "cuda" and (_lib.available() or not _lib.torch_fallback_allowed()):
        return dev
    return torch.device("cpu")


class DCTMapper(SISOMapper):
    """Orthonormal DCT-II (inverse: DCT-III) of a dense vector (``DCTMapper.java``), batched via FFT."""

    def outputType(self):
        return Types.VECTOR

    def mapColumn(self, v):
        if v is None:
            return None
        from scipy.fft import dct, idct
        x = VectorUtil.getVector(v)
        x = x.toDenseVector().data if isinstance(x, SparseVector) else x.data
        inv = bool(_pget(self.params, "inverse", False))
        return DenseVector((idct if inv else dct)(x, type=2, norm="ortho"))

    def _map_columns(self, mt):
        """A dense 2-D tensor column transformed as one batch along its rows (the same scipy transform per
        row); other columns vector by vector."""
        v = mt.cols[self.col_idx].values
        if not (isinstance(v, torch.Tensor) and v.dim() == 2 and v.is_floating_point() and v.shape[1]
                and mt.num_rows):
            return super()._map_columns(mt)
        from scipy.fft import dct, idct
        inv = bool(_pget(self.params, "inverse", False))
        X = v.detach().to("cpu", torch.float64).numpy()
        return [Column(torch.from_numpy(np.ascontiguousarray((idct if inv else dct)(X, type=2, norm="ortho",
                                                                                   axis=1))))]
