"""Tree preprocessing: label encoding, categorical indexing and quantile binning into a uint8 matrix.

Reference: ``A/operator/common/tree/Preprocessing.java`` (distinct labels ``:45-80``; string indexer for
categorical columns ``:157-190``; quantile discretizer over a ``sampleCount4Bin`` sample ``:240-300``,
``SAMPLE_COUNT_4_BIN`` default 500000), ``TableUtil.getCategoricalCols`` (string/boolean feature columns
are categorical even when not listed) and ``DataFormatToArray.java:77-83`` (row-major -> per-feature byte
arrays).

MI355X layout: one row-major ``uint8 [n, F]`` bin matrix per rank, resident in HBM for the whole training
run (1e8 rows x 128 features = 12.8 GB).  Bin ``nbins_f`` .. ``B-2`` are never used by feature ``f``; bin
``B-1`` is the shared missing-value bin.  Continuous features split as ``x <= threshold[j]`` <=> bin <= j.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from ...common.javafmt import java_str
from ...common.params import Params
from ...common.table import MTable
from ...common.types import Types
from ...parallel import comm

__all__ = ["BinnedData", "categorical_cols", "numeric_column", "distinct_labels", "build_bins",
           "quantile_thresholds", "SAMPLE_COUNT_4_BIN"]

SAMPLE_COUNT_4_BIN = 500000
_STRINGISH = (Types.STRING, Types.BOOLEAN)


def categorical_cols(mt_schema, feature_cols: Sequence[str], given: Optional[Sequence[str]]) -> List[str]:
    """``TableUtil.getCategoricalCols``: listed columns plus every string/boolean feature column."""
    given = list(given or [])
    for c in given:
        if c not in feature_cols:
            raise ValueError("CategoricalCols must be included in featureCols!")
    out = []
    for c in feature_cols:
        t = mt_schema.types[mt_schema.names.index(c)]
        if c in given or t in _STRINGISH:
            out.append(c)
    return out


def numeric_column(mt: MTable, c: str, device) -> (torch.Tensor, torch.Tensor):
    """float64 values + null mask (NaN counts as missing) on ``device``."""
    col = mt.col(c)
    if isinstance(col.values, torch.Tensor) and col.values.dim() == 1:
        v = col.values.to(device=device, dtype=torch.float64)
        null = col.nulls.to(device) if col.nulls is not None else torch.zeros(v.shape[0], dtype=torch.bool,
                                                                               device=device)
    else:
        lst = col.to_list()
        null = torch.tensor([x is None for x in lst], dtype=torch.bool, device=device)
        v = torch.tensor([0.0 if x is None else float(x) for x in lst], dtype=torch.float64, device=device)
    null = null | torch.isnan(v)
    return torch.where(null, torch.zeros_like(v), v), null


def _gpu_quantize_ok() -> bool:
    from ...ops import _lib
    return _lib.available() or not _lib.torch_fallback_allowed()


def _raw_column(mt: MTable, c: str, device):
    """Numeric column in its own float dtype on ``device`` (null mask or None) — the quantize kernel reads it
    in place."""
    col = mt.col(c)
    if isinstance(col.values, torch.Tensor) and col.values.dim() == 1:
        v = col.values.to(device)
        if v.dtype not in (torch.float32, torch.float64):
            v = v.to(torch.float64)
        null = col.nulls.to(device) if col.nulls is not None else None
        return v, null
    return numeric_column(mt, c, device)


def _sort_key(v):
    if isinstance(v, (bool, np.bool_)):
        return (0, int(v))
    if isinstance(v, (int, float, np.integer, np.floating)):
        return (0, float(v))
    return (1, str(v))


def distinct_labels(mt: MTable, label_col: str) -> List[Any]:
    """Globally distinct, ascending-sorted labels (``Preprocessing.distinctLabels``)."""
    col = mt.col(label_col)
    if isinstance(col.values, torch.Tensor) and col.values.dim() == 1:
        v = col.values if col.nulls is None else col.values[~col.nulls.to(col.values.device)]
        local = sorted(torch.unique(v).cpu().tolist(), key=_sort_key)
    else:
        local = sorted({v for v in mt.column_values(label_col) if v is not None}, key=_sort_key)
    merged = set()
    for part in comm.all_gather_object(local):
        merged.update(part)
    return sorted(merged, key=_sort_key)


def quantile_thresholds(values: np.ndarray, max_bins: int, exact_midpoints: bool) -> np.ndarray:
    """Split thresholds of one continuous feature.

    * ``exact_midpoints`` and at most ``max_bins`` distinct values: midpoints between consecutive distinct
      values — the exact candidate set of the series CART (``ContinuousSplitter.java:60-95``).
    * otherwise the quantile discretizer's cut points ``sorted[round((n-1) j / q)]``, j = 1..q-1, de-duplicated
      (``QuantileDiscretizerTrainBatchOp`` with ``numBuckets = maxBins``); the split value stored in the model
      is the right border of the left bin (``QuantileDiscretizerModelDataConverter.getFeatureValue``).
    """
    if values.size == 0:
        return np.zeros(0)
    s = np.sort(values)
    if exact_midpoints:
        u = np.unique(s)
        if u.size <= max_bins:
            return (u[:-1] + u[1:]) / 2.0
    n = s.size
    q = max_bins
    idx = np.minimum(n - 1, np.floor((n - 1.0) * np.arange(1, q) / q + 0.5).astype(np.int64))
    return np.unique(s[idx])


@dataclass
class BinnedData:
    bins: torch.Tensor                     # uint8 [n, F] row-major
    B: int                                 # bins per feature incl. the missing bin (index B-1)
    feature_cols: List[str]
    is_cat: List[bool]
    nbins: List[int]                       # used bins per feature (categorical: category count)
    thresholds: List[Optional[np.ndarray]]  # continuous: split values; categorical: None
    cat_tokens: Dict[str, List[str]] = field(default_factory=dict)   # categorical column -> tokens by index
    indexer_rows: List[Any] = field(default_factory=list)           # MultiStringIndexer model rows
    bin_values: List[Optional[np.ndarray]] = field(default_factory=list)

    @property
    def missing_bin(self) -> int:
        return self.B - 1


def _sample_rows(n_local: int, cap_total: int, seed: int) -> np.ndarray:
    total = int(sum(comm.all_gather_object(int(n_local))))
    if total <= cap_total:
        return np.arange(n_local)
    ratio = cap_total / total
    rng = np.random.default_rng(seed + comm.get_rank())
    return np.nonzero(rng.random(n_local) < ratio)[0]


def build_bins(mt: MTable, feature_cols: Sequence[str], cat_cols: Sequence[str], max_bins: int, device,
               exact_midpoints: bool, seed: int = 0, string_order: str = "RANDOM") -> BinnedData:
    """Bin every feature column into ``uint8`` codes (device resident)."""
    from ..feature.encoders import train_multi_string_indexer
    if max_bins > 255:
        raise ValueError("binNum must be less or equal than 255.")
    feature_cols = list(feature_cols)
    n = mt.num_rows
    F = len(feature_cols)
    is_cat = [c in cat_cols for c in feature_cols]
    cat_tokens: Dict[str, List[str]] = {}
    indexer_rows: List[Any] = []
    if cat_cols:
        p = Params().set("selectedCols", list(cat_cols)).set("stringOrderType", string_order)
        model = train_multi_string_indexer(mt, p)
        indexer_rows = [tuple(r) for r in model.rows()]
        for r in indexer_rows:
            ci = int(r[0])
            if ci >= 0:
                cat_tokens.setdefault(cat_cols[ci], {})[r[1]] = int(r[2])
        cat_tokens = {c: [t for t, _ in sorted(cat_tokens.get(c, {}).items(), key=lambda kv: kv[1])]
                      for c in cat_cols}
    # continuous thresholds from a (global) sample
    cont = [c for c, ic in zip(feature_cols, is_cat) if not ic]
    cap = max(1, min(SAMPLE_COUNT_4_BIN, (1 << 25) // max(1, len(cont))))
    sample_idx = _sample_rows(n, cap, seed) if cont else np.zeros(0, dtype=np.int64)
    thresholds: List[Optional[np.ndarray]] = [None] * F
    bin_values: List[Optional[np.ndarray]] = [None] * F
    gpu = torch.device(device).type == "cuda" and _gpu_quantize_ok()
    cols_dev = {}
    if cont:
        sidx = torch.as_tensor(sample_idx, device=device)
        local_samples = []
        for c in cont:
            if gpu:
                v, null = _raw_column(mt, c, device)        # native dtype, no full-column fp64 copy
                cols_dev[c] = (v, null)
                vs = v[sidx].to(torch.float64)
                ok = ~torch.isnan(vs) if null is None else (~null[sidx] & ~torch.isnan(vs))
                local_samples.append(vs[ok].cpu().numpy())
            else:
                v, null = numeric_column(mt, c, device)
                cols_dev[c] = (v, null)
                vs, ns = v[sidx], null[sidx]
                local_samples.append(vs[~ns].cpu().numpy())
        gathered = comm.all_gather_arrays(local_samples)          # tensor collectives, no pickling
        for j, c in enumerate(cont):
            allv = np.concatenate([g[j] for g in gathered]) if gathered else np.zeros(0)
            fi = feature_cols.index(c)
            thresholds[fi] = quantile_thresholds(allv, max_bins, exact_midpoints)
            if exact_midpoints:
                u = np.unique(allv)
                if u.size <= max_bins:
                    bin_values[fi] = u
    nbins = []
    for fi, c in enumerate(feature_cols):
        if is_cat[fi]:
            k = len(cat_tokens.get(c, []))
            if k > 254:
                raise ValueError(f"categorical column {c} has {k} categories; at most 254 are supported "
                                 f"(maxBins {max_bins})")
            nbins.append(max(1, k))
        else:
            nbins.append(len(thresholds[fi]) + 1)
    B = max(nbins) + 1
    bins = torch.empty((n, F), dtype=torch.uint8, device=device)
    if gpu and cont:
        # K5: all continuous columns in one quantize launch (ops/csrc/tree_split.hip)
        from ...ops import tree as tops
        fis = [feature_cols.index(c) for c in cont]
        tops.quantize([cols_dev[c][0] for c in cont], [cols_dev[c][1] for c in cont], [thresholds[fi] for fi in fis],
                      fis, n, F, B - 1, bins)
    for fi, c in enumerate(feature_cols):
        if is_cat[fi]:
            m = {t: i for i, t in enumerate(cat_tokens.get(c, []))}
            codes = [m.get(java_str(v), B - 1) if v is not None else B - 1 for v in mt.column_values(c)]
            bins[:, fi] = torch.tensor(codes, dtype=torch.uint8).to(device)
        elif not gpu:
            v, null = cols_dev[c] if c in cols_dev else numeric_column(mt, c, device)
            thr = torch.as_tensor(thresholds[fi], dtype=torch.float64, device=device)
            b = torch.searchsorted(thr, v.contiguous(), right=False) if thr.numel() else torch.zeros_like(
                v, dtype=torch.long)
            b = torch.where(null, torch.full_like(b, B - 1), b)
            bins[:, fi] = b.to(torch.uint8)
    return BinnedData(bins.contiguous(), B, feature_cols, is_cat, nbins, thresholds, cat_tokens, indexer_rows,
                      bin_values)
