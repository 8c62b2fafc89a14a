"""Data-processing batch ops: sampling/splitting/ids/casts and the vector mapper family.

Reference: ``A/operator/batch/dataproc/*`` — ``SplitBatchOp.java:20-183`` (exact ``round(N*fraction)``
rows chosen with per-partition quotas; the remainder is side output 0), ``AppendIdBatchOp`` (DENSE ids =
global row index, UNIQUE = task-strided), ``SampleBatchOp``/``SampleWithSizeBatchOp``/``WeightSampleBatchOp``,
``FirstNBatchOp``, ``NumericalTypeCastBatchOp`` and the ``vector/*BatchOp`` MapBatchOp wrappers.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from ...common.params import ParamInfo, Params
from ...common.table import Column, MTable
from ...common.types import TableSchema, Types, type_from_str
from ...models.dataproc import vector as V
from ...parallel import comm
from ..base import BatchOperator
from .utils import MapBatchOp

__all__ = ["FirstNBatchOp", "SampleBatchOp", "SampleWithSizeBatchOp", "WeightSampleBatchOp", "SplitBatchOp",
           "AppendIdBatchOp", "NumericalTypeCastBatchOp", "VectorAssemblerBatchOp", "VectorNormalizeBatchOp",
           "VectorSliceBatchOp", "VectorElementwiseProductBatchOp", "VectorInteractionBatchOp",
           "VectorPolynomialExpandBatchOp", "VectorSizeHintBatchOp", "VectorSerializeBatchOp",
           "VectorToColumnsBatchOp", "global_offset", "rank_rng"]


def global_offset(n_local: int):
    """(offset of this rank's first row in global order, global row count, per-rank counts)."""
    counts = comm.all_gather_object(int(n_local))
    r = comm.get_rank()
    return int(sum(counts[:r])), int(sum(counts)), counts


def rank_rng(seed: int = 0) -> np.random.Generator:
    return np.random.default_rng(np.random.SeedSequence([int(seed) & 0xFFFFFFFF, comm.get_rank()]))


class FirstNBatchOp(BatchOperator):
    def __init__(self, params: Optional[Params] = None, **kw):
        if isinstance(params, int):
            n, params = params, None
            super().__init__(params, **kw)
            self.setSize(n)
        else:
            super().__init__(params, **kw)

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        n = self.getSize()
        if mt.replicated:
            self.setOutputTable(mt.slice(0, min(n, mt.num_rows)))
            return self
        off, _, _ = global_offset(mt.num_rows)
        take = max(0, min(mt.num_rows, n - off))
        self.setOutputTable(mt.slice(0, take))
        return self


class SampleBatchOp(BatchOperator):
    EXTRA_PARAMS = [ParamInfo("randomSeed", int, "seed", default=0)]

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        rng = rank_rng(self.getParams().get(self._param_infos["randomSeed"]))
        ratio = self.getRatio()
        if self.getWithReplacement():
            reps = rng.poisson(ratio, mt.num_rows)
            idx = np.repeat(np.arange(mt.num_rows), reps)
        else:
            idx = np.nonzero(rng.random(mt.num_rows) < ratio)[0]
        self.setOutputTable(mt.take(idx))
        return self


class SampleWithSizeBatchOp(BatchOperator):
    EXTRA_PARAMS = [ParamInfo("randomSeed", int, "seed", default=0)]

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        off, total, _ = global_offset(mt.num_rows)
        rng = np.random.default_rng(self.getParams().get(self._param_infos["randomSeed"]))
        size = self.getSize()
        if self.getWithReplacement():
            g = rng.integers(0, total, size) if total else np.zeros(0, dtype=np.int64)
        else:
            g = rng.choice(total, size=min(size, total), replace=False) if total else np.zeros(0, dtype=np.int64)
        g = np.sort(g)
        local = g[(g >= off) & (g < off + mt.num_rows)] - off
        self.setOutputTable(mt.take(local))
        return self


class WeightSampleBatchOp(BatchOperator):
    EXTRA_PARAMS = [ParamInfo("randomSeed", int, "seed", default=0)]

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        w = np.asarray(mt.column_values(self.getWeightCol()), dtype=np.float64)
        tot = float(sum(comm.all_gather_object(float(w.sum()))))
        _, total, _ = global_offset(mt.num_rows)
        ratio = self.getRatio()
        rng = rank_rng(self.getParams().get(self._param_infos["randomSeed"]))
        if self.getWithReplacement():
            reps = rng.poisson(ratio * total * w / max(tot, 1e-300))
            idx = np.repeat(np.arange(mt.num_rows), reps)
        else:
            # A-ES weighted reservoir keys; keep global top ratio*N
            keys = np.log(np.maximum(rng.random(mt.num_rows), 1e-300)) / np.maximum(w, 1e-300)
            target = int(round(total * ratio))
            allk = np.sort(np.concatenate(comm.all_gather_object(keys)))[::-1] if total else np.zeros(0)
            thr = allk[target - 1] if 0 < target <= len(allk) else np.inf
            idx = np.nonzero(keys >= thr)[0]
        self.setOutputTable(mt.take(idx))
        return self


class SplitBatchOp(BatchOperator):
    EXTRA_PARAMS = [ParamInfo("randomSeed", int, "seed", default=0)]

    def __init__(self, params: Optional[Params] = None, **kw):
        if isinstance(params, float):
            f, params = params, None
            super().__init__(params, **kw)
            self.setFraction(f)
        else:
            super().__init__(params, **kw)

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        frac = self.getFraction()
        if frac < 0 or frac > 1:
            raise ValueError(f"invalid fraction {frac}")
        off, total, counts = global_offset(mt.num_rows)
        seed = self.getParams().get(self._param_infos["randomSeed"])
        # per-partition quotas (rank 0 decides, like CountInPartition)
        target = int(round(total * frac))
        sel = [int(np.floor(c * frac)) for c in counts]
        rem = target - sum(sel)
        prng = np.random.default_rng(seed)
        while rem > 0:
            for i in prng.permutation(len(counts)):
                if rem == 0:
                    break
                if sel[i] < counts[i]:
                    sel[i] += 1
                    rem -= 1
        r = comm.get_rank()
        rng = np.random.default_rng(np.random.SeedSequence([seed, r]))
        pick = np.sort(rng.permutation(mt.num_rows)[:sel[r]])
        mask = np.zeros(mt.num_rows, dtype=bool)
        mask[pick] = True
        self.setOutputTable(mt.take(np.nonzero(mask)[0]))
        self.setSideOutputTables([mt.take(np.nonzero(~mask)[0])])
        return self


class AppendIdBatchOp(BatchOperator):
    appendIdColName = "append_id"

    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        col = self.getIdCol() or self.appendIdColName
        off, total, _ = global_offset(mt.num_rows)
        at = self.getAppendType()
        at = at.name if hasattr(at, "name") else str(at)
        if at.upper() == "UNIQUE":
            ws = comm.get_world_size()
            ids = torch.arange(mt.num_rows, dtype=torch.int64) * ws + comm.get_rank()
        else:
            ids = torch.arange(off, off + mt.num_rows, dtype=torch.int64)
        self.setOutputTable(mt.with_columns([col], [Types.LONG], [Column(ids)]))
        return self


def _cast_tensor_column(col, t):
    """``float(v)`` / ``int(float(v))`` over a numeric tensor column at once (through float64, as the row path
    rounds), nulls kept; None (the row path) for other columns, a NaN / infinite value under an integer target
    (the row path raises) or a value outside the integer target's range."""
    import torch
    v = col.values
    dt = getattr(t, "torch_dtype", None)
    if not (isinstance(v, torch.Tensor) and v.dim() == 1 and dt is not None and not v.is_complex()):
        return None
    nm = col.nulls.to(v.device) if col.nulls is not None else None
    x = v.to(torch.float64)
    if t.py is float:
        r = x.to(dt)
    else:
        live = x if nm is None else x[~nm]
        if live.numel() and not bool(torch.isfinite(live).all()):
            return None
        x = torch.trunc(torch.where(nm, torch.zeros_like(x), x) if nm is not None else x)
        info = torch.iinfo(dt)
        if x.numel() and (float(x.min()) < info.min or float(x.max()) > info.max):
            return None
        r = x.to(dt)
    if nm is not None:
        r = torch.where(nm, torch.zeros_like(r), r)
    return Column(r, nm)


class NumericalTypeCastBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        t = self.getTargetType()
        t = type_from_str(t.name if hasattr(t, "name") else str(t))
        sel = self.getSelectedCols()
        names, types, cols = [], [], []
        for n in sel:
            names.append(n)
            types.append(t)
            fast = _cast_tensor_column(mt.col(n), t)
            if fast is not None:
                cols.append(fast)
                continue
            vals = mt.column_values(n)
            conv = [None if v is None else (float(v) if t.py is float else int(float(v))) for v in vals]
            cols.append(Column.from_values(conv, t))
        self.setOutputTable(mt.with_columns(names, types, cols))
        return self


class VectorAssemblerBatchOp(MapBatchOp):
    MAPPER = V.VectorAssemblerMapper


class VectorNormalizeBatchOp(MapBatchOp):
    MAPPER = V.VectorNormalizeMapper


class VectorSliceBatchOp(MapBatchOp):
    MAPPER = V.VectorSliceMapper


class VectorElementwiseProductBatchOp(MapBatchOp):
    MAPPER = V.VectorElementwiseProductMapper


class VectorInteractionBatchOp(MapBatchOp):
    MAPPER = V.VectorInteractionMapper


class VectorPolynomialExpandBatchOp(MapBatchOp):
    MAPPER = V.VectorPolynomialExpandMapper


class VectorSizeHintBatchOp(MapBatchOp):
    MAPPER = V.VectorSizeHintMapper


class VectorSerializeBatchOp(MapBatchOp):
    PARAMS = ()
    MAPPER = V.VectorSerializeMapper


class VectorToColumnsBatchOp(MapBatchOp):
    """Vector flavour (``selectedCol`` + ``outputCols``) or the format flavour (``vectorCol`` + ``schemaStr``,
    ``dataproc/format/VectorToColumnsBatchOp``)."""
    MAPPER = V.VectorToColumnsMapper
    EXTRA_PARAMS = [ParamInfo("vectorCol", str, "Name of a vector column", default=None),
                    ParamInfo("schemaStr", str, "Formatted schema", default=None),
                    ParamInfo("handleInvalid", str, "Strategy to handle unseen token", default="ERROR")]
