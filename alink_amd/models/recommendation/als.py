"""Alternating least squares (reference ``A/operator/common/recommendation/{AlsTrain,AlsPredict,
AlsModelDataConverter,AlsModelMapper}.java``, ``A/operator/batch/recommendation/*``).

Semantics kept from the reference: the rating graph is split into user and item "nodes"; every iteration
updates all user factors (in ``numBlocks`` mini-batches, ``|id| % numBlocks``) and then all item factors;
explicit feedback solves ``(Y_u^T Y_u + lambda n_u I) x = Y_u^T r_u`` (``AlsTrain.java:510-520``), implicit
feedback ``(Y^T Y + Y_u^T C_u Y_u + lambda n_u^+ I) x = Y_u^T (1 + C_u) p_u`` with ``c = alpha r``
(``:521-540``); non-negative solves use NNLS.

MI355X design (SURVEY §2.3 P5 -> RCCL): instead of the reference's per-superstep request/response coGroups,
the ratings are shuffled ONCE into two owner-partitioned CSR copies (by user and by item; one
``all_to_all_single`` each), the small factor tables are replicated in HBM on every rank, each rank builds
and solves the normal equations of the nodes it owns (HIP kernel ``ops/csrc/als.hip`` + batched Cholesky)
and the updated rows are all-gathered.  Model table: ``(userCol LONG, itemCol LONG, factors STRING)`` with
``Float.toString`` factors joined by spaces, user rows have a null item and vice versa.
"""
from __future__ import annotations

import os
import time

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ...ops.gemm import tn_matmul
from ...common.javafmt import java_float_str
from ...common.mapper import ModelMapper, OutputColsHelper, find_col_index
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import TableSchema, Types
from ...ops import als as aops
from ...parallel import comm

__all__ = ["AlsModelData", "AlsModelDataConverter", "AlsModelMapper", "train_als", "als_topk"]


class AlsModelData:
    def __init__(self, user_ids, user_factors, item_ids, item_factors):
        self.user_ids = np.asarray(user_ids, dtype=np.int64)
        self.user_factors = np.asarray(user_factors, dtype=np.float32)
        self.item_ids = np.asarray(item_ids, dtype=np.int64)
        self.item_factors = np.asarray(item_factors, dtype=np.float32)
        self._user_map = self._item_map = None

    # id -> row maps, built on first use (a Python dict over 1e7 user ids costs ~1 s; training never reads them)
    @property
    def user_map(self):
        if self._user_map is None:
            self._user_map = dict(zip(self.user_ids.tolist(), range(len(self.user_ids))))
        return self._user_map

    @property
    def item_map(self):
        if self._item_map is None:
            self._item_map = dict(zip(self.item_ids.tolist(), range(len(self.item_ids))))
        return self._item_map

    # the reference's field names (AlsModelData.java: userIds, userFactors, itemIds, itemFactors)
    userIds = property(lambda self: self.user_ids)
    userFactors = property(lambda self: self.user_factors)
    itemIds = property(lambda self: self.item_ids)
    itemFactors = property(lambda self: self.item_factors)


def _factor_str(f: np.ndarray) -> str:
    return " ".join(java_float_str(float(x)) for x in f)


class AlsModelDataConverter:
    def __init__(self, user_col: str, item_col: str):
        self.user_col, self.item_col = user_col, item_col

    def getModelSchema(self) -> TableSchema:
        return TableSchema([self.user_col, self.item_col, "factors"], [Types.LONG, Types.LONG, Types.STRING])

    def save(self, m: AlsModelData) -> List[tuple]:
        # factor strings in Float.toString form from the C++ formatter (OpenMP row blocks): 1e7 users x rank 64
        # are 6.4e8 values, hours through the per-value Python formatter
        from ... import _native
        us = _native.java_float_rows(m.user_factors.reshape(len(m.user_ids), -1))
        its = _native.java_float_rows(m.item_factors.reshape(len(m.item_ids), -1))
        if us is None or its is None:
            us = [_factor_str(f) for f in m.user_factors]
            its = [_factor_str(f) for f in m.item_factors]
        rows = [(u, None, f) for u, f in zip(m.user_ids.tolist(), us)]
        rows += [(None, i, f) for i, f in zip(m.item_ids.tolist(), its)]
        return rows

    @staticmethod
    def load(rows) -> AlsModelData:
        rows = list(rows)
        fast = AlsModelDataConverter._load_native(rows)
        if fast is not None:
            return fast
        us, uf, its, itf = [], [], [], []
        for r in rows:
            f = np.asarray([float(x) for x in str(r[2]).split(" ")], dtype=np.float32)
            if r[0] is not None:
                us.append(int(r[0]))
                uf.append(f)
            else:
                its.append(int(r[1]))
                itf.append(f)
        rk = len(uf[0]) if uf else (len(itf[0]) if itf else 0)
        return AlsModelData(us, np.stack(uf) if uf else np.zeros((0, rk)), its,
                            np.stack(itf) if itf else np.zeros((0, rk)))

    @staticmethod
    def _load_native(rows) -> Optional[AlsModelData]:
        """The factor strings parsed by the C++ number reader (all rows one rank wide, plain decimal tokens);
        None sends the rows through the per-row path (NaN / Infinity tokens, ragged rows, no library)."""
        from ... import _native
        if not rows or _native.lib is None:
            return None
        user = [r[0] is not None for r in rows]
        strs = [str(r[2]) for r in rows]
        rk = len(strs[0].split(" "))
        res = _native.parse_dense_vectors(strs, rk)
        if res is None:
            return None
        # parse_dense_vectors zero-pads short rows: every row must hold exactly rk values
        if any(s.count(" ") != rk - 1 for s in strs):
            return None
        F = res.astype(np.float32)
        um = np.asarray(user, dtype=bool)
        uid = [int(r[0]) for r in rows if r[0] is not None]
        iid = [int(r[1]) for r in rows if r[0] is None]
        return AlsModelData(uid, F[um], iid, F[~um])


# ---------------------------------------------------------------------------------------------------
def _ids(mt: MTable, c: str, device) -> torch.Tensor:
    col = mt.col(c)
    if isinstance(col.values, torch.Tensor):
        v = col.values.to(device)
        if v.is_floating_point():
            v = v.to(torch.float64).trunc()
        return v.to(torch.int64)
    return torch.tensor([int(float(v)) for v in col.to_list()], dtype=torch.int64, device=device)


def _vals(mt: MTable, c: str, device) -> torch.Tensor:
    col = mt.col(c)
    if isinstance(col.values, torch.Tensor):
        return col.values.to(device).to(torch.float32)
    return torch.tensor([float(v) for v in col.to_list()], dtype=torch.float32, device=device)


class _Side:
    """Owner-partitioned CSR of one side (rows = owned nodes of this rank, ascending global index)."""

    def __init__(self, rows_idx: torch.Tensor, nbr_idx: torch.Tensor, rating: torch.Tensor, raw_ids: torch.Tensor):
        order = torch.argsort(rows_idx * (int(nbr_idx.max()) + 1 if nbr_idx.numel() else 1) + nbr_idx)
        rows_idx, nbr_idx, rating = rows_idx[order], nbr_idx[order], rating[order]
        self.nodes, counts = torch.unique_consecutive(rows_idx, return_counts=True)   # global node indices
        self.indptr = torch.zeros(self.nodes.numel() + 1, dtype=torch.int64, device=rows_idx.device)
        self.indptr[1:] = torch.cumsum(counts, 0)
        self.nbr = nbr_idx.to(torch.int32)
        self.rating = rating
        self.raw = raw_ids[self.nodes]            # original ids of the owned nodes
        # positives per row as a segmented sum over the sorted ratings (cumsum at the row boundaries): an fp64
        # index_add_ here serialises on the atomics of popular items (tens of seconds at 1e7 ratings on ROCm)
        cs = torch.zeros(rating.numel() + 1, dtype=torch.int64, device=rows_idx.device)
        torch.cumsum((rating > 0).to(torch.int64), 0, out=cs[1:])
        self.n_pos = (cs[self.indptr[1:]] - cs[self.indptr[:-1]]).to(torch.float64)
        self.n_all = counts.to(torch.float64)

    def subset_cached(self, key, mask_fn):
        """``subset(mask_fn())`` computed once per key: the row blocks of a side are the same every iteration,
        so the CSR sub-matrices (and the solver's row plan keyed by their identity) are built on the first sweep
        only.  The whole side is the side's own CSR (no copy)."""
        sub = getattr(self, "_subs", None)
        if sub is None:
            sub = self._subs = {}
        if key not in sub:
            mask = mask_fn()
            if bool(mask.all()):
                sub[key] = (torch.arange(mask.numel(), device=mask.device), self.indptr, self.nbr, self.rating)
            else:
                sub[key] = self.subset(mask)
        return sub[key]

    def subset(self, mask: torch.Tensor):
        sel = mask.nonzero().view(-1)
        starts, ends = self.indptr[:-1][sel], self.indptr[1:][sel]
        cnt = ends - starts
        indptr = torch.zeros(sel.numel() + 1, dtype=torch.int64, device=sel.device)
        indptr[1:] = torch.cumsum(cnt, 0)
        if sel.numel():
            pos = torch.repeat_interleave(starts - indptr[:-1], cnt) + torch.arange(int(indptr[-1]), device=sel.device)
        else:
            pos = torch.zeros(0, dtype=torch.int64, device=sel.device)
        return sel, indptr, self.nbr[pos], self.rating[pos]


GATHER_BLOCKS = int(os.environ.get("ALINK_ALS_GATHER_BLOCKS", "4"))


def _update(side: _Side, mask: torch.Tensor, Y: torch.Tensor, X: torch.Tensor, lam: float, implicit: bool,
            alpha: float, nonneg: bool, YtY: Optional[torch.Tensor], key=None):
    """Solve this rank's rows of ``side`` against ``Y`` and replicate them into ``X``.  Over P ranks the rows are
    solved in GATHER_BLOCKS pieces: the all-gather of piece b runs on the comm stream (asynchronous) while piece
    b+1 solves (SURVEY §7.1 compute / communication overlap; the reference's AlsTrain exchanges factor blocks
    by shuffle, ``AlsTrain.java:283-389``)."""
    ws = comm.get_world_size()
    if ws > 1 and GATHER_BLOCKS > 1:
        sel_all = torch.nonzero(mask, as_tuple=False).reshape(-1)
        bounds = [(len(sel_all) * b) // GATHER_BLOCKS for b in range(GATHER_BLOCKS + 1)]
        pend = []
        for b in range(GATHER_BLOCKS):
            def piece(b=b):
                m = torch.zeros_like(mask)
                m[sel_all[bounds[b]:bounds[b + 1]]] = True
                return m
            rows, x = _solve(side, piece, Y, X, lam, implicit, alpha, nonneg, YtY,
                             key=None if key is None else (key, b, GATHER_BLOCKS))
            pend.append((comm.all_gather_varlen_async(rows), comm.all_gather_varlen_async(x)))
        for pr, px in pend:
            X[pr.wait()] = px.wait().to(X.dtype)
        return
    rows, x = _solve(side, lambda: mask, Y, X, lam, implicit, alpha, nonneg, YtY,
                     key=None if key is None else (key, 0, 1))
    rows_all = comm.all_gather_varlen(rows)
    x_all = comm.all_gather_varlen(x)
    X[rows_all] = x_all.to(X.dtype)


def _solve(side: _Side, mask_fn, Y: torch.Tensor, X: torch.Tensor, lam: float, implicit: bool,
           alpha: float, nonneg: bool, YtY: Optional[torch.Tensor], key=None):
    sel, indptr, nbr, rating = side.subset_cached(key, mask_fn) if key is not None else side.subset(mask_fn())
    if sel.numel() and not nonneg and aops.fused_supported(Y):
        # GPU: normal equations + Cholesky fused per row (ops/csrc/als.hip), no [m, r, r] tensor in HBM
        reg = (side.n_pos[sel] if implicit else side.n_all[sel]) * lam
        x = aops.fused_solve(indptr, nbr, rating, Y, reg, implicit, alpha, YtY)
        rows = side.nodes[sel]
    elif sel.numel():
        A, b = aops.normal_equations(indptr, nbr, rating, Y, implicit, alpha)
        A = A.to(torch.float64)
        reg = (side.n_pos[sel] if implicit else side.n_all[sel]) * lam
        if implicit:
            A = A + YtY[None, :, :]
        A = A + reg[:, None, None] * torch.eye(A.shape[1], dtype=A.dtype, device=A.device)[None]
        x = aops.solve(A, b.to(torch.float64), nonneg)
        rows = side.nodes[sel]
    else:
        x = torch.zeros((0, X.shape[1]), dtype=torch.float32, device=X.device)
        rows = torch.zeros(0, dtype=torch.int64, device=X.device)
    return rows, x


ITER_SECONDS: List[float] = []     # wall time of each iteration of the last train_als (ALINK_ALS_TIME_ITERS=1)


def train_als(mt: MTable, params: Params, env) -> AlsModelData:
    t_start = time.perf_counter()
    dev = env.device
    prof = os.environ.get("ALINK_ALS_PROFILE") == "1"

    def mark(what, t0=[t_start]):  # noqa: B006  (per-phase wall time, ALINK_ALS_PROFILE=1)
        if prof:
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            now = time.perf_counter()
            print(f"[als] {what}: {now - t0[0]:.3f} s", flush=True)
            t0[0] = now

    g = lambda k, d: params.get(k) if params.contains(k) and params.get(k) is not None else d  # noqa: E731
    user_col, item_col, rate_col = params.get("userCol"), params.get("itemCol"), params.get("rateCol")
    rank = int(g("rank", 10))
    lam = float(g("lambda", 0.1))
    num_iter = int(g("numIter", 10))
    implicit = bool(g("implicitPrefs", False))
    alpha = float(g("alpha", 40.0))
    nonneg = bool(g("nonnegative", False))
    nblocks = max(1, int(g("numBlocks", 1)))
    seed = int(g("seed", 0)) if params.contains("seed") else 0
    u = _ids(mt, user_col, dev)
    it = _ids(mt, item_col, dev)
    r = _vals(mt, rate_col, dev)
    mark("ids")
    users = torch.unique(comm.all_gather_varlen(torch.unique(u)))
    items = torch.unique(comm.all_gather_varlen(torch.unique(it)))
    ui = torch.searchsorted(users, u)
    ii = torch.searchsorted(items, it)
    ws, me = comm.get_world_size(), comm.get_rank()
    mark("index")

    def shuffle(owner_idx):
        if ws == 1:
            return ui, ii, r
        dest = owner_idx % ws
        order = torch.argsort(dest)
        counts = torch.bincount(dest, minlength=ws).tolist()
        pairs = torch.stack([ui, ii], 1)[order]
        rr = r[order]
        got_p = comm.all_to_all_tensors(list(torch.split(pairs, counts)))
        got_r = comm.all_to_all_tensors([x[:, None] for x in torch.split(rr, counts)])
        p = torch.cat(got_p)
        return p[:, 0], p[:, 1], torch.cat(got_r)[:, 0]

    su, si, sr = shuffle(ui)
    by_user = _Side(su, si, sr, users)
    tu, ti, tr = shuffle(ii)
    by_item = _Side(ti, tu, tr, items)
    mark("csr")
    # random init drawn where the factors live (a 1e7 x 64 host draw + copy costs seconds); the same seed gives
    # the same factors on every rank
    gen = torch.Generator(device=dev).manual_seed(seed)
    U = torch.rand((users.numel(), rank), generator=gen, dtype=torch.float32, device=dev)
    V = torch.rand((items.numel(), rank), generator=gen, dtype=torch.float32, device=dev)
    mark("init factors")
    timed = os.environ.get("ALINK_ALS_TIME_ITERS") == "1"
    ITER_SECONDS.clear()
    for _ in range(num_iter):
        if timed:
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            t_it = time.perf_counter()
        for name, (side, Y, X) in (("users", (by_user, V, U)), ("items", (by_item, U, V))):
            YtY = tn_matmul(Y.to(torch.float64), Y.to(torch.float64)) if implicit else None
            for bb in range(nblocks):
                mask = (side.raw.abs() % nblocks) == bb
                _update(side, mask, Y, X, lam, implicit, alpha, nonneg, YtY, key=("block", bb, nblocks))
            mark(f"update {name}")
        if timed:
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            ITER_SECONDS.append(time.perf_counter() - t_it)
    return AlsModelData(users.cpu().numpy(), U.cpu().numpy(), items.cpu().numpy(), V.cpu().numpy())


# ---------------------------------------------------------------------------------------------------
class AlsModelMapper(ModelMapper):
    """Predicted rating = sum_i (float) u_i * v_i accumulated in double (``AlsModelMapper.predictRating``);
    unknown user or item -> null."""

    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        p = self.params
        self.ucol = find_col_index(dataSchema.names, p.get("userCol"))
        self.icol = find_col_index(dataSchema.names, p.get("itemCol"))
        reserved = p.get("reservedCols") if p.contains("reservedCols") else None
        self.helper = OutputColsHelper(dataSchema, [p.get("predictionCol")], [Types.DOUBLE], reserved)

    def loadModel(self, rows):
        self.model = AlsModelDataConverter.load(rows)

    def _map_columns(self, mt):
        m = self.model
        us = mt.col(self.dataSchema.names[self.ucol]).to_list()
        its = mt.col(self.dataSchema.names[self.icol]).to_list()
        out = []
        for a, b in zip(us, its):
            ui = m.user_map.get(int(a)) if a is not None else None
            ii = m.item_map.get(int(b)) if b is not None else None
            if ui is None or ii is None:
                out.append(None)
            else:
                prod = (m.user_factors[ui] * m.item_factors[ii]).astype(np.float32).astype(np.float64)
                s = 0.0
                for x in prod:
                    s += float(x)
                out.append(s)
        return [Column.from_values(out, Types.DOUBLE)]


def als_topk(model: AlsModelData, users: Sequence[int], k: int, device) -> List[tuple]:
    """Top-``k`` items per requested user by ``u . v`` (reference ``AlsPredict.recommendForUsers`` ->
    ``BlockwiseCross.findTopK``, ``A/operator/common/recommendation/AlsPredict.java:32-103``).

    This rank's users stay on its device; the item table is split into one block per rank and the blocks
    rotate around the RCCL ring (``parallel/cross.py``), each merged by the fused score + top-K kernel, so no
    rank materialises a score matrix or more than two item blocks.  Output ``"item:score,..."``."""
    want = [int(x) for x in users if x is not None and int(x) in model.user_map]
    seen, uniq = set(), []
    for x in want:
        if x not in seen:
            seen.add(x)
            uniq.append(x)
    from ...parallel.cross import blockwise_topk
    ws, me = comm.get_world_size(), comm.get_rank()
    n_items = model.item_factors.shape[0]
    lo, hi = (me * n_items) // ws, ((me + 1) * n_items) // ws
    dev = torch.device(device) if device is not None else torch.device("cpu")
    r = model.item_factors.shape[1] if model.item_factors.ndim == 2 else 0
    U = torch.as_tensor(np.asarray(model.user_factors[[model.user_map[x] for x in uniq]], dtype=np.float32)
                        .reshape(len(uniq), r), device=dev)
    V = torch.as_tensor(np.asarray(model.item_factors[lo:hi], dtype=np.float32).reshape(hi - lo, r), device=dev)
    kk = min(k, n_items)
    if kk <= 0:
        return []
    val, idx = blockwise_topk(U, V, kk)            # collective: every rank takes part, even with no users
    val, idx = val.cpu().numpy(), idx.cpu().numpy()
    from ... import _native
    strs = _native.java_float_kv_rows(model.item_ids[idx], val) if len(uniq) else []
    if strs is None:
        strs = [",".join(f"{int(a)}:{java_float_str(float(b))}" for a, b in zip(model.item_ids[idx[j]], val[j]))
                for j in range(len(uniq))]
    return list(zip(uniq, strs))
