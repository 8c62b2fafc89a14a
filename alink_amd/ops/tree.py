"""Tree-training hot path: binned histograms (K7/K10) and level routing (K9), SURVEY §2.13.

``histogram(bins, slot, stats, nslots, B)`` returns ``hist[nslots, F, B, S]`` with
``hist[slot[r], f, bins[r, f], :] += stats[r, :]`` for every row whose slot is in ``[0, nslots)``.
Reference: ``ConstructLocalBin.java:135-166`` (GBDT ``(g^2, g, h, 1)``) and ``paralleltree/TreeObj.java:321-390``
(RF class counts / moments).

``route(bins, node, feat, base, route_tab)`` moves every row one level down
(``Split.java:64-195``): ``node[r] = base[v] + route_tab[v, bins[r, feat[v]]]`` for an internal node ``v``
and ``node[r] = base[v]`` (a negative leaf code) for a leaf.

On a GPU the HIP kernels in ``csrc/tree_hist.hip`` run: by default ``tree_hist_fm`` (rows grouped by slot, a
workgroup per (row chunk, 32-feature group), int64 fixed-point bank-private LDS histograms — LDS float
atomics are ~30x slower than integer ones on gfx950 — and per-chunk slabs summed exactly); the older fp32
LDS-atomic kernels stay for S > 4 or very wide bins.  On the CPU the fp64 ``index_add_`` reference
below is used.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

__all__ = ["FmStats", "histogram", "histogram_groups", "histogram_torch", "route", "route_torch", "node_sums", "node_sums_torch", "quantize",
           "gbdt_split"]


def gpu_kernels_ok() -> bool:
    """HIP kernels are used on GPU tensors unless the library is missing AND the torch fallback is allowed."""
    return _lib.available() or not _lib.torch_fallback_allowed()


def _num_cus(device) -> int:
    return torch.cuda.get_device_properties(device).multi_processor_count


def histogram_torch(bins: torch.Tensor, slot: torch.Tensor, stats: torch.Tensor, nslots: int, B: int,
                    dtype=torch.float64) -> torch.Tensor:
    n, F = bins.shape
    S = stats.shape[1]
    out = torch.zeros((nslots * F * B, S), dtype=dtype, device=bins.device)
    keep = (slot >= 0) & (slot < nslots)
    if nslots == 0 or not bool(keep.any()):
        return out.view(nslots, F, B, S)
    rows = keep.nonzero().view(-1)
    chunk = max(1, (1 << 22) // max(F, 1))
    farange = torch.arange(F, device=bins.device, dtype=torch.long) * B
    for s in range(0, rows.numel(), chunk):
        r = rows[s:s + chunk]
        idx = (slot[r].long() * (F * B))[:, None] + farange[None, :] + bins[r].long()
        vals = stats[r].to(dtype)
        out.index_add_(0, idx.reshape(-1), vals[:, None, :].expand(-1, F, -1).reshape(-1, S))
    return out.view(nslots, F, B, S)


import os

# 2: fixed-point bank-private feature-group kernel over slot-grouped rows (S <= 4, B * S <= 640; default),
# 0: row-per-lane fp32-atomic kernel, 1: (row, feature)-pair fp32-atomic kernel
HIST_VARIANT = int(os.environ.get("ALINK_TREE_HIST_VARIANT", "2"))
FM_TARGET_BLOCKS = 2048       # histogram workgroups per launch (one 32-feature group x one row chunk each)
FM_MIN_ROWS = 8192            # rows per chunk floor: the LDS clear + slab store amortise over >= 0.5 MB of bins
FM_PACK_MAX_ROWS = 1 << 16    # packed (g, count) histograms: rows per chunk below 2^16 (csrc/tree_hist.hip PACK)
# packed statistic + count LDS atomics for S == 3 with a unit count column (ALINK_TREE_HIST_PACK=0 disables)
FM_PACK = os.environ.get("ALINK_TREE_HIST_PACK", "1") != "0"


def fm_plan(counts, nfg: int, max_rows: int = None, starts=None):
    """Chunking of slot-grouped rows for ``tree_hist_fm``: ``counts[s]`` rows of slot s, starting at row offset
    ``starts[s]`` (default: consecutive, slot after slot); ``max_rows`` caps the rows of a chunk.  Returns
    (chunk bounds [nchunks, 2] (start, end) row offsets, slot_chunk [nslots+1]) as int32 numpy arrays."""
    import numpy as np
    counts = np.asarray(counts, dtype=np.int64)
    total = int(counts.sum())
    R = max(FM_MIN_ROWS, -(-total * nfg // FM_TARGET_BLOCKS)) if total else FM_MIN_ROWS
    if max_rows is not None:
        R = min(R, int(max_rows))
    nch = -(-counts // R)
    slot_chunk = np.zeros(counts.size + 1, dtype=np.int64)
    np.cumsum(nch, out=slot_chunk[1:])
    if starts is None:
        starts = np.zeros(counts.size, dtype=np.int64)
        np.cumsum(counts[:-1], out=starts[1:])
    starts = np.asarray(starts, dtype=np.int64)
    pairs = []
    for s_, c in enumerate(counts):
        if c == 0:
            continue
        k = int(nch[s_])
        edges = starts[s_] + (np.arange(0, k + 1, dtype=np.int64) * c) // k
        pairs.append(np.stack([edges[:-1], edges[1:]], 1))
    bounds = np.concatenate(pairs) if pairs else np.zeros((0, 2), dtype=np.int64)
    return bounds.astype(np.int32), slot_chunk.astype(np.int32)


def gather_rows(q: torch.Tensor, p: torch.Tensor, order: torch.Tensor = None):
    """(q[p], order[p]) for the int32 [n, 4] statistics rows (and the int32 row ids) in one HIP gather; p int64."""
    n = p.numel()
    dev = q.device
    qo = torch.empty((n, 4), dtype=torch.int32, device=dev)
    oo = torch.empty(n, dtype=torch.int32, device=dev) if order is not None else None
    if n:
        L = _lib.require()
        rc = L.alink_tree_gather_rows(q.data_ptr(), None if order is None else order.data_ptr(), p.data_ptr(), n,
                                      qo.data_ptr(), None if oo is None else oo.data_ptr(), _lib.stream_ptr(dev))
        if rc != 0:
            raise RuntimeError(f"alink_tree_gather_rows failed: {rc}")
    return qo, oo


class RowOrder:
    """The rows of the tree being grown, grouped by their node of the current level (stable: ascending row id
    inside a node), and their quantised statistics in that order.  Re-grouped once per level from the previous
    grouping (rows only move inside their parent's segment, so the gathers walk memory almost in order) instead
    of a full sort + random gather of the statistics for every histogram call; the histogram kernel then reads
    the build nodes' segments in place (chunks skip the derived / finished nodes' rows)."""

    def __init__(self, prep: "FmStats", active: torch.Tensor):
        idx = torch.nonzero(active, as_tuple=False).reshape(-1)
        self.order = idx.to(torch.int32)
        self.q = gather_rows(prep.q, idx)[0]
        self.seg = np.asarray([0, int(self.order.numel())], dtype=np.int64)    # node segments
        self.tag = None

    def regroup(self, node_of_row: torch.Tensor, nn: int, tag) -> None:
        """Group by ``node_of_row`` (level node ids 0..nn-1; anything else leaves the order)."""
        if self.tag == tag:
            return
        dev = self.order.device
        key = node_of_row[self.order.long()]
        kt = torch.uint8 if nn < 255 else (torch.int16 if nn < 32767 else torch.int32)
        k = torch.where((key >= 0) & (key < nn), key, torch.full_like(key, nn)).to(kt)
        sk, p = torch.sort(k, stable=True)
        bnd = torch.searchsorted(sk, torch.arange(nn + 1, device=dev, dtype=kt)).cpu().numpy().astype(np.int64)
        keep = int(bnd[nn])
        self.q, self.order = gather_rows(self.q, p[:keep].contiguous(), self.order)
        self.seg = bnd
        self.tag = tag


def _col_absmax(stats: torch.Tensor, blk: int = 4096) -> torch.Tensor:
    """max |stats[:, j]| per column of a row-major [n, S] tensor.  A plain ``amax(dim=0)`` (or ``amax(dim=1)`` of
    the transposed copy) has only S outputs, and the device reduction of S very long rows ran ~3 ms per tree at
    1.25e7 rows; blocking the rows first gives n/blk x S independent reductions, then a tiny second pass."""
    n, S = stats.shape
    m = n // blk * blk
    parts = []
    if m:
        parts.append(stats[:m].abs().view(m // blk, blk, S).amax(1).amax(0))
    if n > m:
        parts.append(stats[m:].abs().amax(0))
    return torch.stack(parts).amax(0)


def fm_scales(stats: torch.Tensor):
    """Per-column power-of-two fixed-point scales for ``tree_hist_fm``: max|column| * scale < 2^30, so every
    row's value fits int32 and no int64 bin sum can overflow below 2^33 rows."""
    import math
    amax = _col_absmax(stats).double().cpu().numpy() if stats.numel() else []
    scales = []
    for m in amax:
        m = float(m)
        if not math.isfinite(m):
            raise ValueError("non-finite tree statistics")
        e = 30 - math.ceil(math.log2(m)) - 1 if m > 0 else 0
        scales.append(math.ldexp(1.0, max(min(e, 1000), -1000)))
    return scales


class FmStats:
    """Row statistics quantised once for ``tree_hist_fm`` (per tree: the statistics do not change between the
    levels): ``q`` [n, 4] int32 fixed point, ``inv`` [S] fp64 device scales back to floats."""

    def __init__(self, stats: torch.Tensor):
        n, S = stats.shape
        self.S = S
        self.n = n
        # the packed kernel keeps the count in the low bits of statistic 0 (exact row counts, 2 atomics per pair)
        self.pack = bool(FM_PACK and S == 3 and n and bool((stats[:, 2] == 1).all()))
        scales = fm_scales(stats)
        dev = stats.device
        self.q = torch.zeros((n, 4), dtype=torch.int32, device=dev)
        self.q[:, :S] = torch.round(stats.double() * torch.tensor(scales, dtype=torch.float64, device=dev)) \
            .to(torch.int32)
        self.inv = torch.tensor([1.0 / x for x in scales], dtype=torch.float64, device=dev)


def _histogram_fm(L, bins, slot, stats, nslots: int, B: int, prep: "FmStats" = None, fgroups=None,
                  tro: "RowOrder" = None, slot_nodes=None) -> torch.Tensor:
    """``tree_hist_fm`` path: rows grouped by slot (stable sort of the slot keys, or the identity when every row
    is in slot 0), statistics quantised to int64 fixed point (``prep``, or here) and gathered into that order,
    chunk plan, kernel + exact fixed-order reduce.  ``fgroups`` (int sequence of 32-feature groups): build only
    those, feature-major ``[len(fgroups) * 32, nslots, B, S]``."""
    dev = bins.device
    n, F = bins.shape
    S = stats.shape[1] if stats is not None else prep.S
    if prep is None:
        prep = FmStats(stats)
    starts = None
    if tro is not None:
        # the tree's node-grouped order: slot s = node slot_nodes[s]'s segment, read in place
        ridx, q = tro.order, tro.q
        starts = [int(tro.seg[i]) for i in slot_nodes]
        counts = [int(tro.seg[i + 1] - tro.seg[i]) for i in slot_nodes]
    elif nslots == 1 and bool(((slot >= 0) & (slot < nslots)).all()):
        ridx = None
        counts = [n]
        q = prep.q
    else:
        act = (slot >= 0) & (slot < nslots)
        # the narrowest key type: the radix sort makes one pass per key byte (uint8 for < 255 slots)
        kt = torch.uint8 if nslots < 255 else (torch.int16 if nslots < 32767 else torch.int32)
        key = torch.where(act, slot, torch.full_like(slot, nslots)).to(kt)
        skey, order = torch.sort(key, stable=True)
        # per-slot counts from the sorted keys (slot boundaries by binary search, no separate histogram pass)
        bnd = torch.searchsorted(skey, torch.arange(nslots + 1, device=dev, dtype=kt))
        counts = (bnd[1:] - bnd[:-1]).cpu().numpy()
        total = int(counts.sum())
        ridx = order[:total].to(torch.int32).contiguous()
        q = gather_rows(prep.q, order[:total].contiguous())[0]
    if fgroups is None:
        nfg, fgl = (F + 31) // 32, None
        hist = torch.empty((nslots, F, B, S), dtype=torch.float32, device=dev)
    else:
        nfg = len(fgroups)
        if any(not 0 <= int(g) < PAD_GROUP + 1 for g in fgroups):
            raise ValueError("feature group out of range")
        fgl = torch.as_tensor(list(fgroups), dtype=torch.int32).to(dev)
        hist = torch.empty((nfg * 32, nslots, B, S), dtype=torch.float32, device=dev)
        if nfg == 0:
            return hist
    chunk_rows, slot_chunk = fm_plan(counts, nfg, FM_PACK_MAX_ROWS - 1 if prep.pack else None, starts)
    nchunks = chunk_rows.shape[0]
    cr = torch.from_numpy(chunk_rows).to(dev)
    scn = torch.from_numpy(slot_chunk).to(dev)
    slab = torch.empty(max(nchunks, 1) * nfg * B * (2 if prep.pack else S) * 32, dtype=torch.int64, device=dev)
    rc = L.alink_tree_hist_fm(bins.data_ptr(), F, None if ridx is None else ridx.data_ptr(), q.data_ptr(),
                              cr.data_ptr(), nchunks, scn.data_ptr(), nslots, S, B,
                              None if fgl is None else fgl.data_ptr(), nfg, int(fgl is not None),
                              prep.inv.data_ptr(), slab.data_ptr(), hist.data_ptr(), _lib.stream_ptr(dev),
                              int(prep.pack))
    if rc != 0:
        raise RuntimeError(f"alink_tree_hist_fm failed: {rc}")
    return hist


PAD_GROUP = 1 << 24       # a 32-feature group index past every feature (zero rows in histogram_groups)


def histogram_groups(bins: torch.Tensor, slot: torch.Tensor, stats: torch.Tensor, nslots: int, B: int,
                     fgroups, prep: "FmStats" = None, tro: "RowOrder" = None, slot_nodes=None) -> torch.Tensor:
    """Feature-major histogram of the 32-feature groups ``fgroups`` only: ``[len(fgroups) * 32, nslots, B, S]``
    (features >= F, e.g. padding groups of the last rank's block, are zero rows) — the unit a per-rank
    feature-block reduce-scatter sends.  GPU: the fixed-point kernel over the listed groups; CPU: the fp64
    reference over the selected columns."""
    n, F = bins.shape
    S = stats.shape[1]
    if prep is None and S == 3 and FM_PACK and fm_eligible(bins, S, B, pack=True):
        prep = FmStats(stats)
    if fm_eligible(bins, S, B, pack=prep is not None and prep.pack):
        return _histogram_fm(_lib.require(), bins, slot.to(torch.int32).contiguous(), stats, nslots, B, prep,
                             fgroups=fgroups, tro=tro, slot_nodes=slot_nodes)
    feats = torch.tensor([g * 32 + l for g in fgroups for l in range(32)], dtype=torch.long)
    out = torch.zeros((feats.numel(), nslots, B, S), dtype=torch.float32 if bins.is_cuda else torch.float64,
                      device=bins.device)
    ok = (feats < F).nonzero().reshape(-1)
    if ok.numel():
        sub = bins[:, feats[ok].to(bins.device)].contiguous()
        h = histogram_torch(sub, slot, stats, nslots, B, dtype=out.dtype) if not bins.is_cuda else \
            histogram(sub, slot, stats, nslots, B)
        out[ok.to(out.device)] = h.transpose(0, 1).to(out.dtype)
    return out


def fm_eligible(bins: torch.Tensor, S: int, B: int, variant: int = None, pack: bool = False) -> bool:
    """The fixed-point kernel fits: its LDS histogram is [B, S, 32] int64 ([B, 2, 32] when packed)."""
    v = HIST_VARIANT if variant is None else int(variant)
    return bins.is_cuda and v == 2 and S <= 4 and B * (2 if pack else S) * 256 <= 160 * 1024 \
        and bins.shape[0] < 2 ** 31 and _lib.available()


def histogram(bins: torch.Tensor, slot: torch.Tensor, stats: torch.Tensor, nslots: int, B: int,
              variant: int = None, prep: FmStats = None, tro: "RowOrder" = None, slot_nodes=None) -> torch.Tensor:
    """[nslots, F, B, S] histogram (fp32 on GPU via HIP, fp64 on CPU).  ``prep``: the statistics already
    quantised for the fixed-point kernel (``FmStats(stats)``, reused across the levels of a tree)."""
    if not bins.is_cuda:
        return histogram_torch(bins, slot, stats, nslots, B)
    if not _lib.available() and _lib.torch_fallback_allowed():
        return histogram_torch(bins, slot, stats, nslots, B, dtype=torch.float32)
    L = _lib.require()
    n, F = bins.shape
    S = stats.shape[1]
    if bins.dtype != torch.uint8 or not bins.is_contiguous():
        raise ValueError("bins must be a contiguous uint8 [n, F] matrix")
    if B > 256:
        raise ValueError("at most 256 bins per feature")
    slot = slot.to(torch.int32).contiguous()
    stats = stats.to(torch.float32).contiguous()
    if slot.shape[0] != n or stats.shape[0] != n:
        raise ValueError("slot/stats row count mismatch")
    if prep is None and S == 3 and FM_PACK and fm_eligible(bins, S, B, variant, pack=True):
        prep = FmStats(stats)               # decides whether the packed (g, count) build applies
    if fm_eligible(bins, S, B, variant, pack=prep is not None and prep.pack) and nslots > 0:
        return _histogram_fm(L, bins, slot, stats, nslots, B, prep, tro=tro, slot_nodes=slot_nodes)
    hist = torch.zeros((nslots, F, B, S), dtype=torch.float32, device=bins.device)
    if n == 0 or nslots == 0:
        return hist
    rc = L.alink_tree_hist_f32(bins.data_ptr(), n, F, slot.data_ptr(), stats.data_ptr(), S, B, nslots,
                               hist.data_ptr(), _num_cus(bins.device),
                               HIST_VARIANT if variant is None else int(variant), _lib.stream_ptr(bins.device))
    if rc != 0:
        raise RuntimeError(f"alink_tree_hist_f32 failed: {rc}")
    return hist


def route_torch(bins, node, feat, base, route_tab):
    nn = feat.shape[0]
    act = (node >= 0) & (node < nn)
    if not bool(act.any()):
        return node
    r = act.nonzero().view(-1)
    v = node[r].long()
    f = feat[v].long()
    leaf = f < 0
    b = bins[r, f.clamp(min=0)].long()
    child = base[v].long() + torch.where(leaf, torch.zeros_like(b), route_tab[v, b].long())
    node = node.clone()
    node[r] = child.to(node.dtype)
    return node


def route(bins: torch.Tensor, node: torch.Tensor, feat: torch.Tensor, base: torch.Tensor,
          route_tab: torch.Tensor) -> torch.Tensor:
    """New int32 node ids (in place on GPU)."""
    if not bins.is_cuda:
        return route_torch(bins, node, feat, base, route_tab)
    if not _lib.available() and _lib.torch_fallback_allowed():
        return route_torch(bins, node, feat, base, route_tab)
    L = _lib.require()
    n, F = bins.shape
    nn = feat.shape[0]
    if route_tab.shape != (nn, 256):
        raise ValueError("route table must be [nnodes, 256]")
    feat = feat.to(torch.int32).contiguous()
    if bool((feat >= F).any()):
        raise ValueError("split feature out of range")
    base = base.to(torch.int32).contiguous()
    route_tab = route_tab.to(torch.int16).contiguous()
    assert node.dtype == torch.int32 and node.is_contiguous() and node.shape[0] == n
    rc = L.alink_tree_route(bins.data_ptr(), n, F, node.data_ptr(), feat.data_ptr(), base.data_ptr(),
                            route_tab.data_ptr(), nn, _num_cus(bins.device), _lib.stream_ptr(bins.device))
    if rc != 0:
        raise RuntimeError(f"alink_tree_route failed: {rc}")
    return node


def node_sums_torch(node: torch.Tensor, sample: torch.Tensor, stats: torch.Tensor, nnodes: int) -> torch.Tensor:
    S = stats.shape[1]
    out = torch.zeros((nnodes + 1, S), dtype=torch.float64, device=stats.device)
    chunk = 1 << 22
    for s0 in range(0, node.shape[0], chunk):
        nd = node[s0:s0 + chunk]
        ok = sample[s0:s0 + chunk] & (nd >= 0) & (nd < nnodes)
        idx = torch.where(ok, nd.long(), torch.full_like(nd, nnodes, dtype=torch.long))
        out.index_add_(0, idx, stats[s0:s0 + chunk].to(torch.float64))
    return out[:nnodes]


def node_sums(node: torch.Tensor, sample: torch.Tensor, stats: torch.Tensor, nnodes: int) -> torch.Tensor:
    """[nnodes, S] fp64 sums of ``stats`` rows per node id (sampled rows only) — node counters."""
    if not stats.is_cuda or (not _lib.available() and _lib.torch_fallback_allowed()):
        return node_sums_torch(node, sample, stats, nnodes)
    L = _lib.require()
    n, S = stats.shape
    node = node.to(torch.int32).contiguous()
    samp = sample.to(torch.uint8).contiguous()
    st = stats.to(torch.float32).contiguous()
    out = torch.zeros((max(nnodes, 1), S), dtype=torch.float64, device=stats.device)
    rc = L.alink_tree_node_sums(node.data_ptr(), samp.data_ptr(), st.data_ptr(), n, S, nnodes, out.data_ptr(),
                                _num_cus(stats.device), _lib.stream_ptr(stats.device))
    if rc != 0:
        raise RuntimeError(f"alink_tree_node_sums failed: {rc}")
    return out[:nnodes]


def f32_threshold_table(thresholds, TP: int) -> np.ndarray:
    """[F, TP] float32: per threshold t the smallest float strictly greater than t, NaN padding; for every fp32 x
    ``t < x  <=>  u <= x``, so an fp32 search counts the fp64 thresholds below x exactly."""
    tab = np.full((len(thresholds), TP), np.nan, dtype=np.float32)
    for i, t in enumerate(thresholds):
        t = np.asarray(t, dtype=np.float64)
        if t.size:
            u = t.astype(np.float32)
            low = u.astype(np.float64) <= t
            u[low] = np.nextafter(u[low], np.float32(np.inf))
            tab[i, :t.size] = u
    return tab


def _quantize_f32(L, cols, nulls, thresholds, out_cols, n, F, missing, out):
    dev = out.device
    T = max(1, max(len(t) for t in thresholds))
    TP = 1
    while TP < T:
        TP <<= 1
    cols = [c.contiguous() for c in cols]
    nulls = [None if m is None else m.to(torch.uint8).contiguous() for m in nulls]
    meta = torch.tensor([[c.data_ptr() for c in cols], [0 if m is None else m.data_ptr() for m in nulls]],
                        dtype=torch.int64).to(dev)
    oc = torch.tensor(list(out_cols), dtype=torch.int32).to(dev)
    thr = torch.from_numpy(f32_threshold_table(thresholds, TP)).to(dev)
    rc = L.alink_tree_quantize_f32(meta[0].data_ptr(), meta[1].data_ptr(), oc.data_ptr(), len(cols), n, F,
                                   thr.data_ptr(), TP, int(missing), out.data_ptr(), _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_tree_quantize_f32 failed: {rc}")
    torch.cuda.current_stream(dev).synchronize()      # the pointer tables must outlive the kernel


def quantize(cols, nulls, thresholds, out_cols, n: int, F: int, missing: int, out: torch.Tensor) -> None:
    """K5: bin continuous columns into ``out`` (uint8 [n, F], row-major) on the GPU.  ``cols`` fp32/fp64 device
    vectors [n], ``nulls`` bool masks or None, ``thresholds`` per column (ascending fp64 numpy), ``out_cols``
    destination column per input (``bin = #thresholds < x``; NaN / null -> ``missing``)."""
    L = _lib.require()
    dev = out.device
    Fc = len(cols)
    if Fc == 0 or n == 0:
        return
    cols = [c if c.dtype in (torch.float32, torch.float64) else c.to(torch.float64) for c in cols]
    f32 = [i for i, c in enumerate(cols) if c.dtype == torch.float32]
    if f32:
        # fp32 columns: exact fp32 threshold tables, half the LDS traffic of the fp64 search (quantize_f32)
        _quantize_f32(L, [cols[i] for i in f32], [nulls[i] for i in f32], [thresholds[i] for i in f32],
                      [out_cols[i] for i in f32], n, F, missing, out)
        rest = [i for i in range(Fc) if cols[i].dtype != torch.float32]
        if not rest:
            return
        cols, nulls = [cols[i] for i in rest], [nulls[i] for i in rest]
        thresholds, out_cols = [thresholds[i] for i in rest], [out_cols[i] for i in rest]
        Fc = len(cols)
    cols = [c.contiguous() for c in cols]
    nulls = [None if m is None else m.to(torch.uint8).contiguous() for m in nulls]
    T = max(1, max(len(t) for t in thresholds))
    thr = torch.full((Fc, T), float("inf"), dtype=torch.float64)
    for i, t in enumerate(thresholds):
        if len(t):
            thr[i, :len(t)] = torch.as_tensor(t, dtype=torch.float64)
    meta = torch.tensor([[c.data_ptr() for c in cols], [0 if m is None else m.data_ptr() for m in nulls]],
                        dtype=torch.int64).to(dev)
    is32 = torch.tensor([int(c.dtype == torch.float32) for c in cols], dtype=torch.int32).to(dev)
    oc = torch.tensor(list(out_cols), dtype=torch.int32).to(dev)
    nt = torch.tensor([len(t) for t in thresholds], dtype=torch.int32).to(dev)
    thr = thr.to(dev)
    rc = L.alink_tree_quantize(meta[0].data_ptr(), meta[1].data_ptr(), is32.data_ptr(), oc.data_ptr(), Fc, n, F,
                               thr.data_ptr(), nt.data_ptr(), T, int(missing), out.data_ptr(), _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_tree_quantize failed: {rc}")
    # keep the pointer tables alive until the kernel has consumed them
    torch.cuda.current_stream(dev).synchronize()


def gbdt_split(H: torch.Tensor, min_leaf: float, min_hess: float, gi: int = 1, hi: int = 2, ci: int = 3):
    """K8: (best gain [m, F] fp64, best bin [m, F] int64) of the GBDT gain over the fp32 histogram H [m,F,B,S]."""
    L = _lib.require()
    m, F, B, S = H.shape
    H = H.to(torch.float32).contiguous()
    gain = torch.empty((m, F), dtype=torch.float64, device=H.device)
    binj = torch.empty((m, F), dtype=torch.int32, device=H.device)
    rc = L.alink_gbdt_split(H.data_ptr(), m, F, B, S, gi, hi, ci, float(min_leaf), float(min_hess),
                            gain.data_ptr(), binj.data_ptr(), _lib.stream_ptr(H.device))
    if rc != 0:
        raise RuntimeError(f"alink_gbdt_split failed: {rc}")
    return gain, binj.to(torch.int64)


SPLIT_S = (3, 4, 5, 6, 8, 11)
_CRIT = {"gbdt": 0, "gini": 1, "infogain": 2, "infogainratio": 3, "mse": 4}


def tree_split(H: torch.Tensor, kind: str, is_cat: torch.Tensor, n_classes: int, min_leaf: float,
               min_hess: float, min_ratio: float, min_gain: float):
    """K8/K10 general split search on the GPU: (best gain [m, F] fp64 (-inf: none), best position [m, F] int64 in
    the per-(node, feature) bin order — the stable (key, bin) order for categorical features, the bin order for
    continuous ones).  ``None`` when the statistic count has no compiled instantiation (torch search)."""
    m, F, B, S = H.shape
    if S not in SPLIT_S or B > 257:
        return None
    L = _lib.require()
    H = H.to(torch.float32).contiguous()
    cat = is_cat.to(device=H.device, dtype=torch.uint8).contiguous()
    gain = torch.empty((m, F), dtype=torch.float64, device=H.device)
    pos = torch.empty((m, F), dtype=torch.int32, device=H.device)
    rc = L.alink_tree_split(H.data_ptr(), m, F, B, S, _CRIT[kind], int(n_classes), cat.data_ptr(), float(min_leaf),
                            float(min_hess), float(min_ratio), float(min_gain), gain.data_ptr(), pos.data_ptr(),
                            _lib.stream_ptr(H.device))
    if rc == 3:
        return None
    if rc != 0:
        raise RuntimeError(f"alink_tree_split failed: {rc}")
    return gain, pos.to(torch.int64)


def split_order_key(h, kind: str, n_classes: int, categorical: bool):
    """Host twin of the kernel's ordering: stable argsort of the candidate bins' keys ([B, S] row of one node and
    feature) — engine._materialise uses it to rebuild the chosen categorical split's left set."""
    import numpy as np
    h = np.asarray(h, dtype=np.float64)
    Hv = h[:-1]
    nb = Hv.shape[0]
    if not categorical:
        return np.arange(nb)
    if kind == "gbdt":
        g, hh = Hv[:, 1], Hv[:, 2]
        key = np.where(hh < 1e-6, -1.0, g / np.where(hh < 1e-6, 1.0, hh))
    else:
        cnt = Hv[:, -1]
        if kind == "mse":
            w = Hv[:, 0]
        else:
            w = np.zeros(nb)
            for k in range(n_classes):            # the kernel's summation order
                w = w + Hv[:, k]
        num = Hv[:, 1] if kind == "mse" else Hv[:, 0]
        key = np.where(cnt > 0, num / np.where(w == 0, 1.0, w), np.inf)
    return np.argsort(key, kind="stable")
