"""Word2Vec: skip-gram with hierarchical softmax (reference ``A/operator/batch/nlp/Word2VecTrainBatchOp.java``,
``A/operator/common/nlp/{Word2VecModelMapper,DocVecGenerator}.java``).

Kept from the reference: vocabulary = words with count >= ``minCount`` (sorted by count, most frequent
first), Huffman coding (``createBinaryTree`` ``:64-139``), input vectors initialised with ``nextFloat`` in
[0, 1) and output (inner-node) vectors with zeros, the update rule of ``CalcModel.update`` (``:450-505``: the
context word's input vector against the Huffman path of the centre word, ``g = (1 - code - sigma(f)) * alpha``
with the 1/84-step sigmoid table and |f| < 6 cut-off, random window shrink ``b = nextInt(window)``), and
``numIter x syncNum`` synchronisation rounds that average input/output vectors across workers
(``AvgInputOutput`` ``:589-604``; SURVEY P2 local SGD + model averaging).

MI355X design: within a rank the skip-gram pairs of a data slice are processed in large batches on the
device — gather ``[P, L, d]`` path vectors, one fused dot/sigmoid/gradient pass, ``index_add_`` scatter of
both gradient sets (Hogwild-style, as the reference's per-pair loop is on one thread) — and the per-round
model average is one RCCL all-reduce of the two ``[V, d]`` tables.
"""
from __future__ import annotations

import heapq
from collections import Counter
from typing import List, Optional, Tuple

import numpy as np
import torch

from ...common.linalg import DenseVector, VectorUtil
from ...common.mapper import SISOMapper, ModelMapper, OutputColsHelper, find_col_index
from ...common.params import Params
from ...common.table import MTable
from ...common.types import TableSchema, Types
from ...ops import w2v as wops
from ...parallel import comm
from .text import java_split

__all__ = ["train_word2vec", "huffman", "Word2VecModelMapper", "MODEL_SCHEMA"]

MODEL_SCHEMA = TableSchema(["word", "vec"], [Types.STRING, Types.VECTOR])


def _pget(p: Params, name, default=None):
    try:
        if p.contains(name):
            v = p.get(name)
            return default if v is None else v
    except KeyError:
        pass
    return default


def huffman(counts: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """word2vec.c Huffman tree over counts sorted descending -> (codes [V, L], points [V, L], lengths [V]).
    Inner nodes are numbered 0..V-2 (the root is V-2), as ``createBinaryTree``."""
    V = len(counts)
    if V == 1:
        return np.zeros((1, 1), np.int64), np.zeros((1, 1), np.int64), np.zeros(1, np.int64)
    count = np.concatenate([counts.astype(np.int64), np.full(V - 1, np.iinfo(np.int64).max // 4)])
    parent = np.zeros(2 * V - 1, np.int64)
    binary = np.zeros(2 * V - 1, np.int64)
    pos1, pos2 = V - 1, V
    for a in range(V - 1):
        mins = []
        for _ in range(2):
            if pos1 >= 0 and count[pos1] < count[pos2]:
                mins.append(pos1)
                pos1 -= 1
            else:
                mins.append(pos2)
                pos2 += 1
        count[V + a] = count[mins[0]] + count[mins[1]]
        parent[mins[0]] = parent[mins[1]] = V + a
        binary[mins[1]] = 1
    codes, points = [], []
    for a in range(V):
        c, p = [], []
        b = a
        while b != 2 * V - 2:
            c.append(binary[b])
            p.append(b)
            b = parent[b]
        n = len(c)
        code = c[::-1]
        point = [V - 2] + [p[n - k] - V for k in range(1, n)]
        codes.append(code)
        points.append(point)
    L = max(len(c) for c in codes)
    C = np.zeros((V, L), np.int64)
    P = np.zeros((V, L), np.int64)
    lens = np.array([len(c) for c in codes], np.int64)
    for i, (c, p) in enumerate(zip(codes, points)):
        C[i, :len(c)] = c
        P[i, :len(p)] = p
    return C, P, lens


def _pairs(docs: List[np.ndarray], window: int, random_window: bool, rng: np.random.Generator):
    """(centre, context) word-id pairs in the reference's loop order."""
    cen, ctx = [], []
    for val in docs:
        n = len(val)
        if n < 2:
            continue
        b = rng.integers(0, window, size=n) if random_window else np.zeros(n, np.int64)
        for i in range(n):
            for a in range(int(b[i]), window * 2 + 1 - int(b[i])):
                if a == window:
                    continue
                c = i - window + a
                if 0 <= c < n:
                    cen.append(val[i])
                    ctx.append(val[c])
    return np.asarray(cen, np.int64), np.asarray(ctx, np.int64)


# Per-batch step bound for ids that repeat inside one batch (see _sgd).  Measured on a 20-topic Zipf corpus
# (V = 2000, d = 100, batch 8192, 3 epochs): HS loss 0.554 with a full mean (one step per id and batch), 0.399
# with DUP_CAP 16, 0.428 for near-sequential batches of 64 pairs; uncapped (DUP_CAP 128+) diverges.
DUP_CAP = 16.0


def _sgd(inp, out, C, P, lens, cen, ctx, alpha, batch):
    dev = inp.device
    Lmax = C.shape[1]
    ar = torch.arange(Lmax, device=dev)
    for s in range(0, cen.numel(), batch):
        c = cen[s:s + batch]
        x = ctx[s:s + batch]
        nodes = P[c]                                  # [B, L]
        code = C[c].to(inp.dtype)
        mask = ar[None, :] < lens[c][:, None]
        h = inp[x]                                    # [B, d]
        o = out[nodes]                                # [B, L, d]
        f = (o * h[:, None, :]).sum(-1)
        valid = mask & (f > -6.0) & (f < 6.0)
        q = torch.floor((f.clamp(-6.0, 6.0 - 1e-9) + 6.0) * 84.0) / 84.0 - 6.0   # sigmoid-table abscissa
        g = (1.0 - code - torch.sigmoid(q)) * alpha * valid
        neu1e = (g[..., None] * o).sum(1)
        # every pair of a batch reads the same stale vectors, so a node / word occurring m times would take m
        # uncorrected steps at once (hot words and the Huffman root diverge), while averaging them (one step per
        # batch) starves exactly those ids — the root is on every path.  Bounded correction: up to DUP_CAP
        # summed steps per id and batch, scaled down to DUP_CAP x the mean beyond that.
        cn = (torch.bincount(nodes[mask], minlength=out.shape[0]).to(g.dtype) / DUP_CAP).clamp(min=1)
        cx = (torch.bincount(x, minlength=inp.shape[0]).to(g.dtype) / DUP_CAP).clamp(min=1)
        out.index_add_(0, nodes.reshape(-1), ((g / cn[nodes])[..., None] * h[:, None, :]).reshape(-1, h.shape[1]))
        inp.index_add_(0, x, neu1e / cx[x][:, None])


def train_word2vec(mt: MTable, params: Params, env) -> List[tuple]:
    col = params.get("selectedCol")
    delim = _pget(params, "wordDelimiter", " ")
    dim = int(_pget(params, "vectorSize", 100))
    alpha = float(_pget(params, "alpha", 0.025))
    min_count = int(_pget(params, "minCount", 5))
    window = int(_pget(params, "window", 5))
    random_window = str(_pget(params, "randomWindow", "true")).lower() == "true"
    num_iter = int(_pget(params, "numIter", 1))
    seed = int(_pget(params, "seed", 0)) if params.contains("seed") else 0
    docs_tok = [[w for w in java_split(str(v), delim) if w] for v in mt.column_values(col) if v is not None]
    cnt = Counter()
    for d in docs_tok:
        cnt.update(d)
    # global vocabulary: counts reduced on one owner rank per word, ordered count desc / word asc
    # (parallel/sort.merged_vocabulary; the reference's pSort, Word2VecTrainBatchOp.java:145)
    from ...parallel.sort import merged_vocabulary
    merged = merged_vocabulary(dict(cnt), keep=lambda w, c: c >= min_count)
    if not merged:
        return []
    total = dict(merged)
    vocab = [w for w, _ in merged]
    index = {w: i for i, w in enumerate(vocab)}
    V = len(vocab)
    C, P, lens = huffman(np.array([total[w] for w in vocab]))
    dev = env.device
    dt = torch.float64 if dev.type == "cpu" else torch.float32
    gen = torch.Generator().manual_seed(seed)
    inp = torch.rand((V, dim), generator=gen, dtype=torch.float64).to(dev, dt)
    out = torch.zeros((max(V - 1, 1), dim), dtype=dt, device=dev)
    Ct, Pt, Lt = (torch.as_tensor(C, device=dev), torch.as_tensor(P, device=dev), torch.as_tensor(lens, device=dev))
    docs = [np.array([index[w] for w in d if w in index], np.int64) for d in docs_tok]
    ndocs_total = sum(comm.all_gather_object(len(docs)))
    sync = max(ndocs_total // 100000, 5)
    rng = np.random.default_rng(seed + 7919 * comm.get_rank())
    ws = comm.get_world_size()
    use_kernel = wops.kernel_supported(dev, dim)
    H = wops.HuffmanDevice(C, P, lens, dev) if use_kernel else None
    for step in range(sync * num_iter):
        k = step % sync
        lo, hi = (len(docs) * k) // sync, (len(docs) * (k + 1)) // sync
        if use_kernel:
            # K20: the window enumeration and every pair's HS update run on the device (Hogwild waves);
            # shrinks drawn exactly as _pairs draws them
            sl = [d for d in docs[lo:hi] if len(d) >= 2]
            shr = [rng.integers(0, window, size=len(d)) if random_window else np.zeros(len(d), np.int64) for d in sl]
            wops.sg_hs_train(sl, shr, window, H, inp, out, alpha)
            cen = np.zeros(0)
        else:
            cen, ctx = _pairs(docs[lo:hi], window, random_window, rng)
        if cen.size:
            # pairs in one batch read the same (stale) vectors; keep a batch to a few updates per word
            _sgd(inp, out, Ct, Pt, Lt, torch.as_tensor(cen, device=dev), torch.as_tensor(ctx, device=dev), alpha,
                 batch=int(min(8192, max(16, 2 * V))))
        if ws > 1:
            comm.all_reduce(inp, "sum")
            comm.all_reduce(out, "sum")
            inp /= ws
            out /= ws
    vecs = inp.to(torch.float64).cpu().numpy()
    return [(w, DenseVector(vecs[i])) for i, w in enumerate(vocab)]


class Word2VecModelMapper(ModelMapper):
    """Document vector = AVG (default) / SUM / MIN / MAX of its known word vectors, as a vector string."""

    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        p = self.params
        self.col = p.get("selectedCol")
        self.col_idx = find_col_index(dataSchema.names, self.col)
        self.delim = _pget(p, "wordDelimiter", " ")
        self.method = str(getattr(_pget(p, "predMethod", "AVG"), "name", _pget(p, "predMethod", "AVG"))).upper()
        out = _pget(p, "outputCol") or self.col
        self.helper = OutputColsHelper(dataSchema, [out], [Types.STRING], _pget(p, "reservedCols"))

    def loadModel(self, rows):
        self.embed = {r[0]: np.asarray(VectorUtil.getVector(r[1]).toDenseVector().data
                                       if hasattr(VectorUtil.getVector(r[1]), "toDenseVector")
                                       else VectorUtil.getVector(r[1]).data, dtype=np.float64) for r in rows}

    def _map_row_values(self, row):
        v = row[self.col_idx]
        if v is None:
            return [None]
        vecs = [self.embed[t] for t in java_split(str(v), self.delim) if t in self.embed]
        if not vecs:
            return [None]
        d = vecs[0].copy()
        for t in vecs[1:]:      # sequential, as DocVecGenerator folds the vectors
            if self.method == "MIN":
                d = np.minimum(d, t)
            elif self.method == "MAX":
                d = np.maximum(d, t)
            else:
                d = d + t
        if self.method == "AVG":
            d = d * (1.0 / len(vecs))
        return [VectorUtil.toString(DenseVector(d))]

    def _map_columns(self, mt):
        """Packed documents with a one-byte delimiter: split on the device, each DISTINCT token looked up once,
        then the fold runs position by position over all documents at once (document d's k-th known word
        joins its vector at step k), so every vector is combined in the row path's order; the results are
        formatted by the C++ Double.toString rows."""
        from ... import _native
        from ...common.strings import StringBlock
        from ...common.table import Column
        from ...ops.strings import split_tokens, unique_ids
        col = mt.cols[self.col_idx]
        blk = col.values
        db = self.delim.encode("utf-8")
        if not (isinstance(blk, StringBlock) and col.nulls is None and len(blk) and len(db) == 1 and db[0] < 0x80
                and self.embed and self.method in ("AVG", "SUM", "MIN", "MAX")):
            return super()._map_columns(mt)
        tok, doc = split_tokens(blk, db[0])
        n = len(blk)
        dev = doc.device
        if len(tok):
            enc = unique_ids(tok)
            if enc is None:
                return super()._map_columns(mt)
            ids, rep = enc
            words = tok.take(rep).to_list()
            dim = len(next(iter(self.embed.values())))
            rows = [self.embed.get(w) for w in words]
            known_w = torch.tensor([r is not None for r in rows], dtype=torch.bool)
            E = torch.as_tensor(np.stack([r if r is not None else np.zeros(dim) for r in rows]), dtype=torch.float64,
                                device=dev)
            keep = known_w.to(dev)[ids]
            kid, kdoc = ids[keep], doc[keep]
        else:
            dim = len(next(iter(self.embed.values())))
            E = torch.zeros((1, dim), dtype=torch.float64, device=dev)
            kid = kdoc = torch.zeros(0, dtype=torch.int64, device=dev)
        cnt = torch.bincount(kdoc, minlength=n)
        first = torch.cumsum(cnt, 0) - cnt
        pos = torch.arange(kid.numel(), device=dev) - first[kdoc]
        D = torch.zeros((n, dim), dtype=torch.float64, device=dev)
        kmax = int(cnt.max()) if n else 0
        for k in range(kmax):
            sel = pos == k
            dk, vk = kdoc[sel], E[kid[sel]]
            if k == 0:
                D[dk] = vk
            elif self.method == "MIN":
                D[dk] = torch.minimum(D[dk], vk)
            elif self.method == "MAX":
                D[dk] = torch.maximum(D[dk], vk)
            else:
                D[dk] = D[dk] + vk
        if self.method == "AVG":
            D = D * (1.0 / cnt.clamp(min=1).to(torch.float64))[:, None]
        nulls = (cnt == 0).cpu()
        if blk.nulls is not None:
            nulls |= blk.nulls.cpu()
        r = _native.java_double_rows_packed(D.cpu().numpy(), " ")
        if r is None:
            return super()._map_columns(mt)
        b, o = np.asarray(r[0], dtype=np.uint8), r[1]
        nm = nulls.numpy()
        if nm.any():
            lens = o[1:] - o[:-1]
            b = b[np.repeat(~nm, lens)]
            o = np.zeros_like(o)
            np.cumsum(np.where(nm, 0, lens), out=o[1:])
        return [Column(StringBlock(torch.from_numpy(np.ascontiguousarray(b)), torch.from_numpy(o),
                                   torch.from_numpy(nm) if nm.any() else None))]
