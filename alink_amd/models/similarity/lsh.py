"""Locality-sensitive hashing: approximate similarity join and top-N nearest neighbours.

Reference: ``A/operator/common/feature/{BaseLSH,MinHashLSH,BucketRandomProjectionLSH,
LocalitySensitiveHashApproxFunctions}.java`` — ``BaseLSH.tableHash`` = Guava ``murmur3_32(0).hashBytes`` of the
big-endian bytes of a table's hash values :63-76; MinHash coefficients ``A = 1 + nextInt(P-1)``,
``B = nextInt(P-1)`` from ``Random(seed)`` :21-31; bucket random projection = unit Gaussian directions and
offsets ``nextDouble()*w`` :21-38; join = equal (table, bucket) candidates, exact distance, ``d < threshold``
:134-225; top-N = per-query sort by distance, rank from 1 :230-262.

MI355X-first: the projections of all rows onto all ``numHashTables x numProjectionsPerTable`` directions are
ONE GEMM on the device; candidate pairs are formed by a bucket hash join on the host-side int keys and their
exact distances are evaluated in one batched gather + reduction on the device.
"""
from __future__ import annotations

from collections import defaultdict
from typing import List, Sequence, Tuple

import numpy as np
import torch

from ...common.jrandom import JavaRandom
from ...common.linalg import DenseVector, SparseVector, VectorUtil

__all__ = ["murmur3_32_words", "MinHashLSH", "BucketRandomProjectionLSH", "approx_similarity_join",
           "approx_nearest_neighbors", "jaccard_distance_sets"]

HASH_PRIME = 2038074743
_M32 = np.uint64(0xFFFFFFFF)


def _rotl(x, r):
    return ((x << np.uint64(r)) | (x >> np.uint64(32 - r))) & _M32


def murmur3_32_words(words: np.ndarray) -> np.ndarray:
    """Guava ``murmur3_32(0).hashBytes`` of each row's int32 values written big-endian (``intToByte4``),
    vectorised over rows; returns signed int32 (``asInt``)."""
    w = np.ascontiguousarray(words, dtype=np.int64) & 0xFFFFFFFF
    n, m = w.shape
    c1, c2 = np.uint64(0xCC9E2D51), np.uint64(0x1B873593)
    h = np.zeros(n, dtype=np.uint64)
    for j in range(m):
        v = w[:, j].astype(np.uint64)
        # big-endian bytes read as a little-endian block == byte swap
        k = (((v & np.uint64(0xFF)) << np.uint64(24)) | (((v >> np.uint64(8)) & np.uint64(0xFF)) << np.uint64(16))
             | (((v >> np.uint64(16)) & np.uint64(0xFF)) << np.uint64(8)) | (v >> np.uint64(24)))
        k = (k * c1) & _M32
        k = _rotl(k, 15)
        k = (k * c2) & _M32
        h ^= k
        h = _rotl(h, 13)
        h = (h * np.uint64(5) + np.uint64(0xE6546B64)) & _M32
    h ^= np.uint64(4 * m)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & _M32
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & _M32
    h ^= h >> np.uint64(16)
    return h.astype(np.int64).astype(np.uint32).view(np.int32).astype(np.int64)


class _Rows:
    """Rows of vectors as CSR (indices/values) + optional dense block."""

    def __init__(self, vecs: Sequence):
        vs = [VectorUtil.getVector(v) for v in vecs]
        self.n = len(vs)
        self.size = 0
        idx, val, ptr = [], [], [0]
        for v in vs:
            if isinstance(v, SparseVector):
                ii = np.asarray(v.getIndices(), dtype=np.int64)
                vv = np.asarray(v.getValues(), dtype=np.float64)
                self.size = max(self.size, v.size() if v.size() > 0 else (int(ii.max()) + 1 if len(ii) else 0))
            else:
                a = np.asarray(v.getData(), dtype=np.float64)
                ii = np.nonzero(a)[0].astype(np.int64)
                vv = a[ii]
                self.size = max(self.size, a.shape[0])
            keep = vv != 0
            idx.append(ii[keep])
            val.append(vv[keep])
            ptr.append(ptr[-1] + int(keep.sum()))
        self.ptr = np.asarray(ptr, dtype=np.int64)
        self.idx = np.concatenate(idx) if idx else np.zeros(0, dtype=np.int64)
        self.val = np.concatenate(val) if val else np.zeros(0, dtype=np.float64)

    def dense(self, d: int, device) -> torch.Tensor:
        out = torch.zeros((self.n, d), dtype=torch.float64, device=device)
        if self.idx.size:
            rows = np.repeat(np.arange(self.n), np.diff(self.ptr))
            sel = self.idx < d
            out[torch.as_tensor(rows[sel], device=device), torch.as_tensor(self.idx[sel], device=device)] = \
                torch.as_tensor(self.val[sel], device=device)
        return out


class MinHashLSH:
    def __init__(self, seed: int, num_proj: int, num_tables: int):
        rnd = JavaRandom(seed)
        self.A = np.zeros((num_tables, num_proj), dtype=np.int64)
        self.B = np.zeros((num_tables, num_proj), dtype=np.int64)
        for i in range(num_tables):
            for j in range(num_proj):
                self.A[i, j] = 1 + rnd.nextInt(HASH_PRIME - 1)
                self.B[i, j] = rnd.nextInt(HASH_PRIME - 1)

    def hash(self, rows: _Rows, device=None) -> np.ndarray:
        T, P = self.A.shape
        out = np.zeros((rows.n, T), dtype=np.int64)
        counts = np.diff(rows.ptr)
        for i in range(T):
            hv = np.full((rows.n, P), HASH_PRIME, dtype=np.int64)
            if rows.idx.size:
                # the reference's (int)((1L + index) * a + b) % HASH_PRIME: the cast to int comes first (the
                # product wraps to 32 bits), then Java's truncating remainder, which keeps the sign
                v = (1 + rows.idx.astype(np.int64))[:, None] * self.A[i][None, :] + self.B[i][None, :]
                w = ((v + (1 << 31)) % (1 << 32)) - (1 << 31)
                cur = np.fmod(w, HASH_PRIME)
                nz = counts > 0
                starts = rows.ptr[:-1][nz]
                hv[nz] = np.minimum.reduceat(cur, starts, axis=0)
            out[:, i] = murmur3_32_words(hv)
        return out

    @staticmethod
    def distance(a_rows: _Rows, ai: np.ndarray, b_rows: _Rows, bi: np.ndarray) -> np.ndarray:
        return np.asarray([jaccard_distance_sets(
            a_rows.idx[a_rows.ptr[x]:a_rows.ptr[x + 1]], b_rows.idx[b_rows.ptr[y]:b_rows.ptr[y + 1]])
            for x, y in zip(ai, bi)], dtype=np.float64)


def jaccard_distance_sets(a: np.ndarray, b: np.ndarray) -> float:
    if len(a) == 0 and len(b) == 0:
        return 0.0
    inter = len(np.intersect1d(a, b, assume_unique=True))
    union = len(a) + len(b) - inter
    return 1.0 - inter / union


class BucketRandomProjectionLSH:
    def __init__(self, seed: int, vector_size: int, num_proj: int, num_tables: int, width: float):
        rnd = JavaRandom(seed)
        self.width = float(width)
        self.R = np.zeros((num_tables, num_proj, vector_size))
        self.r = np.zeros((num_tables, num_proj))
        for i in range(num_tables):
            for j in range(num_proj):
                d = np.asarray([rnd.nextGaussian() for _ in range(vector_size)])
                nrm = np.linalg.norm(d)
                self.R[i, j] = d / nrm if nrm > 0 else d
                self.r[i, j] = rnd.nextDouble() * self.width

    def hash(self, rows: _Rows, device) -> np.ndarray:
        T, P, d = self.R.shape
        X = rows.dense(d, device)
        dots = X @ torch.as_tensor(self.R.reshape(T * P, d).T, device=device)      # one GEMM
        hv = torch.floor((dots + torch.as_tensor(self.r.reshape(-1), device=device)) / self.width)
        hv = hv.to(torch.int64).cpu().numpy().reshape(rows.n, T, P)
        return np.stack([murmur3_32_words(hv[:, i, :]) for i in range(T)], 1)

    def distance_fn(self, device):
        def fn(a_rows: _Rows, ai, b_rows: _Rows, bi):
            if len(ai) == 0:
                return np.zeros(0)
            d = max(a_rows.size, b_rows.size, self.R.shape[2])
            A = a_rows.dense(d, device)
            B = b_rows.dense(d, device)
            ta = torch.as_tensor(ai, device=device)
            tb = torch.as_tensor(bi, device=device)
            return torch.linalg.norm(A[ta] - B[tb], dim=1).cpu().numpy()
        return fn


def _candidates(ha: np.ndarray, hb: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Distinct (a, b) pairs sharing a bucket in at least one table (the join of ``HashData`` outputs)."""
    pairs = set()
    for t in range(ha.shape[1]):
        buckets = defaultdict(list)
        for j, h in enumerate(hb[:, t].tolist()):
            buckets[h].append(j)
        for i, h in enumerate(ha[:, t].tolist()):
            for j in buckets.get(h, ()):
                pairs.add((i, j))
    if not pairs:
        return np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.int64)
    arr = np.asarray(sorted(pairs), dtype=np.int64)
    return arr[:, 0], arr[:, 1]


def _build(distance_type: str, seed, num_proj, num_tables, width, left: _Rows, device):
    if distance_type.upper() == "JACCARD":
        lsh = MinHashLSH(seed, num_proj, num_tables)
        return lsh, MinHashLSH.distance
    lsh = BucketRandomProjectionLSH(seed, left.size, num_proj, num_tables, width)
    return lsh, lsh.distance_fn(device)


def approx_similarity_join(left_vecs, right_vecs, distance_type, seed, num_proj, num_tables, width, threshold,
                           device) -> List[Tuple[int, int, float]]:
    L, R = _Rows(left_vecs), _Rows(right_vecs)
    lsh, dist = _build(distance_type, seed, num_proj, num_tables, width, L, device)
    ai, bi = _candidates(lsh.hash(L, device), lsh.hash(R, device))
    d = dist(L, ai, R, bi)
    keep = d < threshold
    return list(zip(ai[keep].tolist(), bi[keep].tolist(), d[keep].tolist()))


def approx_nearest_neighbors(query_vecs, dict_vecs, distance_type, seed, num_proj, num_tables, width, top_n,
                             device, lsh_basis_vecs=None) -> List[Tuple[int, int, float, int]]:
    """(query index, dict index, distance, rank) for the ``top_n`` nearest candidates of every query."""
    Q, D = _Rows(query_vecs), _Rows(dict_vecs)
    basis = _Rows(lsh_basis_vecs) if lsh_basis_vecs is not None else D
    lsh, dist = _build(distance_type, seed, num_proj, num_tables, width, basis, device)
    qi, di = _candidates(lsh.hash(Q, device), lsh.hash(D, device))
    d = dist(Q, qi, D, di)
    per = defaultdict(list)
    for a, b, x in zip(qi.tolist(), di.tolist(), d.tolist()):
        per[a].append((x, b))
    out = []
    for a in sorted(per):
        lst = sorted(per[a], key=lambda t: t[0])
        for rank, (x, b) in enumerate(lst[:top_n], start=1):
            out.append((a, b, x, rank))
    return out
