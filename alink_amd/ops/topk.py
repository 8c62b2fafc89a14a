"""Running top-K of query·item scores over item blocks.

``TopKState(m, K)`` holds the per-query best scores / item ids; ``merge(state, Q, T, item_base)`` folds the
item block ``T`` (global ids ``item_base + row``) into it; ``finish(state)`` returns rows sorted by
descending score (reference ``BlockwiseCross.findTopK`` pops its PriorityQueue into descending arrays,
``A/operator/common/dataproc/BlockwiseCross.java:221-236``).

GPU: ``alink_topk_cross_f32`` (``csrc/topk.hip``) — f32 MFMA scores against LDS-staged item chunks with the
top-K held in LDS; the score matrix never reaches HBM.  CPU (or rank > 64 / K > 128): chunked GEMM +
``torch.topk`` over [state | block scores].  Ascending order is the same computation on ``-Q``.
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["TopKState", "merge", "finish", "kernel_supported", "pad_rank"]

KMAX = 128
QB = 128            # queries per workgroup (csrc/topk.hip)
WANT_WG = 512       # 2 workgroups per CU on 256 CUs
NEG = float("-inf")


def pad_rank(r: int) -> int:
    return max(16, (r + 15) // 16 * 16)


def kernel_supported(Q: torch.Tensor, K: int) -> bool:
    return Q.is_cuda and pad_rank(Q.shape[1]) <= 64 and 1 <= K <= KMAX and \
        (_lib.available() or not _lib.torch_fallback_allowed())


class TopKState:
    def __init__(self, m: int, K: int, device):
        self.K = int(K)
        self.val = torch.full((m, self.K), NEG, dtype=torch.float32, device=device)
        self.idx = torch.full((m, self.K), -1, dtype=torch.int32, device=device)


def _pad(x: torch.Tensor, R: int) -> torch.Tensor:
    x = x.to(torch.float32)
    if x.shape[1] == R and x.is_contiguous():
        return x
    out = torch.zeros((x.shape[0], R), dtype=torch.float32, device=x.device)
    out[:, :x.shape[1]] = x
    return out


def merge(state: TopKState, Q: torch.Tensor, T: torch.Tensor, item_base: int = 0,
          use_kernel: bool = None) -> TopKState:
    """Fold item block ``T`` [n, r] into the top-K of queries ``Q`` [m, r]."""
    m, n = Q.shape[0], T.shape[0]
    if m == 0 or n == 0:
        return state
    if use_kernel is None:
        use_kernel = kernel_supported(Q, state.K)
    if use_kernel:
        L = _lib.require()
        R = pad_rank(Q.shape[1])
        Qp, Tp = _pad(Q, R), _pad(T.to(Q.device), R)
        # split the items too when the query blocks alone cannot fill the chip (>= 2 workgroups per CU)
        qblocks = (m + QB - 1) // QB
        slices = max(1, min(WANT_WG // qblocks, (n + 4095) // 4096))
        per = ((n + slices - 1) // slices + 63) // 64 * 64
        slices = (n + per - 1) // per
        if slices == 1:
            val, idx = state.val, state.idx
        else:
            val = torch.full((slices, m, state.K), NEG, dtype=torch.float32, device=Q.device)
            idx = torch.full((slices, m, state.K), -1, dtype=torch.int32, device=Q.device)
            val[0].copy_(state.val)
            idx[0].copy_(state.idx)
        rc = L.alink_topk_cross_f32(Qp.data_ptr(), m, Tp.data_ptr(), n, int(item_base), R, state.K,
                                    val.data_ptr(), idx.data_ptr(), slices, per, _lib.stream_ptr(Q.device))
        if rc != 0:
            raise RuntimeError(f"alink_topk_cross_f32 failed: {rc}")
        if slices > 1:
            # plane order = item order, and a stable sort keeps the earlier plane on equal scores
            allv = val.permute(1, 0, 2).reshape(m, slices * state.K)
            alli = idx.permute(1, 0, 2).reshape(m, slices * state.K)
            order = torch.sort(allv, dim=1, descending=True, stable=True).indices[:, :state.K]
            state.val = torch.gather(allv, 1, order)
            state.idx = torch.gather(alli, 1, order)
        return state
    Qf = Q.to(torch.float32)
    Tf = T.to(device=Q.device, dtype=torch.float32)
    chunk = max(1, (1 << 26) // max(1, n))
    for s in range(0, m, chunk):
        sc = Qf[s:s + chunk] @ Tf.T
        kk = min(state.K, n)
        v, i = torch.topk(sc, kk, dim=1)
        allv = torch.cat([state.val[s:s + chunk], v], 1)
        alli = torch.cat([state.idx[s:s + chunk], (i + item_base).to(torch.int32)], 1)
        # stable descending sort: on equal scores the entry already in the state (earlier block) wins
        order = torch.sort(allv, dim=1, descending=True, stable=True).indices[:, :state.K]
        state.val[s:s + chunk] = torch.gather(allv, 1, order)
        state.idx[s:s + chunk] = torch.gather(alli, 1, order)
    return state


def finish(state: TopKState):
    """(values, ids) sorted by descending score; unfilled slots (fewer than K items) have id -1."""
    v, order = torch.sort(state.val, dim=1, descending=True, stable=True)
    return v, torch.gather(state.idx, 1, order)
