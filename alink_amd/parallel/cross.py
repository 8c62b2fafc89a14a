"""Blockwise cross top-K over a ring of item blocks.

Reference: ``BlockwiseCross.findTopK`` (``A/operator/common/dataproc/BlockwiseCross.java:76-240``) tags every
record with its subtask, then runs a P-superstep bulk iteration: in superstep s the target block of subtask
``(t + s) % P`` is co-grouped with the query block of subtask t and every query's PriorityQueue absorbs it.

MI355X design: each rank (one GPU) keeps its query block resident and the item blocks travel around the ring
over RCCL point-to-point (``batch_isend_irecv`` to rank+1 / from rank-1 over xGMI).  The transfer of the next
block is posted before the current block is scored, so the xGMI hop overlaps the fused score + top-K kernel
(``ops/topk.py``); after P-1 hops every query has seen every item and no rank ever holds more than two item
blocks.  Global item ids are ``offset(owner) + row``.  With one rank this is one kernel launch.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist

from . import comm
from ..ops import topk as topk_ops

__all__ = ["blockwise_topk"]


def _comm_device(t: torch.Tensor) -> torch.device:
    if comm._backend() == "nccl":
        return comm.device_for_rank()
    return torch.device("cpu")


def blockwise_topk(Q: torch.Tensor, T_local: torch.Tensor, K: int, descending: bool = True,
                   use_kernel: bool = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Top-``K`` items of every local query ``Q`` [m, r] over the union of all ranks' item blocks.

    ``T_local`` is this rank's block [n_p, r]; the global id of its row i is ``sum(n_q for q < p) + i``.
    Returns ``(scores [m, K], ids [m, K] int64)`` sorted best first (ids -1 where fewer than K items exist).
    """
    dev = Q.device
    Qs = Q.to(torch.float32) if descending else -Q.to(torch.float32)
    state = topk_ops.TopKState(Q.shape[0], K, dev)
    ws, me = comm.get_world_size(), comm.get_rank()
    if ws == 1:
        topk_ops.merge(state, Qs, T_local.to(dev), 0, use_kernel)
    else:
        cdev = _comm_device(T_local)
        sizes = comm.all_gather_tensor(torch.tensor([T_local.shape[0]], dtype=torch.int64, device=cdev)).cpu()
        sizes = [int(x) for x in sizes.tolist()]
        offsets = [sum(sizes[:i]) for i in range(ws)]
        width = T_local.shape[1]
        cap = max(1, max(sizes))
        cur = torch.zeros((cap, width), dtype=torch.float32, device=cdev)
        cur[:sizes[me]] = T_local.to(device=cdev, dtype=torch.float32)
        nxt = torch.empty_like(cur)
        owner = me
        for step in range(ws):
            reqs = None
            if step < ws - 1:
                ops = [dist.P2POp(dist.isend, cur, (me + 1) % ws), dist.P2POp(dist.irecv, nxt, (me - 1) % ws)]
                reqs = dist.batch_isend_irecv(ops)
                comm.STATS.calls += 1
                comm.STATS.bytes += cur.numel() * cur.element_size()
            blk = cur[:sizes[owner]]
            topk_ops.merge(state, Qs, blk if blk.device == dev else blk.to(dev), offsets[owner], use_kernel)
            if reqs is not None:
                for r in reqs:
                    r.wait()
                if cdev.type == "cpu" and dev.type != "cpu":
                    torch.cuda.current_stream(dev).synchronize()
                # the block just scored is free: it becomes the receive buffer of the next hop
                cur, nxt = nxt, cur
                owner = (owner - 1) % ws
    v, i = topk_ops.finish(state)
    if not descending:
        v = -v
    return v, i.to(torch.int64)
