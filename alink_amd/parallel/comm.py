"""Collective communication for the SPMD runtime.

Reference: Alink's only collective is a shuffle-based ``AllReduce`` over Flink's network stack
(``A/common/comqueue/communication/AllReduce.java:42-360``) plus broadcast variables, keyed shuffles and
accumulator-based collect.  Here every partition is one process (one MI355X), and
collectives go through ``torch.distributed``:

* backend ``nccl`` (= RCCL over xGMI on ROCm) for device tensors — one process per GPU;
* a companion ``gloo`` group for host objects (row lists, model rows, small Python state), so object
  traffic never serialises through GPU memory;
* ``gloo`` alone for CPU-only runs / tests (the analogue of Flink's LocalEnvironment).

With world size 1 every call is a local no-op, unless ``ALINK_COMM_FORCE_COLLECTIVE=1``: then a 1-rank process
group is created (``init_distributed``) and every wrapper takes its real collective branch (RCCL on a GPU box,
gloo on the host).  That is how the RCCL branches of an 8-GPU job are exercised on a 1-GPU box: RCCL refuses two
ranks on one device ("Duplicate GPU detected"), but a 1-rank RCCL communicator runs every collective for real.
"""
from __future__ import annotations

import datetime
import functools
import os
import time
from typing import Any, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..utils import trace as _trace

__all__ = ["init_distributed", "get_rank", "get_world_size", "is_distributed", "all_reduce", "all_gather_object",
           "broadcast_object", "barrier", "all_gather_tensor", "all_to_all_objects", "reduce_scatter",
           "object_group", "device_for_rank", "CommStats", "STATS", "shutdown", "all_reduce_coalesced",
           "Pending", "reduce_scatter_async", "all_gather_varlen_async", "all_reduce_async", "all_to_all_bytes", "all_to_all_strings",
           "comm_stream", "force_collective", "device_timing", "device_timing_collect", "host_all_gather"]

_OBJ_GROUP = None


class CommStats:
    """Per-process counters: number of collectives and bytes reduced (observability)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.calls = 0
        self.bytes = 0
        self.oneshot = 0
        self.time_s = 0.0
        self.string_bytes = 0      # packed string bytes sent through all_to_all_strings

    def as_dict(self):
        return {"collectives": self.calls, "bytes": self.bytes, "oneshot": self.oneshot, "time_s": self.time_s,
                "string_bytes": self.string_bytes}


STATS = CommStats()


_DEV_TIMING = {"on": False, "events": [], "folded": (0, 0.0, {})}
_DEV_TIMING_MAX_PENDING = 1024       # older event pairs are resolved into running totals beyond this many


def _fold_events(evs, acc):
    n, tot, per = acc
    per = dict(per)
    for name, s, e in evs:
        e.synchronize()
        dt = s.elapsed_time(e) * 1e-3
        tot += dt
        per[name] = per.get(name, 0.0) + dt
    return n + len(evs), tot, per


def device_timing(on: bool = True):
    """Device-time every outermost collective on a device tensor: a timing event pair around it on the caller's
    stream (the span a compute kernel behind it waits for: RCCL on the comm stream or the one-shot kernel,
    including any wait for slower peers).  Read with ``device_timing_collect``."""
    _DEV_TIMING["on"] = bool(on)


def device_timing_collect():
    """(count, total seconds, per-name totals) of the collectives timed since the last collect; synchronises the
    recorded events."""
    evs, acc = _DEV_TIMING["events"], _DEV_TIMING["folded"]
    _DEV_TIMING["events"], _DEV_TIMING["folded"] = [], (0, 0.0, {})
    return _fold_events(evs, acc)


def _collective(fn):
    """Time a collective (host wall time into ``STATS.time_s``; a ``collective`` span with device timing on the
    tracer's gpu track when tracing is on; device events under ``device_timing``).  Nested collectives (e.g. the
    count exchange inside an all-to-all) are timed once, by the outermost call."""
    name = fn.__name__

    @functools.wraps(fn)
    def wrapper(*a, **kw):
        if not is_distributed():
            return fn(*a, **kw)
        if getattr(_NEST, "v", False):
            return fn(*a, **kw)
        t = a[0] if a and isinstance(a[0], torch.Tensor) else None
        _NEST.v = True
        t0 = time.perf_counter()
        ev = None
        if _DEV_TIMING["on"] and t is not None and t.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(torch.cuda.current_stream(t.device))
        try:
            if _trace.enabled():
                nb = int(t.numel() * t.element_size()) if t is not None else 0
                with _trace.span(name, "collective", device=t is not None and t.is_cuda, bytes=nb,
                                 backend=_backend()):
                    return fn(*a, **kw)
            return fn(*a, **kw)
        finally:
            if ev is not None:
                ev[1].record(torch.cuda.current_stream(t.device))
                evl = _DEV_TIMING["events"]
                evl.append((name, ev[0], ev[1]))
                if len(evl) > _DEV_TIMING_MAX_PENDING:     # bounded: a long timed job holds few live events
                    half = len(evl) // 2
                    _DEV_TIMING["folded"] = _fold_events(evl[:half], _DEV_TIMING["folded"])
                    del evl[:half]
            STATS.time_s += time.perf_counter() - t0
            _NEST.v = False
    return wrapper


import threading as _threading  # noqa: E402
_NEST = _threading.local()


def force_collective() -> bool:
    """``ALINK_COMM_FORCE_COLLECTIVE=1``: a 1-rank group still runs every collective (test / rehearsal switch)."""
    return os.environ.get("ALINK_COMM_FORCE_COLLECTIVE", "0") == "1"


def is_distributed() -> bool:
    """True when collectives must run: a multi-rank group, or any group under ``force_collective()``."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size() > 1 or force_collective()


def get_rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def get_world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def device_for_rank() -> torch.device:
    if torch.cuda.is_available():
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        return torch.device("cuda", lr % max(1, torch.cuda.device_count()))
    return torch.device("cpu")


def init_distributed(backend: Optional[str] = None, timeout_s: float = 1800.0) -> bool:
    """Initialise the default process group from torchrun env vars (RANK/WORLD_SIZE/MASTER_*).

    Returns True if a multi-process group is active.  Safe to call repeatedly.
    """
    global _OBJ_GROUP
    if not dist.is_available():
        return False
    if dist.is_initialized():
        return is_distributed()
    timeout_s = float(os.environ.get("ALINK_DIST_TIMEOUT_S", timeout_s))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1 and not force_collective():
        return False
    if ws <= 1:
        # forced 1-rank group (no launcher): rank 0 of 1 on a private rendezvous port
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("LOCAL_RANK", "0")
        if "MASTER_PORT" not in os.environ:
            import socket
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
    if backend is None:
        backend = os.environ.get("ALINK_DIST_BACKEND")
    if backend is None:
        cpu_only = os.environ.get("ALINK_DEVICE", "").startswith("cpu")
        # RCCL needs one GPU per rank: more local ranks than GPUs (a P-way local env on a smaller box) run their
        # collectives over gloo, with ranks sharing the GPUs round-robin for compute
        local_ws = int(os.environ.get("LOCAL_WORLD_SIZE", str(ws)))
        oversubscribed = torch.cuda.device_count() < local_ws
        backend = "nccl" if torch.cuda.is_available() and not cpu_only and not oversubscribed else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = {}
    if backend == "nccl":
        dev = device_for_rank()
        torch.cuda.set_device(dev)
        kw["device_id"] = dev
    dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    if backend != "gloo":
        _OBJ_GROUP = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))
    else:
        _OBJ_GROUP = None
    return is_distributed()


def shutdown():
    """Tear down the one-shot staging and the process groups.  A one-shot timeout on the job's LAST reduction
    (which no later call would check) is raised here, after the cleanup."""
    global _OBJ_GROUP
    from . import oneshot
    failure = None
    if oneshot._INSTANCE is not None:
        # peers may still be reading this rank's staging slot in their last one-shot call: drain every rank's
        # stream, meet on the host group, then unmap / free
        torch.cuda.synchronize(oneshot._INSTANCE.device)
        try:
            oneshot._INSTANCE.check(wait=True)
        except RuntimeError as e:
            failure = e
        if dist.is_available() and dist.is_initialized():
            dist.barrier(group=_OBJ_GROUP)
    oneshot.reset()
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _OBJ_GROUP = None
    _COMM_STREAMS.clear()
    if failure is not None:
        raise failure


def object_group():
    return _OBJ_GROUP


def collective_device() -> torch.device:
    """Where tensors must live for this job's collectives: the rank's GPU under RCCL, the host under gloo."""
    return device_for_rank() if _backend() == "nccl" else torch.device("cpu")


@_collective
def all_gather_arrays(arrays: List[np.ndarray], dtype=np.float64) -> List[List[np.ndarray]]:
    """Gather a list of variable-length 1-D arrays from every rank as TWO tensor collectives (lengths + one
    packed buffer over RCCL/gloo) instead of a pickled object gather: result[rank][j] = that rank's arrays[j]."""
    ws = get_world_size()
    if not is_distributed():
        return [list(arrays)]
    dev = collective_device()
    lens = torch.tensor([int(a.size) for a in arrays], dtype=torch.int64)
    flat = torch.from_numpy(np.ascontiguousarray(np.concatenate(arrays).astype(dtype)) if arrays else
                            np.zeros(0, dtype))
    all_lens = all_gather_tensor(lens.to(dev)).cpu().view(ws, len(arrays))
    all_flat = all_gather_varlen(flat.to(dev)).cpu().numpy()
    out, off = [], 0
    for r in range(ws):
        part = []
        for j in range(len(arrays)):
            n = int(all_lens[r, j])
            part.append(all_flat[off:off + n])
            off += n
        out.append(part)
    return out


def _backend() -> str:
    return dist.get_backend() if dist.is_initialized() else "none"


_OPS = {"sum": "SUM", "max": "MAX", "min": "MIN", "prod": "PRODUCT"}

# ---------------------------------------------------------------------------------------------------------
# Comm-stream discipline: every RCCL collective is issued from a dedicated high-priority
# communication stream per device.  The comm stream first waits on an event of the caller's (compute) stream
# -- the inputs are ready -- and the caller's stream later waits on an event recorded on the comm stream after
# the collective -- the outputs are ready.  Synchronous calls insert that wait immediately; ``*_async`` calls
# return a ``Pending`` whose ``wait()`` inserts it, so compute launched in between overlaps the collective.
# Tensors touched on the comm stream are ``record_stream``-ed so the caching allocator cannot recycle them early.
_COMM_STREAMS = {}


def comm_stream(dev: torch.device) -> "torch.cuda.Stream":
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _COMM_STREAMS.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=torch.device("cuda", idx), priority=-1)
        _COMM_STREAMS[idx] = s
    return s


def _on_comm_stream(dev: torch.device, tensors, issue, wait_now: bool = True):
    """Run ``issue()`` (which enqueues RCCL work) on the comm stream of ``dev``.  Returns (result, done event)."""
    cur = torch.cuda.current_stream(dev)
    cs = comm_stream(dev)
    ready = torch.cuda.Event()
    ready.record(cur)
    cs.wait_event(ready)
    with torch.cuda.stream(cs):
        res = issue()
        done = torch.cuda.Event()
        done.record(cs)
    for t in tensors:
        if t is not None and t.is_cuda:
            t.record_stream(cs)
    if wait_now:
        cur.wait_event(done)
    return res, done



def _oneshot_max(backend: str) -> int:
    from . import oneshot
    return oneshot.MAX_BYTES if oneshot.enabled(backend) else -1


@_collective
def all_reduce(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """In-place all-reduce of a tensor (SUM/MAX/MIN, reference ``AllReduce.java:125-159``).

    Device tensors use RCCL; on a gloo job, device tensors are staged through host memory.
    """
    if not is_distributed():
        return t
    rop = getattr(dist.ReduceOp, _OPS[op.lower()])
    STATS.calls += 1
    STATS.bytes += t.numel() * t.element_size()
    be = _backend()
    if t.is_cuda and op.lower() in ("sum", "max", "min") and t.dtype in (torch.float32, torch.float64) and \
            t.numel() * t.element_size() <= _oneshot_max(be):
        # small device buffers: one kernel over IPC-mapped peer memory (parallel/oneshot.py, K31) — default on
        # RCCL jobs; on gloo jobs whose ranks share a GPU only when forced (ALINK_ONESHOT_ALLREDUCE=1)
        from . import oneshot
        inst = oneshot.get()
        if inst is not None:
            STATS.oneshot += 1
            return inst.all_reduce_(t, op.lower())
    if t.is_cuda and _backend() != "nccl":
        h = t.cpu()
        dist.all_reduce(h, op=rop)
        t.copy_(h)
        return t
    if (not t.is_cuda) and _backend() == "nccl":
        d = t.to(device_for_rank())
        _on_comm_stream(d.device, [d], lambda: dist.all_reduce(d, op=rop))
        t.copy_(d.cpu())
        return t
    if t.is_cuda:
        _on_comm_stream(t.device, [t], lambda: dist.all_reduce(t, op=rop))
        return t
    dist.all_reduce(t, op=rop)
    return t


@_collective
def all_reduce_coalesced(ts: List[torch.Tensor], op: str = "sum") -> List[torch.Tensor]:
    """Fuse several small same-dtype buffers into one collective (latency-bound regime)."""
    if not is_distributed() or not ts:
        return ts
    flat = torch.cat([t.reshape(-1) for t in ts])
    all_reduce(flat, op)
    off = 0
    for t in ts:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n
    return ts


def scatter_block(n: int, ws: int, r: int):
    """Rows ``[lo, hi)`` of dim 0 that rank ``r`` owns after a reduce-scatter of ``n`` rows over ``ws`` ranks:
    blocks of ``ceil(n / ws)`` rows in rank order, the last ones shorter (possibly empty) when ``ws`` does not
    divide ``n``."""
    b = -(-n // ws)
    lo = min(n, r * b)
    return lo, min(n, lo + b)


def _rs_padded(t: torch.Tensor, ws: int) -> torch.Tensor:
    """``t`` zero-padded along dim 0 to a multiple of ``ws`` (the padding only ever lands in rows no rank keeps)."""
    n = t.shape[0]
    b = -(-n // ws)
    if b * ws == n:
        return t.contiguous()
    pad = torch.zeros((b * ws - n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    return torch.cat([t, pad], 0)


@_collective
def reduce_scatter(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """Reduce-scatter along dim 0; returns this rank's block ``scatter_block(t.shape[0], ws, rank)`` — any row
    count works: a non-divisible buffer is zero-padded to a multiple of the world size and the padding is cut
    off again, never silently dropping the remainder rows."""
    ws = get_world_size()
    if not is_distributed():
        return t
    rop = getattr(dist.ReduceOp, _OPS[op.lower()])
    n = t.shape[0]
    lo, hi = scatter_block(n, ws, get_rank())
    b = -(-n // ws)
    STATS.calls += 1
    STATS.bytes += t.numel() * t.element_size()
    if _backend() == "nccl":
        d = _rs_padded(t if t.is_cuda else t.to(device_for_rank()), ws)
        o = torch.empty((b,) + tuple(t.shape[1:]), dtype=t.dtype, device=d.device)
        _on_comm_stream(d.device, [d, o], lambda: dist.reduce_scatter_tensor(o, d, op=rop))
        o = o[:hi - lo]
        return o if t.is_cuda else o.cpu()
    full = t.clone()
    all_reduce(full, op)
    return full[lo:hi].clone()


def _wait_event(dev, ev, x):
    torch.cuda.current_stream(dev).wait_event(ev)
    return x


class Pending:
    """Handle of an in-flight collective (``*_async``).  Under RCCL the collective is issued from the dedicated
    comm stream (``comm_stream``) after an event wait on the caller's stream, so kernels the caller launches
    afterwards overlap with it; ``wait()`` makes the caller's current stream wait on the event recorded on the
    comm stream after the collective (no host block) and returns the result.  Under gloo the collective runs
    on gloo's thread and ``wait()`` joins it."""

    __slots__ = ("_work", "_result", "_post", "_keep")

    def __init__(self, result, work=None, post=None, keep=()):
        self._work = work
        self._result = result
        self._post = post
        self._keep = keep            # inputs must outlive the collective

    def wait(self) -> torch.Tensor:
        if self._work is not None:
            self._work.wait()
            self._work = None
        if self._post is not None:
            self._result = self._post(self._result)
            self._post = None
        self._keep = ()
        return self._result


def reduce_scatter_async(t: torch.Tensor, op: str = "sum") -> Pending:
    """Asynchronous ``reduce_scatter`` (dim 0 split over ranks as ``scatter_block``; any row count): returns a
    ``Pending`` whose ``wait()`` yields this rank's block.  Used to overlap per-block histogram reductions with building the next block."""
    ws = get_world_size()
    if not is_distributed():
        return Pending(t)
    rop = getattr(dist.ReduceOp, _OPS[op.lower()])
    STATS.calls += 1
    STATS.bytes += t.numel() * t.element_size()
    n = t.shape[0]
    lo, hi = scatter_block(n, ws, get_rank())
    rows = -(-n // ws)
    if _backend() == "nccl":
        d = _rs_padded(t if t.is_cuda else t.to(device_for_rank()), ws)
        o_full = torch.empty((rows,) + tuple(t.shape[1:]), dtype=t.dtype, device=d.device)
        o = o_full[:hi - lo]

        def issue():
            w = dist.reduce_scatter_tensor(o_full, d, op=rop, async_op=True)
            w.wait()                         # comm stream waits on RCCL's stream (no host block)
        _, done = _on_comm_stream(d.device, [d, o_full], issue, wait_now=False)
        dev = d.device
        return Pending(o, None, (lambda x: _wait_event(dev, done, x)) if t.is_cuda else
                       (lambda x: _wait_event(dev, done, x).cpu()), keep=(d,))
    full = t.detach().cpu().clone()
    work = dist.all_reduce(full, op=rop, async_op=True)
    dev = t.device
    return Pending(full, work, lambda x: x[lo:hi].clone().to(dev))


def all_reduce_async(t: torch.Tensor, op: str = "sum") -> Pending:
    """Asynchronous in-place ``all_reduce``: issued from the comm stream (RCCL) or gloo's thread; ``wait()``
    returns ``t`` holding the reduction (the caller's stream waits on the collective's event)."""
    if not is_distributed():
        return Pending(t)
    rop = getattr(dist.ReduceOp, _OPS[op.lower()])
    STATS.calls += 1
    STATS.bytes += t.numel() * t.element_size()
    if _backend() == "nccl":
        d = t if t.is_cuda else t.to(device_for_rank())

        def issue():
            w = dist.all_reduce(d, op=rop, async_op=True)
            w.wait()
        _, done = _on_comm_stream(d.device, [d], issue, wait_now=False)
        dev = d.device
        if t.is_cuda:
            return Pending(t, None, lambda x: _wait_event(dev, done, x))
        return Pending(t, None, lambda x: x.copy_(_wait_event(dev, done, d).cpu()))
    h = t if not t.is_cuda else t.cpu()
    work = dist.all_reduce(h, op=rop, async_op=True)
    return Pending(t, work, (lambda x: x) if h is t else (lambda x: x.copy_(h)), keep=(h,))


def all_gather_varlen_async(t: torch.Tensor) -> Pending:
    """Asynchronous ``all_gather_varlen``: the (tiny) length exchange runs now, the padded payload gather is
    issued from the comm stream (RCCL) or gloo's thread; ``wait()`` returns the rank-order concatenation."""
    ws = get_world_size()
    if not is_distributed():
        return Pending(t)
    n = torch.tensor([t.shape[0]], dtype=torch.int64)
    lens = all_gather_tensor(n).tolist()
    mx = max(lens)
    tail = tuple(t.shape[1:])
    STATS.calls += 1
    STATS.bytes += int(mx * ws * (t.element_size() * (int(np.prod(tail)) if tail else 1)))

    def unpad(full):
        return torch.cat([full[i * mx:i * mx + lens[i]] for i in range(ws)])
    if _backend() == "nccl":
        d = t if t.is_cuda else t.to(device_for_rank())
        pad = torch.zeros((mx,) + tail, dtype=t.dtype, device=d.device)
        pad[:t.shape[0]] = d
        out = torch.empty((ws * mx,) + tail, dtype=t.dtype, device=d.device)

        def issue():
            w = dist.all_gather_into_tensor(out, pad, async_op=True)
            w.wait()
        _, done = _on_comm_stream(d.device, [pad, out], issue, wait_now=False)
        dev, host = d.device, not t.is_cuda
        return Pending(out, None, lambda x: (lambda y: y.cpu() if host else y)(unpad(_wait_event(dev, done, x))),
                       keep=(pad,))
    pad = torch.zeros((mx,) + tail, dtype=t.dtype)
    pad[:t.shape[0]] = t.cpu()
    parts = [torch.empty_like(pad) for _ in range(ws)]
    work = dist.all_gather(parts, pad, async_op=True)
    dev = t.device
    return Pending(parts, work, lambda ps: unpad(torch.cat(ps)).to(dev), keep=(pad,))


@_collective
def all_gather_tensor(t: torch.Tensor) -> torch.Tensor:
    """Concatenate equally-shaped tensors from all ranks along dim 0."""
    ws = get_world_size()
    if not is_distributed():
        return t
    STATS.calls += 1
    if _backend() == "nccl":
        # RCCL has no host path: host inputs are staged through the rank's GPU and the result returned on the host
        d = (t if t.is_cuda else t.to(device_for_rank())).contiguous()
        out = torch.empty((ws * d.shape[0],) + tuple(d.shape[1:]), dtype=d.dtype, device=d.device)
        _on_comm_stream(d.device, [d, out], lambda: dist.all_gather_into_tensor(out, d))
        return out if t.is_cuda else out.cpu()
    parts = [torch.empty_like(t.cpu()) for _ in range(ws)]
    dist.all_gather(parts, t.cpu().contiguous())
    return torch.cat(parts).to(t.device)


@_collective
def host_all_gather(t: torch.Tensor) -> torch.Tensor:
    """All-gather of a small HOST tensor over the host (gloo) group — the control plane of lockstep loops
    (liveness flags, per-rank counts).  Under RCCL this never touches the device: no H2D / D2H copy and no
    synchronisation of the rank's GPU stream, so queued kernels keep running while the ranks agree."""
    ws = get_world_size()
    if not is_distributed():
        return t
    STATS.calls += 1
    h = t.detach().cpu().contiguous()
    parts = [torch.empty_like(h) for _ in range(ws)]
    dist.all_gather(parts, h, group=_OBJ_GROUP)
    return torch.cat(parts)


@_collective
def all_gather_varlen(t: torch.Tensor, lens: Optional[List[int]] = None) -> torch.Tensor:
    """Concatenate tensors whose dim-0 length differs per rank (pads to the max length, one collective).
    ``lens`` (every rank's length, when the caller already knows them) skips the length exchange."""
    ws = get_world_size()
    if not is_distributed():
        return t
    if lens is None:
        n = torch.tensor([t.shape[0]], dtype=torch.int64)
        lens = all_gather_tensor(n).tolist()
    mx = max(lens)
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[:t.shape[0]] = t
    full = all_gather_tensor(pad)
    return torch.cat([full[i * mx:i * mx + lens[i]] for i in range(ws)])


@_collective
def all_to_all_tensors(send: List[torch.Tensor]) -> List[torch.Tensor]:
    """Tensor all-to-all (``send[j]`` -> rank j; same trailing shape/dtype): one ``all_to_all_single`` after a
    count exchange.  This is the request/response shuffle of the reference's ALS (``AlsTrain.java:283-389``)
    done as a single RCCL all-to-all(v)."""
    ws = get_world_size()
    if not is_distributed():
        return [send[0]]
    dev = send[0].device
    tail = tuple(send[0].shape[1:])
    counts = torch.tensor([x.shape[0] for x in send], dtype=torch.int64)
    all_counts = all_gather_tensor(counts).view(ws, ws)
    recv_counts = all_counts[:, get_rank()].tolist()
    width = int(np.prod(tail)) if tail else 1
    flat = torch.cat([x.reshape(x.shape[0], width) for x in send]) if send else torch.empty(0)
    STATS.calls += 1
    STATS.bytes += int(flat.numel() * flat.element_size())
    if _backend() == "nccl":
        cdev = dev if dev.type == "cuda" else device_for_rank()
        out = torch.empty((sum(recv_counts), width), dtype=flat.dtype, device=cdev)
        src = flat.reshape(-1, width).to(cdev).contiguous()
        _on_comm_stream(cdev, [src, out], lambda: dist.all_to_all_single(out, src, recv_counts, counts.tolist()))
        out = out.to(dev)
    else:
        out = torch.empty((sum(recv_counts), width), dtype=flat.dtype)
        dist.all_to_all_single(out, flat.reshape(-1, width).cpu().contiguous(), recv_counts, counts.tolist())
        out = out.to(dev)
    res = list(torch.split(out, recv_counts))
    return [x.reshape((x.shape[0],) + tail) for x in res]


@_collective
def all_gather_object(obj: Any) -> List[Any]:
    ws = get_world_size()
    if not is_distributed():
        return [obj]
    out: List[Any] = [None] * ws
    STATS.calls += 1
    dist.all_gather_object(out, obj, group=_OBJ_GROUP)
    return out


@_collective
def broadcast_object(obj: Any, src: int = 0) -> Any:
    if not is_distributed():
        return obj
    box = [obj]
    STATS.calls += 1
    dist.broadcast_object_list(box, src=src, group=_OBJ_GROUP)
    return box[0]


def _is_str_list(x) -> bool:
    return isinstance(x, list) and all(v is None or isinstance(v, str) for v in x)


@_collective
def all_to_all_bytes(send: List[bytes]) -> List[bytes]:
    """Byte-string all-to-all: ``send[j]`` -> rank j, as one lengths + one packed uint8 ``all_to_all_single``
    (RCCL / gloo) — O(N) bytes in total, no gather of every rank's data on every rank."""
    ws = get_world_size()
    if not is_distributed():
        return [send[0]]
    dev = collective_device()
    lens = [torch.tensor([len(b)], dtype=torch.int64, device=dev) for b in send]
    parts = [torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev) if len(b) else
             torch.zeros(0, dtype=torch.uint8, device=dev) for b in send]
    rl = torch.cat(all_to_all_tensors(lens)).cpu().tolist()
    rb = torch.cat(all_to_all_tensors(parts)).cpu().numpy().tobytes()
    out, off = [], 0
    for n in rl:
        out.append(rb[off:off + n])
        off += n
    return out


def all_to_all_objects(send: List[Any]) -> List[Any]:
    """Object all-to-all: ``send[j]`` goes to rank j; returns the list received from every rank.  Lists of
    strings travel as packed UTF-8 (lengths, -1 = None, + bytes); anything else as one pickled byte string per
    destination — both as tensor all-to-alls whose total traffic is the data itself."""
    ws = get_world_size()
    if not is_distributed():
        return list(send)
    if all(_is_str_list(p) for p in send):
        flags = all_gather_object(True)
        if all(flags):
            from ..common.strings import StringBlock
            blocks = [StringBlock.from_list(p) for p in send]
            got = all_to_all_strings(blocks)
            return [b.to_list() for b in got]
    else:
        all_gather_object(False)
    import pickle
    payload = [pickle.dumps(p, protocol=pickle.HIGHEST_PROTOCOL) for p in send]
    # bytes produced by this job's own ranks (never external input)
    return [pickle.loads(b) for b in all_to_all_bytes(payload)]


def all_to_all_strings(send) -> list:
    """``StringBlock`` all-to-all: ``send[j]`` -> rank j; returns the blocks received from every rank (source
    order).  Two tensor all-to-alls: per-string byte lengths (-1 marks NULL) and the concatenated bytes."""
    from ..common.strings import StringBlock
    ws = get_world_size()
    if not is_distributed():
        return [send[0]]
    lens = [torch.where(b.null_mask(), torch.full_like(b.lengths(), -1), b.lengths()) for b in send]
    rl = all_to_all_tensors(lens)
    rb = all_to_all_tensors([b.data for b in send])
    out = []
    for L, B in zip(rl, rb):
        nulls = L < 0
        out.append(StringBlock.from_parts(L.clamp(min=0), B, nulls if bool(nulls.any()) else None))
    STATS.string_bytes += sum(b.nbytes for b in send)
    return out


@_collective
def barrier():
    if is_distributed():
        if _backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()
