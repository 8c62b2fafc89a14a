"""One-shot xGMI all-reduce for small buffers (kernel ``ops/csrc/allreduce.hip``).

Every rank allocates an uncached staging area (two slots of ``cap_bytes`` + per-block flags), exports it with
``hipIpcGetMemHandle``, the handles are exchanged once over the host (gloo) group and opened on every peer.  An
all-reduce is then one kernel on the caller's stream: copy-in, release a sequence number to every peer, poll
the own flags (wrap-safe: a flag at or past the call's sequence number counts), sum the P staging slots in rank order (for P <= 8 the P remote loads of an element are issued
together, so a slice costs one xGMI round trip, not P).  No RCCL call, no host round trip, bit-identical results
on all ranks.

Used by ``comm.all_reduce`` for device tensors of at most ``ALINK_ONESHOT_MAX_BYTES`` (default 1 MiB):

* ``ALINK_ONESHOT_ALLREDUCE`` unset / ``auto`` (default): on ``nccl`` (RCCL) jobs;
* ``1``: also on ``gloo`` jobs whose ranks hold device tensors (several ranks sharing a GPU — the multi-process
  rehearsal of an 8-GPU job on one card; the IPC handles are real either way);
* ``0``: never (RCCL / gloo for everything).

Setup is collective and validated on a probe buffer against the exact rank-order sum; if any rank fails, every
rank disables the path (the decision is agreed by a MIN all-reduce over the host group, so ranks never diverge
between the two implementations).  A peer that does not arrive within ``ALINK_ONESHOT_TIMEOUT_S`` (300 s) makes
the kernel write NaN and set an error word, on the device and in a mapped pinned host word; the host polls the
host word (a plain memory read, no copy) at the start of every call and raises (``ALINK_ONESHOT_CHECK=1``:
synchronously, on the same call).  The reduction runs in place on the caller's tensor: each workgroup copies its
slice to the staging slot before signalling and writes the same slice of the result only after every rank's
signal.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import torch

from ..ops import _lib

__all__ = ["OneShot", "get", "enabled", "MAX_BYTES"]

MAX_BYTES = int(os.environ.get("ALINK_ONESHOT_MAX_BYTES", str(1 << 20)))
BLOCKS = 64
TIMEOUT_S = float(os.environ.get("ALINK_ONESHOT_TIMEOUT_S", "300"))
# the setup probe waits at most this long for peers: a node whose cross-GPU stores never become visible falls back
# to RCCL after seconds instead of stalling the job for TIMEOUT_S
PROBE_TIMEOUT_S = float(os.environ.get("ALINK_ONESHOT_PROBE_TIMEOUT_S", "20"))
SYNC_CHECK = os.environ.get("ALINK_ONESHOT_CHECK", "0") == "1"
_DT = {torch.float32: 0, torch.float64: 1}
_OP = {"sum": 0, "max": 1, "min": 2}


def _sigs(L):
    c_vp, c_i64, c_int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    L.alink_ar_alloc.argtypes = [c_i64, ctypes.POINTER(c_vp)]
    L.alink_ar_ipc_handle.argtypes = [c_vp, c_vp]
    L.alink_ar_ipc_open.argtypes = [c_vp, ctypes.POINTER(c_vp)]
    L.alink_ar_ipc_close.argtypes = [c_vp]
    L.alink_ar_free.argtypes = [c_vp]
    L.alink_oneshot_allreduce.argtypes = [c_vp, c_vp, c_i64, c_int, c_int, c_int, c_int, ctypes.c_uint32, c_vp, c_vp,
                                          c_i64, c_int, c_int, ctypes.c_double, c_vp, c_vp, c_vp]
    L.alink_ar_host_word_alloc.argtypes = [ctypes.POINTER(c_vp), ctypes.POINTER(c_vp)]
    L.alink_ar_host_word_free.argtypes = [c_vp]
    for f in ("alink_ar_alloc", "alink_ar_ipc_handle", "alink_ar_ipc_open", "alink_ar_ipc_close", "alink_ar_free",
              "alink_oneshot_allreduce", "alink_ar_handle_size", "alink_ar_host_word_alloc", "alink_ar_host_word_free"):
        getattr(L, f).restype = c_int


class OneShot:
    """Staging buffers + peer tables for ``P`` ranks.  ``bases[p]`` are device addresses valid in this process
    (IPC-opened for peers, own allocation for ``rank``); a single process may also pass P local allocations
    (single-GPU tests of the reduction)."""

    def __init__(self, device, P: int, rank: int, cap_bytes: int, bases: List[int], owned: List[int],
                 opened: List[int]):
        self.L = _lib.require()
        _sigs(self.L)
        self.device, self.P, self.rank, self.cap = device, P, rank, int(cap_bytes)
        self.owned, self.opened = owned, opened
        self.flag_off = 2 * self.cap
        self.peer_data = torch.tensor(bases, dtype=torch.int64, device=device)
        self.peer_flags = torch.tensor([b + self.flag_off for b in bases], dtype=torch.int64, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        # the kernel also sets a mapped host word on a timeout, so the per-call check is a host read (no copy)
        self._hword, self._hword_dev, self._hview = None, None, None
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        if self.L.alink_ar_host_word_alloc(ctypes.byref(h), ctypes.byref(d)) == 0 and d.value:
            import numpy as np
            self._hword, self._hword_dev = h.value, d.value
            self._hview = np.ctypeslib.as_array((ctypes.c_int32 * 1).from_address(h.value))
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=torch.cuda.is_available())
        self._err_ev = None
        self.seq = 0
        self.calls = 0

    @staticmethod
    def region_bytes(cap_bytes: int, P: int) -> int:
        return 2 * cap_bytes + BLOCKS * max(P, 1) * 4 + 256

    @staticmethod
    def alloc(cap_bytes: int, P: int) -> int:
        L = _lib.require()
        _sigs(L)
        p = ctypes.c_void_p()
        rc = L.alink_ar_alloc(OneShot.region_bytes(cap_bytes, P), ctypes.byref(p))
        if rc != 0:
            raise RuntimeError(f"alink_ar_alloc failed: {rc}")
        return int(p.value)

    def launch(self, t: torch.Tensor, out: torch.Tensor, op: str = "sum", rank: Optional[int] = None,
               phases: int = 3, seq: Optional[int] = None, timeout_s: Optional[float] = None) -> torch.Tensor:
        n = t.numel()
        if t.dtype not in _DT or n * t.element_size() > self.cap:
            raise ValueError("one-shot all-reduce: unsupported dtype or buffer larger than the staging slot")
        if seq is None:
            self.seq += 1
            seq = self.seq
        from ..utils import trace as _trace
        tmo = TIMEOUT_S if timeout_s is None else float(timeout_s)
        with _trace.span("oneshot_allreduce", "kernel", device=True, bytes=int(n * t.element_size()), P=self.P):
            rc = self.L.alink_oneshot_allreduce(t.data_ptr(), out.data_ptr(), n, _DT[t.dtype], _OP[op], self.P,
                                                self.rank if rank is None else rank, seq & 0xFFFFFFFF,
                                                self.peer_data.data_ptr(), self.peer_flags.data_ptr(), self.cap,
                                                BLOCKS, phases, tmo, self.err.data_ptr(), self._hword_dev,
                                                _lib.stream_ptr(self.device))
        if rc != 0:
            raise RuntimeError(f"alink_oneshot_allreduce failed: {rc}")
        self.calls += 1
        return out

    def _raise_if_failed(self, value: int):
        if value != 0:
            self.err.zero_()
            self._err_host.zero_()
            if self._hview is not None:
                self._hview[0] = 0
            self._err_ev = None
            raise RuntimeError("one-shot all-reduce timed out waiting for a peer (results were poisoned with NaN)")

    def check(self, wait: bool = False):
        """Raise if an earlier call timed out.  Non-blocking by default: the error word of the previous call is
        read back asynchronously (pinned copy + event) and examined once that copy has landed."""
        if self._hview is not None:
            if wait:
                torch.cuda.current_stream(self.device).synchronize()
            self._raise_if_failed(int(self._hview[0]))
            return
        if self._err_ev is not None and (wait or self._err_ev.query()):
            self._err_ev.synchronize()
            self._raise_if_failed(int(self._err_host[0]))
            self._err_ev = None

    def all_reduce_(self, t: torch.Tensor, op: str = "sum", timeout_s: Optional[float] = None) -> torch.Tensor:
        self.check()
        # in place: a block copies its slice of the input to the staging slot before it signals, and writes the
        # same slice of the result only after every rank's signal (no result buffer, no copy back)
        flat = t.view(-1) if t.is_contiguous() else t.reshape(-1).contiguous()
        self.launch(flat, flat, op, timeout_s=timeout_s)
        if SYNC_CHECK:
            self._raise_if_failed(int(self.err.item()))
        elif self._hview is None and self._err_ev is None:
            self._err_host.copy_(self.err, non_blocking=True)
            self._err_ev = torch.cuda.Event()
            self._err_ev.record(torch.cuda.current_stream(self.device))
        if flat.data_ptr() != t.data_ptr():
            t.copy_(flat.view_as(t))
        return t

    def close(self):
        if self._hword is not None:
            self._hview = None
            self.L.alink_ar_host_word_free(ctypes.c_void_p(self._hword))
            self._hword, self._hword_dev = None, None
        for p in self.opened:
            self.L.alink_ar_ipc_close(ctypes.c_void_p(p))
        for p in self.owned:
            self.L.alink_ar_free(ctypes.c_void_p(p))
        self.opened, self.owned = [], []


_INSTANCE: Optional[OneShot] = None
_TRIED = False


def mode() -> str:
    v = os.environ.get("ALINK_ONESHOT_ALLREDUCE", "auto").lower()
    return {"1": "force", "0": "off", "auto": "auto", "force": "force", "off": "off"}.get(v, "auto")


def enabled(backend: str = "nccl") -> bool:
    """Whether comm.all_reduce routes small device buffers through the one-shot kernel on this backend."""
    m = mode()
    return m == "force" or (m == "auto" and backend == "nccl")


def _host_min(x: float) -> float:
    """MIN all-reduce of one float over the host (gloo) group: valid on nccl and gloo jobs alike."""
    import torch.distributed as dist
    from . import comm
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=comm.object_group())
    return float(t.item())


def reset():
    """Drop the instance (tests; a new process group needs a new setup)."""
    global _INSTANCE, _TRIED
    if _INSTANCE is not None:
        _INSTANCE.close()
    _INSTANCE, _TRIED = None, False


SETUP_ERROR: Optional[str] = None     # why the last setup fell back to the collective library (diagnostics)


def get() -> Optional[OneShot]:
    """Collective on first use: every rank of the job must call it at the same point (comm.all_reduce does)."""
    global _INSTANCE, _TRIED, SETUP_ERROR
    if _TRIED:
        return _INSTANCE
    _TRIED = True
    SETUP_ERROR = None
    from . import comm
    P, rank = comm.get_world_size(), comm.get_rank()
    dev = comm.device_for_rank()
    ok, inst, base, opened = 1.0, None, None, []
    handles = None
    L = None
    try:
        L = _lib.require()
        _sigs(L)
        base = OneShot.alloc(MAX_BYTES, P)
        hs = int(L.alink_ar_handle_size())
        buf = ctypes.create_string_buffer(hs)
        rc = L.alink_ar_ipc_handle(ctypes.c_void_p(base), buf)
        if rc != 0:
            raise RuntimeError(f"hipIpcGetMemHandle failed: {rc}")
        mine = bytes(buf.raw)
    except Exception as e:
        ok, mine = 0.0, b""
        SETUP_ERROR = f"alloc/handle: {e!r}"
    handles = comm.all_gather_object(mine)
    bases = []
    if ok:
        try:
            for p in range(P):
                if p == rank:
                    bases.append(base)
                    continue
                if not handles[p]:
                    raise RuntimeError("peer has no handle")
                q = ctypes.c_void_p()
                rc = L.alink_ar_ipc_open(ctypes.create_string_buffer(handles[p], len(handles[p])), ctypes.byref(q))
                if rc != 0:
                    raise RuntimeError(f"hipIpcOpenMemHandle failed: {rc}")
                opened.append(int(q.value))
                bases.append(int(q.value))
            inst = OneShot(dev, P, rank, MAX_BYTES, bases, [base], opened)
        except Exception as e:
            ok = 0.0
            SETUP_ERROR = f"ipc open: {e!r}"
    if _host_min(ok) < 1.0:
        SETUP_ERROR = SETUP_ERROR or "a peer failed to set up"
        if inst is not None:
            inst.close()
        else:                       # failure paths: release what this rank did allocate / open
            for q in opened:
                L.alink_ar_ipc_close(ctypes.c_void_p(q))
            if base is not None:
                L.alink_ar_free(ctypes.c_void_p(base))
        return None
    # validate on a probe buffer: the exact rank-order sum every rank can compute locally (integers in fp64)
    probe = torch.arange(1000, dtype=torch.float64, device=dev) * (rank + 1) + 0.25
    ref = torch.arange(1000, dtype=torch.float64, device=dev) * (P * (P + 1) // 2) + 0.25 * P
    try:
        got = inst.all_reduce_(probe.clone(), timeout_s=min(TIMEOUT_S, PROBE_TIMEOUT_S))
        torch.cuda.synchronize(dev)
        good = 1.0 if torch.equal(got, ref) and int(inst.err.item()) == 0 else 0.0
        if not good:
            SETUP_ERROR = "probe mismatch"
    except Exception as e:
        good = 0.0
        SETUP_ERROR = f"probe: {e!r}"
    if _host_min(good) < 1.0:
        SETUP_ERROR = SETUP_ERROR or "a peer's probe failed"
        inst.close()
        return None
    _INSTANCE = inst
    return inst
