"""Tracing / profiling: a per-rank timeline of operators, supersteps, collectives and HIP kernels.

Reference: the reference has no tracer at all — only Flink operator names in the web UI
(``A/common/comqueue/BaseComQueue.java:172,195,225,255,301``, ``communication/AllReduce.java:98-119``),
``LOG.info`` at compute-function boundaries (``KMeansAssignCluster.java:31,64``) and ad-hoc wall clocks in
``A/operator/common/dataproc/BlockwiseCross.java:172-213``.

MI355X design (SURVEY §5.1 "Ours"):

* every span is a Chrome-trace ``"X"`` event (``chrome://tracing`` / Perfetto JSON), one ``pid`` per rank, so
  the per-rank files of an SPMD job can be merged into one timeline (:func:`merge`);
* spans nest: ``op`` (each ``BatchOperator.linkFrom`` / ``StreamOperator.linkFrom``) > ``superstep`` (BSP
  engine) > ``item`` (compute / communicate functions) > ``collective`` (RCCL / gloo / one-shot) and ``kernel``
  (every call into ``libalink_hip.so``);
* the same names are pushed as roctx ranges (``torch.cuda.nvtx`` is roctx on ROCm), so a
  ``rocprofv3 --marker-trace`` run shows them next to the kernel rows;
* device time without synchronising: ``kernel`` and ``collective`` spans also record a pair of HIP events on
  the current stream; :func:`dump` resolves them against an anchor event recorded at :func:`enable` and
  emits them on a separate ``gpu`` track (the host track shows launch cost, the gpu track execution).

Enable with ``ALINK_TRACE=/path/trace_{rank}.json`` (dumped at exit) or :func:`enable`.  Disabled, every hook
costs one attribute check.
"""
from __future__ import annotations

import atexit
import contextlib
import json
import os
import threading
import time
from typing import Any, Dict, List, Optional

__all__ = ["enable", "disable", "enabled", "span", "instant", "counter", "dump", "events", "merge", "reset",
           "traced_call"]


class _Tracer:
    def __init__(self):
        self.enabled = False
        self.path: Optional[str] = None
        self.roctx = True
        self.gpu_events = True
        self.events: List[Dict[str, Any]] = []
        self.pending_gpu: List[tuple] = []     # (name, cat, args, start_event, end_event)
        self.anchor = None                     # (host_us, torch.cuda.Event) pair for device timestamps
        self.t0 = time.perf_counter()
        self.lock = threading.Lock()
        self.depth = threading.local()


_T = _Tracer()


def _rank() -> int:
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:  # pragma: no cover
        pass
    return int(os.environ.get("RANK", "0"))


def _now_us() -> float:
    return (time.perf_counter() - _T.t0) * 1e6


def _cuda_ready() -> bool:
    try:
        import torch
        return torch.cuda.is_available() and torch.cuda.is_initialized()
    except Exception:  # pragma: no cover
        return False


def enable(path: Optional[str] = None, roctx: bool = True, gpu_events: bool = True):
    """Start recording.  ``path`` (``{rank}`` substituted) is where :func:`dump` writes at exit."""
    _T.enabled = True
    _T.path = path
    _T.roctx = roctx
    _T.gpu_events = gpu_events
    _T.anchor = None
    if path:
        atexit.register(_dump_at_exit)


def disable():
    _T.enabled = False


def enabled() -> bool:
    return _T.enabled


def reset():
    with _T.lock:
        _T.events.clear()
        _T.pending_gpu.clear()
        _T.anchor = None
        _T.t0 = time.perf_counter()


def _anchor():
    """Host time <-> device time reference: a synchronised event at a known host time (lazily, on the first
    device span, so CPU-only jobs never touch HIP)."""
    if _T.anchor is None:
        import torch
        torch.cuda.synchronize()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        ev.synchronize()
        _T.anchor = (_now_us(), ev)
    return _T.anchor


def _roctx_push(name):
    if not _T.roctx:
        return False
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            return True
    except Exception:
        _T.roctx = False
    return False


def _roctx_pop():
    try:
        import torch
        torch.cuda.nvtx.range_pop()
    except Exception:  # pragma: no cover
        pass


@contextlib.contextmanager
def span(name: str, cat: str = "op", device: bool = False, **args):
    """Record ``name`` as one timeline event.  ``device=True`` also times it on the current HIP stream."""
    if not _T.enabled:
        yield
        return
    pushed = _roctx_push(name)
    evs = None
    if device and _T.gpu_events and _cuda_ready():
        import torch
        _anchor()
        evs = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        evs[0].record()
    depth = getattr(_T.depth, "v", 0)
    _T.depth.v = depth + 1
    ts = _now_us()
    try:
        yield
    finally:
        dur = _now_us() - ts
        _T.depth.v = depth
        if evs is not None:
            evs[1].record()
        if pushed:
            _roctx_pop()
        ev = {"name": name, "cat": cat, "ph": "X", "ts": ts, "dur": dur, "pid": _rank(),
              "tid": threading.get_ident() if threading.current_thread() is not threading.main_thread() else 0,
              "args": dict(args, depth=depth)}
        with _T.lock:
            _T.events.append(ev)
            if evs is not None:
                _T.pending_gpu.append((name, cat, dict(args), evs[0], evs[1]))


def instant(name: str, cat: str = "mark", **args):
    if not _T.enabled:
        return
    with _T.lock:
        _T.events.append({"name": name, "cat": cat, "ph": "i", "s": "p", "ts": _now_us(), "pid": _rank(),
                          "tid": 0, "args": args})


def counter(name: str, **values):
    """A counter track (e.g. bytes all-reduced per superstep, rows/s)."""
    if not _T.enabled:
        return
    with _T.lock:
        _T.events.append({"name": name, "ph": "C", "ts": _now_us(), "pid": _rank(), "tid": 0,
                          "args": {k: float(v) for k, v in values.items()}})


def traced_call(fn, name: str, cat: str = "kernel", device: bool = True):
    """Wrap ``fn`` so every call is a span (used for the ctypes entry points of ``libalink_hip.so``)."""
    def wrapper(*a, **kw):
        if not _T.enabled:
            return fn(*a, **kw)
        with span(name, cat, device=device):
            return fn(*a, **kw)
    wrapper.__name__ = name
    wrapper.__wrapped__ = fn
    return wrapper


def _resolve_gpu() -> List[Dict[str, Any]]:
    """Turn the recorded event pairs into device-time events (one synchronisation, at dump time)."""
    if not _T.pending_gpu or _T.anchor is None:
        return []
    import torch
    torch.cuda.synchronize()
    host0, ev0 = _T.anchor
    out = []
    for name, cat, args, s, e in _T.pending_gpu:
        try:
            start_ms = ev0.elapsed_time(s)
            dur_ms = s.elapsed_time(e)
        except Exception:  # event never recorded (e.g. a failed launch)
            continue
        out.append({"name": name, "cat": cat + ".gpu", "ph": "X", "ts": host0 + start_ms * 1e3,
                    "dur": dur_ms * 1e3, "pid": _rank(), "tid": "gpu", "args": args})
    _T.pending_gpu.clear()
    return out


def events() -> List[Dict[str, Any]]:
    """All events so far (device events resolved)."""
    with _T.lock:
        _T.events.extend(_resolve_gpu())
        return list(_T.events)


def dump(path: Optional[str] = None) -> str:
    """Write the Chrome-trace JSON of this rank; returns the path."""
    path = (path or _T.path or "alink_trace_{rank}.json").replace("{rank}", str(_rank()))
    evs = events()
    meta = [{"name": "process_name", "ph": "M", "pid": _rank(), "tid": 0, "args": {"name": f"rank {_rank()}"}},
            {"name": "thread_name", "ph": "M", "pid": _rank(), "tid": "gpu", "args": {"name": "gpu stream"}}]
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump({"traceEvents": meta + evs, "displayTimeUnit": "ms",
                   "otherData": {"producer": "alink_amd", "rank": _rank()}}, f)
    os.replace(tmp, path)
    return path


def merge(paths: List[str], out: str) -> str:
    """Concatenate per-rank trace files into one timeline (one process row per rank)."""
    allev = []
    for p in paths:
        with open(p) as f:
            allev.extend(json.load(f)["traceEvents"])
    with open(out, "w") as f:
        json.dump({"traceEvents": allev, "displayTimeUnit": "ms"}, f)
    return out


def _dump_at_exit():
    if _T.enabled and _T.path:
        try:
            dump()
        except Exception as e:  # pragma: no cover - exit path
            print(f"alink trace dump failed: {e}")


if os.environ.get("ALINK_TRACE"):
    enable(os.environ["ALINK_TRACE"], roctx=os.environ.get("ALINK_TRACE_ROCTX", "1") == "1")
