"""Structured metrics: per-superstep records (wall time, collective bytes / calls / time, rows/s, loss) exposed to
Python, optionally streamed as JSON lines and as Prometheus gauges.

Reference: the reference logs through slf4j inside compute functions (e.g. loss, gradient norm and learning
rate per iteration in ``A/operator/common/optim/subfunc/UpdateModel.java:192``) and has no metric groups
(SURVEY §5.5).  Here every BSP superstep (``parallel/comqueue.py``) produces one record; algorithms add their
own fields (``queue.logMetric("loss", v)``) and declare the rows a superstep touches (``queue.setRowsPerStep``),
from which ``rows_per_s`` is derived.

Sinks:
* in memory — :func:`records` (always, bounded to the newest ``ALINK_METRICS_KEEP`` records, default 100000);
* ``ALINK_METRICS=/path/metrics_{rank}.jsonl`` — one JSON object per line, flushed per record;
* ``ALINK_METRICS_PROMETHEUS=<port>`` — ``prometheus_client`` gauges per (job, field) on that port (rank 0 only
  listens; skipped when the client is not importable).
"""
from __future__ import annotations

import json
import os
import threading
from collections import deque
from typing import Any, Dict, List, Optional

__all__ = ["record", "records", "clear", "set_sink", "summary"]

_LOCK = threading.Lock()
_KEEP = int(os.environ.get("ALINK_METRICS_KEEP", "100000"))
_RECORDS: deque = deque(maxlen=_KEEP)
_SINK = None
_SINK_PATH: Optional[str] = None
_PROM = None


def _rank() -> int:
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:  # pragma: no cover
        pass
    return int(os.environ.get("RANK", "0"))


def set_sink(path: Optional[str]):
    """Stream every record to ``path`` (``{rank}`` substituted) as JSON lines; ``None`` closes the sink."""
    global _SINK, _SINK_PATH
    with _LOCK:
        if _SINK is not None:
            _SINK.close()
        _SINK, _SINK_PATH = None, None
        if path:
            _SINK_PATH = path.replace("{rank}", str(_rank()))
            d = os.path.dirname(os.path.abspath(_SINK_PATH))
            os.makedirs(d, exist_ok=True)
            _SINK = open(_SINK_PATH, "a", buffering=1)


def _prometheus(rec: Dict[str, Any]):
    global _PROM
    port = os.environ.get("ALINK_METRICS_PROMETHEUS")
    if not port:
        return
    if _PROM is None:
        try:
            import prometheus_client as pc
        except Exception:
            _PROM = False
            return
        if _rank() == 0:
            pc.start_http_server(int(port))
        _PROM = (pc, {})
    if _PROM is False:
        return
    pc, gauges = _PROM
    for k, v in rec.items():
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            key = "alink_" + "".join(ch if ch.isalnum() else "_" for ch in k)
            g = gauges.get(key)
            if g is None:
                g = gauges[key] = pc.Gauge(key, f"alink_amd metric {k}", ["job", "rank"])
            g.labels(job=str(rec.get("job", "")), rank=str(rec.get("rank", 0))).set(float(v))


def record(kind: str, **fields) -> Dict[str, Any]:
    """Append one record ``{"kind": kind, "rank": r, **fields}`` to every sink."""
    rec = {"kind": kind, "rank": _rank()}
    rec.update(fields)
    with _LOCK:
        _RECORDS.append(rec)
        if _SINK is not None:
            _SINK.write(json.dumps(rec, default=float) + "\n")
    _prometheus(rec)
    return rec


def records(kind: Optional[str] = None, job: Optional[str] = None) -> List[Dict[str, Any]]:
    with _LOCK:
        return [r for r in _RECORDS if (kind is None or r["kind"] == kind) and (job is None or r.get("job") == job)]


def clear():
    with _LOCK:
        _RECORDS.clear()


def summary(kind: str = "superstep", job: Optional[str] = None) -> Dict[str, float]:
    """Totals / means over the matching records (steps, wall, bytes, mean rows/s)."""
    rs = records(kind, job)
    if not rs:
        return {"steps": 0}
    wall = sum(r.get("wall_s", 0.0) for r in rs)
    out = {"steps": len(rs), "wall_s": wall, "comm_bytes": sum(r.get("comm_bytes", 0) for r in rs),
           "comm_calls": sum(r.get("comm_calls", 0) for r in rs), "comm_s": sum(r.get("comm_s", 0.0) for r in rs)}
    rows = sum(r.get("rows", 0) for r in rs)
    if rows and wall > 0:
        out["rows_per_s"] = rows / wall
    return out


if os.environ.get("ALINK_METRICS"):
    set_sink(os.environ["ALINK_METRICS"])
