"""GPU clock / power / temperature telemetry sampled next to a benchmark (``amdsmi`` gpu_metrics).

``GpuTelemetry(device)`` finds the amdsmi handle of a torch device (by PCI bus id), ``start()`` runs a daemon
thread that reads the SMU's gpu_metrics table every ``interval_s``, ``mark(name)`` time-stamps a phase boundary
(e.g. the timed window of bench.py) and ``stop()`` returns a JSON-ready summary.  ``process=True`` (bench.py) runs
the sampler as a child process instead (``telemetry_child.py``): decoding a gpu_metrics table is Python work that
holds the GIL, and a thread doing it every 5 ms cost the host-heavy KMeans convergence run ~0.9 ms of 43
(profiles/kmeans_telemetry_r6.txt); the child shares only the monotonic clock.  The summary holds:

* per phase: min / median / max of the gfx clock (over XCDs: ``current_gfxclks``), memory clock (``current_uclk``),
  socket power, hotspot and HBM temperature;
* throttle residency deltas over the run (PPT / thermal / PROCHOT accumulators and the per-XCP "gfx clock below
  host limit" counters), so a slow window can be told from a power / thermal cap;
* optionally the raw series ``[t_s, gfxclk_min, gfxclk_max, uclk, power_w, hotspot_c, hbm_c]`` (``series()``).

Absent ``amdsmi`` (or no matching device) the sampler is a no-op whose summary says why.  The reference has no
device telemetry; it plays the role of the Flink metric reporters of ``A/common/MLEnvironment.java`` for a GPU
job (SURVEY §5.5 metrics).
"""
from __future__ import annotations

import json
import os
import statistics
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional

__all__ = ["GpuTelemetry"]

_RESIDENCY = ("ppt_residency_acc", "socket_thm_residency_acc", "vr_thm_residency_acc", "hbm_thm_residency_acc",
              "prochot_residency_acc", "accumulation_counter")
_XCP = ("xcp_stats.gfx_below_host_limit_ppt_acc", "xcp_stats.gfx_below_host_limit_thm_acc",
        "xcp_stats.gfx_below_host_limit_total_acc", "xcp_stats.gfx_low_utilization_acc")


def _num(v) -> Optional[float]:
    """amdsmi reports an unsupported field as the string "N/A"."""
    try:
        return float(v)
    except (TypeError, ValueError):
        return None


def _valid_list(v) -> List[float]:
    if not isinstance(v, (list, tuple)):
        x = _num(v)
        return [] if x is None else [x]
    out = []
    for e in v:
        x = _num(e)
        if x is not None and x > 0:
            out.append(x)
    return out


def _sum_list(v) -> Optional[float]:
    vals = [x for x in (_num(e) for e in (v if isinstance(v, (list, tuple)) else [v])) if x is not None]
    return sum(vals) if vals else None


class GpuTelemetry:
    def __init__(self, device=None, interval_s: float = 0.005, process: bool = False):
        self.interval_s = float(interval_s)
        self.process = bool(process)
        self._child: Optional[subprocess.Popen] = None
        self._bdf = "-"
        self.error: Optional[str] = None
        self._h = None
        self._smi = None
        self._rows: List[tuple] = []
        self._marks: Dict[str, float] = {}
        self._first = self._last = None
        self._stop = threading.Event()
        self._thr: Optional[threading.Thread] = None
        self._t0 = 0.0
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self._smi = amdsmi
            handles = amdsmi.amdsmi_get_processor_handles()
            self._h = self._match(amdsmi, handles, device)
            if self._h is None:
                self.error = f"no amdsmi handle matches {device}"
            elif len(handles) > 1:
                self._bdf = amdsmi.amdsmi_get_gpu_device_bdf(self._h)
        except Exception as e:      # not installed / no driver access on this host
            self.error = f"amdsmi unavailable: {type(e).__name__}: {e}"

    @staticmethod
    def _match(amdsmi, handles, device):
        if not handles:
            return None
        if len(handles) == 1:
            return handles[0]
        try:
            import torch
            p = torch.cuda.get_device_properties(device)
            bus = getattr(p, "pci_bus_id", None)
            dom = getattr(p, "pci_domain_id", 0) or 0
        except Exception:
            bus = None
        if bus is None:
            return None
        for h in handles:
            try:
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)          # "dddd:bb:dd.f"
                d, b = bdf.split(":")[0], bdf.split(":")[1]
                if int(b, 16) == int(bus) and int(d, 16) == int(dom):
                    return h
            except Exception:
                continue
        return None

    @property
    def available(self) -> bool:
        return self._h is not None

    def _read(self):
        return self._smi.amdsmi_get_gpu_metrics_info(self._h)

    def _loop(self):
        nxt = time.perf_counter()
        while not self._stop.is_set():
            try:
                m = self._read()
            except Exception as e:          # keep the bench alive; record why the series stopped
                self.error = f"gpu_metrics read failed: {type(e).__name__}: {e}"
                return
            t = time.perf_counter() - self._t0
            clk = _valid_list(m.get("current_gfxclks", m.get("current_gfxclk")))
            self._rows.append((t, min(clk) if clk else None, max(clk) if clk else None,
                               _num(m.get("current_uclk")), _num(m.get("current_socket_power")),
                               _num(m.get("temperature_hotspot")), _num(m.get("temperature_mem"))))
            if self._first is None:
                self._first = m
            self._last = m
            nxt += self.interval_s
            d = nxt - time.perf_counter()
            if d > 0:
                self._stop.wait(d)
            else:
                nxt = time.perf_counter()

    def start(self) -> "GpuTelemetry":
        self._t0 = time.perf_counter()
        if self.available and self.process and self._child is None:
            child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "telemetry_child.py")
            self._child = subprocess.Popen([sys.executable, child, str(self._bdf), str(self.interval_s)]
                                           + list(_RESIDENCY + _XCP + ("throttle_status",)),
                                           stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
            self._child.stdout.readline()          # "ready": the first sample is taken
        elif self.available and self._thr is None:
            self._thr = threading.Thread(target=self._loop, name="alink-gpu-telemetry", daemon=True)
            self._thr.start()
        return self

    def _stop_child(self):
        c, self._child = self._child, None
        try:
            out, _ = c.communicate("stop\n", timeout=10.0)
            res = json.loads(out.strip().splitlines()[-1])
        except Exception as e:                     # keep the bench alive; say why the series is missing
            c.kill()
            c.wait()
            self.error = f"telemetry child failed: {type(e).__name__}: {e}"
            return
        self._rows = [tuple([r[0] - self._t0] + r[1:]) for r in res.get("rows", [])]
        self._first, self._last = res.get("first"), res.get("last")
        if res.get("error"):
            self.error = res["error"]

    def mark(self, name: str) -> None:
        self._marks[name] = time.perf_counter() - self._t0

    def stop(self) -> dict:
        if self._child is not None:
            self._stop_child()
        if self._thr is not None:
            self._stop.set()
            self._thr.join(timeout=2.0)
            self._thr = None
        return self.summary()

    def _phase(self, lo: float, hi: float) -> dict:
        rows = [r for r in self._rows if lo <= r[0] < hi]
        out = {"samples": len(rows)}
        for j, name in ((1, "gfxclk_min_mhz"), (2, "gfxclk_max_mhz"), (3, "uclk_mhz"), (4, "socket_power_w"),
                        (5, "hotspot_c"), (6, "hbm_c")):
            v = [r[j] for r in rows if r[j] is not None]
            if v:
                out[name] = {"min": min(v), "median": statistics.median(v), "max": max(v)}
        return out

    def series(self) -> list:
        return [[round(r[0], 4)] + [None if v is None else round(v, 1) for v in r[1:7]] for r in self._rows]

    def summary(self, with_series: bool = False) -> dict:
        if not self.available:
            return {"available": False, "error": self.error}
        res = {"available": True, "interval_s": self.interval_s, "samples": len(self._rows), "marks": self._marks}
        if self.error:
            res["error"] = self.error
        edges = sorted(self._marks.items(), key=lambda kv: kv[1])
        bounds = [("all", 0.0, float("inf"))]
        prev_name, prev_t = "start", 0.0
        for name, t in edges:
            bounds.append((f"{prev_name}->{name}", prev_t, t))
            prev_name, prev_t = name, t
        bounds.append((f"{prev_name}->end", prev_t, float("inf")))
        res["phases"] = {n: self._phase(lo, hi) for n, lo, hi in bounds}
        if self._first is not None and self._last is not None:
            d = {}
            for key in _RESIDENCY + _XCP:
                a, b = _sum_list(self._first.get(key)), _sum_list(self._last.get(key))
                if a is not None and b is not None:
                    d[key] = b - a
            res["residency_delta"] = d
            res["throttle_status_last"] = self._last.get("throttle_status")
        if with_series:
            res["series"] = self.series()
        return res
