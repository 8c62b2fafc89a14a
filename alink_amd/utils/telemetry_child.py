"""Sampler process of ``utils/telemetry.py`` (``GpuTelemetry(process=True)``): a standalone script -- it imports
neither torch nor this package -- so the amdsmi reads and the Python work of decoding every gpu_metrics table run
outside the benchmark's interpreter and never contend for its GIL.

    python telemetry_child.py <bdf | -> <interval_s> <keys...>

Reads ``amdsmi_get_gpu_metrics_info`` every interval (the device whose BDF matches, or the only one), stamps each
row with ``time.perf_counter()`` (CLOCK_MONOTONIC: the parent's clock too), keeps the residency counters ``keys``
of the first and last table, and on a line on stdin (or stdin closing) writes everything as ONE JSON document to
stdout and exits.  ``ALINK_AMDSMI_MODULE`` names a stand-in module (tests).
"""
import importlib
import json
import os
import select
import sys
import time


def _num(v):
    try:
        return float(v)
    except (TypeError, ValueError):
        return None


def _clocks(v):
    vals = v if isinstance(v, (list, tuple)) else [v]
    out = [x for x in (_num(e) for e in vals) if x is not None and x > 0]
    return (min(out), max(out)) if out else (None, None)


def main():
    bdf, interval, keys = sys.argv[1], float(sys.argv[2]), sys.argv[3:]
    res = {"rows": [], "first": None, "last": None, "error": None}
    try:
        smi = importlib.import_module(os.environ.get("ALINK_AMDSMI_MODULE", "amdsmi"))
        smi.amdsmi_init()
        handles = smi.amdsmi_get_processor_handles()
        h = None
        if bdf == "-" and len(handles) == 1:
            h = handles[0]
        else:
            for c in handles:
                try:
                    if smi.amdsmi_get_gpu_device_bdf(c).lower() == bdf.lower():
                        h = c
                        break
                except Exception:
                    continue
        if h is None:
            raise RuntimeError(f"no amdsmi handle with BDF {bdf}")
    except Exception as e:
        res["error"] = f"{type(e).__name__}: {e}"
        h = None
    print("ready", flush=True)
    nxt = time.perf_counter()
    while True:
        if h is not None:
            try:
                m = smi.amdsmi_get_gpu_metrics_info(h)
                lo, hi = _clocks(m.get("current_gfxclks", m.get("current_gfxclk")))
                res["rows"].append([time.perf_counter(), lo, hi, _num(m.get("current_uclk")),
                                    _num(m.get("current_socket_power")), _num(m.get("temperature_hotspot")),
                                    _num(m.get("temperature_mem"))])
                sub = {k: m.get(k) for k in keys if k in m}
                if res["first"] is None:
                    res["first"] = sub
                res["last"] = sub
            except Exception as e:
                res["error"] = f"gpu_metrics read failed: {type(e).__name__}: {e}"
                h = None
        nxt += interval
        wait = max(0.0, nxt - time.perf_counter())
        if wait == 0.0:
            nxt = time.perf_counter()
        r, _, _ = select.select([sys.stdin], [], [], wait if h is not None else None)
        if r:
            break
    sys.stdout.write(json.dumps(res) + "\n")
    sys.stdout.flush()


if __name__ == "__main__":
    main()
