"""utils/telemetry.py against a fake amdsmi (the real one needs a GPU driver): phase split by marks, XCD clock
min/max, "N/A" fields, residency deltas; and the no-amdsmi path degrades to a summary that says why."""
import sys
import time
import types

from alink_amd.utils.telemetry import GpuTelemetry


def _fake_amdsmi():
    m = types.ModuleType("amdsmi")
    state = {"n": 0}
    m.amdsmi_init = lambda: None
    m.amdsmi_get_processor_handles = lambda: ["h0"]

    def metrics(h):
        state["n"] += 1
        n = state["n"]
        return {"current_gfxclks": [2400, 2300 - n % 2, "N/A", 0], "current_uclk": 1900,
                "current_socket_power": 900 + n, "temperature_hotspot": 70, "temperature_mem": "N/A",
                "ppt_residency_acc": 10 * n, "xcp_stats.gfx_below_host_limit_ppt_acc": [n, n, "N/A"]}
    m.amdsmi_get_gpu_metrics_info = metrics
    return m


def test_telemetry_phases_and_deltas(monkeypatch):
    monkeypatch.setitem(sys.modules, "amdsmi", _fake_amdsmi())
    t = GpuTelemetry("cpu", interval_s=0.002).start()
    time.sleep(0.03)
    t.mark("window_start")
    time.sleep(0.03)
    t.mark("window_end")
    s = t.stop()
    assert s["available"] and s["samples"] >= 5
    w = s["phases"]["window_start->window_end"]
    assert w["samples"] >= 2
    assert w["gfxclk_max_mhz"]["max"] == 2400 and w["gfxclk_min_mhz"]["min"] >= 2299
    assert "hbm_c" not in w and w["uclk_mhz"]["median"] == 1900
    d = s["residency_delta"]
    assert d["ppt_residency_acc"] == 10 * (s["samples"] - 1)
    assert d["xcp_stats.gfx_below_host_limit_ppt_acc"] == 2 * (s["samples"] - 1)
    assert len(t.series()) == s["samples"] and len(t.series()[0]) == 7


def test_telemetry_without_amdsmi(monkeypatch):
    bad = types.ModuleType("amdsmi")

    def boom():
        raise RuntimeError("no driver")
    bad.amdsmi_init = boom
    monkeypatch.setitem(sys.modules, "amdsmi", bad)
    t = GpuTelemetry("cpu").start()
    t.mark("x")
    s = t.stop()
    assert s["available"] is False and "no driver" in s["error"]


_FAKE_SRC = """
state = {"n": 0}


def amdsmi_init():
    pass


def amdsmi_get_processor_handles():
    return ["h0"]


def amdsmi_get_gpu_metrics_info(h):
    state["n"] += 1
    n = state["n"]
    return {"current_gfxclks": [2400, 2300 - n % 2, "N/A", 0], "current_uclk": 1900,
            "current_socket_power": 900 + n, "temperature_hotspot": 70, "temperature_mem": "N/A",
            "ppt_residency_acc": 10 * n, "xcp_stats.gfx_below_host_limit_ppt_acc": [n, n, "N/A"]}
"""


def test_telemetry_child_process(monkeypatch, tmp_path):
    """process=True: the sampler runs as a child process (no GIL shared with the caller) with the same summary --
    rows on the parent's clock, phase split by the parent's marks, residency deltas from the child's first / last
    tables."""
    (tmp_path / "fake_amdsmi_child.py").write_text(_FAKE_SRC)
    monkeypatch.setitem(sys.modules, "amdsmi", _fake_amdsmi())
    monkeypatch.setenv("ALINK_AMDSMI_MODULE", "fake_amdsmi_child")
    monkeypatch.setenv("PYTHONPATH", str(tmp_path))
    t = GpuTelemetry("cpu", interval_s=0.002, process=True).start()
    time.sleep(0.05)
    t.mark("window_start")
    time.sleep(0.05)
    t.mark("window_end")
    s = t.stop()
    assert s["available"] and s["samples"] >= 10, s
    w = s["phases"]["window_start->window_end"]
    assert w["samples"] >= 5 and w["gfxclk_max_mhz"]["max"] == 2400 and w["uclk_mhz"]["median"] == 1900
    d = s["residency_delta"]
    assert d["ppt_residency_acc"] == 10 * (s["samples"] - 1)
    assert d["xcp_stats.gfx_below_host_limit_ppt_acc"] == 2 * (s["samples"] - 1)
    assert all(0.0 <= r[0] < 1.0 for r in t.series())
