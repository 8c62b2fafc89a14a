"""Every ``parallel/comm.py`` wrapper through its real collective branch (tests/comm_check.py).

* host: gloo at world 1 (forced collective), 2 and 3 — the rank arithmetic of every wrapper;
* GPU: a 1-rank RCCL (``nccl``) group with ``ALINK_COMM_FORCE_COLLECTIVE=1`` — the RCCL branches an 8-GPU job
  runs (device and host-staged tensors, comm-stream event discipline, async handles), once with the one-shot
  kernel serving small device all-reduces (the default on RCCL jobs) and once with RCCL for everything.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, tmp_path, tag, extra_env=None, timeout=240):
    port = _free_port()
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "ALINK_COMM_FORCE_COLLECTIVE",
              "MASTER_PORT"):
        env.pop(k, None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(extra_env or {})
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "comm_check.py"), str(r), str(world), str(port),
                               str(tmp_path), tag], env=env) for r in range(world)]
    try:
        for p in procs:
            p.wait(timeout=timeout)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    outs = []
    for r in range(world):
        with open(os.path.join(str(tmp_path), f"comm_{tag}_{world}_{r}.json")) as f:
            o = json.load(f)
        assert "error" not in o, o["error"]
        assert "shutdown_error" not in o, o["shutdown_error"]
        bad = [k for k, v in o["checks"].items() if not v]
        assert not bad, (r, bad)
        outs.append(o)
    return outs


@pytest.mark.parametrize("world", [1, 2, 3])
def test_comm_wrappers_gloo(tmp_path, world):
    outs = _run(world, tmp_path, "gloo", {"ALINK_DEVICE": "cpu", "ALINK_DIST_BACKEND": "gloo"})
    for o in outs:
        assert o["backend"] == "gloo" and o["is_distributed"] and o["world"] == world
        assert len(o["checks"]) >= 40
        assert o["stats"]["collectives"] > 30


@pytest.mark.gpu
def test_comm_wrappers_rccl_one_rank_with_oneshot(tmp_path):
    o = _run(1, tmp_path, "rccl_oneshot")[0]
    assert o["backend"] == "nccl" and o["is_distributed"]
    assert o["oneshot_instance"], o["oneshot_setup_error"]
    assert o["stats"]["oneshot"] > 0


@pytest.mark.gpu
def test_comm_wrappers_rccl_one_rank_no_oneshot(tmp_path):
    o = _run(1, tmp_path, "rccl_plain", {"ALINK_ONESHOT_ALLREDUCE": "0"})[0]
    assert o["backend"] == "nccl" and o["is_distributed"]
    assert not o["oneshot_instance"] and o["stats"]["oneshot"] == 0


def test_device_timing_event_list_is_bounded():
    """Device timing folds old event pairs into running totals: a long timed job never holds more than the cap of
    live events, and collect() still returns every collective's count and time."""
    from alink_amd.parallel import comm

    class _Ev:
        def synchronize(self):
            pass

        def elapsed_time(self, other):
            return 2.0                                          # ms

    saved = dict(comm._DEV_TIMING)
    try:
        comm._DEV_TIMING.update({"events": [], "folded": (0, 0.0, {})})
        cap = comm._DEV_TIMING_MAX_PENDING
        for i in range(3 * cap):
            evl = comm._DEV_TIMING["events"]
            evl.append(("all_reduce", _Ev(), _Ev()))
            if len(evl) > cap:
                half = len(evl) // 2
                comm._DEV_TIMING["folded"] = comm._fold_events(evl[:half], comm._DEV_TIMING["folded"])
                del evl[:half]
            assert len(comm._DEV_TIMING["events"]) <= cap
        n, tot, per = comm.device_timing_collect()
        assert n == 3 * cap and abs(tot - 3 * cap * 2e-3) < 1e-9 and set(per) == {"all_reduce"}
        assert comm.device_timing_collect()[0] == 0
    finally:
        comm._DEV_TIMING.clear()
        comm._DEV_TIMING.update(saved)
