#!/usr/bin/env python3
"""Multi-process rehearsal on one GPU with per-rank tracing: P rank processes of a tests/mp_gpu_helpers.py
scenario share the card (gloo host group, device tensors, small all-reduces through the one-shot IPC kernel),
each with ALINK_TRACE on, and the per-rank Chrome traces are merged and summarised.

    python tools/mp_rehearsal.py --world 2 --scenario kmeans --out gpurun_out/rehearsal
Writes <out>/trace_<rank>.json, <out>/merged.json and prints one JSON summary line: per rank the one-shot
kernel spans on the gpu track (count, mean / p50 device us), the collective spans (host track), and RCCL-free
all-reduce counts from the scenario itself.  The launcher only spawns children: it never touches the GPU."""
import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--scenario", default="kmeans")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "rehearsal"))
    ap.add_argument("--timeout", type=int, default=240)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    port = _port()
    procs = []
    for r in range(a.world):
        env = dict(os.environ)
        env["ALINK_TRACE"] = os.path.join(a.out, "trace_{rank}.json")
        env["ALINK_TRACE_ROCTX"] = "0"
        # ranks sharing one GPU run gloo: the one-shot IPC kernel is opt-in there (default on under RCCL)
        env.setdefault("ALINK_ONESHOT_ALLREDUCE", "1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_gpu_helpers.py"), str(r),
                                       str(a.world), str(port), a.scenario, a.out], env=env))
    rc = 0
    for p in procs:
        try:
            rc |= p.wait(timeout=a.timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            print(json.dumps({"error": "timeout"}))
            return 1
    if rc:
        print(json.dumps({"error": f"rank exit code {rc}"}))
        return 1
    from alink_amd.utils import trace
    paths = [os.path.join(a.out, f"trace_{r}.json") for r in range(a.world)]
    trace.merge(paths, os.path.join(a.out, "merged.json"))
    summary = {"world": a.world, "scenario": a.scenario, "ranks": []}
    for r, pth in enumerate(paths):
        with open(pth) as f:
            ev = json.load(f)["traceEvents"]
        gpu = [e for e in ev if e.get("tid") == "gpu" and e.get("ph") == "X"]
        one = sorted(e["dur"] for e in gpu if "oneshot" in e["name"])
        coll = [e for e in ev if e.get("cat") == "collective" and e.get("tid") != "gpu"]
        kern = {}
        for e in gpu:
            kern.setdefault(e["name"], []).append(e["dur"])
        with open(os.path.join(a.out, f"{a.scenario}_{a.world}_{r}.json")) as f:
            res = json.load(f)
        summary["ranks"].append({
            "rank": r, "oneshot_kernel_spans_gpu_track": len(one),
            "oneshot_us_mean": round(sum(one) / len(one), 2) if one else None,
            "oneshot_us_p50": round(one[len(one) // 2], 2) if one else None,
            "collective_spans_host_track": len(coll),
            "collective_names": sorted({e["name"] for e in coll}),
            "gpu_track_kernels": {k: {"n": len(v), "mean_us": round(sum(v) / len(v), 2)} for k, v in sorted(kern.items())},
            "scenario_oneshot_calls": res.get("oneshot_calls"), "backend": res.get("backend"),
            "oneshot_setup_error": res.get("oneshot_setup_error"), "error": (res.get("error") or "")[-400:]})
    print(json.dumps(summary))
    return 0


if __name__ == "__main__":
    sys.exit(main())
