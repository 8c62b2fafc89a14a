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
    ap.add_argument("--compare", default=None, help="a <scenario>_1_0.json of a 1-rank run: compare the KMeans "
                    "model of every rank with it (tests/test_multiprocess_gpu.py tolerances)")
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
    if a.compare:
        summary["compare"] = _compare(a.compare, [os.path.join(a.out, f"{a.scenario}_{a.world}_{r}.json")
                                                  for r in range(a.world)])
    print(json.dumps(summary))
    return 0


def _compare(ref_path, rank_paths):
    """Every rank's model bit-identical to rank 0's; rank 0's centroids equal to the 1-rank run's up to fp32
    partial-sum rounding (weights within max(2, 1e-4 w), coordinates rtol = atol = 1e-4)."""
    import numpy as np
    with open(ref_path) as f:
        one = json.load(f)
    outs = []
    for p in rank_paths:
        with open(p) as f:
            outs.append(json.load(f))
    a = [json.loads(r[1]) for r in one["model"] if r[0] > 0]
    b = [json.loads(r[1]) for r in outs[0]["model"] if r[0] > 0]
    res = {"ranks_identical": all(o["model"] == outs[0]["model"] for o in outs),
           "iterations": [one.get("iterations"), outs[0].get("iterations")], "k": [len(a), len(b)]}
    if len(a) == len(b):
        dw = [abs(x["weight"] - y["weight"]) for x, y in zip(a, b)]
        dv = [float(np.max(np.abs(np.asarray(x["vec"]["data"]) - np.asarray(y["vec"]["data"])))) for x, y in zip(a, b)]
        res["max_weight_diff"] = max(dw)
        res["max_coord_diff"] = max(dv)
        res["within_tolerance"] = all(d <= max(2.0, 1e-4 * x["weight"]) for d, x in zip(dw, a)) and \
            all(np.allclose(np.asarray(x["vec"]["data"]), np.asarray(y["vec"]["data"]), rtol=1e-4, atol=1e-4)
                for x, y in zip(a, b))
    else:
        res["within_tolerance"] = False
    return res


if __name__ == "__main__":
    sys.exit(main())
