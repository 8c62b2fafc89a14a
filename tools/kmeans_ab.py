#!/usr/bin/env python3
"""Same-box A/B timing of builds of libalink_hip.so (KMeans v10 variants): every build runs the fused kernel on
the same synthetic 1e8 x 128 bf16 table (tools/kmeans_kernel_bench.py in a child process with ALINK_HIP_LIB),
in ``--rounds`` alternating rounds, so clock drift and box-to-box spread hit all builds alike.

    python tools/kmeans_ab.py --libs base=alink_amd/ops/libalink_hip.so,pk=variants/libalink_hip_pk.so \
        [--rounds 3] [--rows 100000000] [--modes 0] [--iters 15]

Prints one JSON line per (round, build, mode) and a summary line with the median ms per build and mode.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--modes", default="0")
    ap.add_argument("--iters", type=int, default=15)
    ap.add_argument("--sub-rows", default="")
    a = ap.parse_args()
    libs = [kv.split("=", 1) for kv in a.libs.split(",")]
    res = {}
    for r in range(a.rounds):
        for name, path in libs:
            env = dict(os.environ)
            env["ALINK_HIP_LIB"] = os.path.join(ROOT, path) if not os.path.isabs(path) else path
            cmd = [sys.executable, os.path.join(ROOT, "tools", "kmeans_kernel_bench.py"), "--rows", str(a.rows),
                   "--configs", "v10:1", "--modes", a.modes, "--iters", str(a.iters)]
            if a.sub_rows:
                cmd += ["--sub-rows", a.sub_rows]
            out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                print(json.dumps({"build": name, "round": r, "error": out.stderr[-2000:]}), flush=True)
                return 1
            for line in out.stdout.splitlines():
                if line.startswith("{"):
                    d = json.loads(line)
                    d.update({"build": name, "round": r})
                    print(json.dumps(d), flush=True)
                    res.setdefault((name, d["rows"], d["mode"]), []).append(d["ms"])
    summ = {f"{k[0]}|rows={k[1]}|mode={k[2]}": sorted(v)[len(v) // 2] for k, v in res.items()}
    print(json.dumps({"summary_median_ms": summ}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
