#!/bin/bash
# round-5 GPU call: per-launch KMeans kernel durations across a run (warm-up length, per-rank shape)
set -o pipefail
R=$PWD
tools/gpu.sh prof w3 300 python $R/bench.py --steps 40 --warmup 3 --converge-iters 0 || exit 1
tools/gpu.sh prof w125 300 python $R/bench.py --rows 12500000 --steps 100 --warmup 30 --converge-iters 0 || exit 1
python - <<'PY'
import sqlite3, glob
for name in ("w3", "w125"):
    p = glob.glob(f"gpurun_out/prof_{name}/*.db")[0]
    c = sqlite3.connect(p)
    rows = c.execute("select name,start,end from kernels order by start").fetchall()
    v = [(s, e) for n, s, e in rows if "kmeans_v10" in n]
    gaps = [round((v[i + 1][0] - v[i][1]) / 1e3, 1) for i in range(len(v) - 1)]
    print(name, "v10_us", [round((e - s) / 1e3) for s, e in v])
    print(name, "gap_us", gaps)
PY
