#!/bin/bash
# round-5 GPU call: what else runs on the GPU while the 1.25e7-row supersteps slow down (kernels + copies)
set -o pipefail
R=$PWD
O=$R/gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/prof_w125b -o w125b -- python $R/bench.py --rows 12500000 --steps 60 --warmup 5 --converge-iters 0 > $O/prof_w125b.log 2>&1 || exit 1
cd $R && python - > $O/w125b_window.txt 2>&1 <<'PY'
import sqlite3, glob
p = glob.glob("gpurun_out/prof_w125b/*.db")[0]
c = sqlite3.connect(p)
ks = c.execute("select name,start,end,stream_id,queue_id from kernels order by start").fetchall()
v = [k for k in ks if "kmeans_v10" in k[0]]
print("v10_us", [round((k[2] - k[1]) / 1e3) for k in v])
t0, t1 = v[3][1], v[14][2]
print("kernels in the window of launches 4..15:")
for k in ks:
    if k[2] >= t0 and k[1] <= t1:
        print(round((k[1] - t0) / 1e3, 1), round((k[2] - k[1]) / 1e3, 1), "stream", k[3], "queue", k[4], k[0][:80])
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
mc = [t for t in tabs if "memory_copy" in t.lower() and not t[-1].isdigit()]
print("copy tables", mc)
for t in mc[:1]:
    cols = [r[1] for r in c.execute(f"pragma table_info({t})")]
    print(cols)
    rows = c.execute(f"select * from {t}").fetchall()
    si, ei = cols.index("start"), cols.index("end")
    for r in rows:
        if r[ei] >= t0 and r[si] <= t1:
            print("copy", round((r[si] - t0) / 1e3, 1), round((r[ei] - r[si]) / 1e3, 1), r)
PY
rm -rf $O/prof_w125b
cat $O/w125b_window.txt | head -80
