#!/usr/bin/env python3
"""Summarise rocprofv3 CSV outputs (kernel stats / PMC counters) into a compact text report."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root, out):
    lines = []
    for f in sorted(glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)):
        lines.append(f"== kernel stats {os.path.relpath(f, root)}")
        rows = list(csv.DictReader(open(f)))
        rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0) or 0))
        for r in rows[:25]:
            lines.append(f"{r.get('Name','')[:90]:90s} calls={r.get('Calls')} total_ms={float(r.get('TotalDurationNs',0))/1e6:.3f} "
                         f"avg_us={float(r.get('AverageNs',0))/1e3:.1f} pct={float(r.get('Percentage',0)):.1f}")
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        lines.append(f"== counters {os.path.relpath(f, root)}")
        agg = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", r.get("Kernel-Name", ""))[:80]
            agg[k][r.get("Counter_Name", "")] += float(r.get("Counter_Value", 0) or 0)
        for k, d in agg.items():
            if "kmeans" not in k and "assign" not in k:
                continue
            lines.append(k)
            for c, v in sorted(d.items()):
                lines.append(f"   {c:32s} {v:.4g}")
    for f in sorted(glob.glob(os.path.join(root, "**", "*.db"), recursive=True)):
        import sqlite3
        c = sqlite3.connect(f)
        lines.append(f"== kernel stats (rocpd db) {os.path.relpath(f, root)}")
        for name, calls, tot, avg, pct in c.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels limit 25"):
            lines.append(f"{name[:90]:90s} calls={calls} total_ms={tot/1e3:.3f} avg_us={avg:.1f} pct={pct:.1f}")
    txt = "\n".join(lines)
    open(out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
