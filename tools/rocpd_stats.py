#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite output (``*_results.db``) as a per-kernel stats table (calls, total/avg/min/max
µs, % of GPU time).  Usage: python tools/rocpd_stats.py DB [--top N] [--match SUBSTR] [--timeline ANCHOR]

--timeline ANCHOR prints, for the last two launches of the kernel whose name contains ANCHOR, every kernel in
between with its start offset and duration (one superstep of an iterative job, launch gaps included)."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--match", default=None)
    ap.add_argument("--timeline", default=None)
    ap.add_argument("--steady", type=int, default=40, help="periods of the --timeline kernel to summarise")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     f"from kernels group by {name} order by sum(end-start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print(f"{'calls':>6} {'total_us':>11} {'avg_us':>10} {'min_us':>10} {'max_us':>10} {'pct':>6}  kernel")
    for r in rows[:a.top]:
        if a.match and a.match not in r[0]:
            continue
        print(f"{r[1]:6d} {r[2]/1e3:11.1f} {r[3]/1e3:10.2f} {r[4]/1e3:10.2f} {r[5]/1e3:10.2f} {100*r[2]/total:6.2f}  {r[0][:110]}")
    print(f"total GPU kernel time: {total/1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches")
    if a.timeline:
        ks = c.execute(f"select {name}, start, end from kernels order by start").fetchall()
        anchors = [i for i, k in enumerate(ks) if a.timeline in k[0]]
        if len(anchors) >= 2:
            i0, i1 = anchors[-2], anchors[-1]
            t0 = ks[i0][1]
            print(f"\ntimeline between the last two '{a.timeline}' launches (offset_us, dur_us, kernel):")
            for k in ks[i0:i1 + 1]:
                print(f"  {(k[1] - t0) / 1e3:10.1f} {(k[2] - k[1]) / 1e3:9.1f}  {k[0][:100]}")
            # steady state over the last launches: anchor duration, launch-to-launch period, time outside it
            last = anchors[-min(len(anchors), a.steady + 1):]
            if len(last) >= 3:
                durs = sorted((ks[i][2] - ks[i][1]) / 1e3 for i in last[:-1])
                pers = sorted((ks[j][1] - ks[i][1]) / 1e3 for i, j in zip(last[:-1], last[1:]))
                med = lambda v: v[len(v) // 2]  # noqa: E731
                print(f"\nsteady state over the last {len(last) - 1} '{a.timeline}' periods: kernel median "
                      f"{med(durs):.1f} us (min {durs[0]:.1f}, max {durs[-1]:.1f}), period median {med(pers):.1f} us "
                      f"(min {pers[0]:.1f}, max {pers[-1]:.1f}), outside the kernel {med(pers) - med(durs):.1f} us")


if __name__ == "__main__":
    main()
