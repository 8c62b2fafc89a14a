#!/usr/bin/env python3
"""Summarise an alink_amd Chrome-trace file (utils/trace.py): time per category / name on the host track, device
time per kernel on the gpu track, and the idle gaps between consecutive device spans (launch / sync bubbles).
Usage: python tools/trace_summary.py trace_0.json [--top 15]"""
import argparse
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    evs = [e for e in json.load(open(a.path))["traceEvents"] if e.get("ph") == "X"]
    host = [e for e in evs if e.get("tid") != "gpu"]
    gpu = sorted([e for e in evs if e.get("tid") == "gpu"], key=lambda e: e["ts"])
    by = defaultdict(lambda: [0, 0.0])
    for e in host:
        k = (e["cat"], e["name"] if e["cat"] not in ("superstep",) else "superstep")
        by[k][0] += 1
        by[k][1] += e["dur"]
    print("host spans (cat, name): calls, total ms, mean us")
    for (c, n), (cnt, tot) in sorted(by.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {c:10s} {n[:60]:60s} {cnt:6d} {tot / 1e3:10.3f} {tot / cnt:10.1f}")
    if gpu:
        kb = defaultdict(lambda: [0, 0.0])
        for e in gpu:
            kb[e["name"]][0] += 1
            kb[e["name"]][1] += e["dur"]
        print("device spans (gpu track): calls, total ms, mean us")
        for n, (cnt, tot) in sorted(kb.items(), key=lambda kv: -kv[1][1])[:a.top]:
            print(f"  {n[:70]:70s} {cnt:6d} {tot / 1e3:10.3f} {tot / cnt:10.1f}")
        busy = sum(e["dur"] for e in gpu)
        span = gpu[-1]["ts"] + gpu[-1]["dur"] - gpu[0]["ts"]
        gaps = [max(0.0, b["ts"] - (a_["ts"] + a_["dur"])) for a_, b in zip(gpu, gpu[1:])]
        print(f"gpu-track span {span / 1e3:.3f} ms, traced device time {busy / 1e3:.3f} ms "
              f"({100 * busy / max(span, 1e-9):.1f} %), gaps between traced spans: "
              f"mean {sum(gaps) / max(1, len(gaps)):.1f} us, max {max(gaps, default=0):.1f} us")


if __name__ == "__main__":
    main()
