"""LDS-table histogram kernels of ops/csrc/tree_hist.hip (the non-fixed-point path: S > 4 statistics, e.g.
random-forest class counts, or B*S too wide for the fixed-point kernel): ms per histogram call, checked
against the fp64 torch histogram.  Usage: python tools/hist_lds_bench.py  (ALINK_HIP_LIB selects a library)"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from alink_amd.ops import tree as tops
    g = torch.Generator(device="cuda").manual_seed(0)
    for n, F, B, S, nslots, variant in [(4_000_000, 64, 64, 6, 8, 1), (4_000_000, 64, 64, 3, 8, 0),
                                         (2_000_000, 128, 256, 4, 4, 0), (2_000_000, 32, 32, 12, 16, 1)]:
        bins = torch.randint(0, B, (n, F), device="cuda", generator=g, dtype=torch.int32).to(torch.uint8)
        slot = torch.randint(0, nslots, (n,), device="cuda", generator=g, dtype=torch.int32)
        stats = torch.rand(n, S, device="cuda", generator=g)
        h = tops.histogram(bins, slot, stats, nslots, B, variant=variant)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            tops.histogram(bins, slot, stats, nslots, B, variant=variant)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        m = 200_000
        ref = tops.histogram_torch(bins[:m].cpu(), slot[:m].cpu(), stats[:m].cpu().double(), nslots, B)
        part = tops.histogram(bins[:m].contiguous(), slot[:m].contiguous(), stats[:m].contiguous(), nslots, B,
                              variant=variant).cpu().double()
        err = float((part - ref).abs().max() / ref.abs().max())
        print(json.dumps({"lib": os.environ.get("ALINK_HIP_LIB", "tree"), "n": n, "F": F, "B": B, "S": S,
                          "nslots": nslots, "variant": variant, "ms": round(sorted(ts)[2], 3),
                          "bin_GBps": round(n * F / sorted(ts)[2] / 1e6, 1), "max_rel_err_2e5": err,
                          "checksum": float(h.double().sum())}), flush=True)


if __name__ == "__main__":
    main()
