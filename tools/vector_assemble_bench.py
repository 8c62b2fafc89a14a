#!/usr/bin/env python3
"""K24 VectorAssembler: HIP kernel vs the vectorised torch path on the same device columns.

    python tools/vector_assemble_bench.py --rows 2000000
Parts: 8 numeric columns, one [n, 16] dense vector block, one 1000-dim sparse block (~12 nnz/row).
Prints one JSON line (ms per call for each path, output nnz, GB/s of CSR written by the kernel)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from alink_amd.common.linalg.block import SparseBlock  # noqa: E402
from alink_amd.ops.feature import vector_assemble  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    n, dev = a.rows, torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    parts = [torch.randn(n, device=dev, generator=g, dtype=torch.float64) for _ in range(8)]
    parts.append(torch.randn(n, 16, device=dev, generator=g, dtype=torch.float32))
    ln = torch.randint(6, 19, (n,), device=dev, generator=g)
    crow = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(ln, 0, out=crow[1:])
    nnz = int(crow[-1])
    col = torch.sort(torch.randint(0, 1000, (nnz,), device=dev, generator=g, dtype=torch.int32))[0]
    parts.append(SparseBlock(crow, col, torch.randn(nnz, device=dev, generator=g, dtype=torch.float64), 1000))
    res = {"rows": n}
    out = {}
    import alink_amd.ops.feature as FE
    for name, uk, var in (("kernel_v1", True, 1), ("kernel", True, 2), ("torch", False, 2)):
        FE.VA_VARIANT = var
        sb, _ = vector_assemble(parts, n, use_kernel=uk)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            t0 = time.perf_counter()
            sb, _ = vector_assemble(parts, n, use_kernel=uk)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name] = sb
        res[name + "_ms"] = round(sorted(ts)[len(ts) // 2] * 1e3, 3)
    a_, b_ = out["kernel"], out["torch"]
    res["equal"] = bool(torch.equal(a_.crow, b_.crow) and torch.equal(a_.col, b_.col) and torch.equal(a_.val, b_.val))
    res["nnz"] = int(a_.crow[-1])
    res["speedup"] = round(res["torch_ms"] / res["kernel_ms"], 2)
    res["v1_equal"] = bool(torch.equal(out["kernel_v1"].col, a_.col) and torch.equal(out["kernel_v1"].val, a_.val))
    res["kernel_GBps_written"] = round(res["nnz"] * 12 / (res["kernel_ms"] * 1e-3) / 1e9, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
