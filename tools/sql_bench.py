#!/usr/bin/env python3
"""Relational ops: columnar SQL evaluation (operator/common/sql/vexpr.py, columnar groupBy / distinct) vs the row
evaluator on the same table.  python tools/sql_bench.py --rows 1000000 [--device cuda]
Prints one JSON line per operation (ms for each path, rows/s of the columnar path)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alink_amd.common.table import Column, MTable  # noqa: E402
from alink_amd.common.types import TableSchema, Types  # noqa: E402
from alink_amd.operator.common.sql import engine as E  # noqa: E402
from alink_amd.operator.common.sql import vexpr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--row-rows", type=int, default=100_000, help="rows for the (slow) row-path timing")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    a = ap.parse_args()
    rng = np.random.default_rng(0)

    def table(n, dev):
        cols = [Column(torch.as_tensor(rng.integers(0, 1000, n)).to(dev)),
                Column(torch.as_tensor(rng.normal(size=n)).to(dev)),
                Column(torch.as_tensor(rng.integers(0, 50, n)).to(dev))]
        return MTable(TableSchema(["id", "x", "g"], [Types.LONG, Types.DOUBLE, Types.LONG]), cols)

    ops = {"where": lambda t: E.sql_where(t, "x > 0.5 AND id % 7 <> 3"),
           "select": lambda t: E.sql_select(t, "id * 2 + g AS k, CASE WHEN x > 0 THEN x ELSE -x END AS ax"),
           "groupBy": lambda t: E.sql_group_by(t, "g", "g, COUNT(*) AS c, SUM(x) AS s, MAX(id) AS m")}
    big, small = table(a.rows, a.device), table(a.row_rows, "cpu")
    sync = torch.cuda.synchronize if a.device.startswith("cuda") else (lambda: None)
    for name, fn in ops.items():
        fn(big)
        sync()
        t0 = time.perf_counter()
        fn(big)
        sync()
        col_ms = (time.perf_counter() - t0) * 1e3
        saved = (vexpr.try_evaluate, E._group_by_columnar)
        vexpr.try_evaluate, E._group_by_columnar = (lambda *x: None), (lambda *x: None)
        t0 = time.perf_counter()
        fn(small)
        row_ms = (time.perf_counter() - t0) * 1e3
        vexpr.try_evaluate, E._group_by_columnar = saved
        print(json.dumps({"op": name, "device": a.device, "columnar_rows": a.rows, "columnar_ms": round(col_ms, 3),
                          "columnar_rows_per_s": a.rows / (col_ms * 1e-3), "row_path_rows": a.row_rows,
                          "row_path_ms": round(row_ms, 1), "row_path_rows_per_s": a.row_rows / (row_ms * 1e-3)}),
              flush=True)


if __name__ == "__main__":
    main()
