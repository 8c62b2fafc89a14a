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
    ap.add_argument("--join-left", type=int, default=10_000_000)
    ap.add_argument("--join-right", type=int, default=1_000_000)
    ap.add_argument("--only-join", action="store_true")
    a = ap.parse_args()
    if a.only_join:
        return join_bench(a)
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
    join_bench(a)


def join_bench(a):
    """1e7 x 1e6 equi-join (each left row matches one right row) + intersect / minus on the device: the
    columnar path (joint key codes, sorted right codes, searchsorted ranges) vs the row path at 1/100 scale."""
    rng = np.random.default_rng(1)
    sync = torch.cuda.synchronize if a.device.startswith("cuda") else (lambda: None)

    def sides(nl, nr, dev):
        L = MTable(TableSchema(["id", "x"], [Types.LONG, Types.DOUBLE]),
                   [Column(torch.as_tensor(rng.integers(0, nr, nl)).to(dev)),
                    Column(torch.as_tensor(rng.normal(size=nl)).to(dev))])
        R = MTable(TableSchema(["key", "w"], [Types.LONG, Types.DOUBLE]),
                   [Column(torch.as_tensor(rng.permutation(nr)).to(dev)),
                    Column(torch.as_tensor(rng.normal(size=nr)).to(dev))])
        return L, R
    L, R = sides(a.join_left, a.join_right, a.device)
    Ls, Rs = sides(a.join_left // 100, a.join_right // 100, "cpu")
    ops = {"join_inner": lambda l, r: E.sql_join(l, r, "a.id = b.key", "a.id, a.x, b.w", "inner"),
           "join_left_residual": lambda l, r: E.sql_join(l, r, "a.id = b.key AND a.x > b.w", "a.id, b.w", "left"),
           "intersect": lambda l, r: E.sql_intersect(l.select(["id"]), r.select(["key"]), False),
           "minus_all": lambda l, r: E.sql_minus(l.select(["id"]), r.select(["key"]), True)}
    for name, fn in ops.items():
        fn(L, R)
        sync()
        t0 = time.perf_counter()
        out = fn(L, R)
        sync()
        col_s = time.perf_counter() - t0
        saved = (E._join_columnar, E._set_op_columnar)
        E._join_columnar, E._set_op_columnar = (lambda *x, **k: None), (lambda *x, **k: None)
        t0 = time.perf_counter()
        outs = fn(Ls, Rs)
        row_s = time.perf_counter() - t0
        E._join_columnar, E._set_op_columnar = saved
        print(json.dumps({"op": name, "device": a.device, "left_rows": a.join_left, "right_rows": a.join_right,
                          "output_rows": out.num_rows, "columnar_ms": round(col_s * 1e3, 2),
                          "columnar_output_rows_per_s": out.num_rows / col_s,
                          "columnar_input_rows_per_s": (a.join_left + a.join_right) / col_s,
                          "row_path_left_rows": a.join_left // 100, "row_path_ms": round(row_s * 1e3, 1),
                          "row_path_output_rows_per_s": outs.num_rows / row_s}), flush=True)


if __name__ == "__main__":
    main()
