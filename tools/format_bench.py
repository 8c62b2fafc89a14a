#!/usr/bin/env python3
"""Format-conversion throughput: the columnar fast paths of ``models/dataproc/format.py`` vs the per-row
reader -> map -> writer path on the same table (``--rows`` x ``--cols`` doubles).  Host-side work (string
formatting / parsing), so it runs anywhere; prints one JSON line per conversion.

    python tools/format_bench.py --rows 200000 --cols 10
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=200_000)
    ap.add_argument("--cols", type=int, default=10)
    ap.add_argument("--slow-rows", type=int, default=20_000, help="rows timed on the per-row path")
    a = ap.parse_args()
    from alink_amd.common.mapper import Mapper
    from alink_amd.common.params import Params
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.dataproc import format as F
    rng = np.random.default_rng(0)
    names = [f"c{i}" for i in range(a.cols)]
    X = rng.normal(size=(a.rows, a.cols))
    num = MTable(TableSchema(names, [Types.DOUBLE] * a.cols), [Column(torch.from_numpy(X[:, i].copy()))
                                                               for i in range(a.cols)])
    schema_str = ", ".join(f"{c} double" for c in names)
    p_vec = Params().set("fromFormat", "COLUMNS").set("toFormat", "VECTOR").set("selectedCols", names) \
        .set("vectorCol", "vec")
    p_csv = Params().set("fromFormat", "COLUMNS").set("toFormat", "CSV").set("selectedCols", names) \
        .set("csvCol", "csv").set("schemaStr", schema_str)
    vec = F.FormatTransMapper(num.schema, p_vec).map_table(num)
    csv = F.FormatTransMapper(num.schema, p_csv).map_table(num)
    vt = MTable(TableSchema(["vec"], [Types.STRING]), [vec.col("vec")])
    ct = MTable(TableSchema(["csv"], [Types.STRING]), [csv.col("csv")])
    cases = [("columns_to_vector", num, F.FormatTransMapper(num.schema, p_vec)),
             ("columns_to_csv", num, F.FormatTransMapper(num.schema, p_csv)),
             ("vector_to_columns", vt, F.FormatTransMapper(vt.schema, Params().set("fromFormat", "VECTOR")
                                                           .set("toFormat", "COLUMNS").set("vectorCol", "vec")
                                                           .set("schemaStr", schema_str))),
             ("csv_to_columns", ct, F.FormatTransMapper(ct.schema, Params().set("fromFormat", "CSV")
                                                        .set("toFormat", "COLUMNS").set("csvCol", "csv")
                                                        .set("schemaStr", schema_str))),
             ("CsvToColumns", ct, F.CsvToColumnsMapper(ct.schema, Params().set("selectedCol", "csv")
                                                       .set("schemaStr", schema_str)))]
    for name, mt, m in cases:
        t = time.perf_counter()
        fast = m.map_table(mt)
        tf = time.perf_counter() - t
        sub = MTable(mt.schema, [c.take(slice(0, a.slow_rows)) for c in mt.cols])
        t = time.perf_counter()
        slow = m.helper.result_table(sub, Mapper._map_columns(m, sub))
        ts = time.perf_counter() - t
        same = [tuple(map(repr, r)) for r in fast.rows()[:a.slow_rows]] == [tuple(map(repr, r)) for r in slow.rows()]
        print(json.dumps({"conversion": name, "rows": a.rows, "cols": a.cols,
                          "fast_rows_per_s": round(a.rows / tf), "row_path_rows_per_s": round(a.slow_rows / ts),
                          "speedup": round((a.rows / tf) / (a.slow_rows / ts), 1), "identical": same}), flush=True)


if __name__ == "__main__":
    main()
