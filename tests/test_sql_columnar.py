"""Columnar SQL evaluation (operator/common/sql/vexpr.py) equals the row evaluator on select and where,
including NULLs, integer division, three-valued logic, CASE, BETWEEN / IN and casts."""
import math

import numpy as np
import pytest
import torch

from alink_amd.common.table import Column, MTable
from alink_amd.common.types import TableSchema, Types
from alink_amd.operator.common.sql import engine as E
from alink_amd.operator.common.sql import vexpr

EXPRS = [
    "a + b", "a - 2 * b", "a / b", "x / y", "a % 3", "x * 1.5 + a", "-x", "a / 0", "x / 0",
    "a > b", "x <= y", "a = 3", "a <> b AND x > 0", "a > 2 OR x < 0", "NOT (a > b)",
    "x IS NULL", "a IS NOT NULL", "a BETWEEN 1 AND 4", "b NOT BETWEEN 0 AND 2", "a IN (1, 3, 5)",
    "CASE WHEN a > 3 THEN x WHEN a > 1 THEN y ELSE 0.5 END", "CAST(x AS INT)", "CAST(a AS DOUBLE) / 2",
    "ABS(x)", "FLOOR(y)", "SIGN(a - 3)", "f AND a > 1", "NOT f OR x > 0",
]


def _table(n=300, seed=0, dev="cpu"):
    rng = np.random.default_rng(seed)
    a = torch.as_tensor(rng.integers(-2, 7, n), dtype=torch.int32)
    b = torch.as_tensor(rng.integers(-3, 4, n), dtype=torch.int64)
    x = torch.as_tensor(np.round(rng.normal(size=n), 3))
    y = torch.as_tensor(rng.normal(size=n).astype(np.float32))
    f = torch.as_tensor(rng.random(n) < 0.5)
    nx = torch.as_tensor(rng.random(n) < 0.1)
    na = torch.as_tensor(rng.random(n) < 0.1)
    cols = [Column(a.to(dev), na.to(dev)), Column(b.to(dev)), Column(x.to(dev), nx.to(dev)), Column(y.to(dev)),
            Column(f.to(dev))]
    return MTable(TableSchema(["a", "b", "x", "y", "f"], [Types.INT, Types.LONG, Types.DOUBLE, Types.FLOAT,
                                                          Types.BOOLEAN]), cols)


def _same(u, v):
    if u is None or v is None:
        return u is None and v is None
    if isinstance(u, float) or isinstance(v, float):
        return (math.isnan(u) and math.isnan(v)) or u == v or abs(u - v) <= 1e-12 * max(1.0, abs(v))
    return u == v and type(u) is type(v) or (isinstance(u, bool) == isinstance(v, bool) and u == v)


@pytest.mark.parametrize("expr", EXPRS)
def test_columnar_select_equals_row_path(expr):
    mt = _table()
    out = E.sql_select(mt, f"{expr} AS r")
    assert isinstance(out.cols[0].values, torch.Tensor), "columnar path expected"
    rows, schema = E._select_rows(mt.rows(), mt.schema, f"{expr} AS r")
    got = out.cols[0].to_list()
    ref = [r[0] for r in rows]
    assert all(_same(g, r) for g, r in zip(got, ref)), [(g, r) for g, r in zip(got, ref) if not _same(g, r)][:5]
    assert out.schema.types[0] == schema.types[0]


@pytest.mark.parametrize("expr", [e for e in EXPRS if any(op in e for op in ("<", ">", "=", "IS", "IN", "AND",
                                                                              "OR", "NOT", "BETWEEN"))])
def test_columnar_where_equals_row_path(expr, monkeypatch):
    mt = _table(seed=1)
    got = E.sql_where(mt, expr).rows()
    monkeypatch.setattr(vexpr, "try_evaluate", lambda *a: None)
    ref = E.sql_where(mt, expr).rows()
    assert [tuple(map(str, r)) for r in got] == [tuple(map(str, r)) for r in ref]


def test_unsupported_falls_back():
    mt = _table()
    assert vexpr.try_evaluate(__import__("alink_amd.operator.common.sql.expr", fromlist=["x"]).parse_expr(
        "UPPER('a')"), mt, E._resolver(mt.schema.names)) is None


@pytest.mark.gpu
@pytest.mark.parametrize("expr", ["a > b AND x > 0", "CASE WHEN a > 3 THEN x ELSE y END", "a / b", "x IS NULL OR f"])
def test_columnar_sql_on_device_table(expr):
    """A GPU-resident table is projected / filtered on the device and equals the host evaluation."""
    host, dev = _table(seed=2), _table(seed=2, dev="cuda")
    s_dev = E.sql_select(dev, f"{expr} AS r")
    assert s_dev.cols[0].values.is_cuda
    assert [str(v) for v in s_dev.cols[0].to_list()] == [str(v) for v in E.sql_select(host, f"{expr} AS r").cols[0].to_list()]
    if "CASE" not in expr and "/" not in expr:
        assert [tuple(map(str, r)) for r in E.sql_where(dev, expr).rows()] == \
               [tuple(map(str, r)) for r in E.sql_where(host, expr).rows()]


@pytest.mark.parametrize("by,sel", [
    ("b", "b, COUNT(*) AS c, SUM(a) AS s, AVG(x) AS m, MIN(y) AS lo, MAX(a) AS hi, COUNT(x) AS cx"),
    ("b, f", "f, b, SUM(x) AS s"),
    ("a", "a, COUNT(*) AS c"),            # NULL keys form their own group
    ("s", "s, COUNT(*) AS c, MAX(b) AS mb"),
])
def test_columnar_group_by_equals_row_path(by, sel, monkeypatch):
    mt = _table(seed=3)
    rng = np.random.default_rng(4)
    strs = [None if i % 17 == 0 else f"k{int(v)}" for i, v in enumerate(rng.integers(0, 6, mt.num_rows))]
    mt = mt.with_columns(["s"], [Types.STRING], [Column(strs)])
    got = E.sql_group_by(mt, by, sel)
    assert E._group_by_columnar(mt, by, sel) is not None
    monkeypatch.setattr(E, "_group_by_columnar", lambda *a: None)
    ref = E.sql_group_by(mt, by, sel)
    assert got.schema.types == ref.schema.types
    for rg, rr in zip(got.rows(), ref.rows()):
        assert all(_same(u, v) for u, v in zip(rg, rr)), (rg, rr)
    assert got.num_rows == ref.num_rows


def test_columnar_distinct_equals_row_path(monkeypatch):
    mt = _table(n=500, seed=5)
    mt = mt.select(["b", "f"]).with_columns(["s"], [Types.STRING],
                                           [Column([None if i % 9 == 0 else f"v{i % 4}" for i in range(500)])])
    got = E.sql_distinct(mt).rows()
    monkeypatch.setattr(E, "_row_codes", lambda *a: None)
    ref = E.sql_distinct(mt).rows()
    assert [tuple(r) for r in got] == [tuple(r) for r in ref]


def test_groupby_distinct_packed_string_keys_equal_list_keys():
    """GROUP BY / DISTINCT on a packed string key (device dictionary codes) give the rows and order of the list
    key (first appearance), nulls and empty strings as their own groups."""
    import torch
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.common.sql.engine import sql_distinct
    import alink_amd as A
    from alink_amd.operator.batch.source import TableSourceBatchOp
    keys = ["b", "a", None, "", "b", "c", None, "a", "", "b"] * 3
    x = torch.arange(len(keys), dtype=torch.float64)
    outs = []
    for kc in (Column(StringBlock.from_list(keys)), Column(list(keys))):
        mt = MTable(TableSchema(["k", "x"], [Types.STRING, Types.DOUBLE]), [kc, Column(x)])
        g = A.GroupByBatchOp().setGroupByPredicate("k").setSelectClause("k, COUNT(*) AS n, SUM(x) AS s") \
            .linkFrom(TableSourceBatchOp(mt)).collect()
        d = sql_distinct(MTable(TableSchema(["k"], [Types.STRING]), [kc])).col("k").to_list()
        outs.append(([tuple(r) for r in g], d))
    assert outs[0] == outs[1]


@pytest.mark.parametrize("clause,order", [("a", "asc"), ("a", "desc"), ("a desc, b", "asc"), ("b, a asc", "desc"),
                                          ("a + b", "asc")])
def test_order_by_columnar_matches_row_path(monkeypatch, clause, order):
    """ORDER BY on tensor keys (stable device sorts) gives the row path's order: ties in input order, NULLs
    first ascending / last descending, -0.0 equal to 0.0, offset/limit applied after."""
    import torch
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.common.sql import engine as E
    g = torch.Generator().manual_seed(5)
    n = 300
    a = torch.randint(0, 7, (n,), generator=g).to(torch.float64)
    a[::17] = -0.0
    b = torch.randint(0, 4, (n,), generator=g)
    an = torch.zeros(n, dtype=torch.bool)
    an[5::23] = True
    mt = MTable(TableSchema(["a", "b", "i"], [Types.DOUBLE, Types.LONG, Types.LONG]),
                [Column(a, an), Column(b), Column(torch.arange(n))])
    for off, lim in [(None, None), (3, 50)]:
        fast = E.sql_order_by(mt, clause, order, limit=lim, offset=off)
        with monkeypatch.context() as m:
            m.setattr(E, "_order_columnar", lambda *x: None)
            slow = E.sql_order_by(mt, clause, order, limit=lim, offset=off)
        assert fast.col("i").values.tolist() == slow.col("i").values.tolist()


@pytest.mark.parametrize("clause", ["UPPER(c) AS u, CONCAT(c, '_', d) AS cd", "LOWER(CONCAT(d, c)) AS x",
                                    "CONCAT('[', UPPER(d), ']') AS b, c", "UPPER(c) AS u, LOWER(e) AS l"])
def test_select_string_functions_columnar(monkeypatch, clause):
    """UPPER / LOWER / CONCAT on packed strings (byte operations on the device) select the row path's values:
    NULLs propagate, empty strings, literals; non-ASCII text goes back to the row path."""
    from alink_amd.common.strings import StringBlock
    cs = ["aB", None, "", "xyz", "Q r"] * 3
    ds = ["d1", "E", None, "", "zz"] * 3
    es = ["Ünï", "b", "c", None, "É"] * 3
    schema = TableSchema(["c", "d", "e"], [Types.STRING] * 3)
    mt = MTable(schema, [Column(StringBlock.from_list(cs)), Column(StringBlock.from_list(ds)),
                         Column(StringBlock.from_list(es))])
    fast = E.sql_select(mt, clause)
    with monkeypatch.context() as m:
        m.setattr(E, "_select_columnar", lambda *a, **k: None)
        slow = E.sql_select(mt, clause)
    assert fast.schema.names == slow.schema.names and fast.schema.types == slow.schema.types
    assert [tuple(r) for r in fast.rows()] == [tuple(r) for r in slow.rows()]


@pytest.mark.gpu
def test_select_string_functions_device():
    from alink_amd.common.strings import StringBlock
    cs = ["aB", None, "", "xyz", "Q r"] * 50
    ds = ["d1", "E", None, "", "zz"] * 50
    schema = TableSchema(["c", "d"], [Types.STRING] * 2)
    host = MTable(schema, [Column(StringBlock.from_list(cs)), Column(StringBlock.from_list(ds))])
    dev = MTable(schema, [Column(StringBlock.from_list(cs).to("cuda")), Column(StringBlock.from_list(ds).to("cuda"))])
    clause = "UPPER(c) AS u, CONCAT(c, '_', LOWER(d)) AS cd"
    a, b = E.sql_select(host, clause), E.sql_select(dev, clause)
    assert b.cols[0].values.device.type == "cuda"
    assert [tuple(r) for r in a.rows()] == [tuple(r) for r in b.rows()]
