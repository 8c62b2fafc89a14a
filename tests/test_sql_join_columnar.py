"""Columnar equi-join and set operations (operator/common/sql/engine.py ``_join_columnar`` /
``_set_op_columnar``) equal the row path row for row, in order: inner / left / right / full joins with
duplicate keys, NULL keys on both sides, residual predicates, multi-column and mixed int/float keys, string
keys; intersect / minus with and without ALL (NULLs equal in set operations).  The device variants run the same
comparison on GPU-resident tables."""
import numpy as np
import pytest
import torch

from alink_amd.common.strings import StringBlock
from alink_amd.common.table import Column, MTable
from alink_amd.common.types import TableSchema, Types
from alink_amd.operator.common.sql import engine as E


def _tables(dev="cpu", n=400, m=300, seed=0):
    rng = np.random.default_rng(seed)
    k1 = torch.as_tensor(rng.integers(0, 40, n), dtype=torch.int64)
    k2 = torch.as_tensor(rng.integers(0, 3, n), dtype=torch.int32)
    v = torch.as_tensor(np.round(rng.normal(size=n), 3))
    s = [f"s{int(x)}" if x % 11 else None for x in rng.integers(0, 30, n)]
    nk = torch.as_tensor(rng.random(n) < 0.08)
    A = MTable(TableSchema(["id", "g", "v", "s"], [Types.LONG, Types.INT, Types.DOUBLE, Types.STRING]),
               [Column(k1.to(dev), nk.to(dev)), Column(k2.to(dev)), Column(v.to(dev)), Column(StringBlock.from_list(s))])
    key = torch.as_tensor(rng.integers(0, 50, m).astype(np.float64))      # float keys vs the int left keys
    g = torch.as_tensor(rng.integers(0, 3, m), dtype=torch.int64)
    w = torch.as_tensor(rng.integers(0, 5, m).astype(np.float64))
    t = [f"s{int(x)}" if x % 7 else None for x in rng.integers(0, 30, m)]
    nkey = torch.as_tensor(rng.random(m) < 0.08)
    B = MTable(TableSchema(["key", "g", "w", "t"], [Types.DOUBLE, Types.LONG, Types.DOUBLE, Types.STRING]),
               [Column(key.to(dev), nkey.to(dev)), Column(g.to(dev)), Column(w.to(dev)), Column(t)])
    return A, B


CASES = [
    ("a.id = b.key", "a.id, a.v, b.w"),
    ("a.id = b.key AND a.g = b.g", "*"),
    ("a.id = b.key AND b.w > 1", "a.id, b.key, a.g, b.w"),
    ("b.key = a.id AND a.v < b.w", "a.v, b.w, a.s"),
    ("a.s = b.t", "a.id, a.s, b.t, b.w"),
    ("a.s = b.t AND a.g = b.g AND a.v > 0", "a.s, b.g, a.v"),
    ("a.id = b.key AND a.s = b.t", "a.id, b.t"),
]


def _rows(mt):
    return [tuple(r) for r in mt.rows()]


@pytest.mark.parametrize("how", ["inner", "left", "right", "full"])
@pytest.mark.parametrize("pred,select", CASES)
def test_join_columnar_equals_row_path(monkeypatch, how, pred, select):
    A, B = _tables()
    got = E.sql_join(A, B, pred, select, how)
    monkeypatch.setattr(E, "_join_columnar", lambda *a, **k: None)
    monkeypatch.setattr(E, "_join_blocked", lambda *a, **k: None)
    ref = E.sql_join(A, B, pred, select, how)
    assert got.schema.names == ref.schema.names
    assert _rows(got) == _rows(ref)
    assert len(_rows(ref)) > 0


THETA = [
    ("a.v < b.w", "a.id, a.v, b.w"),
    ("a.v < b.w AND a.g = 1", "*"),
    ("a.id > b.key AND b.g = 2 OR a.v > 1.5", "a.id, b.key, a.g, b.g"),
    ("a.s = b.t OR a.v > b.w", "a.s, b.t, a.v"),
]


@pytest.mark.parametrize("how", ["inner", "left", "right", "full"])
@pytest.mark.parametrize("pred,select", THETA)
def test_theta_join_blocked_equals_row_path(monkeypatch, how, pred, select):
    """Joins without equality keys run the left x right pairs in blocks with the predicate evaluated columnar
    (``_join_blocked``): the same rows in the same order as the nested loop, NULLs (three-valued logic) and outer
    padding included; small blocks exercise the block boundaries."""
    A, B = _tables(n=120, m=90)
    real = E._join_blocked
    monkeypatch.setattr(E, "_join_blocked", lambda *a, **k: real(*a, **{**k, "pairs": 1000}))
    got = E.sql_join(A, B, pred, select, how)
    monkeypatch.setattr(E, "_join_blocked", lambda *a, **k: None)
    ref = E.sql_join(A, B, pred, select, how)
    assert got.schema.names == ref.schema.names
    assert _rows(got) == _rows(ref)


def test_join_columnar_keeps_tensor_columns():
    A, B = _tables()
    out = E.sql_join(A, B, "a.id = b.key", "a.id, a.v, b.w", "left")
    assert all(isinstance(c.values, torch.Tensor) for c in out.cols)
    assert out.cols[2].nulls is not None                    # unmatched left rows padded with NULL


@pytest.mark.parametrize("fn", ["intersect", "minus"])
@pytest.mark.parametrize("all_", [False, True])
def test_set_ops_columnar_equal_row_path(monkeypatch, fn, all_):
    def tab(n, seed, hi):
        r = np.random.default_rng(seed)
        x = torch.as_tensor(r.integers(0, hi, n), dtype=torch.int64)
        nx = torch.as_tensor(r.random(n) < 0.15)
        s = [f"k{int(v)}" if v else None for v in r.integers(0, 4, n)]
        return MTable(TableSchema(["x", "s"], [Types.LONG, Types.STRING]), [Column(x, nx), Column(s)])
    a, b = tab(300, 1, 9), tab(200, 2, 6)
    f = getattr(E, "sql_" + fn)
    got = f(a, b, all_)
    monkeypatch.setattr(E, "_set_op_columnar", lambda *x, **k: None)
    ref = f(a, b, all_)
    assert _rows(got) == _rows(ref) and len(_rows(ref)) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["inner", "left", "right", "full"])
def test_join_columnar_on_device(monkeypatch, how):
    A, B = _tables("cuda")
    for pred, select in CASES[:4]:
        got = E.sql_join(A, B, pred, select, how)
        assert any(isinstance(c.values, torch.Tensor) and c.values.is_cuda for c in got.cols)
        with monkeypatch.context() as m:
            m.setattr(E, "_join_columnar", lambda *a, **k: None)
            ref = E.sql_join(A, B, pred, select, how)
        assert _rows(got) == _rows(ref), pred
