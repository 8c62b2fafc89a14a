"""VectorAssembler (K24): the columnar assembler (ops/feature.vector_assemble — HIP kernel on a GPU, torch on the
host) equals the per-row reference rule of VectorAssemblerMapper.java:50-106 (dense/sparse output by RATIO,
NULL handling)."""
import numpy as np
import pytest
import torch

from alink_amd.common.linalg import DenseVector, SparseVector, VectorUtil
from alink_amd.common.linalg.block import SparseBlock
from alink_amd.common.table import Column, MTable
from alink_amd.common.types import TableSchema, Types
from alink_amd.models.dataproc.vector import VectorAssemblerMapper
from alink_amd.common.params import Params


def _table(n, seed, nulls=False, dev="cpu"):
    rng = np.random.default_rng(seed)
    x = torch.as_tensor(rng.normal(size=n))
    k = torch.as_tensor(rng.integers(0, 5, n))
    dense = torch.as_tensor(rng.normal(size=(n, 3)) * (rng.random((n, 3)) < 0.5))
    rows = []
    for _ in range(n):
        idx = sorted(rng.choice(10, rng.integers(0, 4), replace=False).tolist())
        rows.append(SparseVector(10, idx, rng.normal(size=len(idx)).tolist()))
    sb = SparseBlock.from_vectors(rows, 10) if hasattr(SparseBlock, "from_vectors") else None
    strs = [" ".join(f"{v:.3f}" for v in rng.normal(size=2)) for _ in range(n)]
    cols = [Column(x.to(dev)), Column(k.to(dev)), Column(dense.to(dev)),
            Column(sb.to(dev) if sb is not None else rows), Column(strs)]
    if nulls:
        m = torch.zeros(n, dtype=torch.bool)
        m[::7] = True
        cols[0] = Column(x.to(dev), m.to(dev))
        strs2 = list(strs)
        strs2[3::11] = [None] * len(strs2[3::11])
        cols[4] = Column(strs2)
    schema = TableSchema(["x", "k", "d", "s", "t"], [Types.DOUBLE, Types.LONG, Types.DENSE_VECTOR,
                                                     Types.SPARSE_VECTOR, Types.STRING])
    return MTable(schema, cols)


def _mapper(mt, handle):
    p = Params().set("selectedCols", ["x", "k", "d", "s", "t"]).set("outputCol", "o").set("handleInvalid", handle)
    return VectorAssemblerMapper(mt.schema, p)


def _per_row(m, mt):
    cols = [c.to_list() for c in mt.cols]
    out = []
    for r in range(mt.num_rows):
        try:
            out.append(m.mapColumns([c[r] for c in cols]))
        except ValueError:
            raise
    return out


def _eq(a, b):
    if a is None or b is None:
        return a is None and b is None
    return type(a) is type(b) and VectorUtil.toString(a) == VectorUtil.toString(b)


@pytest.mark.parametrize("handle,nulls", [("ERROR", False), ("SKIP", True), ("KEEP", False)])
def test_columnar_assembler_equals_per_row_rule(handle, nulls):
    mt = _table(400, 3, nulls)
    m = _mapper(mt, handle)
    col = m._map_columns(mt)[0]
    assert isinstance(col.values, SparseBlock)             # the columnar path ran, not the per-row fallback
    got = col.to_list()
    ref = _per_row(m, mt)
    assert len(got) == len(ref)
    assert all(_eq(a, b) for a, b in zip(got, ref))


def test_columnar_assembler_error_on_null():
    mt = _table(50, 4, True)
    with pytest.raises(ValueError):
        _mapper(mt, "ERROR")._map_columns(mt)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("handle,nulls", [("ERROR", False), ("SKIP", True)])
def test_hip_vector_assemble_equals_host(handle, nulls, variant, monkeypatch):
    """The HIP kernel paths (device columns; v1 thread per (part, row), v2 element-parallel workgroups) equal
    the host columnar path and the per-row rule."""
    import alink_amd.ops.feature as FE
    monkeypatch.setattr(FE, "VA_VARIANT", variant)
    host = _table(3000, 5, nulls)
    dev = _table(3000, 5, nulls, dev="cuda")
    m = _mapper(host, handle)
    a = m._map_columns(host)[0].to_list()
    out = m._map_columns(dev)[0]
    assert out.values.crow.is_cuda
    b = out.to_list()
    assert all(_eq(x, y) for x, y in zip(a, b))
