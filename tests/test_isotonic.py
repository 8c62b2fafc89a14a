import pytest



def test_isotonic_predict_columnar_matches_scalar():
    """Whole-column prediction (searchsorted) equals the per-value bisect path: exact boundaries, duplicates,
    ends, NaN, nulls."""
    import numpy as np
    import torch
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.regression.isotonic import IsotonicRegressionModelMapper as M
    m = M.__new__(M)
    m.vector_col, m.feature_col, m.index = None, "x", 0
    m.b = np.array([0.0, 1.0, 1.0, 2.5, 4.0])
    m.v = np.array([0.1, 0.2, 0.3, 0.35, 0.9])
    x = torch.tensor([-1.0, 0.0, 0.5, 1.0, 1.7, 2.5, 3.9, 4.0, 9.0, float("nan"), 7.0], dtype=torch.float64)
    nm = torch.zeros(len(x), dtype=torch.bool)
    nm[-1] = True
    mt = MTable(TableSchema(["x"], [Types.DOUBLE]), [Column(x, nm)])
    out = m._map_columns(mt)[0]
    got = out.to_list()
    want = [None if k else m._predict(float(v)) for v, k in zip(x.tolist(), nm.tolist())]
    assert got[:-1] == want[:-1] and got[-1] is None


@pytest.mark.gpu
def test_isotonic_predict_device_bitwise():
    import numpy as np
    import torch
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.regression.isotonic import IsotonicRegressionModelMapper as M
    m = M.__new__(M)
    m.vector_col, m.feature_col, m.index = None, "x", 0
    rng = np.random.default_rng(0)
    m.b = np.sort(rng.standard_normal(50))
    m.v = np.sort(rng.random(50))
    x = torch.from_numpy(rng.standard_normal(10000) * 1.5)
    x[::97] = torch.from_numpy(np.resize(m.b, x[::97].numel()))      # exact boundary hits
    schema = TableSchema(["x"], [Types.DOUBLE])
    host = m._map_columns(MTable(schema, [Column(x)]))[0].values
    dev = m._map_columns(MTable(schema, [Column(x.cuda())]))[0].values
    assert dev.is_cuda and torch.equal(host.view(torch.int64), dev.cpu().view(torch.int64))
