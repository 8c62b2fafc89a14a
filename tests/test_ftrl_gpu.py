"""Hogwild FTRL kernel (ops/csrc/ftrl.hip) vs the sequential fp64 rule of FtrlTrainStreamOp."""
import numpy as np
import pytest
import torch

from alink_amd.operator.stream.onlinelearning import _ftrl_python

pytestmark = pytest.mark.gpu


def _csr(rows):
    indptr, idx, val = [0], [], []
    for r in rows:
        for i, v in r:
            idx.append(i)
            val.append(v)
        indptr.append(len(idx))
    return np.asarray(indptr, np.int64), np.asarray(idx, np.int32), np.asarray(val, np.float64)


def _run_gpu(indptr, idx, val, y, w0, prm):
    from alink_amd.ops.ftrl import ftrl_hogwild
    st = [torch.tensor(a, dtype=torch.float64, device="cuda") for a in (w0, np.zeros_like(w0), np.zeros_like(w0))]
    ftrl_hogwild(torch.as_tensor(indptr), torch.as_tensor(idx), torch.as_tensor(val), torch.as_tensor(y), *st, *prm)
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in st]


def test_ftrl_hogwild_disjoint_coordinates_match_sequential():
    """Samples touching disjoint coordinates have no Hogwild race: the result equals the sequential rule."""
    rng = np.random.default_rng(1)
    nrows, per = 3000, 7                       # 7..(7+63) non-zeros per row, all coordinates distinct
    rows, base = [], 0
    for r in range(nrows):
        k = per + int(rng.integers(0, 64))
        rows.append([(base + j, float(rng.normal())) for j in range(k)])
        base += k
    indptr, idx, val = _csr(rows)
    y = (rng.random(nrows) < 0.5).astype(np.float64)
    w0 = rng.normal(size=base) * 0.1
    prm = (0.1, 1.0, 0.05, 0.1)
    got = _run_gpu(indptr, idx, val, y, w0, prm)
    ref = [w0.copy(), np.zeros(base), np.zeros(base)]
    _ftrl_python(indptr, idx, val, y, *ref, *prm)
    for g, r in zip(got, ref):
        np.testing.assert_allclose(g, r, rtol=1e-12, atol=1e-14)


def test_ftrl_hogwild_shared_coordinates_close_to_sequential():
    """Worst-case contention: 20000 samples over only 200 coordinates (~1000 updates per coordinate, all in
    flight at once), so most samples read stale weights.  Measured on MI355X: log-loss 0.447 (Hogwild) vs 0.374
    (sequential) vs 0.693 (untrained).  The model must still learn and stay within 25 % of the sequential loss;
    at realistic CTR sparsity (1e6-dim, few updates per coordinate in flight) the gap vanishes (the
    disjoint-coordinate test above is exact)."""
    rng = np.random.default_rng(2)
    d, nrows = 200, 20000
    wt = rng.normal(size=d)
    rows, ys = [], []
    for _ in range(nrows):
        cols = rng.choice(d, size=10, replace=False)
        v = rng.normal(size=10)
        rows.append(list(zip(cols.tolist(), v.tolist())))
        ys.append(float(rng.random() < 1 / (1 + np.exp(-float(v @ wt[cols])))))
    indptr, idx, val = _csr(rows)
    y = np.asarray(ys)
    prm = (0.5, 1.0, 0.0, 0.0)
    w_gpu = _run_gpu(indptr, idx, val, y, np.zeros(d), prm)[0]
    ref = [np.zeros(d), np.zeros(d), np.zeros(d)]
    _ftrl_python(indptr, idx, val, y, *ref, *prm)

    def logloss(w):
        m = np.asarray([sum(v * w[i] for i, v in r) for r in rows])
        return float(np.mean(np.log1p(np.exp(-np.where(y > 0, m, -m)))))

    assert np.isfinite(w_gpu).all()
    assert logloss(w_gpu) < 0.8 * np.log(2.0)
    assert logloss(w_gpu) <= logloss(ref[0]) * 1.25


def test_ftrl_hogwild_rejects_bad_index():
    from alink_amd.ops.ftrl import ftrl_hogwild
    st = [torch.zeros(4, dtype=torch.float64, device="cuda") for _ in range(3)]
    with pytest.raises(ValueError):
        ftrl_hogwild(torch.tensor([0, 2]), torch.tensor([1, 9], dtype=torch.int32), torch.ones(2), torch.ones(1), *st,
                     0.1, 1.0, 0.0, 0.0)
