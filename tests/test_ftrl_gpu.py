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


def _prox(z, n, alpha, beta, l1, l2):
    return np.where(np.abs(z) <= l1, 0.0, (np.sign(z) * l1 - z) / (beta + np.sqrt(n) / alpha + l2))


def test_ftrl_hogwild_weights_consistent_with_n_z_after_contention():
    """after a contended batch the racing w stores are reconciled — w == prox(z, n) exactly."""
    rng = np.random.default_rng(5)
    d, nrows = 50, 20000
    rows = [list(zip(rng.choice(d, 8, replace=False).tolist(), rng.normal(size=8).tolist())) for _ in range(nrows)]
    indptr, idx, val = _csr(rows)
    y = (rng.random(nrows) < 0.5).astype(np.float64)
    prm = (0.3, 1.0, 0.02, 0.05)
    w, n, z = _run_gpu(indptr, idx, val, y, np.zeros(d), prm)
    np.testing.assert_allclose(w, _prox(z, n, *prm), rtol=1e-13, atol=1e-15)


def _random_csr(rng, nrows, dim, hot=3):
    rows = []
    for _ in range(nrows):
        k = int(rng.integers(1, 30))
        cols = set(rng.choice(dim, size=k, replace=False).tolist()) | set(range(hot))   # hot coords in every row
        rows.append([(c, float(rng.normal())) for c in sorted(cols)])
    return _csr(rows)


@pytest.mark.parametrize("lo,hi", [(0, 5000), (0, 1700), (1700, 5000), (2500, 2600)])
def test_ftrl_sharded_kernels_match_native(lo, hi):
    """SHARDED micro-batch FTRL: partial-margin kernel and per-coordinate replay kernel vs the native host rule
    on one coefficient shard [lo, hi)."""
    from alink_amd import _native
    from alink_amd.ops.ftrl import ftrl_partial_margin_hip, ftrl_shard_update_hip
    rng = np.random.default_rng(lo + hi)
    dim, nrows = 5000, 3000
    indptr, idx, val = _random_csr(rng, nrows, dim)
    y = (rng.random(nrows) < 0.5).astype(np.float64)
    w0 = rng.normal(size=hi - lo) * 0.1
    prm = (0.1, 1.0, 0.01, 0.02)
    ref_m = _native.ftrl_partial_margin(indptr, idx, val, w0, lo, hi)
    dev = [torch.as_tensor(a).cuda() for a in (indptr, idx, val)]
    st = [torch.tensor(a, dtype=torch.float64, device="cuda") for a in (w0, np.zeros_like(w0), np.zeros_like(w0))]
    m = ftrl_partial_margin_hip(*dev, st[0], lo, hi)
    np.testing.assert_allclose(m.cpu().numpy(), ref_m, rtol=1e-12, atol=1e-13)
    full = ref_m + rng.normal(size=nrows) * 0.2          # stand-in for the other shards' all-reduced margins
    err = 1.0 / (1.0 + np.exp(-full)) - y
    ref = [w0.copy(), np.zeros_like(w0), np.zeros_like(w0)]
    _native.ftrl_shard_update(indptr, idx, val, err, *ref, lo, hi, *prm)
    ftrl_shard_update_hip(*dev, torch.as_tensor(err).cuda(), *st, lo, hi, *prm)
    torch.cuda.synchronize()
    for g, r in zip(st, ref):
        np.testing.assert_allclose(g.cpu().numpy(), r, rtol=1e-12, atol=1e-14)


def test_ftrl_shard_update_long_segments_match_native():
    """Coordinates with more than LONG_SEGMENT entries replay on one wave each (lane-parallel n / sigma /
    reciprocal, serial z -> w chain); lengths straddle the threshold and the 64-entry chunking."""
    from alink_amd import _native
    from alink_amd.ops.ftrl import LONG_SEGMENT, ftrl_shard_update_hip
    rng = np.random.default_rng(11)
    nrows, dim = 1100, 40
    lens = {0: nrows, 1: LONG_SEGMENT + 1, 2: LONG_SEGMENT, 3: 64, 4: 65, 5: 129, 6: 640, 7: 1}
    rows = []
    for r in range(nrows):
        cols = {c for c, L in lens.items() if r < L} | set(rng.choice(np.arange(8, dim), 3, replace=False).tolist())
        rows.append([(c, float(rng.normal())) for c in sorted(cols)])
    indptr, idx, val = _csr(rows)
    err = rng.normal(size=nrows) * 0.5
    prm = (0.1, 1.0, 0.01, 0.02)
    w0 = rng.normal(size=dim) * 0.1
    ref = [w0.copy(), np.zeros(dim), np.zeros(dim)]
    _native.ftrl_shard_update(indptr, idx, val, err, *ref, 0, dim, *prm)
    dev = [torch.as_tensor(a).cuda() for a in (indptr, idx, val)]
    st = [torch.tensor(a, dtype=torch.float64, device="cuda") for a in (w0, np.zeros(dim), np.zeros(dim))]
    ftrl_shard_update_hip(*dev, torch.as_tensor(err).cuda(), *st, 0, dim, *prm)
    torch.cuda.synchronize()
    for g, r in zip(st, ref):
        np.testing.assert_allclose(g.cpu().numpy(), r, rtol=1e-11, atol=1e-13)


def test_ftrl_train_stream_sharded_on_gpu_equals_cpu():
    """FtrlTrainStreamOp(updateMode=SHARDED) end to end: GPU env (HIP kernels) == CPU env (native host)."""
    import pandas as pd
    from alink_amd import (useLocalEnv, BatchOperator, StreamOperator, LogisticRegressionTrainBatchOp,
                           FtrlTrainStreamOp, CollectStreamOp)
    from alink_amd.common.mlenv import resetEnv
    rng = np.random.default_rng(9)
    X = rng.normal(size=(3000, 6))
    df = pd.DataFrame({f"f{i}": X[:, i] for i in range(6)})
    df["label"] = (X @ rng.normal(size=6) > 0).astype(int)
    schema = ", ".join(f"f{i} double" for i in range(6)) + ", label int"
    cols = [f"f{i}" for i in range(6)]
    out = {}
    for dev in ("cpu", "cuda:0"):
        resetEnv()
        useLocalEnv(1, device=dev)
        model = LogisticRegressionTrainBatchOp().setFeatureCols(cols).setLabelCol("label").setMaxIter(3) \
            .linkFrom(BatchOperator.fromDataframe(df.iloc[:100], schemaStr=schema))
        snaps = []
        FtrlTrainStreamOp(model).setFeatureCols(cols).setLabelCol("label").setTimeInterval(1e9) \
            .setUpdateMode("SHARDED").setAlpha(0.1).setBeta(1.0).setL1(0.01).setL2(0.01) \
            .linkFrom(StreamOperator.fromDataframe(df, schemaStr=schema)).link(CollectStreamOp(snaps))
        StreamOperator.execute()
        last = max(r[0] for r in snaps)
        out[dev] = [r for r in snaps if r[0] == last and r[2] == 1048576][0][3]
    import json
    a = np.asarray(json.loads(out["cpu"])["coefVector"]["data"])
    b = np.asarray(json.loads(out["cuda:0"])["coefVector"]["data"])
    assert np.abs(a).max() > 0
    np.testing.assert_allclose(b, a, rtol=1e-9, atol=1e-12)


def test_gpu_scoring_to_evaluation_stays_on_device_and_matches_host():
    """LR scoring on the GPU keeps margins, labels and the detail block on the device (no per-micro-batch host
    copy), the binary evaluation bins them on the device, and the metrics equal the host path's (AUC / KS exactly,
    log loss to fp64 summation order)."""
    import numpy as np
    import pandas as pd
    from alink_amd import (BatchOperator, StreamOperator, LogisticRegressionTrainBatchOp,
                           LogisticRegressionPredictBatchOp, LogisticRegressionPredictStreamOp,
                           EvalBinaryClassBatchOp, EvalBinaryClassStreamOp, CollectStreamOp, useLocalEnv)
    from alink_amd.common.detail import DetailBlock
    rng = np.random.default_rng(0)
    X = rng.normal(size=(20000, 4))
    df = pd.DataFrame({f"x{i}": X[:, i] for i in range(4)})
    df["y"] = (X @ np.array([1.0, -0.5, 0.3, 0.0]) + 0.5 * rng.normal(size=len(df)) > 0).astype(int)
    schema = "x0 double, x1 double, x2 double, x3 double, y int"
    feats = [f"x{i}" for i in range(4)]
    res = {}
    useLocalEnv(1, device="cpu")
    model = LogisticRegressionTrainBatchOp().setFeatureCols(feats).setLabelCol("y") \
        .linkFrom(BatchOperator.fromDataframe(df, schemaStr=schema))
    model.getOutputTable()
    from alink_amd.common.table import Column, MTable
    from alink_amd.operator.batch.source import TableSourceBatchOp
    from alink_amd.operator.stream.source import TableSourceStreamOp
    for dev in ("cpu", "cuda:0"):
        useLocalEnv(1, device=dev)
        host = BatchOperator.fromDataframe(df, schemaStr=schema).getOutputTable()
        mt = MTable(host.schema, [Column(c.values.to(dev)) for c in host.cols])      # device-resident rows
        src = TableSourceBatchOp(mt)
        pred = LogisticRegressionPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d") \
            .linkFrom(model, src)
        blk = pred.getOutputTable().col("d").values
        assert isinstance(blk, DetailBlock)
        if dev != "cpu":
            assert blk._probs_t is not None and blk._probs_t.is_cuda and blk.trusted
        m = EvalBinaryClassBatchOp().setLabelCol("y").setPredictionDetailCol("d").linkFrom(pred).collectMetrics()
        box = []
        EvalBinaryClassStreamOp().setLabelCol("y").setPredictionDetailCol("d").setTimeInterval(1e9).linkFrom(
            LogisticRegressionPredictStreamOp(model).setPredictionCol("p").setPredictionDetailCol("d")
            .linkFrom(TableSourceStreamOp(mt))).link(CollectStreamOp(box))
        StreamOperator.execute()
        import json
        res[dev] = (m.getAuc(), m.getKs(), m.getLogLoss(), m.getTotalSamples(), json.loads(box[-1][1]))
    useLocalEnv(1)
    a, b = res["cpu"], res["cuda:0"]
    # probabilities may differ in the last ulp (device exp): a row may land in the neighbouring 1e-5 bin
    assert abs(a[0] - b[0]) < 1e-6 and abs(a[1] - b[1]) < 1e-4 and a[3] == b[3]
    assert abs(a[2] - b[2]) < 1e-9 * abs(a[2])
    assert abs(float(a[4]["AUC"]) - float(b[4]["AUC"])) < 1e-6
    assert int(a[4]["TotalSamples"]) == int(b[4]["TotalSamples"]) == 20000


@pytest.mark.parametrize("l1", [0.01, 3.0])
@pytest.mark.parametrize("drift", [0.0, 0.3])
def test_ftrl_shard_update_block_scan_matches_native(l1, drift, monkeypatch):
    """Segments above SCAN_SEGMENT run the whole-segment speculative block scan (ftrl_coord_scan_kernel): equal
    to the native sequential replay, both when z stays in one prox regime (drift 0.3: one-signed errors) and when
    it crosses |z| = l1 inside the segment (the scan falls back to the chunk walk from the first failing entry)."""
    from alink_amd import _native
    from alink_amd.ops import ftrl as F
    monkeypatch.setattr(F, "SCAN_SEGMENT", 600)
    rng = np.random.default_rng(21)
    nrows, dim = 20000, 30
    lens = {0: nrows, 1: 5000, 2: 601, 3: 600, 4: 1500}
    rows = []
    for r in range(nrows):
        cols = {c for c, L in lens.items() if r < L} | set(rng.choice(np.arange(5, dim), 2, replace=False).tolist())
        rows.append([(c, float(rng.normal()) if c else 1.0) for c in sorted(cols)])
    indptr, idx, val = _csr(rows)
    err = rng.normal(size=nrows) * 0.5 + drift
    prm = (0.1, 1.0, l1, 0.02)
    w0 = rng.normal(size=dim) * 0.1
    ref = [w0.copy(), np.zeros(dim), np.zeros(dim)]
    _native.ftrl_shard_update(indptr, idx, val, err, *ref, 0, dim, *prm)
    dev = [torch.as_tensor(a).cuda() for a in (indptr, idx, val)]
    st = [torch.tensor(a, dtype=torch.float64, device="cuda") for a in (w0, np.zeros(dim), np.zeros(dim))]
    F.ftrl_shard_update_hip(*dev, torch.as_tensor(err).cuda(), *st, 0, dim, *prm)
    torch.cuda.synchronize()
    for g, r in zip(st, ref):
        np.testing.assert_allclose(g.cpu().numpy(), r, rtol=1e-10, atol=1e-12)


def test_ftrl_default_mode_is_device_independent_and_auto_is_sharded():
    """The default updateMode (SEQUENTIAL) trains the bit-identical model on a CPU and a GPU environment; AUTO is
    the opt-in GPU throughput path (SHARDED there), whose step-start margins change the model (~0.2 in a
    coefficient here) -- the difference this pins."""
    import json
    import pandas as pd
    from alink_amd import (useLocalEnv, BatchOperator, StreamOperator, LogisticRegressionTrainBatchOp,
                           FtrlTrainStreamOp, CollectStreamOp)
    from alink_amd.common.mlenv import resetEnv
    rng = np.random.default_rng(4)
    X = rng.normal(size=(3000, 6))
    df = pd.DataFrame({f"f{i}": X[:, i] for i in range(6)})
    df["label"] = (X @ rng.normal(size=6) > 0).astype(int)
    schema = ", ".join(f"f{i} double" for i in range(6)) + ", label int"
    cols = [f"f{i}" for i in range(6)]

    from alink_amd.common.table import MTable
    from alink_amd.operator.batch.source import TableSourceBatchOp
    resetEnv()
    useLocalEnv(1, device="cpu")
    init = LogisticRegressionTrainBatchOp().setFeatureCols(cols).setLabelCol("label").setMaxIter(3) \
        .linkFrom(BatchOperator.fromDataframe(df.iloc[:100], schemaStr=schema))
    init_rows, init_schema = init.collect(), init.getOutputTable().schema       # one initial model for every run

    def run(dev, mode):
        resetEnv()
        useLocalEnv(1, device=dev)
        model = TableSourceBatchOp(MTable.from_rows(init_rows, init_schema, replicated=True))
        snaps = []
        op = FtrlTrainStreamOp(model).setFeatureCols(cols).setLabelCol("label").setTimeInterval(1e9) \
            .setAlpha(0.1).setBeta(1.0).setL1(0.01).setL2(0.01)
        if mode is not None:
            op = op.setUpdateMode(mode)
        op.linkFrom(StreamOperator.fromDataframe(df, schemaStr=schema)).link(CollectStreamOp(snaps))
        StreamOperator.execute()
        last = max(r[0] for r in snaps)
        row = [r for r in snaps if r[0] == last and r[2] == 1048576][0][3]
        return np.asarray(json.loads(row)["coefVector"]["data"])
    cpu, gpu = run("cpu", None), run("cuda:0", None)
    assert np.array_equal(cpu, gpu)
    auto, sharded = run("cuda:0", "AUTO"), run("cuda:0", "SHARDED")
    assert np.array_equal(auto, sharded)
    assert not np.array_equal(auto, cpu)
    assert np.abs(auto - cpu).max() < 0.5 and np.array_equal(np.sign(auto[1:]), np.sign(cpu[1:]))
