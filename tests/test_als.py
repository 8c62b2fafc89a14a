"""ALS vs the reference docs (docs/en/als*.md) + format / mode / kernel checks."""
import numpy as np
import pandas as pd
import pytest
import torch

from alink_amd import *  # noqa: F401,F403
from alink_amd.models.recommendation.als import AlsModelDataConverter
from alink_amd.ops import als as aops

DATA = np.array([[1, 1, 0.6], [2, 2, 0.8], [2, 3, 0.6], [4, 1, 0.6], [4, 2, 0.3], [4, 3, 0.4]])
REF = [0.579622, 0.766851, 0.581079, 0.574481, 0.298500, 0.382157]


def _src():
    df = pd.DataFrame({"user": DATA[:, 0].astype(int), "item": DATA[:, 1].astype(int), "rating": DATA[:, 2]})
    return BatchOperator.fromDataframe(df, schemaStr="user bigint, item bigint, rating double"), df


def _train(**kw):
    op = AlsTrainBatchOp().setUserCol("user").setItemCol("item").setRateCol("rating").setNumIter(10) \
        .setRank(10).setLambda(0.01)
    for k, v in kw.items():
        getattr(op, "set" + k[0].upper() + k[1:])(v)
    return op


def test_als_doc_example_predictions():
    src, df = _src()
    model = _train().linkFrom(src)
    rows = model.collect()
    assert [(r[0], r[1]) for r in rows] == [(1, None), (2, None), (4, None), (None, 1), (None, 2), (None, 3)]
    assert len(rows[0][2].split(" ")) == 10
    out = AlsPredictBatchOp().setUserCol("user").setItemCol("item").setPredictionCol("p") \
        .linkFrom(model, src).collect()
    # factor initialisation is random in the reference too; the fitted ratings agree to ~1e-2
    np.testing.assert_allclose([r[3] for r in out], REF, atol=1e-2)
    # unseen user -> null
    df2 = pd.DataFrame({"user": [99], "item": [1], "rating": [0.0]})
    miss = AlsPredictBatchOp().setUserCol("user").setItemCol("item").setPredictionCol("p").linkFrom(
        model, BatchOperator.fromDataframe(df2, schemaStr="user bigint, item bigint, rating double")).collect()
    assert miss[0][3] is None


def test_als_topk_stream_and_pipeline():
    src, df = _src()
    model = _train().linkFrom(src)
    top = AlsTopKPredictBatchOp().setUserCol("user").setPredictionCol("rec").setTopK(2).linkFrom(model, src).collect()
    assert [r[0] for r in top] == [1, 2, 4]
    for _, rec in top:
        parts = [p.split(":") for p in rec.split(",")]
        assert len(parts) == 2 and float(parts[0][1]) >= float(parts[1][1])
    box = []
    AlsPredictStreamOp(model).setUserCol("user").setItemCol("item").setPredictionCol("p") \
        .linkFrom(StreamOperator.fromDataframe(df, schemaStr="user bigint, item bigint, rating double")) \
        .link(CollectStreamOp(box))
    StreamOperator.execute()
    np.testing.assert_allclose(sorted(r[3] for r in box), sorted(REF), atol=1e-2)
    m = ALS().setUserCol("user").setItemCol("item").setRateCol("rating").setRank(10).setLambda(0.01) \
        .setPredictionCol("p").fit(src)
    np.testing.assert_allclose([r[3] for r in m.transform(src).collect()], REF, atol=1e-2)


def test_als_modes_and_roundtrip():
    src, _ = _src()
    nn = AlsModelDataConverter.load(_train(nonnegative=True, numBlocks=2).linkFrom(src).collect())
    assert (nn.user_factors >= 0).all() and (nn.item_factors >= 0).all()
    imp = AlsModelDataConverter.load(_train(implicitPrefs=True, alpha=10.0).linkFrom(src).collect())
    # implicit preference: observed pairs score higher than unobserved ones for user 1 (rated only item 1)
    s = imp.user_factors[imp.user_map[1]] @ imp.item_factors.T
    assert s[imp.item_map[1]] > max(s[imp.item_map[2]], s[imp.item_map[3]])


def test_als_recovers_low_rank_matrix():
    rng = np.random.default_rng(0)
    nu, ni, k = 60, 40, 4
    U, V = rng.normal(size=(nu, k)), rng.normal(size=(ni, k))
    R = U @ V.T
    mask = rng.random((nu, ni)) < 0.5
    uu, ii = np.nonzero(mask)
    df = pd.DataFrame({"u": uu, "i": ii, "r": R[uu, ii]})
    src = BatchOperator.fromDataframe(df, schemaStr="u bigint, i bigint, r double")
    model = AlsTrainBatchOp().setUserCol("u").setItemCol("i").setRateCol("r").setRank(k).setLambda(1e-4) \
        .setNumIter(30).linkFrom(src)
    m = AlsModelDataConverter.load(model.collect())
    pred = m.user_factors @ m.item_factors.T
    held = ~mask
    rmse = np.sqrt(((pred[np.ix_(m.user_ids, m.item_ids)] - R)[held] ** 2).mean())
    assert rmse < 0.05 * R.std()



def _pipeline_als(**kw):
    als = ALS().setUserCol("user").setItemCol("item").setRateCol("rating").setLambda(0.01).setRank(10) \
        .setNumIter(10).setPredictionCol("predicted_rating")
    for k, v in kw.items():
        getattr(als, "set" + k[0].upper() + k[1:])(v)
    return als


def _mae(pred):
    return EvalRegressionBatchOp().setLabelCol("rating").setPredictionCol("predicted_rating").linkFrom(pred) \
        .collectMetrics().getMae()


def test_als_pipeline_reference_cases():
    """pipeline/recommendation/ALSTest: explicit and non-negative fits reach MAE < 0.02 through the pipeline model
    and AlsPredictBatchOp over ``model.getModelData()``; non-negative factors are >= 0; an unseen user predicts
    null; implicit preferences separate positive from non-positive ratings (MAE < 0.02 on the 0/1 labels)."""
    from alink_amd.operator.batch.source import MemSourceBatchOp
    data = MemSourceBatchOp([(1, 1, 0.6), (2, 2, 0.8), (2, 3, 0.6), (3, 1, 0.6), (3, 2, 0.3), (3, 3, 0.4)],
                            "user bigint, item bigint, rating double")
    predict = AlsPredictBatchOp().setUserCol("user").setItemCol("item").setPredictionCol("predicted_rating")
    model = _pipeline_als().fit(data)
    assert _mae(model.transform(data)) < 0.02
    assert _mae(predict.linkFrom(model.getModelData(), data)) < 0.02

    model = _pipeline_als(nonnegative=True).fit(data)
    assert _mae(model.transform(data)) < 0.02
    md = AlsModelDataConverter.load(BatchOperator.fromTable(model.getModelData()).collect())
    assert (np.asarray(md.userFactors) >= 0).all() and (np.asarray(md.itemFactors) >= 0).all()
    unseen = MemSourceBatchOp([(4, 1)], "user bigint, item bigint")
    for out in (model.transform(unseen), AlsPredictBatchOp().setUserCol("user").setItemCol("item")
                .setPredictionCol("predicted_rating").linkFrom(model.getModelData(), unseen)):
        assert [tuple(r) for r in out.collect()] == [(4, 1, None)]

    rows2 = [(1, 1, 6.0), (1, 2, -10.0), (1, 3, -5.0), (2, 1, 0.0), (2, 2, 8.0), (2, 3, 6.0), (3, 1, 6.0),
             (3, 2, 3.0), (3, 3, 0.1)]
    data2 = MemSourceBatchOp(rows2, "user bigint, item bigint, rating double")
    pred = _pipeline_als(implicitPrefs=True).fit(data2).transform(data2) \
        .select("(case rating > 0 when true then 1 else 0 end) as rating, predicted_rating")
    assert _mae(pred) < 0.02

def test_normal_equations_torch_matches_dense():
    rng = np.random.default_rng(1)
    Y = torch.as_tensor(rng.normal(size=(7, 5)), dtype=torch.float32)
    indptr = torch.tensor([0, 3, 3, 6])
    nbr = torch.tensor([0, 2, 6, 1, 2, 3], dtype=torch.int32)
    rt = torch.tensor([1.0, -2.0, 0.5, 0.0, 3.0, 1.5])
    A, b = aops.normal_equations(indptr, nbr, rt, Y, implicit=False)
    Yd = Y.double()
    np.testing.assert_allclose(A[0].numpy(), (Yd[[0, 2, 6]].T @ Yd[[0, 2, 6]]).numpy(), atol=1e-12)
    np.testing.assert_allclose(b[2].numpy(), (Yd[[1, 2, 3]].T @ rt[3:].double()).numpy(), atol=1e-12)
    assert float(A[1].abs().sum()) == 0.0
    x = aops.nnls(torch.eye(2, dtype=torch.float64)[None] * 2, torch.tensor([[2.0, -4.0]], dtype=torch.float64))
    np.testing.assert_allclose(x.numpy(), [[1.0, 0.0]])


@pytest.mark.gpu
@pytest.mark.parametrize("r", [3, 10, 16, 40, 64])
@pytest.mark.parametrize("implicit", [False, True])
def test_hip_als_normal_equations(r, implicit):
    import alink_amd.ops._lib as L
    assert L.available()
    rng = np.random.default_rng(r)
    m, n = 300, 500
    counts = rng.integers(0, 90, size=m)
    indptr = torch.zeros(m + 1, dtype=torch.int64)
    indptr[1:] = torch.as_tensor(np.cumsum(counts))
    nnz = int(indptr[-1])
    nbr = torch.as_tensor(rng.integers(0, n, size=nnz), dtype=torch.int32)
    rt = torch.as_tensor(rng.normal(size=nnz), dtype=torch.float32)
    Y = torch.as_tensor(rng.normal(size=(n, r)), dtype=torch.float32)
    A0, b0 = aops.normal_equations_torch(indptr, nbr, rt, Y, implicit, 3.0)
    A1, b1 = aops.normal_equations(indptr.cuda(), nbr.cuda(), rt.cuda(), Y.cuda(), implicit, 3.0)
    np.testing.assert_allclose(A1.cpu().double().numpy(), A0.numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(b1.cpu().double().numpy(), b0.numpy(), rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("r", [10, 64])
def test_hip_als_normal_equations_high_degree_row(r):
    """ADVICE r1 (als.hip fp32 accumulation): one row with 1e5 neighbours against the fp64 torch Gram. Tile
    partials fold into fp64, so the error stays near one fp32 rounding of the result (plain fp32 running sums
    drift to ~1e-5 relative at this degree)."""
    import alink_amd.ops._lib as L
    assert L.available()
    rng = np.random.default_rng(7)
    n, deg = 4000, 100_000
    indptr = torch.tensor([0, deg, deg + 5], dtype=torch.int64)
    nbr = torch.as_tensor(rng.integers(0, n, size=deg + 5), dtype=torch.int32)
    rt = torch.as_tensor(rng.uniform(0.5, 5.0, size=deg + 5), dtype=torch.float32)
    Y = torch.as_tensor(1.0 + 0.3 * rng.normal(size=(n, r)), dtype=torch.float32)
    A0, b0 = aops.normal_equations_torch(indptr, nbr, rt, Y, False, 0.0)
    A1, b1 = aops.normal_equations(indptr.cuda(), nbr.cuda(), rt.cuda(), Y.cuda(), False, 0.0)
    np.testing.assert_allclose(A1.cpu().double().numpy(), A0.numpy(), rtol=2e-6)
    np.testing.assert_allclose(b1.cpu().double().numpy(), b0.numpy(), rtol=2e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("r", [3, 10, 16, 40, 64])
@pytest.mark.parametrize("implicit", [False, True])
def test_hip_als_fused_solve_matches_fp64_torch(r, implicit):
    """Fused normal equations + Cholesky kernel vs fp64 torch (index_add_ Gram + cholesky_solve), including a
    row with 20000 neighbours (fp64 accumulation) and empty rows (pure regularisation -> x = 0)."""
    rng = np.random.default_rng(100 + r)
    m, n = 400, 3000
    counts = rng.integers(0, 60, size=m)
    counts[5] = 20000                 # > HEAVY_DEGREE: split across waves
    counts[9] = 40000
    counts[7] = 0
    indptr = torch.zeros(m + 1, dtype=torch.int64)
    indptr[1:] = torch.as_tensor(np.cumsum(counts))
    nnz = int(indptr[-1])
    nbr = torch.as_tensor(rng.integers(0, n, size=nnz), dtype=torch.int32)
    rt = torch.as_tensor(rng.integers(1, 6, size=nnz).astype(np.float32))
    if implicit:
        rt[torch.as_tensor(rng.random(nnz) < 0.2)] = 0.0
    Y = torch.as_tensor(rng.normal(size=(n, r)) * 0.3, dtype=torch.float32)
    lam = 0.05
    reg = torch.as_tensor(np.maximum(counts, 1) * lam, dtype=torch.float64)
    YtY = (Y.double().T @ Y.double()) if implicit else None
    A, b = aops.normal_equations_torch(indptr, nbr, rt, Y, implicit, 2.0)
    if implicit:
        A = A + YtY[None]
    A = A + reg[:, None, None] * torch.eye(r, dtype=torch.float64)[None]
    ref = torch.cholesky_solve(b[:, :, None], torch.linalg.cholesky(A))[:, :, 0]
    got = aops.fused_solve(indptr.cuda(), nbr.cuda(), rt.cuda(), Y.cuda(), reg.cuda(), implicit, 2.0,
                           None if YtY is None else YtY.cuda())
    np.testing.assert_allclose(got.cpu().double().numpy(), ref.float().double().numpy(), rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
def test_als_train_on_gpu_matches_docs():
    """AlsTrainBatchOp on cuda (fused solve path) reproduces the docs/en/als.md predictions."""
    from alink_amd import useLocalEnv, BatchOperator, AlsTrainBatchOp, AlsPredictBatchOp
    useLocalEnv(1, device="cuda:0")
    df = pd.DataFrame([[1, 1, 0.6], [2, 2, 0.8], [2, 3, 0.6], [4, 1, 0.6], [4, 2, 0.3], [4, 3, 0.4]],
                      columns=["user", "item", "rating"])
    data = BatchOperator.fromDataframe(df, schemaStr="user bigint, item bigint, rating double")
    model = AlsTrainBatchOp().setUserCol("user").setItemCol("item").setRateCol("rating").setNumIter(10) \
        .setRank(10).setLambda(0.01).linkFrom(data)
    out = AlsPredictBatchOp().setUserCol("user").setItemCol("item").setPredictionCol("pred") \
        .linkFrom(model, data).collect()
    np.testing.assert_allclose([r[3] for r in out], REF, atol=1e-2)   # random init, as the CPU doc test


@pytest.mark.gpu
@pytest.mark.parametrize("implicit", [False, True])
def test_hip_als_heavy_mfma_gram_matches_valu(implicit, monkeypatch):
    """Heavy rows at rank 64: the MFMA partial Gram (bf16 x3 exact split, per-step fp64 folding) gives the same
    solutions as the fp64 VALU Gram to fp32 resolution."""
    rng = np.random.default_rng(3)
    m, n, r = 6, 5000, 64
    counts = np.array([30000, 17000, 5, 50000, 0, 20001])
    indptr = torch.zeros(m + 1, dtype=torch.int64)
    indptr[1:] = torch.as_tensor(np.cumsum(counts))
    nnz = int(indptr[-1])
    nbr = torch.as_tensor(rng.integers(0, n, size=nnz), dtype=torch.int32)
    rt = torch.as_tensor(rng.integers(1, 6, size=nnz).astype(np.float32))
    Y = torch.as_tensor(rng.normal(size=(n, r)) * 0.3, dtype=torch.float32)
    reg = torch.as_tensor(np.maximum(counts, 1) * 0.05, dtype=torch.float64)
    YtY = (Y.double().T @ Y.double()).cuda() if implicit else None
    args = (indptr.cuda(), nbr.cuda(), rt.cuda(), Y.cuda(), reg.cuda(), implicit, 2.0, YtY)
    monkeypatch.setattr(aops, "HEAVY_MFMA", 1)
    a = aops.fused_solve(*args).cpu().double().numpy()
    monkeypatch.setattr(aops, "HEAVY_MFMA", 0)
    b = aops.fused_solve(*args).cpu().double().numpy()
    np.testing.assert_allclose(a, b, rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("r", [24, 40, 64])
def test_hip_als_woodbury_small_rows_match_rxr(r, monkeypatch):
    """Explicit rows with <= 32 neighbours take the m x m push-through solve; it equals the r x r fused solve and
    fp64 Cholesky (rows with 0, 1, 16, 17, 32 and 33 neighbours, repeated neighbours, and lambda = 0 rows that
    fall back to pinv: the minimum-norm solution either way)."""
    rng = np.random.default_rng(7 + r)
    n = 900
    counts = np.concatenate([[0, 1, 16, 17, 32, 33, 2, 5], rng.integers(0, 40, size=3000)])
    m = counts.size
    indptr = torch.zeros(m + 1, dtype=torch.int64)
    indptr[1:] = torch.as_tensor(np.cumsum(counts))
    nnz = int(indptr[-1])
    nbr = rng.integers(0, n, size=nnz)
    nbr[int(indptr[6]):int(indptr[7])] = nbr[int(indptr[6])]          # the 2-neighbour row repeats one item
    nbr = torch.as_tensor(nbr, dtype=torch.int32)
    rt = torch.as_tensor(rng.integers(1, 6, size=nnz).astype(np.float32))
    Y = torch.as_tensor(rng.normal(size=(n, r)) * 0.3, dtype=torch.float32)
    reg = torch.as_tensor(counts * 0.05, dtype=torch.float64)
    reg[7] = 0.0                                                        # 5 neighbours, no regulariser
    args = (indptr.cuda(), nbr.cuda(), rt.cuda(), Y.cuda(), reg.cuda(), False, 0.0, None)
    monkeypatch.setattr(aops, "WOODBURY", 1)
    a = aops.fused_solve(*args).cpu().double().numpy()
    monkeypatch.setattr(aops, "WOODBURY", 0)
    b = aops.fused_solve(*args).cpu().double().numpy()
    np.testing.assert_allclose(a, b, rtol=2e-5, atol=2e-6)
    A, bb = aops.normal_equations_torch(indptr, nbr, rt, Y, False, 0.0)
    A = A + reg[:, None, None] * torch.eye(r, dtype=torch.float64)[None]
    ref = (torch.linalg.pinv(A) @ bb[:, :, None])[:, :, 0].numpy()
    np.testing.assert_allclose(a, ref, rtol=2e-4, atol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("r", [33, 40, 62, 64])
@pytest.mark.parametrize("implicit", [False, True])
def test_hip_als_mfma_light_solve_matches_fp64(r, implicit, monkeypatch):
    """Rank 33..64 light rows on the f64 matrix cores (permuted-basis MFMA Gram + block LDL^T, alink_als_mfma_solve)
    vs fp64 Cholesky and vs the VALU Gauss-Jordan kernel: rows with 0 .. 300 neighbours (past-the-end steps of the
    4-neighbour loop), one with 5000, r not a multiple of 4 (scalar loads), repeated neighbours, implicit Y^T Y."""
    rng = np.random.default_rng(31 + r + implicit)
    n = 2000
    counts = np.concatenate([[0, 1, 3, 4, 5, 33, 34, 35, 36, 37, 5000], rng.integers(33, 300, size=600)])
    m = counts.size
    indptr = torch.zeros(m + 1, dtype=torch.int64)
    indptr[1:] = torch.as_tensor(np.cumsum(counts))
    nnz = int(indptr[-1])
    nbr = rng.integers(0, n, size=nnz)
    nbr[int(indptr[6]):int(indptr[7])] = nbr[int(indptr[6])]
    nbr = torch.as_tensor(nbr, dtype=torch.int32)
    rt = torch.as_tensor(rng.integers(1, 6, size=nnz).astype(np.float32))
    if implicit:
        rt[torch.as_tensor(rng.random(nnz) < 0.2)] = 0.0
    Y = torch.as_tensor(rng.normal(size=(n, r)) * 0.3, dtype=torch.float32)
    reg = torch.as_tensor(np.maximum(counts, 1) * 0.05, dtype=torch.float64)
    YtY = (Y.double().T @ Y.double()) if implicit else None
    args = (indptr.cuda(), nbr.cuda(), rt.cuda(), Y.cuda(), reg.cuda(), implicit, 2.0,
            None if YtY is None else YtY.cuda())
    monkeypatch.setattr(aops, "WOODBURY", 0)           # every row through the r x r kernels
    monkeypatch.setattr(aops, "MFMA_LIGHT", 1)
    a = aops.fused_solve(*args).cpu().double().numpy()
    monkeypatch.setattr(aops, "MFMA_LIGHT", 0)
    b = aops.fused_solve(*args).cpu().double().numpy()
    A, bb = aops.normal_equations_torch(indptr, nbr, rt, Y, implicit, 2.0)
    if implicit:
        A = A + YtY[None]
    A = A + reg[:, None, None] * torch.eye(r, dtype=torch.float64)[None]
    ref = torch.cholesky_solve(bb[:, :, None], torch.linalg.cholesky(A))[:, :, 0].float().double().numpy()
    np.testing.assert_allclose(a, ref, rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(a, b, rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("r", [10, 24, 62, 64])
def test_hip_als_woodbury16_mfma_matches_lds_kernel(r, monkeypatch):
    """Explicit rows with 9..16 ratings on the f64 matrix cores (alink_als_woodbury16_mfma: MFMA Gram, sweep
    inverse, reduce-scatter Y^T a) == the LDS-staged push-through kernel and fp64 Cholesky; r % 4 != 0 takes the
    scalar loads; repeated neighbours; a lambda = 0 row."""
    rng = np.random.default_rng(70 + r)
    n = 700
    counts = np.concatenate([[9, 16, 12, 16, 10], rng.integers(9, 17, size=3000)])
    m = counts.size
    indptr = torch.zeros(m + 1, dtype=torch.int64)
    indptr[1:] = torch.as_tensor(np.cumsum(counts))
    nnz = int(indptr[-1])
    nbr = rng.integers(0, n, size=nnz)
    nbr[int(indptr[2]):int(indptr[3])] = nbr[int(indptr[2])]
    nbr = torch.as_tensor(nbr, dtype=torch.int32)
    rt = torch.as_tensor(rng.integers(1, 6, size=nnz).astype(np.float32))
    Y = torch.as_tensor(rng.normal(size=(n, r)) * 0.3, dtype=torch.float32)
    reg = torch.as_tensor(counts * 0.05, dtype=torch.float64)
    reg[4] = 0.0
    args = (indptr.cuda(), nbr.cuda(), rt.cuda(), Y.cuda(), reg.cuda(), False, 0.0, None)
    monkeypatch.setattr(aops, "WOODBURY", 1)
    monkeypatch.setattr(aops, "WOODBURY_MFMA", 1)
    a = aops.fused_solve(*args).cpu().double().numpy()
    monkeypatch.setattr(aops, "WOODBURY_MFMA", 0)
    b = aops.fused_solve(*args).cpu().double().numpy()
    np.testing.assert_allclose(a, b, rtol=2e-5, atol=2e-6)
    A, bb = aops.normal_equations_torch(indptr, nbr, rt, Y, False, 0.0)
    A = A + reg[:, None, None] * torch.eye(r, dtype=torch.float64)[None]
    ref = (torch.linalg.pinv(A) @ bb[:, :, None])[:, :, 0].numpy()
    np.testing.assert_allclose(a, ref, rtol=2e-4, atol=2e-5)


def test_als_model_rows_native_format_and_parse():
    """ALS model rows: factor strings from the C++ Float.toString formatter equal the per-value formatter's, and
    the C++ reader loads them back bit-exactly (NaN tokens fall back to the per-row path)."""
    import numpy as np
    from alink_amd.common.javafmt import java_float_str
    from alink_amd.models.recommendation.als import AlsModelData, AlsModelDataConverter
    rng = np.random.default_rng(1)
    uf = (rng.normal(size=(300, 16)) * 10.0 ** rng.integers(-9, 9, size=(300, 16))).astype(np.float32)
    itf = rng.normal(size=(50, 16)).astype(np.float32)
    m = AlsModelData(np.arange(300) * 7, uf, np.arange(50) + 1000, itf)
    conv = AlsModelDataConverter("u", "i")
    rows = conv.save(m)
    assert rows[5][2] == " ".join(java_float_str(float(v)) for v in uf[5]) and rows[5][:2] == (35, None)
    assert rows[300 + 3][:2] == (None, 1003)
    got = conv.load(rows)
    assert np.array_equal(got.user_factors, uf) and np.array_equal(got.item_factors, itf)
    assert got.user_ids.tolist() == (np.arange(300) * 7).tolist() and got.user_map[14] == 2
    uf[3, 2] = np.nan
    rows = conv.save(AlsModelData(np.arange(300), uf, np.arange(50), itf))
    assert "NaN" in rows[3][2]
    got = conv.load(rows)
    assert np.array_equal(got.user_factors, uf, equal_nan=True)
