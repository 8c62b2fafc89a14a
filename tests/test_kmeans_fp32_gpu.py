"""KMeans on fp32 / fp64 feature matrices on the GPU: the fp32 GEMM-assign + HIP accumulate-by-index path
(ops/kmeans.assign_accumulate_f32_hip, csrc/kmeans_accum.hip alink_kmeans_accum_f32) against the fp64 PyTorch
reference, and the ALINK_KMEANS_INPUT opt-in casts of fp64 training data."""
import numpy as np
import pytest
import torch

from alink_amd.ops import kmeans as K

pytestmark = pytest.mark.gpu


def _data(n, d, k, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    centers = torch.randn(k, d, device="cuda", generator=g, dtype=torch.float64) * 6
    lab = torch.randint(0, k, (n,), device="cuda", generator=g)
    X = centers[lab] + torch.randn(n, d, device="cuda", generator=g, dtype=torch.float64)
    C = centers + 0.3 * torch.randn(k, d, device="cuda", generator=g, dtype=torch.float64)
    return X, C


@pytest.mark.parametrize("n,d,k,weighted", [(300_000, 128, 100, False), (200_001, 64, 300, True),
                                            (100_000, 256, 50, False)])
def test_fp32_assign_accumulate_matches_fp64(n, d, k, weighted):
    X64, C = _data(n, d, k)
    X = X64.float().contiguous()
    w = torch.rand(n, device="cuda") + 0.5 if weighted else None
    assert K.f32_supported(X, k)
    calls = K.F32_CALLS
    got = K.assign_accumulate(X, C, w)
    assert K.F32_CALLS == calls + 1
    ref = K.assign_accumulate_torch(X.double(), C, None if w is None else w.double())
    torch.cuda.synchronize()
    # the fp32 GEMM may flip a near-tie row; counts (weights) agree to a handful of rows
    assert float((got[:, -1] - ref[:, -1]).abs().sum()) <= 4.0 * (2.0 if weighted else 1.0)
    scale = ref[:, :-1].abs().max()
    assert float((got[:, :-1] - ref[:, :-1]).abs().max() / scale) < 2e-3


def test_kmeans_train_fp64_input_casts(monkeypatch):
    """fp64 vector column (what VectorAssembler produces): the default stays on the fp64 path; the opt-in fp32
    cast runs the HIP fp32 path and lands within 1e-2 of the fp64 centroids (closer than bf16), bf16 on the fused
    kernel within 0.2 % of the fp64 objective (SSE)."""
    from alink_amd import useLocalEnv, KMeansTrainBatchOp
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    from alink_amd.models.clustering.kmeans import KMeansModelDataConverter
    useLocalEnv(1, device="cuda:0")
    X64, _ = _data(400_000, 128, 20, seed=3)
    mt = MTable(TableSchema(["vec"], [Types.DENSE_VECTOR]), [Column(X64)])

    def fit(mode):
        if mode:
            monkeypatch.setenv("ALINK_KMEANS_INPUT", mode)
        else:
            monkeypatch.delenv("ALINK_KMEANS_INPUT", raising=False)
        op = KMeansTrainBatchOp().setVectorCol("vec").setK(20).setMaxIter(8).setEpsilon(-1.0) \
            .setInitMode("RANDOM").linkFrom(TableSourceBatchOp(mt))
        md = KMeansModelDataConverter().load(op.collect())
        return md.centroids[np.argsort(md.centroids[:, 0])], md.weights
    c64, w64 = fit(None)
    calls = K.F32_CALLS
    c32, w32 = fit("fp32")
    assert K.F32_CALLS > calls
    # 8 Lloyd steps: the few boundary rows whose fp32 / fp64 nearest centroids differ move the means by ~1e-3
    np.testing.assert_allclose(c32, c64, rtol=1e-2, atol=1e-2)
    np.testing.assert_allclose(w32, w64, rtol=1e-2)
    cb, _ = fit("bf16")

    def sse(c):
        return float(torch.cdist(X64, torch.as_tensor(c, device=X64.device)).min(1).values.square().sum())
    # bf16 rounding moves a boundary here and there (a centroid can drift by ~0.1): judge it by the objective
    s64, s32, sb = sse(c64), sse(c32), sse(cb)
    assert abs(s32 - s64) / s64 < 1e-5
    assert abs(sb - s64) / s64 < 2e-3
    assert np.abs(c32 - c64).mean() < np.abs(cb - c64).mean()
