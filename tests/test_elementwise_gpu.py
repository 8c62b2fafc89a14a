"""Fused elementwise HIP kernels (ops/csrc/elementwise.hip: K6 GBDT g/h + leaf update, K27 column transforms)
against the plain torch chains they replace (bit-identical), plus an end-to-end GBDT / scaler run on cuda."""
import numpy as np
import pytest
import torch

from alink_amd.ops import _lib
from alink_amd.ops import elementwise as ew

pytestmark = pytest.mark.gpu


def _loaded():
    _lib.require()


@pytest.mark.parametrize("n", [1, 1000, 257 * 1024 + 3])
@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("weighted", [False, True])
def test_gbdt_grad_stats_bitwise(n, algo, weighted):
    _loaded()
    g = torch.Generator(device="cuda").manual_seed(n + algo)
    pred = torch.randn(n, device="cuda", generator=g) * 4
    y = (torch.rand(n, device="cuda", generator=g) < 0.4).float() if algo else torch.randn(n, device="cuda",
                                                                                        generator=g)
    w = torch.rand(n, device="cuda", generator=g) + 0.5 if weighted else None
    a = ew.gbdt_grad_stats(pred, y, w, algo)
    b = ew.gbdt_grad_stats_torch(pred, y, w, algo)
    torch.cuda.synchronize()
    assert a.shape == (n, 4)
    # logistic uses fp64 exp on both sides; allow one fp32 ulp in case the libm paths round differently
    torch.testing.assert_close(a, b, rtol=1.2e-7 if algo else 0, atol=1e-30 if algo else 0)


def test_gbdt_leaf_update_matches_torch():
    _loaded()
    n = 100003
    g = torch.Generator(device="cuda").manual_seed(3)
    pred = torch.randn(n, device="cuda", generator=g)
    codes = torch.randint(-40, 5, (n,), device="cuda", dtype=torch.int32, generator=g)
    vals = torch.randn(37, device="cuda", dtype=torch.float64, generator=g)   # codes below -37 clamp to the last
    ref = ew.gbdt_leaf_update_torch(pred.clone(), codes, vals)
    out = ew.gbdt_leaf_update(pred.clone(), codes, vals)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("mode", ["standard", "minmax", "maxabs", "impute", "binarize"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("shape", [(5000, 7), (1, 1), (70001,), (3000, 129)])
def test_col_transform_bitwise(mode, dtype, shape):
    _loaded()
    g = torch.Generator(device="cuda").manual_seed(sum(shape))
    X = (torch.randn(*shape, device="cuda", generator=g, dtype=torch.float64) * 3 + 1).to(dtype)
    d = shape[1] if len(shape) == 2 else 1
    if mode == "impute":
        X.view(-1)[::11] = float("nan")
    a = torch.randn(d, dtype=torch.float64, device="cuda", generator=g)
    b = a + torch.rand(d, dtype=torch.float64, device="cuda", generator=g) * 5
    if d > 2:
        a[1] = 0.0
        b[2] = a[2]          # zero range / zero std / zero max-abs columns take the constant branch
        b[1] = 0.0
    out = ew.col_transform(X, mode, a, b, -1.0, 2.0)
    ref = ew.col_transform_torch(X, mode, a, b, -1.0, 2.0)
    torch.cuda.synchronize()
    assert out.dtype == torch.float64 and out.shape == X.shape
    assert torch.equal(torch.nan_to_num(out, nan=123.0), torch.nan_to_num(ref, nan=123.0))


def test_gbdt_and_scalers_end_to_end_on_cuda():
    """GBDT (logistic) and the column / vector scalers on a cuda local env: same model and outputs as on CPU."""
    _loaded()
    from alink_amd import (useLocalEnv, GbdtTrainBatchOp, GbdtPredictBatchOp, StandardScalerTrainBatchOp,
                           StandardScalerPredictBatchOp, MinMaxScalerTrainBatchOp, MinMaxScalerPredictBatchOp)
    from alink_amd.operator.batch.source import MemSourceBatchOp
    rng = np.random.default_rng(0)
    rows = [[float(a), float(b), int(a + b > 0)] for a, b in rng.normal(size=(400, 2))]
    outs = {}
    for dev in ("cpu", "cuda:0"):
        useLocalEnv(1, device=dev)
        src = MemSourceBatchOp(rows, "f0 double, f1 double, label int")
        model = GbdtTrainBatchOp().setFeatureCols(["f0", "f1"]).setLabelCol("label").setNumTrees(5) \
            .setMinSamplesPerLeaf(5).linkFrom(src)
        pred = GbdtPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d").linkFrom(model, src)
        sm = StandardScalerTrainBatchOp().setSelectedCols(["f0", "f1"]).linkFrom(src)
        sp = StandardScalerPredictBatchOp().linkFrom(sm, src)
        mm = MinMaxScalerTrainBatchOp().setSelectedCols(["f0", "f1"]).linkFrom(src)
        mp = MinMaxScalerPredictBatchOp().linkFrom(mm, src)
        outs[dev] = (pred.collect(), sp.collect(), mp.collect())
    useLocalEnv(1, device="cpu")
    p_cpu, s_cpu, m_cpu = outs["cpu"]
    p_gpu, s_gpu, m_gpu = outs["cuda:0"]
    assert [r[-2] for r in p_cpu] == [r[-2] for r in p_gpu]
    np.testing.assert_allclose(np.array([r[:2] for r in s_cpu], dtype=float),
                               np.array([r[:2] for r in s_gpu], dtype=float), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(np.array([r[:2] for r in m_cpu], dtype=float),
                               np.array([r[:2] for r in m_gpu], dtype=float), rtol=1e-12, atol=1e-12)
