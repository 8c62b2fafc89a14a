"""Sparse (CSR/CSC) linear-model gradient kernels (ops/csrc/linear.hip) vs fp64 torch, and LR training on
hashed sparse features in a GPU environment vs the CPU environment."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _fm(n, d, nnz_row, seed, dev):
    from alink_amd.models.common.features import FeatureMatrix
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(1, nnz_row, (n,), generator=g)
    crow = torch.zeros(n + 1, dtype=torch.int64)
    crow[1:] = torch.cumsum(lens + 1, 0)
    cols, vals = [], []
    for i in range(n):
        c = torch.randint(1, d, (int(lens[i]),), generator=g).unique()
        cols.append(torch.cat([torch.zeros(1, dtype=torch.int64), c]))     # column 0 in every row (hot)
        vals.append(torch.randn(c.numel() + 1, generator=g, dtype=torch.float64))
    crow[1:] = torch.cumsum(torch.tensor([x.numel() for x in cols]), 0)
    return FeatureMatrix(crow=crow.to(dev), col=torch.cat(cols).to(dev), val=torch.cat(vals).to(dev), ncols=d)


@pytest.mark.parametrize("loss", ["log", "square", "hinge", "smooth", "huber"])
def test_sparse_grad_kernel_matches_fp64_torch(loss):
    from alink_amd.models.linear import objfunc as O
    from alink_amd.ops import linear as lops
    fn = {"log": O.LogLossFunc(), "square": O.SquareLossFunc(), "hinge": O.HingeLossFunc(),
          "smooth": O.SmoothHingeLossFunc(), "huber": O.HuberLossFunc(0.7)}[loss]
    n, d = 20000, 5000
    fm = _fm(n, d, 30, 1, "cuda")
    g = torch.Generator().manual_seed(2)
    y = (torch.randint(0, 2, (n,), generator=g) * 2 - 1).double().cuda()
    w = torch.rand(n, generator=g, dtype=torch.float64).cuda()
    coef = (0.1 * torch.randn(d, generator=g, dtype=torch.float64)).cuda()
    code, prm = lops.loss_code(fn)
    got, lsum, wsum = lops.sparse_grad_hip(fm, y, w, coef, code, prm)
    eta = fm.mv(coef)
    ref = fm.rmv(w * fn.derivative(eta, y), d)
    torch.testing.assert_close(got, ref, rtol=1e-10, atol=1e-9)
    torch.testing.assert_close(lsum, (w * fn.loss(eta, y)).sum(), rtol=1e-10, atol=1e-9)
    again, _, _ = lops.sparse_grad_hip(fm, y, w, coef, code, prm)
    assert torch.equal(got, again)                         # no atomics: bitwise deterministic


def test_lr_on_hashed_sparse_features_gpu_equals_cpu():
    import pandas as pd
    from alink_amd import useLocalEnv, BatchOperator, FeatureHasherBatchOp, LogisticRegressionTrainBatchOp
    from alink_amd.common.mlenv import resetEnv
    rng = np.random.default_rng(3)
    n = 5000
    df = pd.DataFrame({f"c{i}": rng.choice([f"v{j}" for j in range(200)], n) for i in range(6)})
    df["label"] = (rng.random(n) < 0.4).astype(int)
    out = {}
    for dev in ("cpu", "cuda:0"):
        resetEnv()
        useLocalEnv(1, device=dev)
        src = BatchOperator.fromDataframe(df, schemaStr=", ".join(f"c{i} string" for i in range(6)) + ", label int")
        h = FeatureHasherBatchOp().setSelectedCols([f"c{i}" for i in range(6)]).setOutputCol("v") \
            .setNumFeatures(30000).linkFrom(src)
        m = LogisticRegressionTrainBatchOp().setVectorCol("v").setLabelCol("label").setMaxIter(15).setL2(0.01) \
            .linkFrom(h)
        from alink_amd.models.linear.model import LinearModelDataConverter
        out[dev] = np.asarray(LinearModelDataConverter().load(m.collect()).coefVector.data)
    np.testing.assert_allclose(out["cuda:0"], out["cpu"], rtol=1e-7, atol=1e-9)
