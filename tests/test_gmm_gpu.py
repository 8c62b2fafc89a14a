"""K22 GMM E-step (one GEMM + ops/csrc/gmm.hip fused log-density / responsibilities) against the per-component
fp64 torch formula, plus a GMM training run on cuda equal to the CPU run."""
import math

import numpy as np
import pytest
import torch

from alink_amd.models.clustering.gmm import _root_inv
from alink_amd.ops import _lib
from alink_amd.ops import gmm as G

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,k,d", [(1, 1, 1), (1000, 3, 2), (20001, 10, 50), (4097, 64, 7), (3000, 5, 130)])
def test_gmm_estep_matches_torch(n, k, d):
    _lib.require()
    g = torch.Generator(device="cuda").manual_seed(n + k + d)
    X0 = torch.randn(n, d, device="cuda", dtype=torch.float64, generator=g)
    mu0 = torch.randn(k, d, device="cuda", dtype=torch.float64, generator=g)
    A = torch.randn(k, d, d, device="cuda", dtype=torch.float64, generator=g)
    S = A @ A.transpose(1, 2) / d + 0.1 * torch.eye(d, device="cuda", dtype=torch.float64)
    if d > 3:
        S[0] = S[0] * 0
        S[0, :3, :3] = torch.eye(3, device="cuda", dtype=torch.float64)   # rank-deficient component
    W, logdet, rank = _root_inv(S)
    logw = torch.log(torch.softmax(torch.randn(k, device="cuda", dtype=torch.float64, generator=g), 0))
    R, ll = G.estep(X0, mu0, W, logdet, rank, logw)
    R0, ll0 = G.estep_torch(X0, mu0, W, logdet, rank, logw)
    torch.testing.assert_close(R, R0, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(float(ll), float(ll0), rtol=1e-11)


def test_gmm_train_cuda_equals_cpu():
    _lib.require()
    from alink_amd import useLocalEnv, GmmTrainBatchOp, GmmPredictBatchOp
    from alink_amd.operator.batch.source import MemSourceBatchOp
    rng = np.random.default_rng(5)
    pts = np.concatenate([rng.normal(-3, 1, size=(300, 2)), rng.normal(3, 0.5, size=(300, 2))])
    rows = [["%f %f" % (a, b)] for a, b in pts]
    preds = {}
    for dev in ("cpu", "cuda:0"):
        useLocalEnv(1, device=dev)
        src = MemSourceBatchOp(rows, "vec string")
        m = GmmTrainBatchOp().setVectorCol("vec").setK(2).setMaxIter(20).linkFrom(src)
        preds[dev] = [r[-1] for r in GmmPredictBatchOp().setPredictionCol("p").linkFrom(m, src).collect()]
    useLocalEnv(1, device="cpu")
    assert preds["cpu"] == preds["cuda:0"]


def test_weighted_syrk_matches_einsum():
    from alink_amd.models.clustering.gmm import _weighted_syrk
    g = torch.Generator(device="cuda").manual_seed(11)
    R = torch.rand(40001, 6, device="cuda", dtype=torch.float64, generator=g)
    X = torch.randn(40001, 9, device="cuda", dtype=torch.float64, generator=g)
    torch.testing.assert_close(_weighted_syrk(R, X), torch.einsum("nk,nd,ne->kde", R, X, X), rtol=1e-11, atol=1e-9)
