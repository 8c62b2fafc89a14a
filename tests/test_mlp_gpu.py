"""K17 MLP backprop (GEMMs + ops/csrc/elementwise.hip bias-sigmoid / sigmoid-backward + pivot-free K16 softmax)
against torch autograd of the same network, plus an MLP classifier run on cuda against the CPU run."""
import numpy as np
import pytest
import torch

from alink_amd.models.classification.mlp import mlp_forward, weight_size
from alink_amd.ops import _lib
from alink_amd.ops import mlp as M
from alink_amd.ops import softmax as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,K", [(1, 2), (5000, 3), (70001, 10), (999, 32)])
def test_softmax_full_grad_matches_torch(n, K):
    L = _lib.require()
    g = torch.Generator(device="cuda").manual_seed(n + K)
    z = torch.randn(n, K, device="cuda", dtype=torch.float64, generator=g) * 4
    y = torch.randint(0, K, (n,), device="cuda", generator=g).double()
    w = torch.rand(n, device="cuda", dtype=torch.float64, generator=g) + 0.5
    R = torch.empty_like(z)
    part = torch.zeros(L.alink_softmax_grid(n), dtype=torch.float64, device="cuda")
    assert L.alink_softmax_full_grad_f64(z.data_ptr(), y.data_ptr(), w.data_ptr(), n, K, R.data_ptr(),
                                         part.data_ptr(), _lib.stream_ptr()) == 0
    R0, loss0 = S.softmax_full_grad_torch(z, y, w)
    torch.testing.assert_close(R, R0, rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(float(part.sum()), float(loss0), rtol=1e-12)


@pytest.mark.parametrize("layers", [[4, 3], [5, 7, 3], [16, 32, 8, 10], [3, 6, 2]])
def test_mlp_grad_matches_autograd(layers):
    _lib.require()
    n = 3001
    g = torch.Generator(device="cuda").manual_seed(sum(layers))
    X = torch.randn(n, layers[0], device="cuda", dtype=torch.float64, generator=g)
    y = torch.randint(0, layers[-1], (n,), device="cuda", generator=g).double()
    w = torch.rand(n, device="cuda", dtype=torch.float64, generator=g) + 0.5
    coef = torch.randn(weight_size(layers), device="cuda", dtype=torch.float64, generator=g) * 0.5
    grad, loss = M.mlp_grad(X, y, w, coef, layers)

    wt = coef.clone().requires_grad_(True)
    P = mlp_forward(X, wt, layers)
    ce = -torch.log(P.gather(1, y.long()[:, None])[:, 0])
    (g0,) = torch.autograd.grad((ce * w).sum(), wt)
    torch.testing.assert_close(grad, g0, rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(float(loss), float((ce * w).sum()), rtol=1e-11)


def test_mlp_classifier_cuda_equals_cpu():
    _lib.require()
    from alink_amd import useLocalEnv, MultilayerPerceptronTrainBatchOp, MultilayerPerceptronPredictBatchOp
    from alink_amd.operator.batch.source import MemSourceBatchOp
    rng = np.random.default_rng(2)
    X = rng.normal(size=(500, 4))
    lab = (X[:, 0] * X[:, 1] > 0).astype(int) + (X[:, 2] > 1).astype(int)
    rows = [[float(a), float(b), float(c), float(e), int(l)] for (a, b, c, e), l in zip(X, lab)]
    preds = {}
    for dev in ("cpu", "cuda:0"):
        useLocalEnv(1, device=dev)
        src = MemSourceBatchOp(rows, "f0 double, f1 double, f2 double, f3 double, label int")
        m = MultilayerPerceptronTrainBatchOp().setFeatureCols(["f0", "f1", "f2", "f3"]).setLabelCol("label") \
            .setLayers([4, 8, 3]).setMaxIter(50).linkFrom(src)
        preds[dev] = [r[-1] for r in MultilayerPerceptronPredictBatchOp().setPredictionCol("p").linkFrom(m, src)
                      .collect()]
    useLocalEnv(1, device="cpu")
    agree = np.mean(np.array(preds["cpu"]) == np.array(preds["cuda:0"]))
    assert agree > 0.98, agree
