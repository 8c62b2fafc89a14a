"""K16 fused softmax epilogues (ops/csrc/softmax.hip) against the fp64 torch formulas, plus a Softmax
training run on cuda equal to the CPU run."""
import numpy as np
import pytest
import torch

from alink_amd.ops import _lib
from alink_amd.ops import softmax as S

pytestmark = pytest.mark.gpu


def _data(n, k1, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    eta = torch.randn(n, k1, device="cuda", dtype=torch.float64, generator=g) * 3
    y = torch.randint(0, k1 + 1, (n,), device="cuda", generator=g).double()   # k1 = the pivot class
    w = torch.rand(n, device="cuda", dtype=torch.float64, generator=g) + 0.25
    return eta, y, w


@pytest.mark.parametrize("n", [1, 777, 300001])
@pytest.mark.parametrize("k1", [1, 2, 4, 9, 16, 31])
def test_softmax_grad_matches_torch(n, k1):
    _lib.require()
    eta, y, w = _data(n, k1, n + k1)
    R, loss = S.softmax_grad(eta, y, w)
    R0, loss0 = S.softmax_grad_torch(eta.clone(), y, w)
    torch.testing.assert_close(R, R0, rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(float(loss), float(loss0), rtol=1e-12)


@pytest.mark.parametrize("k1", [1, 3, 16, 32])
@pytest.mark.parametrize("nsteps", [1, 5, 11])
def test_softmax_search_matches_torch(k1, nsteps):
    _lib.require()
    ec, y, w = _data(50001, k1, 7 * k1 + nsteps)
    ed = torch.randn_like(ec)
    a = S.softmax_search(ec, ed, y, w, 0.37, nsteps)
    b = S.softmax_search_torch(ec, ed, y, w, 0.37, nsteps)
    assert a.shape == (nsteps,)
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-12)


def test_softmax_train_cuda_equals_cpu():
    _lib.require()
    from alink_amd import useLocalEnv, SoftmaxTrainBatchOp, SoftmaxPredictBatchOp
    from alink_amd.operator.batch.source import MemSourceBatchOp
    rng = np.random.default_rng(1)
    X = rng.normal(size=(600, 3))
    lab = np.argmax(X @ rng.normal(size=(3, 4)) + 0.3 * rng.normal(size=(600, 4)), 1)
    rows = [[float(a), float(b), float(c), int(l)] for (a, b, c), l in zip(X, lab)]
    preds = {}
    for dev in ("cpu", "cuda:0"):
        useLocalEnv(1, device=dev)
        src = MemSourceBatchOp(rows, "f0 double, f1 double, f2 double, label int")
        m = SoftmaxTrainBatchOp().setFeatureCols(["f0", "f1", "f2"]).setLabelCol("label").setMaxIter(30) \
            .linkFrom(src)
        preds[dev] = [r[-1] for r in SoftmaxPredictBatchOp().setPredictionCol("p").linkFrom(m, src).collect()]
    useLocalEnv(1, device="cpu")
    agree = np.mean(np.array(preds["cpu"]) == np.array(preds["cuda:0"]))
    assert agree > 0.995, agree
