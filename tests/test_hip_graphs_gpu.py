"""hipGraph replay of the L-BFGS two-loop recursion (models/linear/optim._two_loop_graph) against the eager
ops: identical directions, including after the history buffers change in place between replays and across the
rotation of the circular history (k > m, the rotation is a device scalar inside one captured graph)."""
import pytest
import torch

from alink_amd.models.linear import optim

pytestmark = pytest.mark.gpu


class _Ctx:
    def __init__(self, sK, yK):
        self.o = {optim.SKYK: (sK, yK)}

    def getObj(self, name):
        return self.o[name]


@pytest.mark.parametrize("d", [7, 1000, 70000])
def test_two_loop_graph_matches_eager(monkeypatch, d):
    g = torch.Generator(device="cuda").manual_seed(d)
    m = optim.NUM_CORRECTIONS
    sK = torch.randn(m, d, device="cuda", dtype=torch.float64, generator=g)
    yK = sK + 0.1 * torch.randn(m, d, device="cuda", dtype=torch.float64, generator=g)
    yK[3] = -sK[3]                               # s.y < 0: that pair is skipped (rho = 0) on both paths
    ctx = _Ctx(sK, yK)
    c0, r0 = optim.GRAPH_STATS["captures"], optim.GRAPH_STATS["replays"]
    for k in [1, 4, 10, 11, 17, 10, 23]:
        gv = torch.randn(d, device="cuda", dtype=torch.float64, generator=g)
        monkeypatch.setenv("ALINK_HIP_GRAPHS", "1")
        a = optim._two_loop(ctx, gv, gv, k)
        monkeypatch.setenv("ALINK_HIP_GRAPHS", "0")
        b = optim._two_loop(ctx, gv, gv, k)
        torch.cuda.synchronize()
        assert torch.equal(a, b), k
        # the history changes in place between supersteps: the replayed graph must read the new values
        sK[k % m].mul_(0.5)
        yK[(k + 3) % m].add_(0.25)
    # one capture for this history (first full-history superstep), replayed for every k >= m whatever the rotation
    assert optim.GRAPH_STATS["captures"] == c0 + 1
    assert optim.GRAPH_STATS["replays"] == r0 + 5


def test_logistic_regression_graphs_on_off_identical(monkeypatch):
    from alink_amd import useLocalEnv
    from alink_amd.common.params import Params
    from alink_amd.models.common.features import FeatureMatrix
    from alink_amd.models.linear.objfunc import LabeledData, LogLossFunc, UnaryLossObjFunc
    env = useLocalEnv(1, device="cuda:0")
    g = torch.Generator(device="cuda").manual_seed(0)
    n, d = 20000, 24
    X = torch.randn(n, d, device="cuda", generator=g, dtype=torch.float64)
    wt = torch.randn(d, device="cuda", generator=g, dtype=torch.float64)
    y = torch.where(X @ wt + 0.5 * torch.randn(n, device="cuda", generator=g, dtype=torch.float64) > 0, 1.0, -1.0)
    data = LabeledData(FeatureMatrix(dense=X), y, torch.ones(n, device="cuda", dtype=torch.float64))
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("ALINK_HIP_GRAPHS", flag)
        coef, curve = optim.optimize(UnaryLossObjFunc(LogLossFunc(), 0.0, 0.0), data, d,
                                     Params().set("maxIter", 25).set("epsilon", 1e-30), env=env)
        import numpy as np
        c = coef.cpu() if torch.is_tensor(coef) else torch.as_tensor(np.asarray(getattr(coef, "data", coef)))
        res[flag] = (c, np.asarray([float(v) for v in curve]).tolist())
    assert torch.equal(res["1"][0], res["0"][0])
    assert res["1"][1] == res["0"][1]
