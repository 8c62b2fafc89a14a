"""BSP engine tests after the reference's ``core/src/test/java/com/alibaba/alink/common/comqueue/
{IterativeComQueueTest,BaseComQueueTest}.java``: Monte-Carlo pi with per-task state, linear regression by
gradient + ``AllReduce("grads")`` + update over local tasks, the compute-fusion optimizer seen through ``str``,
and the stop criterion of task 0."""
import numpy as np
import torch

from alink_amd import useLocalEnv
from alink_amd.parallel.comqueue import (AllReduce, CompareCriterionFunction, CompleteResultFunction,
                                         ComputeFunction, IterativeComQueue)


class _Noop(ComputeFunction):
    def calc(self, ctx):
        pass


class _Comm(AllReduce):
    def __init__(self):
        super().__init__("x")


def test_compute_fusion_optimizer_through_str():
    """BaseComQueueTest: adjacent compute functions fuse into one ChainedComputation; communication items
    split the chains; the queue prints as the reference's JSON."""
    import re
    q = IterativeComQueue().add(_Noop()).add(_Noop()).add(_Comm()).add(_Comm()).add(_Noop()).add(_Noop()) \
        .add(_Comm())
    assert re.fullmatch(r'\{"completeResult":null,"maxIter":2147483647,"sessionId":[0-9]*,"queue":'
                        r'"ChainedComputation,_Comm,_Comm,ChainedComputation,_Comm","compareCriterion":null\}', str(q))
    assert '"queue":""' in str(IterativeComQueue())
    assert '"queue":"_Noop"' in str(IterativeComQueue().add(_Noop()))
    assert '"queue":"_Comm"' in str(IterativeComQueue().add(_Comm()))


def test_pi_with_per_task_state():
    env = useLocalEnv(4)

    class Sample(ComputeFunction):
        def calc(self, ctx):
            g = torch.Generator().manual_seed(17 * ctx.getTaskId() + ctx.getStepNo())
            p = torch.rand((5000, 2), generator=g, dtype=torch.float64)
            inside = float(((p ** 2).sum(1) <= 1.0).sum())
            steps = (ctx.getObj("steps") or 0) + 1                   # per-task state survives supersteps
            ctx.putObj("steps", steps)
            acc = ctx.getObj("acc")
            acc = torch.tensor([inside, 5000.0], dtype=torch.float64) + (0 if acc is None else acc)
            ctx.putObj("acc", acc)
            ctx.putObj("sum", acc.clone())

    class Out(CompleteResultFunction):
        def calc(self, ctx):
            s = ctx.getObj("sum")
            return [(ctx.getTaskId(), ctx.getObj("steps"), float(4.0 * s[0] / s[1]))]

    rows = IterativeComQueue().setMLEnvironment(env).add(Sample()).add(AllReduce("sum")).closeWith(Out()) \
        .setMaxIter(6).exec()
    assert sorted(r[0] for r in rows) == [0, 1, 2, 3]
    assert all(r[1] == 6 for r in rows)
    assert len({r[2] for r in rows}) == 1 and abs(rows[0][2] - np.pi) < 0.02


def _icq_linear_regression(n, m=10000, iters=100, lr=1.0, tasks=4):
    env = useLocalEnv(tasks)
    rng = np.random.default_rng(0)
    X = np.concatenate([rng.random((m, n)), np.ones((m, 1))], 1)
    y = X[:, :n].sum(1)
    data = torch.as_tensor(np.concatenate([X, y[:, None]], 1))

    class Grad(ComputeFunction):
        def calc(self, ctx):
            part, coef = ctx.getObj("train"), ctx.getObj("coef")
            Xp, yp = part[:, :-1], part[:, -1]
            ctx.putObj("grads", Xp.T @ (yp - Xp @ coef))

    class Update(ComputeFunction):
        def calc(self, ctx):
            ctx.putObj("coef", ctx.getObj("coef") + ctx.getObj("grads") * (lr / ctx.getObj("count")))

    class Out(CompleteResultFunction):
        def calc(self, ctx):
            return [(ctx.getObj("coef").numpy(),)] if ctx.getTaskId() == 0 else None

    rows = IterativeComQueue().setMLEnvironment(env).setMaxIter(iters) \
        .initWithPartitionedData("train", data) \
        .initWithBroadcastData("coef", torch.zeros(n + 1, dtype=torch.float64)) \
        .initWithBroadcastData("count", float(m)) \
        .add(Grad()).add(AllReduce("grads")).add(Update()).closeWith(Out()).exec()
    assert len(rows) == 1
    return X, y, rows[0][0]


def test_icq_linear_regression():
    X, y, coef = _icq_linear_regression(3)
    assert abs(float(X[0] @ coef) - y[0]) < 2.0                   # the reference's tolerance
    assert np.abs(X @ coef - y).mean() < 0.05                      # and it actually fits


def test_icq_linear_regression_20_features_same_on_one_and_four_tasks():
    _, _, c4 = _icq_linear_regression(20, iters=30, tasks=4)
    _, _, c1 = _icq_linear_regression(20, iters=30, tasks=1)
    np.testing.assert_allclose(c4, c1, rtol=1e-9, atol=1e-12)


def test_stop_criterion_of_task0():
    env = useLocalEnv(2)

    class Count(ComputeFunction):
        def calc(self, ctx):
            ctx.putObj("n", ctx.getStepNo())

    class Stop(CompareCriterionFunction):
        def calc(self, ctx):
            return ctx.getObj("n") >= 4

    class Out(CompleteResultFunction):
        def calc(self, ctx):
            return [(ctx.getTaskId(), ctx.getObj("n"))]

    rows = IterativeComQueue().setMLEnvironment(env).add(Count()).setCompareCriterionOfNode0(Stop()) \
        .closeWith(Out()).setMaxIter(100).exec()
    assert sorted(rows) == [(0, 4), (1, 4)]
