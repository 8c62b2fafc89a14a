"""Device tree-ensemble prediction (``ops/csrc/tree_predict.hip``) against the host walk of the same mapper: GBDT
(binary and regression), random forest (multi-class, regression) with categorical splits and missing values."""
import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu


def _frame(n=3000, seed=0, classes=2):
    rng = np.random.default_rng(seed)
    x0 = rng.normal(size=n)
    x1 = rng.normal(size=n)
    cat = rng.choice(["a", "b", "c", "d", "e"], n)
    y_num = x0 - 0.5 * x1 + (cat == "c") * 1.5 + 0.2 * rng.normal(size=n)
    q = np.quantile(y_num, np.linspace(0, 1, classes + 1)[1:-1])
    y = np.searchsorted(q, y_num)
    df = pd.DataFrame({"x0": x0, "x1": x1, "c": cat, "y": y, "t": y_num})
    return df


def _with_missing(df, seed=1):
    rng = np.random.default_rng(seed)
    df = df.copy().astype({"x0": object, "c": object})
    m0 = rng.random(len(df)) < 0.1
    m1 = rng.random(len(df)) < 0.1
    df.loc[m0, "x0"] = None
    df.loc[m1, "c"] = None
    df.loc[rng.random(len(df)) < 0.03, "c"] = "unseen"
    return df


SCHEMA = "x0 double, x1 double, c string, y int, t double"


def _predict_both(train_op, pred_cls, df_train, df_pred, detail=True):
    from alink_amd import BatchOperator, useLocalEnv
    from alink_amd.models.tree import model as tm
    useLocalEnv(1, device="cuda:0")
    model = train_op.linkFrom(BatchOperator.fromDataframe(df_train, schemaStr=SCHEMA))
    src = BatchOperator.fromDataframe(df_pred, schemaStr=SCHEMA)

    def run():
        op = pred_cls().setPredictionCol("p")
        if detail:
            op = op.setPredictionDetailCol("d")
        return op.linkFrom(model, src).collect()
    calls = {"dev": 0}
    orig = tm.TreeModelMapper._accumulate_device
    orig_device = tm.TreeModelMapper._device

    def spy(self, *a):
        calls["dev"] += 1
        return orig(self, *a)
    tm.TreeModelMapper._accumulate_device = spy
    try:
        dev = run()
        tm.TreeModelMapper._device = lambda self, mt: None          # host walk
        host = run()
    finally:
        tm.TreeModelMapper._accumulate_device = orig
        tm.TreeModelMapper._device = orig_device
    assert calls["dev"] >= 1
    return dev, host


def _compare(dev, host, detail, exact_pred=True):
    assert len(dev) == len(host)
    for a, b in zip(dev, host):
        if exact_pred:
            assert a[5] == b[5]
        else:
            assert a[5] == pytest.approx(b[5], rel=1e-12, abs=1e-12)
        if detail:
            da, db = (None if x is None else __import__("json").loads(x) for x in (a[6], b[6]))
            assert da.keys() == db.keys()
            for k in da:
                assert da[k] == pytest.approx(db[k], rel=1e-12, abs=1e-12)


def test_gbdt_binary_device_predict_matches_host():
    from alink_amd import GbdtTrainBatchOp, GbdtPredictBatchOp
    df = _frame()
    tr = GbdtTrainBatchOp().setFeatureCols(["x0", "x1", "c"]).setCategoricalCols(["c"]).setLabelCol("y") \
        .setNumTrees(20).setMaxDepth(5).setMinSamplesPerLeaf(10)
    dev, host = _predict_both(tr, GbdtPredictBatchOp, df, _with_missing(df))
    _compare(dev, host, True)


def test_gbdt_regression_device_predict_matches_host():
    from alink_amd import GbdtRegTrainBatchOp, GbdtRegPredictBatchOp
    df = _frame(seed=3)
    tr = GbdtRegTrainBatchOp().setFeatureCols(["x0", "x1", "c"]).setCategoricalCols(["c"]).setLabelCol("t") \
        .setNumTrees(15).setMaxDepth(6).setMinSamplesPerLeaf(10)
    dev, host = _predict_both(tr, GbdtRegPredictBatchOp, df, _with_missing(df), detail=False)
    _compare(dev, host, False, exact_pred=False)


@pytest.mark.parametrize("classes", [2, 3, 6])
def test_random_forest_device_predict_matches_host(classes):
    from alink_amd import RandomForestTrainBatchOp, RandomForestPredictBatchOp
    df = _frame(seed=5, classes=classes)
    tr = RandomForestTrainBatchOp().setFeatureCols(["x0", "x1", "c"]).setCategoricalCols(["c"]).setLabelCol("y") \
        .setNumTrees(12).setMaxDepth(7)
    dev, host = _predict_both(tr, RandomForestPredictBatchOp, df, _with_missing(df))
    _compare(dev, host, True)


def test_random_forest_regression_device_predict_matches_host():
    from alink_amd import RandomForestRegTrainBatchOp, RandomForestRegPredictBatchOp
    df = _frame(seed=7)
    tr = RandomForestRegTrainBatchOp().setFeatureCols(["x0", "x1", "c"]).setCategoricalCols(["c"]) \
        .setLabelCol("t").setNumTrees(8).setMaxDepth(8)
    dev, host = _predict_both(tr, RandomForestRegPredictBatchOp, df, _with_missing(df), detail=False)
    _compare(dev, host, False, exact_pred=False)


def test_tree_predict_kernel_rows_not_multiple_of_block():
    from alink_amd import GbdtTrainBatchOp, GbdtPredictBatchOp
    df = _frame(n=131)
    tr = GbdtTrainBatchOp().setFeatureCols(["x0", "x1", "c"]).setCategoricalCols(["c"]).setLabelCol("y") \
        .setNumTrees(5).setMaxDepth(3).setMinSamplesPerLeaf(3)
    dev, host = _predict_both(tr, GbdtPredictBatchOp, df, df.iloc[:67])
    _compare(dev, host, True)


def test_random_forest_memory_bound_identical_trees_gpu():
    """RF with the default unbounded depth on the GPU: maxMemoryInMB 8 (node-batched histogram passes, level
    histograms parked in host memory) grows exactly the trees of an unbounded budget."""
    from tests.test_tree import _rf_trees
    from alink_amd.models.tree.engine import TreeBuilder
    from alink_amd import useLocalEnv
    rng = np.random.default_rng(1)
    n, F = 200_000, 100
    X = rng.normal(size=(n, F)).astype(np.float32)
    df = pd.DataFrame({f"f{i}": X[:, i].astype(np.float64) for i in range(F)})
    df["label"] = ((X[:, 0] + np.sin(3 * X[:, 1]) + X[:, 2] * X[:, 3] + 0.5 * rng.normal(size=n)) > 0).astype(int)
    TreeBuilder.LEVEL_STATS.clear()
    small = _rf_trees(df, 8, n_trees=1, dev="cuda:0")
    widest = max(nodes for _, nodes, _, _ in TreeBuilder.LEVEL_STATS)
    big = _rf_trees(df, 1 << 20, n_trees=1, dev="cuda:0")
    useLocalEnv(1)
    assert widest * F * 128 * 3 * 4 > 8 << 20          # some level really exceeded the budget
    assert small[1:] == big[1:]


def _forest(trees, depth, F, seed, decimals):
    from alink_amd.models.tree.model import LabelCounter, Node
    rng = np.random.default_rng(seed)

    def build(d):
        if d == depth:
            return Node(-1, 0.0, LabelCounter(1.0, 1, [float(rng.normal())]))
        nd = Node(int(rng.integers(F)), 1.0, LabelCounter(2.0, 1, [0.0]), None,
                  float(np.round(rng.normal(), decimals)))
        nd.nextNodes = [build(d + 1), build(d + 1)]
        return nd
    return [build(0) for _ in range(trees)]


@pytest.mark.parametrize("decimals,F,n,row0", [(2, 40, 1000, 0), (2, 40, 4099, 131), (4, 3, 777, 64)])
def test_device_row_codes_equal_searchsorted(decimals, F, n, row0):
    """alink_tree_codes (ops/csrc/tree_predict.hip) == the torch searchsorted + scatter form, bit for bit: values
    exactly on thresholds, NaN (MISS), +-inf, uint8 codes and uint16 codes (> 254 thresholds on a feature),
    row offsets and row counts off the 64-row block."""
    from alink_amd.models.tree.model import _DeviceForest, _FlatForest
    flat = _FlatForest(_forest(60 if decimals == 4 else 30, 6, F, seed=decimals + F, decimals=decimals), 1)
    dfo = _DeviceForest(flat, [], [0] * F, "cuda:0")
    assert dfo.code_bytes == (2 if decimals == 4 else 1)
    g = torch.Generator(device="cpu").manual_seed(n)
    cols = {}
    for f in dfo.cont:
        x = torch.randn(row0 + n, generator=g, dtype=torch.float64)
        T = torch.from_numpy(dfo.thresholds[f])
        k = torch.randint(0, len(T), (row0 + n,), generator=g)
        on = torch.rand(row0 + n, generator=g) < 0.2
        x = torch.where(on, T[k], x)                            # exactly on a threshold
        x[torch.rand(row0 + n, generator=g) < 0.05] = float("nan")
        x[3] = float("inf")
        x[5] = -float("inf")
        cols[f] = x.cuda()
    a = dfo.codes(cols, {}, n, row0=row0, use_kernel=True)
    b = dfo.codes(cols, {}, n, row0=row0, use_kernel=False)
    torch.cuda.synchronize()
    assert a.dtype == b.dtype and a.shape == b.shape
    assert torch.equal(a, b)


@pytest.mark.parametrize("missing", [0.0, 0.05])
@pytest.mark.parametrize("nd_classes", [1, 3, 6])
def test_tree_split_predict_kernel_bit_identical_to_one_wave(missing, nd_classes, monkeypatch):
    """tree_predict2_kernel (4 waves walk different trees of the same staged rows, wave 0 adds the leaves in tree
    order and redoes fan-out trees in place) == the one-wave kernel bit for bit: GBDT-like 1-value leaves and
    multi-class distributions, with and without missing values, more trees than one 64-tree group."""
    from alink_amd.models.tree.model import LabelCounter, Node, _DeviceForest, _FlatForest
    from alink_amd.ops import _lib
    rng = np.random.default_rng(nd_classes)
    F = 50

    def build(d):
        if d == 5:
            return Node(-1, 0.0, LabelCounter(float(rng.integers(1, 50)), 1, list(rng.normal(size=nd_classes))))
        nd = Node(int(rng.integers(F)), 1.0, LabelCounter(1.0, 1, [0.0] * nd_classes), None,
                  float(np.round(rng.normal(), 2)))
        nd.nextNodes = [build(d + 1), build(d + 1)]
        nd.counter.weightSum = nd.nextNodes[0].counter.weightSum + nd.nextNodes[1].counter.weightSum
        return nd
    flat = _FlatForest([build(0) for _ in range(150)], nd_classes)
    dfo = _DeviceForest(flat, [], [0] * F, "cuda:0")
    n = 3001
    cols = {}
    for f in dfo.cont:
        x = torch.randn(n, dtype=torch.float64)
        x[torch.rand(n) < missing] = float("nan")
        cols[f] = x.cuda()
    codes = dfo.codes(cols, {}, n)
    L = _lib.require()
    out = {}
    for v in ("1", "2"):
        monkeypatch.setenv("ALINK_TREE_PREDICT_KERNEL", v)
        acc = torch.full((n, dfo.nd), 7.0, dtype=torch.float64, device="cuda")
        wacc = torch.full((n,), 7.0, dtype=torch.float64, device="cuda")
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        assert L.alink_tree_predict(codes.data_ptr(), n, dfo.stride, dfo.code_bytes, dfo.nodes.data_ptr(),
                                    dfo.dist.data_ptr(), dfo.nd, dfo.wsum.data_ptr(), dfo.cat.data_ptr(),
                                    int(dfo.cat.shape[1]), dfo.roots.data_ptr(), int(dfo.roots.numel()),
                                    acc.data_ptr(), wacc.data_ptr(), err.data_ptr(), _lib.stream_ptr("cuda:0")) == 0
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        out[v] = (acc.cpu(), wacc.cpu())
    assert torch.equal(out["1"][0].view(torch.int64), out["2"][0].view(torch.int64))
    assert torch.equal(out["1"][1].view(torch.int64), out["2"][1].view(torch.int64))
    if missing == 0.0:
        assert bool((out["2"][1] == 150.0).all())
