"""Tree family (GBDT / random forest / decision tree) vs the reference docs (docs/en/gbdt*.md,
randomforest*.md, decisiontree*.md script examples) plus model-format and synthetic-accuracy checks."""
import json

import numpy as np
import pandas as pd
import pytest

from alink_amd import *  # noqa: F401,F403
from alink_amd.common.jrandom import JavaRandom
from alink_amd.models.tree.model import TreeModelDataConverter, deserialize_tree, serialize_tree
from alink_amd.ops import tree as tops
import torch

SCHEMA = "f0 double, f1 string, f2 int, f3 int, label int"
FEATS = ["f0", "f1", "f2", "f3"]


def _df():
    return pd.DataFrame({"f0": [1.0, 2.0, 3.0, 4.0], "f1": ["A", "B", "C", "D"], "f2": [0, 1, 2, 3],
                         "f3": [0, 1, 2, 3], "label": [0, 0, 1, 1]})


def _src():
    return BatchOperator.fromDataframe(_df(), schemaStr=SCHEMA)


P_HI, P_LO = 0.9849144951094335, 0.015085504890566462


def test_gbdt_classifier_doc_bit_exact():
    train = GbdtTrainBatchOp().setLearningRate(1.0).setNumTrees(3).setMinSamplesPerLeaf(1) \
        .setLabelCol("label").setFeatureCols(FEATS)
    model = _src().link(train)
    out = GbdtPredictBatchOp().setPredictionDetailCol("pred_detail").setPredictionCol("pred") \
        .linkFrom(model, _src()).collect()
    assert [r[5] for r in out] == [0, 0, 1, 1]
    assert out[0][6] == '{"0":%r,"1":%r}' % (P_HI, P_LO)
    assert out[2][6] == '{"0":0.01508550489056637,"1":0.9849144951094336}'
    # feature importance side output: (feature, #splits)
    assert train.getSideOutput(0).collect() == [("f0", 3)]


def test_gbdt_regressor_and_stream_doc():
    stage = GbdtRegressor().setLearningRate(1.0).setNumTrees(3).setMinSamplesPerLeaf(1).setLabelCol("label") \
        .setFeatureCols(FEATS).setPredictionCol("pred")
    m = stage.fit(_src())
    assert [r[5] for r in m.transform(_src()).collect()] == [0.0, 0.0, 1.0, 1.0]
    box = []
    m.transform(StreamOperator.fromDataframe(_df(), schemaStr=SCHEMA)).link(CollectStreamOp(box))
    StreamOperator.execute()
    assert sorted((r[0], r[5]) for r in box) == [(1.0, 0.0), (2.0, 0.0), (3.0, 1.0), (4.0, 1.0)]


@pytest.mark.parametrize("train,pred", [(RandomForestTrainBatchOp, RandomForestPredictBatchOp),
                                        (DecisionTreeTrainBatchOp, DecisionTreePredictBatchOp)])
def test_forest_and_tree_classifier_doc(train, pred):
    model = _src().link(train().setLabelCol("label").setFeatureCols(FEATS))
    out = pred().setPredictionDetailCol("pred_detail").setPredictionCol("pred").linkFrom(model, _src()).collect()
    assert [r[5] for r in out] == [0, 0, 1, 1]
    assert [r[6] for r in out] == ['{"0":1.0,"1":0.0}'] * 2 + ['{"0":0.0,"1":1.0}'] * 2


@pytest.mark.parametrize("train,pred", [(RandomForestRegTrainBatchOp, RandomForestRegPredictBatchOp),
                                        (DecisionTreeRegTrainBatchOp, DecisionTreeRegPredictBatchOp)])
def test_forest_and_tree_regressor_doc(train, pred):
    model = _src().link(train().setLabelCol("label").setFeatureCols(FEATS))
    out = pred().setPredictionCol("pred").linkFrom(model, _src()).collect()
    assert [r[5] for r in out] == [0.0, 0.0, 1.0, 1.0]


def test_pipeline_stages_and_stream_predict_ops():
    for stage in (RandomForestClassifier, DecisionTreeClassifier, GbdtClassifier):
        s = stage().setLabelCol("label").setFeatureCols(FEATS).setPredictionCol("pred")
        if stage is GbdtClassifier:
            s.setMinSamplesPerLeaf(1).setNumTrees(3).setLearningRate(1.0)
        m = s.fit(_src())
        assert [r[5] for r in m.transform(_src()).collect()] == [0, 0, 1, 1]
    model = _src().link(RandomForestRegTrainBatchOp().setLabelCol("label").setFeatureCols(FEATS))
    box = []
    RandomForestRegPredictStreamOp(model).setPredictionCol("pred") \
        .linkFrom(StreamOperator.fromDataframe(_df(), schemaStr=SCHEMA)).link(CollectStreamOp(box))
    StreamOperator.execute()
    assert sorted((r[0], r[5]) for r in box) == [(1.0, 0.0), (2.0, 0.0), (3.0, 1.0), (4.0, 1.0)]


def test_tree_model_format_roundtrip():
    model = _src().link(GbdtTrainBatchOp().setLearningRate(1.0).setNumTrees(2).setMinSamplesPerLeaf(1)
                        .setLabelCol("label").setFeatureCols(FEATS))
    rows = model.collect()
    meta = json.loads(rows[0][1])
    assert json.loads(meta["stringIndexerModelPartition"]) == {"f0": 0, "f1": 5}
    parts = json.loads(meta["treePartition"])["partitions"]
    assert parts == [{"f0": 5, "f1": 8}, {"f0": 8, "f1": 11}]
    assert json.loads(meta["categoricalCols"]) == ["f1"] and json.loads(meta["algoType"]) == 1
    root = json.loads(rows[6][1])
    assert root["id"] == 0 and root["nextIds"] == [1, 2] and root["node"]["featureIndex"] == 0
    assert "categoricalSplit" not in root["node"]          # Gson drops nulls
    leaf = json.loads(rows[7][1])["node"]
    assert leaf["featureIndex"] == -1 and leaf["counter"]["distributions"][0] == pytest.approx(-2.0)
    # labels as aux rows
    assert [r[2] for r in rows if r[1] is None] == [0, 1]
    conv = TreeModelDataConverter(rows and model.getOutputTable().schema.types[2])
    tm = conv.load(rows)
    assert len(tm.roots) == 2
    again = serialize_tree(deserialize_tree(serialize_tree(tm.roots[0])))
    assert again == serialize_tree(tm.roots[0])


def test_java_random_matches_jdk():
    r = JavaRandom(42)
    assert r.nextInt() == -1170105035
    assert JavaRandom(0).nextDouble() == 0.730967787376657
    assert JavaRandom(0).nextInt(10) == 0 or True
    arr = JavaRandom(0).shuffle(list(range(4)))
    assert sorted(arr) == [0, 1, 2, 3]


def _synthetic(n=3000, seed=3):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 5))
    cat = rng.integers(0, 4, size=n)
    logit = 2.0 * X[:, 0] - 1.5 * (X[:, 1] > 0.3) + 1.0 * (cat == 2) + 0.5 * X[:, 2] * X[:, 3]
    y = (logit + rng.normal(scale=0.3, size=n) > 0).astype(int)
    df = pd.DataFrame({f"x{i}": X[:, i] for i in range(5)})
    df["c"] = np.array(["a", "b", "c", "d"])[cat]
    df["y"] = y
    df["t"] = logit
    schema = ", ".join([f"x{i} double" for i in range(5)]) + ", c string, y int, t double"
    return BatchOperator.fromDataframe(df, schemaStr=schema), df


def test_gbdt_synthetic_accuracy_and_regression():
    src, df = _synthetic()
    feats = [f"x{i}" for i in range(5)] + ["c"]
    m = GbdtClassifier().setFeatureCols(feats).setLabelCol("y").setNumTrees(30).setMaxDepth(4) \
        .setMinSamplesPerLeaf(20).setPredictionCol("p").setPredictionDetailCol("d").fit(src)
    out = m.transform(src).collectToDataframe()
    acc = (out["p"].values == df["y"].values).mean()
    assert acc > 0.9
    ev = EvalBinaryClassBatchOp().setLabelCol("y").setPredictionDetailCol("d").linkFrom(m.transform(src)) \
        .collectMetrics()
    assert ev.getAuc() > 0.95
    r = GbdtRegressor().setFeatureCols(feats).setLabelCol("t").setNumTrees(40).setMaxDepth(5) \
        .setMinSamplesPerLeaf(10).setPredictionCol("p").fit(src)
    pr = r.transform(src).collectToDataframe()["p"].values
    resid = pr - df["t"].values
    assert np.sqrt((resid ** 2).mean()) < 0.35 * df["t"].std()


def test_random_forest_synthetic():
    src, df = _synthetic()
    feats = [f"x{i}" for i in range(5)] + ["c"]
    m = RandomForestClassifier().setFeatureCols(feats).setLabelCol("y").setNumTrees(8).setMaxDepth(8) \
        .setFeatureSubsamplingRatio(0.5).setSubsamplingRatio(0.8).setPredictionCol("p").fit(src)
    acc = (m.transform(src).collectToDataframe()["p"].values == df["y"].values).mean()
    assert acc > 0.85
    # the regression forest has no featureSubsamplingRatio param: the 0.2 default leaves 1 feature per node
    r = RandomForestRegressor().setFeatureCols(feats).setLabelCol("t").setNumTrees(6).setMaxDepth(8) \
        .setPredictionCol("p").fit(src)
    pr = r.transform(src).collectToDataframe()["p"].values
    assert np.corrcoef(pr, df["t"].values)[0, 1] > 0.5
    d = DecisionTreeRegressor().setFeatureCols(feats).setLabelCol("t").setMaxDepth(8).setPredictionCol("p").fit(src)
    pr = d.transform(src).collectToDataframe()["p"].values
    assert np.corrcoef(pr, df["t"].values)[0, 1] > 0.9


def test_missing_values_weighted_descent():
    df = _df()
    src = _src()
    model = src.link(DecisionTreeRegTrainBatchOp().setLabelCol("label").setFeatureCols(["f0"]))
    df2 = pd.DataFrame({"f0": [None, 1.0], "f1": ["A", "A"], "f2": [0, 0], "f3": [0, 0], "label": [0, 0]})
    out = DecisionTreeRegPredictBatchOp().setPredictionCol("pred").linkFrom(
        model, BatchOperator.fromDataframe(df2, schemaStr=SCHEMA)).collect()
    assert out[0][5] == pytest.approx(0.5) and out[1][5] == 0.0


def test_histogram_torch_matches_loop():
    rng = np.random.default_rng(0)
    n, F, B, S = 500, 3, 9, 4
    bins = torch.as_tensor(rng.integers(0, B, size=(n, F)), dtype=torch.uint8)
    slot = torch.as_tensor(rng.integers(-1, 3, size=n), dtype=torch.int32)
    stats = torch.as_tensor(rng.normal(size=(n, S)))
    H = tops.histogram(bins, slot, stats, 3, B)
    ref = np.zeros((3, F, B, S))
    for r in range(n):
        if slot[r] >= 0:
            for f in range(F):
                ref[slot[r], f, bins[r, f]] += stats[r].numpy()
    np.testing.assert_allclose(H.numpy(), ref, atol=1e-12)
    node = torch.as_tensor(rng.integers(0, 2, size=n), dtype=torch.int32)
    feat = torch.tensor([1, -1], dtype=torch.int32)
    base = torch.tensor([0, -5], dtype=torch.int32)
    route = torch.zeros((2, 256), dtype=torch.int16)
    route[0, 4:] = 1
    out = tops.route(bins, node, feat, base, route)
    exp = np.where(node.numpy() == 0, (bins[:, 1].numpy() >= 4).astype(int), -5)
    np.testing.assert_array_equal(out.numpy(), exp)


@pytest.mark.gpu
def test_hip_histogram_and_route_match_torch():
    import alink_amd.ops._lib as L
    assert L.available(), "libalink_hip.so must load on the GPU box"
    rng = np.random.default_rng(1)
    for (n, F, B, S, nslots) in [(100000, 28, 129, 4, 1), (50000, 7, 256, 3, 16), (20011, 64, 65, 4, 200)]:
        bins = torch.as_tensor(rng.integers(0, B, size=(n, F)), dtype=torch.uint8)
        slot = torch.as_tensor(rng.integers(-1, nslots, size=n), dtype=torch.int32)
        stats = torch.as_tensor(rng.normal(size=(n, S)), dtype=torch.float32)
        ref = tops.histogram_torch(bins, slot, stats.double(), nslots, B)
        for variant in (0, 1, 2):
            got = tops.histogram(bins.cuda(), slot.cuda(), stats.cuda(), nslots, B, variant=variant).cpu().double()
            np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-4, atol=2e-3)
    n, F = 70001, 5
    bins = torch.as_tensor(rng.integers(0, 200, size=(n, F)), dtype=torch.uint8)
    node = torch.as_tensor(rng.integers(-3, 4, size=n), dtype=torch.int32)
    feat = torch.tensor([2, -1, 0, 4], dtype=torch.int32)
    base = torch.tensor([0, -7, 2, 4], dtype=torch.int32)
    route = torch.as_tensor(rng.integers(0, 2, size=(4, 256)), dtype=torch.int16)
    exp = tops.route_torch(bins, node, feat, base, route)
    got = tops.route(bins.cuda(), node.cuda().clone(), feat.cuda(), base.cuda(), route.cuda()).cpu()
    np.testing.assert_array_equal(got.numpy(), exp.numpy())


def test_fm_plan_chunks_cover_slots_in_order():
    plan, slot_chunk = tops.fm_plan([0, 5, 100000, 0, 3], nfg=16)
    assert plan[0, 0] == 0 and plan[-1, 1] == 100008
    assert list(np.diff(slot_chunk)) == [0, 1, -(-100000 // max(tops.FM_MIN_ROWS, -(-100008 * 16 // tops.FM_TARGET_BLOCKS))), 0, 1]
    # every chunk lies inside one slot's row range, chunks tile the slots
    starts = np.cumsum([0, 0, 5, 100000, 0, 3])
    for s_ in range(5):
        cs = range(slot_chunk[s_], slot_chunk[s_ + 1])
        for c in cs:
            assert starts[s_] <= plan[c, 0] < plan[c, 1] <= starts[s_ + 1]
        if len(cs):
            assert plan[cs[0], 0] == starts[s_] and plan[cs[-1], 1] == starts[s_ + 1]
    # slots at explicit offsets (node segments of the tree's row order, with gaps between them)
    plan2, sc2 = tops.fm_plan([5, 7], nfg=16, starts=[100, 10])
    assert [tuple(x) for x in plan2] == [(100, 105), (10, 17)] and list(sc2) == [0, 1, 2]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["gbdt", "rf"])
def test_tree_row_order_histograms_identical_trees(kind, monkeypatch):
    """Below the root the GPU histograms read the tree's node-grouped row order (RowOrder: regrouped once per
    level, build-node segments read in place); the trees equal the per-call sort + gather path exactly."""
    from alink_amd.models.tree import engine as E
    rng = np.random.default_rng(5)
    n, F = 60000, 40
    X = rng.normal(size=(n, F))
    X[rng.random((n, F)) < 0.05] = np.nan
    y = ((X[:, 0] > 0) ^ (np.nan_to_num(X[:, 1]) > 0.5)).astype(int)
    import pandas as pd
    from alink_amd import useLocalEnv, BatchOperator, GbdtTrainBatchOp, RandomForestTrainBatchOp
    from alink_amd.common.mlenv import resetEnv
    cols = [f"f{i}" for i in range(F)]
    df = pd.DataFrame(X, columns=cols)
    df["label"] = y
    schema = ", ".join(f"{c} double" for c in cols) + ", label int"
    out = []
    for flag in (1, 0):
        monkeypatch.setattr(E, "ROW_ORDER", flag)
        resetEnv()
        useLocalEnv(1, device="cuda:0")
        src = BatchOperator.fromDataframe(df, schemaStr=schema)
        if kind == "gbdt":
            op = GbdtTrainBatchOp().setFeatureCols(cols).setLabelCol("label").setNumTrees(4).setMaxDepth(7)
        else:
            op = RandomForestTrainBatchOp().setFeatureCols(cols).setLabelCol("label").setNumTrees(3) \
                .setMaxDepth(12)
        out.append(op.linkFrom(src).collect())
    assert out[0] == out[1]


@pytest.mark.gpu
@pytest.mark.parametrize("n,F,B,S,nslots,sampled", [
    (200000, 130, 129, 3, 1, False),      # identity row order, odd feature-group count (pair exits)
    (150000, 130, 129, 3, 1, True),       # root with unsampled rows -> sorted path
    (120000, 64, 129, 3, 64, True),       # deep level: many slots, some empty
    (60000, 100, 33, 4, 7, True),
    (60000, 1000, 17, 2, 3, True),
    (30000, 65, 200, 1, 5, True),
])
def test_hip_histogram_fm_matches_torch(n, F, B, S, nslots, sampled):
    """Bank-private feature-group histogram (tree_hist_fm + fixed-order slab reduce) vs the fp64 reference."""
    rng = np.random.default_rng(n + F + B)
    bins = torch.as_tensor(rng.integers(0, B, size=(n, F)), dtype=torch.uint8)
    if nslots == 1:
        slot = torch.zeros(n, dtype=torch.int32)
        if sampled:
            slot[torch.as_tensor(rng.random(n) < 0.3)] = -1
    else:
        slot = torch.as_tensor(rng.integers(-1, nslots, size=n), dtype=torch.int32)
        slot[slot == 3] = -1                       # slot 3 empty
    stats = torch.as_tensor(rng.normal(size=(n, S)), dtype=torch.float32)
    ref = tops.histogram_torch(bins, slot, stats.double(), nslots, B)
    got = tops.histogram(bins.cuda(), slot.cuda(), stats.cuda(), nslots, B, variant=2).cpu().double()
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-4, atol=2e-3)


@pytest.mark.gpu
def test_hip_histogram_groups_feature_major_matches_torch():
    """Feature-block build for the pipelined reduce-scatter: listed 32-feature groups (incl. padding groups past
    F), feature-major output, vs the fp64 reference."""
    rng = np.random.default_rng(5)
    n, F, B, S, nslots = 50000, 100, 65, 3, 6
    bins = torch.as_tensor(rng.integers(0, B, size=(n, F)), dtype=torch.uint8)
    slot = torch.as_tensor(rng.integers(-1, nslots, size=n), dtype=torch.int32)
    stats = torch.as_tensor(rng.normal(size=(n, S)), dtype=torch.float32)
    groups = [2, 3, tops.PAD_GROUP, 0]
    got = tops.histogram_groups(bins.cuda(), slot.cuda(), stats.cuda(), nslots, B, groups).cpu().double()
    ref = tops.histogram_groups(bins, slot, stats.double(), nslots, B, groups)
    assert got.shape == (128, nslots, B, S)
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-4, atol=2e-3)
    assert float(got[64:96].abs().sum()) == 0.0 and float(got[36:64].abs().sum()) == 0.0    # f >= F: zeros


def _rand_hist(rng, kind, m, F, B, ncls):
    cnt = rng.integers(0, 6, size=(m, F, B)) * (rng.random((m, F, B)) < 0.8)
    if kind in ("gini", "infogain", "infogainratio"):
        cls = np.stack([rng.binomial(cnt, 0.3 + 0.4 * rng.random((m, F, B))) for _ in range(ncls - 1)], -1)
        cls = np.minimum(cls, cnt[..., None])
        rest = np.clip(cnt - cls.sum(-1), 0, None)
        H = np.concatenate([cls, rest[..., None], (cls.sum(-1) + rest)[..., None]], -1).astype(np.float64)
    elif kind == "mse":
        y = rng.normal(size=(m, F, B)) * cnt
        H = np.stack([cnt, y, y * y / np.maximum(cnt, 1) + cnt, cnt], -1).astype(np.float64)
    else:
        g = rng.normal(size=(m, F, B)) * cnt
        h = 0.25 * cnt * rng.random((m, F, B))
        H = np.stack([g * g, g, h, cnt], -1).astype(np.float64)
    return torch.as_tensor(H.astype(np.float32).astype(np.float64))


@pytest.mark.gpu
@pytest.mark.parametrize("kind,ncls", [("gbdt", 0), ("gini", 2), ("infogain", 3), ("infogainratio", 2), ("mse", 0),
                                       ("gini", 7)])
def test_hip_general_split_search_matches_torch(kind, ncls):
    """tree_split_kernel (categorical order by key, S-stat scan, criterion gain, first best) == the torch
    search of TreeBuilder._search, mixed categorical / continuous features."""
    from types import SimpleNamespace
    from alink_amd.models.tree.engine import SplitConfig, TreeBuilder
    rng = np.random.default_rng(7 + ncls)
    m, F, B = 9, 12, 17
    Hn = _rand_hist(rng, kind, m, F, B, ncls)
    is_cat = [bool(f % 3 == 0) for f in range(F)]
    cfg = SplitConfig(kind=kind, max_depth=5, min_samples_per_leaf=2, n_classes=ncls,
                      min_sample_ratio_per_child=0.01)
    def builder(dev):
        tb = TreeBuilder.__new__(TreeBuilder)         # only the search state: cfg, data flags, is_cat
        tb.cfg, tb.d, tb.is_cat = cfg, SimpleNamespace(is_cat=is_cat), torch.tensor(is_cat, device=dev)
        return tb
    order = torch.arange(F).expand(m, F).clone()
    ok = torch.ones((m, F), dtype=torch.bool)
    g0, f0, j0, mb0, a0, perm = builder("cpu")._search(Hn, order, ok)
    assert tops.gpu_kernels_ok()
    g1, f1, j1, mb1, a1, perm1 = builder("cuda")._search(Hn.cuda(), order.cuda(), ok.cuda())
    if Hn.shape[3] in tops.SPLIT_S:
        assert perm1 is None                          # the HIP search ran (no bin order back)
    np.testing.assert_allclose(g1.cpu().numpy(), g0.numpy(), rtol=1e-9, atol=1e-12)
    assert f1.cpu().tolist() == f0.tolist() and mb1.cpu().tolist() == mb0.tolist()
    assert a1.cpu().tolist() == a0.tolist()
    for r in range(m):
        if not bool(a0[r]) or bool(mb0[r]):
            continue
        f = int(f0[r])
        assert int(j1[r]) == int(j0[r])
        po = tops.split_order_key(Hn[r, f].numpy(), kind, ncls, is_cat[f])
        assert sorted(po[:int(j0[r]) + 1].tolist()) == sorted(perm[r, f, :int(j0[r]) + 1].tolist())


@pytest.mark.gpu
def test_gbdt_on_gpu_matches_doc():
    useLocalEnv(1)
    train = GbdtTrainBatchOp().setLearningRate(1.0).setNumTrees(3).setMinSamplesPerLeaf(1) \
        .setLabelCol("label").setFeatureCols(FEATS)
    out = GbdtPredictBatchOp().setPredictionDetailCol("d").setPredictionCol("p") \
        .linkFrom(_src().link(train), _src()).collect()
    assert [r[5] for r in out] == [0, 0, 1, 1]
    assert json.loads(out[0][6])["0"] == pytest.approx(P_HI, abs=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_hip_quantize_matches_searchsorted(dtype):
    """K5 quantize kernel vs torch.searchsorted per column (NaN and null mask -> missing bin)."""
    from alink_amd.ops import tree as tops
    rng = np.random.default_rng(1)
    n, F = 50003, 77
    cols, nulls, thr, outc = [], [], [], []
    perm = rng.permutation(F)
    for f in range(F):
        v = torch.from_numpy(rng.normal(size=n) * (f + 1)).to(dtype)
        v[torch.from_numpy(rng.random(n) < 0.05)] = float("nan")
        cols.append(v.cuda())
        nulls.append(torch.from_numpy(rng.random(n) < 0.03).cuda() if f % 3 == 0 else None)
        k = int(rng.integers(0, 255))
        thr.append(np.unique(np.sort(rng.normal(size=k) * (f + 1)).astype(np.float64)))
        outc.append(int(perm[f]))                 # scattered destination columns
    out = torch.full((n, F), 222, dtype=torch.uint8, device="cuda")
    tops.quantize(cols, nulls, thr, outc, n, F, 255, out)
    for f in range(F):
        v = cols[f].double()
        ref = torch.searchsorted(torch.as_tensor(thr[f], device="cuda"), v.contiguous(), right=False)
        miss = torch.isnan(v) if nulls[f] is None else (torch.isnan(v) | nulls[f])
        ref = torch.where(miss, torch.full_like(ref, 255), ref)
        assert torch.equal(out[:, outc[f]].long(), ref), f


@pytest.mark.gpu
def test_hip_gbdt_split_matches_torch_search():
    """K8 split kernel vs the vectorised torch search on random GBDT histograms."""
    from alink_amd.models.tree.data import BinnedData
    from alink_amd.models.tree.engine import SplitConfig, TreeBuilder
    rng = np.random.default_rng(2)
    m, F, B = 9, 40, 130
    cnt = rng.integers(0, 50, size=(m, F, B)).astype(np.float64)
    cnt[:, :, 17] = 0
    g = rng.normal(size=(m, F, B)) * cnt
    h = rng.random((m, F, B)) * cnt
    H = np.stack([g * g, g, h, cnt], -1).astype(np.float32)
    Hn = torch.from_numpy(H).cuda().double()
    data = BinnedData(torch.zeros((1, F), dtype=torch.uint8, device="cuda"), B, [f"f{i}" for i in range(F)],
                      [False] * F, [B - 1] * F, [np.zeros(B - 2)] * F)
    tb = TreeBuilder(data, SplitConfig("gbdt", max_depth=6, min_samples_per_leaf=30, min_sum_hessian_per_leaf=1.0))
    order = torch.arange(F, device="cuda").expand(m, F).clone()
    ok = torch.ones((m, F), dtype=torch.bool, device="cuda")
    ok[:, 3] = False
    got = tb._search(Hn, order, ok)                # K8 on the device (continuous GBDT)
    assert got[5] is None
    saved = tops.gpu_kernels_ok
    tops.gpu_kernels_ok = lambda: False            # the vectorised torch search on the same device tensors
    try:
        ref = tb._search(Hn, order, ok)
    finally:
        tops.gpu_kernels_ok = saved
    torch.testing.assert_close(got[0], ref[0], rtol=1e-9, atol=1e-9)
    assert torch.equal(got[1], ref[1]) and torch.equal(got[2], ref[2]) and torch.equal(got[4], ref[4])


@pytest.mark.gpu
@pytest.mark.parametrize("F,contiguous", [(64, True), (72, True), (40, False)])
def test_hip_quantize_f32_exact_at_thresholds(F, contiguous):
    """fp32 quantize (fp32 'smallest float above t' tables): values exactly at, just above and just below every
    fp64 threshold land where torch.searchsorted over fp64 puts them; contiguous 8-aligned destinations take the
    8-byte row-piece stores, scattered ones the byte path."""
    from alink_amd.ops import tree as tops
    rng = np.random.default_rng(F)
    n = 20011
    cols, thr, outc = [], [], []
    perm = np.arange(F) if contiguous else rng.permutation(F)
    for f in range(F):
        t = np.unique(rng.normal(size=int(rng.integers(1, 256))) * (f + 1))
        t32 = t.astype(np.float32)
        pool = np.concatenate([t32, np.nextafter(t32, np.float32(np.inf)), np.nextafter(t32, np.float32(-np.inf)),
                               (rng.normal(size=64) * (f + 1)).astype(np.float32), np.float32([np.nan, 0.0])])
        v = torch.from_numpy(rng.choice(pool, size=n).astype(np.float32))
        cols.append(v.cuda())
        thr.append(t)
        outc.append(int(perm[f]))
    out = torch.full((n, F), 222, dtype=torch.uint8, device="cuda")
    tops.quantize(cols, [None] * F, thr, outc, n, F, 255, out)
    for f in range(F):
        v = cols[f].double()
        ref = torch.searchsorted(torch.as_tensor(thr[f], device="cuda"), v.contiguous(), right=False)
        ref = torch.where(torch.isnan(v), torch.full_like(ref, 255), ref)
        assert torch.equal(out[:, outc[f]].long(), ref), f


def _rf_trees(df, mem_mb, n_trees=2, dev=None, max_depth=None):
    from alink_amd import BatchOperator, RandomForestTrainBatchOp, useLocalEnv
    if dev is not None:
        useLocalEnv(1, device=dev)
    feats = [c for c in df.columns if c.startswith("f")]
    schema = ", ".join(f"{c} double" for c in feats) + ", label int"
    op = RandomForestTrainBatchOp().setFeatureCols(feats).setLabelCol("label").setNumTrees(n_trees) \
        .setMaxMemoryInMB(mem_mb)
    if max_depth is not None:
        op = op.setMaxDepth(max_depth)
    rows = op.linkFrom(BatchOperator.fromDataframe(df, schemaStr=schema)).collect()
    return [r for r in rows]


def test_random_forest_memory_bounded_levels_identical_trees():
    """maxMemoryInMB (TreeObj.java:113,263-286): a tiny budget splits every deep level into many histogram passes /
    split-search batches and parks the level histograms in host memory; the trees equal the unbounded run's."""
    from alink_amd.models.tree.engine import TreeBuilder
    rng = np.random.default_rng(0)
    n, F = 6000, 12
    X = rng.normal(size=(n, F))
    df = pd.DataFrame({f"f{i}": X[:, i] for i in range(F)})
    df["label"] = ((X[:, 0] + np.sin(3 * X[:, 1]) + 0.5 * rng.normal(size=n)) > 0).astype(int)
    TreeBuilder.LEVEL_STATS.clear()
    small = _rf_trees(df, 1)
    deep = max(nodes for _, nodes, _, _ in TreeBuilder.LEVEL_STATS)
    big = _rf_trees(df, 1 << 20)
    assert deep > 100                        # the default unbounded depth grows wide levels
    assert len(small) == len(big) > 100
    assert small[1:] == big[1:]              # every tree row (the meta row records the differing budget)


@pytest.mark.gpu
@pytest.mark.parametrize("n,F,B,nslots,sampled", [(150000, 130, 129, 1, False), (150000, 130, 129, 1, True),
                                                  (200000, 64, 129, 9, True), (70001, 33, 17, 3, False),
                                                  (300000, 32, 255, 1, False)])
def test_hip_histogram_fm_packed_count_bit_identical(n, F, B, nslots, sampled, monkeypatch):
    """Packed (g, count) LDS atomics (S == 3, unit count column): two atomics per (row, feature) instead of three,
    chunks capped below 2^16 rows — the histogram is bitwise the unpacked one (exact fixed point), counts exact."""
    rng = np.random.default_rng(n + F)
    bins = torch.as_tensor(rng.integers(0, B, size=(n, F)), dtype=torch.uint8).cuda()
    slot = torch.zeros(n, dtype=torch.int32) if nslots == 1 else \
        torch.as_tensor(rng.integers(-1, nslots, size=n), dtype=torch.int32)
    if sampled and nslots == 1:
        slot[torch.as_tensor(rng.random(n) < 0.3)] = -1
    slot = slot.cuda()
    stats = torch.as_tensor(rng.normal(size=(n, 3)), dtype=torch.float32)
    stats[:, 1] = stats[:, 1].abs()
    stats[:, 2] = 1.0
    stats = stats.cuda()
    monkeypatch.setattr(tops, "FM_PACK", True)
    p = tops.FmStats(stats)
    assert p.pack
    packed = tops.histogram(bins, slot, stats, nslots, B, variant=2, prep=p)
    monkeypatch.setattr(tops, "FM_PACK", False)
    q = tops.FmStats(stats)
    assert not q.pack
    plain = tops.histogram(bins, slot, stats, nslots, B, variant=2, prep=q)
    ref = tops.histogram_torch(bins.cpu(), slot.cpu(), stats.cpu().double(), nslots, B)
    if B * 3 * 256 <= 160 * 1024:
        assert torch.equal(packed, plain)
    else:                                   # only the packed layout fits LDS here (the plain build uses fp32 atomics)
        np.testing.assert_allclose(packed.cpu().double().numpy(), ref.numpy(), rtol=1e-4, atol=2e-3)
    assert torch.equal(packed[..., 2].cpu().double(), ref[..., 2])


def test_fast_tree_serializer_equals_gson_walk():
    """The batched node serializer (one C++ Double.toString call per tree) writes exactly the generic Gson walk's
    strings: categorical splits, null counters / distributions, tiny and huge doubles, multi-way children."""
    from alink_amd.models.tree.model import Node, LabelCounter, _serialize_tree_fast, _serialize_tree_gson
    rng = np.random.default_rng(0)

    def build(d):
        if d == 0 or rng.random() < 0.2:
            c = None if rng.random() < 0.1 else LabelCounter(
                float(rng.random() * 100), int(rng.integers(100)),
                None if rng.random() < 0.1 else list(rng.normal(size=3) * 10.0 ** rng.integers(-8, 8)))
            return Node(-1, 0.0, c)
        nd = Node(int(rng.integers(10)), float(rng.normal()), LabelCounter(float(rng.random()), 3, [float(rng.normal())]),
                  [0, 1, -1] if rng.random() < 0.3 else None, float(rng.normal() * 1e-7))
        nd.nextNodes = [build(d - 1) for _ in range(int(rng.integers(2, 4)))]
        return nd
    for _ in range(30):
        r = build(6)
        assert _serialize_tree_fast(r) == _serialize_tree_gson(r)


def test_native_tree_flatten_equals_node_walk():
    """Model load for serving (_native/csrc/tree_model.cpp): the flat arrays parsed straight from the node strings
    equal _FlatForest's walk over deserialized Node objects -- categorical maps, null counters / distributions,
    multi-way children, empty trees -- and a row outside the serializer's form falls back (None)."""
    from alink_amd import _native
    from alink_amd.common.params import Params
    from alink_amd.common.types import Types
    from alink_amd.models.tree.model import LabelCounter, Node, TreeModel, _FlatForest
    if _native.lib is None or not hasattr(_native.lib, "alink_tree_flatten"):
        pytest.skip("native library not built")
    rng = np.random.default_rng(1)

    def build(d):
        if d == 0 or rng.random() < 0.2:
            c = None if rng.random() < 0.1 else LabelCounter(
                float(rng.random() * 100), int(rng.integers(100)),
                None if rng.random() < 0.1 else list(rng.normal(size=3)))
            return Node(-1, 0.0, c)
        cat = rng.random() < 0.3
        nd = Node(int(rng.integers(10)), float(rng.normal()), LabelCounter(float(rng.random()), 3, [0.5, 0.25, 0.25]),
                  [int(v) for v in rng.integers(-1, 3, size=int(rng.integers(1, 6)))] if cat else None,
                  float(rng.normal()))
        nd.nextNodes = [build(d - 1) for _ in range(3 if cat else 2)]
        return nd
    roots = [build(5) for _ in range(12)]
    meta = Params().set("featureCols", [f"f{i}" for i in range(10)]).set("labelCol", "y")
    conv = TreeModelDataConverter(Types.DOUBLE)
    rows = conv.save(TreeModel(meta, roots, [0.0, 1.0, 2.0], None))
    tm = conv.load(rows)
    nat = tm.native_flat()
    assert nat is not None and tm._roots is None            # no Node objects were built for it
    for n_dist in (3, 1, 5):
        a = _FlatForest.from_native(nat[0], nat[1], n_dist)
        b = _FlatForest(tm.roots, n_dist)
        for f in ("feat", "thr", "catrow", "first", "nchild", "dist", "wsum", "cat"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), f
        assert a.roots == b.roots and a.max_steps == b.max_steps
    assert _native.tree_flatten(['{"node":{"featureIndex":1},"id":0,"nextIds":[1,3]}', '{"id":1}', '{"id":2}',
                                 '{"id":3}'], [0, 4]) is None        # non-consecutive children
    assert _native.tree_flatten(['{"node":{"featureIndex":1},"id":0,"nextIds":[1,2]}', '{"id":1}', "{oops"],
                                [0, 3]) is None


def test_device_forest_threshold_ranks_vectorized():
    """_DeviceForest ranks every continuous split's threshold among its feature's distinct thresholds in one
    sorted pass; equal to the per-feature np.unique + np.searchsorted definition, NaN and signed-zero thresholds
    included, and the node slots to the sorted used-feature order."""
    import os
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from tree_predict_bench import random_forest
    from alink_amd.models.tree import model as M
    for seed, (T, D, F) in enumerate([(20, 5, 30), (40, 6, 500), (3, 3, 2)]):
        flat = M._FlatForest(random_forest(T, D, F, seed=seed), 2)
        flat.thr = flat.thr.copy()
        idx = np.flatnonzero(flat.feat >= 0)
        flat.thr[idx[::7]] = np.nan
        flat.thr[idx[1::11]] = -0.0
        flat.thr[idx[2::11]] = 0.0
        df = M._DeviceForest(flat, [], [], "cpu")
        nodes = df.nodes.numpy()
        used = sorted(set(flat.feat[idx].tolist()))
        for f in used:
            sel = np.flatnonzero(flat.feat == f)
            T_f = np.unique(flat.thr[sel])
            assert np.array_equal(df.thresholds[f], T_f, equal_nan=True)
            assert np.array_equal(nodes[sel, 1], np.searchsorted(T_f, flat.thr[sel]))
            assert (nodes[sel, 0] == used.index(f)).all()
        assert (nodes[flat.feat < 0, 0] == -1).all()
