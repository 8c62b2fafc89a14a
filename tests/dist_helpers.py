"""Multi-process (gloo, CPU) scenarios for tests/test_distributed.py — each rank is one process, exactly
like one-process-per-GPU on MI355X but with the gloo backend (the analogue of Flink's LocalEnvironment)."""
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _data_frame():
    import numpy as np
    import pandas as pd
    rng = np.random.default_rng(7)
    X = rng.normal(size=(600, 4))
    y = (X @ np.array([1.0, -2.0, 0.5, 0.0]) + 0.2 > 0).astype(int)
    df = pd.DataFrame({f"x{i}": X[:, i] for i in range(4)})
    df["y"] = y
    return df


def scenario_pi(out):
    import torch
    from alink_amd.parallel.comqueue import (AllReduce, ComputeFunction, CompleteResultFunction,
                                             IterativeComQueue)
    from alink_amd import useLocalEnv

    env = useLocalEnv(4)   # 2 processes x 2 local tasks

    class Sample(ComputeFunction):
        def calc(self, ctx):
            g = torch.Generator().manual_seed(1000 + ctx.getTaskId() * 31 + ctx.getStepNo())
            pts = torch.rand((20000, 2), generator=g, dtype=torch.float64)
            inside = float(((pts ** 2).sum(1) <= 1.0).sum())
            acc = ctx.getObj("acc")
            if acc is None:
                acc = torch.zeros(2, dtype=torch.float64)
            acc = acc + torch.tensor([inside, 20000.0], dtype=torch.float64)
            ctx.putObj("acc", acc)
            ctx.putObj("buf", torch.tensor([inside, 20000.0], dtype=torch.float64))

    class Out(CompleteResultFunction):
        def calc(self, ctx):
            b = ctx.getObj("buf")
            return [(ctx.getTaskId(), ctx.getNumTask(), float(4.0 * b[0] / b[1]))]

    rows = IterativeComQueue().setMLEnvironment(env).add(Sample()).add(AllReduce("buf")).closeWith(Out()) \
        .setMaxIter(3).exec()
    out["rows"] = rows


def scenario_kmeans(out):
    from alink_amd import useLocalEnv, BatchOperator, KMeansTrainBatchOp, VectorAssemblerBatchOp
    from alink_amd.operator.batch.source import MemSourceBatchOp
    df = _data_frame()
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr="x0 double, x1 double, x2 double, x3 double, y int")
    va = VectorAssemblerBatchOp().setSelectedCols(["x0", "x1", "x2", "x3"]).setOutputCol("v").linkFrom(src)
    m = KMeansTrainBatchOp().setVectorCol("v").setK(4).setInitMode("RANDOM").setMaxIter(15).linkFrom(va)
    out["model"] = [list(r) for r in m.collect()]


def scenario_lr(out):
    from alink_amd import useLocalEnv, BatchOperator, LogisticRegressionTrainBatchOp
    df = _data_frame()
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr="x0 double, x1 double, x2 double, x3 double, y int")
    m = LogisticRegressionTrainBatchOp().setFeatureCols(["x0", "x1", "x2", "x3"]).setLabelCol("y").linkFrom(src)
    rows = m.collect()
    out["coef"] = json.loads(rows[1][1])["coefVector"]["data"]


def scenario_gbdt(out):
    from alink_amd import useLocalEnv, BatchOperator, GbdtTrainBatchOp, GbdtPredictBatchOp
    df = _data_frame()
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr="x0 double, x1 double, x2 double, x3 double, y int")
    m = GbdtTrainBatchOp().setFeatureCols(["x0", "x1", "x2", "x3"]).setLabelCol("y").setNumTrees(5) \
        .setMinSamplesPerLeaf(5).setMaxDepth(4).linkFrom(src)
    out["model"] = [list(r) for r in m.collect()]


def scenario_gbdt_rank(out):
    """LambdaMART-NDCG over queries spread across ranks: rows are exchanged so each query lives on one rank."""
    import numpy as np
    import pandas as pd
    from alink_amd import useLocalEnv, BatchOperator, GbdtRegTrainBatchOp
    useLocalEnv(1)
    rng = np.random.default_rng(4)
    X = rng.normal(size=(480, 3))
    rel = np.clip(np.round(1.5 + X[:, 0] - 0.5 * X[:, 1]), 0, 3)
    df = pd.DataFrame({"f0": X[:, 0], "f1": X[:, 1], "f2": X[:, 2], "qid": (np.arange(480) * 7) % 40, "rel": rel})
    src = BatchOperator.fromDataframe(df, schemaStr="f0 double, f1 double, f2 double, qid int, rel double")
    m = GbdtRegTrainBatchOp(algoType=int(os.environ.get("ALINK_TEST_ALGO", "2"))) \
        .setFeatureCols(["f0", "f1", "f2"]).setLabelCol("rel").setGroupCol("qid").setNumTrees(4) \
        .setMinSamplesPerLeaf(5).setMaxDepth(3).linkFrom(src)
    out["model"] = [list(r) for r in m.collect()]

def scenario_gbdt_wide(out):
    """7 continuous features (not a multiple of the world size): feature-sharded histograms with a padded block."""
    import numpy as np
    import pandas as pd
    from alink_amd import useLocalEnv, BatchOperator, GbdtTrainBatchOp
    from alink_amd.models.tree.engine import TreeBuilder
    rng = np.random.default_rng(11)
    X = rng.normal(size=(900, 7))
    y = (X @ np.array([1.0, -2.0, 0.5, 0.0, 1.5, -0.7, 0.3]) + 0.3 * np.sin(3 * X[:, 3]) > 0).astype(int)
    df = pd.DataFrame({f"x{i}": X[:, i] for i in range(7)})
    df["y"] = y
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr=", ".join(f"x{i} double" for i in range(7)) + ", y int")
    before = TreeBuilder.SHARDED_SEARCHES
    m = GbdtTrainBatchOp().setFeatureCols([f"x{i}" for i in range(7)]).setLabelCol("y").setNumTrees(4) \
        .setMinSamplesPerLeaf(5).setMaxDepth(5).linkFrom(src)
    out["model"] = [list(r) for r in m.collect()]
    out["sharded"] = TreeBuilder.SHARDED_SEARCHES - before


def scenario_gbdt_many(out):
    """200 continuous features: rank blocks of 4 x 32-feature groups, reduce-scattered in 4 pipelined pieces."""
    import numpy as np
    import pandas as pd
    from alink_amd import useLocalEnv, BatchOperator, GbdtTrainBatchOp
    from alink_amd.models.tree.engine import TreeBuilder
    rng = np.random.default_rng(12)
    X = rng.normal(size=(600, 200))
    w = rng.normal(size=200) * (rng.random(200) < 0.1)
    y = (X @ w + 0.2 * rng.normal(size=600) > 0).astype(int)
    df = pd.DataFrame({f"x{i}": X[:, i] for i in range(200)})
    df["y"] = y
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr=", ".join(f"x{i} double" for i in range(200)) + ", y int")
    before = TreeBuilder.SHARDED_SEARCHES
    nrs = TreeBuilder.RS_CALLS
    m = GbdtTrainBatchOp().setFeatureCols([f"x{i}" for i in range(200)]).setLabelCol("y").setNumTrees(2) \
        .setMinSamplesPerLeaf(5).setMaxDepth(4).linkFrom(src)
    out["model"] = [list(r) for r in m.collect()]
    out["sharded"] = TreeBuilder.SHARDED_SEARCHES - before
    out["rs_calls"] = TreeBuilder.RS_CALLS - nrs


def _tree_cat(out, kind):
    """Mixed categorical / continuous features under feature sharding (categorical bin orders are per (node,
    feature), so the owner of the feature computes them): ``kind`` = gbdt | gini | infogain | mse."""
    import numpy as np
    import pandas as pd
    from alink_amd import (useLocalEnv, BatchOperator, GbdtTrainBatchOp, RandomForestTrainBatchOp,
                           RandomForestRegTrainBatchOp)
    from alink_amd.models.tree.engine import TreeBuilder
    rng = np.random.default_rng(31)
    n = 1200
    c1 = rng.integers(0, 6, n)
    c2 = rng.integers(0, 9, n)
    X = rng.normal(size=(n, 5))
    score = X @ np.array([1.0, -1.0, 0.5, 0.0, 0.8]) + np.array([0.9, -0.8, 0.1, 1.2, -1.1, 0.0])[c1] \
        + 0.4 * np.cos(c2)
    df = pd.DataFrame({f"x{i}": X[:, i] for i in range(5)})
    df["c1"] = [f"a{v}" for v in c1]
    df["c2"] = [f"b{v}" for v in c2]
    df["y"] = (score > 0).astype(int) if kind != "mse" else np.round(score, 4)
    useLocalEnv(1)
    feats = [f"x{i}" for i in range(5)] + ["c1", "c2"]
    schema = ", ".join(f"x{i} double" for i in range(5)) + ", c1 string, c2 string, " + \
        ("y double" if kind == "mse" else "y int")
    src = BatchOperator.fromDataframe(df, schemaStr=schema)
    s0, r0, h0 = TreeBuilder.SHARDED_SEARCHES, sum(TreeBuilder.RS_BYTES), sum(TreeBuilder.HIST_BYTES)
    nr, nh = len(TreeBuilder.RS_BYTES), len(TreeBuilder.HIST_BYTES)
    if kind == "gbdt":
        op = GbdtTrainBatchOp().setNumTrees(3).setMinSamplesPerLeaf(10).setMaxDepth(4)
    elif kind == "mse":
        op = RandomForestRegTrainBatchOp().setNumTrees(2).setMaxDepth(4).setCreateTreeMode("parallel") \
            .setSubsamplingRatio(1.0)
    else:
        op = RandomForestTrainBatchOp().setNumTrees(2).setMaxDepth(4).setCreateTreeMode("parallel") \
            .setTreeType(kind.upper()).setSubsamplingRatio(1.0)
    m = op.setFeatureCols(feats).setCategoricalCols(["c1", "c2"]).setLabelCol("y").linkFrom(src)
    out["model"] = [list(r) for r in m.collect()]
    out["sharded"] = TreeBuilder.SHARDED_SEARCHES - s0
    out["rs_bytes"] = sum(list(TreeBuilder.RS_BYTES)[nr:]) if len(TreeBuilder.RS_BYTES) > nr else 0
    out["hist_bytes"] = sum(list(TreeBuilder.HIST_BYTES)[nh:])


def scenario_tree_cat_gbdt(out):
    _tree_cat(out, "gbdt")


def scenario_tree_cat_gini(out):
    _tree_cat(out, "gini")


def scenario_tree_cat_infogain(out):
    _tree_cat(out, "infogain")


def scenario_tree_cat_mse(out):
    _tree_cat(out, "mse")


def scenario_rf(out):
    from alink_amd import useLocalEnv, BatchOperator, RandomForestTrainBatchOp
    df = _data_frame()
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr="x0 double, x1 double, x2 double, x3 double, y int")
    m = RandomForestTrainBatchOp().setFeatureCols(["x0", "x1", "x2", "x3"]).setLabelCol("y").setNumTrees(3) \
        .setMaxDepth(5).linkFrom(src)
    out["model"] = [list(r) for r in m.collect()]


def scenario_rf_parallel(out):
    from alink_amd import useLocalEnv, BatchOperator, RandomForestTrainBatchOp
    df = _data_frame()
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr="x0 double, x1 double, x2 double, x3 double, y int")
    m = RandomForestTrainBatchOp().setFeatureCols(["x0", "x1", "x2", "x3"]).setLabelCol("y").setNumTrees(3) \
        .setMaxDepth(5).setCreateTreeMode("parallel").linkFrom(src)
    out["model"] = [list(r) for r in m.collect()]


def scenario_rf_sampled(out):
    """Tree-parallel forest with row subsampling: tree t's sample does not depend on which rank grows it."""
    from alink_amd import useLocalEnv, BatchOperator, RandomForestTrainBatchOp
    df = _data_frame()
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr="x0 double, x1 double, x2 double, x3 double, y int")
    m = RandomForestTrainBatchOp().setFeatureCols(["x0", "x1", "x2", "x3"]).setLabelCol("y").setNumTrees(5) \
        .setMaxDepth(4).setSubsamplingRatio(0.6).linkFrom(src)
    out["model"] = [list(r) for r in m.collect()]


def scenario_als(out):
    import numpy as np
    import pandas as pd
    from alink_amd import useLocalEnv, BatchOperator, AlsTrainBatchOp
    rng = np.random.default_rng(5)
    uu, ii = np.nonzero(rng.random((40, 30)) < 0.4)
    df = pd.DataFrame({"u": uu * 3 + 1, "i": ii * 7 + 2, "r": rng.normal(size=uu.size)})
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr="u bigint, i bigint, r double")
    m = AlsTrainBatchOp().setUserCol("u").setItemCol("i").setRateCol("r").setRank(6).setNumIter(5) \
        .setNumBlocks(2).linkFrom(src)
    out["model"] = [list(r) for r in m.collect()]


def scenario_cross(out):
    """Ring blockwise top-K: queries and items split unevenly over the ranks."""
    import numpy as np
    import torch
    from alink_amd.parallel import comm
    from alink_amd.parallel.cross import blockwise_topk
    comm.init_distributed()
    ws, me = comm.get_world_size(), comm.get_rank()
    g = torch.Generator().manual_seed(3)
    Q = torch.randn(37, 10, generator=g)
    T = torch.randn(53, 10, generator=g)
    qb = [0, 5, 20, 37] if ws == 3 else [0, 37]
    ib = [0, 30, 31, 53] if ws == 3 else [0, 53]
    for desc in (True, False):
        v, i = blockwise_topk(Q[qb[me]:qb[me + 1]], T[ib[me]:ib[me + 1]], 7, descending=desc)
        out["desc" if desc else "asc"] = {"v": v.tolist(), "i": i.tolist(), "q0": qb[me]}


def run(rank, world, port, scenario, outdir):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "ALINK_DEVICE": "cpu"})
    out = {}
    try:
        globals()["scenario_" + scenario](out)
    except Exception:
        out["error"] = traceback.format_exc()
    with open(os.path.join(outdir, f"{scenario}_{world}_{rank}.json"), "w") as f:
        json.dump(out, f)
    from alink_amd.parallel import comm
    comm.shutdown()


def scenario_glm(out):
    import json as _j
    from alink_amd import useLocalEnv, BatchOperator, GlmTrainBatchOp
    df = _data_frame()
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr="x0 double, x1 double, x2 double, x3 double, y int")
    op = GlmTrainBatchOp().setFamily("binomial").setFeatureCols(["x0", "x1", "x2", "x3"]).setLabelCol("y")
    model = src.link(op)
    out["summary"] = _j.loads(model.getSideOutput(1).collect()[0][0])


def scenario_isotonic(out):
    import json as _j
    from alink_amd import useLocalEnv, BatchOperator, IsotonicRegTrainBatchOp
    df = _data_frame()
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr="x0 double, x1 double, x2 double, x3 double, y int")
    rows = sorted(src.link(IsotonicRegTrainBatchOp().setFeatureCol("x1").setLabelCol("x0")).collect(),
                  key=lambda r: r[0])
    out["b"] = _j.loads(rows[1][1])
    out["v"] = _j.loads(rows[2][1])


def scenario_fm(out):
    from alink_amd import useLocalEnv, BatchOperator, FmClassifierTrainBatchOp, FmClassifierPredictBatchOp
    df = _data_frame()
    useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr="x0 double, x1 double, x2 double, x3 double, y int")
    model = src.link(FmClassifierTrainBatchOp().setFeatureCols(["x0", "x1", "x2", "x3"]).setLabelCol("y")
                     .setNumEpochs(20).setLearnRate(0.1).setNumFactor(2))
    pred = FmClassifierPredictBatchOp().setPredictionCol("p").linkFrom(model, src).collect()
    out["model"] = [list(r) for r in model.collect()]
    out["acc"] = sum(int(r[-1] == r[-2]) for r in pred) / max(len(pred), 1)


def scenario_eval_stream_windows(out):
    """EvalBinaryClassStreamOp with 1 s windows while rank 1 stalls 0.3 s per micro-batch: the window decision
    is agreed over the host group, so both ranks emit the same windows with the same (all-reduced) metrics."""
    import time
    import numpy as np
    import pandas as pd
    os.environ["ALINK_STREAM_BATCH"] = "40"
    from alink_amd import useLocalEnv, StreamOperator, EvalBinaryClassStreamOp, CollectStreamOp
    from alink_amd.parallel import comm
    useLocalEnv(1)
    rng = np.random.default_rng(5)
    p = rng.random(480)
    y = (rng.random(480) < p).astype(int)
    df = pd.DataFrame({"label": y, "detail": [f'{{"1":{v},"0":{1 - v}}}' for v in p]})
    box = []
    ev = EvalBinaryClassStreamOp().setLabelCol("label").setPredictionDetailCol("detail").setTimeInterval(1)
    ev.linkFrom(StreamOperator.fromDataframe(df, schemaStr="label int, detail string")).link(CollectStreamOp(box))
    if comm.get_rank() == 1:
        orig = ev.on_batch

        def slow(port, mt):
            time.sleep(0.3)
            return orig(port, mt)
        ev.on_batch = slow
    StreamOperator.execute()
    out["rows"] = [list(r) for r in box]


def _ftrl_run(mode, rows, batch, async_reduce=False):
    import numpy as np
    import pandas as pd
    os.environ["ALINK_STREAM_BATCH"] = str(batch)
    from alink_amd import (useLocalEnv, BatchOperator, StreamOperator, LogisticRegressionTrainBatchOp,
                           FtrlTrainStreamOp, CollectStreamOp)
    useLocalEnv(1)
    rng = np.random.default_rng(3)
    X = rng.normal(size=(rows, 5))
    y = (X @ np.array([1.0, -1.0, 0.5, 0.0, 2.0]) + 0.3 * rng.normal(size=rows) > 0).astype(int) + 1
    df = pd.DataFrame({f"f{i}": X[:, i] for i in range(5)})
    df["label"] = y
    schema = ", ".join(f"f{i} double" for i in range(5)) + ", label int"
    batch_op = BatchOperator.fromDataframe(df.iloc[:40], schemaStr=schema)
    stream = StreamOperator.fromDataframe(df, schemaStr=schema)
    cols = [f"f{i}" for i in range(5)]
    model = LogisticRegressionTrainBatchOp().setFeatureCols(cols).setLabelCol("label").setMaxIter(3).linkFrom(batch_op)
    snaps = []
    op = FtrlTrainStreamOp(model).setFeatureCols(cols).setLabelCol("label").setTimeInterval(1e9).setAlpha(0.1) \
        .setBeta(0.1).setL1(0.01).setL2(0.01).setWithIntercept(True).setUpdateMode(mode)
    if async_reduce:
        op.set("asyncGradReduce", True)
    op.linkFrom(stream).link(CollectStreamOp(snaps))
    StreamOperator.execute()
    last = max(r[0] for r in snaps)
    _ftrl_run.recv_nnz = list(op.recv_nnz)
    return [list(r[2:]) for r in snaps if r[0] == last], sorted({r[0] for r in snaps})


def scenario_ftrl_seq(out):
    out["model"], out["bids"] = _ftrl_run("SEQUENTIAL", 64, 4096)


def scenario_ftrl_sharded(out):
    out["model"], out["bids"] = _ftrl_run("SHARDED", 64, 4096)


def scenario_ftrl_sharded_split(out):
    """SplitVector exchange: each shard receives only the nonzeros in its coefficient range."""
    out["model"], out["bids"] = _ftrl_run("SHARDED", 400, 30)
    out["recv_nnz"] = _ftrl_run.recv_nnz


def scenario_ftrl_sharded_allgather(out):
    """The same steps with the whole micro-batch all-gathered to every shard (the round-2 exchange)."""
    os.environ["ALINK_FTRL_SHARDED_EXCHANGE"] = "allgather"
    out["model"], out["bids"] = _ftrl_run("SHARDED", 400, 30)


def scenario_ftrl_dp(out):
    out["model"], out["bids"] = _ftrl_run("DATA_PARALLEL", 400, 4096)


def scenario_ftrl_dp_async(out):
    """DATA_PARALLEL with the gradient all-reduce overlapped with the next step (one-step-stale gradients)."""
    out["model"], out["bids"] = _ftrl_run("DATA_PARALLEL", 400, 25, async_reduce=True)
    out["sync"], _ = _ftrl_run("DATA_PARALLEL", 400, 25)
    out["one_async"], _ = _ftrl_run("DATA_PARALLEL", 400, 4096, async_reduce=True)
    out["one_sync"], _ = _ftrl_run("DATA_PARALLEL", 400, 4096)


def scenario_ftrl_uneven(out):
    # 9 rows, 2-row micro-batches: rank 0 has 3 batches, rank 1 has 2 -> lockstep with empty steps
    out["model"], out["bids"] = _ftrl_run("SHARDED", 9, 2)


def scenario_ftrl_ckpt(out):
    """Lockstep stream checkpoint on P ranks (phase from ALINK_TEST_PHASE): ``ref`` runs through, ``crash`` dies
    inside the 6th FTRL step on every rank, ``resume`` restarts from the agreed checkpoint round."""
    import numpy as np
    import pandas as pd
    from alink_amd import (useLocalEnv, BatchOperator, StreamOperator, LogisticRegressionTrainBatchOp,
                           FtrlTrainStreamOp, CollectStreamOp)
    from alink_amd.operator.stream import onlinelearning as ol
    phase = os.environ["ALINK_TEST_PHASE"]
    os.environ["ALINK_STREAM_BATCH"] = "7"
    useLocalEnv(1)
    rng = np.random.default_rng(5)
    X = rng.normal(size=(150, 4))
    df = pd.DataFrame({f"f{i}": X[:, i] for i in range(4)})
    df["label"] = (X @ np.array([1.0, -1.0, 0.5, 0.2]) > 0).astype(int)
    schema = ", ".join(f"f{i} double" for i in range(4)) + ", label int"
    cols = [f"f{i}" for i in range(4)]
    model = LogisticRegressionTrainBatchOp().setFeatureCols(cols).setLabelCol("label").setMaxIter(3) \
        .linkFrom(BatchOperator.fromDataframe(df.iloc[:40], schemaStr=schema))
    ckdir = os.path.join(os.environ["ALINK_TEST_TMP"], "ck_" + ("ref" if phase == "ref" else "run"))
    StreamOperator.setCheckPointConf(interval_s=1e9, directory=ckdir, every_batches=2)
    snaps = []
    FtrlTrainStreamOp(model).setFeatureCols(cols).setLabelCol("label").setTimeInterval(1e9) \
        .setUpdateMode("SHARDED").linkFrom(StreamOperator.fromDataframe(df, schemaStr=schema)) \
        .link(CollectStreamOp(snaps))
    if phase == "crash":
        # the per-step entry (the SHARDED multi-rank step goes through _sharded_step, one rank through _apply)
        orig = ol.FtrlTrainStreamOp._step
        calls = {"n": 0}

        def boom(self, *a):
            calls["n"] += 1
            if calls["n"] > 5:
                raise RuntimeError("injected crash")
            return orig(self, *a)
        ol.FtrlTrainStreamOp._step = boom
    try:
        StreamOperator.execute()
    except RuntimeError as e:
        out["crashed"] = str(e)
        out["files"] = sorted(os.listdir(ckdir))
        return
    last = max(r[0] for r in snaps)
    out["model"] = [list(r[2:]) for r in snaps if r[0] == last]
    out["left"] = sorted(os.listdir(ckdir))


def scenario_shuffle_strings(out):
    """Hash partition of a string-keyed table: packed UTF-8 all-to-all, device-independent key hashes."""
    import numpy as np
    import torch
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.parallel import comm, shuffle
    comm.init_distributed()
    ws, me = comm.get_world_size(), comm.get_rank()
    rng = np.random.default_rng(100 + me)
    n = 20000
    keys = [f"user-{int(k):06d}-\u00e9" for k in rng.integers(0, 50000, n)]
    payload = ["x" * int(l) for l in rng.integers(0, 40, n)]
    payload[::97] = [None] * len(payload[::97])
    vals = torch.as_tensor(rng.normal(size=n))
    mt = MTable(TableSchema(["k", "p", "v"], [Types.STRING, Types.STRING, Types.DOUBLE]),
                [Column(keys), Column(StringBlock.from_list(payload)), Column(vals)])
    shuffle.STATS.reset()
    part = shuffle.hash_partition(mt, [0])
    out["is_block"] = [isinstance(c.values, StringBlock) for c in part.cols[:2]]
    out["rows"] = part.num_rows
    out["keys"] = sorted(set(part.cols[0].to_list()))
    out["sent_rows"] = [list(r) for r in zip(keys, payload, vals.tolist())]
    out["recv_rows"] = [list(r) for r in part.rows()]
    out["string_bytes_recv"] = shuffle.STATS.string_bytes_recv
    out["string_bytes_total_local"] = sum(len(k.encode()) for k in keys) + sum(len(p) for p in payload if p)
    fixed = ["a", "", "user-000001-\u00e9", "\U0001F600", None, "longer key with spaces"]
    fmt = MTable(TableSchema(["k", "n"], [Types.STRING, Types.LONG]),
                 [Column(fixed), Column(torch.arange(len(fixed), dtype=torch.int64))])
    out["hash_sample"] = shuffle.key_hash(fmt, [0, 1]).tolist()
    out["hash_keys"] = [str(x) for x in fixed]


def scenario_shuffle_partial_nulls(out):
    """Only rank 0's value column carries a NULL mask, and the object key column holds numbers on rank 0 but a
    mix of numbers and strings on rank 1: every rank must issue the same collectives (no deadlock) and equal
    keys must co-locate (one agreed hash family per column)."""
    import torch
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.parallel import comm, shuffle
    comm.init_distributed()
    me = comm.get_rank()
    n = 40
    v = torch.arange(n, dtype=torch.float64) + 1000 * me
    nulls = (torch.arange(n) % 5 == 0) if me == 0 else None
    keys = [i % 7 for i in range(n)] if me == 0 else [(i % 7 if i % 3 else str(i % 7)) for i in range(n)]
    mt = MTable(TableSchema(["k", "v"], [Types.STRING, Types.DOUBLE]), [Column(keys), Column(v, nulls)])
    part = shuffle.hash_partition(mt, [0])
    out["rows"] = [[str(r[0]), r[1]] for r in part.rows()]
    out["sent"] = [[str(k), (None if nulls is not None and bool(nulls[i]) else float(v[i]))]
                   for i, k in enumerate(keys)]


def scenario_gather(out):
    """gather_table moves columns in native form (no whole-table pickle): tensors, null masks, sparse blocks,
    packed strings; object columns alone pickled."""
    import torch
    from alink_amd.common.linalg import DenseVector
    from alink_amd.common.linalg.block import SparseBlock
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.base import gather_table
    from alink_amd.parallel import comm
    comm.init_distributed()
    me = comm.get_rank()
    n = 5 + me
    x = torch.arange(n, dtype=torch.float64) + 100 * me
    nm = torch.zeros(n, dtype=torch.bool)
    nm[1] = True
    s = [f"r{me}-{i}-\u00e9" if i != 2 else None for i in range(n)]
    crow = torch.arange(n + 1, dtype=torch.int64)
    sb = SparseBlock(crow, torch.full((n,), me, dtype=torch.int32), torch.ones(n, dtype=torch.float64), 8)
    objs = [{"k": me, "i": i} for i in range(n)]
    mt = MTable(TableSchema(["x", "s", "v", "o"], [Types.DOUBLE, Types.STRING, Types.SPARSE_VECTOR, Types.STRING]),
                [Column(x, nm), Column(s), Column(sb), Column(objs)], False)
    full = gather_table(mt)
    out["kinds"] = [type(c.values).__name__ for c in full.cols]
    out["rows"] = [[str(v) for v in r] for r in full.rows()]


def scenario_sql(out):
    """Distributed relational ops: each rank returns its partition of every result."""
    import numpy as np
    import pandas as pd
    from alink_amd import (useLocalEnv, BatchOperator, JoinBatchOp, GroupByBatchOp, DistinctBatchOp,
                           OrderByBatchOp, UnionBatchOp, IntersectBatchOp, MinusBatchOp, LeftOuterJoinBatchOp)
    useLocalEnv(1)
    rng = np.random.default_rng(11)
    n = 97
    a = pd.DataFrame({"id": rng.integers(0, 30, n), "name": [f"n{x}" for x in rng.integers(0, 7, n)],
                      "v": np.round(rng.normal(size=n), 3)})
    b = pd.DataFrame({"key": rng.integers(0, 40, 61), "w": rng.integers(0, 5, 61).astype(float)})
    A = BatchOperator.fromDataframe(a, schemaStr="id long, name string, v double")
    B = BatchOperator.fromDataframe(b, schemaStr="key long, w double")
    res = {}
    res["join"] = JoinBatchOp().setJoinPredicate("a.id = b.key").setSelectClause("a.id, a.name, b.w") \
        .linkFrom(A, B).collect()
    res["ljoin"] = LeftOuterJoinBatchOp().setJoinPredicate("a.id = b.key").setSelectClause("a.id, b.w") \
        .linkFrom(A, B).collect()
    res["group"] = GroupByBatchOp().setGroupByPredicate("name").setSelectClause("name, count(*) as c, sum(v) as s") \
        .linkFrom(A).collect()
    res["distinct"] = DistinctBatchOp().linkFrom(A.select("name")).collect()
    res["order"] = OrderByBatchOp().setClause("v").setOrder("desc").linkFrom(A).collect()
    res["order_lim"] = OrderByBatchOp().setClause("id, v").setLimit(13).linkFrom(A).collect()
    ids = A.select("id")
    keys = B.select("key")
    res["union"] = UnionBatchOp().linkFrom(ids, keys).collect()
    res["intersect"] = IntersectBatchOp().linkFrom(ids, keys).collect()
    res["minus"] = MinusBatchOp().linkFrom(ids, keys).collect()
    A.registerTableName("ta")
    B.registerTableName("tb")
    res["order_sqlquery"] = BatchOperator.sqlQuery(
        "select t.name, count(*) c, sum(w) sw from ta t join tb u on t.id = u.key "
        "where u.w > 0 group by t.name having count(*) > 1 order by sw desc, name").collect()
    out["res"] = {k: [list(r) for r in v] for k, v in res.items()}


def scenario_csv(out):
    """Byte-range sharded CSV read: every rank parses only its split; gathered rows equal the file."""
    import os
    from alink_amd import useLocalEnv, CsvSourceBatchOp
    from alink_amd.parallel import comm
    useLocalEnv(1)
    path = os.path.join(os.environ["ALINK_TEST_TMP"], "data.csv")
    if comm.get_rank() == 0 and not os.path.exists(path):
        with open(path + ".tmp", "w") as f:
            f.write("id,name,v\n")
            for i in range(503):
                f.write(f"{i},name{i % 17},{i * 0.5}\n")
        os.replace(path + ".tmp", path)
    comm.barrier()
    op = CsvSourceBatchOp().setFilePath(path).setSchemaStr("id long, name string, v double").setIgnoreFirstLine(True)
    out["local_rows"] = op.getOutputTable().num_rows
    out["rows"] = [list(r) for r in op.collect()]


def scenario_trace(out):
    """Timeline + metrics on a 2-rank KMeans: op / superstep / item / collective spans per rank."""
    import os
    from alink_amd.utils import trace, metrics
    trace.reset()
    trace.enable(os.path.join(os.environ["ALINK_TEST_TMP"], "trace_{rank}.json"))
    metrics.clear()
    scenario_kmeans({})
    path = trace.dump()
    trace.disable()
    out["trace"] = path
    out["steps"] = [r for r in metrics.records("superstep") if r.get("job") == "KMeans"]


def scenario_eval_uneven(out):
    """Binary evaluation where rank 0 holds 200 rows and rank 1 60 (P=1 holds all 260), as a stream (40-row
    micro-batches, windows after every batch; phase ``ckpt`` adds a stream checkpoint conf) and as a batch op.
    Phase ``mixed``: rank 0's detail column is a columnar DetailBlock, rank 1's plain strings — the ranks must
    agree on one summary branch instead of issuing different collectives."""
    import numpy as np
    os.environ["ALINK_STREAM_BATCH"] = "40"
    from alink_amd import useLocalEnv, StreamOperator, EvalBinaryClassStreamOp, EvalBinaryClassBatchOp, \
        CollectStreamOp
    from alink_amd.common.detail import DetailBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    from alink_amd.operator.stream.source import TableSourceStreamOp
    from alink_amd.parallel import comm
    import torch
    phase = os.environ.get("ALINK_TEST_PHASE", "plain")
    useLocalEnv(1)
    rng = np.random.default_rng(11)
    p = rng.random(260)
    y = (rng.random(260) < p).astype(np.int64)
    ws, r = comm.get_world_size(), comm.get_rank()
    sl = slice(0, 260) if ws == 1 else (slice(0, 200) if r == 0 else slice(200, 260))
    blk = DetailBlock(["1", "0"], np.stack([p[sl], 1.0 - p[sl]], 1))
    dcol = Column(blk) if (phase == "mixed" and r == 0) or ws == 1 else Column(blk.to_list())
    mt = MTable(TableSchema(["label", "detail"], [Types.LONG, Types.STRING]),
                [Column(torch.from_numpy(y[sl].copy())), dcol])
    if phase == "ckpt":
        StreamOperator.setCheckPointConf(interval_s=1e9, directory=os.path.join(os.environ["ALINK_TEST_TMP"],
                                         "ck_eval"), every_batches=2)
    box = []
    EvalBinaryClassStreamOp().setLabelCol("label").setPredictionDetailCol("detail").setTimeInterval(0) \
        .linkFrom(TableSourceStreamOp(mt)).link(CollectStreamOp(box))
    StreamOperator.execute()
    out["stream"] = [list(rw) for rw in box]
    m = EvalBinaryClassBatchOp().setLabelCol("label").setPredictionDetailCol("detail") \
        .linkFrom(TableSourceBatchOp(mt)).collectMetrics()
    out["batch"] = {"auc": m.getAuc(), "logloss": m.getLogLoss(), "total": m.getTotalSamples()}


def scenario_stream_ops_uneven(out):
    """Lockstep micro-batches through the common stream operators when the ranks' streams differ in length (rank 0:
    150 rows, rank 1: 20 rows, or none with ALINK_TEST_PHASE=empty; 40-row micro-batches): rank 1 feeds empty
    batches for most rounds.  Every branch's rows on a rank must equal the batch ops over that rank's rows."""
    import numpy as np
    import pandas as pd
    os.environ["ALINK_STREAM_BATCH"] = "40"
    from alink_amd import (useLocalEnv, BatchOperator, StreamOperator, CollectStreamOp, CsvSinkStreamOp,
                           VectorAssemblerStreamOp, VectorAssemblerBatchOp, LogisticRegressionTrainBatchOp,
                           LogisticRegressionPredictStreamOp, LogisticRegressionPredictBatchOp,
                           StandardScalerTrainBatchOp, StandardScalerPredictStreamOp, StandardScalerPredictBatchOp,
                           StringIndexerTrainBatchOp, StringIndexerPredictStreamOp, StringIndexerPredictBatchOp,
                           KMeansTrainBatchOp, KMeansPredictStreamOp, KMeansPredictBatchOp, GbdtTrainBatchOp,
                           GbdtPredictStreamOp, GbdtPredictBatchOp, TokenizerStreamOp, TokenizerBatchOp,
                           EvalBinaryClassStreamOp)
    from alink_amd.common.table import MTable
    from alink_amd.operator.batch.source import TableSourceBatchOp
    from alink_amd.operator.stream.source import TableSourceStreamOp
    from alink_amd.parallel import comm
    useLocalEnv(1)
    rng = np.random.default_rng(3)
    n = 170
    X = rng.normal(size=(n, 3))
    df = pd.DataFrame({"x0": X[:, 0], "x1": X[:, 1], "x2": X[:, 2],
                       "y": (X @ np.array([1.0, -1.0, 0.5]) > 0).astype(int),
                       "s": [["Alpha Beta", "beta", "GAMMA x"][i % 3] for i in range(n)]})
    schema = "x0 double, x1 double, x2 double, y int, s string"
    feats = ["x0", "x1", "x2"]
    train = BatchOperator.fromDataframe(df, schemaStr=schema)
    lr = LogisticRegressionTrainBatchOp().setFeatureCols(feats).setLabelCol("y").setMaxIter(5).linkFrom(train)
    sc = StandardScalerTrainBatchOp().setSelectedCols(feats).linkFrom(train)
    si = StringIndexerTrainBatchOp().setSelectedCol("s").linkFrom(train)
    km = KMeansTrainBatchOp().setVectorCol("v").setK(3).setMaxIter(5).linkFrom(
        VectorAssemblerBatchOp().setSelectedCols(feats).setOutputCol("v").linkFrom(train))
    gb = GbdtTrainBatchOp().setFeatureCols(feats).setLabelCol("y").setNumTrees(3).setMinSamplesPerLeaf(5) \
        .linkFrom(train)
    ws, r = comm.get_world_size(), comm.get_rank()
    phase = os.environ.get("ALINK_TEST_PHASE", "short")
    local = df.iloc[:150] if r == 0 else (df.iloc[150:] if phase == "short" else df.iloc[:0])
    mt = MTable.from_rows([tuple(x) for x in local.itertuples(index=False)], schema)
    mt.replicated = False
    branches = {
        "lr": (lambda s: LogisticRegressionPredictStreamOp(lr).setPredictionCol("p").setPredictionDetailCol("d")
               .linkFrom(s),
               lambda b: LogisticRegressionPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d")
               .linkFrom(lr, b)),
        "scaler": (lambda s: StandardScalerPredictStreamOp(sc).linkFrom(s),
                   lambda b: StandardScalerPredictBatchOp().linkFrom(sc, b)),
        "indexer": (lambda s: StringIndexerPredictStreamOp(si).setSelectedCol("s").setOutputCol("si").linkFrom(s),
                    lambda b: StringIndexerPredictBatchOp().setSelectedCol("s").setOutputCol("si").linkFrom(si, b)),
        "kmeans": (lambda s: KMeansPredictStreamOp(km).setPredictionCol("c").linkFrom(
                       VectorAssemblerStreamOp().setSelectedCols(feats).setOutputCol("v").linkFrom(s)),
                   lambda b: KMeansPredictBatchOp().setPredictionCol("c").linkFrom(
                       km, VectorAssemblerBatchOp().setSelectedCols(feats).setOutputCol("v").linkFrom(b))),
        "gbdt": (lambda s: GbdtPredictStreamOp(gb).setPredictionCol("g").linkFrom(s),
                 lambda b: GbdtPredictBatchOp().setPredictionCol("g").linkFrom(gb, b)),
        "sql_tok": (lambda s: TokenizerStreamOp().setSelectedCol("s").setOutputCol("t").linkFrom(
                        s.where("x0 > -0.5").select("x0, y, s")),
                    lambda b: TokenizerBatchOp().setSelectedCol("s").setOutputCol("t").linkFrom(
                        b.where("x0 > -0.5").select("x0, y, s"))),
    }
    src = TableSourceStreamOp(mt)
    boxes = {k: [] for k in branches}
    for k, (sf, _) in branches.items():
        sf(src).link(CollectStreamOp(boxes[k]))
    ev_box = []
    EvalBinaryClassStreamOp().setLabelCol("y").setPredictionDetailCol("d").setTimeInterval(0).linkFrom(
        branches["lr"][0](src)).link(CollectStreamOp(ev_box))
    CsvSinkStreamOp().setFilePath(os.path.join(os.environ["ALINK_TEST_TMP"], f"uneven_{phase}_{ws}.csv")) \
        .setOverwriteSink(True).linkFrom(branches["indexer"][0](src))
    StreamOperator.execute()
    out["ok"] = {}
    for k, (_, bf) in branches.items():
        want = [list(x) for x in bf(TableSourceBatchOp(mt)).getOutputTable().rows()]
        got = [list(x) for x in boxes[k]]
        out["ok"][k] = got == want
        out.setdefault("rows", {})[k] = len(got)
    out["eval_windows"] = len(ev_box)


if __name__ == "__main__":
    run(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5])
