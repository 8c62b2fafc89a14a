"""Rank processes for tests/test_multiprocess_gpu.py: P processes sharing ONE MI355X (gloo host group, device
tensors on cuda:0, collectives of small device buffers through the one-shot IPC kernel) — the rehearsal of an
8-GPU job on a 1-GPU box.  Each rank writes <outdir>/<scenario>_<world>_<rank>.json."""
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def _rank_tensor(r, n, dtype, seed):
    import torch
    g = torch.Generator().manual_seed(seed * 7919 + r)
    return (torch.randn(n, generator=g, dtype=torch.float64) * (r + 1)).to(dtype)


def scenario_oneshot(out):
    """Bit-exact rank-order reductions through the one-shot kernel, several sizes / dtypes / ops."""
    import torch
    from alink_amd.parallel import comm, oneshot
    comm.init_distributed()
    ws, me = comm.get_world_size(), comm.get_rank()
    dev = comm.device_for_rank()
    checks = []
    for seed, (n, dtype, op) in enumerate([(1, torch.float64, "sum"), (129 * 100, torch.float64, "sum"),
                                           (5000, torch.float32, "sum"), (77777, torch.float64, "max"),
                                           (3, torch.float32, "min"), (131072, torch.float64, "sum")]):
        for rep in range(3):                      # the staging slots alternate with the sequence number
            x = _rank_tensor(me, n, dtype, seed * 10 + rep).to(dev)
            comm.all_reduce(x, op)
            parts = [_rank_tensor(r, n, dtype, seed * 10 + rep) for r in range(ws)]
            ref = parts[0].clone()
            for p in parts[1:]:
                ref = ref + p if op == "sum" else (torch.maximum(ref, p) if op == "max" else torch.minimum(ref, p))
            checks.append(bool(torch.equal(x.cpu(), ref)))
    inst = oneshot._INSTANCE
    out["checks"] = checks
    out["oneshot_calls"] = comm.STATS.oneshot
    out["instance"] = inst is not None
    out["backend"] = comm._backend()
    out["peers_opened"] = len(inst.opened) if inst is not None else -1


def scenario_kmeans(out):
    """KMeans on bf16 [N,128] (v10 fused kernel) with the [k,129] all-reduce on the one-shot path."""
    from alink_amd import useLocalEnv, KMeansTrainBatchOp, RandomVectorSourceBatchOp
    from alink_amd.parallel import comm
    env = useLocalEnv(1)
    src = RandomVectorSourceBatchOp().setNumRows(200_003).setSize(128).setNumClusters(20).setClusterStd(1.0) \
        .setCenterScale(4.0).setDtype("bf16").setSeed(17).setOutputCol("vec")
    op = KMeansTrainBatchOp().setVectorCol("vec").setK(20).setMaxIter(12).setEpsilon(-1.0).setInitMode("RANDOM") \
        .linkFrom(src)
    rows = op.collect()
    out["model"] = [[r[0], r[1]] for r in rows]
    out["iterations"] = op.getTrainInfo()["iterations"]
    out["oneshot_calls"] = comm.STATS.oneshot
    out["backend"] = comm._backend()
    from alink_amd.parallel import oneshot
    out["oneshot_setup_error"] = oneshot.SETUP_ERROR
    out["device"] = str(env.device)


def scenario_kmeans_headline(out):
    """The bench's configuration (bf16 Gaussian mixture, k=100, d=128, k-means|| init with the reference
    seeding) at ``ALINK_REH_ROWS`` rows (default 1e8) for ``ALINK_REH_ITERS`` Lloyd supersteps: the model, the
    one-shot count and the device time of the supersteps' collectives."""
    import torch
    from alink_amd import useLocalEnv, KMeansTrainBatchOp, RandomVectorSourceBatchOp
    from alink_amd.operator.batch.source import TableSourceBatchOp
    from alink_amd.parallel import comm, oneshot
    env = useLocalEnv(1)
    rows = int(float(os.environ.get("ALINK_REH_ROWS", "1e8")))
    iters = int(os.environ.get("ALINK_REH_ITERS", "8"))
    src = RandomVectorSourceBatchOp().setNumRows(rows).setSize(128).setNumClusters(100).setClusterStd(1.0) \
        .setCenterScale(4.0).setDtype("bf16").setSeed(2024).setOutputCol("vec")
    import time
    t0 = time.time()
    data = src.getOutputTable()
    print(f"[rank {env.rank}] data {data.num_rows} rows {time.time() - t0:.1f}s", flush=True)
    comm.device_timing(env.device.type == "cuda")
    op = KMeansTrainBatchOp().setVectorCol("vec").setK(100).setMaxIter(iters).setEpsilon(-1.0)
    op._on_step = lambda step, q: print(f"[rank {env.rank}] superstep {step} {time.time() - t0:.1f}s", flush=True)
    op.linkFrom(TableSourceBatchOp(data))
    res = op.collect()
    comm.device_timing(False)
    n_ev, dev_s, per = comm.device_timing_collect()
    out["model"] = [[r[0], r[1]] for r in res]
    out["iterations"] = op.getTrainInfo()["iterations"]
    out["oneshot_calls"] = comm.STATS.oneshot
    out["oneshot_P"] = oneshot._INSTANCE.P if oneshot._INSTANCE is not None else None
    out["oneshot_setup_error"] = oneshot.SETUP_ERROR
    out["backend"] = comm._backend()
    out["rows_local"] = int(data.num_rows)
    out["collective_device_us"] = {k: round(v * 1e6, 1) for k, v in per.items()}
    out["collectives_timed"] = n_ev
    out["device"] = str(env.device)
    if env.device.type == "cuda":
        torch.cuda.synchronize()


def scenario_als(out):
    """ALS with device tensors over the ranks sharing the GPU: owner-partitioned ratings, the request/response
    all-to-all and the pipelined factor all-gather on device tensors; plus the reference doc example
    (docs/en/als.md) predictions."""
    import numpy as np
    import pandas as pd
    from alink_amd import useLocalEnv, BatchOperator, AlsTrainBatchOp, AlsPredictBatchOp
    from alink_amd.parallel import comm
    env = useLocalEnv(1)
    rng = np.random.default_rng(5)
    uu, ii = np.nonzero(rng.random((600, 400)) < 0.05)
    df = pd.DataFrame({"u": uu * 3 + 1, "i": ii * 7 + 2, "r": np.round(rng.normal(size=uu.size), 3)})
    src = BatchOperator.fromDataframe(df, schemaStr="u bigint, i bigint, r double")
    m = AlsTrainBatchOp().setUserCol("u").setItemCol("i").setRateCol("r").setRank(8).setNumIter(6) \
        .setLambda(0.1).linkFrom(src)
    out["model"] = [list(r) for r in m.collect()]
    doc = np.array([[1, 1, 0.6], [2, 2, 0.8], [2, 3, 0.6], [4, 1, 0.6], [4, 2, 0.3], [4, 3, 0.4]])
    ddf = pd.DataFrame({"user": doc[:, 0].astype(int), "item": doc[:, 1].astype(int), "rating": doc[:, 2]})
    dsrc = BatchOperator.fromDataframe(ddf, schemaStr="user bigint, item bigint, rating double")
    dm = AlsTrainBatchOp().setUserCol("user").setItemCol("item").setRateCol("rating").setNumIter(10).setRank(10) \
        .setLambda(0.01).linkFrom(dsrc)
    pred = AlsPredictBatchOp().setUserCol("user").setItemCol("item").setPredictionCol("p").linkFrom(dm, dsrc)
    out["doc_pred"] = sorted((int(r[0]), int(r[1]), float(r[3])) for r in pred.collect())
    out["backend"] = comm._backend()
    out["device"] = str(env.device)
    out["comm_calls"] = comm.STATS.calls


def scenario_tree_cat_gbdt(out):
    """Categorical GBDT, feature-sharded over the ranks sharing the GPU (tests/dist_helpers._tree_cat)."""
    from dist_helpers import _tree_cat
    _tree_cat(out, "gbdt")


def scenario_tree_cat_gini(out):
    """Parallel-mode RF (gini, categorical features), feature-sharded on the GPU."""
    from dist_helpers import _tree_cat
    _tree_cat(out, "gini")


def scenario_gbdt(out):
    """GBDT with 160 continuous features on the GPU: the feature-sharded histogram (fixed-point kernel over this
    rank's 32-feature pieces) and the pipelined asynchronous reduce-scatter with device tensors."""
    import numpy as np
    import pandas as pd
    from alink_amd import useLocalEnv, BatchOperator, GbdtTrainBatchOp
    from alink_amd.models.tree.engine import TreeBuilder
    from alink_amd.parallel import comm
    rng = np.random.default_rng(21)
    X = rng.normal(size=(20000, 160))
    w = rng.normal(size=160) * (rng.random(160) < 0.2)
    y = (X @ w + 0.3 * rng.normal(size=20000) > 0).astype(int)
    df = pd.DataFrame({f"x{i}": X[:, i] for i in range(160)})
    df["y"] = y
    env = useLocalEnv(1)
    src = BatchOperator.fromDataframe(df, schemaStr=", ".join(f"x{i} double" for i in range(160)) + ", y int")
    before = TreeBuilder.SHARDED_SEARCHES
    nrs = TreeBuilder.RS_CALLS
    m = GbdtTrainBatchOp().setFeatureCols([f"x{i}" for i in range(160)]).setLabelCol("y").setNumTrees(3) \
        .setMinSamplesPerLeaf(10).setMaxDepth(5).linkFrom(src)
    out["model"] = [list(r) for r in m.collect()]
    out["sharded"] = TreeBuilder.SHARDED_SEARCHES - before
    out["rs_calls"] = TreeBuilder.RS_CALLS - nrs
    out["backend"] = comm._backend()
    out["device"] = str(env.device)


def scenario_ftrl_hogwild(out):
    """FTRL updateMode HOGWILD over P ranks sharing the GPU: local Hogwild kernel + all-reduced (dn, dz)."""
    _ftrl_mode(out, "HOGWILD")


def scenario_ftrl_sharded(out):
    """FTRL updateMode SHARDED over P ranks sharing the GPU: SplitVector all-to-all of device CSR entries,
    partial-margin HIP kernel, margin all-reduce, per-coordinate replay kernel on each rank's range."""
    _ftrl_mode(out, "SHARDED")


def scenario_ftrl_dp_async(out):
    """FTRL DATA_PARALLEL with asyncGradReduce: the (sum g, sum g^2) all-reduce runs on the comm stream while the
    next micro-batch scores."""
    _ftrl_mode(out, "DATA_PARALLEL", async_reduce=True)


def _ftrl_mode(out, mode, async_reduce=False):
    import numpy as np
    import pandas as pd
    from alink_amd import (useLocalEnv, BatchOperator, StreamOperator, LogisticRegressionTrainBatchOp,
                           FtrlTrainStreamOp, CollectStreamOp)
    from alink_amd.parallel import comm
    os.environ["ALINK_STREAM_BATCH"] = "64"
    env = useLocalEnv(1)
    rng = np.random.default_rng(5)
    X = rng.normal(size=(2000, 6))
    wt = np.array([1.0, -1.0, 0.5, 0.2, -0.7, 0.0])
    df = pd.DataFrame({f"f{i}": X[:, i] for i in range(6)})
    df["label"] = (X @ wt + 0.3 * rng.normal(size=2000) > 0).astype(int)
    schema = ", ".join(f"f{i} double" for i in range(6)) + ", label int"
    cols = [f"f{i}" for i in range(6)]
    model = LogisticRegressionTrainBatchOp().setFeatureCols(cols).setLabelCol("label").setMaxIter(2) \
        .linkFrom(BatchOperator.fromDataframe(df.iloc[:50], schemaStr=schema))
    snaps = []
    op = FtrlTrainStreamOp(model).setFeatureCols(cols).setLabelCol("label").setTimeInterval(1e9) \
        .setUpdateMode(mode).setAlpha(0.1).setBeta(1.0)
    if async_reduce:
        op.set("asyncGradReduce", True)
    op.linkFrom(StreamOperator.fromDataframe(df, schemaStr=schema)).link(CollectStreamOp(snaps))
    StreamOperator.execute()
    last = max(r[0] for r in snaps)
    coef = [r for r in snaps if r[0] == last and r[2] == 1048576][0][3]
    w = np.asarray(json.loads(coef)["coefVector"]["data"])
    out["coef"] = w.tolist()
    m = X @ w[1:] + w[0] if w.size == 7 else X @ w[:6]
    y = df["label"].to_numpy()
    out["acc"] = float(((m > 0).astype(int) == y).mean())
    out["backend"] = comm._backend()
    out["device"] = str(env.device)


def _ftrl_pipeline(out, mode):
    """The BASELINE config-5 StreamOp pipeline at test size (tools/ftrl_pipeline_bench.py): every rank streams
    its block of one synthetic click log -> FeatureHasher -> FtrlTrainStreamOp (``mode``) -> FtrlPredictStreamOp
    -> EvalBinaryClassStreamOp; the final cumulative metrics and the last snapshot's coefficients."""
    import json as _json
    import numpy as np
    from alink_amd import (useLocalEnv, FeatureHasherBatchOp, LogisticRegressionTrainBatchOp, FtrlTrainStreamOp,
                           FtrlPredictStreamOp, EvalBinaryClassStreamOp, FeatureHasherStreamOp, StreamOperator,
                           CollectStreamOp)
    from alink_amd.operator.batch.source import TableSourceBatchOp
    from alink_amd.operator.stream.source import TableSourceStreamOp
    from alink_amd.parallel import comm
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from ftrl_pipeline_bench import click_table
    os.environ["ALINK_STREAM_BATCH"] = os.environ.get("ALINK_TEST_BATCH", "4096")
    env = useLocalEnv(1)
    fields = [f"C{f + 1}" for f in range(8)]
    full = click_table(20_000 + 122_880, 8, 500, env.device, seed=7)
    init_tab = full.slice(0, 20_000)
    ws, me = comm.get_world_size(), comm.get_rank()
    # rank r streams the r-th micro-batch of every group of ws consecutive ones: global step t of P ranks then holds
    # exactly the rows one rank streams at P x the micro-batch (rank order == row order)
    import torch
    mb = int(os.environ["ALINK_STREAM_BATCH"])
    rows = torch.arange(122_880).view(-1, mb)[me::ws].reshape(-1) + 20_000
    part = full.take(rows)

    def hasher(cls):
        return cls().setSelectedCols(fields).setCategoricalCols(fields).setOutputCol("vec").setNumFeatures(20000) \
            .setReservedCols(["label"])
    init_vec = hasher(FeatureHasherBatchOp).linkFrom(TableSourceBatchOp(init_tab))
    # the warm start model is trained on the replicated first rows (identical on every rank)
    init_vec.getOutputTable().replicated = True
    init_model = LogisticRegressionTrainBatchOp().setVectorCol("vec").setLabelCol("label").setMaxIter(10) \
        .linkFrom(init_vec)
    hashed = hasher(FeatureHasherStreamOp).linkFrom(TableSourceStreamOp(part))
    # a snapshot every micro-batch: the predictor serves the model of the previous step (prequential evaluation)
    train = FtrlTrainStreamOp(init_model).setVectorCol("vec").setLabelCol("label").setTimeInterval(0.0) \
        .setAlpha(0.1).setBeta(0.1).setL1(0.01).setL2(0.01).setUpdateMode(mode).linkFrom(hashed)
    snaps = []
    train.link(CollectStreamOp(snaps))
    pred = FtrlPredictStreamOp(init_model).setVectorCol("vec").setPredictionCol("pred") \
        .setPredictionDetailCol("detail").setReservedCols(["label"]).linkFrom(train, hashed)
    box = []
    EvalBinaryClassStreamOp().setLabelCol("label").setPredictionDetailCol("detail").linkFrom(pred) \
        .link(CollectStreamOp(box))
    StreamOperator.execute()
    last = _json.loads([r for r in box if r[0] == "all"][-1][1])
    out["auc"] = float(last["AUC"])
    out["logloss"] = float(last["LogLoss"])
    out["total"] = int(last["TotalSamples"])
    from alink_amd.models.linear.model import LinearModelDataConverter
    lb = max(r[0] for r in snaps)
    m = LinearModelDataConverter().load([tuple(r[2:]) for r in snaps if r[0] == lb])
    out["coef_head"] = np.asarray(m.coefVector.data)[:50].tolist()
    out["backend"] = comm._backend()
    out["device"] = str(env.device)


def scenario_ftrl_pipeline_sharded(out):
    _ftrl_pipeline(out, "SHARDED")


def scenario_ftrl_pipeline_dp(out):
    _ftrl_pipeline(out, "DATA_PARALLEL")


def scenario_cross_gpu(out):
    """Ring blockwise top-K with device query / item blocks (the top-K merge kernel on the GPU)."""
    import torch
    from alink_amd.parallel import comm
    from alink_amd.parallel.cross import blockwise_topk
    comm.init_distributed()
    ws, me = comm.get_world_size(), comm.get_rank()
    g = torch.Generator().manual_seed(3)
    Q = torch.randn(300, 16, generator=g)
    T = torch.randn(5000, 16, generator=g)
    qb = [round(i * 300 / ws) for i in range(ws + 1)]
    ib = [0] + sorted(int(x) for x in torch.randint(1, 5000, (ws - 1,), generator=g).tolist()) + [5000]
    dev = comm.device_for_rank()
    v, i = blockwise_topk(Q[qb[me]:qb[me + 1]].to(dev), T[ib[me]:ib[me + 1]].to(dev), 10)
    ref_v, ref_i = torch.topk(Q[qb[me]:qb[me + 1]] @ T.T, 10, dim=1)
    out["ids_equal"] = bool(torch.equal(i.cpu(), ref_i))
    out["max_abs_diff"] = float((v.cpu() - ref_v).abs().max())
    out["on_device"] = v.is_cuda


def run(rank, world, port, scenario, outdir):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    out = {}
    try:
        globals()["scenario_" + scenario](out)
    except Exception:
        out["error"] = traceback.format_exc()
    with open(os.path.join(outdir, f"{scenario}_{world}_{rank}.json"), "w") as f:
        json.dump(out, f)
    from alink_amd.parallel import comm
    comm.shutdown()


if __name__ == "__main__":
    run(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5])
