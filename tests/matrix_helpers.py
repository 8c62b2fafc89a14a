"""Multi-rank correctness matrix (gloo, CPU): one launch of P processes runs EVERY scenario in sequence on one
process group, each rank writing one JSON result per scenario; ``tests/test_multirank_matrix.py`` compares the
P-rank results with the 1-rank ones.  P = 8 is where uneven splits, ranks with no rows of a class / word /
item, and world-size divisibility bite (reference harness: ``BaseComQueue.java:154-308`` runs every algorithm
at the environment's parallelism).

    python tests/matrix_helpers.py RANK WORLD PORT OUTDIR name1,name2,...
"""
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402


# ------------------------------------------------------------------------------------------------ data
def _dense(n=613, d=4, seed=7):
    """n rows (613: not a multiple of 2, 3 or 8), d features, a binary and a 3-class label."""
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d))
    df = pd.DataFrame({f"x{i}": X[:, i] for i in range(d)})
    s = X @ np.linspace(1.0, -1.0, d) + 0.3 * rng.normal(size=n)
    df["y"] = (s > 0).astype(int)
    df["c3"] = np.digitize(s, [-0.7, 0.7])
    df["vec"] = [" ".join(f"{v:.6f}" for v in row) for row in X]
    return df


DENSE_SCHEMA = "x0 double, x1 double, x2 double, x3 double, y int, c3 int, vec string"
FEATS = ["x0", "x1", "x2", "x3"]


def _src(df=None, schema=DENSE_SCHEMA):
    from alink_amd import BatchOperator
    return BatchOperator.fromDataframe(_dense() if df is None else df, schemaStr=schema)


def _docs(n=301, seed=3):
    rng = np.random.default_rng(seed)
    vocab = [f"w{i}" for i in range(40)]
    p = 1.0 / np.arange(1, 41)
    p /= p.sum()
    return pd.DataFrame({"id": np.arange(n),
                         "doc": [" ".join(rng.choice(vocab, size=int(rng.integers(3, 12)), p=p)) for _ in range(n)]})


def _rows(op):
    return [list(r) for r in op.collect()]


def _num(x):
    """JSON-safe nested numbers (numpy scalars / arrays to python)."""
    if isinstance(x, dict):
        return {str(k): _num(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_num(v) for v in x]
    if isinstance(x, np.ndarray):
        return _num(x.tolist())
    if isinstance(x, (np.floating, np.integer)):
        return x.item()
    return x


# ------------------------------------------------------------------------------------------------ scenarios
def s_kmeans(out):
    from alink_amd import KMeansTrainBatchOp, VectorAssemblerBatchOp
    va = VectorAssemblerBatchOp().setSelectedCols(FEATS).setOutputCol("v").linkFrom(_src())
    out["model"] = _rows(KMeansTrainBatchOp().setVectorCol("v").setK(4).setMaxIter(20).linkFrom(va))


def s_bisecting(out):
    from alink_amd import BisectingKMeansTrainBatchOp, BisectingKMeansPredictBatchOp
    src = _src()
    m = BisectingKMeansTrainBatchOp().setVectorCol("vec").setK(4).setMaxIter(10).linkFrom(src)
    out["pred"] = [r[-1] for r in BisectingKMeansPredictBatchOp().setPredictionCol("p").linkFrom(m, src).collect()]


def s_gmm(out):
    from alink_amd import GmmTrainBatchOp, GmmPredictBatchOp
    src = _src()
    m = GmmTrainBatchOp().setVectorCol("vec").setK(3).setMaxIter(8).linkFrom(src)
    out["pred"] = [r[-1] for r in GmmPredictBatchOp().setPredictionCol("p").linkFrom(m, src).collect()]


def s_lr(out):
    from alink_amd import LogisticRegressionTrainBatchOp
    m = LogisticRegressionTrainBatchOp().setFeatureCols(FEATS).setLabelCol("y").linkFrom(_src())
    out["coef"] = json.loads(m.collect()[1][1])["coefVector"]["data"]


def s_softmax(out):
    from alink_amd import SoftmaxTrainBatchOp, SoftmaxPredictBatchOp
    src = _src()
    m = SoftmaxTrainBatchOp().setFeatureCols(FEATS).setLabelCol("c3").setMaxIter(30).linkFrom(src)
    out["pred"] = [r[-1] for r in SoftmaxPredictBatchOp().setPredictionCol("p").linkFrom(m, src).collect()]


def s_mlp(out):
    from alink_amd import MultilayerPerceptronTrainBatchOp, MultilayerPerceptronPredictBatchOp
    src = _src()
    m = MultilayerPerceptronTrainBatchOp().setFeatureCols(FEATS).setLabelCol("c3").setLayers([4, 6, 3]) \
        .setMaxIter(40).linkFrom(src)
    pred = [r[-1] for r in MultilayerPerceptronPredictBatchOp().setPredictionCol("p").linkFrom(m, src).collect()]
    df = _dense()
    out["acc"] = float(np.mean(np.asarray(pred) == df["c3"].values))


def s_pca(out):
    from alink_amd import PcaTrainBatchOp, PcaPredictBatchOp
    src = _src()
    m = PcaTrainBatchOp().setK(2).setSelectedCols(FEATS).linkFrom(src)
    out["pred"] = [r[-1] for r in PcaPredictBatchOp().setPredictionCol("p").linkFrom(m, src).collect()]


def s_summarizer(out):
    from alink_amd import SummarizerBatchOp
    s = SummarizerBatchOp().setSelectedCols(FEATS).linkFrom(_src()).collectSummary()
    out["mean"] = [float(s.mean(c)) for c in FEATS]
    out["var"] = [float(s.variance(c)) for c in FEATS]
    out["min"] = [float(s.min(c)) for c in FEATS]
    out["count"] = int(s.count())


def s_correlation(out):
    from alink_amd import CorrelationBatchOp
    for m in ("PEARSON", "SPEAMAN"):
        c = CorrelationBatchOp().setSelectedCols(FEATS + ["c3"]).setMethod(m).linkFrom(_src()) \
            .collectCorrelation().getCorrelation()
        out[m] = _num(np.asarray(c))


def s_quantile(out):
    from alink_amd import QuantileDiscretizerTrainBatchOp
    df = _dense()
    df["xi"] = (df["x0"] * 3).round()          # many ties
    m = QuantileDiscretizerTrainBatchOp().setSelectedCols(["x0", "xi"]).setNumBuckets(7) \
        .linkFrom(_src(df, DENSE_SCHEMA + ", xi double"))
    out["model"] = _rows(m)


def s_naive_bayes(out):
    from alink_amd import NaiveBayesTextTrainBatchOp, VectorAssemblerBatchOp
    df = _dense()
    for c in FEATS:
        df[c] = df[c].abs().round(3)
    va = VectorAssemblerBatchOp().setSelectedCols(FEATS).setOutputCol("v").linkFrom(_src(df))
    out["model"] = _rows(NaiveBayesTextTrainBatchOp().setVectorCol("v").setLabelCol("c3").linkFrom(va))


def s_onehot_indexer(out):
    from alink_amd import OneHotTrainBatchOp, StringIndexerTrainBatchOp
    df = _dense()
    df["cat"] = [f"k{int(abs(v) * 4) % 9}" for v in df["x1"]]
    src = _src(df, DENSE_SCHEMA + ", cat string")
    out["onehot"] = _rows(OneHotTrainBatchOp().setSelectedCols(["cat", "c3"]).linkFrom(src))
    out["indexer"] = _rows(StringIndexerTrainBatchOp().setSelectedCol("cat").setStringOrderType("frequency_desc")
                           .linkFrom(src))


def s_doccount(out):
    from alink_amd import BatchOperator, DocCountVectorizerTrainBatchOp
    src = BatchOperator.fromDataframe(_docs(), schemaStr="id long, doc string")
    out["model"] = _rows(DocCountVectorizerTrainBatchOp().setSelectedCol("doc").setMinDF(2.0).linkFrom(src))
    from alink_amd import DocHashCountVectorizerTrainBatchOp
    out["hash"] = _rows(DocHashCountVectorizerTrainBatchOp().setSelectedCol("doc").setNumFeatures(64)
                        .setMinDF(2.0).linkFrom(src))


def s_word2vec(out):
    from alink_amd import BatchOperator, Word2VecTrainBatchOp
    src = BatchOperator.fromDataframe(_docs(), schemaStr="id long, doc string")
    m = Word2VecTrainBatchOp().setSelectedCol("doc").setMinCount(3).setVectorSize(8).setNumIter(2).linkFrom(src)
    out["vocab"] = [r[0] for r in m.collect()]


def s_lda(out):
    from alink_amd import BatchOperator, LdaTrainBatchOp
    src = BatchOperator.fromDataframe(_docs(), schemaStr="id long, doc string")
    for method in ("em", "online"):
        m = LdaTrainBatchOp().setSelectedCol("doc").setTopicNum(4).setMethod(method).setNumIter(6) \
            .linkFrom(src)
        out[method] = len(m.collect())


def s_fpgrowth(out):
    from alink_amd import BatchOperator, FpGrowthBatchOp
    rng = np.random.default_rng(5)
    items = [",".join(sorted(set(rng.choice(list("ABCDEFG"), size=int(rng.integers(1, 5)))))) for _ in range(211)]
    src = BatchOperator.fromDataframe(pd.DataFrame({"items": items}), schemaStr="items string")
    f = FpGrowthBatchOp().setItemsCol("items").setMinSupportPercent(0.1).setMinConfidence(0.3).linkFrom(src)
    out["patterns"] = sorted(_rows(f))
    out["rules"] = sorted(_rows(f.getSideOutput(0)))


def s_prefixspan(out):
    from alink_amd import BatchOperator, PrefixSpanBatchOp
    rng = np.random.default_rng(6)
    seqs = [";".join(",".join(sorted(set(rng.choice(list("abcde"), size=int(rng.integers(1, 3))))))
                     for _ in range(int(rng.integers(1, 4)))) for _ in range(97)]
    src = BatchOperator.fromDataframe(pd.DataFrame({"s": seqs}), schemaStr="s string")
    out["patterns"] = sorted(_rows(PrefixSpanBatchOp().setItemsCol("s").setMinSupportCount(8).linkFrom(src)))


def s_sos(out):
    from alink_amd import SosBatchOp
    df = _dense(n=157)
    df["id"] = np.arange(len(df))
    rows = SosBatchOp().setVectorCol("vec").setPredictionCol("s").setPerplexity(5.0) \
        .linkFrom(_src(df, DENSE_SCHEMA + ", id long")).collect()
    out["scores"] = sorted((int(r[-2]), float(r[-1])) for r in rows)


def s_lsh_join(out):
    from alink_amd import BatchOperator, ApproxVectorSimilarityJoinLSHBatchOp
    df = _dense(n=131)
    df["id"] = np.arange(len(df))
    src = BatchOperator.fromDataframe(df, schemaStr=DENSE_SCHEMA + ", id long")
    j = ApproxVectorSimilarityJoinLSHBatchOp().setLeftIdCol("id").setRightIdCol("id").setLeftCol("vec") \
        .setRightCol("vec").setDistanceThreshold(1.5).setOutputCol("d").linkFrom(src, src)
    out["pairs"] = sorted([int(r[0]), int(r[1]), round(float(r[2]), 9)] for r in j.collect())


def s_eval_binary(out):
    from alink_amd import LogisticRegressionTrainBatchOp, LogisticRegressionPredictBatchOp, EvalBinaryClassBatchOp
    src = _src()
    m = LogisticRegressionTrainBatchOp().setFeatureCols(FEATS).setLabelCol("y").linkFrom(src)
    p = LogisticRegressionPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d").linkFrom(m, src)
    e = EvalBinaryClassBatchOp().setLabelCol("y").setPredictionDetailCol("d").linkFrom(p).collectMetrics()
    out["m"] = {"auc": e.getAuc(), "ks": e.getKs(), "ll": e.getLogLoss(), "acc": e.getAccuracy(),
                "n": e.getTotalSamples()}


def s_gbdt_fshard(out):
    from alink_amd import GbdtTrainBatchOp
    m = GbdtTrainBatchOp().setFeatureCols(FEATS).setLabelCol("y").setNumTrees(4).setMinSamplesPerLeaf(5) \
        .setMaxDepth(4).linkFrom(_src())
    out["model"] = _rows(m)


def s_gbdt_rank(out):
    from alink_amd import GbdtRegTrainBatchOp
    df = _dense()
    df["q"] = np.arange(len(df)) % 37
    m = GbdtRegTrainBatchOp(algoType=2).setFeatureCols(FEATS).setLabelCol("c3").setGroupCol("q") \
        .setNumTrees(3).setMinSamplesPerLeaf(5).setMaxDepth(3).linkFrom(_src(df, DENSE_SCHEMA + ", q int"))
    out["model"] = _rows(m)


def s_als(out):
    from alink_amd import BatchOperator, AlsTrainBatchOp
    rng = np.random.default_rng(2)
    n = 700
    df = pd.DataFrame({"u": rng.integers(0, 40, n), "i": rng.integers(0, 25, n), "r": rng.integers(1, 6, n) * 1.0})
    src = BatchOperator.fromDataframe(df, schemaStr="u long, i long, r double")
    m = AlsTrainBatchOp().setUserCol("u").setItemCol("i").setRateCol("r").setRank(4).setNumIter(4).linkFrom(src)
    out["n"] = len(m.collect())


def s_ftrl(out):
    from alink_amd import LogisticRegressionTrainBatchOp, StreamOperator, FtrlTrainStreamOp, CollectStreamOp
    os.environ["ALINK_STREAM_BATCH"] = "37"
    df = _dense()
    schema = DENSE_SCHEMA
    init = LogisticRegressionTrainBatchOp().setFeatureCols(FEATS).setLabelCol("y").setMaxIter(2) \
        .linkFrom(_src(df.iloc[:50]))
    res = {}
    for mode in ("SHARDED", "DATA_PARALLEL"):
        snaps = []
        FtrlTrainStreamOp(init).setFeatureCols(FEATS).setLabelCol("y").setTimeInterval(1e9).setUpdateMode(mode) \
            .linkFrom(StreamOperator.fromDataframe(df, schemaStr=schema)).link(CollectStreamOp(snaps))
        StreamOperator.execute()
        last = [r for r in snaps if r[0] == max(x[0] for x in snaps)]
        res[mode] = len(last)
    out["snap_rows"] = res


SCENARIOS = {k[2:]: v for k, v in globals().items() if k.startswith("s_") and callable(v)}


def main(rank, world, port, outdir, names):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "ALINK_DEVICE": "cpu",
                       "ALINK_DIST_TIMEOUT_S": os.environ.get("ALINK_DIST_TIMEOUT_S", "240")})
    from alink_amd import useLocalEnv
    useLocalEnv(1)
    for name in names:
        out = {}
        try:
            SCENARIOS[name](out)
        except Exception:
            out["error"] = traceback.format_exc()
        with open(os.path.join(outdir, f"{name}_{world}_{rank}.json"), "w") as f:
            json.dump(_num(out), f)
    from alink_amd.parallel import comm
    comm.shutdown()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5].split(","))
