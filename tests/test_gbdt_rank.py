"""GBDT learning to rank (algoType 2 LambdaMART-NDCG, 3 LambdaMART-DCG, 4 GBRank; reference
``operator/common/tree/parallelcart/ConstructLocalBin.java:296-460``, ``BaseGbdtTrainBatchOp.java:63-66,245-252``).

The oracle is a direct transcription of the reference's ranking branch in numpy with Java's float / double
semantics spelled out (float accumulators, float prediction differences, the float discount table)."""
import math

import numpy as np
import pytest
import torch


def _disc(n):
    r = np.arange(n, dtype=np.float64)
    return (np.log(2.0) / np.log(2.0 + r)).astype(np.float32)


def _reference_grad(pred, gain, offsets, algo):
    """ConstructLocalBin.java:296-430, line by line."""
    f32 = np.float32
    disc = _disc(10000)
    G = np.zeros(len(pred), np.float32)
    H = np.zeros(len(pred), np.float32)
    for q in range(len(offsets) - 1):
        b, e = int(offsets[q]), int(offsets[q + 1])
        n = e - b
        P = pred[b:e].astype(np.float32)
        Y = gain[b:e].astype(np.float32)
        by_label = sorted(range(n), key=lambda i: -float(Y[i]))          # stable, descending
        max_dcg = 0.0
        for r in range(n):
            max_dcg += float(f32(disc[r] * Y[by_label[r]]))
        inv = 1.0 / max_dcg if max_dcg != 0 else math.inf
        by_pred = sorted(range(n), key=lambda i: -float(P[i]))
        rank = [0] * n
        for r, i in enumerate(by_pred):
            rank[i] = r
        best, worst = float(P[by_pred[0]]), float(P[by_pred[-1]])
        g = np.zeros(n, np.float32)
        h = np.zeros(n, np.float32)
        for i1 in range(n):
            hl, hp, hr = float(Y[i1]), P[i1], rank[i1]
            for i2 in range(n):
                if i2 == i1:
                    continue
                lp, ll, lr = P[i2], float(Y[i2]), rank[i2]
                if ll >= hl:
                    continue
                ds = float(f32(hp - lp))
                if algo == 4:
                    if ds >= 0.6:
                        continue
                    g[i1] = f32(float(g[i1]) + -(float(lp) + 0.6))
                    g[i2] = f32(float(g[i2]) + -(float(hp) - 0.6))
                    h[i1] = f32(float(h[i1]) + 1)
                    h[i2] = f32(float(h[i2]) + 1)
                    continue
                dn = (hl - ll) * float(abs(f32(disc[hr] - disc[lr])))
                if hl != ll and best != worst:
                    dn /= (float(f32(0.01)) + abs(ds))
                if algo == 2:
                    dn *= inv
                lam = 2.0 / (1.0 + math.exp(2.0 * ds))
                hes = lam * (2.0 - lam)
                lam *= -dn
                hes *= 2 * dn
                g[i1] = f32(float(g[i1]) + lam)
                g[i2] = f32(float(g[i2]) - lam)
                h[i1] = f32(float(h[i1]) + hes)
                h[i2] = f32(float(h[i2]) + hes)
        z = ((g < 1e-7) & (g > -1e-7)) | ((h < 1e-7) & (h > -1e-7))
        g[z] = 0
        h[z] = 0
        G[b:e], H[b:e] = g, h
    return G, H


def _queries(nq=12, seed=0, max_len=9, ties=True):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(1, max_len + 1, nq)
    offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    n = int(offsets[-1])
    pred = rng.normal(size=n).astype(np.float32)
    if ties:                                           # equal predictions: the stable-rank tie order matters
        m = (n - 1) // 4
        pred[0:4 * m:4] = pred[1:4 * m + 1:4]
    labels = rng.integers(0, 4, n).astype(np.float64)
    gain = (np.power(2.0, np.minimum(labels, 31)) - 1.0).astype(np.float32)
    return pred, gain, offsets


@pytest.mark.parametrize("algo", [2, 3, 4])
@pytest.mark.parametrize("seed", [0, 1])
def test_rank_gradients_match_reference_transcription(algo, seed):
    from alink_amd.ops import elementwise as ew
    pred, gain, offsets = _queries(seed=seed)
    g_ref, h_ref = _reference_grad(pred, gain, offsets, algo)
    st = ew.gbdt_rank_stats(torch.from_numpy(pred), torch.from_numpy(gain), None, torch.from_numpy(offsets), algo)
    g, h = st[:, 1].numpy(), st[:, 2].numpy()
    np.testing.assert_allclose(g, g_ref, rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(h, h_ref, rtol=2e-6, atol=1e-7)
    np.testing.assert_array_equal(st[:, 0].numpy(), (g * g).astype(np.float32))
    np.testing.assert_array_equal(st[:, 3].numpy(), np.ones(len(pred), np.float32))


def test_rank_gradients_all_equal_predictions_first_tree():
    """Before the first tree every prediction is 0: the |delta score| scaling is skipped (bestScore == worstScore)."""
    from alink_amd.ops import elementwise as ew
    _, gain, offsets = _queries(seed=3)
    pred = np.zeros(len(gain), np.float32)
    for algo in (2, 3, 4):
        g_ref, h_ref = _reference_grad(pred, gain, offsets, algo)
        st = ew.gbdt_rank_stats(torch.from_numpy(pred), torch.from_numpy(gain), None, torch.from_numpy(offsets), algo)
        np.testing.assert_allclose(st[:, 1].numpy(), g_ref, rtol=2e-6, atol=1e-7)
        np.testing.assert_allclose(st[:, 2].numpy(), h_ref, rtol=2e-6, atol=1e-7)


def _rank_frame(nq=60, per=8, seed=0):
    import pandas as pd
    rng = np.random.default_rng(seed)
    rows = []
    for q in range(nq):
        x = rng.normal(size=(per, 3))
        rel = np.clip(np.round(1.5 + x[:, 0] - 0.5 * x[:, 1] + 0.3 * rng.normal(size=per)), 0, 3)
        for i in range(per):
            rows.append((float(x[i, 0]), float(x[i, 1]), float(x[i, 2]), int(1000 + (q * 7919) % 997), float(rel[i])))
    return pd.DataFrame(rows, columns=["f0", "f1", "f2", "qid", "rel"])


def _ndcg(df, score):
    tot, cnt = 0.0, 0
    for _, g in df.assign(s=score).groupby("qid"):
        gains = 2.0 ** g["rel"].values - 1
        order = np.argsort(-g["s"].values, kind="stable")
        disc = 1.0 / np.log2(np.arange(len(g)) + 2)
        ideal = np.sort(gains)[::-1]
        if ideal.sum() > 0:
            tot += (gains[order] * disc).sum() / (ideal * disc).sum()
            cnt += 1
    return tot / cnt


@pytest.mark.parametrize("algo", [2, 3, 4])
def test_rank_training_learns_ordering_and_model_round_trips(algo):
    """Ranking GBDT trains through the public op (``algoType`` field + groupCol), the model meta carries the algo
    type, and predictions (tree sums, GbdtModelMapper.java:79) rank the queries far better than chance."""
    from alink_amd import BatchOperator, GbdtRegTrainBatchOp, GbdtRegPredictBatchOp, useLocalEnv
    useLocalEnv(1)
    df = _rank_frame()
    src = BatchOperator.fromDataframe(df, schemaStr="f0 double, f1 double, f2 double, qid int, rel double")
    op = GbdtRegTrainBatchOp(algoType=algo).setFeatureCols(["f0", "f1", "f2"]).setLabelCol("rel") \
        .setGroupCol("qid").setNumTrees(12).setMaxDepth(4).setMinSamplesPerLeaf(5).setLearningRate(0.3)
    model = op.linkFrom(src)
    meta = model.collect()[0]
    assert f'"algoType":"{algo}"' in str(meta[1]) or f'"algoType":{algo}' in str(meta[1])
    pred = GbdtRegPredictBatchOp().setPredictionCol("s").linkFrom(model, src).collectToDataframe()
    rnd = _ndcg(df, np.random.default_rng(1).normal(size=len(df)))
    got = _ndcg(df, pred["s"].values)
    assert got > rnd + 0.1, (got, rnd)


def test_rank_needs_group_col():
    from alink_amd import BatchOperator, GbdtRegTrainBatchOp, useLocalEnv
    useLocalEnv(1)
    df = _rank_frame(nq=5)
    src = BatchOperator.fromDataframe(df, schemaStr="f0 double, f1 double, f2 double, qid int, rel double")
    with pytest.raises(ValueError, match="groupCol"):
        GbdtRegTrainBatchOp(algoType=2).setFeatureCols(["f0"]).setLabelCol("rel").linkFrom(src)


def test_rank_query_rows_regrouped_stably():
    """Rows of one query become contiguous in input order whatever the input interleaving; the query offsets and
    per-row query index agree."""
    from alink_amd.common.params import Params
    from alink_amd.common.table import MTable
    from alink_amd.models.tree.train import _rank_groups
    mt = MTable.from_rows([(3, 0.0), (1, 1.0), (3, 2.0), (2, 3.0), (1, 4.0), (3, 5.0)], "q int, v double")
    out, off, qidx = _rank_groups(mt, Params().set("groupCol", "q"), torch.device("cpu"))
    assert [r[1] for r in out.rows()] == [1.0, 4.0, 3.0, 0.0, 2.0, 5.0]
    assert off.tolist() == [0, 2, 3, 6] and qidx.tolist() == [0, 0, 1, 2, 2, 2]
