"""Multi-process SPMD runs on CPU (gloo, world_size 2) must agree with the single-process run.

Each rank is a separate Python process started exactly like ``torchrun`` would (RANK/WORLD_SIZE/MASTER_*
with 127.0.0.1) — the CPU stand-in for one process per MI355X over RCCL."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(scenario, world, tmp_path):
    port = _free_port()
    env = dict(os.environ)
    env["ALINK_TEST_TMP"] = str(tmp_path)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_helpers.py"), str(r), str(world), str(port),
                               scenario, str(tmp_path)], env=env) for r in range(world)]
    for p in procs:
        p.wait(timeout=300)
    outs = []
    for r in range(world):
        with open(os.path.join(str(tmp_path), f"{scenario}_{world}_{r}.json")) as f:
            o = json.load(f)
        assert "error" not in o, o.get("error")
        outs.append(o)
    return outs


def test_comqueue_pi_two_processes(tmp_path):
    outs = _run("pi", 2, tmp_path)
    rows = outs[0]["rows"]
    assert outs[1]["rows"] == rows                 # closeWith results gathered on every rank
    assert sorted(r[0] for r in rows) == [0, 1, 2, 3] and all(r[1] == 4 for r in rows)
    assert len({r[2] for r in rows}) == 1          # every task sees the all-reduced buffer
    assert abs(rows[0][2] - np.pi) < 0.05


def test_kmeans_two_processes_equal_single(tmp_path):
    one = _run("kmeans", 1, tmp_path)[0]["model"]
    two = _run("kmeans", 2, tmp_path)
    assert two[0]["model"] == two[1]["model"]
    c1 = [json.loads(r[1]) for r in one[1:]]
    c2 = [json.loads(r[1]) for r in two[0]["model"][1:]]
    assert len(c1) == len(c2)
    for a, b in zip(c1, c2):
        np.testing.assert_allclose(a["vec"]["data"], b["vec"]["data"], atol=1e-9)
        assert a["weight"] == b["weight"]


def test_logistic_regression_two_processes_equal_single(tmp_path):
    one = _run("lr", 1, tmp_path)[0]["coef"]
    two = _run("lr", 2, tmp_path)
    np.testing.assert_allclose(two[0]["coef"], two[1]["coef"], rtol=0, atol=0)
    np.testing.assert_allclose(one, two[0]["coef"], rtol=1e-6, atol=1e-8)


def _tree_nodes(model_rows):
    out = []
    for r in model_rows[1:]:
        if r[1] is None or not r[1].startswith('{"node"'):
            continue
        out.append(json.loads(r[1]))
    return out


@pytest.mark.parametrize("scenario", ["gbdt", "gbdt_wide", "rf", "rf_parallel", "rf_sampled", "gbdt_rank"])
def test_trees_two_processes_equal_single(tmp_path, scenario):
    """Histogram all-reduce over 2 ranks (gbdt, rf_parallel) and tree-parallel forests (rf, rf_sampled: each rank
    grows its own trees on the all-gathered bins) give the same trees as one rank."""
    one = _tree_nodes(_run(scenario, 1, tmp_path)[0]["model"])
    two = _run(scenario, 2, tmp_path)
    assert two[0]["model"] == two[1]["model"]
    t2 = _tree_nodes(two[0]["model"])
    assert len(one) == len(t2)
    for a, b in zip(one, t2):
        assert a["id"] == b["id"] and a.get("nextIds") == b.get("nextIds")
        assert a["node"]["featureIndex"] == b["node"]["featureIndex"]
        assert a["node"].get("continuousSplit") == pytest.approx(b["node"].get("continuousSplit"))
        np.testing.assert_allclose(a["node"]["counter"]["distributions"], b["node"]["counter"]["distributions"],
                                   rtol=1e-5, atol=1e-7)


def test_gbdt_feature_sharded_histograms_three_ranks(tmp_path):
    """GBDT over 3 ranks reduce-scatters histograms by feature block (7 features -> 32-feature blocks, the other
    ranks' blocks all padding) and grows the same trees as one rank."""
    one = _run("gbdt_wide", 1, tmp_path)[0]
    three = _run("gbdt_wide", 3, tmp_path)
    assert one["sharded"] == 0 and all(o["sharded"] > 0 for o in three)
    assert three[0]["model"] == three[1]["model"] == three[2]["model"]
    ta, tb = _tree_nodes(one["model"]), _tree_nodes(three[0]["model"])
    assert len(ta) == len(tb)
    for a, b in zip(ta, tb):
        assert a["node"]["featureIndex"] == b["node"]["featureIndex"]
        assert a["node"].get("continuousSplit") == pytest.approx(b["node"].get("continuousSplit"))
        np.testing.assert_allclose(a["node"]["counter"]["distributions"], b["node"]["counter"]["distributions"],
                                   rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("kind,world", [("gbdt", 2), ("gbdt", 3), ("gini", 2), ("infogain", 2), ("mse", 3)])
def test_feature_sharded_categorical_and_rf_criteria(tmp_path, kind, world):
    """Feature-sharded histograms + split search for categorical GBDT and the parallel-mode RF criteria (gini,
    C4.5 information gain with multi-way categorical splits, MSE): the same trees as one rank, and every rank
    reduce-scatters exactly the full (padded) histogram: it sends (P-1)/P of it and keeps its own 1/P block,
    instead of all-reducing the whole histogram."""
    one = _run("tree_cat_" + kind, 1, tmp_path)[0]
    many = _run("tree_cat_" + kind, world, tmp_path)
    assert one["sharded"] == 0 and all(o["sharded"] > 0 for o in many)
    assert all(o["model"] == many[0]["model"] for o in many)
    ta, tb = _tree_nodes(one["model"]), _tree_nodes(many[0]["model"])
    assert len(ta) == len(tb) and len(ta) > 3
    for a, b in zip(ta, tb):
        assert a["id"] == b["id"] and a.get("nextIds") == b.get("nextIds")
        assert a["node"]["featureIndex"] == b["node"]["featureIndex"]
        assert a["node"].get("categoricalSplit") == b["node"].get("categoricalSplit")
        assert a["node"].get("continuousSplit") == pytest.approx(b["node"].get("continuousSplit"))
        np.testing.assert_allclose(a["node"]["counter"]["distributions"], b["node"]["counter"]["distributions"],
                                   rtol=1e-5, atol=1e-7)
    assert any(a["node"].get("categoricalSplit") for a in ta)          # categorical splits were chosen
    F, Fb = 7, 32                                                      # 7 features -> one 32-feature block per rank
    for o in many:
        assert o["rs_bytes"] == o["hist_bytes"] * world * Fb // F


def test_gbdt_pipelined_feature_block_reduce_scatter_two_ranks(tmp_path):
    """200 features over 2 ranks: each histogram is built and reduce-scattered in 4 feature pieces (the
    reduce-scatter of piece c in flight while piece c+1 builds); the trees equal the 1-rank trees."""
    one = _run("gbdt_many", 1, tmp_path)[0]
    two = _run("gbdt_many", 2, tmp_path)
    assert one["sharded"] == 0 and all(o["sharded"] > 0 for o in two)
    assert all(o["rs_calls"] >= 4 and o["rs_calls"] % 4 == 0 for o in two)      # 4 pieces per histogram
    assert two[0]["model"] == two[1]["model"]
    ta, tb = _tree_nodes(one["model"]), _tree_nodes(two[0]["model"])
    assert len(ta) == len(tb)
    for a, b in zip(ta, tb):
        assert a["node"]["featureIndex"] == b["node"]["featureIndex"]
        assert a["node"].get("continuousSplit") == pytest.approx(b["node"].get("continuousSplit"))
        np.testing.assert_allclose(a["node"]["counter"]["distributions"], b["node"]["counter"]["distributions"],
                                   rtol=1e-5, atol=1e-7)


def test_als_two_processes_equal_single(tmp_path):
    """Owner-partitioned CSR + all-to-all shuffle + all-gathered factor rows == single-process ALS."""
    one = _run("als", 1, tmp_path)[0]["model"]
    two = _run("als", 2, tmp_path)
    assert two[0]["model"] == two[1]["model"]
    assert [r[:2] for r in one] == [r[:2] for r in two[0]["model"]]
    a = np.array([[float(x) for x in r[2].split()] for r in one])
    b = np.array([[float(x) for x in r[2].split()] for r in two[0]["model"]])
    np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("world", [1, 3])
def test_blockwise_topk_ring(tmp_path, world):
    """Item blocks rotating around the ring give every query the brute-force top-K (reference
    BlockwiseCross.findTopK), for uneven query/item blocks and both orders."""
    import torch
    outs = _run("cross", world, tmp_path)
    g = torch.Generator().manual_seed(3)
    Q = torch.randn(37, 10, generator=g)
    T = torch.randn(53, 10, generator=g)
    S = (Q @ T.T).numpy()
    for key, desc in (("desc", True), ("asc", False)):
        for o in outs:
            part = o[key]
            for r, (vals, ids) in enumerate(zip(part["v"], part["i"])):
                q = part["q0"] + r
                order = np.argsort(-S[q] if desc else S[q], kind="stable")[:7]
                np.testing.assert_allclose(vals, S[q][order], rtol=1e-5, atol=1e-5)
                assert sorted(ids) == sorted(order.tolist())


def test_glm_two_processes_equal_single(tmp_path):
    one = _run("glm", 1, tmp_path)[0]["summary"]
    two = _run("glm", 2, tmp_path)
    assert two[0]["summary"] == two[1]["summary"]
    np.testing.assert_allclose(one["coefficients"], two[0]["summary"]["coefficients"], rtol=1e-9)
    np.testing.assert_allclose(one["deviance"], two[0]["summary"]["deviance"], rtol=1e-9)


def test_isotonic_two_processes_equal_single(tmp_path):
    one = _run("isotonic", 1, tmp_path)[0]
    two = _run("isotonic", 2, tmp_path)
    assert two[0]["b"] == two[1]["b"] == one["b"]
    np.testing.assert_allclose(one["v"], two[0]["v"], rtol=1e-5, atol=1e-6)  # float32 block sums, as in the reference


def test_fm_two_processes_model_averaging(tmp_path):
    two = _run("fm", 2, tmp_path)
    assert two[0]["model"] == two[1]["model"]
    assert two[0]["acc"] > 0.8


def _coef(model_rows):
    meta = [json.loads(r[1]) for r in model_rows if r[0] == 0][0]
    data = [json.loads(r[1]) for r in model_rows if r[0] == 1048576]
    return meta, np.asarray(data[0]["coefVector"]["data"] if "coefVector" in data[0] else data[0]["data"])


@pytest.mark.parametrize("scenario", ["ftrl_seq", "ftrl_sharded"])
def test_ftrl_two_processes_equal_single(tmp_path, scenario):
    """FTRL on 2 ranks (SEQUENTIAL: replicated, all-gathered micro-batches; SHARDED: feature-sharded partial
    margins + all-reduce) equals the 1-rank model when the global micro-batch sequence is the same."""
    one = _run(scenario, 1, tmp_path)[0]
    two = _run(scenario, 2, tmp_path)
    assert two[0]["model"] == two[1]["model"]           # every rank emits the full model snapshot
    assert one["bids"] == two[0]["bids"]
    assert len(one["model"]) == len(two[0]["model"])
    for a, b in zip(one["model"], two[0]["model"]):
        assert a[0] == b[0]
        if a[1] != b[1]:
            ja, jb = json.loads(a[1]), json.loads(b[1])
            assert ja.keys() == jb.keys()
            np.testing.assert_allclose(np.asarray(ja.get("coefVector", {}).get("data", [])),
                                       np.asarray(jb.get("coefVector", {}).get("data", [])), rtol=1e-12,
                                       atol=1e-14)


@pytest.mark.parametrize("world", [2, 4])
def test_ftrl_sharded_split_vector_exchange(tmp_path, world):
    """SHARDED with the SplitVector exchange (each shard receives only the nonzeros of its coefficient range,
    ``FtrlTrainStreamOp.java:174-267``) equals the all-gather exchange on the same global steps, while every shard
    receives ~1/P of each step's nonzeros."""
    split = _run("ftrl_sharded_split", world, tmp_path)
    ag = _run("ftrl_sharded_allgather", world, tmp_path)
    for o in split[1:]:
        assert o["model"] == split[0]["model"]
    assert split[0]["bids"] == ag[0]["bids"]
    for a, b in zip(ag[0]["model"], split[0]["model"]):
        assert a[0] == b[0]
        if a[1] != b[1]:
            ja, jb = json.loads(a[1]), json.loads(b[1])
            np.testing.assert_allclose(np.asarray(ja.get("coefVector", {}).get("data", [])),
                                       np.asarray(jb.get("coefVector", {}).get("data", [])), rtol=1e-12, atol=1e-14)
    # 6 coefficients (intercept + 5 dense features): shard j owns ceil(6/P) columns and gets only those entries
    per_rank = np.asarray([o["recv_nnz"] for o in split], dtype=float)     # [P, steps]
    step_total = per_rank.sum(0)
    per = -(-6 // world)
    for r in range(world):
        owned = max(0, min(6, (r + 1) * per) - r * per)
        np.testing.assert_allclose(per_rank[r], step_total * owned / 6.0)


@pytest.mark.parametrize("world", [2, 4])
def test_ftrl_data_parallel_equal_single(tmp_path, world):
    """DATA_PARALLEL (replicated w, all-reduced mini-batch gradients): P ranks whose micro-batches form the
    same global step as one rank's batch give the same model up to summation order."""
    one = _run("ftrl_dp", 1, tmp_path)[0]
    outs = _run("ftrl_dp", world, tmp_path)
    for o in outs[1:]:
        assert o["model"] == outs[0]["model"]
    assert one["bids"] == outs[0]["bids"]
    for a, b in zip(one["model"], outs[0]["model"]):
        if a[1] != b[1]:
            ja, jb = json.loads(a[1]), json.loads(b[1])
            np.testing.assert_allclose(np.asarray(ja.get("coefVector", {}).get("data", [])),
                                       np.asarray(jb.get("coefVector", {}).get("data", [])), rtol=1e-10, atol=1e-12)


def _coefs(model):
    for r in model:
        if r[1] and "coefVector" in r[1]:
            return np.asarray(json.loads(r[1])["coefVector"]["data"])
    raise AssertionError("no coefficient row in the model")


def test_ftrl_data_parallel_async_grad_reduce(tmp_path):
    """asyncGradReduce: ranks stay identical; one global step equals the synchronous mode; many steps stay close
    to it (gradients one step stale)."""
    outs = _run("ftrl_dp_async", 2, tmp_path)
    assert outs[0]["model"] == outs[1]["model"]
    np.testing.assert_allclose(_coefs(outs[0]["one_async"]), _coefs(outs[0]["one_sync"]), rtol=1e-12, atol=1e-14)
    a, s = _coefs(outs[0]["model"]), _coefs(outs[0]["sync"])
    assert np.all(np.isfinite(a))
    assert np.corrcoef(a, s)[0, 1] > 0.95
    assert not np.allclose(a, s, rtol=1e-9, atol=1e-12)          # the overlap really changed the schedule


def test_ftrl_uneven_micro_batches_lockstep(tmp_path):
    """Rank 0 has 3 micro-batches, rank 1 has 2: the finished rank joins steps with an empty batch (no hang)."""
    one = _run("ftrl_uneven", 1, tmp_path)[0]
    two = _run("ftrl_uneven", 2, tmp_path)
    assert two[0]["model"] == two[1]["model"]
    assert two[0]["bids"] == [0, 1]
    assert len(one["model"]) == len(two[0]["model"])


def test_stream_checkpoint_lockstep_resume_two_ranks(tmp_path, monkeypatch):
    """Multi-rank stream checkpoint: every rank saves at the same micro-batch round (a consistent cut), keeps the
    last two rounds, and a restart agrees on the newest round EVERY rank holds (rank 1's newest file is deleted
    here, as if it died before writing it) — the resumed model equals an uninterrupted run."""
    monkeypatch.setenv("ALINK_TEST_PHASE", "ref")
    ref = _run("ftrl_ckpt", 2, tmp_path)
    monkeypatch.setenv("ALINK_TEST_PHASE", "crash")
    crashed = _run("ftrl_ckpt", 2, tmp_path)
    assert all("crashed" in o for o in crashed), crashed
    ck = tmp_path / "ck_run"
    r1 = sorted(ck.glob("stream_ckpt_rank1_round*.pt"), key=lambda p: int(p.stem.split("round")[1]))
    r0 = sorted(ck.glob("stream_ckpt_rank0_round*.pt"), key=lambda p: int(p.stem.split("round")[1]))
    assert len(r0) == 2 and len(r1) == 2, (r0, r1, crashed)   # the last two rounds are kept per rank
    assert [p.name.split("_round")[1] for p in r0] == [p.name.split("_round")[1] for p in r1]
    r1[-1].unlink()
    monkeypatch.setenv("ALINK_TEST_PHASE", "resume")
    resumed = _run("ftrl_ckpt", 2, tmp_path)
    assert resumed[0]["model"] == resumed[1]["model"] == ref[0]["model"], (resumed, ref)
    assert not list(ck.iterdir()) and not list((tmp_path / "ck_ref").iterdir())   # cleared after completed runs


@pytest.mark.parametrize("world", [2, 4])
def test_sql_relational_ops_partitioned_equal_single(tmp_path, world):
    """join / left join / groupBy / distinct / union / intersect / minus (hash-partitioned) and orderBy (range
    partitioned, concatenated in rank order) on P ranks equal the 1-rank results."""
    one = _run("sql", 1, tmp_path)[0]["res"]
    many = _run("sql", world, tmp_path)
    for k, ref in one.items():
        got = many[0]["res"][k]                                # collect(): partitions gathered in rank order
        assert all(o["res"][k] == got for o in many)
        if k.startswith("order"):
            assert got == ref, k
        else:
            key = lambda r: [str(x) for x in r]  # noqa: E731
            assert sorted(got, key=key) == sorted(ref, key=key), k


@pytest.mark.parametrize("world", [2, 4])
def test_string_shuffle_packed_bytes_balanced(tmp_path, world):
    """Hash shuffle of a string-keyed table: string columns move as packed UTF-8 (received as StringBlock), every
    key lands on exactly one rank, no row is lost or altered, each rank receives ~1/P of all string bytes, and
    the key hash is the same function on every rank."""
    outs = _run("shuffle_strings", world, tmp_path)
    assert all(o["is_block"] == [True, True] for o in outs)
    sent = sorted(map(json.dumps, (r for o in outs for r in o["sent_rows"])))
    recv = sorted(map(json.dumps, (r for o in outs for r in o["recv_rows"])))
    assert sent == recv
    seen = {}
    for r, o in enumerate(outs):
        for k in o["keys"]:
            assert seen.setdefault(k, r) == r                 # co-partitioned: one owner per key
    total = sum(o["string_bytes_total_local"] for o in outs)
    for o in outs:
        assert abs(o["string_bytes_recv"] - total / world) <= 0.08 * total / world, (o["string_bytes_recv"], total)
    # same key -> same hash on every rank (no per-process salt)
    assert all(o["hash_sample"] == outs[0]["hash_sample"] for o in outs)
    assert len(set(outs[0]["hash_sample"])) == len(outs[0]["hash_sample"])


@pytest.mark.parametrize("world", [2, 3])
def test_shuffle_nulls_on_some_ranks_and_mixed_key_kinds(tmp_path, world):
    """NULL masks on a subset of ranks and per-rank differing object-key kinds: the exchange completes, no row is
    lost, NULLs survive, and every key (1 and '1' hash alike as strings once any rank mixes kinds) has one owner."""
    outs = _run("shuffle_partial_nulls", world, tmp_path)
    sent = sorted(map(json.dumps, (r for o in outs for r in o["sent"])))
    recv = sorted(map(json.dumps, (r for o in outs for r in o["rows"])))
    assert sent == recv
    assert any(r[1] is None for o in outs for r in o["rows"])
    owner = {}
    for r, o in enumerate(outs):
        for k, _ in o["rows"]:
            assert owner.setdefault(k, r) == r, k


def test_gather_table_columnar_three_ranks(tmp_path):
    """gather_table (collect, sinks, tuning, pipeline save) concatenates partitions in rank order with native
    column transport: tensors + null masks, sparse blocks and packed strings; objects pickled."""
    outs = _run("gather", 3, tmp_path)
    assert all(o["rows"] == outs[0]["rows"] for o in outs)
    assert outs[0]["kinds"] == ["Tensor", "StringBlock", "SparseBlock", "list"]
    rows = outs[0]["rows"]
    assert len(rows) == 5 + 6 + 7
    assert rows[0][0] == "0.0" and rows[1][0] == "None" and rows[5][0] == "100.0"
    assert rows[2][1] == "None" and rows[5][1] == "r1-0-\u00e9"
    assert rows[17][3] == str({"k": 2, "i": 6})


def test_csv_source_byte_range_split(tmp_path):
    one = _run("csv", 1, tmp_path)[0]
    three = _run("csv", 3, tmp_path)
    assert len(one["rows"]) == 503 and one["rows"][0] == [0, "name0", 0.0]
    assert all(o["rows"] == one["rows"] for o in three)
    assert sum(o["local_rows"] for o in three) == 503 and max(o["local_rows"] for o in three) < 503


def test_eval_stream_windows_agree_across_ranks(tmp_path):
    outs = _run("eval_stream_windows", 2, tmp_path)
    a, b = outs[0]["rows"], outs[1]["rows"]
    assert [r[0] for r in a] == [r[0] for r in b]
    assert len(a) >= 4                                   # rank 1's stalls close at least one window early
    assert json.loads(a[-1][1])["TotalSamples"] == json.loads(b[-1][1])["TotalSamples"]


@pytest.mark.parametrize("phase", ["plain", "ckpt", "mixed"])
def test_eval_uneven_ranks_and_mixed_detail_kinds(tmp_path, monkeypatch, phase):
    """Binary evaluation on ranks of unequal length (the shorter rank's stream ends first and keeps joining the
    collectives with empty micro-batches), with and without a stream checkpoint, and with one rank's detail column
    columnar and the other's strings: no hang, and the final cumulative metrics equal one rank over all rows."""
    monkeypatch.setenv("ALINK_TEST_PHASE", phase)
    one = _run("eval_uneven", 1, tmp_path)[0]
    two = _run("eval_uneven", 2, tmp_path)
    assert two[0]["stream"] == two[1]["stream"]
    fin1 = json.loads([r for r in one["stream"] if r[0] == "all"][-1][1])
    fin2 = json.loads([r for r in two[0]["stream"] if r[0] == "all"][-1][1])
    assert int(fin2["TotalSamples"]) == int(fin1["TotalSamples"]) == 260
    assert float(fin2["AUC"]) == float(fin1["AUC"])
    assert abs(float(fin2["LogLoss"]) - float(fin1["LogLoss"])) < 1e-12
    assert two[0]["batch"]["total"] == two[1]["batch"]["total"] == one["batch"]["total"] == 260
    assert two[0]["batch"]["auc"] == one["batch"]["auc"]
    assert abs(two[0]["batch"]["logloss"] - one["batch"]["logloss"]) < 1e-12


@pytest.mark.parametrize("phase", ["short", "empty"])
def test_stream_ops_uneven_rank_streams_lockstep(tmp_path, monkeypatch, phase):
    """Two ranks whose streams differ in length (rank 1 ends early, or holds no rows at all) run common stream
    operators -- predictors, scaler, indexer, SQL where/select, tokenizer, KMeans over a vector assembler, the
    binary evaluation (a collective per window) and a CSV sink -- through the lockstep rounds' empty micro-batches:
    every branch equals the batch ops on the rank's own rows."""
    monkeypatch.setenv("ALINK_TEST_PHASE", phase)
    outs = _run("stream_ops_uneven", 2, tmp_path)
    for r, o in enumerate(outs):
        assert all(o["ok"].values()), (r, o["ok"])
    assert outs[0]["rows"]["lr"] == 150 and outs[1]["rows"]["lr"] == (20 if phase == "short" else 0)
    assert outs[0]["eval_windows"] == outs[1]["eval_windows"] > 0
