"""Collectives between real GPU processes: P ranks (2 and 4) share the box's MI355X, exchange real
hipIpcGetMemHandle handles and reduce through the one-shot kernel (ops/csrc/allreduce.hip) — the path an 8-GPU
RCCL job uses for its small BSP buffers (KMeans [k, d+1] sums, criterion scalars)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _tree_nodes(model_rows):
    return [json.loads(r[1]) for r in model_rows[1:] if r[1] is not None and r[1].startswith('{"node"')]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(scenario, world, tmp_path, timeout=150):
    port = _free_port()
    env = dict(os.environ)
    env["ALINK_ONESHOT_ALLREDUCE"] = "1"          # gloo host group + device tensors: force the one-shot path
    env["ALINK_ONESHOT_TIMEOUT_S"] = "30"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "mp_gpu_helpers.py"), str(r), str(world),
                               str(port), scenario, str(tmp_path)], env=env) for r in range(world)]
    try:
        for p in procs:
            p.wait(timeout=timeout)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    outs = []
    for r in range(world):
        with open(os.path.join(str(tmp_path), f"{scenario}_{world}_{r}.json")) as f:
            o = json.load(f)
        assert "error" not in o, o.get("error")
        outs.append(o)
    return outs


@pytest.mark.parametrize("world", [2, 4])
def test_oneshot_between_processes_bit_exact(tmp_path, world):
    outs = _run("oneshot", world, tmp_path)
    for o in outs:
        assert o["backend"] == "gloo" and o["instance"] and o["peers_opened"] == world - 1
        assert all(o["checks"]), o["checks"]
        assert o["oneshot_calls"] >= len(o["checks"])


def test_kmeans_multiprocess_gpu_matches_one_rank(tmp_path):
    one = _run("kmeans", 1, tmp_path)[0]
    for world in (2, 4):
        outs = _run("kmeans", world, tmp_path)
        for o in outs:
            assert o["iterations"] == one["iterations"]
            assert o["oneshot_calls"] > 0
            assert o["model"] == outs[0]["model"]            # bit-identical on every rank
        # per-rank fp32 partial sums differ from the 1-rank partition: centroids agree to rounding (a near-tie
        # row may flip between two centroids)
        a = [json.loads(r[1]) for r in one["model"] if r[0] > 0]
        b = [json.loads(r[1]) for r in outs[0]["model"] if r[0] > 0]
        assert len(a) == len(b)
        for x, y in zip(a, b):
            assert abs(x["weight"] - y["weight"]) <= max(2.0, 1e-4 * x["weight"])
            np.testing.assert_allclose(np.asarray(x["vec"]["data"]), np.asarray(y["vec"]["data"]), rtol=1e-4,
                                       atol=1e-4)


def test_gbdt_feature_sharded_multiprocess_gpu_matches_one_rank(tmp_path):
    """2 ranks on one GPU: device histograms of each rank's feature pieces, asynchronous per-piece
    reduce-scatter, and the same trees as one rank (the fixed-point histogram sums are exact, so the split
    choices cannot depend on the partitioning)."""
    one = _run("gbdt", 1, tmp_path)[0]
    two = _run("gbdt", 2, tmp_path)
    assert "cuda" in one["device"]
    assert one["sharded"] == 0 and all(o["sharded"] > 0 and o["rs_calls"] > 0 for o in two)
    assert two[0]["model"] == two[1]["model"]
    ta, tb = _tree_nodes(one["model"]), _tree_nodes(two[0]["model"])
    assert len(ta) == len(tb) and len(ta) > 3
    for a, b in zip(ta, tb):
        # exact fixed-point histograms: identical split features and thresholds on every node
        assert a["id"] == b["id"] and a.get("nextIds") == b.get("nextIds")
        assert a["node"]["featureIndex"] == b["node"]["featureIndex"]
        assert a["node"].get("continuousSplit") == b["node"].get("continuousSplit")
        np.testing.assert_allclose(a["node"]["counter"]["distributions"], b["node"]["counter"]["distributions"],
                                   rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("kind", ["gbdt", "gini"])
def test_feature_sharded_categorical_trees_multiprocess_gpu(tmp_path, kind):
    """Categorical GBDT / parallel-mode RF over 2 ranks on the GPU: feature-block reduce-scatter of the device
    histograms, K8/K10 split kernels on each rank's block, owner-side categorical bin order -> the 1-rank trees."""
    one = _run("tree_cat_" + kind, 1, tmp_path)[0]
    two = _run("tree_cat_" + kind, 2, tmp_path)
    assert one["sharded"] == 0 and all(o["sharded"] > 0 for o in two)
    assert two[0]["model"] == two[1]["model"]
    ta, tb = _tree_nodes(one["model"]), _tree_nodes(two[0]["model"])
    assert len(ta) == len(tb) and len(ta) > 3
    for a, b in zip(ta, tb):
        assert a["id"] == b["id"] and a.get("nextIds") == b.get("nextIds")
        assert a["node"]["featureIndex"] == b["node"]["featureIndex"]
        assert a["node"].get("categoricalSplit") == b["node"].get("categoricalSplit")
        assert a["node"].get("continuousSplit") == b["node"].get("continuousSplit")
    assert any(a["node"].get("categoricalSplit") for a in ta)
    assert all(o["rs_bytes"] == o["hist_bytes"] * 2 * 32 // 7 for o in two)


def test_ftrl_hogwild_multiprocess_gpu(tmp_path):
    """HOGWILD FTRL over 2 ranks on one GPU: every rank ends with the same replicated model, and it learns as
    well as the 1-rank Hogwild model (cross-rank staleness is one micro-batch)."""
    one = _run("ftrl_hogwild", 1, tmp_path)[0]
    two = _run("ftrl_hogwild", 2, tmp_path)
    assert "cuda" in one["device"]
    assert two[0]["coef"] == two[1]["coef"]
    assert one["acc"] > 0.85 and two[0]["acc"] > one["acc"] - 0.03


def test_ftrl_sharded_multiprocess_gpu(tmp_path):
    """SHARDED FTRL with device tensors over 2 ranks (SplitVector all-to-all, partial-margin and replay HIP
    kernels per coefficient range): both ranks assemble the same model and it learns as well as 1 rank (the
    ranks' micro-batches form different global steps than one rank's, so the models are not bit-equal)."""
    one = _run("ftrl_sharded", 1, tmp_path)[0]
    two = _run("ftrl_sharded", 2, tmp_path)
    assert two[0]["coef"] == two[1]["coef"]
    assert one["acc"] > 0.85 and two[0]["acc"] > one["acc"] - 0.03


def test_ftrl_dp_async_multiprocess_gpu(tmp_path):
    """DATA_PARALLEL FTRL with asyncGradReduce (the (sum g, sum g^2) all-reduce of step t in flight while step
    t+1 scores): replicated model identical on both ranks, learns as well as 1 rank.  The ranks share one GPU, so
    the job runs on gloo and the in-flight reduce is gloo's async work (device tensors staged through the host);
    the RCCL comm-stream variant of all_reduce_async is exercised by
    tests/test_comm_wrappers.py::test_comm_wrappers_rccl_one_rank_* (a 1-rank RCCL group)."""
    one = _run("ftrl_dp_async", 1, tmp_path)[0]
    two = _run("ftrl_dp_async", 2, tmp_path)
    assert two[0]["coef"] == two[1]["coef"]
    assert one["acc"] > 0.85 and two[0]["acc"] > one["acc"] - 0.03


def test_als_multiprocess_gpu_matches_one_rank(tmp_path):
    """ALS over 2 ranks sharing the GPU (device factor tensors through the all-to-all request/response exchange
    and the pipelined all-gather) == 1 rank within the solve tolerance, and the reference doc predictions."""
    one = _run("als", 1, tmp_path)[0]
    two = _run("als", 2, tmp_path)
    assert "cuda" in one["device"] and two[0]["comm_calls"] > 0
    assert two[0]["model"] == two[1]["model"]
    assert [r[:2] for r in one["model"]] == [r[:2] for r in two[0]["model"]]
    a = np.array([[float(x) for x in r[2].split()] for r in one["model"]])
    b = np.array([[float(x) for x in r[2].split()] for r in two[0]["model"]])
    np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
    ref = [0.579622, 0.766851, 0.581079, 0.574481, 0.298500, 0.382157]
    for o in [one] + two:
        np.testing.assert_allclose([p for _, _, p in o["doc_pred"]], ref, atol=1e-2)


@pytest.mark.parametrize("mode", ["sharded", "dp"])
def test_ftrl_stream_pipeline_multiprocess_gpu(tmp_path, mode, monkeypatch):
    """The config-5 StreamOp pipeline (source -> FeatureHasher -> FtrlTrain -> FtrlPredict -> EvalBinaryClass) over
    2 ranks on the GPU, each streaming 4096-row micro-batches, against 1 rank streaming 8192-row micro-batches of
    the same rows (the same global steps): every rank ends with the same model, the prequential evaluation covers
    the whole stream on every rank (all-reduced bins), and model and AUC match 1 rank."""
    monkeypatch.setenv("ALINK_TEST_BATCH", "8192")
    one = _run("ftrl_pipeline_" + mode, 1, tmp_path, timeout=240)[0]
    monkeypatch.setenv("ALINK_TEST_BATCH", "4096")
    two = _run("ftrl_pipeline_" + mode, 2, tmp_path, timeout=240)
    assert "cuda" in one["device"]
    assert two[0]["coef_head"] == two[1]["coef_head"]
    assert one["total"] == 122_880 and all(o["total"] == 122_880 for o in two)
    assert one["auc"] > 0.65 and abs(two[0]["auc"] - one["auc"]) < 0.01
    np.testing.assert_allclose(two[0]["coef_head"], one["coef_head"], rtol=1e-6, atol=1e-9)


def test_ring_topk_multiprocess_gpu(tmp_path):
    """Ring blockwise top-K with device blocks over 2 ranks == torch.topk of the full score matrix."""
    for o in _run("cross_gpu", 2, tmp_path):
        assert o["on_device"] and o["ids_equal"] and o["max_abs_diff"] < 1e-4
