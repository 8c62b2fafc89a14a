"""Self-launching SPMD jobs (parallel/launch.py): ``bench.py --gpus N`` and ``alink_amd.launch(P, fn)``
start N real ranks by themselves (gloo on CPU here, one process per MI355X on a GPU node)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _kmeans_centroids(rows, k, seed):
    """Rank body: KMeans on the synthetic mixture; returns (world size, centroids, iterations)."""
    from alink_amd import useLocalEnv, KMeansTrainBatchOp, RandomVectorSourceBatchOp
    from alink_amd.operator.batch.source import TableSourceBatchOp
    env = useLocalEnv(1, device="cpu")
    src = RandomVectorSourceBatchOp().setNumRows(rows).setSize(16).setNumClusters(k).setClusterStd(0.5) \
        .setCenterScale(4.0).setSeed(seed).setOutputCol("vec")
    op = KMeansTrainBatchOp().setVectorCol("vec").setK(k).setMaxIter(8).setEpsilon(-1.0) \
        .linkFrom(TableSourceBatchOp(src.getOutputTable()))
    C = op._queue.final_contexts[0].getObj("centroid1")[1].cpu().numpy()
    C2 = op._queue.final_contexts[0].getObj("centroid2")[1].cpu().numpy()
    return env.world_size, np.stack([C, C2]), op.getTrainInfo()["iterations"]


def _fail_on_rank1():
    from alink_amd import useLocalEnv
    env = useLocalEnv(1, device="cpu")
    if env.rank == 1:
        raise ValueError("boom")
    return env.rank


def test_launch_kmeans_agrees_across_world_sizes():
    from alink_amd import launch
    ref = launch(1, _kmeans_centroids, 6000, 5, 11)
    for p in (2, 4):
        res = launch(p, _kmeans_centroids, 6000, 5, 11, timeout_s=300)
        assert [r[0] for r in res] == [p] * p
        for r in res:
            assert r[2] == ref[0][2]
            np.testing.assert_allclose(r[1], ref[0][1], rtol=0, atol=1e-9)


def test_launch_reports_failing_rank():
    from alink_amd import launch
    with pytest.raises(RuntimeError, match="boom"):
        launch(2, _fail_on_rank1, timeout_s=120)


def _bench(n, extra=()):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env["ALINK_DEVICE"] = "cpu"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--rows", "40000", "--k", "8",
           "--steps", "2", "--warmup", "1", "--converge-iters", "0", "--timeout", "300"] + list(extra)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_self_launches_n_ranks():
    res = _bench(4)
    assert res["n_gpus"] == 4
    assert res["steps"] == 2 and res["warmup"] == 1
    assert res["config"]["parallelism"] == "dp4"
    k = res["live_k"]
    # one [k, d+1] fp64 centroid buffer per superstep (the criterion needs no collective: replicated)
    assert res["allreduce_bytes_per_step"] == k * (128 + 1) * 8
    assert res["hip_kernels"] is False           # CPU run: the torch path ran, and the JSON says so
    assert res["effective_config"]["rows_per_rank"] == 10000


def test_bench_self_launches_eight_ranks_like_the_driver():
    """The driver's 8-GPU shape of the headline bench (N=8, strong scaling), rehearsed on the CPU: 8 ranks, a row
    count that does not divide by 8, the convergence run included; every rank holds its share of the rows."""
    res = _bench(8, ["--rows", "40003", "--converge-iters", "20"])
    assert res["n_gpus"] == 8 and res["config"]["parallelism"] == "dp8"
    assert res["effective_config"]["rows_per_rank"] == 40003 // 8
    # straggler split: every rank's timed assign time, max / min / spread consistent with them
    by = res["assign_ms_per_step_by_rank"]
    assert len(by) == 8 and all(v > 0 for v in by)
    assert res["assign_ms_per_step_max"] == max(by) and res["assign_ms_per_step_min"] == min(by)
    assert abs(res["straggler_ms_per_step"] - (max(by) - min(by))) < 1e-9
    assert res["assign_calls_timed"] == res["steps"]
    assert res["telemetry"]["available"] is False
    assert res["allreduce_bytes_per_step"] == res["live_k"] * (128 + 1) * 8
    assert 1 <= res["iters_to_converge"] <= 20 and res["convergence"]["reference"]["sse"] > 0


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, ALINK_DEVICE="cpu", WORLD_SIZE="1", RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29999")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rows", "1000",
                        "--converge-iters", "0"], env=env, capture_output=True, text=True, timeout=200, cwd=ROOT)
    assert r.returncode != 0
