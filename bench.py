#!/usr/bin/env python3
"""Headline benchmark: KMeans k=100 on 1e8 synthetic rows x 128 dims (bf16), data-parallel over N MI355X.

Metric (BASELINE.json): rows/sec/node + iterations-to-converge.  One *step* = one Lloyd superstep of the
framework's ``KMeansTrainBatchOp`` BSP queue: fused HIP assign+accumulate over this rank's rows, RCCL
all-reduce of the [k, d+1] sums, centroid update and the convergence criterion.  The 1e8-row table is fixed
(strong scaling: each of N ranks holds 1e8/N rows, generated on its own GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R] [--k 100] [--dims 128]
    torchrun --nproc-per-node N bench.py --gpus N ...

``--gpus N`` without a launcher around it starts the N ranks itself (``alink_amd/parallel/launch.py``: N
child processes with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, started before this process touches the
GPU; rank 0's JSON line is the job's output; a failing or hung rank fails the job).

Prints ONE JSON line on rank 0.  ``value`` = total rows processed per second by the whole job
(rows x K / max-over-ranks elapsed).  Also reports ``iters_to_converge`` from a separate untimed run with
epsilon 1e-4 at the reference defaults (k-means|| initSteps=2 and the reference's sampled k-means++ seeding over
the candidates, ``convergence.reference``), plus the opt-in greedy seeding (``convergence.greedy``) and
initSteps=5 for comparison; every run reports its final SSE (sum of squared distances to the nearest centroid)
and live k.  The fused update holds each bf16 centroid operand while its fp64 centroid stays within one bf16 ulp
(ops/csrc/kmeans_common.hip), so Lloyd reaches an exactly stationary assignment.

Communication fields: ``comm_backend`` (nccl = RCCL, gloo, or none for a 1-rank job), ``oneshot_used`` (the
[k, d+1] all-reduce went through the one-shot xGMI kernel), ``allreduce_us_per_step`` (device time of the
superstep's collectives, event-timed on the compute stream, i.e. including the wait for the slowest rank) and
``allreduce_calls_per_step``.  ``ALINK_COMM_FORCE_COLLECTIVE=1`` makes a 1-rank job run its collectives for
real (the RCCL path of a multi-GPU job, on one GPU).

Straggler split: ``assign_ms_per_step_{max,min}`` are the max / min over ranks of the assign+accumulate device time
per timed superstep (HIP events around the fused kernel and its slab reduction), ``assign_ms_per_step_by_rank`` the
per-rank values and ``straggler_ms_per_step`` their spread — so a multi-GPU step time splits into the slowest
rank's kernel, the wait for it (inside ``allreduce_us_per_step``) and the collective itself.

Telemetry (``--telemetry 1``, default on a GPU): an ``amdsmi`` sampling process (``alink_amd/utils/telemetry.py``)
records gfx / memory clocks, socket power and temperatures every 5 ms; ``telemetry`` holds per-phase min / median /
max (data generation, warm-up, timed window, convergence runs) and the throttle-residency deltas of rank 0, plus
every rank's timed-window medians.  ``ALINK_TELEMETRY_OUT=path`` also writes rank 0's raw series there.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

METRIC = "rows/sec/node + iters-to-converge, KMeans k=100 1e8-row×128-dim at 1/2/4/8 MI355X"


def _sse(data, op, dev) -> float:
    """Sum over all rows (all ranks) of the squared Euclidean distance to the nearest centroid of ``op``'s model
    (fp32 GEMM in 4M-row chunks, fp64 accumulation)."""
    from alink_amd.models.clustering.kmeans import KMeansModelDataConverter
    from alink_amd.parallel import comm
    md = KMeansModelDataConverter().load(op.collect())
    X = data.col("vec").values
    C = torch.as_tensor(md.centroids, dtype=torch.float32, device=X.device)
    cn = (C * C).sum(1)
    tot = torch.zeros((), dtype=torch.float64, device=X.device)
    for lo in range(0, X.shape[0], 1 << 22):
        x = X[lo:lo + (1 << 22)].to(torch.float32)
        d = (x * x).sum(1, keepdim=True) - 2.0 * (x @ C.T) + cn[None, :]
        tot += d.min(1).values.clamp_min(0).sum(dtype=torch.float64)
    t = tot.reshape(1).to(comm.collective_device())
    comm.all_reduce(t)
    return float(t.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--dims", type=int, default=128)
    ap.add_argument("--converge-iters", type=int, default=100, help="maxIter of the convergence run (0 = skip)")
    ap.add_argument("--timeout", type=float, default=1500.0, help="self-launched job time limit (s)")
    ap.add_argument("--convergence-first", type=int, default=0,
                    help="1: the untimed convergence runs before the timed run (0: after it)")
    ap.add_argument("--telemetry", type=int, default=1, help="1: sample GPU clocks / power (amdsmi) during the run")
    ap.add_argument("--kernel-timing", type=int, default=1,
                    help="1: HIP events around every assign launch in the window (per-rank kernel time fields)")
    a = ap.parse_args()

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # self-launch: this parent never initialises the GPU; each child is one rank (one MI355X)
        from alink_amd.parallel.launch import launch_script
        sys.exit(launch_script(a.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                               timeout_s=a.timeout))

    from alink_amd import useLocalEnv, KMeansTrainBatchOp, RandomVectorSourceBatchOp
    from alink_amd.parallel import comm
    from alink_amd.ops import _lib

    from alink_amd.ops import kmeans as kops
    env = useLocalEnv(1)
    if env.world_size != a.gpus:
        raise SystemExit(f"[bench] --gpus {a.gpus} but the job has WORLD_SIZE={env.world_size}")
    dev = env.device
    if dev.type == "cuda":
        _lib.require()

    tel = None
    if dev.type == "cuda" and a.telemetry:
        from alink_amd.utils.telemetry import GpuTelemetry
        # a sampler process per rank keeps the amdsmi decoding off the rank's GIL; above 4 ranks a thread, so a node
        # never carries more than 8 extra processes next to the ranks
        tel = GpuTelemetry(dev, process=comm.get_world_size() <= 4).start()

    def mark(name):
        if tel is not None:
            tel.mark(name)

    src = RandomVectorSourceBatchOp().setNumRows(a.rows).setSize(a.dims).setNumClusters(a.k) \
        .setClusterStd(1.0).setCenterScale(4.0).setDtype("bf16").setSeed(2024).setOutputCol("vec")
    t_gen = time.perf_counter()
    data = src.getOutputTable()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t_gen = time.perf_counter() - t_gen
    mark("datagen_end")

    from alink_amd.operator.batch.source import TableSourceBatchOp

    def convergence_runs():
        iters, conv = None, {}
        # ---- convergence runs (epsilon 1e-4): the reference defaults (k-means|| initSteps=2, the reference's sampled
        # k-means++ seeding over the candidates), the opt-in greedy seeding, and initSteps=5 ----
        if a.converge_iters > 0:
            for tag, steps, seeding in (("reference", 2, "reference"), ("greedy", 2, "greedy"),
                                        ("initSteps5", 5, "reference")):
                old = os.environ.get("ALINK_KMEANS_SEEDING")
                os.environ["ALINK_KMEANS_SEEDING"] = seeding
                t_c = time.perf_counter()
                op2 = KMeansTrainBatchOp().setVectorCol("vec").setK(a.k).setMaxIter(a.converge_iters) \
                    .setInitSteps(steps)
                op2.linkFrom(TableSourceBatchOp(data))
                wall = time.perf_counter() - t_c
                info = op2.getTrainInfo()
                if old is None:
                    os.environ.pop("ALINK_KMEANS_SEEDING", None)
                else:
                    os.environ["ALINK_KMEANS_SEEDING"] = old
                shift = (info["max_shift"] or [None])[-1]
                conv[tag] = {"iters": info["iterations"], "wall_s": wall, "initSteps": steps,
                             "final_max_shift": shift, "converged": shift is not None and shift < 1e-4,
                             "seeding": seeding, "live_k": int(op2._queue.final_contexts[0].getObj("k")),
                             "sse": _sse(data, op2, dev)}
            iters = conv["reference"]["iters"]

        return iters, conv

    if a.convergence_first:
        iters, conv = convergence_runs()

    # ---- timed run: W warmup supersteps + exactly K timed supersteps (no early convergence) ----
    marks = {}

    step_t = []

    def on_step(step, q):
        if a.warmup < step < a.warmup + a.steps:
            step_t.append(time.perf_counter())         # host superstep boundaries inside the window
        if step == a.warmup or step == a.warmup + a.steps:
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            comm.barrier()
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            marks[step] = time.perf_counter()
            if step == a.warmup:
                mark("window_start")
                comm.device_timing_collect()                  # drop warmup events
                kops.kernel_timing_collect()
                marks["oneshot0"] = comm.STATS.oneshot
                comm.device_timing(dev.type == "cuda")
                kops.kernel_timing(bool(a.kernel_timing))
            else:
                mark("window_end")
                comm.device_timing(False)
                kops.kernel_timing(False)

    op = KMeansTrainBatchOp().setVectorCol("vec").setK(a.k).setMaxIter(a.warmup + a.steps).setEpsilon(-1.0)
    op._on_step = on_step
    op._sync_steps = (a.warmup, a.warmup + a.steps)   # nothing queued across the timing marks
    t_tot = time.perf_counter()
    hip0 = kops.HIP_CALLS
    op.linkFrom(TableSourceBatchOp(data))
    hip_used = kops.HIP_CALLS > hip0
    t_tot = time.perf_counter() - t_tot
    if a.warmup == 0:
        raise SystemExit("--warmup must be >= 1 (the first superstep includes one-time setup)")
    elapsed = marks[a.warmup + a.steps] - marks[a.warmup]
    el = torch.tensor([elapsed], dtype=torch.float64)
    n_ev, dev_comm_s, _ = comm.device_timing_collect()
    n_kt, kern_s = kops.kernel_timing_collect()
    mark("timed_run_end")
    kern_by_rank = [float(v) for v in comm.all_gather_object(kern_s / a.steps * 1e3)]
    oneshot_calls = comm.STATS.oneshot - marks.get("oneshot0", comm.STATS.oneshot)
    comm_backend = comm._backend() if comm.is_distributed() else "none"
    el_max = el.clone()
    comm.all_reduce(el_max, "max")
    elapsed = float(el_max.item())
    cst = torch.tensor([dev_comm_s], dtype=torch.float64)
    comm.all_reduce(cst, "max")
    dev_comm_s = float(cst.item())
    stats = op._queue.stats[a.warmup:a.warmup + a.steps]
    live_k = int(op._queue.final_contexts[0].getObj("k"))
    comm_bytes = sum(s["comm_bytes"] for s in stats) / max(1, len(stats))
    timed_sse = _sse(data, op, dev)

    if not a.convergence_first:
        iters, conv = convergence_runs()
    mark("convergence_end")
    telemetry = None
    if tel is not None:
        tel.stop()
        telemetry = tel.summary()
        out_path = os.environ.get("ALINK_TELEMETRY_OUT")
        if out_path and env.rank == 0:
            with open(out_path, "w") as f:
                json.dump({"summary": telemetry, "series": tel.series(),
                           "columns": ["t_s", "gfxclk_min_mhz", "gfxclk_max_mhz", "uclk_mhz", "socket_power_w",
                                       "hotspot_c", "hbm_c"]}, f)
    if telemetry is not None and len(step_t) >= 2:
        # host-side superstep periods through the window (speculation keeps the GPU one step ahead, so these
        # follow the device within a step): the first and last fifth, to set against the clock series
        ts = [marks[a.warmup]] + step_t + [marks[a.warmup + a.steps]]
        per = [1e3 * (b - x) for x, b in zip(ts[:-1], ts[1:])]
        q5 = max(1, len(per) // 5)
        telemetry["step_ms_first_fifth"] = sum(per[:q5]) / q5
        telemetry["step_ms_last_fifth"] = sum(per[-q5:]) / q5
    win = (telemetry or {}).get("phases", {}).get("window_start->window_end", {})
    per_rank_win = comm.all_gather_object({k: v.get("median") for k, v in win.items() if isinstance(v, dict)})
    if telemetry is not None:
        telemetry["window_median_by_rank"] = per_rank_win

    rows_per_s = a.rows * a.steps / elapsed
    res = {
        "metric": METRIC,
        "value": rows_per_s,
        "unit": "rows/s",
        "n_gpus": env.world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": f"synthetic (Gaussian mixture, {a.k} components, generated on {dev.type})",
        "config": {"model": "KMeans k=100 (Lloyd, EUCLIDEAN, k-means|| init)", "global_batch": a.rows,
                   "seq_len": a.dims, "rows": a.rows, "dims": a.dims, "k": a.k,
                   "parallelism": f"dp{env.world_size}"},
        "rows_per_s_per_gpu": rows_per_s / env.world_size,
        "iters_to_converge": iters,
        "iters_to_converge_setting": "epsilon 1e-4 (max centroid shift), maxIter 100, k-means|| initSteps=2 with "
                                     "the reference's sampled k-means++ seeding over the candidates (the "
                                     "reference defaults); convergence.greedy = opt-in greedy seeding, "
                                     "convergence.initSteps5 = initSteps 5",
        "converged": conv.get("reference", {}).get("converged"),
        "convergence": conv,
        "live_k": live_k,
        "sse_timed_run": timed_sse,
        "effective_config": {"k_requested": a.k, "k_live_in_timed_run": live_k, "init": "K_MEANS_PARALLEL",
                             "initSteps_timed_run": 2, "seeding": "reference", "epsilon_timed_run": -1.0,
                             "rows_per_rank": a.rows // env.world_size, "device": str(dev)},
        "comm_backend": comm_backend,
        "oneshot_used": oneshot_calls > 0,
        "allreduce_us_per_step": dev_comm_s / a.steps * 1e6,
        "allreduce_calls_per_step": n_ev / a.steps,
        "allreduce_bytes_per_step": comm_bytes,
        "assign_ms_per_step_max": max(kern_by_rank),
        "assign_ms_per_step_min": min(kern_by_rank),
        "assign_ms_per_step_by_rank": kern_by_rank,
        "straggler_ms_per_step": max(kern_by_rank) - min(kern_by_rank),
        "assign_calls_timed": n_kt,
        "hip_kernels": bool(hip_used),
        "datagen_s": t_gen,
        "train_wall_s": t_tot,
        "telemetry": telemetry if telemetry is not None else {"available": False,
                                                              "error": "disabled" if dev.type == "cuda" else "cpu"},
    }
    if env.rank == 0:
        print(json.dumps(res), flush=True)
    comm.shutdown()


if __name__ == "__main__":
    main()
