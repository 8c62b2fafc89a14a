"""KMeans: model data, converter, BSP training (Lloyd with k-means|| init) and batched prediction.

Reference behaviour (cited per piece):
* model format — ``KMeansModelDataConverter.java:16-33``: meta = ``ParamSummary.toParams``
  (distanceType, k, vectorSize, vectorCol, latitudeCol, longitudeCol), one JSON ``ClusterSummary``
  ``{"clusterId","weight","vec":{"data":[..]}}`` per centroid;
* superstep — ``KMeansTrainBatchOp.java:58-81``: preallocate -> assign+accumulate -> AllReduce ->
  update (drops empty clusters, ``KMeansUpdateCentroids.java:52-69``) -> task-0 criterion
  (max per-centroid shift < epsilon, ``KMeansIterTermination.java:28-44``) -> output;
  the two centroid buffers alternate by step parity;
* init — ``KMeansInitCentroids.java``: RANDOM (sample k rows) or K_MEANS_PARALLEL (k-means||: one random
  center, ``initSteps-1`` rounds sampling each point with probability ``2k*cost/sum(cost)``, weights =
  nearest-candidate counts, then weighted local k-means++ + Lloyd (``LocalKmeansFunc.java``, 30 iters));
  the k-means|| oversampling cost is the FastDistance value as in the reference, and the default weighted
  k-means++ over the candidates is the reference's rule (one candidate sampled per pick with probability
  weight x plain distance, ``LocalKmeansFunc.java:41,88``).  ``ALINK_KMEANS_SEEDING=greedy`` opts into a
  greedy k-means++ over squared distances (Arthur & Vassilvitskii), which places the seeds of well-separated
  clusters more reliably;
* predict — ``KMeansModelMapper.java:61-97``: prediction (cluster id), optional detail
  (``KMeansUtil.getProbArrayFromDistanceArray``) and distance columns.

MI355X path: rows stay on the GPU; the assign/accumulate step is the fused HIP kernel
(``ops/csrc/kmeans_v10.hip`` for bf16 rows with d = 128, ``kmeans_accum.hip`` for other bf16 shapes, see
``ops/kmeans.py``), the [k, d+1] all-reduce is the one-shot xGMI kernel (``ops/csrc/allreduce.hip``) or RCCL,
and the update/criterion is one fused HIP kernel (``kmeans_common.hip``) — no per-sample host work.
"""
from __future__ import annotations

import json
import math
import os
from typing import List, Optional

import numpy as np
import torch

from ...common.linalg import DenseVector, VectorUtil
from ...common.mapper import RichModelMapper, ModelMapper, OutputColsHelper
from ...common.model import SimpleModelDataConverter
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import TableSchema, Types
from ...params import get_enum, param
from ...parallel import comm
from ...parallel.comqueue import (AllReduce, CompareCriterionFunction, CompleteResultFunction, ComputeFunction,
                                  IterativeComQueue)
from ...ops import _lib, kmeans as kops

__all__ = ["ClusterSummary", "KMeansTrainModelData", "KMeansModelDataConverter", "KMeansPredictModelData",
           "KMeansModelMapper", "train_kmeans", "kmeans_init", "pairwise_distance"]

TRAIN_DATA = "trainData"
INIT_CENTROID = "initCentroid"
CENTROID1 = "centroid1"
CENTROID2 = "centroid2"
CENTROID_ALL_REDUCE = "centroidAllReduce"
VECTOR_SIZE = "vectorSize"
K = "k"


class ClusterSummary:
    __gson_fields__ = ("clusterId", "weight", "vec")

    def __init__(self, vec: DenseVector, clusterId: int, weight: float):
        self.vec, self.clusterId, self.weight = vec, int(clusterId), float(weight)


class KMeansTrainModelData:
    def __init__(self, centroids: List[ClusterSummary], k: int, vectorSize: int, distanceType: str,
                 vectorColName: Optional[str], latitudeColName=None, longitudeColName=None):
        self.centroids = centroids
        self.k = k
        self.vectorSize = vectorSize
        self.distanceType = distanceType
        self.vectorColName = vectorColName
        self.latitudeColName = latitudeColName
        self.longitudeColName = longitudeColName

    def to_params(self) -> Params:
        dt = get_enum("DistanceType", "HasKMeansWithHaversineDistanceType")[self.distanceType]
        p = Params()
        p.set("distanceType", dt)
        p.set("k", self.k)
        p.set("vectorSize", self.vectorSize)
        p.set("vectorCol", self.vectorColName)
        p.set("latitudeCol", self.latitudeColName)
        p.set("longitudeCol", self.longitudeColName)
        return p


class KMeansPredictModelData:
    def __init__(self, centroids: np.ndarray, ids: np.ndarray, weights: np.ndarray, params: Params):
        self.centroids = centroids  # [k, d] float64
        self.ids = ids
        self.weights = weights
        self.params = params
        self.k = int(params.get("k", int))
        self.distanceType = params.get("distanceType", str)
        self.vectorColName = params.get("vectorCol", str) if params.contains("vectorCol") else None
        self.latitudeColName = params.get("latitudeCol", str) if params.contains("latitudeCol") else None
        self.longitudeColName = params.get("longitudeCol", str) if params.contains("longitudeCol") else None


class KMeansModelDataConverter(SimpleModelDataConverter):
    def serializeModel(self, model: KMeansTrainModelData):
        from ...common.javafmt import gson_dumps
        return model.to_params(), [gson_dumps(c) for c in model.centroids]

    def deserializeModel(self, meta: Params, data: List[str]) -> KMeansPredictModelData:
        vecs, ids, ws = [], [], []
        for s in data:
            o = json.loads(s)
            if "vec" in o and o["vec"] is not None:
                v = o["vec"]["data"] if isinstance(o["vec"], dict) else o["vec"]
            else:  # legacy OldClusterSummary with "center" string (KMeansUtil.java:278-310)
                c = o.get("center")
                v = json.loads(c)["data"] if "data" in c else json.loads(c)
            vecs.append(np.asarray(v, dtype=np.float64))
            ids.append(int(o["clusterId"]))
            ws.append(float(o.get("weight", 0.0)))
        C = np.stack(vecs) if vecs else np.zeros((0, 0))
        if str(meta.get("distanceType", str)).upper() == "COSINE":
            n = np.linalg.norm(C, axis=1, keepdims=True)
            C = np.where(n > 0, C / np.where(n > 0, n, 1), C)
        return KMeansPredictModelData(C, np.asarray(ids), np.asarray(ws), meta)


# ---------------------------------------------------------------------------------------------------
# distances
# ---------------------------------------------------------------------------------------------------
def pairwise_distance(X: torch.Tensor, C: torch.Tensor, distance_type: str) -> torch.Tensor:
    """[n, k] FastDistance values (EUCLIDEAN: sqrt|x-c|^2, COSINE: 1 - x.c on normalised inputs,
    HAVERSINE: great-circle km on (lat, lon) degrees)."""
    dt = distance_type.upper()
    if dt == "COSINE":
        return 1.0 - X @ C.T
    if dt == "HAVERSINE":
        lat1 = torch.deg2rad(X[:, 0:1])
        lon1 = torch.deg2rad(X[:, 1:2])
        lat2 = torch.deg2rad(C[:, 0])[None, :]
        lon2 = torch.deg2rad(C[:, 1])[None, :]
        a = torch.sin((lat2 - lat1) / 2) ** 2 + torch.cos(lat1) * torch.cos(lat2) * torch.sin((lon2 - lon1) / 2) ** 2
        return 2 * 6371.0 * torch.asin(torch.sqrt(a.clamp(0, 1)))
    xn = (X * X).sum(1, keepdim=True)
    cn = (C * C).sum(1)[None, :]
    return torch.sqrt((xn + cn - 2.0 * (X @ C.T)).abs())


def _normalize_rows(X: torch.Tensor) -> torch.Tensor:
    n = X.norm(dim=1, keepdim=True)
    return torch.where(n > 0, X / torch.where(n > 0, n, torch.ones_like(n)), X)


# ---------------------------------------------------------------------------------------------------
# initialisation
# ---------------------------------------------------------------------------------------------------
def _seed_cost(d: torch.Tensor, dist_type: str) -> torch.Tensor:
    return d * d if dist_type.upper() == "EUCLIDEAN" else d


def _hip_nearest_ok(X: torch.Tensor, dist_type: str) -> bool:
    return dist_type.upper() == "EUCLIDEAN" and kops.nearest_supported(X) and _lib.available()


def _min_dist_to(X: torch.Tensor, C: torch.Tensor, dist_type: str, chunk=1 << 20) -> torch.Tensor:
    if _hip_nearest_ok(X, dist_type):
        if C.shape[0] == 1:      # the first k-means|| cost: one streaming pass, fp64 distances straight out
            return kops.cost1_hip(X, C[0])
        return kops.nearest_hip(X, C)[1].to(torch.float64).sqrt_()
    out = []
    Cf = C.to(torch.float32 if X.dtype in (torch.bfloat16, torch.float16) else X.dtype)
    for s in range(0, X.shape[0], chunk):
        xc = X[s:s + chunk].to(Cf.dtype)
        out.append(pairwise_distance(xc, Cf, dist_type).min(1).values.to(torch.float64))
    return torch.cat(out) if out else torch.zeros(0, dtype=torch.float64, device=X.device)


def _nearest(X: torch.Tensor, C: torch.Tensor, dist_type: str, chunk=1 << 20) -> torch.Tensor:
    if _hip_nearest_ok(X, dist_type):
        return kops.nearest_hip(X, C)[0].to(torch.int64)
    out = []
    Cf = C.to(torch.float32 if X.dtype in (torch.bfloat16, torch.float16) else X.dtype)
    for s in range(0, X.shape[0], chunk):
        xc = X[s:s + chunk].to(Cf.dtype)
        out.append(pairwise_distance(xc, Cf, dist_type).argmin(1))
    return torch.cat(out) if out else torch.zeros(0, dtype=torch.int64, device=X.device)


def _global_count(n_local: int) -> List[int]:
    t = torch.tensor([int(n_local)], dtype=torch.int64)
    return [int(v) for v in comm.all_gather_tensor(t).tolist()]


_M64 = (1 << 64) - 1


def _round_key(seed: int, rnd: int) -> int:
    key = (seed * 0x9E3779B97F4A7C15 + rnd * 0xBF58476D1CE4E5B9 + 0x94D049BB133111EB) & _M64
    return key - (1 << 64) if key >= (1 << 63) else key


def _row_uniform(first_row: int, n: int, seed: int, rnd: int, device) -> torch.Tensor:
    """Counter-based U(0,1) per *global* row index (splitmix64 of (seed, round, row)): the k-means||
    oversampling draws are the same for any world size / partitioning, so a P-rank job picks exactly
    the candidates a 1-rank job picks (the reference's per-subtask Random makes them P-dependent)."""
    key = _round_key(seed, rnd)
    z = torch.arange(first_row, first_row + n, dtype=torch.int64, device=device) * 0x2545F491 + key

    def _shr(x, k):  # logical shift right on int64
        return (x >> k) & ((1 << (64 - k)) - 1)
    z = (z ^ _shr(z, 30)) * -4658895280553007687      # 0xBF58476D1CE4E5B9 as int64
    z = (z ^ _shr(z, 27)) * -7723592293110705685      # 0x94D049BB133111EB as int64
    z = z ^ _shr(z, 31)
    return (_shr(z, 11).to(torch.float64) + 0.5) * (1.0 / (1 << 53))


def _fetch_global_rows(X: torch.Tensor, global_idx: List[int], counts: List[int]) -> torch.Tensor:
    """Rows by global index (rank-order concatenation), replicated on every rank: each rank writes the rows
    it owns into a zero [m, d] fp64 block and one SUM all-reduce (RCCL on GPU) assembles it — no pickling."""
    rank = comm.get_rank()
    offs = np.concatenate([[0], np.cumsum(counts)])
    d = max(1, int(X.shape[1])) if X.dim() == 2 else 1
    out = torch.zeros((len(global_idx), d), dtype=torch.float64, device=X.device)
    mine = [(j, g - offs[rank]) for j, g in enumerate(global_idx) if offs[rank] <= g < offs[rank + 1]]
    if mine:
        dst = torch.as_tensor([j for j, _ in mine], dtype=torch.long, device=X.device)
        src = torch.as_tensor([int(i) for _, i in mine], dtype=torch.long, device=X.device)
        out.index_copy_(0, dst, X.index_select(0, src).to(torch.float64))
    comm.all_reduce(out)
    return out


def _seed_reference_device(D: torch.Tensor, w: torch.Tensor, k: int, rng, idx0: int) -> Optional[torch.Tensor]:
    """Picks 1..k-1 of the reference seeding rule without a host round trip per pick: the k-1 uniforms are drawn
    up front (the same values, in the same order, that the per-pick ``rng.random(1)`` calls return) and every
    pick's cumulative weight x cost, scaled draw, ``searchsorted`` and cost update run as device ops.  Returns the
    [k] candidate indices, or None (rng untouched) when some pick met an all-zero total — the per-pick host loop
    then runs instead, since that case consumes the generator differently."""
    n = D.shape[0]
    state = rng.bit_generator.state
    U = torch.as_tensor(rng.random(k - 1), dtype=torch.float64, device=D.device)
    chosen = torch.empty(k, dtype=torch.int64, device=D.device)
    mintot = torch.full((1,), float("inf"), dtype=torch.float64, device=D.device)
    if D.is_cuda and n <= 4096 and _lib.available():
        # all k-1 picks in one single-workgroup launch (csrc/kmeans_nearest.hip kmeans_seed_ref_kernel)
        L = _lib.require()
        Dc, wc = D.contiguous(), w.contiguous()
        rc = L.alink_kmeans_seed_ref(Dc.data_ptr(), wc.data_ptr(), U.data_ptr(), n, k, int(idx0), chosen.data_ptr(),
                                     mintot.data_ptr(), _lib.stream_ptr(D.device))
        if rc != 0:
            raise RuntimeError(f"alink_kmeans_seed_ref failed: {rc}")
        if not float(mintot.item()) > 0:
            rng.bit_generator.state = state
            return None
        return chosen
    chosen[0] = idx0
    costs = D[idx0].clone()
    for j in range(1, k):
        cw = torch.cumsum(w * costs, 0)
        tot = cw[-1:]
        torch.minimum(mintot, tot, out=mintot)
        i = torch.searchsorted(cw, U[j - 1:j] * tot).clamp_(max=n - 1)
        chosen[j:j + 1] = i
        costs = torch.minimum(costs, D.index_select(0, i)[0])
    if not float(mintot.item()) > 0:
        rng.bit_generator.state = state
        return None
    return chosen


def _local_kmeans_kernels(samples: torch.Tensor, w: torch.Tensor, D: torch.Tensor, k: int, max_iter: int,
                          rng) -> Optional[torch.Tensor]:
    """``_local_kmeans`` (reference rule, EUCLIDEAN) as two one-workgroup launches and ONE device -> host read:
    the seeding kernel makes all k picks, the first one included (from the same ``rng.random()`` draw over the
    sequential cumulative weights), and the Lloyd kernel runs the iterations on the chip
    (``ops/kmeans.py`` ``seed_ref_hip`` / ``local_lloyd_hip``).  Only an empty cluster brings the host back in,
    to refill it from the same generator draws in ascending cluster order, as the torch loop does.  Returns None
    with ``rng`` restored when a pick met an all-zero total or an input is not finite: the caller then runs the
    torch path, which handles both."""
    state = rng.bit_generator.state
    r0 = float(rng.random())
    # the uniforms go up from pinned memory without blocking: the host queues the seeding and Lloyd kernels while
    # the weights pass is still running (a pageable copy would wait for it)
    U = torch.as_tensor(rng.random(k - 1), dtype=torch.float64).pin_memory().to(samples.device, non_blocking=True)
    chosen, mintot = kops.seed_ref_hip(D, w, U, k, idx0=-1, r0=r0)
    C, assign, status, live = kops.local_lloyd_hip(samples, w, k, chosen=chosen, max_iter=max_iter, mintot=mintot)
    st = status.cpu().tolist()
    if st[3] != 0 or not st[4] > 0:
        rng.bit_generator.state = state
        return None
    n = samples.shape[0]
    it = int(st[0])
    while True:
        changed, empty = st[1] != 0, st[2] != 0
        if empty:
            for c in np.flatnonzero(live.cpu().numpy() == 0).tolist():
                C[c] = samples[int(rng.integers(n))]
        if not changed or it >= max_iter:
            return C
        C, assign, status, live = kops.local_lloyd_hip(samples, w, k, C=C, assign=assign, max_iter=max_iter - it)
        st = status.cpu().tolist()
        it += int(st[0])


def _local_kmeans(samples: torch.Tensor, weights: torch.Tensor, k: int, dist_type: str,
                  max_iter: int = 30, seed: int = 0) -> torch.Tensor:
    """Weighted k-means++ seeding + Lloyd on the k-means|| candidate set (LocalKmeansFunc.java:36-141).

    Default (``ALINK_KMEANS_SEEDING`` unset / ``reference``): the reference's rule — one candidate per pick,
    sampled with probability proportional to weight x cost, the cost being the PLAIN distance as in
    ``LocalKmeansFunc.sampleInitialCentroids`` (``LocalKmeansFunc.java:41,88``).

    ``ALINK_KMEANS_SEEDING=greedy``: every pick takes the candidate that lowers the weighted *squared*-distance
    potential most — over ALL candidates when the set is small (<= 4096, the usual k-means|| output, O(k m^2)
    on the device), else over 2 + ln k sampled trials.

    Device-resident: the reference rule's picks (``_seed_reference_device``) and every Lloyd iteration issue no
    per-centroid or per-pick host read — one 2-flag read per Lloyd iteration (changed assignment, empty cluster);
    an empty cluster is refilled from a random candidate in ascending cluster order, as before.  On the GPU the
    cluster sums are a one-hot fp64 GEMM (run-to-run deterministic)."""
    import os
    rng = np.random.default_rng(seed)
    n = samples.shape[0]
    w = weights.to(torch.float64)
    reference_rule = os.environ.get("ALINK_KMEANS_SEEDING", "reference").lower() != "greedy"
    D = pairwise_distance(samples, samples, dist_type)                                      # [n, n]
    if (reference_rule and k > 1 and dist_type.upper() == "EUCLIDEAN" and kops.local_lloyd_ok(samples, k)
            and os.environ.get("ALINK_KMEANS_LOCAL_KERNEL", "1") != "0"):
        C = _local_kmeans_kernels(samples, w, D, k, max_iter, rng)
        if C is not None:
            return C
    if not reference_rule:
        D = _seed_cost(D, dist_type)
    trials = 1 if reference_rule else 2 + int(np.log(max(k, 2)))
    exhaustive = n <= 4096 and not reference_rule
    cum = torch.cumsum(w, 0).cpu().numpy()
    idx = int(min(np.searchsorted(cum, rng.random() * cum[-1], side="left"), n - 1))
    chosen_t = _seed_reference_device(D, w, k, rng, idx) if reference_rule and k > 1 else None
    if chosen_t is not None:
        C = samples.index_select(0, chosen_t)
    else:
        chosen = [idx]
        costs = D[idx].clone()
        for _ in range(1, k):
            if exhaustive:
                pot = (torch.minimum(costs[None, :], D) * w[None, :]).sum(1)
                pot[chosen] = float("inf")
                b = int(pot.argmin().item())
                chosen.append(b)
                costs = torch.minimum(costs, D[b])
                continue
            cw = torch.cumsum(w * costs, 0).cpu().numpy()
            tot = cw[-1]
            if tot <= 0:
                cand = rng.integers(n, size=trials)
            else:
                cand = np.minimum(np.searchsorted(cw, rng.random(trials) * tot, side="left"), n - 1)
            cand_t = torch.as_tensor(cand, device=samples.device)
            newc = torch.minimum(costs[None, :], D[cand_t])  # [trials, n]
            pot = (newc * w[None, :]).sum(1)
            b = int(pot.argmin().item())
            chosen.append(int(cand[b]))
            costs = newc[b]
        C = samples[chosen].clone()
    assign = torch.full((n,), -1, dtype=torch.int64, device=samples.device)
    for _ in range(max_iter):
        a = pairwise_distance(samples, C, dist_type).argmin(1)
        if samples.is_cuda:
            # one-hot fp64 GEMM: a fixed summation order (device index_add_ sums by atomics in any order)
            oh = (a[None, :] == torch.arange(k, device=a.device)[:, None]).to(torch.float64)
            S = oh @ (samples * w[:, None])
            cnt = oh @ w
        else:
            S = torch.zeros_like(C)
            S.index_add_(0, a, samples * w[:, None])
            cnt = torch.zeros(k, dtype=torch.float64, device=samples.device).index_add_(0, a, w)
        live = cnt > 0
        flags = torch.stack([(a != assign).any(), (~live).any()]).cpu()
        changed, any_empty = bool(flags[0]), bool(flags[1])
        assign = a
        C = torch.where(live[:, None], S / torch.where(live, cnt, torch.ones_like(cnt))[:, None], C)
        if any_empty:
            for c in np.flatnonzero(~live.cpu().numpy()).tolist():
                C[c] = samples[int(rng.integers(n))]
        if dist_type.upper() == "COSINE":
            C = _normalize_rows(C)
        if not changed:
            break
    return C


def kmeans_init(X: torch.Tensor, k: int, init_mode: str, init_steps: int, dist_type: str,
                seed: int = 0) -> torch.Tensor:
    """Initial centroids [k', d] float64 (identical on every rank)."""
    counts = _global_count(X.shape[0])
    n = int(sum(counts))
    if n == 0:
        raise ValueError("The train dataset is empty!")
    rng = np.random.default_rng(seed)
    if init_mode.upper() == "RANDOM" or n <= k:
        gidx = sorted(rng.choice(n, size=min(k, n), replace=False).tolist())
        return _fetch_global_rows(X, gidx, counts)
    # k-means||
    centers = _fetch_global_rows(X, [int(rng.integers(n))], counts)
    psum = None
    if _hip_nearest_ok(X, dist_type):
        # the first cost pass also leaves per-wave sums: the threshold's total without a second pass over cost
        cost, psum = kops.cost1_hip(X, centers[0], with_sum=True)
    else:
        cost = _min_dist_to(X, centers, dist_type)
    first_row = int(sum(counts[:comm.get_rank()]))
    rounds = max(0, init_steps - 1)
    for rnd in range(rounds):
        local = psum.sum() if psum is not None else cost.sum()
        psum = None
        tot = torch.tensor([float(local.item())], dtype=torch.float64)
        comm.all_reduce(tot)
        thre = 2.0 * k / max(float(tot.item()), 1e-300)
        if cost.is_cuda and _lib.available():
            pick = kops.par_pick_hip(cost, first_row, _round_key(seed, rnd), thre)
        else:
            u = _row_uniform(first_row, X.shape[0], seed, rnd, X.device)
            pick = torch.nonzero(u < cost * thre).reshape(-1)
        new = comm.all_gather_varlen(X[pick].to(torch.float64))   # rank order == global row order
        if new.shape[0] == 0:
            continue
        centers = torch.cat([centers, new])
        if rnd + 1 < rounds:           # the last round's costs would never be read: no pass over X for them
            cost = torch.minimum(cost, _min_dist_to(X, new, dist_type))
    if centers.shape[0] <= k:
        return centers
    if _hip_nearest_ok(X, dist_type):
        w = kops.nearest_counts_hip(X, centers).to(torch.float64)      # one pass, no per-row output
    else:
        w = torch.bincount(_nearest(X, centers, dist_type), minlength=centers.shape[0]).to(torch.float64)
    comm.all_reduce(w)
    return _local_kmeans(centers, w, k, dist_type, seed=seed)


# ---------------------------------------------------------------------------------------------------
# BSP queue items
# ---------------------------------------------------------------------------------------------------
class KMeansPreallocateCentroid(ComputeFunction):
    def calc(self, ctx):
        if ctx.getStepNo() == 1:
            C = ctx.getObj(INIT_CENTROID)
            ctx.putObj(CENTROID1, [0, C.clone()])
            ctx.putObj(CENTROID2, [0, C.clone()])
            ctx.putObj(K, C.shape[0])


class KMeansAssignCluster(ComputeFunction):
    def calc(self, ctx):
        cur = ctx.getObj(CENTROID1) if ctx.getStepNo() % 2 == 0 else ctx.getObj(CENTROID2)
        k = ctx.getObj(K)
        X = ctx.getObj(TRAIN_DATA)
        C = cur[1][:k]
        spec = ctx.getObj(SPEC_BUF)
        ctx.removeObj(SPEC_BUF)
        if spec is not None and spec[0][0] == ctx.getStepNo() and kops.key_matches(spec[0][1], C):
            ctx.putObj(CENTROID_ALL_REDUCE, spec[1])    # launched by the previous superstep's update
            return
        if X is None or X.shape[0] == 0:
            buf = torch.zeros((k, C.shape[1] + 1), dtype=torch.float64, device=C.device)
        else:
            buf = kops.assign_accumulate(X, C, reverse=kops.serpentine_reverse(ctx.getStepNo()))
        ctx.putObj(CENTROID_ALL_REDUCE, buf)


def _lib_ok() -> bool:
    return kops._lib.available()


SPEC_BUF = "speculativeAllReduceBuf"


class KMeansUpdateCentroids(ComputeFunction):
    """``speculate``: after the fused HIP update, the NEXT superstep's assign kernel is queued on the new
    centroids before the host waits for the update's 16-byte stats (empty flag, max shift), so the GPU runs
    straight through the host's criterion / engine bookkeeping.  The queued result is used only if that next
    superstep runs with exactly these centroids (no empty-cluster compaction, not converged, not the last
    step); otherwise it is dropped — results are identical either way.  ``sync_steps``: supersteps after which
    nothing may be queued ahead (a caller that times supersteps, e.g. bench.py, synchronises there).
    ``tol`` (the termination epsilon): the update kernel also leaves a device word "the next superstep will not
    use this launch" (an empty cluster, or max shift < tol) that the queued kernel reads first, returning at once —
    so neither the compaction superstep nor the run's last one pays for a pass over X nobody reads.  Its result is
    then dropped on the host by the same test.  An empty cluster is compacted on the host (k x 129 values)."""

    def __init__(self, dist_type: str, max_iter: int = 2 ** 31 - 1, sync_steps=(), speculate: bool = True,
                 tol: Optional[float] = None):
        self.dist_type = dist_type
        self.max_iter = int(max_iter)
        self.sync_steps = set(sync_steps or ())
        self.speculate = speculate
        self.tol = None if tol is None else float(tol)

    def calc(self, ctx):
        tgt = ctx.getObj(CENTROID2) if ctx.getStepNo() % 2 == 0 else ctx.getObj(CENTROID1)
        old = ctx.getObj(CENTROID1) if ctx.getStepNo() % 2 == 0 else ctx.getObj(CENTROID2)
        buf = ctx.getObj(CENTROID_ALL_REDUCE)
        d = buf.shape[1] - 1
        cnt = buf[:, d]
        prev = old[1] if old is not None and old[1] is not None else None
        if self.dist_type == "EUCLIDEAN" and kops.update_supported(buf) and \
                (_lib_ok() or not kops._lib.torch_fallback_allowed()):
            # fused HIP update: C, the shift vs prev, the empty flag and the next step's MFMA operands in one
            # launch + one 16-byte read
            step = ctx.getStepNo()
            X = ctx.getObj(TRAIN_DATA)
            spec_ok = (self.speculate and step >= 2 and step < self.max_iter and step not in self.sync_steps
                       and X is not None and X.shape[0] > 0 and kops.hip_supported(X, buf.shape[0]))
            C, read = kops.update_centroids_hip(buf, prev, deferred=True,
                                                skip_tol=self.tol if spec_ok and self.tol is not None else None)
            if spec_ok:
                ctx.putObj(SPEC_BUF, ((step + 1, kops._ckey(C)),
                                      kops.assign_accumulate_hip(X, C, reverse=kops.serpentine_reverse(step + 1),
                                                                 skip=read.skip)))
            shift, has_empty = read()
            if has_empty or (read.skip is not None and shift is not None and shift < self.tol):
                ctx.removeObj(SPEC_BUF)     # not used (compaction) / possibly skipped on the device (converged)
            if has_empty:
                # drop the empty clusters on the host (k x 129 values): the fused update's C rows are the same
                # fp64 quotients the generic path computes, and the rare path issues no torch kernel that the
                # supersteps do not already use (a first use of e.g. norm / nonzero costs a lazy code-object load,
                # ~100 ms, inside the first job's supersteps)
                # one stream sync for all three reads (async copies into pinned buffers), one H2D copy back
                kk, dd = C.shape
                use_prev = prev is not None and prev.shape[1] == dd and prev.dtype == C.dtype
                pin = C.is_cuda
                h_cnt = torch.empty(cnt.shape, dtype=cnt.dtype, pin_memory=pin)
                h_C = torch.empty(C.shape, dtype=C.dtype, pin_memory=pin)
                h_prev = torch.empty((min(prev.shape[0], kk) if use_prev else 0, dd), dtype=C.dtype, pin_memory=pin)
                h_cnt.copy_(cnt, non_blocking=pin)
                h_C.copy_(C, non_blocking=pin)
                if use_prev:
                    h_prev.copy_(prev[:h_prev.shape[0]], non_blocking=pin)
                if pin:
                    torch.cuda.current_stream(C.device).synchronize()
                cnt_h = h_cnt.numpy()
                keep = np.flatnonzero(cnt_h > 0)
                C_h = h_C.numpy()[keep]
                # the criterion's shift (first k rows of the previous centroids vs the new ones), on the host too
                shift_h = None
                if use_prev and h_prev.shape[0] >= len(keep):
                    dlt = h_prev.numpy()[:len(keep)] - C_h
                    shift_h = float(np.sqrt((dlt * dlt).sum(1)).max()) if len(keep) else None
                # the kept centroids and their weights in one pinned block -> one copy; C / weights are views of it
                kk2 = len(keep)
                h_pack = torch.empty(kk2 * dd + kk2, dtype=C.dtype, pin_memory=pin)
                hp = h_pack.numpy()
                hp[:kk2 * dd] = C_h.reshape(-1)
                hp[kk2 * dd:] = cnt_h[keep]
                pack = h_pack.to(C.device, non_blocking=pin)
                C = pack[:kk2 * dd].view(kk2, dd)
                ctx.putObj("maxShift", shift_h)
                tgt[0] = ctx.getStepNo()
                tgt[1] = C
                ctx.putObj("lastWeights", pack[kk2 * dd:].to(cnt.dtype))
                ctx.putObj(K, int(C.shape[0]))
                return
            if not has_empty:
                ctx.putObj("maxShift", shift)
                tgt[0] = ctx.getStepNo()
                tgt[1] = C
                ctx.putObj("lastWeights", cnt)
                ctx.putObj(K, int(C.shape[0]))
                return
        # ONE small D2H read per superstep: the (rare) empty-cluster flag together with the max centroid shift
        # the termination criterion needs (the criterion then reads the host float instead of syncing again)
        C = buf[:, :d] / cnt[:, None]
        if self.dist_type == "COSINE":
            C = _normalize_rows(C)
        empty_any = (cnt <= 0).any().to(C.dtype)
        shift = None
        if prev is not None and prev.shape == C.shape and self.dist_type not in ("COSINE", "HAVERSINE"):
            flag, shift = torch.stack([empty_any, (C - prev).norm(dim=1).max()]).tolist()
        else:
            flag = empty_any.item()
        empty = (cnt <= 0).nonzero().reshape(-1).tolist() if flag > 0 else []
        ctx.putObj("maxShift", None if empty else shift)
        if not empty:
            tgt[0] = ctx.getStepNo()
            tgt[1] = C
            ctx.putObj("lastWeights", cnt)
            ctx.putObj(K, int(C.shape[0]))
            return
        if empty:
            keep = torch.as_tensor([i for i in range(buf.shape[0]) if i not in set(empty)], dtype=torch.long,
                                   device=buf.device)
            buf = buf.index_select(0, keep)
            cnt = buf[:, d]
        C = buf[:, :d] / cnt[:, None]
        if self.dist_type == "COSINE":
            C = _normalize_rows(C)
        tgt[0] = ctx.getStepNo()
        tgt[1] = C
        ctx.putObj("lastWeights", cnt)
        ctx.putObj(K, int(C.shape[0]))


class KMeansIterTermination(CompareCriterionFunction):
    def __init__(self, dist_type: str, tol: float):
        self.dist_type, self.tol = dist_type, tol
        self.history = []  # max centroid movement per superstep (diagnostics / train info)

    def calc(self, ctx) -> bool:
        k = ctx.getObj(K)
        a = ctx.getObj(CENTROID1)[1][:k]
        b = ctx.getObj(CENTROID2)[1][:k]
        if a.shape != b.shape:
            return False
        pre = ctx.getObj("maxShift")          # computed with the update's single D2H read (EUCLIDEAN)
        if pre is not None and self.dist_type not in ("COSINE", "HAVERSINE"):
            self.history.append(float(pre))
            return float(pre) < self.tol
        if self.dist_type == "COSINE":
            d = 1.0 - (a * b).sum(1)
        elif self.dist_type == "HAVERSINE":
            d = torch.diagonal(pairwise_distance(a, b, "HAVERSINE"))
        else:
            d = (a - b).norm(dim=1)
        mx = float(d.max().item())
        self.history.append(mx)
        return mx < self.tol


class KMeansOutputModel(CompleteResultFunction):
    def __init__(self, dist_type, vector_col, lat_col=None, lon_col=None):
        self.dist_type, self.vector_col, self.lat_col, self.lon_col = dist_type, vector_col, lat_col, lon_col

    def calc(self, ctx):
        if ctx.getTaskId() != 0:
            return None
        c1, c2 = ctx.getObj(CENTROID1), ctx.getObj(CENTROID2)
        cur = c1 if c1[0] > c2[0] else c2
        k = ctx.getObj(K)
        C = cur[1][:k].to(torch.float64).cpu().numpy()
        w = ctx.getObj("lastWeights")
        w = w.cpu().numpy() if w is not None else np.zeros(k)
        cents = [ClusterSummary(DenseVector(C[i]), i, float(w[i]) if i < len(w) else 0.0) for i in range(k)]
        md = KMeansTrainModelData(cents, k, int(ctx.getObj(VECTOR_SIZE)), self.dist_type, self.vector_col,
                                  self.lat_col, self.lon_col)
        return KMeansModelDataConverter().save(md)


def train_kmeans(X: torch.Tensor, k: int, max_iter: int, tol: float, dist_type: str, init_mode: str,
                 init_steps: int, vector_col: Optional[str], env, lat_col=None, lon_col=None,
                 init_centroids: Optional[torch.Tensor] = None, on_step=None, seed: int = 0, sync_steps=()):
    """Run the KMeans BSP queue on this rank's rows ``X`` ([n, d] on the env device); returns
    (model rows, queue)."""
    dist_type = dist_type.upper()
    # opt-in device precision for fp64 feature matrices (VectorAssembler output): ALINK_KMEANS_INPUT=fp32 runs the
    # fp32 GEMM-assign + HIP accumulate path, =bf16 the fused bf16 MFMA kernels (a one-time cast of this rank's
    # rows; profiles/kmeans_fp32_r4.txt records the centroid deltas against fp64)
    cast = os.environ.get("ALINK_KMEANS_INPUT", "").lower()
    if cast in ("fp32", "bf16") and X.is_cuda and X.dtype == torch.float64 and dist_type == "EUCLIDEAN":
        X = X.to(torch.float32 if cast == "fp32" else torch.bfloat16).contiguous()
    if dist_type == "COSINE":
        X = _normalize_rows(X.to(torch.float64)) if X.dtype == torch.float64 else \
            _normalize_rows(X.float()).to(X.dtype)
    vs = torch.tensor([float(X.shape[1]) if X.shape[0] else 0.0], dtype=torch.float64)
    vector_size = int(comm.all_reduce(vs, "max").item())
    init = init_centroids if init_centroids is not None else kmeans_init(X, k, init_mode, init_steps, dist_type,
                                                                         seed=seed)
    init = init.to(device=X.device, dtype=torch.float64)
    q = (IterativeComQueue()
         .setMLEnvironment(env)
         .setJobName("KMeans")
         .setRowsPerStep(int(X.shape[0]))
         .initWithPartitionedData(TRAIN_DATA, X)
         .initWithBroadcastData(INIT_CENTROID, init)
         .add(KMeansPreallocateCentroid())
         .add(KMeansAssignCluster())
         .add(AllReduce(CENTROID_ALL_REDUCE))
         .add(KMeansUpdateCentroids(dist_type, max_iter, sync_steps, tol=tol))
         .setCompareCriterionOfNode0(KMeansIterTermination(dist_type, tol), replicated=True)
         .closeWith(KMeansOutputModel(dist_type, vector_col, lat_col, lon_col))
         .setMaxIter(max_iter))
    q.initWithBroadcastData(VECTOR_SIZE, vector_size)
    # VECTOR_SIZE is consumed by the output function; mirror the reference's KMEANS_STATISTICS broadcast
    if on_step is not None:
        q.addStepCallback(on_step)
    rows = q.exec()
    return rows, q


# ---------------------------------------------------------------------------------------------------
# prediction
# ---------------------------------------------------------------------------------------------------
def prob_from_distances(d: torch.Tensor) -> torch.Tensor:
    """Row-wise ``getProbArrayFromDistanceArray`` (KMeansUtil.java)."""
    k = d.shape[1]
    s = d.sum(1, keepdim=True)
    return 1.0 / (k - 1) - d / s / (k - 1)


class KMeansModelMapper(ModelMapper):
    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        p = self.params
        reserved = p.get("reservedCols") if p.contains("reservedCols") else None
        self.pred_col = p.get("predictionCol")
        self.detail_col = p.get("predictionDetailCol") if p.contains("predictionDetailCol") else None
        self.dist_col = p.get("predictionDistanceCol") if p.contains("predictionDistanceCol") else None
        names, types = [self.pred_col], [Types.LONG]
        if self.detail_col:
            names.append(self.detail_col)
            types.append(Types.STRING)
        if self.dist_col:
            names.append(self.dist_col)
            types.append(Types.DOUBLE)
        self.helper = OutputColsHelper(dataSchema, names, types, reserved)

    def loadModel(self, modelRows):
        self.model = KMeansModelDataConverter().load(modelRows)
        self.C = torch.from_numpy(self.model.centroids)

    def _input_block(self, mt: MTable):
        m = self.model
        if m.vectorColName is not None:
            c = mt.col(m.vectorColName)
            v = c.values
            if isinstance(v, torch.Tensor) and v.dim() == 2:
                return v, None
            d = self.C.shape[1]
            from ...common.linalg.block import SparseBlock
            if isinstance(v, SparseBlock):
                dense = v.to_dense(torch.float64)
                if dense.shape[1] >= d:
                    dense = dense[:, :d]        # indices past the model's size are ignored, as the per-row path
                else:
                    dense = torch.cat([dense, dense.new_zeros((dense.shape[0], d - dense.shape[1]))], 1)
                nl = c.nulls.cpu().tolist() if c.nulls is not None else None
                return dense, nl
            vals = c.to_list()
            if vals and all(isinstance(x, str) and "$" not in x and ":" not in x for x in vals):
                # dense vector strings ("1.0 2.0 ..."): the C++ parser, no per-row Python vectors
                from ... import _native
                arr = _native.parse_dense_vectors(vals, d)
                if arr is not None:
                    return torch.from_numpy(arr), None
            vecs = [VectorUtil.getVector(x) for x in vals]
            nulls = [x is None for x in vecs]
            arr = np.zeros((len(vecs), d))
            for i, x in enumerate(vecs):
                if x is None:
                    continue
                if hasattr(x, "indices"):
                    sel = x.indices < d
                    arr[i, x.indices[sel]] = x.values[sel]
                else:
                    arr[i, :min(d, x.size())] = x.data[:d]
            return torch.from_numpy(arr), nulls
        lat = mt.col(m.latitudeColName).to_list()
        lon = mt.col(m.longitudeColName).to_list()
        return torch.tensor(np.stack([np.asarray(lat, float), np.asarray(lon, float)], 1)), None

    def _map_columns(self, mt: MTable):
        X, nulls = self._input_block(mt)
        dev = X.device
        dt = self.model.distanceType.upper()
        if X.dtype in (torch.bfloat16, torch.float16) and dt == "EUCLIDEAN" and X.is_cuda:
            C = self.C.to(dev)
            idx, d2 = kops.assign(X, C)
            dist_all = None
            if self.detail_col:
                dist_all = torch.cat([pairwise_distance(X[s:s + (1 << 20)].float(), C.float(), dt).double()
                                      for s in range(0, X.shape[0], 1 << 20)])
            best = d2.sqrt()
        else:
            Xf = X.to(torch.float64)
            if dt == "COSINE":
                Xf = _normalize_rows(Xf)
            C = self.C.to(Xf.device)
            dist_all = pairwise_distance(Xf, C, dt)
            best, idx = dist_all.min(1)
        ids = torch.as_tensor(self.model.ids, device=idx.device)[idx]
        outs = [Column(ids.to(torch.int64).cpu())]
        if nulls is not None and any(nulls):
            outs[0] = Column.from_values([None if nl else int(v) for v, nl in zip(outs[0].to_list(), nulls)],
                                         Types.LONG)
        if self.detail_col:
            probs = prob_from_distances(dist_all).cpu().numpy()
            full = np.zeros_like(probs)
            full[:, self.model.ids] = probs          # cluster-id order, as the per-row DenseVector was
            from ... import _native
            r = _native.java_double_rows_packed(full, " ") if len(full) else None
            if r is not None:
                # left packed as a StringBlock; null rows emptied
                from ...common.strings import StringBlock
                b, o = np.asarray(r[0], dtype=np.uint8), r[1]
                nm = None
                if nulls is not None and any(nulls):
                    nm = np.asarray(nulls, dtype=bool)
                    lens = o[1:] - o[:-1]
                    b = b[np.repeat(~nm, lens)]
                    o = np.zeros_like(o)
                    np.cumsum(np.where(nm, 0, lens), out=o[1:])
                    nm = torch.from_numpy(nm)
                outs.append(Column(StringBlock(torch.from_numpy(np.ascontiguousarray(b)), torch.from_numpy(o), nm)))
            else:
                det = [VectorUtil.toString(DenseVector(r)) for r in full]
                if nulls is not None and any(nulls):
                    det = [None if nl else s_ for s_, nl in zip(det, nulls)]
                outs.append(Column(det))
        if self.dist_col:
            bd = best.to(torch.float64).cpu()
            if nulls is not None and any(nulls):
                outs.append(Column.from_values([None if nl else float(v) for v, nl in zip(bd.tolist(), nulls)],
                                               Types.DOUBLE))
            else:
                outs.append(Column(bd))
        return outs
