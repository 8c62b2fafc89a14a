"""Online learning: FTRL-proximal logistic regression on a stream (reference
``A/operator/stream/onlinelearning/{FtrlTrainStreamOp,FtrlPredictStreamOp}.java``).

``FtrlTrainStreamOp(initModel)`` warm-starts from a batch-trained linear model (collected once, as the
reference's ``DirectReader``), updates the coefficients per micro-batch in one of four ``updateMode``s (see the
class docstring: SEQUENTIAL = the reference's sample-by-sample rule in the native C++ loop
``_native/csrc/ftrl.cpp``; SHARDED = the reference's feature-sharded design with HIP partial-margin / replay
kernels; DATA_PARALLEL = replicated mini-batch FTRL with an (optionally asynchronous) RCCL gradient all-reduce;
HOGWILD = one GPU wave per sample) and emits a model snapshot at the first step, every ``timeInterval`` seconds
and when the stream ends.  Snapshot rows are ``(bid, ntab, model_id, model_info, label_value)``: ``bid`` =
snapshot number, ``ntab`` = rows per snapshot.  ``FtrlPredictStreamOp(initModel).linkFrom(models, data)``
re-assembles snapshots and hot-swaps the ``LinearModelMapper`` between micro-batches; a snapshot produced in
the same process also carries its coefficient vector, so the hot swap skips re-parsing the JSON rows.

Per step the ranks agree on liveness, snapshot due-ness and per-rank sample counts with one host-group
all-gather (``comm.host_all_gather``: never a device copy or a GPU-stream sync under RCCL).

Deviation: the reference scales each gradient by ``1/sqrt(ms between the forward and the feedback pass)``
(``FtrlTrainStreamOp.java:428``), a wall-clock artefact of its Flink feedback loop; here the scale is 1.
Multi-rank: see ``FtrlTrainStreamOp`` (replicated SEQUENTIAL, feature-sharded SHARDED).
"""
from __future__ import annotations

import os
import time
from typing import List, Optional

import numpy as np

from ... import _native
from ...common.linalg import DenseVector
from ...common.params import ParamInfo, Params
from ...common.table import MTable
from ...common.types import TableSchema, Types
from ...models.common.features import extract_features
from ...models.linear.model import LinearModelDataConverter, LinearModelMapper
from ...parallel import comm
from .base import StreamOperator, _register_upstream_sources

__all__ = ["FtrlTrainStreamOp", "FtrlPredictStreamOp"]


def _pget(p: Params, name, default=None):
    try:
        if p.contains(name):
            v = p.get(name)
            return default if v is None else v
    except KeyError:
        pass
    return default


def _model_rows(op):
    """Warm-start model through DirectReader (reference FtrlTrainStreamOp reads its init model with
    ``DirectReader.collect`` / ``directRead``)."""
    from ...common.directreader import DirectReader
    return DirectReader.collect(op).readTable()


def _ftrl_python(indptr, indices, values, label, w, n, z, alpha, beta, l1, l2):
    for r in range(len(indptr) - 1):
        s, e = indptr[r], indptr[r + 1]
        idx, val = indices[s:e], values[s:e]
        p = 1.0 / (1.0 + np.exp(-float(np.dot(val, w[idx]))))
        for i, x in zip(idx, val):
            g = (p - label[r]) * x
            sigma = (np.sqrt(n[i] + g * g) - np.sqrt(n[i])) / alpha
            z[i] += g - sigma * w[i]
            n[i] += g * g
            w[i] = 0.0 if abs(z[i]) <= l1 else (np.sign(z[i]) * l1 - z[i]) / (beta + np.sqrt(n[i]) / alpha + l2)


class FtrlTrainStreamOp(StreamOperator):
    """Online FTRL-proximal logistic regression (``FtrlTrainStreamOp.java``).

    ``updateMode``:

    * ``SEQUENTIAL`` (default): sample-by-sample rule in stream order (native host loop), every margin on the
      latest weights — the same model on every device, so a job trains identically on CPU and GPU.  With P ranks every
      step all-gathers the ranks' micro-batches (rank order) and every rank applies the identical update to a
      replicated coefficient vector, so the model equals the 1-rank model on the same global batch sequence.
    * ``SHARDED``: the reference's distributed design (``FtrlTrainStreamOp.java:72-85`` split info,
      ``:174-267`` SplitVector, ``:396-420`` partial margins, ``:488-567`` keyed reduce + feedback) at micro-batch
      granularity: rank r owns the coefficient range [lo_r, hi_r).  Per step every rank splits its OWN samples by
      coefficient range and sends shard j only the entries in j's range (one all-to-all: each rank receives
      ~1/P of the global batch's nonzeros); each shard computes partial margins of the global batch on its range
      (HIP kernel on GPU), the margins are summed per sample (all-reduce), and each shard replays its
      coordinates in global sample order with the margins of the step start — the reference's feedback
      staleness bounded to one micro-batch.  Deterministic and independent of the number of ranks.  Its
      step-start margins are the reference's own kind of staleness (a sample's margin is computed on arrival,
      ``FtrlTrainStreamOp.java:396-420``, and the coefficients updated when the reduced margin comes back through
      the feedback edge, ``:424-480``), so its model differs from SEQUENTIAL's (by ~0.2 in a coefficient on the
      6-feature stream of tests/test_ftrl_gpu.py).
    * ``AUTO`` (opt-in): ``SHARDED`` when the environment's device is a GPU, else ``SEQUENTIAL`` — the GPU
      throughput path (profiles/ftrl_r5.txt), whose model then depends on the device.
    * ``DATA_PARALLEL``: replicated coefficients, the ranks' micro-batches form one global step: every rank
      scores its own samples, the per-coordinate gradient sums (g, g^2) are all-reduced as one dense buffer
      (RCCL), and every rank applies the same mini-batch FTRL-proximal update (n += sum g^2, z += sum g - sigma w).
      Throughput grows with P; per-sample ordering inside a micro-batch is not kept (a different, mini-batch
      rule than SEQUENTIAL / SHARDED).
    * ``HOGWILD`` (GPU): ``ops/csrc/ftrl.hip``, one wave per sample, exact atomic n/z, prox pass; with P ranks
      every rank runs it on its own micro-batch and the (dn, dz) increments are all-reduced each step.

    Every step (and every snapshot decision) is a collective over the ranks, so ranks with different numbers of
    micro-batches stay in lockstep: a rank whose stream ended keeps joining steps with an empty batch until all
    ranks are done.  Snapshots: at the first step, whenever any rank's ``timeInterval`` elapsed, and at the end.
    """
    EXTRA_PARAMS = [ParamInfo("updateMode", str, "SEQUENTIAL (default), AUTO (SHARDED on a GPU, else "
                                                 "SEQUENTIAL), SHARDED (feature-sharded micro-batch), "
                                                 "DATA_PARALLEL (replicated, all-reduced mini-batch gradients) or "
                                                 "HOGWILD (GPU, one wave per sample)", default="SEQUENTIAL"),
                    ParamInfo("asyncGradReduce", bool, "DATA_PARALLEL: overlap the gradient all-reduce of a step "
                                                       "with scoring the next (one-step-stale gradients)",
                              default=False)]

    def __init__(self, model=None, params: Optional[Params] = None, **kw):
        if isinstance(model, Params):
            model, params = None, model
        super().__init__(params, **kw)
        if model is None:
            raise ValueError("Ftrl algo: initial model is null. Please set a valid initial model.")
        self._init_model = model

    def linkFrom(self, *inputs):
        import torch
        (inp,) = self._connect(*inputs)
        p = self.getParams()
        mt = _model_rows(self._init_model)
        conv = LinearModelDataConverter(LinearModelDataConverter.extractLabelType(mt.schema))
        self._model = conv.load(mt.rows())
        self._label_type = inp.getSchema().types[inp.getSchema().names.index(p.get("labelCol"))]
        self._conv = LinearModelDataConverter(self._label_type)
        base = self._conv.getModelSchema()
        self._schema = TableSchema(["bid", "ntab"] + list(base.names), [Types.LONG, Types.LONG] + list(base.types))
        w0 = np.array(self._model.coefVector.data, dtype=np.float64)
        self._dim = int(w0.size)
        self._bid = 0
        self._first = True
        self._t0 = time.time()
        self._alpha = float(_pget(p, "alpha", 0.1))
        self._beta = float(_pget(p, "beta", 1.0))
        self._l1 = float(_pget(p, "l1", 0.0))
        self._l2 = float(_pget(p, "l2", 0.0))
        self._interval = float(_pget(p, "timeInterval", 1800))
        self._intercept = bool(_pget(p, "withIntercept", True))
        self._vec_col = _pget(p, "vectorCol")
        self._feat_cols = _pget(p, "featureCols")
        self._vsize = _pget(p, "vectorSize")
        self._mode = str(_pget(p, "updateMode", "SEQUENTIAL")).upper()
        if self._mode == "AUTO":
            self._mode = "SHARDED" if self.env.device.type == "cuda" else "SEQUENTIAL"
        self._async_reduce = bool(_pget(p, "asyncGradReduce", False))
        self._pending = None
        if self._mode not in ("SEQUENTIAL", "SHARDED", "DATA_PARALLEL", "HOGWILD"):
            raise ValueError(f"unknown updateMode {self._mode}")
        self._ws, self._rank = comm.get_world_size(), comm.get_rank()
        self.recv_nnz = []          # SHARDED: nonzeros this shard received per step (observability / tests)
        self.snapshot_log = []      # per snapshot: bid, perf_counter at its start and at its emission
        # SEQUENTIAL keeps its state on the host (the rule is a serial loop); the others on the rank's GPU
        gpu = self.env.device.type == "cuda" and self._mode != "SEQUENTIAL"
        self._dev = self.env.device if gpu else torch.device("cpu")
        if self._mode == "HOGWILD" and self._dev.type != "cuda":
            raise RuntimeError("FTRL updateMode HOGWILD needs a GPU")
        # owned coordinate range (the whole vector unless SHARDED)
        if self._mode == "SHARDED":
            per = -(-self._dim // self._ws)
            self._lo, self._hi = min(self._dim, self._rank * per), min(self._dim, (self._rank + 1) * per)
        else:
            self._lo, self._hi = 0, self._dim
        shard = w0[self._lo:self._hi].copy()
        if self._dev.type == "cuda":
            self._state = [torch.as_tensor(a, device=self._dev).clone() for a in (shard, np.zeros_like(shard),
                                                                                  np.zeros_like(shard))]
        else:
            self._state = [shard, np.zeros_like(shard), np.zeros_like(shard)]
        _register_upstream_sources(inp)
        return self

    # ---------------------------------------------------------------- model state
    def _full_w(self) -> np.ndarray:
        import torch
        w = self._state[0]
        if self._mode != "SHARDED" or self._ws == 1:
            return (w.cpu().numpy() if isinstance(w, torch.Tensor) else w).copy()
        per = -(-self._dim // self._ws)
        t = torch.as_tensor(w, dtype=torch.float64)
        pad = torch.zeros(per, dtype=torch.float64, device=t.device)
        pad[:t.shape[0]] = t
        full = comm.all_gather_tensor(pad if comm._backend() == "nccl" and pad.is_cuda else pad.cpu())
        return full.cpu().numpy()[:self._dim].copy()

    def _snapshot(self):
        t_begin = time.perf_counter()
        w = self._full_w()
        m = self._model
        m.coefVector = DenseVector(w)
        m.hasInterceptItem = self._intercept
        m.vectorColName = self._vec_col
        m.featureNames = list(self._feat_cols) if self._feat_cols else None
        m.modelName = "Logistic Regression"
        m.vectorSize = w.size - 1 if self._intercept else w.size
        rows = self._conv.save(m)
        out = [(self._bid, len(rows)) + tuple(r) for r in rows]
        snap = MTable.from_rows(out, self._schema)
        # in-process subscribers (FtrlPredictStreamOp) hot-swap from the vector itself, not by re-parsing JSON
        snap.ftrl_coef = (self._bid, w, rows[0][1])
        self.snapshot_log.append({"bid": self._bid, "t_begin": t_begin, "t_emit": time.perf_counter()})
        self._bid += 1
        self._emit(snap)

    # ---------------------------------------------------------------- checkpoint state
    def _state_dict(self):
        import torch
        self._drain()
        w, n, z = (torch.as_tensor(a).detach().cpu().clone() for a in self._state)
        return {"w": w, "n": n, "z": z, "bid": int(self._bid), "first": bool(self._first)}

    def _load_state_dict(self, st):
        import torch
        for k, key in enumerate(("w", "n", "z")):
            if isinstance(self._state[k], torch.Tensor):
                self._state[k].copy_(st[key].to(self._state[k].device))
            else:
                self._state[k][:] = st[key].numpy()
        self._bid = int(st["bid"])
        self._first = bool(st["first"])

    # ---------------------------------------------------------------- stream protocol
    def on_batch(self, port, mt):
        self._step(mt if mt.num_rows else None)

    def on_finish(self, port):
        while self._step(None):
            pass
        self._drain()
        self._snapshot()

    def _step(self, mt) -> bool:
        """One lockstep step over the ranks; False once every rank's stream has ended (nothing applied)."""
        import torch
        csr = self._local_csr(mt) if mt is not None else None
        due = time.time() - self._t0 > self._interval
        nloc = 0 if csr is None else int(csr[0].numel() - 1)
        info = torch.tensor([[0 if csr is None else 1, 1 if due else 0, nloc]], dtype=torch.int64)
        if self._ws > 1:
            # [P, 3]: live, due, samples per rank — over the host group: the rank's GPU stream is never synced
            info = comm.host_all_gather(info)
        active, due = bool(info[:, 0].max()), bool(info[:, 1].max())
        counts = [int(c) for c in info[:, 2].tolist()]
        if not active:
            return False
        if self._first:
            self._snapshot()
            self._first = False
        if self._mode == "DATA_PARALLEL":
            self._dp_step(csr)
        elif self._mode == "HOGWILD" and self._ws > 1:
            self._hogwild_step(csr)
        elif self._ws == 1:
            if csr is not None and csr[0].shape[0] > 1:
                self._apply(*csr)
        elif self._mode == "SHARDED" and os.environ.get("ALINK_FTRL_SHARDED_EXCHANGE", "split") != "allgather":
            self._sharded_step(csr, counts)
        else:                           # SEQUENTIAL (and SHARDED's all-gather exchange, kept for comparison)
            batch = self._gather(csr)
            if batch is not None and batch[0].shape[0] > 1:
                self._apply(*batch)
        if due:
            self._t0 = time.time()
            self._drain()
            self._snapshot()
        return True

    def _sharded_step(self, csr, counts):
        """SplitVector exchange (``FtrlTrainStreamOp.java:174-267``): this rank's samples split by coefficient
        range, shard j receiving only the entries in [lo_j, hi_j) (one all-to-all), then partial margins over the
        global batch, a per-sample margin all-reduce and the in-order replay of the owned coordinates."""
        import torch
        P = self._ws
        per = -(-self._dim // P)
        cd = self._comm_dev()
        offset = sum(counts[:self._rank])
        G = sum(counts)
        if csr is None:
            send = [torch.zeros((0, 3), dtype=torch.int64, device=cd) for _ in range(P)]
            lab = torch.zeros(0, dtype=torch.float64, device=cd)
        else:
            indptr, idx, val, lab = (t.to(cd) for t in csr)
            rows = torch.repeat_interleave(torch.arange(indptr.numel() - 1, device=cd, dtype=torch.int64) + offset,
                                           indptr[1:] - indptr[:-1])
            owner = idx.to(torch.int64) // per
            # one int64 entry per nonzero: global row id, coordinate, and the fp64 value's bits (exact)
            ent = torch.stack([rows, idx.to(torch.int64), val.to(torch.float64).view(torch.int64)], 1)
            order = torch.argsort(owner, stable=True)            # by destination, sample order kept inside
            ent = ent[order]
            split = torch.bincount(owner, minlength=P).tolist()
            send = list(torch.split(ent, split))
        recv = comm.all_to_all_tensors(send)                     # from every source rank, in rank order
        ent = torch.cat(recv) if recv else torch.zeros((0, 3), dtype=torch.int64, device=cd)
        self.recv_nnz.append(int(ent.shape[0]))
        # labels of the global batch in rank order; the per-rank counts are known from the step's control gather
        glab = comm.all_gather_varlen(lab.to(torch.float64), lens=counts)
        grow = ent[:, 0]
        gptr = torch.zeros(G + 1, dtype=torch.int64, device=cd)
        if ent.shape[0]:
            torch.cumsum(torch.bincount(grow, minlength=G), 0, out=gptr[1:])
        gidx = ent[:, 1].to(torch.int32).contiguous()
        gval = ent[:, 2].contiguous().view(torch.float64)
        dev = self._dev
        gptr, gidx, gval, glab = (t.to(dev) for t in (gptr, gidx, gval, glab))
        a, b, l1, l2 = self._alpha, self._beta, self._l1, self._l2
        w, n, z = self._state
        if isinstance(w, torch.Tensor):
            from ...ops.ftrl import ftrl_partial_margin_hip, ftrl_shard_update_hip
            margin = ftrl_partial_margin_hip(gptr, gidx, gval, w, self._lo, self._hi)
            margin = comm.all_reduce(margin.to(cd), "sum").to(dev)
            err = (torch.sigmoid(margin) - glab).contiguous()
            ftrl_shard_update_hip(gptr, gidx, gval, err, w, n, z, self._lo, self._hi, a, b, l1, l2)
        else:
            args = (gptr.numpy(), gidx.numpy(), gval.numpy())
            margin = torch.from_numpy(_native.ftrl_partial_margin(*args, w, self._lo, self._hi))
            margin = comm.all_reduce(margin, "sum")
            err = (1.0 / (1.0 + np.exp(-margin.numpy()))) - glab.numpy()
            _native.ftrl_shard_update(*args, err, w, n, z, self._lo, self._hi, a, b, l1, l2)

    def _dp_step(self, csr):
        """DATA_PARALLEL: local scoring, one dense all-reduce of the per-coordinate (sum g, sum g^2), identical
        mini-batch FTRL-proximal update on every rank (``ops/ftrl.py``).  ``asyncGradReduce``: the all-reduce of
        step t runs on the comm stream while step t+1 scores (gradients one micro-batch stale, BASELINE config 5's
        async RCCL gradient reduce); step t's update is applied when step t+1's reduce is issued."""
        import torch
        from ...ops.ftrl import ftrl_dp_gradients, ftrl_dp_update
        w, n, z = (a if isinstance(a, torch.Tensor) else torch.from_numpy(a) for a in self._state)
        dev = w.device
        if csr is not None and csr[0].numel() > 1:
            gq, _ = ftrl_dp_gradients(*(t.to(dev) for t in csr), w)
        else:
            gq = torch.zeros((2, self._dim), dtype=torch.float64, device=dev)
        if self._ws > 1 and self._async_reduce:
            prev = self._pending
            self._pending = comm.all_reduce_async(gq.to(self._comm_dev()), "sum")
            if prev is not None:
                ftrl_dp_update(prev.wait().to(dev), w, n, z, self._alpha, self._beta, self._l1, self._l2)
            return
        if self._ws > 1:
            gq = comm.all_reduce(gq.to(self._comm_dev()), "sum").to(dev)
        ftrl_dp_update(gq, w, n, z, self._alpha, self._beta, self._l1, self._l2)

    def _drain(self):
        """Apply the last in-flight asynchronous gradient reduce (before a snapshot or the end)."""
        if getattr(self, "_pending", None) is not None:
            import torch
            from ...ops.ftrl import ftrl_dp_update
            w, n, z = (a if isinstance(a, torch.Tensor) else torch.from_numpy(a) for a in self._state)
            ftrl_dp_update(self._pending.wait().to(w.device), w, n, z, self._alpha, self._beta, self._l1, self._l2)
            self._pending = None

    def _hogwild_step(self, csr):
        """HOGWILD over P ranks: every rank runs the one-wave-per-sample Hogwild kernel on its OWN micro-batch
        from the shared state of the step start, the per-coordinate increments (dn, dz) of all ranks are summed
        (one dense all-reduce) and added to that state, and w = prox(z, n) is re-derived.  Within a rank samples
        race as in the single-GPU mode; across ranks a sample sees the other ranks' updates one micro-batch late
        (the reference's asynchronous feedback loop, bounded staleness)."""
        import torch
        from ...ops.ftrl import ftrl_hogwild, ftrl_prox_hip
        w, n, z = self._state
        n0, z0 = n.clone(), z.clone()
        if csr is not None and csr[0].numel() > 1:
            ftrl_hogwild(*(t.to(self._dev) for t in csr), w, n, z, self._alpha, self._beta, self._l1, self._l2)
        d = torch.stack([n - n0, z - z0])
        d = comm.all_reduce(d.to(self._comm_dev()), "sum").to(self._dev)
        n.copy_(n0 + d[0])
        z.copy_(z0 + d[1])
        ftrl_prox_hip(w, n, z, self._alpha, self._beta, self._l1, self._l2)

    def _comm_dev(self):
        import torch
        return self._dev if (comm._backend() == "nccl" and self._dev.type == "cuda") else torch.device("cpu")

    def _gather(self, csr):
        """All-gather the ranks' CSR micro-batches in rank order (empty for finished ranks)."""
        import torch
        cd = self._comm_dev()
        if csr is None:
            csr = (torch.zeros(1, dtype=torch.int64), torch.zeros(0, dtype=torch.int32),
                   torch.zeros(0, dtype=torch.float64), torch.zeros(0, dtype=torch.float64))
        indptr, idx, val, lab = (t.to(cd) for t in csr)
        lens = comm.all_gather_varlen(indptr[1:] - indptr[:-1])
        gidx = comm.all_gather_varlen(idx)
        gval = comm.all_gather_varlen(val)
        glab = comm.all_gather_varlen(lab)
        gptr = torch.zeros(lens.shape[0] + 1, dtype=torch.int64, device=lens.device)
        torch.cumsum(lens, 0, out=gptr[1:])
        return tuple(t.to(self._dev) for t in (gptr, gidx, gval, glab))

    def _local_csr(self, mt: MTable):
        import torch
        p = self.getParams()
        fm = extract_features(mt, self._feat_cols if self._vec_col is None else None, self._vec_col, self._dev,
                              vector_size=self._vsize)
        if self._intercept:
            fm = fm.prefix_one()
        if fm.is_sparse:
            indptr, indices, values = fm.crow.to(torch.int64), fm.col.to(torch.int32), fm.val.to(torch.float64)
        else:
            X = fm.to_dense().to(torch.float64)
            nrow, d = X.shape
            indptr = torch.arange(nrow + 1, dtype=torch.int64, device=X.device) * d
            indices = torch.arange(d, dtype=torch.int32, device=X.device).repeat(nrow)
            values = X.reshape(-1)
        l0 = self._model.labelValues[0]
        col = mt.col(p.get("labelCol"))
        if isinstance(col.values, torch.Tensor) and isinstance(l0, (int, float)) and not isinstance(l0, bool):
            labels = (col.values.to(torch.float64) == float(l0)).to(torch.float64)
        else:
            vals = col.to_list()
            if isinstance(l0, (int, float)) and not isinstance(l0, bool):
                labels = torch.tensor([1.0 if float(v) == float(l0) else 0.0 for v in vals], dtype=torch.float64)
            else:
                labels = torch.tensor([1.0 if str(v) == str(l0) else 0.0 for v in vals], dtype=torch.float64)
        if indices.numel() and int(indices.max()) >= self._dim:
            raise ValueError("feature index out of range of the initial model")
        return (indptr.contiguous(), indices.contiguous(), values.contiguous(),
                labels.to(indptr.device).contiguous())

    def _apply(self, indptr, idx, val, lab):
        import torch
        a, b, l1, l2 = self._alpha, self._beta, self._l1, self._l2
        w, n, z = self._state
        if self._mode == "HOGWILD":
            from ...ops.ftrl import ftrl_hogwild
            ftrl_hogwild(indptr, idx, val, lab, w, n, z, a, b, l1, l2)
            return
        if self._mode == "SEQUENTIAL":
            args = (indptr.numpy(), idx.numpy(), val.numpy(), lab.numpy())
            if not _native.ftrl_update_csr(*args, w, n, z, a, b, l1, l2):
                _ftrl_python(*args, w, n, z, a, b, l1, l2)
            return
        # SHARDED: partial margins on the owned range -> all-reduce -> per-coordinate replay
        if isinstance(w, torch.Tensor):
            from ...ops.ftrl import ftrl_partial_margin_hip, ftrl_shard_update_hip
            margin = ftrl_partial_margin_hip(indptr, idx, val, w, self._lo, self._hi)
            if self._ws > 1:
                margin = comm.all_reduce(margin.to(self._comm_dev()), "sum").to(self._dev)
            err = (torch.sigmoid(margin) - lab).contiguous()
            ftrl_shard_update_hip(indptr, idx, val, err, w, n, z, self._lo, self._hi, a, b, l1, l2)
        else:
            args = (indptr.numpy(), idx.numpy(), val.numpy())
            margin = torch.from_numpy(_native.ftrl_partial_margin(*args, w, self._lo, self._hi))
            if self._ws > 1:
                margin = comm.all_reduce(margin, "sum")
            err = (1.0 / (1.0 + np.exp(-margin.numpy()))) - lab.numpy()
            _native.ftrl_shard_update(*args, err, w, n, z, self._lo, self._hi, a, b, l1, l2)


class FtrlPredictStreamOp(StreamOperator):
    def __init__(self, model=None, params: Optional[Params] = None, **kw):
        if isinstance(model, Params):
            model, params = None, model
        super().__init__(params, **kw)
        if model is None:
            raise ValueError("Ftrl algo: initial model is null. Please set a valid initial model.")
        self._init_model = model

    def linkFrom(self, *inputs):
        models, data = self._connect(*inputs)
        mt = _model_rows(self._init_model)
        ms = models.getSchema()
        self._model_schema = TableSchema(list(ms.names[2:5]), list(ms.types[2:5]))
        self._mapper = LinearModelMapper(self._model_schema, data.getSchema(), self.getParams())
        self._mapper.loadModel(mt.rows())
        self._schema = self._mapper.getOutputSchema()
        self._buffers = {}
        self._meta = None
        self.swap_log = {}          # bid -> perf_counter when the snapshot became the serving model
        _register_upstream_sources(models)
        _register_upstream_sources(data)
        return self

    def on_batch(self, port, mt):
        if port == 0:
            fast = getattr(mt, "ftrl_coef", None)
            if fast is not None and self._meta == fast[2] and not self._buffers:
                # same meta as the serving model: swap the coefficient vector only (rows stay the record)
                self._mapper.swapCoef(fast[1])
                self.swap_log[int(fast[0])] = time.perf_counter()
                return
            for r in mt.rows():
                bid, ntab = int(r[0]), int(r[1])
                buf = self._buffers.setdefault(bid, [])
                buf.append(tuple(r[2:]))
                if len(buf) == ntab:
                    self._mapper.loadModel(buf)
                    self._meta = next((x[1] for x in buf if int(x[0]) == 0), None)
                    del self._buffers[bid]
                    self.swap_log[bid] = time.perf_counter()
        else:
            self._emit(self._mapper.map_table(mt))
