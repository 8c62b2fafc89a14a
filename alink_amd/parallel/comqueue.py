"""BSP iteration engine: ``IterativeComQueue`` / ``ComContext`` / queue items.

Reference: ``A/common/comqueue/BaseComQueue.java:39-549`` (declarative superstep queue over a Flink bulk
iteration; per-task state in a JVM-static map, ``SessionSharedObjs``/``IterTaskObjKeeper``),
``ComContext.java``, ``ComputeFunction/CommunicateFunction/CompareCriterionFunction/
CompleteResultFunction`` and ``communication/AllReduce.java``.

MI355X design: the queue is plain SPMD.  Each process owns ``local_tasks`` BSP tasks (1 per GPU in
production) whose state lives in ``ComContext`` dictionaries (device tensors stay on the device between
supersteps — no serialisation, no barrier edges).  A superstep is: run every item in order for every
local task; ``CommunicateFunction`` items first combine the local tasks, then issue one collective over
RCCL (GPU) / gloo (CPU).  The criterion of task 0 decides termination; when the queue state is
bit-identical on every rank after an all-reduce (``criterion_replicated=True``) each rank evaluates it
locally and no broadcast is needed.

Observability: every superstep produces one structured record (``queue.stats`` and
``utils.metrics``: wall time, collective calls / bytes / time, ``rows_per_s`` when the algorithm declared
``setRowsPerStep``, plus fields logged by items through ``logMetric``); with tracing on
(``utils.trace``) each superstep and each compute / communicate item is a timeline span and a roctx range.

Fault tolerance (the reference has none: ComQueue state lives in the JVM heap and any failure restarts the
job):
* ``setCheckpoint(dir, every)`` — after every ``every``-th superstep each rank atomically writes its task
  state (everything except the partitioned/broadcast inputs, which are rebuilt from the DAG) plus the
  tensor / plain-data state of the queue items and criterion (no pickled objects: loaded with
  ``weights_only=True``), the criterion's stop decision and a fingerprint of the job (queue structure,
  max_iter, layout, partition sizes — a directory of another job is rejected); ``exec`` resumes from the
  newest step ALL ranks have (agreed with one MIN all-reduce), so a killed job restarts at a superstep
  boundary, and a job whose checkpoint is the converged superstep returns its result without running on;
* ``setWatchdog(seconds)`` — a superstep (its collectives included) that exceeds the limit dumps every
  thread's stack and terminates the process instead of hanging the job (a stuck RCCL peer);
* fault injection for tests: ``ALINK_FAULT_INJECT="<rank>:<step>"`` raises ``InjectedFault`` on that rank
  at the start of that superstep.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import time
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

from . import comm
from ..utils import metrics as _metrics
from ..utils import trace as _trace

__all__ = ["InjectedFault", "ComContext", "ComputeFunction", "CommunicateFunction", "CompareCriterionFunction",
           "CompleteResultFunction", "AllReduce", "BaseComQueue", "IterativeComQueue", "ComQueue",
           "ChainedComputation", "AllGather", "Broadcast", "SUM", "MAX", "MIN"]

SUM, MAX, MIN = "sum", "max", "min"


class InjectedFault(RuntimeError):
    """Raised by the ``ALINK_FAULT_INJECT`` hook (tests of checkpoint/resume)."""


class _Skip(Exception):
    pass


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


_NULL = _NullCtx()


_SCALARS = (bool, int, float, str, type(None))


def _plain(v):
    """Checkpointable form of ``v``: tensors (on CPU), numpy arrays (as ``{"__np__": tensor}``), scalars and
    lists / tuples / str-keyed dicts of those.  Anything else raises ``_Skip`` — checkpoints hold no
    pickled objects, so they load with ``torch.load(weights_only=True)`` (no code runs from the file)."""
    if isinstance(v, torch.Tensor):
        return v.detach().cpu()
    if isinstance(v, np.ndarray):
        if v.dtype == object:
            raise _Skip
        return {"__np__": torch.from_numpy(np.ascontiguousarray(v))}
    if isinstance(v, np.generic):
        return v.item()
    if isinstance(v, _SCALARS):
        return v
    if isinstance(v, list):
        return [_plain(x) for x in v]
    if isinstance(v, tuple):
        return tuple(_plain(x) for x in v)
    if isinstance(v, dict) and all(isinstance(k, str) for k in v):
        return {k: _plain(x) for k, x in v.items()}
    raise _Skip


def _unplain(v, dev):
    if isinstance(v, torch.Tensor):
        return v.to(dev) if dev is not None else v
    if isinstance(v, dict):
        if set(v) == {"__np__"}:
            return v["__np__"].numpy()
        return {k: _unplain(x, dev) for k, x in v.items()}
    if isinstance(v, list):
        return [_unplain(x, dev) for x in v]
    if isinstance(v, tuple):
        return tuple(_unplain(x, dev) for x in v)
    return v


def _plain_items(d: Dict[str, Any], skip=()) -> Dict[str, Any]:
    out = {}
    for k, v in d.items():
        if k in skip:
            continue
        try:
            out[k] = _plain(v)
        except _Skip:
            pass
    return out


class ComContext:
    def __init__(self, store: Dict[str, Any], task_id: int, num_task: int, queue: "BaseComQueue"):
        self._store = store
        self._task_id = task_id
        self._num_task = num_task
        self._queue = queue

    def getTaskId(self) -> int:
        return self._task_id

    def getNumTask(self) -> int:
        return self._num_task

    def getStepNo(self) -> int:
        return self._queue.step_no

    def getObj(self, name: str):
        return self._store.get(name)

    def putObj(self, name: str, obj):
        self._store[name] = obj

    def removeObj(self, name: str):
        self._store.pop(name, None)

    def containsObj(self, name: str) -> bool:
        return name in self._store

    @property
    def device(self):
        return self._queue.device

    def logMetric(self, name: str, value):
        """Attach ``name=value`` to this superstep's metrics record (``utils.metrics``)."""
        self._queue.logMetric(name, value)


class ComputeFunction:
    def calc(self, context: ComContext):
        raise NotImplementedError

    def name(self):
        return type(self).__name__


class ChainedComputation(ComputeFunction):
    """Adjacent compute items fused into one (reference ``ChainedComputation.java:10-39``)."""

    def __init__(self, fns: Sequence[ComputeFunction]):
        self.fns = list(fns)

    def calc(self, context):
        for f in self.fns:
            f.calc(context)

    def name(self):
        return "chained computation@" + "->".join(f.name() for f in self.fns)


class CommunicateFunction:
    def communicate(self, contexts: List[ComContext], queue: "BaseComQueue"):
        raise NotImplementedError

    def name(self):
        return type(self).__name__


class CompareCriterionFunction:
    def calc(self, context: ComContext) -> bool:
        raise NotImplementedError


class CompleteResultFunction:
    def calc(self, context: ComContext) -> Optional[List]:
        raise NotImplementedError


def _as_tensor(buf):
    if isinstance(buf, torch.Tensor):
        return buf, "torch"
    if isinstance(buf, np.ndarray):
        return torch.from_numpy(buf), "numpy"
    if isinstance(buf, list):
        return torch.tensor(buf, dtype=torch.float64), "list"
    raise TypeError(f"AllReduce buffer must be tensor/ndarray/list, got {type(buf)}")


class AllReduce(CommunicateFunction):
    """Element-wise SUM/MAX/MIN of buffer ``bufferName`` across all tasks; optionally only the prefix
    ``[0, ctx.getObj(lengthName))``.  Local tasks are folded on-device before one collective."""

    def __init__(self, bufferName: str, lengthName: Optional[str] = None, op: str = SUM):
        self.buffer = bufferName
        self.length = lengthName
        self.op = op if isinstance(op, str) else str(op)

    def name(self):
        return f"AllReduce({self.buffer})"

    def communicate(self, contexts, queue):
        bufs = [c.getObj(self.buffer) for c in contexts]
        present = [b for b in bufs if b is not None]
        if not present:
            raise RuntimeError(f"AllReduce buffer {self.buffer} missing")
        n = None
        if self.length is not None:
            n = int(contexts[0].getObj(self.length))
        t0, kind = _as_tensor(present[0])
        if len(bufs) == 1 and n is None and kind == "torch" and t0.is_contiguous():
            comm.all_reduce(t0.view(-1), self.op)      # one task per process (one GPU): reduce in place
            return
        view = (lambda t: t.reshape(-1)[:n]) if n is not None else (lambda t: t.reshape(-1))
        acc = view(t0).clone()
        for b in present[1:]:
            tb, _ = _as_tensor(b)
            tb = view(tb).to(acc.device)
            if self.op == SUM:
                acc += tb
            elif self.op == MAX:
                torch.maximum(acc, tb, out=acc)
            else:
                torch.minimum(acc, tb, out=acc)
        comm.all_reduce(acc, self.op)
        for c, b in zip(contexts, bufs):
            if b is None:
                continue
            tb, kind = _as_tensor(b)
            view(tb).copy_(acc.to(tb.device))
            if kind == "list":
                c.putObj(self.buffer, tb.tolist())


class AllGather(CommunicateFunction):
    """Every task ends with the list of all tasks' ``bufferName`` objects (in task order)."""

    def __init__(self, bufferName: str, outName: Optional[str] = None):
        self.buffer, self.out = bufferName, outName or bufferName + "_all"

    def communicate(self, contexts, queue):
        local = [c.getObj(self.buffer) for c in contexts]
        allv = [x for part in comm.all_gather_object(local) for x in part]
        for c in contexts:
            c.putObj(self.out, list(allv))


class Broadcast(CommunicateFunction):
    """Object in task 0's ``bufferName`` copied to every task."""

    def __init__(self, bufferName: str):
        self.buffer = bufferName

    def communicate(self, contexts, queue):
        v = contexts[0].getObj(self.buffer) if comm.get_rank() == 0 else None
        v = comm.broadcast_object(v, 0)
        for c in contexts:
            c.putObj(self.buffer, v)


def _split(data, parts: int) -> List[Any]:
    """Split a partition into ``parts`` contiguous sub-partitions."""
    if parts == 1:
        return [data]
    from ..common.table import MTable
    n = len(data) if not isinstance(data, torch.Tensor) else data.shape[0]
    bounds = [(i * n) // parts for i in range(parts + 1)]
    out = []
    for i in range(parts):
        lo, hi = bounds[i], bounds[i + 1]
        if isinstance(data, MTable):
            out.append(data.slice(lo, hi))
        else:
            out.append(data[lo:hi])
    return out


class BaseComQueue:
    def __init__(self):
        self.items: List[Any] = []
        self.criterion: Optional[CompareCriterionFunction] = None
        self.criterion_replicated = False
        self.complete: Optional[CompleteResultFunction] = None
        self.max_iter = 2 ** 31 - 1
        self.partitioned: List = []
        self.broadcast: List = []
        self.step_no = 0
        self.stats: List[Dict[str, float]] = []
        self.on_step: List[Callable[[int, "BaseComQueue"], None]] = []
        self.env = None
        self.device = None
        self.sync_device_per_step = False
        self.ckpt_dir: Optional[str] = None
        self.ckpt_every = 1
        self.watchdog_s: Optional[float] = None
        self.resumed_from = 0
        self.resumed_stop = False
        self.rows_per_step = 0
        self.job_name = None
        self._step_metrics: Dict[str, Any] = {}

    # ---- fault tolerance ----
    def setCheckpoint(self, directory: str, every: int = 1):
        self.ckpt_dir, self.ckpt_every = directory, max(1, int(every))
        return self

    def setWatchdog(self, seconds: float):
        self.watchdog_s = float(seconds)
        return self

    def _ckpt_file(self, rank: int, step: int) -> str:
        return os.path.join(self.ckpt_dir, f"rank{rank}", f"step{step:08d}.pt")

    def _item_states(self, items):
        return [_plain_items(getattr(it, "__dict__", {})) for it in list(items) + [self.criterion]]

    def _fingerprint(self, items, stores) -> str:
        """Identity of the job a checkpoint belongs to: queue structure, max_iter, world / task layout and
        the size of every partitioned input (a reused directory from another job is rejected)."""
        sizes = []
        for name, data in self.partitioned:
            sizes.append([name] + [(len(st[name]) if not isinstance(st[name], torch.Tensor)
                                    else int(st[name].shape[0])) if st.get(name) is not None else -1
                                   for st in stores])
        from ..common.mlenv import MLEnvironmentFactory
        env = self.env or MLEnvironmentFactory.getDefault()
        return repr(("->".join(it.name() for it in items), type(self.criterion).__name__, self.max_iter,
                     env.world_size, env.local_tasks, sizes))

    def _save_checkpoint(self, rank, stores, items, skip, stop=False):
        state = {"step": self.step_no, "stop": bool(stop), "fingerprint": self._fingerprint(items, stores),
                 "stores": [_plain_items(st, skip) for st in stores],
                 "items": self._item_states(items)}
        path = self._ckpt_file(rank, self.step_no)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = path + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)
        for old in os.listdir(os.path.dirname(path)):      # keep the newest two
            full = os.path.join(os.path.dirname(path), old)
            if old.endswith(".pt") and full < self._ckpt_file(rank, self.step_no - self.ckpt_every):
                os.remove(full)

    def _try_resume(self, rank, stores, items) -> int:
        d = os.path.join(self.ckpt_dir, f"rank{rank}")
        steps = sorted(int(f[4:12]) for f in os.listdir(d) if f.endswith(".pt")) if os.path.isdir(d) else []
        mine = torch.tensor([float(steps[-1]) if steps else 0.0], dtype=torch.float64)
        comm.all_reduce(mine, MIN)
        step = int(mine.item())
        if step <= 0 or step not in steps:
            return 0
        state = torch.load(self._ckpt_file(rank, step), map_location="cpu", weights_only=True)
        fp = self._fingerprint(items, stores)
        if state.get("fingerprint") != fp:
            raise RuntimeError(f"checkpoint {self._ckpt_file(rank, step)} belongs to another job "
                               f"({state.get('fingerprint')!r} != {fp!r}); use an empty checkpoint directory")
        for st, saved in zip(stores, state["stores"]):
            st.update(_unplain(saved, self.device))
        for it, saved in zip(list(items) + [self.criterion], state["items"]):
            if it is not None:
                it.__dict__.update(_unplain(saved, None if isinstance(it, CompareCriterionFunction)
                                            else self.device))
        self.resumed_stop = bool(state.get("stop", False))
        return step

    # ---- builder API (names as in the reference) ----
    def initWithPartitionedData(self, name: str, data):
        self.partitioned.append((name, data))
        return self

    def initWithBroadcastData(self, name: str, data):
        self.broadcast.append((name, data))
        return self

    def add(self, item):
        self.items.append(item)
        return self

    def setCompareCriterionOfNode0(self, criterion: CompareCriterionFunction, replicated: bool = False):
        self.criterion = criterion
        self.criterion_replicated = replicated
        return self

    def closeWith(self, complete: CompleteResultFunction):
        self.complete = complete
        return self

    def setMaxIter(self, n: int):
        self.max_iter = int(n)
        return self

    def setMLEnvironment(self, env):
        self.env = env
        return self

    def addStepCallback(self, fn: Callable[[int, "BaseComQueue"], None]):
        self.on_step.append(fn)
        return self

    # ---- metrics ----
    def setRowsPerStep(self, n: int):
        """Rows one superstep processes on this rank (the per-step record then carries ``rows_per_s``)."""
        self.rows_per_step = int(n)
        return self

    def setJobName(self, name: str):
        self.job_name = name
        return self

    def logMetric(self, name: str, value):
        """Attach ``name=value`` to the current superstep's record (e.g. the loss of an optimizer step)."""
        if isinstance(value, torch.Tensor):
            value = value.item()
        self._step_metrics[name] = value
        return self

    def optimize(self) -> List[Any]:
        """Fuse runs of adjacent compute items (reference ``BaseComQueue.optimize`` :470-495)."""
        out: List[Any] = []
        run: List[ComputeFunction] = []
        for it in self.items:
            if isinstance(it, ComputeFunction):
                run.append(it)
                continue
            if run:
                out.append(run[0] if len(run) == 1 else ChainedComputation(run))
                run = []
            out.append(it)
        if run:
            out.append(run[0] if len(run) == 1 else ChainedComputation(run))
        return out

    def __str__(self):
        """The reference's ``BaseComQueue.toString`` JSON: complete-result and criterion class names, maxIter,
        the session (ML environment) id and the optimized queue as class names (fused runs of compute
        functions show as ``ChainedComputation``)."""
        import json

        def cls(o):
            return None if o is None else type(o).__name__
        env_id = getattr(self.env, "env_id", 0) if self.env is not None else 0
        return json.dumps({"completeResult": cls(self.complete), "maxIter": self.max_iter, "sessionId": env_id,
                           "queue": ",".join(cls(it) for it in self.optimize()),
                           "compareCriterion": cls(self.criterion)}, separators=(",", ":"))

    # ---- execution ----
    def exec(self) -> List:
        from ..common.mlenv import MLEnvironmentFactory
        from ..common.table import MTable
        from ..operator.base import gather_table
        env = self.env or MLEnvironmentFactory.getDefault()
        self.device = env.device
        lt = env.local_tasks
        ws = env.world_size
        num_task = ws * lt
        first_task = env.rank * lt
        stores: List[Dict[str, Any]] = [dict() for _ in range(lt)]
        ctxs = [ComContext(stores[i], first_task + i, num_task, self) for i in range(lt)]
        for name, data in self.partitioned:
            for s, part in zip(stores, _split(data, lt)):
                s[name] = part
        for name, data in self.broadcast:
            full = gather_table(data) if isinstance(data, MTable) else data
            for s in stores:
                s[name] = full
        items = self.optimize()
        self.step_no = 0
        if self.ckpt_dir is not None:
            self.resumed_from = self._try_resume(env.rank, stores, items)
        inject = os.environ.get("ALINK_FAULT_INJECT")
        inject = tuple(int(x) for x in inject.split(":")) if inject else None
        skip = {n for n, _ in self.partitioned} | {n for n, _ in self.broadcast}
        use_roctx = self.device is not None and self.device.type == "cuda" and hasattr(torch.cuda, "nvtx")
        job = self.job_name or "->".join(it.name() for it in items)
        self.step_no = self.resumed_from
        stop = self.resumed_stop        # a checkpoint written at the converged superstep ends the run
        while not stop and self.step_no < self.max_iter:
            self.step_no += 1
            if inject is not None and inject == (env.rank, self.step_no):
                raise InjectedFault(f"injected fault on rank {env.rank} at superstep {self.step_no}")
            if self.watchdog_s is not None:
                faulthandler.dump_traceback_later(self.watchdog_s, exit=True, file=sys.stderr)
            t0 = time.perf_counter()
            b0, c0, s0 = comm.STATS.bytes, comm.STATS.calls, comm.STATS.time_s
            self._step_metrics = {}
            tracing = _trace.enabled()
            if use_roctx and not tracing:
                try:
                    torch.cuda.nvtx.range_push(f"superstep {self.step_no}")
                except Exception:
                    use_roctx = False
            step_span = _trace.span(f"superstep {self.step_no}", "superstep", job=job) if tracing else None
            if step_span is not None:
                step_span.__enter__()
            for it in items:
                with (_trace.span(it.name(), "item") if tracing else _NULL):
                    if isinstance(it, CommunicateFunction):
                        it.communicate(ctxs, self)
                    else:
                        for c in ctxs:
                            it.calc(c)
            if self.criterion is not None:
                if self.criterion_replicated or ws == 1:
                    dec = bool(self.criterion.calc(ctxs[0]))
                else:
                    # task 0 decides; one 1-element MAX all-reduce (RCCL on GPU) instead of a pickled broadcast
                    dec = bool(self.criterion.calc(ctxs[0])) if env.rank == 0 else False
                    flag = torch.tensor([1.0 if dec else 0.0], dtype=torch.float64,
                                        device=self.device if self.device is not None and
                                        self.device.type == "cuda" else "cpu")
                    dec = bool(comm.all_reduce(flag, MAX).item() > 0)
                stop = dec
            if step_span is not None:
                step_span.__exit__(None, None, None)
            elif use_roctx:
                torch.cuda.nvtx.range_pop()
            if self.sync_device_per_step and self.device is not None and self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            if self.watchdog_s is not None:
                faulthandler.cancel_dump_traceback_later()
            wall = time.perf_counter() - t0
            rec = {"job": job, "step": self.step_no, "wall_s": wall, "comm_bytes": comm.STATS.bytes - b0,
                   "comm_calls": comm.STATS.calls - c0, "comm_s": comm.STATS.time_s - s0}
            if self.rows_per_step:
                rec["rows"] = self.rows_per_step
                rec["rows_per_s"] = self.rows_per_step / wall if wall > 0 else 0.0
            rec.update(self._step_metrics)
            self.stats.append(rec)
            _metrics.record("superstep", **rec)
            if tracing:
                _trace.counter("comm_bytes", bytes=rec["comm_bytes"])
            if self.ckpt_dir is not None and (self.step_no % self.ckpt_every == 0 or stop):
                self._save_checkpoint(env.rank, stores, items, skip, stop)
            for fn in self.on_step:
                fn(self.step_no, self)
        result: List = []
        if self.complete is not None:
            local = []
            for c in ctxs:
                r = self.complete.calc(c)
                if r is not None:
                    local.extend(r)
            parts = comm.all_gather_object(local) if ws > 1 else [local]
            for p in parts:
                result.extend(p)
        self.final_contexts = ctxs
        return result


class IterativeComQueue(BaseComQueue):
    pass


class ComQueue(BaseComQueue):
    def __init__(self):
        super().__init__()
        self.max_iter = 1
