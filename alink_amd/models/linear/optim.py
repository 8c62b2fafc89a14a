"""Distributed optimizers on the BSP queue: L-BFGS, OWL-QN, GD, SGD, Newton.

Each optimizer is an ``IterativeComQueue`` with the same items, buffers and update rules as the reference:

* ``Lbfgs.java:55-175``  — CalcGradient -> AllReduce(grad) -> two-loop direction (m = 10 corrections,
  no initial Hessian scaling) -> CalcLosses at ``numSearchStep + 1`` step sizes -> AllReduce(losses) ->
  ``UpdateModel`` (adaptive learning rate, ``subfunc/UpdateModel.java:68-176``);
* ``Owlqn.java`` — the same with the L1 pseudo-gradient, direction sign projection and orthant-wise
  coefficient clipping;
* ``Gd.java`` — steepest descent with the same search;
* ``Sgd.java:82-200`` — sampled mini-batch gradient, ``eta = lr / (|g|_inf + sqrt(step))``;
* ``Newton.java`` — gradient + Hessian all-reduce, ``H x = g`` solve, full step.

MI355X design: all state (coefficients, the L-BFGS ``s_k / y_k`` history, directions) is a device tensor;
the gradient of a partition is one GEMV pair (or CSR segment-sum) and the line search evaluates all step
sizes from ONE pass over the samples (``X @ [coef, dir]``).  The only host synchronisations per superstep
are the scalar decisions of ``UpdateModel`` (which step won, convergence), exactly the values the reference
computes on every task.  All tasks hold bit-identical state after each all-reduce, so the termination
criterion is evaluated locally (no broadcast).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import numpy as np
import torch

from ...common.params import Params
from ...parallel.comqueue import (AllReduce, ComputeFunction, CompareCriterionFunction, CompleteResultFunction,
                                  IterativeComQueue)
from .objfunc import LabeledData, OptimObjFunc

__all__ = ["optimize", "OptimMethodName", "NUM_CORRECTIONS", "LEARNING_RATE"]

NUM_CORRECTIONS = 10        # OptimVariable.numCorrections
LEARNING_RATE = 0.1         # OptimVariable.learningRate
EPS = 1.0e-18               # UpdateModel.EPS

TRAIN, MODEL, OBJ = "trainData", "model", "objFunc"
CUR, MIN, CURVE = "currentCoef", "minCoef", "lossCurve"
DIR, GRAD, PSE = "direction", "gradient", "pseGradient"
GRAD_AR, LOSS_AR, SKYK, GH_AR = "gradAllReduce", "lossAllReduce", "sKyK", "gradHessAllReduce"


class OptimMethodName:
    LBFGS, OWLQN, GD, SGD, NEWTON = "LBFGS", "OWLQN", "GD", "SGD", "Newton"


class _State:
    """(vector, scalars) pair — the reference's ``Tuple2<DenseVector, double[]>`` / ``Tuple2<DenseVector,Double>``."""
    __slots__ = ("v", "f")

    def __init__(self, v, f):
        self.v, self.f = v, f


# ---------------------------------------------------------------------------------------------------
# preallocation
# ---------------------------------------------------------------------------------------------------
class _Preallocate(ComputeFunction):
    def __init__(self, max_iter: int, method: str):
        self.max_iter, self.method = max_iter, method

    def calc(self, ctx):
        if ctx.getStepNo() != 1:
            return
        coef = ctx.getObj(MODEL)
        coef = coef.to(device=ctx.device or coef.device, dtype=torch.float64).clone()
        ctx.putObj(CUR, _State(coef.clone(), 1.7976931348623157e308))
        ctx.putObj(MIN, _State(coef.clone(), 1.7976931348623157e308))
        ctx.putObj(CURVE, np.full(self.max_iter, np.inf))
        ctx.putObj(DIR, _State(torch.zeros_like(coef), [0.0, LEARNING_RATE if self.method != OptimMethodName.SGD
                                                          else 0.0]))
        ctx.putObj(GRAD, _State(torch.zeros_like(coef), [0.0]))
        ctx.putObj(PSE, _State(torch.zeros_like(coef), [0.0]))
        if self.method in (OptimMethodName.LBFGS, OptimMethodName.OWLQN):
            d = coef.shape[0]
            ctx.putObj(SKYK, (torch.zeros((NUM_CORRECTIONS, d), dtype=torch.float64, device=coef.device),
                              torch.zeros((NUM_CORRECTIONS, d), dtype=torch.float64, device=coef.device)))
            ctx.putObj("oldGradient", None)


# ---------------------------------------------------------------------------------------------------
# gradient / losses
# ---------------------------------------------------------------------------------------------------
class CalcGradient(ComputeFunction):
    def calc(self, ctx):
        data: LabeledData = ctx.getObj(TRAIN)
        obj: OptimObjFunc = ctx.getObj(OBJ)
        coef = ctx.getObj(CUR).v
        g, ws = obj.calc_gradient(data, coef)
        ctx.getObj(DIR).v = g
        buf = torch.empty(coef.shape[0] + 1, dtype=torch.float64, device=coef.device)
        buf[:-1] = g * ws
        buf[-1] = ws
        ctx.putObj(GRAD_AR, buf)


class CalcLosses(ComputeFunction):
    def __init__(self, method: str, num_search_step: int):
        self.method, self.ns = method, num_search_step

    def calc(self, ctx):
        data = ctx.getObj(TRAIN)
        obj = ctx.getObj(OBJ)
        d = ctx.getObj(DIR)
        coef = ctx.getObj(CUR).v
        beta = d.f[1] / self.ns
        if self.method == OptimMethodName.OWLQN:
            vec = obj.constraint_calc_search_values(data, coef, d.v, beta, self.ns)
        else:
            vec = obj.calc_search_values(data, coef, d.v, beta, self.ns)
        ctx.putObj(LOSS_AR, vec.to(torch.float64).clone())


def _two_loop_body(S, Y, dirv):
    """S, Y: [l, d] corrections in order (oldest first)."""
    dots = (S * Y).sum(1)
    rho = torch.where(dots > 0, 1.0 / torch.where(dots <= 0, torch.ones_like(dots), dots),
                      torch.zeros_like(dots))
    l = S.shape[0]
    alpha = [None] * l
    for i in range(l - 1, -1, -1):
        alpha[i] = rho[i] * (S[i] * dirv).sum()
        dirv = dirv - alpha[i] * Y[i]
    for i in range(l):
        beta_i = rho[i] * (Y[i] * dirv).sum()
        dirv = dirv + (alpha[i] - beta_i) * S[i]
    return dirv


# ---- hipGraph replay of the two-loop ----------------------------------------------------------------------
# The recursion is ~6 l + 4 small kernels (l <= 10 corrections) whose launch cost, not their bytes, sets the time
# of an L-BFGS superstep at moderate sizes.  Once the history is full (l = m, every superstep from k = m + 1 on)
# it is captured ONCE per history as a HIP graph and replayed as a single launch: the history tensors are
# updated in place between supersteps; the rotation of the circular history is a device scalar set by a fill
# kernel before each replay (order = (0..m-1 + delta) mod m gathered inside the graph, no host->device copy);
# inputs / outputs go through static vectors.  The first m supersteps (l < m, each l seen once) run eagerly.
# ALINK_HIP_GRAPHS=0 runs everything eagerly.
import gc as _gc  # noqa: E402
import os as _os  # noqa: E402
import weakref as _weakref  # noqa: E402

_GRAPHS = {}      # id(sK) -> (weakref to sK, {(yK ptr, d, dtype): (graph, static dir, delta, static out)})
GRAPH_MAX_DIM = 1 << 20            # above this each op is bandwidth-bound (launch cost no longer matters) and the
#                                    graph pool would hold 2 x m x d fp64 of gathered history
GRAPH_STATS = {"captures": 0, "replays": 0}


def graphs_enabled() -> bool:
    return _os.environ.get("ALINK_HIP_GRAPHS", "1") != "0"


def _two_loop_rotating(sK, yK, dirv, delta):
    m = sK.shape[0]
    order = torch.remainder(torch.arange(m, device=sK.device) + delta, m)
    return _two_loop_body(sK.index_select(0, order), yK.index_select(0, order), dirv)


def _two_loop_graph(sK, yK, start_dir, delta: int):
    hit = _GRAPHS.get(id(sK))
    if hit is not None and hit[0]() is sK:
        per = hit[1]
    else:                    # identity, not tensor equality; the entry (and its graphs) dies with the history
        per = {}
        key_id = id(sK)
        _GRAPHS[key_id] = (_weakref.ref(sK, lambda _r, i=key_id: _GRAPHS.pop(i, None)), per)
    key = (yK.data_ptr(), start_dir.shape[0], start_dir.dtype)
    ent = per.get(key)
    if ent is None:
        din = start_dir.clone()
        dl = torch.zeros((), dtype=torch.int64, device=start_dir.device)
        dl.fill_(delta)
        cur = torch.cuda.current_stream(start_dir.device)
        side = torch.cuda.Stream(device=start_dir.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):            # warm-up outside capture (lazy module / kernel loads)
            _two_loop_rotating(sK, yK, din.clone(), dl)
        cur.wait_stream(side)
        g = torch.cuda.CUDAGraph()
        # no Python GC inside the capture: a collected object that releases a HIP resource (an event, an older
        # graph of a dead history) would issue a HIP call on the capturing stream and abort the capture
        gc_was = _gc.isenabled()
        _gc.disable()
        try:
            with torch.cuda.graph(g):
                dout = _two_loop_rotating(sK, yK, din.clone(), dl)
        finally:
            if gc_was:
                _gc.enable()
        ent = (g, din, dl, dout)
        per[key] = ent
        GRAPH_STATS["captures"] += 1
    g, din, dl, dout = ent
    din.copy_(start_dir)
    dl.fill_(delta)
    g.replay()
    GRAPH_STATS["replays"] += 1
    return dout.clone()


def _two_loop(ctx, grad_vec, start_dir, k):
    """L-BFGS two-loop recursion over the stored corrections (``Lbfgs.CalDirection`` :109-175).

    Kept entirely on the device: a correction pair with ``s.y == 0`` is skipped in the reference; here its
    ``rho`` is 0, which makes the same update a no-op without a host round trip.  Pairs with ``s.y < 0``
    (impossible for the convex linear losses, common for the MLP objective) are skipped the same way so
    the direction stays a descent direction.  On a GPU the recursion replays as one HIP graph."""
    sK, yK = ctx.getObj(SKYK)
    m = NUM_CORRECTIONS
    delta = k - m if k > m else 0
    l = k if k <= m else m
    if l == 0:
        return start_dir.clone()
    order = [(i + delta) % m for i in range(l)]
    if l == m and start_dir.is_cuda and graphs_enabled() and start_dir.dim() == 1 and \
            start_dir.shape[0] <= GRAPH_MAX_DIM and sK.is_contiguous() and yK.is_contiguous():
        return _two_loop_graph(sK, yK, start_dir.contiguous(), delta)
    return _two_loop_body(sK[order], yK[order], start_dir.clone())


def _update_history(ctx, grad_vec, k):
    sK, yK = ctx.getObj(SKYK)
    old = ctx.getObj("oldGradient")
    if k > 0:
        yK[(k - 1) % NUM_CORRECTIONS] = grad_vec - old
    ctx.putObj("oldGradient", grad_vec.clone())


class LbfgsDirection(ComputeFunction):
    def calc(self, ctx):
        arr = ctx.getObj(GRAD_AR)
        size = arr.shape[0] - 1
        ws = float(arr[size].item())
        g = arr[:size] / ws
        ctx.getObj(GRAD).v = g
        d = ctx.getObj(DIR)
        d.f[0] = ws
        k = ctx.getStepNo() - 1
        _update_history(ctx, g, k)
        d.v = _two_loop(ctx, g, g, k)


class OwlqnDirection(ComputeFunction):
    def __init__(self, l1: float):
        self.l1 = float(l1)

    def calc(self, ctx):
        arr = ctx.getObj(GRAD_AR)
        size = arr.shape[0] - 1
        ws = float(arr[size].item())
        g = arr[:size] / ws
        ctx.getObj(GRAD).v = g
        d = ctx.getObj(DIR)
        d.f[0] = ws
        coef = ctx.getObj(CUR).v
        if abs(self.l1) > 0.0:
            pse = torch.where(coef == 0.0,
                              torch.where(g - self.l1 > 0, g - self.l1,
                                          torch.where(g + self.l1 < 0, g + self.l1, torch.zeros_like(g))), g)
        else:
            pse = g.clone()
        ctx.getObj(PSE).v = pse
        k = ctx.getStepNo() - 1
        _update_history(ctx, g, k)
        dirv = _two_loop(ctx, g, pse, k)
        if abs(self.l1) > 0.0:
            dirv = torch.where(dirv * pse < 0, torch.zeros_like(dirv), dirv)
        d.v = dirv


class GdDirection(ComputeFunction):
    def calc(self, ctx):
        arr = ctx.getObj(GRAD_AR)
        size = arr.shape[0] - 1
        d = ctx.getObj(DIR)
        d.v = arr[:size] / arr[size]
        d.f[0] = float(arr[size].item())


class UpdateModel(ComputeFunction):
    """Adaptive-step line search result + stopping rules (``subfunc/UpdateModel.java:47-176``)."""

    def __init__(self, method: str, grad_name: str, num_search_step: int, epsilon: float, max_iter: int):
        self.method, self.grad_name, self.ns = method, grad_name, num_search_step
        self.epsilon, self.max_iter = epsilon, max_iter

    def calc(self, ctx):
        losses = (ctx.getObj(LOSS_AR) / ctx.getObj(DIR).f[0]).cpu().tolist()
        d = ctx.getObj(DIR)
        cur, mn = ctx.getObj(CUR), ctx.getObj(MIN)
        curve = ctx.getObj(CURVE)
        ratio = 1.0
        pos = -1
        for j in range(len(losses)):
            if losses[j] < losses[0]:
                losses[0] = losses[j]
                pos = j
        beta = d.f[1] / self.ns
        if pos == -1:
            eta = 0.0
            d.f[1] *= 1.0 / (self.ns * self.ns)
            cur.f = losses[0]
        elif pos == self.ns:
            eta = beta * pos
            d.f[1] *= self.ns
            d.f[1] = min(d.f[1], float(self.ns))
            ratio = abs((cur.f - losses[pos]) / cur.f)
            cur.f = losses[self.ns]
        else:
            eta = beta * pos
            ratio = abs((cur.f - losses[pos]) / cur.f)
            cur.f = losses[pos]
        step = ctx.getStepNo()
        curve[step - 1] = cur.f
        if ctx.getTaskId() == 0:
            ctx.logMetric("loss", cur.f)
        k = step - 1
        if self.method == OptimMethodName.OWLQN:
            sK, _ = ctx.getObj(SKYK)
            val = cur.v
            new = val - d.v * eta
            pse = ctx.getObj(PSE).v
            new = torch.where(val.abs() > 0.0, torch.where(new * val < 0, torch.zeros_like(new), new),
                              torch.where(new * pse > 0, torch.zeros_like(new), new))
            sK[k % NUM_CORRECTIONS] = new - val
            cur.v = new
        elif self.method == OptimMethodName.LBFGS:
            sK, _ = ctx.getObj(SKYK)
            sK[k % NUM_CORRECTIONS] = d.v * (-eta)
            cur.v = cur.v - eta * d.v
        else:
            cur.v = cur.v - eta * d.v
        if cur.f < mn.f:
            mn.f = cur.f
            mn.v = cur.v.clone()
        # stopping rules
        gnorm = float(ctx.getObj(self.grad_name).v.norm().item())
        if cur.f < self.epsilon or gnorm < self.epsilon:
            d.f[0] = -1.0
        elif step > self.max_iter - 1:
            d.f[0] = -1.0
        elif d.f[1] < EPS:
            d.f[0] = -1.0
        elif ratio < self.epsilon and gnorm < math.sqrt(self.epsilon):
            d.f[0] = -1.0
        hist = ctx.getObj("history")
        if hist is not None:
            hist.append({"step": step, "loss": cur.f, "gradNorm": gnorm, "learningRate": d.f[1]})


class SgdSubGradient(ComputeFunction):
    def __init__(self, fraction: float, seed: int = 0):
        self.fraction, self.seed = fraction, seed

    def calc(self, ctx):
        data: LabeledData = ctx.getObj(TRAIN)
        obj: OptimObjFunc = ctx.getObj(OBJ)
        n = len(data)
        bs = int(n * self.fraction)
        gen = ctx.getObj("sgdGen")
        if gen is None:
            gen = torch.Generator(device="cpu").manual_seed(self.seed * 1000003 + ctx.getTaskId())
            ctx.putObj("sgdGen", gen)
        coef = ctx.getObj(MIN).v
        if bs > 0:
            idx = torch.randint(0, n, (bs,), generator=gen).to(data.device)
            mb = data[idx]
            g, ws = obj.calc_gradient(mb, coef)
            loss, _ = obj.calc_obj_value(mb, coef)
        else:
            g, ws, loss = torch.zeros_like(coef), 0.0, 0.0
        buf = torch.empty(coef.shape[0] + 2, dtype=torch.float64, device=coef.device)
        buf[:-2] = g * ws
        buf[-2] = ws
        buf[-1] = loss
        ctx.putObj(GRAD_AR, buf)


class SgdUpdate(ComputeFunction):
    def __init__(self, max_iter: int, epsilon: float, lr: float):
        self.max_iter, self.epsilon, self.lr = max_iter, epsilon, lr

    def calc(self, ctx):
        arr = ctx.getObj(GRAD_AR)
        size = arr.shape[0] - 2
        d = ctx.getObj(DIR)
        ws = float(arr[size].item())
        d.v = arr[:size] / ws if ws != 0 else torch.zeros_like(arr[:size])
        d.f = [ws, float(arr[size + 1].item())]
        m = ctx.getObj(MIN)
        step = ctx.getStepNo()
        eta = self.lr / (float(d.v.abs().max().item()) + math.sqrt(step))
        m.v = m.v - eta * d.v
        gnorm = float(d.v.norm().item())
        if gnorm < self.epsilon or step > self.max_iter - 1:
            d.f[0] = -1.0


class NewtonGradHess(ComputeFunction):
    def calc(self, ctx):
        data = ctx.getObj(TRAIN)
        obj = ctx.getObj(OBJ)
        coef = ctx.getObj(CUR).v
        H, g, ws, loss = obj.calc_hessian_gradient_loss(data, coef)
        size = coef.shape[0]
        buf = torch.empty(size + size * size + 2, dtype=torch.float64, device=coef.device)
        buf[:size] = g
        buf[size:size + size * size] = H.reshape(-1)
        buf[-2] = ws
        buf[-1] = loss
        ctx.putObj(GH_AR, buf)


class NewtonUpdate(ComputeFunction):
    def __init__(self, max_iter: int, epsilon: float):
        self.max_iter, self.epsilon = max_iter, epsilon

    def calc(self, ctx):
        arr = ctx.getObj(GH_AR)
        cur, mn, d = ctx.getObj(CUR), ctx.getObj(MIN), ctx.getObj(DIR)
        size = cur.v.shape[0]
        ws = float(arr[-2].item())
        g = arr[:size] / ws
        H = arr[size:size + size * size].reshape(size, size) / ws
        loss = float(arr[-1].item()) / ws
        gnorm = float(g.norm().item())
        norm = 1.0 / float(g.abs().sum().item()) if float(g.abs().sum().item()) > 0 else 1.0
        H = H * norm
        g = g * norm
        x = torch.linalg.lstsq(H.cpu(), g.cpu()[:, None]).solution[:, 0].to(g.device)
        cur.v = cur.v - x
        cur.f = loss
        d.v = x
        d.f = [ws, loss]
        curve = ctx.getObj(CURVE)
        step = ctx.getStepNo()
        curve[step - 1] = loss
        if cur.f < mn.f:
            mn.f = cur.f
            mn.v = cur.v.clone()
        if cur.f < self.epsilon or gnorm < self.epsilon or step > self.max_iter - 1:
            d.f[0] = -1.0


class IterTermination(CompareCriterionFunction):
    def calc(self, ctx) -> bool:
        return ctx.getObj(DIR).f[0] < 0.0


class OutputModel(CompleteResultFunction):
    def calc(self, ctx):
        if ctx.getTaskId() != 0:
            return None
        mn = ctx.getObj(MIN)
        curve = ctx.getObj(CURVE)
        eff = len(curve)
        for i, v in enumerate(curve):
            if np.isinf(v):
                eff = i
                break
        coef = mn.v.detach().cpu().numpy().astype(np.float64)
        if not np.all(np.isfinite(coef)):
            raise RuntimeError("Optimization result has NAN or infinite value, coefficient is invalid")
        return [(coef, np.asarray(curve[:eff], dtype=np.float64))]


def optimize(obj: OptimObjFunc, data: LabeledData, dim: int, params: Params, method: Optional[str] = None,
             env=None, init_coef: Optional[torch.Tensor] = None, history: Optional[list] = None
             ) -> Tuple[np.ndarray, np.ndarray]:
    """Run the selected optimizer over this rank's partition; returns (coef, lossCurve) on every rank.

    Method selection mirrors ``BaseLinearModelTrainBatchOp.optimize`` :229-269: explicit ``optimMethod``,
    else OWL-QN when ``l1 > 0``, else L-BFGS."""
    from ...common.mlenv import MLEnvironmentFactory

    def pget(name, default):
        return params.get(name) if params.contains(name) and params.get(name) is not None else default

    if method is None:
        om = pget("optimMethod", None)
        method = (om.name if hasattr(om, "name") else str(om)) if om is not None else \
            (OptimMethodName.OWLQN if obj.l1 > 0 else OptimMethodName.LBFGS)
    method = {"LBFGS": "LBFGS", "OWLQN": "OWLQN", "GD": "GD", "SGD": "SGD", "NEWTON": "Newton"}[method.upper()]
    max_iter = int(pget("maxIter", 100))
    epsilon = float(pget("epsilon", 1.0e-6))
    ns = int(pget("numSearchStep", 4))
    env = env or MLEnvironmentFactory.getDefault()
    dev = data.device
    if init_coef is None:
        init_coef = torch.zeros(dim, dtype=torch.float64, device=dev)
        init_coef[0] = 1.0e-3   # Optimizer.initCoefZeros
    q = IterativeComQueue().setMLEnvironment(env).setJobName(f"optim.{method}")
    q.initWithPartitionedData(TRAIN, data)
    try:
        q.setRowsPerStep(len(data))
    except TypeError:
        pass
    q.initWithBroadcastData(MODEL, init_coef.to(dev))
    q.initWithBroadcastData(OBJ, obj)
    q.add(_Preallocate(max_iter, method))
    if method == OptimMethodName.SGD:
        lr = float(pget("learningRate", 0.1))
        frac = float(pget("miniBatchFraction", 0.1))
        q.add(SgdSubGradient(frac, int(pget("randomSeed", 0)))).add(AllReduce(GRAD_AR)) \
            .add(SgdUpdate(max_iter, epsilon, lr))
    elif method == OptimMethodName.NEWTON:
        q.add(NewtonGradHess()).add(AllReduce(GH_AR)).add(NewtonUpdate(max_iter, epsilon))
    else:
        q.add(CalcGradient()).add(AllReduce(GRAD_AR))
        if method == OptimMethodName.LBFGS:
            q.add(LbfgsDirection())
            gname = GRAD
        elif method == OptimMethodName.OWLQN:
            q.add(OwlqnDirection(obj.l1))
            gname = GRAD
        else:
            q.add(GdDirection())
            gname = DIR
        q.add(CalcLosses(method, ns)).add(AllReduce(LOSS_AR)) \
            .add(UpdateModel(method, gname, ns, epsilon, max_iter))
    if history is not None:
        q.initWithBroadcastData("history", history)
    q.setCompareCriterionOfNode0(IterTermination(), replicated=True).closeWith(OutputModel()).setMaxIter(max_iter)
    rows = q.exec()
    coef, curve = rows[0]
    return coef, curve
