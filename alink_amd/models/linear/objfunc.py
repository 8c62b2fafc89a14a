"""Loss functions and optimisation objectives, vectorised over a partition's sample matrix.

Reference semantics (per-sample Java loops) — ``A/operator/common/optim/objfunc/OptimObjFunc.java:21-266``,
``A/operator/common/linear/UnaryLossObjFunc.java:17-140``, ``unarylossfunc/*.java``,
``SoftmaxObjFunc.java`` and ``AftRegObjFunc.java``.  Every quantity here is one batched tensor expression
(GEMV/GEMM + elementwise) over ``LabeledData`` living on the rank's device; the optimizers in ``optim.py``
all-reduce the partial sums exactly where the reference does.

Conventions kept from the reference:
* ``calc_gradient`` returns the *local* gradient normalised by the local weight sum plus the L1/L2 terms,
  together with the weight sum; the optimizer ships ``grad * weightSum`` (so regularisation is counted once
  after the global division).
* ``calc_search_values`` returns UNNORMALISED weighted data losses (no regularisation) at
  ``coef - i * beta * dir`` for ``i = 0..numStep``.
* L2 term is ``l2 * |w|^2`` (gradient ``2 * l2 * w``), L1 is ``l1 * |w|_1``.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from ...ops import softmax as softmax_ops
from ..common.features import FeatureMatrix

__all__ = ["LabeledData", "UnaryLossFunc", "LogLossFunc", "LogisticLossFunc", "SquareLossFunc", "HingeLossFunc",
           "SmoothHingeLossFunc", "PerceptronLossFunc", "ExponentialLossFunc", "HuberLossFunc", "SvrLossFunc",
           "ZeroOneLossFunc", "OptimObjFunc", "UnaryLossObjFunc", "SoftmaxObjFunc", "AftRegObjFunc"]


class LabeledData:
    """(weight, label, features) of one partition: ``X`` FeatureMatrix, ``y``/``w`` [n] float64."""

    def __init__(self, X: FeatureMatrix, y: torch.Tensor, w: torch.Tensor):
        self.X, self.y, self.w = X, y, w

    def __len__(self):
        return self.X.nrows

    def __getitem__(self, sl):
        if isinstance(sl, slice):
            return LabeledData(self.X[sl], self.y[sl], self.w[sl])
        return LabeledData(self.X.take(sl), self.y[sl], self.w[sl])

    @property
    def device(self):
        return self.y.device


# ---------------------------------------------------------------------------------------------------
# unary losses  l(eta, y)  (eta = x . w)
# ---------------------------------------------------------------------------------------------------
class UnaryLossFunc:
    def loss(self, eta, y):
        raise NotImplementedError

    def derivative(self, eta, y):
        raise NotImplementedError

    def second_derivative(self, eta, y):
        raise NotImplementedError


class LogLossFunc(UnaryLossFunc):
    """log(1 + exp(-y eta)) with the reference's cut-offs (d < -37 -> -d, d > 34 -> 0)."""

    def loss(self, eta, y):
        d = eta * y
        mid = torch.log1p(torch.exp(-d.clamp(-37.0, 34.0)))
        return torch.where(d < -37, -d, torch.where(d > 34, torch.zeros_like(d), mid))

    def derivative(self, eta, y):
        d = eta * y
        mid = -y / (torch.exp(d.clamp(-37.0, 34.0)) + 1.0)
        return torch.where(d < -37, -y, torch.where(d > 34, torch.zeros_like(d), mid))

    def second_derivative(self, eta, y):
        t = y / (1.0 + torch.exp((eta * y).clamp(max=700.0)))
        return t * (y - t)


class LogisticLossFunc(LogLossFunc):
    _ln2 = math.log(2.0)

    def loss(self, eta, y):
        return super().loss(eta, y) / self._ln2

    def derivative(self, eta, y):
        d = eta * y
        return torch.where(d < -37, -y / self._ln2, -y / (torch.exp(d.clamp(max=700.0)) + 1.0) / self._ln2)

    def second_derivative(self, eta, y):
        return super().second_derivative(eta, y) / self._ln2


class SquareLossFunc(UnaryLossFunc):
    def loss(self, eta, y):
        return 0.5 * (eta - y) ** 2

    def derivative(self, eta, y):
        return eta - y

    def second_derivative(self, eta, y):
        return torch.ones_like(eta)


class HingeLossFunc(UnaryLossFunc):
    def loss(self, eta, y):
        return torch.clamp(1 - eta * y, min=0.0)

    def derivative(self, eta, y):
        return torch.where(eta * y < 1, -y, torch.zeros_like(y))

    def second_derivative(self, eta, y):
        return torch.zeros_like(eta)


class SmoothHingeLossFunc(UnaryLossFunc):
    def loss(self, eta, y):
        d = eta * y
        return torch.where(d <= 0, 0.5 - d, torch.where(d >= 1.0, torch.zeros_like(d), 0.5 * (1 - d) ** 2))

    def derivative(self, eta, y):
        d = eta * y
        return torch.where(d <= 0, -y, torch.where(d >= 1.0, torch.zeros_like(d), (1 - d) * (-y)))

    def second_derivative(self, eta, y):
        d = eta * y
        return torch.where((d >= 1.0) | (d <= 0.0), torch.zeros_like(d), y * y)


class PerceptronLossFunc(UnaryLossFunc):
    def loss(self, eta, y):
        return torch.clamp(-eta * y, min=0.0)

    def derivative(self, eta, y):
        return torch.where(eta * y < 0, -y, torch.zeros_like(y))

    def second_derivative(self, eta, y):
        return torch.zeros_like(eta)


class ExponentialLossFunc(UnaryLossFunc):
    def loss(self, eta, y):
        return torch.exp(-eta * y)

    def derivative(self, eta, y):
        return -y * torch.exp(-eta * y)

    def second_derivative(self, eta, y):
        return y * y * torch.exp(-eta * y)


class HuberLossFunc(UnaryLossFunc):
    def __init__(self, delta: float):
        if delta <= 0:
            raise ValueError("Parameter delta must be positive.")
        self.delta = float(delta)

    def loss(self, eta, y):
        x = (eta - y).abs()
        return torch.where(x > self.delta, self.delta * (x - self.delta / 2), x * x / 2)

    def derivative(self, eta, y):
        x = eta - y
        return torch.where(x.abs() > self.delta, torch.sign(x) * self.delta, x)

    def second_derivative(self, eta, y):
        return torch.where((eta - y).abs() > self.delta, torch.zeros_like(eta), torch.ones_like(eta))


class SvrLossFunc(UnaryLossFunc):
    def __init__(self, epsilon: float):
        if epsilon < 0:
            raise ValueError("Parameter epsilon can not be negtive.")
        self.epsilon = float(epsilon)

    def loss(self, eta, y):
        return torch.clamp((eta - y).abs() - self.epsilon, min=0.0)

    def derivative(self, eta, y):
        x = eta - y
        return torch.where(x.abs() > self.epsilon, torch.sign(x), torch.zeros_like(x))

    def second_derivative(self, eta, y):
        return torch.zeros_like(eta)


class ZeroOneLossFunc(UnaryLossFunc):
    def loss(self, eta, y):
        return (eta * y < 0).to(eta.dtype)

    def derivative(self, eta, y):
        return torch.zeros_like(eta)

    def second_derivative(self, eta, y):
        return torch.zeros_like(eta)


# ---------------------------------------------------------------------------------------------------
# objectives
# ---------------------------------------------------------------------------------------------------
class OptimObjFunc:
    def __init__(self, l1: float = 0.0, l2: float = 0.0):
        self.l1 = float(l1 or 0.0)
        self.l2 = float(l2 or 0.0)

    def has_second_derivative(self) -> bool:
        return False

    # -- to implement --
    def loss_per_sample(self, data: LabeledData, coef: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def grad_sum(self, data: LabeledData, coef: torch.Tensor) -> torch.Tensor:
        """sum_i (sample-weighted) d loss_i / d coef  (no regularisation)."""
        raise NotImplementedError

    def hessian_sum(self, data: LabeledData, coef: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError("loss function can't support second derivative, newton precondition can "
                                  "not work.")

    def sample_weight(self, data: LabeledData) -> torch.Tensor:
        return data.w

    # -- reference API --
    def _reg_grad(self, coef):
        g = torch.zeros_like(coef)
        if self.l2 != 0.0:
            g = g + 2.0 * self.l2 * coef
        if self.l1 != 0.0:
            g = g + torch.sign(coef) * self.l1
        return g

    def calc_gradient(self, data: LabeledData, coef: torch.Tensor) -> Tuple[torch.Tensor, float]:
        ws = float(self.sample_weight(data).sum().item()) if len(data) else 0.0
        g = self.grad_sum(data, coef) if len(data) else torch.zeros_like(coef)
        if ws > 0.0:
            g = g / ws
        return g + self._reg_grad(coef), ws

    def calc_obj_value(self, data: LabeledData, coef: torch.Tensor) -> Tuple[float, float]:
        ws = float(self.sample_weight(data).sum().item()) if len(data) else 0.0
        f = float((self.loss_per_sample(data, coef) * self.sample_weight(data)).sum().item()) if len(data) else 0.0
        if ws != 0.0:
            f /= ws
        if self.l1 != 0.0:
            f += self.l1 * float(coef.abs().sum().item())
        if self.l2 != 0.0:
            f += self.l2 * float((coef * coef).sum().item())
        return f, ws

    def calc_hessian_gradient_loss(self, data: LabeledData, coef: torch.Tensor):
        """(hessian_sum, grad_sum, weightSum, lossSum) with L1/L2 scaled by the weight sum."""
        if not self.has_second_derivative():
            raise NotImplementedError("loss function can't support second derivative, newton precondition can "
                                      "not work.")
        d = coef.shape[0]
        if len(data):
            H = self.hessian_sum(data, coef)
            g = self.grad_sum(data, coef)
            ws = float(self.sample_weight(data).sum().item())
            loss = float(self.loss_per_sample(data, coef).sum().item())
        else:
            H = torch.zeros((d, d), dtype=coef.dtype, device=coef.device)
            g, ws, loss = torch.zeros_like(coef), 0.0, 0.0
        if self.l1 != 0.0:
            g = g + torch.sign(coef) * self.l1 * ws
        if self.l2 != 0.0:
            t = self.l2 * 2 * ws
            g = g + coef * t
            H = H + torch.eye(d, dtype=H.dtype, device=H.device) * t
        return H, g, ws, loss

    def _losses_at(self, data, coefs: torch.Tensor) -> torch.Tensor:
        """weighted data loss for each column of coefs [d, S]."""
        return torch.stack([(self.loss_per_sample(data, coefs[:, i]) * self.sample_weight(data)).sum()
                            for i in range(coefs.shape[1])])

    def calc_search_values(self, data: LabeledData, coef, dirv, beta: float, num_step: int) -> torch.Tensor:
        steps = torch.arange(num_step + 1, dtype=coef.dtype, device=coef.device) * beta
        coefs = coef[:, None] - dirv[:, None] * steps[None, :]
        if not len(data):
            return torch.zeros(num_step + 1, dtype=coef.dtype, device=coef.device)
        return self._losses_at(data, coefs)

    def constraint_calc_search_values(self, data: LabeledData, coef, dirv, beta: float, num_step: int):
        steps = torch.arange(num_step + 1, dtype=coef.dtype, device=coef.device) * beta
        coefs = coef[:, None] - dirv[:, None] * steps[None, :]
        coefs = torch.where(coefs * coef[:, None] < 0, torch.zeros_like(coefs), coefs)
        if not len(data):
            return torch.zeros(num_step + 1, dtype=coef.dtype, device=coef.device)
        return self._losses_at(data, coefs)


class UnaryLossObjFunc(OptimObjFunc):
    """Generalised linear loss l(x.w, y) — LR (log loss), SVM (smooth hinge), LinearReg (square), SVR,
    Perceptron (``BaseLinearModelTrainBatchOp.getObjFunction`` :276-311)."""

    def __init__(self, loss: UnaryLossFunc, l1: float = 0.0, l2: float = 0.0):
        super().__init__(l1, l2)
        self.unary = loss

    def has_second_derivative(self):
        return True

    def loss_per_sample(self, data, coef):
        return self.unary.loss(data.X.mv(coef), data.y)

    def grad_sum(self, data, coef):
        from ...ops import _lib, linear as lops
        X = data.X.dense
        code = lops.loss_code(self.unary)
        if code is not None and lops.hip_linear_supported(X) and (_lib.available()
                                                                  or not _lib.torch_fallback_allowed()):
            return lops.linear_grad_hip(X, data.y, data.w, coef, code[0], code[1])[0]   # one pass over X
        if code is not None and lops.hip_sparse_supported(data.X):
            return lops.sparse_grad_hip(data.X, data.y, data.w, coef, code[0], code[1])[0]   # CSR + CSC kernels
        eta = data.X.mv(coef)
        return data.X.rmv(data.w * self.unary.derivative(eta, data.y), coef.shape[0])

    def hessian_sum(self, data, coef):
        eta = data.X.mv(coef)
        return data.X.gram(self.unary.second_derivative(eta, data.y) * data.w, coef.shape[0])

    def calc_search_values(self, data, coef, dirv, beta, num_step):
        if not len(data):
            return torch.zeros(num_step + 1, dtype=coef.dtype, device=coef.device)
        from ...ops import _lib, linear as lops
        X = data.X.dense
        code = lops.loss_code(self.unary)
        if code is not None and lops.hip_linear_supported(X) and num_step + 1 <= lops.SEARCH_MAX_STEPS and \
                (_lib.available() or not _lib.torch_fallback_allowed()) and not lops.k14_disabled():
            # K14: both margins and all num_step+1 losses in one pass over X
            return lops.search_losses_hip(X, data.y, data.w, coef, dirv, code[0], code[1], beta, num_step + 1)
        E = data.X.mm(torch.stack([coef, dirv], 1))  # one pass over X for both margins
        steps = torch.arange(num_step + 1, dtype=coef.dtype, device=coef.device)
        etas = E[:, :1] - steps[None, :] * (E[:, 1:2] * beta)
        return (self.unary.loss(etas, data.y[:, None]) * data.w[:, None]).sum(0)


class SoftmaxObjFunc(OptimObjFunc):
    """Multinomial logistic loss with K-1 free coefficient blocks (class K-1 is the pivot),
    coef layout ``[k][featDim]`` flattened (``SoftmaxObjFunc.java``)."""

    def __init__(self, num_classes: int, l1: float = 0.0, l2: float = 0.0):
        super().__init__(l1, l2)
        self.k1 = int(num_classes) - 1

    def has_second_derivative(self):
        return True

    def _eta(self, data, coef):
        W = coef.reshape(self.k1, -1)
        return data.X.mm(W.T)  # [n, k1]

    @staticmethod
    def _logsumexp1(eta):
        z = torch.zeros((eta.shape[0], 1), dtype=eta.dtype, device=eta.device)
        return torch.logsumexp(torch.cat([eta, z], 1), 1)

    def loss_per_sample(self, data, coef):
        eta = self._eta(data, coef)
        yk = data.y.long()
        lin = torch.where(yk < self.k1, eta.gather(1, yk.clamp(max=self.k1 - 1)[:, None])[:, 0],
                          torch.zeros_like(data.y))
        return self._logsumexp1(eta) - lin

    def _phi(self, eta):
        lse = self._logsumexp1(eta)
        return torch.exp(eta - lse[:, None])

    def grad_sum(self, data, coef):
        # K16: w * (softmax - onehot) in one fused pass over the logits (torch formulas on the CPU)
        R, _ = softmax_ops.softmax_grad(self._eta(data, coef), data.y, data.w)
        G = data.X.rmm(R, coef.shape[0] // self.k1)  # [m, k1]
        return G.T.reshape(-1)

    def hessian_sum(self, data, coef):
        m = coef.shape[0] // self.k1
        phi = self._phi(self._eta(data, coef))
        H = torch.zeros((self.k1 * m, self.k1 * m), dtype=coef.dtype, device=coef.device)
        for s in range(self.k1):
            for t in range(s, self.k1):
                scale = (phi[:, s] - phi[:, s] ** 2) if s == t else -phi[:, s] * phi[:, t]
                blk = data.X.gram(scale * data.w, m)
                H[s * m:(s + 1) * m, t * m:(t + 1) * m] = blk
                if s != t:
                    H[t * m:(t + 1) * m, s * m:(s + 1) * m] = blk.T
        return H

    def calc_search_values(self, data, coef, dirv, beta, num_step):
        if not len(data):
            return torch.zeros(num_step + 1, dtype=coef.dtype, device=coef.device)
        # every trial step's loss from one read of the two logit blocks (K16 search epilogue)
        return softmax_ops.softmax_search(self._eta(data, coef), self._eta(data, dirv), data.y, data.w, beta,
                                          num_step + 1)


class AftRegObjFunc(OptimObjFunc):
    """Accelerated-failure-time (Weibull) negative log-likelihood; the last coefficient is log(sigma) and the
    sample "weight" slot carries the censor indicator, exactly as ``AftRegObjFunc.java`` uses ``f0``."""

    def has_second_derivative(self):
        return True

    def sample_weight(self, data):
        # every sample counts once (AftRegObjFunc overrides calcObjValue/calcGradient/calcSearchValues with
        # weightSum += 1.0); the weight slot is the censor indicator used inside the loss
        return torch.ones_like(data.w)

    def _parts(self, data, coef):
        # x . coef over the vector's own length (AftRegObjFunc.getDotProduct): training vectors have d - 1
        # entries, so log(sigma) stays out of the product
        log_sigma = coef[-1]
        sigma = torch.exp(log_sigma)
        eps = (data.y - data.X.mv(coef)) / sigma
        return log_sigma, sigma, eps

    def loss_per_sample(self, data, coef):
        log_sigma, _, eps = self._parts(data, coef)
        return data.w * (log_sigma - eps) + torch.exp(eps)

    def grad_sum(self, data, coef):
        d = coef.shape[0]
        _, sigma, eps = self._parts(data, coef)
        mult = data.w - torch.exp(eps)
        g = data.X.rmv(mult / sigma, d).clone()
        g[d - 1] += (data.w + mult * eps).sum()
        return g

    def hessian_sum(self, data, coef):
        d = coef.shape[0]
        _, sigma, eps = self._parts(data, coef)
        H = data.X.gram(torch.exp(eps) / (sigma * sigma), d).clone()
        H[d - 1, d - 1] += (eps * (torch.exp(eps) * (1 + eps) - data.w)).sum()
        return H
