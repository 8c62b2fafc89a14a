"""Generalized linear models: IRLS over device-resident sufficient statistics.

Reference: ``A/operator/common/regression/glm/GlmUtil.java`` (IRLS ``train`` :133-186, weighted least squares
from ``WeightStat`` :1190-1435, residuals :346-425, summary / AIC :215-335, :505-692), ``FamilyLink.java``
(working label / weight :151-167), families ``glm/famliy/*`` and links ``glm/link/*``,
``GlmTrainBatchOp.java``, ``GlmEvaluationBatchOp.java``, ``GlmModelMapper.java``, ``GlmModelDataConverter.java``.

MI355X-first design: the reference reduces a ``WeightStat`` (sums, packed ``A^T W A``, ``A^T W b``) to ONE
task and solves there (``setParallelism(1)``).  Here every rank builds its statistics as one
``[X|1|b]^T diag(w) [X|1|b]`` GEMM on its device shard, the statistics are summed with a single all-reduce,
and every rank solves the (k+1)x(k+1) system itself — no gather to one node, no broadcast of the model.
"""
from __future__ import annotations

import json
import math
from typing import List, Optional, Sequence

import numpy as np
import torch

from ...ops.gemm import tn_matmul
from ...common.javafmt import gson_dumps
from ...common.mapper import ModelMapper, OutputColsHelper
from ...common.model import SimpleModelDataConverter
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import Types
from ...parallel import comm

__all__ = ["FamilyLink", "GlmModelData", "GlmModelDataConverter", "GlmModelMapper", "train_glm", "glm_residuals",
           "glm_summary", "preprocess", "family_link_of", "RESIDUAL_COLS", "WlsModel"]

EPSILON = 1e-16
DELTA = 0.1
JAVA_MIN_VALUE = 4.9e-324
JAVA_MAX_VALUE = 1.7976931348623157e308
RESIDUAL_COLS = ["label", "weight", "offset", "pred", "residualdevianceResiduals", "pearsonResiduals",
                 "workingResiduals", "responseResiduals"]


def _name(v) -> Optional[str]:
    if v is None:
        return None
    return v.name if hasattr(v, "name") else str(v)


# ---------------------------------------------------------------------------------------------------
# links (vectorised over torch tensors)
# ---------------------------------------------------------------------------------------------------
class _Link:
    name = ""


class Identity(_Link):
    name = "identity"

    def link(self, mu):
        return mu

    def unlink(self, eta):
        return eta

    def derivative(self, mu):
        return torch.ones_like(mu)


class Log(_Link):
    name = "log"

    def link(self, mu):
        return torch.log(mu)

    def unlink(self, eta):
        return torch.exp(eta)

    def derivative(self, mu):
        return 1.0 / mu


class Logit(_Link):
    name = "logit"

    def link(self, mu):
        return torch.log(mu / (1.0 - mu))

    def unlink(self, eta):
        return 1.0 / (1.0 + torch.exp(-eta))

    def derivative(self, mu):
        return 1.0 / (mu * (1.0 - mu))


class Inverse(_Link):
    name = "inverse"

    def link(self, mu):
        return 1.0 / mu

    def unlink(self, eta):
        return 1.0 / eta

    def derivative(self, mu):
        return -torch.pow(mu, -2.0)


class Sqrt(_Link):
    name = "sqrt"

    def link(self, mu):
        return torch.sqrt(mu)

    def unlink(self, eta):
        return eta * eta

    def derivative(self, mu):
        return 1.0 / (2.0 * torch.sqrt(mu))


class CLogLog(_Link):
    name = "cloglog"

    def link(self, mu):
        return torch.log(-torch.log(1 - mu))

    def unlink(self, eta):
        return 1.0 - torch.exp(-torch.exp(eta))

    def derivative(self, mu):
        return 1.0 / ((mu - 1.0) * torch.log(1.0 - mu))


class Probit(_Link):
    name = "probit"

    def link(self, mu):
        return torch.special.ndtri(mu)

    def unlink(self, eta):
        return torch.special.ndtr(eta)

    def derivative(self, mu):
        z = torch.special.ndtri(mu)
        return math.sqrt(2 * math.pi) * torch.exp(0.5 * z * z)


class Power(_Link):
    name = "power"

    def __init__(self, p: float):
        self.p = float(p)

    def link(self, mu):
        return torch.log(mu) if self.p == 0 else torch.pow(mu, self.p)

    def unlink(self, eta):
        return torch.exp(eta) if self.p == 0 else torch.pow(eta, 1.0 / self.p)

    def derivative(self, mu):
        return 1.0 / mu if self.p == 0 else self.p * torch.pow(mu, self.p - 1.0)


# ---------------------------------------------------------------------------------------------------
# families
# ---------------------------------------------------------------------------------------------------
def _clamp_pos(mu):
    mu = torch.where(mu < EPSILON, torch.full_like(mu, EPSILON), mu)
    return torch.where(torch.isinf(mu), torch.full_like(mu, JAVA_MAX_VALUE), mu)


class Gaussian:
    name = "gaussian"

    def __init__(self):
        self.default_link = Identity()

    def initialize(self, y, w):
        return y

    def variance(self, mu):
        return torch.ones_like(mu)

    def deviance(self, y, mu, w):
        return w * (y - mu) * (y - mu)

    def project(self, mu):
        mu = torch.where(mu == float("inf"), torch.full_like(mu, JAVA_MAX_VALUE), mu)
        return torch.where(mu == float("-inf"), torch.full_like(mu, JAVA_MIN_VALUE), mu)


class Binomial:
    name = "binomial"

    def __init__(self):
        self.default_link = Logit()

    def initialize(self, y, w):
        mu = (w * y + 0.5) / (w + 1.0)
        if bool(((mu <= 0) | (mu >= 1.0)).any()):
            raise RuntimeError("mu must be in (0, 1).")
        return mu

    def variance(self, mu):
        return mu * (1 - mu)

    def deviance(self, y, mu, w):
        def ylogy(a, b):
            return torch.where(a == 0, torch.zeros_like(a), a * torch.log(a / b))
        return 2.0 * w * (ylogy(y, mu) + ylogy(1.0 - y, 1.0 - mu))

    def project(self, mu):
        return mu.clamp(EPSILON, 1.0 - EPSILON)


class Poisson:
    name = "poisson"

    def __init__(self):
        self.default_link = Log()

    def initialize(self, y, w):
        if bool((y < 0).any()):
            raise RuntimeError("y of poisson family must be non-negative.")
        return torch.clamp(y, min=DELTA)

    def variance(self, mu):
        return mu

    def deviance(self, y, mu, w):
        ylog = torch.where(y == 0, torch.zeros_like(y), y * torch.log(y / mu))
        return 2.0 * w * (ylog - (y - mu))

    def project(self, mu):
        return _clamp_pos(mu)


class Gamma:
    name = "gamma"

    def __init__(self):
        self.default_link = Inverse()

    def initialize(self, y, w):
        if bool((y <= 0).any()):
            raise RuntimeError("y of gamma family must be positive.")
        return y

    def variance(self, mu):
        return mu * mu

    def deviance(self, y, mu, w):
        return -2.0 * w * (torch.log(y / mu) - (y - mu) / mu)

    def project(self, mu):
        return _clamp_pos(mu)


class Tweedie:
    name = "tweedie"

    def __init__(self, vp: float):
        self.vp = float(vp)
        self.default_link = Power(1 - self.vp)

    def initialize(self, y, w):
        return torch.where(y == 0, torch.full_like(y, DELTA), y)

    def variance(self, mu):
        return torch.pow(mu, self.vp)

    def deviance(self, y, mu, w):
        y1 = torch.where(y == 0, torch.ones_like(y), y)
        p1, p2 = 1 - self.vp, 2 - self.vp
        theta = torch.log(y1 / mu) if self.vp == 1 else (torch.pow(y1, p1) - torch.pow(mu, p1)) / p1
        kappa = torch.log(y1 / mu) if self.vp == 2 else (torch.pow(y, p2) - torch.pow(mu, p2)) / p2
        d = 2 * w * (y * theta - kappa)
        return torch.where(d < EPSILON, torch.full_like(d, EPSILON), d)

    def project(self, mu):
        return _clamp_pos(mu)


_LINKS = {"identity": Identity, "log": Log, "logit": Logit, "inverse": Inverse, "sqrt": Sqrt,
          "cloglog": CLogLog, "probit": Probit}


class FamilyLink:
    """``FamilyLink.java`` — family (+ variance power) and link (default = the family's canonical link)."""

    def __init__(self, family, variance_power: float = 0.0, link=None, link_power: float = 1.0):
        f = (_name(family) or "gaussian").lower()
        fams = {"gaussian": Gaussian, "binomial": Binomial, "poisson": Poisson, "gamma": Gamma}
        if f in fams:
            self.family = fams[f]()
        elif f == "tweedie":
            self.family = Tweedie(variance_power)
        else:
            raise RuntimeError("family is not support. ")
        ln = _name(link)
        if not ln:
            self.link = self.family.default_link
        elif ln.lower() == "power":
            self.link = Power(link_power)
        elif ln.lower() in _LINKS:
            self.link = _LINKS[ln.lower()]()
        else:
            raise RuntimeError("link is not support. ")

    @property
    def familyName(self):
        return self.family.name

    @property
    def linkName(self):
        return self.link.name

    def predict(self, mu):
        return self.link.link(self.family.project(mu))

    def fitted(self, eta):
        return self.family.project(self.link.unlink(eta))


def family_link_of(p) -> FamilyLink:
    def g(name, default=None):
        v = p.get(name) if p.contains(name) else default
        return default if v is None else v
    return FamilyLink(g("family", "gaussian"), float(g("variancePower", 0.0)), g("link"), float(g("linkPower", 1.0)))


# ---------------------------------------------------------------------------------------------------
# weighted least squares on all-reduced statistics (GlmUtil.WeightedLeastSquares)
# ---------------------------------------------------------------------------------------------------
class WlsModel:
    def __init__(self, coefficients, intercept, diag_inv, fit_intercept, n):
        self.coefficients = np.asarray(coefficients, dtype=np.float64)
        self.intercept = float(intercept)
        self.diagInvAtWA = np.asarray(diag_inv, dtype=np.float64)
        self.fitIntercept = bool(fit_intercept)
        self.numInstances = int(n)


def _weight_stats(X: torch.Tensor, b: torch.Tensor, w: torch.Tensor) -> np.ndarray:
    """All-reduced ``[count, wwSum, G]`` with ``G = [X|1|b]^T diag(w) [X|1|b]`` (one GEMM per rank)."""
    n = X.shape[0]
    Z = torch.cat([X, torch.ones((n, 1), dtype=X.dtype, device=X.device), b[:, None]], 1)
    G = tn_matmul(Z, Z * w[:, None])
    head = torch.stack([torch.tensor(float(n), dtype=X.dtype, device=X.device), (w * w).sum()])
    buf = torch.cat([head, G.reshape(-1)])
    comm.all_reduce(buf, "sum")
    return buf.cpu().numpy()


def _wls(stats: np.ndarray, k: int, fit_intercept: bool, reg: float, std_features: bool,
         std_label: bool) -> WlsModel:
    count = stats[0]
    G = stats[2:].reshape(k + 2, k + 2)
    aa, a_sum, ab_sum = G[:k, :k], G[:k, k], G[:k, k + 1]
    w_sum, b_sum, bb_sum = G[k, k], G[k, k + 1], G[k + 1, k + 1]
    b_mean_raw = b_sum / w_sum
    b_std_raw = math.sqrt(max(bb_sum / w_sum - b_mean_raw * b_mean_raw, 0.0))
    b_std = b_std_raw if b_std_raw != 0.0 else abs(b_mean_raw)
    if b_std == 0.0:
        b_std = 1.0
    b_mean = b_mean_raw / b_std
    a_mean_raw = a_sum / w_sum
    a_std = np.sqrt(np.maximum(np.diag(aa) / w_sum - a_mean_raw * a_mean_raw, 0.0))
    nz = a_std != 0.0
    safe = np.where(nz, a_std, 1.0)
    a_means = np.where(nz, a_mean_raw / safe, 0.0)
    ab_means = np.where(nz, ab_sum / w_sum / (safe * b_std), 0.0)
    denom = np.outer(safe, safe)
    aa_means = np.where(np.outer(nz, nz), aa / w_sum / denom, 0.0)
    lam = np.full(k, reg / b_std)
    if not std_features:
        lam = np.where(nz, lam / (safe * safe), 0.0)
    if not std_label:
        lam = lam * b_std
    aa_means = aa_means + np.diag(lam)
    if fit_intercept:
        M = np.zeros((k + 1, k + 1))
        M[:k, :k] = aa_means
        M[:k, k] = a_means
        M[k, :k] = a_means
        M[k, k] = 1.0
        rhs = np.concatenate([ab_means, [b_mean]])
    else:
        M, rhs = aa_means, ab_means
    try:
        L = np.linalg.cholesky(M)
        x = np.linalg.solve(L.T, np.linalg.solve(L, rhs))
        inv = np.linalg.inv(M)
    except np.linalg.LinAlgError:
        x = np.linalg.lstsq(M, rhs, rcond=None)[0]
        inv = np.linalg.pinv(M)
    coef = np.where(nz, x[:k] * b_std / safe, 0.0)
    intercept = x[k] * b_std if fit_intercept else 0.0
    mult = np.concatenate([a_std * a_std, [1.0]]) if fit_intercept else a_std * a_std
    with np.errstate(divide="ignore", invalid="ignore"):
        diag = np.diag(inv) / (w_sum * mult)
    return WlsModel(coef, intercept, diag, fit_intercept, count)


class GlmData:
    """One rank's preprocessed rows (``GlmUtil.preProc``): features [n,k], label, weight, offset."""

    def __init__(self, X, y, w, off):
        self.X, self.y, self.w, self.off = X, y, w, off


def _col(mt: MTable, name: Optional[str], default: float, device) -> torch.Tensor:
    if not name:
        return torch.full((mt.num_rows,), default, dtype=torch.float64, device=device)
    v = mt.col(name).values
    if isinstance(v, torch.Tensor):
        return v.to(device=device, dtype=torch.float64).reshape(-1)
    return torch.tensor([default if x is None else float(x) for x in v], dtype=torch.float64, device=device)


def preprocess(mt: MTable, feature_cols: Sequence[str], label_col: str, weight_col: Optional[str],
               offset_col: Optional[str], device) -> GlmData:
    if not feature_cols:
        raise RuntimeError("featureColNames must be set.")
    if label_col is None:
        raise RuntimeError("labelColName must be set.")
    X = torch.stack([_col(mt, c, 0.0, device) for c in feature_cols], 1)
    return GlmData(X, _col(mt, label_col, 0.0, device), _col(mt, weight_col, 1.0, device),
                   _col(mt, offset_col, 0.0, device))


def _irls(d: GlmData, fl: FamilyLink, reg: float, fit_intercept: bool, num_iter: int, eps: float) -> WlsModel:
    k = d.X.shape[1]
    if fl.familyName == "gaussian" and fl.linkName == "identity":
        return _wls(_weight_stats(d.X, d.y - d.off, d.w), k, fit_intercept, reg, True, True)
    eta0 = fl.predict(fl.family.initialize(d.y, d.w)) - d.off
    model = _wls(_weight_stats(d.X, eta0, d.w), k, fit_intercept, reg, True, True)
    for _ in range(int(num_iter)):
        beta = torch.as_tensor(model.coefficients, dtype=torch.float64, device=d.X.device)
        eta = d.X @ beta + model.intercept + d.off
        mu = fl.fitted(eta)
        deriv = fl.link.derivative(mu)
        z = eta - d.off + (d.y - mu) * deriv
        ww = d.w / (deriv * deriv * fl.family.variance(mu))
        new = _wls(_weight_stats(d.X, z, ww), k, fit_intercept, reg, False, False)
        tol = max([abs(new.intercept - model.intercept)]
                  + [abs(a - b) for a, b in zip(new.coefficients, model.coefficients)])
        model = new
        if tol <= eps:
            break
    return model


def train_glm(d: GlmData, p: Params) -> WlsModel:
    return _irls(d, family_link_of(p), float(p.get("regParam")), bool(p.get("fitIntercept")),
                 int(p.get("maxIter")), float(p.get("epsilon")))


def glm_residuals(d: GlmData, model: WlsModel, fl: FamilyLink) -> List[torch.Tensor]:
    """[pred, deviance, pearson, working, response] residual columns (``GlmUtil.residualRow``)."""
    beta = torch.as_tensor(model.coefficients, dtype=torch.float64, device=d.X.device)
    eta = d.X @ beta + model.intercept + d.off
    pred = fl.fitted(eta)
    dr = torch.sqrt(torch.clamp(fl.family.deviance(d.y, pred, d.w), min=0.0))
    dr = torch.where(d.y <= pred, -dr, dr)
    pr = (d.y - pred) * torch.sqrt(d.w) / torch.sqrt(fl.family.variance(pred))
    wr = (d.y - pred) * fl.link.derivative(pred)
    return [pred, dr, pr, wr, d.y - pred]


def _allsum(vals: List[float]) -> List[float]:
    t = torch.tensor(vals, dtype=torch.float64)
    comm.all_reduce(t, "sum")
    return t.tolist()


def glm_summary(d: GlmData, model: WlsModel, fl: FamilyLink, reg: float, num_iter: int, eps: float,
                fit_intercept: bool) -> str:
    """Summary JSON of ``GlmUtil.aggSummary``: deviance, null deviance, dispersion, AIC, standard errors,
    t- and p-values (``diagInvAtWA`` is the true diagonal of ``(A^T W A)^-1``)."""
    from scipy import stats as st
    k = d.X.shape[1]
    pred, _, pr, _, _ = glm_residuals(d, model, fl)
    if fit_intercept:
        if fl.familyName == "gaussian" and fl.linkName == "identity":
            s = _allsum([float((d.w * (d.y - d.off)).sum()), float(d.w.sum())])
            intercept = s[0] / s[1]
        else:
            intercept = _irls(GlmData(d.X[:, :0], d.y, d.w, d.off), fl, reg, True, num_iter, eps).intercept
    else:
        intercept = 0.0
    null_dev = fl.family.deviance(d.y, fl.link.unlink(intercept + d.off), d.w)
    dev = fl.family.deviance(d.y, pred, d.w)
    disp = torch.ones_like(pred) if fl.familyName in ("binomial", "poisson") else pr * pr
    null_dev_s, dev_s, disp_s, w_s, cnt = _allsum([float(null_dev.sum()), float(dev.sum()), float(disp.sum()),
                                                  float(d.w.sum()), float(d.y.shape[0])])
    count = int(round(cnt))
    fam = fl.familyName
    if fam == "tweedie":
        aic = None
    elif fam == "binomial":
        wt, kk = torch.round(d.w), torch.round(d.y * d.w)
        lp = (torch.lgamma(wt + 1) - torch.lgamma(kk + 1) - torch.lgamma(wt - kk + 1)
              + kk * torch.log(pred) + (wt - kk) * torch.log(1 - pred))
        aic = -2.0 * _allsum([float(torch.where(wt == 0, torch.zeros_like(lp), lp).sum())])[0]
    elif fam == "gamma":
        dd = dev_s / w_s
        a = 1.0 / dd
        theta = 1.0 / (pred * dd)
        logd = (a - 1) * torch.log(d.y) - d.y / theta - math.lgamma(a) - a * torch.log(theta)
        aic = -2.0 * _allsum([float((d.w * logd).sum())])[0] + 2.0
    elif fam == "poisson":
        kk = torch.floor(d.y)
        aic = -2.0 * _allsum([float((d.w * (kk * torch.log(pred) - pred - torch.lgamma(kk + 1))).sum())])[0]
    else:
        wt = _allsum([float(torch.log(d.w).sum())])[0]
        aic = count * (math.log(dev_s / count * 2.0 * math.pi) + 1.0) + 2.0 - wt
    rank = k + 1 if fit_intercept else k
    dof = count - rank
    dispersion = 1.0 if fam in ("binomial", "poisson") else disp_s / dof
    stderr = np.sqrt(model.diagInvAtWA * dispersion)
    tvals = np.zeros_like(stderr)
    with np.errstate(divide="ignore", invalid="ignore"):
        tvals[:k] = model.coefficients / stderr[:k]
        if fit_intercept:
            tvals[k] = model.intercept / stderr[k]
    if fam in ("binomial", "poisson"):
        pvals = 2.0 * (1.0 - st.norm.cdf(np.abs(tvals)))
    else:
        pvals = 2.0 * (1.0 - st.t.cdf(np.abs(tvals), max(dof, 1)))
    summary = {
        "rank": rank, "degreeOfFreedom": dof, "residualDegreeOfFreeDom": dof,
        "residualDegreeOfFreedomNull": count - 1 if fit_intercept else count,
        "aic": JAVA_MAX_VALUE if aic is None else aic + 2 * rank, "dispersion": dispersion, "deviance": dev_s,
        "nullDeviance": JAVA_MIN_VALUE if math.isnan(null_dev_s) else null_dev_s,
        "coefficients": model.coefficients.tolist(), "intercept": model.intercept,
        "coefficientStandardErrors": stderr.tolist(), "tValues": tvals.tolist(), "pValues": pvals.tolist()}
    return gson_dumps(summary, java_map_order=False)


# ---------------------------------------------------------------------------------------------------
# model format + predict
# ---------------------------------------------------------------------------------------------------
class GlmModelData:
    def __init__(self):
        self.featureColNames = None
        self.offsetColName = None
        self.weightColName = None
        self.labelColName = None
        self.familyName = "Gaussian"
        self.variancePower = 0.0
        self.linkName = None
        self.linkPower = 1.0
        self.coefficients = None
        self.intercept = 0.0
        self.diagInvAtWA = None
        self.fitIntercept = True
        self.regParam = 0.0
        self.numIter = 10
        self.epsilon = 1e-5


class GlmModelDataConverter(SimpleModelDataConverter):
    """Meta = train params; data = [coefficients, intercept, diagInvAtWA] JSON (``GlmModelDataConverter.java``)."""

    def serializeModel(self, m: GlmModelData):
        meta = Params()
        meta.set("featureCols", list(m.featureColNames))
        meta.set("offsetCol", m.offsetColName)
        meta.set("weightCol", m.weightColName)
        meta.set("labelCol", m.labelColName)
        meta.set("family", _name(m.familyName))
        meta.set("variancePower", float(m.variancePower))
        meta.set("link", _name(m.linkName))
        meta.set("linkPower", float(m.linkPower))
        meta.set("fitIntercept", bool(m.fitIntercept))
        meta.set("regParam", float(m.regParam))
        meta.set("epsilon", float(m.epsilon))
        meta.set("maxIter", int(m.numIter))
        data = [gson_dumps([float(x) for x in m.coefficients]), gson_dumps(float(m.intercept)),
                gson_dumps([float(x) for x in m.diagInvAtWA])]
        return meta, data

    def deserializeModel(self, meta: Params, data: List[str]) -> GlmModelData:
        m = GlmModelData()

        def g(name, default=None):
            v = meta.get(name) if meta.contains(name) else default
            return default if v is None else v
        m.featureColNames = g("featureCols")
        m.offsetColName = g("offsetCol")
        m.weightColName = g("weightCol")
        m.labelColName = g("labelCol")
        m.familyName = g("family", "Gaussian")
        m.variancePower = float(g("variancePower", 0.0))
        m.linkName = g("link")
        m.linkPower = float(g("linkPower", 1.0))
        m.fitIntercept = bool(g("fitIntercept", True))
        m.regParam = float(g("regParam", 0.0))
        m.numIter = int(g("maxIter", 10))
        m.epsilon = float(g("epsilon", 1e-5))
        m.coefficients = np.asarray(json.loads(data[0]), dtype=np.float64)
        m.intercept = float(json.loads(data[1]))
        m.diagInvAtWA = np.asarray(json.loads(data[2]), dtype=np.float64)
        return m

    def from_wls(self, wls: WlsModel, p: Params) -> GlmModelData:
        m = GlmModelData()

        def g(name, default=None):
            v = p.get(name) if p.contains(name) else default
            return default if v is None else v
        m.featureColNames = list(p.get("featureCols"))
        m.offsetColName = g("offsetCol")
        m.weightColName = g("weightCol")
        m.labelColName = p.get("labelCol")
        m.familyName = g("family", "Gaussian")
        m.variancePower = float(g("variancePower", 0.0))
        m.linkName = g("link")
        m.linkPower = float(g("linkPower", 1.0))
        m.fitIntercept = bool(g("fitIntercept", True))
        m.regParam = float(g("regParam", 0.0))
        m.numIter = int(g("maxIter", 10))
        m.epsilon = float(g("epsilon", 1e-5))
        m.coefficients, m.intercept, m.diagInvAtWA = wls.coefficients, wls.intercept, wls.diagInvAtWA
        return m


class GlmModelMapper(ModelMapper):
    """``GlmModelMapper.java`` — appends ``predictionCol`` (fitted mean) and optionally ``linkPredResultCol``
    (linear predictor); batched as one GEMV per partition."""

    def __init__(self, modelSchema, dataSchema, params=None):
        super().__init__(modelSchema, dataSchema, params)
        p = self.params
        self.pred_col = p.get("predictionCol")
        self.link_col = p.get("linkPredResultCol") if p.contains("linkPredResultCol") else None
        names = [self.pred_col] + ([self.link_col] if self.link_col else [])
        self.helper = OutputColsHelper(dataSchema, names, [Types.DOUBLE] * len(names),
                                       p.get("reservedCols") if p.contains("reservedCols") else None)

    def loadModel(self, modelRows):
        self.model = GlmModelDataConverter().load(modelRows)
        m = self.model
        self.fl = FamilyLink(m.familyName, m.variancePower, m.linkName, m.linkPower)

    def _map_columns(self, mt: MTable):
        m = self.model
        cpu = torch.device("cpu")
        X = torch.stack([_col(mt, c, 0.0, cpu) for c in m.featureColNames], 1)
        eta = X @ torch.as_tensor(m.coefficients, dtype=torch.float64) + m.intercept + _col(mt, m.offsetColName, 0.0, cpu)
        outs = [Column(self.fl.fitted(eta))]
        if self.link_col:
            outs.append(Column(eta))
        return outs
