"""Evaluation metrics: binary / multi-class / regression summaries and their Params-backed metric objects.

Reference: ``A/operator/common/evaluation/{EvaluationUtil,ClassificationEvaluationUtil,BinaryMetricsSummary,
MultiMetricsSummary,RegressionMetricsSummary,ConfusionMatrix,ClassificationMetricComputers,EvaluationCurve,
BaseMetrics,BinaryClassMetrics,MultiClassMetrics,RegressionMetrics}.java``.

MI355X design: a partition's sufficient statistics are built with device kernels — the binary summary is a
100000-bin probability histogram per class (``bincount`` on the device), the multi-class summary a
confusion matrix (``bincount`` of ``pred * K + label``), regression a handful of sums — then ONE all-reduce
merges them across ranks (the reference's ``ReduceBaseMetrics``).  Curves, thresholds and the ~60 derived
metrics are computed on the host from the merged histograms, with the reference's bin, sampling and
threshold rules, and stored as a ``Params`` JSON row (``BaseMetrics.serialize``).
"""
from __future__ import annotations

import json
import math
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from ... import _native
from ...common.javafmt import gson_dumps
from ...common.params import Params
from ...parallel import comm

__all__ = ["DETAIL_BIN_NUMBER", "BaseMetrics", "BinaryClassMetrics", "MultiClassMetrics", "RegressionMetrics",
           "ClusterMetrics", "build_label_index", "binary_summary", "multi_summary_from_detail",
           "multi_summary_from_pred", "regression_summary", "binary_metrics", "multi_metrics",
           "regression_metrics", "parse_detail"]

DETAIL_BIN_NUMBER = 100000
PROBABILITY_INTERVAL = 0.001
PROBABILITY_ERROR = 0.00001
LOG_LOSS_EPS = 1e-15
PROB_SUM_EPS = 0.01


# ---------------------------------------------------------------------------------------------------
# metric objects
# ---------------------------------------------------------------------------------------------------
def _camel(name: str) -> str:
    return name[0].upper() + name[1:]


class BaseMetrics:
    """Params holder; ``getXxx()`` returns the param named ``Xxx`` (or an alias below)."""
    _ALIASES: Dict[str, str] = {}

    def __init__(self, params: Optional[Params] = None):
        self.params = params if params is not None else Params()

    @classmethod
    def fromRow(cls, row):
        return cls(Params.fromJson(row[0]))

    def serialize(self):
        return (self.params.toJson(),)

    def getParams(self) -> Params:
        return self.params

    def _get(self, name):
        if not self.params.contains(name):
            raise KeyError(name)
        return json.loads(self.params._m[name]) if self.params._m[name] is not None else None

    def __getattr__(self, item):
        if item.startswith("get") and len(item) > 3:
            key = self._ALIASES.get(item[3:], item[3:])
            return lambda *a: self._get_metric(key, *a)
        raise AttributeError(item)

    def _get_metric(self, key, *args):
        return self._get(key)

    def __str__(self):
        return self.params.toJson()


class _ClassifierMetrics(BaseMetrics):
    _ALIASES = {"LabelArray": "LabelArray", "Ks": "K-S", "Auc": "AUC", "Prc": "PRC"}

    def _label_index(self, label):
        labels = self._get("LabelArray")
        return labels.index(str(label))

    def _get_metric(self, key, *args):
        if args:   # per-label value from the *Array param
            arr = self._get(key + "Array")
            return arr[self._label_index(args[0])]
        return self._get(key)

    def getConfusionMatrix(self):
        return np.asarray(self._get("ConfusionMatrix"), dtype=np.int64)


class BinaryClassMetrics(_ClassifierMetrics):
    def getRocCurve(self):
        return self._get("RocCurve")

    def getRecallPrecisionCurve(self):
        return self._get("RecallPrecisionCurve")

    def getLiftChart(self):
        return self._get("LiftChart")

    def getThresholdArray(self):
        return self._get("ThresholdArray")


class MultiClassMetrics(_ClassifierMetrics):
    pass


class RegressionMetrics(BaseMetrics):
    _ALIASES = {"Sse": "SSE", "Sst": "SST", "Ssr": "SSR", "Sae": "SAE", "Mse": "MSE", "Rmse": "RMSE", "Mae": "MAE",
                "Mape": "MAPE", "Count": "count", "YMean": "yMean", "PredictionMean": "predictionMean",
                "ExplainedVariance": "Explained Variance"}


class ClusterMetrics(BaseMetrics):
    _ALIASES = {"K": "k", "Count": "count", "Ssw": "SSW", "Ssb": "SSB", "ClusterArray": "clusterArray",
                "CountArray": "countArray", "Nmi": "NMI", "Purity": "purity", "Ri": "ri", "Ari": "ari",
                "SilhouetteCoefficient": "silhouetteCoefficient", "CalinskiHarabaz": "calinskiHarabaz",
                "Compactness": "compactness", "Seperation": "seperation", "DaviesBouldin": "daviesBouldin"}


# ---------------------------------------------------------------------------------------------------
# label handling
# ---------------------------------------------------------------------------------------------------
def build_label_index(labels, binary: bool, positive: Optional[str] = None):
    """Distinct labels sorted in reverse string order; binary + positiveValue puts it first
    (``ClassificationEvaluationUtil.buildLabelIndexLabelArray``)."""
    labels = sorted({str(l) for l in labels}, reverse=True)
    if len(labels) < 2:
        raise ValueError("The distinct label number less than 2!")
    if binary and len(labels) != 2:
        raise ValueError("The number of labels must be equal to 2!")
    if binary and positive is not None:
        if labels[1] == positive:
            labels[1] = labels[0]
            labels[0] = positive
        elif labels[0] != positive:
            raise ValueError("Not contain positiveValue")
    return labels


def parse_detail(s: str) -> Dict[str, float]:
    try:
        m = json.loads(s)
    except Exception:
        raise RuntimeError(f"Fail to deserialize detail column {s}!")
    m = {str(k): float(v) for k, v in m.items()}
    for v in m.values():
        if not (0.0 <= v <= 1.0):
            raise ValueError(f"Probibality in {s} not in range [0, 1]!")
    if abs(sum(m.values()) - 1.0) >= PROB_SUM_EPS:
        raise ValueError(f"Probability sum in {s} not equal to 1.0!")
    return m


# ---------------------------------------------------------------------------------------------------
# summaries (device histograms + one all-reduce)
# ---------------------------------------------------------------------------------------------------
def binary_summary(labels_col: Sequence[Any], details: Sequence[str], label_array: List[str], device=None):
    """(positiveBin, negativeBin, logLoss, total) over all ranks."""
    dev = device or torch.device("cpu")
    fast = _binary_detail_native(labels_col, details, label_array)
    if fast is not None:
        pos_p, is_pos, ll, keep = fast
        return _binary_bins(pos_p, is_pos, ll, keep, dev)
    pos_p, is_pos, ll, keep = [], [], 0.0, 0
    for lab, det in zip(labels_col, details):
        if lab is None or det is None:
            continue
        m = parse_detail(det)
        if len(m) != 2:
            raise ValueError("The number of labels must be equal to 2!")
        lab = str(lab)
        if lab not in label_array:
            continue
        p = m.get(label_array[0])
        pl = m.get(lab, 0.0)
        ll += -math.log(max(min(pl, 1 - LOG_LOSS_EPS), LOG_LOSS_EPS))
        pos_p.append(p)
        is_pos.append(lab == label_array[0])
        keep += 1
    return _binary_bins(pos_p, is_pos, ll, keep, dev)


def _label_codes(label_col):
    """(distinct label strings, per-row index into them, null mask) of a label Column, computed per distinct value
    (torch.unique on tensor columns) instead of per row."""
    vals = label_col.values
    if isinstance(vals, torch.Tensor) and vals.dim() == 1:
        lab = vals.detach().cpu()
        lnull = label_col.nulls.cpu().numpy() if label_col.nulls is not None else np.zeros(len(lab), bool)
        if lab.dtype in (torch.int8, torch.int16, torch.int32, torch.int64, torch.uint8) and len(lab):
            a = lab.numpy().astype(np.int64)
            lo = int(a.min())
            span = int(a.max()) - lo + 1
            if span <= 1 << 16:                   # small integer range: presence table instead of a sort
                present = np.bincount(a - lo, minlength=span) > 0
                slot = np.cumsum(present) - 1
                return [str(v) for v in (np.flatnonzero(present) + lo).tolist()], slot[a - lo], lnull
        uniq, inv = torch.unique(lab, return_inverse=True)
        return [str(v) for v in uniq.tolist()], inv.numpy(), lnull
    lst = label_col.to_list()
    ustr = sorted({str(v) for v in lst if v is not None})
    pos = {u: i for i, u in enumerate(ustr)}
    inv = np.asarray([pos[str(v)] if v is not None else 0 for v in lst], dtype=np.int64)
    return ustr, inv, np.asarray([v is None for v in lst], dtype=bool)


def detail_block_keys(label_col, blk) -> set:
    """Label strings a ``DetailBlock`` detail column and its label column contribute to the label index (the
    keys every row's detail map would show, plus the labels of the rows that have a detail)."""
    ustr, inv, lnull = _label_codes(label_col)
    ok = ~lnull if blk.nulls is None else (~lnull & ~blk.nulls)
    keys = {str(x) for x in blk.labels}
    if ok.any():
        keys |= {ustr[i] for i in np.unique(inv[ok]).tolist()}
    return keys


def detail_block_valid(blk, label_array: List[str]) -> bool:
    """This rank's block can be summarised columnar: its two labels are the index's, probabilities in [0, 1]
    summing to 1 (``parse_detail``'s checks)."""
    keys = [str(x) for x in blk.labels]
    if len(keys) != 2 or set(keys) != set(label_array):
        return False
    pr = blk.probs
    if not len(pr):
        return True
    c0, c1 = keys.index(label_array[0]), keys.index(label_array[1])
    return bool(np.all((pr >= 0.0) & (pr <= 1.0)) and np.all(np.abs(pr[:, c0] + pr[:, c1] - 1.0) < PROB_SUM_EPS))


def binary_summary_block(label_col, blk, label_array: List[str], device=None):
    """``binary_summary`` straight from a ``common/detail.DetailBlock`` (no detail strings): the same
    (positiveBin, negativeBin, logLoss, total) over all ranks — the strings are ``Double.toString`` of these same
    doubles, which parse back exactly.  None when the block's labels are not the two of ``label_array`` or a
    probability is out of range (the caller then takes the string path and its exact errors)."""
    # the fall-back decision is collective (the string path's all-reduce must run on every rank or on none);
    # ``blk`` None = this rank's micro-batch is empty (it contributes zero bins)
    dev_res = _binary_block_device(label_col, blk, label_array)
    if dev_res is not None and not comm.is_distributed():
        return dev_res
    valid = float(blk is None or len(blk) == 0 or (dev_res is not None) or detail_block_valid(blk, label_array))
    if comm.is_distributed():
        valid = min(comm.all_gather_object(valid))
    if valid < 1.0:
        return None
    if blk is None or len(blk) == 0:
        return _reduce_bins(np.zeros(2 * DETAIL_BIN_NUMBER), 0.0, 0, device or torch.device("cpu"))
    if dev_res is not None:
        pb, nb, ll, keep = dev_res
        buf = torch.cat([pb.to(torch.float64), nb.to(torch.float64), ll.reshape(1), keep.reshape(1).to(torch.float64)])
        comm.all_reduce(buf, "sum")
        B = DETAIL_BIN_NUMBER
        return buf[:B].to(torch.int64), buf[B:2 * B].to(torch.int64), buf[-2], buf[-1].to(torch.int64)
    keys = [str(x) for x in blk.labels]
    ustr, inv, lnull = _label_codes(label_col)
    ok = ~lnull if blk.nulls is None else (~lnull & ~blk.nulls)
    c0, c1 = keys.index(label_array[0]), keys.index(label_array[1])
    pr = blk.probs
    code = np.array([0 if u == label_array[0] else (1 if u == label_array[1] else -1) for u in ustr],
                    dtype=np.int64)
    rc = code[inv] if len(code) else np.zeros(0, np.int64)
    nat = _native.binary_bins(pr, c0, c1, rc, ok, DETAIL_BIN_NUMBER, LOG_LOSS_EPS)
    if nat is not None:                           # one C++ pass: bins + row-order log loss
        bins, ll, keep = nat
        return _reduce_bins(bins.astype(np.float64), ll, keep, device or torch.device("cpu"))
    sel = ok & (rc >= 0)
    is_pos = rc[sel] == 0
    p0 = pr[sel, c0]
    pl = np.where(is_pos, p0, pr[sel, c1])
    terms = -np.log(np.clip(pl, LOG_LOSS_EPS, 1 - LOG_LOSS_EPS))
    ll = float(np.cumsum(terms)[-1]) if len(terms) else 0.0       # the loop's left-to-right summation order
    return _binary_bins(p0, is_pos, ll, int(sel.sum()), device or torch.device("cpu"))


def host_value(x):
    """numpy array / python scalar of a (device) tensor summary part; anything else unchanged."""
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu()
        return x.numpy() if x.dim() else x.item()
    return x


def _numeric_label_value(s: str, dtype):
    """The numeric value whose Alink string form is ``s`` for a label column of torch ``dtype``, or None."""
    from ...common.javafmt import java_str
    try:
        v = float(s)
    except ValueError:
        return None
    if dtype.is_floating_point:
        return v if java_str(v) == s else None
    return int(v) if v == int(v) and str(int(v)) == s else None


def _binary_block_device(label_col, blk, label_array: List[str]):
    """The binary summary of a device-resident, trusted ``DetailBlock`` (a GPU scorer's output) with a numeric device
    label column, computed on the device: (positive bins int64 [B], negative bins int64 [B], log loss fp64 0-dim,
    kept rows int64 0-dim), all device tensors — a scoring -> evaluation stream never copies the micro-batch to the
    host.  The log loss is a device sum (fp64, any order) instead of the row-order loop.  None when not applicable."""
    if blk is None or len(blk) == 0 or not blk.trusted or blk._probs_t is None or not blk._probs_t.is_cuda:
        return None
    lab = label_col.values
    if not (isinstance(lab, torch.Tensor) and lab.dim() == 1 and lab.device == blk._probs_t.device) \
            or label_col.nulls is not None or blk.nulls is not None:
        return None
    keys = [str(x) for x in blk.labels]
    if len(keys) != 2 or set(keys) != set(label_array):
        return None
    v0, v1 = (_numeric_label_value(x, lab.dtype) for x in label_array)
    if v0 is None or v1 is None:
        return None
    pr = blk._probs_t
    c0, c1 = keys.index(label_array[0]), keys.index(label_array[1])
    is_pos = lab == v0
    sel = is_pos | (lab == v1)
    B = DETAIL_BIN_NUMBER
    p0 = pr[:, c0]
    idx = torch.where(p0 == 1.0, torch.full_like(p0, B - 1), torch.floor(p0 * B)).to(torch.int64)
    ok = sel & (idx >= 0) & (idx < B)
    slot = torch.where(is_pos, idx, idx + B)
    bins = torch.bincount(torch.where(ok, slot, torch.full_like(slot, 2 * B)), minlength=2 * B + 1)[:2 * B]
    pl = torch.where(is_pos, p0, pr[:, c1])
    terms = -torch.log(torch.clamp(pl, LOG_LOSS_EPS, 1 - LOG_LOSS_EPS))
    ll = torch.where(sel, terms, torch.zeros_like(terms)).sum()
    return bins[:B], bins[B:], ll, sel.sum()


def _binary_detail_native(labels_col, details, label_array: List[str]):
    """Bulk path of the per-row detail parsing above: the host C++ parser reads plain two-entry detail strings
    (``_native.parse_binary_detail``) and the checks run vectorised; None -> the caller's JSON loop (which also
    produces the exact error messages)."""
    from ... import _native
    if len(label_array) != 2:
        return None
    labs = [None if l is None else str(l) for l in labels_col]
    lset = set(label_array)
    # parse and check EVERY non-null (label, detail) row, as the JSON loop does, so both paths accept and
    # reject the same inputs; only then keep the rows whose label is one of the two
    nn_idx = [i for i, (l, d) in enumerate(zip(labs, details)) if l is not None and d is not None]
    dets = [details[i] for i in nn_idx]
    if any(not isinstance(d, str) for d in dets):
        return None
    parsed = _native.parse_binary_detail(dets, label_array[0], label_array[1])
    if parsed is None:
        return None
    p0, p1 = parsed
    if not (np.all((p0 >= 0.0) & (p0 <= 1.0) & (p1 >= 0.0) & (p1 <= 1.0))
            and np.all(np.abs(p0 + p1 - 1.0) < PROB_SUM_EPS)):
        return None
    sel = np.array([labs[i] in lset for i in nn_idx], dtype=bool)
    keep_idx = [i for i, m in zip(nn_idx, sel) if m]
    p0, p1 = p0[sel], p1[sel]
    is_pos = np.array([labs[i] == label_array[0] for i in keep_idx], dtype=bool)
    pl = np.where(is_pos, p0, p1)
    terms = -np.log(np.clip(pl, LOG_LOSS_EPS, 1 - LOG_LOSS_EPS))
    ll = float(np.cumsum(terms)[-1]) if len(terms) else 0.0       # the loop's left-to-right summation order
    return p0, is_pos, ll, len(keep_idx)


def _binary_bins(pos_p, is_pos, ll, keep, dev):
    """(positiveBin, negativeBin, logLoss, total) summed over ranks: one numpy bincount over 2 * BINS slots
    (positive rows in the first half); the all-reduce only runs under a process group."""
    p = np.asarray(pos_p, dtype=np.float64)
    lbl = np.asarray(is_pos, dtype=bool)
    B = DETAIL_BIN_NUMBER
    idx = np.where(p == 1.0, B - 1, np.floor(p * B))
    ok = (idx >= 0) & (idx < B)
    slot = idx[ok].astype(np.int64) + np.where(lbl[ok], 0, B)
    return _reduce_bins(np.bincount(slot, minlength=2 * B).astype(np.float64), ll, keep, dev)


def _reduce_bins(bins2, ll, keep, dev):
    B = DETAIL_BIN_NUMBER
    buf = np.zeros(2 * B + 2, dtype=np.float64)
    buf[:2 * B] = bins2
    buf[-2:] = (ll, float(keep))
    if comm.is_distributed():
        t = torch.from_numpy(buf).to(dev)
        comm.all_reduce(t, "sum")
        buf = t.cpu().numpy()
    return buf[:B].astype(np.int64), buf[B:2 * B].astype(np.int64), float(buf[-2]), int(buf[-1])


def multi_summary_from_detail(labels_col, details, label_array: List[str], device=None):
    dev = device or torch.device("cpu")
    K = len(label_array)
    index = {l: i for i, l in enumerate(label_array)}
    pi, li, ll, n = [], [], 0.0, 0
    for lab, det in zip(labels_col, details):
        if lab is None or det is None:
            continue
        m = parse_detail(det)
        lab = str(lab)
        if lab not in index:
            continue
        best, pred = -math.inf, None
        for k in sorted(m):           # TreeMap iteration order, first max wins
            if m[k] > best:
                best, pred = m[k], k
        pl = m.get(lab, 0.0)
        ll += -math.log(max(min(pl, 1 - LOG_LOSS_EPS), LOG_LOSS_EPS))
        pi.append(index[pred])
        li.append(index[lab])
        n += 1
    return _confusion(pi, li, K, ll, n, dev)


def multi_summary_from_pred(labels_col, preds, label_array: List[str], device=None):
    dev = device or torch.device("cpu")
    index = {l: i for i, l in enumerate(label_array)}
    pi, li = [], []
    for lab, pr in zip(labels_col, preds):
        if lab is None or pr is None:
            continue
        pi.append(index[str(pr)])
        li.append(index[str(lab)])
    return _confusion(pi, li, len(label_array), -1.0, len(pi), dev)


def multi_summary_pred_tensors(lc, pc, binary: bool, pos, device=None):
    """(confusion matrix, -1, rows, label array) of integer / bool label and prediction tensor columns with no
    per-row Python: the label set from the distinct values of each column (as ``str`` of the value, every rank's
    union), the codes by ``searchsorted`` over the distinct values.  None for other column types."""
    a, b = lc.values, pc.values
    ok_t = lambda v: isinstance(v, torch.Tensor) and v.dim() == 1 and not v.is_floating_point() and \
        not v.is_complex()
    if not (ok_t(a) and ok_t(b)) or a.dtype != b.dtype:
        return None
    dev = device or torch.device("cpu")
    a, b = a.to(dev), b.to(dev)
    nl = lc.nulls.to(dev) if lc.nulls is not None else torch.zeros(a.shape, dtype=torch.bool, device=dev)
    npd = pc.nulls.to(dev) if pc.nulls is not None else torch.zeros(b.shape, dtype=torch.bool, device=dev)
    uniq = torch.unique(torch.cat([a[~nl], b[~npd]]))
    strs = [str(v) for v in uniq.tolist()]
    label_set = set()
    for part in comm.all_gather_object(sorted(set(strs))):
        label_set.update(part)
    arr = build_label_index(label_set, binary, pos)
    index = {l: i for i, l in enumerate(arr)}
    lut = torch.tensor([index[x] for x in strs] or [0], dtype=torch.long, device=dev)
    ok = ~(nl | npd)
    la, pa = a[ok], b[ok]
    li = lut[torch.searchsorted(uniq, la)] if la.numel() else la.long()
    pi = lut[torch.searchsorted(uniq, pa)] if pa.numel() else pa.long()
    mat, ll, n = _confusion(pi, li, len(arr), -1.0, int(la.numel()), dev)
    return mat, ll, n, arr


def _confusion(pi, li, K, ll, n, dev):
    p = torch.as_tensor(pi, dtype=torch.long, device=dev)
    l = torch.as_tensor(li, dtype=torch.long, device=dev)
    mat = torch.bincount(p * K + l, minlength=K * K).double()
    buf = torch.cat([mat, torch.tensor([max(ll, 0.0), float(n)], dtype=torch.float64, device=dev)])
    comm.all_reduce(buf, "sum")
    b = buf.cpu().numpy()
    return b[:K * K].reshape(K, K).astype(np.int64), (float(b[-2]) if ll >= 0 else -1.0), int(b[-1])


def regression_summary(y, pred, device=None):
    dev = device or torch.device("cpu")
    yv = y.to(dev, torch.float64) if isinstance(y, torch.Tensor) else \
        torch.as_tensor(np.asarray(y, dtype=np.float64), device=dev)
    pv = pred.to(dev, torch.float64) if isinstance(pred, torch.Tensor) else \
        torch.as_tensor(np.asarray(pred, dtype=np.float64), device=dev)
    diff = (yv - pv).abs()
    buf = torch.stack([yv.sum(), (yv * yv).sum(), pv.sum(), (pv * pv).sum(), diff.sum(), (diff * diff).sum(),
                       (diff / yv).abs().sum(), torch.tensor(float(yv.shape[0]), dtype=torch.float64, device=dev)])
    comm.all_reduce(buf, "sum")
    return buf.cpu().numpy()


# ---------------------------------------------------------------------------------------------------
# confusion-matrix metrics (ConfusionMatrix.java + ClassificationMetricComputers.java)
# ---------------------------------------------------------------------------------------------------
class _CM:
    def __init__(self, m: np.ndarray):
        self.m = np.asarray(m, dtype=np.float64)
        self.k = self.m.shape[0]
        self.actual = self.m.sum(0)
        self.pred = self.m.sum(1)
        self.total = float(self.m.sum())
        d = np.diag(self.m)
        self.tp_i = d
        self.fp_i = self.pred - d
        self.fn_i = self.actual - d
        self.tn_i = d + self.total - self.pred - self.actual
        self.tp, self.fp, self.fn, self.tn = self.tp_i.sum(), self.fp_i.sum(), self.fn_i.sum(), self.tn_i.sum()

    def counts(self, i):
        if i is None:
            return self.tp, self.fp, self.fn, self.tn
        return self.tp_i[i], self.fp_i[i], self.fn_i[i], self.tn_i[i]

    def proportion(self):
        return self.actual / self.total if self.total else np.zeros(self.k)

    def accuracy(self):
        return float(np.trace(self.m) / self.total) if self.total else float("nan")

    def kappa(self):
        pe = float((self.pred * self.actual).sum()) / (self.total * self.total)
        pa = float(np.trace(self.m)) / self.total
        return (pa - pe) / (1 - pe) if pe < 1 else 1.0


def _div(a, b):
    return 0.0 if b == 0 else a / b


def _tpr(c, i):
    tp, fp, fn, tn = c.counts(i)
    return _div(tp, tp + fn)


def _tnr(c, i):
    tp, fp, fn, tn = c.counts(i)
    return _div(tn, fp + tn)


def _fpr(c, i):
    tp, fp, fn, tn = c.counts(i)
    return _div(fp, fp + tn)


def _fnr(c, i):
    tp, fp, fn, tn = c.counts(i)
    return _div(fn, tp + fn)


def _precision(c, i):
    tp, fp, fn, tn = c.counts(i)
    return _div(tp, tp + fp)


def _f1(c, i):
    tp, fp, fn, tn = c.counts(i)
    return _div(2 * tp, 2 * tp + fp + fn)


def _acc(c, i):
    tp, fp, fn, tn = c.counts(i)
    return (tp + tn) / (tp + fp + fn + tn)


def _kappa(c, i):
    tp, fp, fn, tn = c.counts(i)
    total = tp + fp + fn + tn
    pa = (tp + tn) / total
    pe = ((tp + fn) * (tp + fp) + (tn + fp) * (tn + fn)) / (total * total)
    return (pa - pe) / (1 - pe) if pe < 1 else 1.0


# (array param, weighted, macro, micro, computer) in ClassificationEvaluationUtil.Computations order
_COMPUTATIONS = [
    ("TrueNegativeRate", _tnr), ("TruePositiveRate", _tpr), ("FalseNegativeRate", _fnr),
    ("FalsePositiveRate", _fpr), ("Precision", _precision), ("Specificity", _tnr), ("Sensitivity", _tpr),
    ("Recall", _tpr), ("F1", _f1), ("Accuracy", _acc), ("Kappa", _kappa)]


def _weighted(fn, c):
    prop = c.proportion()
    return float(sum(fn(c, i) * prop[i] for i in range(c.k)))


def _macro(fn, c):
    return float(sum(fn(c, i) for i in range(c.k)) / c.k)


def _set(params: Params, name, value):
    params.set(name, value)


def _common(params: Params, c: _CM, labels: List[str]):
    _set(params, "LabelArray", list(labels))
    _set(params, "ActualLabelFrequency", [int(x) for x in c.actual])
    _set(params, "ActualLabelProportion", [float(x) for x in c.proportion()])
    _set(params, "ConfusionMatrix", [[int(x) for x in row] for row in c.m])
    _set(params, "TotalSamples", int(c.total))
    for name, fn in _COMPUTATIONS:
        _set(params, "Weighted" + name, _weighted(fn, c))
        _set(params, "Macro" + name, _macro(fn, c))
        _set(params, "Micro" + name, float(fn(c, None)))
    _set(params, "Accuracy", c.accuracy())
    _set(params, "Kappa", c.kappa())


def multi_metrics(matrix: np.ndarray, labels: List[str], logloss: float, total: int) -> MultiClassMetrics:
    params = Params()
    c = _CM(matrix)
    _set(params, "PredictLabelFrequency", [int(x) for x in c.pred])
    _set(params, "PredictLabelProportion", [float(x) for x in (c.pred / c.total if c.total else c.pred)])
    for name, fn in _COMPUTATIONS:
        vals = [float(fn(c, i)) for i in range(c.k)] + [_weighted(fn, c), _macro(fn, c), float(fn(c, None))]
        _set(params, name + "Array", vals)
    _common(params, c, labels)
    if logloss >= 0:
        _set(params, "LogLoss", logloss / total)
    return MultiClassMetrics(params)


def _area(x, y):
    return float(np.sum((x[1:] - x[:-1]) * (y[1:] + y[:-1]) / 2)) if len(x) > 1 else 0.0


def _sample_thresholds(thr: np.ndarray) -> List[int]:
    """Indices kept by the reference's threshold sampling over the descending thresholds (index 0, then every
    threshold at least PROBABILITY_INTERVAL below the last kept one, plus any within PROBABILITY_ERROR of 0.5).
    Jumps between kept points with a binary search (the predicate is monotone in i) and settles the exact
    boundary with the scalar comparison, so the result equals the per-element scan."""
    n1 = len(thr)
    step = PROBABILITY_INTERVAL - PROBABILITY_ERROR
    halves = np.nonzero(np.abs(thr - 0.5) < PROBABILITY_ERROR)[0].tolist()
    neg = -thr                                           # ascending
    keep, pre, i, h = [0], thr[0], 0, 0
    while i < n1:
        j = int(np.searchsorted(neg, -(pre - step), side="left"))
        j = max(j, i)
        while j > i and abs(pre - thr[j - 1]) >= step:
            j -= 1
        while j < n1 and not abs(pre - thr[j]) >= step:
            j += 1
        while h < len(halves) and halves[h] < i:
            h += 1
        if h < len(halves) and halves[h] < j:
            j = halves[h]
        if j >= n1:
            break
        keep.append(j)
        pre = thr[j]
        i = j + 1
    return keep


def _vdiv(a, b):
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(b == 0, 0.0, a / np.where(b == 0, 1.0, b))


def _binary_arrays(TP, FP, FN, TN):
    """``_COMPUTATIONS`` of class 0 over arrays of 2x2 confusion counts."""
    total = TP + FP + FN + TN
    pa = (TP + TN) / total
    pe = ((TP + FN) * (TP + FP) + (TN + FP) * (TN + FN)) / (total * total)
    with np.errstate(divide="ignore", invalid="ignore"):
        kappa = np.where(pe < 1, (pa - pe) / np.where(pe < 1, 1 - pe, 1.0), 1.0)
    tnr, tpr = _vdiv(TN, FP + TN), _vdiv(TP, TP + FN)
    return {"TrueNegativeRate": tnr, "TruePositiveRate": tpr, "FalseNegativeRate": _vdiv(FN, TP + FN),
            "FalsePositiveRate": _vdiv(FP, FP + TN), "Precision": _vdiv(TP, TP + FP), "Specificity": tnr,
            "Sensitivity": tpr, "Recall": tpr, "F1": _vdiv(2 * TP, 2 * TP + FP + FN), "Accuracy": (TP + TN) / total,
            "Kappa": kappa}


def binary_metrics(posb: np.ndarray, negb: np.ndarray, labels: List[str], logloss: float, total: int
                   ) -> BinaryClassMetrics:
    """``BinaryMetricsSummary.toMetrics`` :72-...: full curves for AUC/PRC/KS, 0.001-sampled curves and
    threshold arrays, confusion matrix at the threshold nearest 0.5.  Device-tensor summaries (the GPU columnar
    path) are read back here, once per emitted window."""
    posb, negb, logloss, total = (host_value(x) for x in (posb, negb, logloss, total))
    eff = np.nonzero((posb != 0) | (negb != 0))[0]
    mid = DETAIL_BIN_NUMBER // 2
    at = int(np.searchsorted(eff, mid))
    if at == len(eff) or eff[at] != mid:
        eff = np.insert(eff, at, mid)
    total_true, total_false = int(posb[eff].sum()), int(negb[eff].sum())
    if total_true + total_false != total:
        raise ValueError("The effective number in bins must be equal to total!")
    rev = eff[::-1]
    cur_t = np.cumsum(posb[rev]).astype(np.float64)
    cur_f = np.cumsum(negb[rev]).astype(np.float64)
    n1 = len(rev) + 1
    thr = np.empty(n1)
    thr[0] = 1.0
    thr[1:] = rev * (1.0 / DETAIL_BIN_NUMBER)
    tp = np.concatenate([[0.0], cur_t])
    fp = np.concatenate([[0.0], cur_f])
    tpr = tp / total_true if total_true else np.ones(n1)
    fpr = fp / total_false if total_false else np.ones(n1)
    roc_x, roc_y = fpr.copy(), tpr.copy()
    roc_x[0], roc_y[0] = 0.0, 0.0
    prec = np.where(tp == 0, 1.0, tp / np.where(tp + fp == 0, 1.0, tp + fp))
    pr_x, pr_y = tpr.copy(), prec.copy()
    pr_x[0], pr_y[0] = 0.0, prec[1] if n1 > 1 else 1.0
    lift_x = (tp + fp) / total
    lift_y = tp.copy()
    lift_x[0], lift_y[0] = 0.0, 0.0
    params = Params()
    _set(params, "AUC", _area(roc_x, roc_y))
    _set(params, "PRC", _area(pr_x, pr_y))
    _set(params, "K-S", float(np.max(np.abs(roc_x - roc_y))))
    # sampling of thresholds at 0.001 resolution (plus the 0.5 point); float64 arrays go to the Params JSON
    # writer as they are (same Double.toString digits as their tolist(), formatted in C++ when long)
    keep = _native.sample_thresholds(thr, PROBABILITY_INTERVAL - PROBABILITY_ERROR, PROBABILITY_ERROR)
    if keep is None:
        keep = np.asarray(_sample_thresholds(thr))
    _set(params, "RocCurve", [roc_x[keep], roc_y[keep]])
    _set(params, "RecallPrecisionCurve", [pr_x[keep], pr_y[keep]])
    _set(params, "LiftChart", [lift_x[keep], lift_y[keep]])
    sk = keep[1:]
    s_thr = thr[sk]
    _set(params, "ThresholdArray", s_thr)
    # per-threshold 2x2 confusion counts of class 0, every computation vectorised over the thresholds (the same
    # float64 operations, in the same order, as the per-matrix _CM computers)
    TP, FP = tp[sk], fp[sk]
    FN, TN = float(total_true) - TP, float(total_false) - FP
    for name, arr in _binary_arrays(TP, FP, FN, TN).items():
        _set(params, name + "Array", arr)
    if logloss >= 0:
        _set(params, "LogLoss", logloss / total)
    mid_i = int(np.argmin(np.abs(s_thr - 0.5)))
    i = sk[mid_i]
    c = _CM(np.array([[tp[i], fp[i]], [total_true - tp[i], total_false - fp[i]]]))
    _set(params, "Precision", float(_precision(c, 0)))
    _set(params, "Recall", float(_tpr(c, 0)))
    _set(params, "F1", float(_f1(c, 0)))
    _common(params, c, labels)
    return BinaryClassMetrics(params)


def regression_metrics(s: np.ndarray) -> RegressionMetrics:
    y_sum, y_sum2, p_sum, p_sum2, mae, sse, mape, total = [float(v) for v in s]
    params = Params()
    sst = y_sum2 - y_sum * y_sum / total
    ssr = p_sum2 - 2 * y_sum * p_sum / total + y_sum * y_sum / total
    r2 = 1 - sse / sst if sst != 0 else float("nan")
    _set(params, "SST", sst)
    _set(params, "SSE", sse)
    _set(params, "SSR", ssr)
    _set(params, "R2", r2)
    _set(params, "R", math.sqrt(r2) if r2 >= 0 else float("nan"))
    _set(params, "MSE", sse / total)
    _set(params, "RMSE", math.sqrt(sse / total))
    _set(params, "SAE", mae)
    _set(params, "MAE", mae / total)
    _set(params, "count", total)
    _set(params, "MAPE", mape * 100 / total)
    _set(params, "yMean", y_sum / total)
    _set(params, "predictionMean", p_sum / total)
    _set(params, "Explained Variance", ssr / total)
    return RegressionMetrics(params)
