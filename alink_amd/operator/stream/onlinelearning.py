"""Online learning: FTRL-proximal logistic regression on a stream (reference
``A/operator/stream/onlinelearning/{FtrlTrainStreamOp,FtrlPredictStreamOp}.java``).

``FtrlTrainStreamOp(initModel)`` warm-starts from a batch-trained linear model (collected once, as the
reference's ``DirectReader``), updates coefficients sample by sample with FTRL-proximal (native C++ loop
``_native/csrc/ftrl.cpp`` — the update is inherently sequential) and emits a model snapshot at the first
sample, every ``timeInterval`` seconds and when the stream ends.  Snapshot rows are
``(bid, ntab, model_id, model_info, label_value)``: ``bid`` = snapshot number, ``ntab`` = rows per snapshot.
``FtrlPredictStreamOp(initModel).linkFrom(models, data)`` re-assembles snapshots and hot-swaps the
``LinearModelMapper`` between micro-batches.

Deviation: the reference scales each gradient by ``1/sqrt(ms between the forward and the feedback pass)``
(``FtrlTrainStreamOp.java:428``), a wall-clock artefact of its Flink feedback loop; here the scale is 1.
With more than one rank the coefficient vector is sharded by feature range only for the margin;
each rank applies the identical update to the full vector after an all-gather of the micro-batch.
"""
from __future__ import annotations

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
    from ..base import gather_table
    return gather_table(op.getOutputTable())


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
    """``updateMode``: ``SEQUENTIAL`` (default; the native host loop, sample order as the reference) or
    ``HOGWILD`` (the micro-batch is applied on the GPU by ``ops/csrc/ftrl.hip``, one wave per sample, with the
    model state resident in HBM; needs a GPU)."""
    EXTRA_PARAMS = [ParamInfo("updateMode", str, "SEQUENTIAL or HOGWILD (GPU, one wave per sample)",
                              default="SEQUENTIAL")]

    def __init__(self, model=None, params: Optional[Params] = None, **kw):
        if isinstance(model, Params):
            model, params = None, model
        super().__init__(params, **kw)
        if model is None:
            raise ValueError("Ftrl algo: initial model is null. Please set a valid initial model.")
        self._init_model = model

    def linkFrom(self, *inputs):
        (inp,) = self._connect(*inputs)
        p = self.getParams()
        mt = _model_rows(self._init_model)
        conv = LinearModelDataConverter(LinearModelDataConverter.extractLabelType(mt.schema))
        self._model = conv.load(mt.rows())
        self._label_type = inp.getSchema().types[inp.getSchema().names.index(p.get("labelCol"))]
        self._conv = LinearModelDataConverter(self._label_type)
        base = self._conv.getModelSchema()
        self._schema = TableSchema(["bid", "ntab"] + list(base.names), [Types.LONG, Types.LONG] + list(base.types))
        self._w = np.array(self._model.coefVector.data, dtype=np.float64)
        self._n = np.zeros_like(self._w)
        self._z = np.zeros_like(self._w)
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
        self._hogwild = str(_pget(p, "updateMode", "SEQUENTIAL")).upper() == "HOGWILD"
        self._dev_state = None
        _register_upstream_sources(inp)
        return self

    def _snapshot(self):
        if self._dev_state is not None:
            self._w = self._dev_state[0].cpu().numpy().copy()
        m = self._model
        m.coefVector = DenseVector(self._w.copy())
        m.hasInterceptItem = self._intercept
        m.vectorColName = self._vec_col
        m.featureNames = list(self._feat_cols) if self._feat_cols else None
        m.modelName = "Logistic Regression"
        m.vectorSize = self._w.size - 1 if self._intercept else self._w.size
        rows = self._conv.save(m)
        out = [(self._bid, len(rows)) + tuple(r) for r in rows]
        self._bid += 1
        self._emit(MTable.from_rows(out, self._schema))

    def on_batch(self, port, mt):
        if self._first:
            self._snapshot()
            self._first = False
        if mt.num_rows:
            self._update(mt)
        if time.time() - self._t0 > self._interval:
            self._t0 = time.time()
            self._snapshot()

    def on_finish(self, port):
        self._snapshot()

    def _update(self, mt: MTable):
        import torch
        p = self.getParams()
        fm = extract_features(mt, self._feat_cols if self._vec_col is None else None, self._vec_col,
                              torch.device("cpu"), vector_size=self._vsize)
        if self._intercept:
            fm = fm.prefix_one()
        if fm.is_sparse:
            indptr = fm.crow.cpu().numpy()
            indices = fm.col.cpu().numpy()
            values = fm.val.cpu().double().numpy()
        else:
            X = fm.to_dense().double().numpy()
            nrow, d = X.shape
            indptr = np.arange(nrow + 1, dtype=np.int64) * d
            indices = np.tile(np.arange(d, dtype=np.int32), nrow)
            values = X.reshape(-1)
        l0 = self._model.labelValues[0]
        labels = []
        for v in mt.column_values(p.get("labelCol")):
            if isinstance(l0, (int, float)) and not isinstance(l0, bool):
                labels.append(1.0 if float(v) == float(l0) else 0.0)
            else:
                labels.append(1.0 if str(v) == str(l0) else 0.0)
        if indices.size and int(indices.max()) >= self._w.size:
            raise ValueError("feature index out of range of the initial model")
        if self._hogwild:
            from ...ops.ftrl import ftrl_hogwild
            if not torch.cuda.is_available():
                raise RuntimeError("FTRL updateMode HOGWILD needs a GPU")
            if self._dev_state is None:
                dev = torch.device("cuda", torch.cuda.current_device())
                self._dev_state = [torch.as_tensor(a, device=dev).clone() for a in (self._w, self._n, self._z)]
            ftrl_hogwild(torch.as_tensor(indptr), torch.as_tensor(indices), torch.as_tensor(values),
                         torch.as_tensor(np.asarray(labels, dtype=np.float64)), *self._dev_state,
                         self._alpha, self._beta, self._l1, self._l2)
            return
        if not _native.ftrl_update_csr(indptr, indices, values, np.asarray(labels), self._w, self._n, self._z,
                                       self._alpha, self._beta, self._l1, self._l2):
            _ftrl_python(indptr, indices, values, labels, self._w, self._n, self._z, self._alpha, self._beta,
                         self._l1, self._l2)


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
        _register_upstream_sources(models)
        _register_upstream_sources(data)
        return self

    def on_batch(self, port, mt):
        if port == 0:
            for r in mt.rows():
                bid, ntab = int(r[0]), int(r[1])
                buf = self._buffers.setdefault(bid, [])
                buf.append(tuple(r[2:]))
                if len(buf) == ntab:
                    self._mapper.loadModel(buf)
                    del self._buffers[bid]
        else:
            self._emit(self._mapper.map_table(mt))
