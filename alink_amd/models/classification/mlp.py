"""Multilayer perceptron classifier (reference ``A/operator/batch/classification/
MultilayerPerceptronTrainBatchOp.java``, ``A/operator/common/classification/ann/*``).

Kept: topology ``layers[0] -> ... -> layers[-1]`` of affine layers with sigmoid activations and a softmax +
cross-entropy top (``FeedForwardTopology.multiLayerPerceptron(layers, true)``); the flat weight vector packs
every affine layer as ``W [in x out]`` row-major followed by ``b [out]`` (``AffineLayerModel.pack``);
initial weights ``N(0, 0.05^2)`` from ``java.util.Random(1).nextGaussian`` (or ``initialWeights``);
training = the shared L-BFGS (``models/linear/optim.py``, 3 line-search steps as ``FeedForwardTrainer``)
over the mean cross-entropy with optional L1/L2.  Model: meta ``{vectorCol, isVectorInput, layers,
featureCols}`` + the weight ``DenseVector`` JSON + label rows.

MI355X design: the whole partition is one ``[n, d]`` device matrix; forward/backward are GEMMs
(rocBLAS/hipBLASLt) with fused elementwise sigmoid/softmax, the gradient comes from autograd on the flat
weight vector, and the line search evaluates the loss for all step sizes with one batched forward each.
"""
from __future__ import annotations

import json
from typing import List, Sequence

import numpy as np
import torch

from ...ops import mlp as mlp_ops
from ...common.javafmt import gson_dumps, java_str
from ...common.jrandom import JavaRandom
from ...common.linalg import DenseVector
from ...common.mapper import OutputColsHelper, RichModelMapper
from ...common.model.converter import LabeledModelDataConverter
from ...common.params import Params
from ...common.table import Column, MTable
from ...common.types import Types
from ...parallel import comm
from ..common.features import extract_features
from ..linear.model import _recover_label
from ..linear.objfunc import LabeledData, OptimObjFunc
from ..linear.optim import optimize

__all__ = ["MlpObjFunc", "mlp_forward", "train_mlp", "MlpcModelDataConverter", "MlpcModelMapper", "weight_size"]


def weight_size(layers: Sequence[int]) -> int:
    return sum(layers[i] * layers[i + 1] + layers[i + 1] for i in range(len(layers) - 1))


def _unpack(w: torch.Tensor, layers):
    out, off = [], 0
    for i in range(len(layers) - 1):
        a, b = layers[i], layers[i + 1]
        W = w[off:off + a * b].reshape(a, b)
        off += a * b
        bias = w[off:off + b]
        off += b
        out.append((W, bias))
    return out


def mlp_forward(X: torch.Tensor, w: torch.Tensor, layers) -> torch.Tensor:
    """Class probabilities [n, C]."""
    h = X
    params = _unpack(w, layers)
    for i, (W, b) in enumerate(params):
        z = h @ W + b
        h = torch.softmax(z, dim=1) if i == len(params) - 1 else torch.sigmoid(z)
    return h


class MlpObjFunc(OptimObjFunc):
    def __init__(self, layers, l1=0.0, l2=0.0):
        super().__init__(l1, l2)
        self.layers = list(layers)

    def _ce(self, data, coef):
        P = mlp_forward(data.X.to_dense(), coef, self.layers)
        idx = data.y.long()
        return -torch.log(P.gather(1, idx[:, None])[:, 0].clamp_min(1e-300))

    def loss_per_sample(self, data, coef):
        with torch.no_grad():
            return self._ce(data, coef)

    def grad_sum(self, data, coef):
        X = data.X.to_dense()
        if mlp_ops.kernel_supported(X, self.layers):   # K17: explicit backprop, GEMMs + fused HIP epilogues
            return mlp_ops.mlp_grad(X, data.y, data.w, coef.detach(), self.layers)[0]
        w = coef.detach().clone().requires_grad_(True)
        loss = (self._ce(data, w) * data.w).sum()
        (g,) = torch.autograd.grad(loss, w)
        return g.detach()


def train_mlp(mt: MTable, params: Params, env):
    dev = env.device
    label_col = params.get("labelCol")
    vcol = params.get("vectorCol") if params.contains("vectorCol") else None
    vcol = vcol if vcol else None
    fcols = params.get("featureCols") if (params.contains("featureCols") and params.get("featureCols")) else None
    if vcol is None and fcols is None:
        from ...common.types import is_numeric
        fcols = [n for n, t in zip(mt.schema.names, mt.schema.types) if n != label_col and is_numeric(t)]
    layers = [int(x) for x in params.get("layers")]
    keys = {}
    for part in comm.all_gather_object(sorted({java_str(v): v for v in mt.column_values(label_col)}.items())):
        for k, v in part:
            keys.setdefault(k, v)
    from ..tree.data import _sort_key
    labels = sorted(keys.values(), key=_sort_key)
    index = {java_str(v): i for i, v in enumerate(labels)}
    y = torch.tensor([float(index[java_str(v)]) for v in mt.column_values(label_col)], dtype=torch.float64,
                     device=dev)
    fm = extract_features(mt, fcols if vcol is None else None, vcol, dev)
    if fm.is_sparse:
        fm.set_ncols(layers[0])
    X = fm.to_dense().to(torch.float64)
    if X.shape[1] != layers[0]:
        X = torch.nn.functional.pad(X, (0, max(0, layers[0] - X.shape[1])))[:, :layers[0]]
    from ..common.features import FeatureMatrix
    data = LabeledData(FeatureMatrix(dense=X), y, torch.ones_like(y))
    nw = weight_size(layers)
    if params.contains("initialWeights") and params.get("initialWeights") is not None:
        iw = params.get("initialWeights")
        init = torch.as_tensor(np.asarray(getattr(iw, "data", iw), dtype=np.float64), device=dev)
        if init.numel() != nw:
            raise RuntimeError("Invalid initial weights, size mismatch")
    else:
        r = JavaRandom(1)
        init = torch.tensor([r.nextGaussian() * 0.05 for _ in range(nw)], dtype=torch.float64, device=dev)
    p = params.clone().set("numSearchStep", 3)
    obj = MlpObjFunc(layers, float(params.get("l1") or 0.0) if params.contains("l1") else 0.0,
                     float(params.get("l2") or 0.0) if params.contains("l2") else 0.0)
    coef, curve = optimize(obj, data, nw, p, method="LBFGS", env=env, init_coef=init)
    meta = Params().set("vectorCol", vcol).set("isVectorInput", vcol is not None).set("layers", layers) \
        .set("featureCols", fcols if vcol is None else None)
    return meta, np.asarray(coef), labels, mt.col_type(label_col)


class MlpcModelDataConverter(LabeledModelDataConverter):
    def serializeModel(self, m):
        meta, w, labels = m
        return meta, [gson_dumps(DenseVector(w), java_map_order=False)], labels

    def deserializeModel(self, meta, data, labels):
        return meta, np.asarray(json.loads(data[0])["data"], dtype=np.float64), list(labels)


class MlpcModelMapper(RichModelMapper):
    model = None

    def loadModel(self, rows):
        from ..linear.model import LinearModelDataConverter
        lt = LinearModelDataConverter.extractLabelType(self.modelSchema)
        meta, w, labels = MlpcModelDataConverter(lt).load(rows)
        self.meta, self.w = meta, torch.as_tensor(w)
        self.labels = [_recover_label(v, lt) for v in labels]
        self.layers = [int(x) for x in meta.get("layers")]
        self.vcol = meta.get("vectorCol") if meta.contains("vectorCol") else None
        self.fcols = meta.get("featureCols") if meta.contains("featureCols") else None
        if self.params.contains("vectorCol") and self.params.get("vectorCol"):
            self.vcol = self.params.get("vectorCol")
        names = [self.pred_col] + ([self.detail_col] if self.detail_col else [])
        types = [lt or Types.STRING] + ([Types.STRING] if self.detail_col else [])
        self.helper = OutputColsHelper(self.dataSchema, names, types, self.params.get("reservedCols")
                                       if self.params.contains("reservedCols") else None)

    def _map_row_values(self, row):
        mt = MTable.from_rows([tuple(row)], self.dataSchema)
        return [c.to_list()[0] for c in self._map_columns(mt)]

    def _map_columns(self, mt):
        fm = extract_features(mt, self.fcols if not self.vcol else None, self.vcol, torch.device("cpu"))
        if fm.is_sparse:
            fm.set_ncols(self.layers[0])
        X = fm.to_dense().double()
        if X.shape[1] != self.layers[0]:
            X = torch.nn.functional.pad(X, (0, max(0, self.layers[0] - X.shape[1])))[:, :self.layers[0]]
        P = mlp_forward(X, self.w, self.layers).numpy()
        preds = [self.labels[int(i)] for i in P.argmax(1)]
        cols = [Column.from_values(preds, self.helper.out_types[0])]
        if self.detail_col:
            cols.append(Column.from_values(
                [gson_dumps({java_str(self.labels[j]): float(p[j]) for j in range(len(self.labels))}) for p in P],
                Types.STRING))
        return cols
