"""Clustering batch operators (reference ``A/operator/batch/clustering/*``)."""
from __future__ import annotations

from typing import Optional

import torch

from ...common.params import ParamInfo, Params
from ...common.table import MTable
from ...models.clustering.kmeans import KMeansModelDataConverter, KMeansModelMapper, train_kmeans
from ..base import BatchOperator
from .utils import ModelMapBatchOp

__all__ = ["KMeansTrainBatchOp", "KMeansPredictBatchOp", "vector_tensor", "GmmTrainBatchOp", "GmmPredictBatchOp",
           "BisectingKMeansTrainBatchOp", "BisectingKMeansPredictBatchOp", "LdaTrainBatchOp", "LdaPredictBatchOp"]


def vector_tensor(mt: MTable, col: str, device) -> torch.Tensor:
    """This rank's rows of a vector column as an [n, d] device tensor (bf16/fp32 blocks keep their dtype)."""
    c = mt.col(col)
    v = c.values
    if isinstance(v, torch.Tensor) and v.dim() == 2:
        return v.to(device) if v.device != device else v
    if isinstance(v, torch.Tensor):
        return v.reshape(-1, 1).to(device=device, dtype=torch.float64)
    from ...parallel import comm
    # vector sizes must agree across ranks: use the global max size
    blk = mt.vector_block(col, dtype=torch.float64)
    d = max(comm.all_gather_object(int(blk.shape[1]) if blk.shape[0] else 0))
    if blk.shape[1] < d:
        blk = torch.nn.functional.pad(blk, (0, d - blk.shape[1]))
    return blk.to(device)


class KMeansTrainBatchOp(BatchOperator):
    """k-means on the BSP engine (see ``models/clustering/kmeans.py``)."""
    EXTRA_PARAMS = [ParamInfo("randomSeed", int, "seed of the k-means|| / random initialisation", default=0)]

    def linkFrom(self, *inputs):
        inp = self.checkAndGetFirst(inputs)
        mt = inp.getOutputTable()
        env = self.env
        X = vector_tensor(mt, self.getVectorCol(), env.device)
        dt = str(self.getDistanceType().name if hasattr(self.getDistanceType(), "name") else self.getDistanceType())
        im = self.getInitMode()
        im = im.name if hasattr(im, "name") else str(im)
        rows, q = train_kmeans(X, self.getK(), self.getMaxIter(), self.getEpsilon(), dt, im, self.getInitSteps(),
                               self.getVectorCol(), env, seed=self.getParams().get(self._param_infos["randomSeed"]),
                               on_step=getattr(self, "_on_step", None),
                               sync_steps=getattr(self, "_sync_steps", ()))
        self._queue = q
        self.setOutputTable(MTable.from_rows(rows, KMeansModelDataConverter().getModelSchema(), replicated=True))
        return self

    def getTrainInfo(self):
        q = getattr(self, "_queue", None)
        crit = getattr(q, "criterion", None) if q else None
        return {"iterations": q.step_no if q else None, "steps": q.stats if q else None,
                "max_shift": list(getattr(crit, "history", []))}


class KMeansPredictBatchOp(ModelMapBatchOp):
    MAPPER = KMeansModelMapper


class GmmTrainBatchOp(BatchOperator):
    """EM for a Gaussian mixture (``models/clustering/gmm.py``)."""

    def linkFrom(self, *inputs):
        from ...common.model.converter import SimpleModelDataConverter
        from ...models.clustering.gmm import train_gmm
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        rows = train_gmm(mt, self.getParams(), self.env)
        self.setOutputTable(MTable.from_rows(rows, SimpleModelDataConverter().getModelSchema(), replicated=True))
        return self


class BisectingKMeansTrainBatchOp(BatchOperator):
    """Bisecting k-means (``models/clustering/bisecting.py``)."""

    def linkFrom(self, *inputs):
        from ...common.model.converter import SimpleModelDataConverter
        from ...models.clustering.bisecting import train_bisecting_kmeans
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        rows = train_bisecting_kmeans(mt, self.getParams(), self.env)
        self.setOutputTable(MTable.from_rows(rows, SimpleModelDataConverter().getModelSchema(), replicated=True))
        return self


from ...models.clustering.bisecting import BisectingKMeansModelMapper  # noqa: E402
from ...models.clustering.gmm import GmmModelMapper  # noqa: E402


class GmmPredictBatchOp(ModelMapBatchOp):
    MAPPER = GmmModelMapper


class BisectingKMeansPredictBatchOp(ModelMapBatchOp):
    MAPPER = BisectingKMeansModelMapper


class LdaTrainBatchOp(BatchOperator):
    """LDA, collapsed Gibbs ("em") or online variational Bayes (``models/clustering/lda.py``)."""

    def linkFrom(self, *inputs):
        from ...common.model.converter import SimpleModelDataConverter
        from ...models.clustering.lda import train_lda
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        rows = train_lda(mt, self.getParams(), self.env)
        self.setOutputTable(MTable.from_rows(rows, SimpleModelDataConverter().getModelSchema(), replicated=True))
        return self


from ...models.clustering.lda import LdaModelMapper  # noqa: E402


class LdaPredictBatchOp(ModelMapBatchOp):
    MAPPER = LdaModelMapper
