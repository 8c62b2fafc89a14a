"""Clustering pipeline stages (reference ``A/pipeline/clustering/*``)."""
from ..models.clustering.kmeans import KMeansModelMapper
from ..operator.batch.clustering import KMeansTrainBatchOp
from .base import MapModel, Trainer

__all__ = ["KMeans", "KMeansModel"]


class KMeans(Trainer):
    TRAIN_OP = KMeansTrainBatchOp
    MODEL = "KMeansModel"


class KMeansModel(MapModel):
    MAPPER = KMeansModelMapper
