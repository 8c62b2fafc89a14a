"""Clustering pipeline stages (reference ``A/pipeline/clustering/*``)."""
from ..models.clustering.kmeans import KMeansModelMapper
from ..operator.batch.clustering import KMeansTrainBatchOp
from .base import MapModel, Trainer

__all__ = ["KMeans", "KMeansModel", "GaussianMixture", "GaussianMixtureModel", "BisectingKMeans",
           "BisectingKMeansModel", "Lda", "LdaModel"]


class KMeans(Trainer):
    TRAIN_OP = KMeansTrainBatchOp
    MODEL = "KMeansModel"


class KMeansModel(MapModel):
    MAPPER = KMeansModelMapper


from ..models.clustering.bisecting import BisectingKMeansModelMapper  # noqa: E402
from ..models.clustering.gmm import GmmModelMapper  # noqa: E402
from ..operator.batch.clustering import BisectingKMeansTrainBatchOp, GmmTrainBatchOp  # noqa: E402


class GaussianMixture(Trainer):
    TRAIN_OP = GmmTrainBatchOp
    MODEL = "GaussianMixtureModel"


class GaussianMixtureModel(MapModel):
    MAPPER = GmmModelMapper


class BisectingKMeans(Trainer):
    TRAIN_OP = BisectingKMeansTrainBatchOp
    MODEL = "BisectingKMeansModel"


class BisectingKMeansModel(MapModel):
    MAPPER = BisectingKMeansModelMapper


from ..models.clustering.lda import LdaModelMapper  # noqa: E402
from ..operator.batch.clustering import LdaTrainBatchOp  # noqa: E402


class Lda(Trainer):
    TRAIN_OP = LdaTrainBatchOp
    MODEL = "LdaModel"


class LdaModel(MapModel):
    MAPPER = LdaModelMapper
