"""ALS pipeline stages (reference ``A/pipeline/recommendation/{ALS,ALSModel}.java``)."""
from ..models.recommendation.als import AlsModelMapper
from ..operator.batch.recommendation import AlsTrainBatchOp
from .base import MapModel, Trainer

__all__ = ["ALS", "ALSModel"]


class ALS(Trainer):
    TRAIN_OP = AlsTrainBatchOp
    MODEL = "ALSModel"


class ALSModel(MapModel):
    MAPPER = AlsModelMapper
