"""Pipeline stages of the non-linear classifiers (reference ``A/pipeline/classification/*``)."""
from ..models.classification.naive_bayes import NaiveBayesTextModelMapper
from ..operator.batch import classification_extra as C
from .base import MapModel, Trainer

__all__ = ["NaiveBayesTextClassifier", "NaiveBayesTextModel"]


class NaiveBayesTextClassifier(Trainer):
    TRAIN_OP = C.NaiveBayesTextTrainBatchOp
    MODEL = "NaiveBayesTextModel"


class NaiveBayesTextModel(MapModel):
    MAPPER = NaiveBayesTextModelMapper
