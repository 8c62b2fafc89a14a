"""Pipeline stages of the non-linear classifiers (reference ``A/pipeline/classification/*``)."""
from ..models.classification.naive_bayes import NaiveBayesTextModelMapper
from ..operator.batch import classification_extra as C
from .base import MapModel, Trainer

__all__ = ["FmClassifier", "FmRegressor", "FmModel", "NaiveBayesTextClassifier", "NaiveBayesTextModel", "MultilayerPerceptronClassifier",
           "MultilayerPerceptronClassificationModel"]


class NaiveBayesTextClassifier(Trainer):
    TRAIN_OP = C.NaiveBayesTextTrainBatchOp
    MODEL = "NaiveBayesTextModel"


class NaiveBayesTextModel(MapModel):
    MAPPER = NaiveBayesTextModelMapper


from ..models.classification.mlp import MlpcModelMapper  # noqa: E402


class MultilayerPerceptronClassifier(Trainer):
    TRAIN_OP = C.MultilayerPerceptronTrainBatchOp
    MODEL = "MultilayerPerceptronClassificationModel"


class MultilayerPerceptronClassificationModel(MapModel):
    MAPPER = MlpcModelMapper


from ..models.recommendation.fm import FmModelMapper  # noqa: E402


class FmClassifier(Trainer):
    TRAIN_OP = C.FmClassifierTrainBatchOp
    MODEL = "FmModel"


class FmRegressor(Trainer):
    TRAIN_OP = C.FmRegressorTrainBatchOp
    MODEL = "FmModel"


class FmModel(MapModel):
    MAPPER = FmModelMapper
