"""GLM / isotonic-regression pipeline stages (reference ``A/pipeline/regression/{GeneralizedLinearRegression,
IsotonicRegression}*.java``)."""
from ..models.regression.glm import GlmModelMapper
from ..models.regression.isotonic import IsotonicRegressionModelMapper
from ..operator.batch import regression_extra as R
from .base import MapModel, Trainer

__all__ = ["GeneralizedLinearRegression", "GeneralizedLinearRegressionModel", "IsotonicRegression",
           "IsotonicRegressionModel"]


class GeneralizedLinearRegression(Trainer):
    TRAIN_OP = R.GlmTrainBatchOp
    MODEL = "GeneralizedLinearRegressionModel"


class GeneralizedLinearRegressionModel(MapModel):
    MAPPER = GlmModelMapper


class IsotonicRegression(Trainer):
    TRAIN_OP = R.IsotonicRegTrainBatchOp
    MODEL = "IsotonicRegressionModel"


class IsotonicRegressionModel(MapModel):
    MAPPER = IsotonicRegressionModelMapper
