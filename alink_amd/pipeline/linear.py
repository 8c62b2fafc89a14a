"""Linear-family pipeline stages (reference ``A/pipeline/classification/{LogisticRegression,LinearSvm,Softmax}``,
``A/pipeline/regression/{LinearRegression,RidgeRegression,LassoRegression,AftSurvivalRegression}`` + models)."""
from ..models.linear.model import AFTModelMapper, LinearModelMapper, SoftmaxModelMapper
from ..operator.batch import linear as L
from .base import MapModel, Trainer

__all__ = ["LogisticRegression", "LogisticRegressionModel", "LinearSvm", "LinearSvmModel", "LinearRegression",
           "LinearRegressionModel", "RidgeRegression", "RidgeRegressionModel", "LassoRegression",
           "LassoRegressionModel", "Softmax", "SoftmaxModel", "AftSurvivalRegression", "AftSurvivalRegressionModel"]


class LogisticRegression(Trainer):
    TRAIN_OP = L.LogisticRegressionTrainBatchOp
    MODEL = "LogisticRegressionModel"


class LogisticRegressionModel(MapModel):
    MAPPER = LinearModelMapper


class LinearSvm(Trainer):
    TRAIN_OP = L.LinearSvmTrainBatchOp
    MODEL = "LinearSvmModel"


class LinearSvmModel(MapModel):
    MAPPER = LinearModelMapper


class LinearRegression(Trainer):
    TRAIN_OP = L.LinearRegTrainBatchOp
    MODEL = "LinearRegressionModel"


class LinearRegressionModel(MapModel):
    MAPPER = LinearModelMapper


class RidgeRegression(Trainer):
    TRAIN_OP = L.RidgeRegTrainBatchOp
    MODEL = "RidgeRegressionModel"


class RidgeRegressionModel(MapModel):
    MAPPER = LinearModelMapper


class LassoRegression(Trainer):
    TRAIN_OP = L.LassoRegTrainBatchOp
    MODEL = "LassoRegressionModel"


class LassoRegressionModel(MapModel):
    MAPPER = LinearModelMapper


class Softmax(Trainer):
    TRAIN_OP = L.SoftmaxTrainBatchOp
    MODEL = "SoftmaxModel"


class SoftmaxModel(MapModel):
    MAPPER = SoftmaxModelMapper


class AftSurvivalRegression(Trainer):
    TRAIN_OP = L.AftSurvivalRegTrainBatchOp
    MODEL = "AftSurvivalRegressionModel"


class AftSurvivalRegressionModel(MapModel):
    MAPPER = AFTModelMapper
