"""Tree pipeline stages (reference ``A/pipeline/classification/{GbdtClassifier,RandomForestClassifier,
DecisionTreeClassifier}``, ``A/pipeline/regression/{GbdtRegressor,RandomForestRegressor,DecisionTreeRegressor}``
+ their models)."""
from ..models.tree.model import GbdtModelMapper, RandomForestModelMapper
from ..operator.batch import tree as T
from .base import MapModel, Trainer

__all__ = ["GbdtClassifier", "GbdtClassificationModel", "GbdtRegressor", "GbdtRegressionModel",
           "RandomForestClassifier", "RandomForestClassificationModel", "RandomForestRegressor",
           "RandomForestRegressionModel", "DecisionTreeClassifier", "DecisionTreeClassificationModel",
           "DecisionTreeRegressor", "DecisionTreeRegressionModel"]


class GbdtClassifier(Trainer):
    TRAIN_OP = T.GbdtTrainBatchOp
    MODEL = "GbdtClassificationModel"


class GbdtClassificationModel(MapModel):
    MAPPER = GbdtModelMapper


class GbdtRegressor(Trainer):
    TRAIN_OP = T.GbdtRegTrainBatchOp
    MODEL = "GbdtRegressionModel"


class GbdtRegressionModel(MapModel):
    MAPPER = GbdtModelMapper


class RandomForestClassifier(Trainer):
    TRAIN_OP = T.RandomForestTrainBatchOp
    MODEL = "RandomForestClassificationModel"


class RandomForestClassificationModel(MapModel):
    MAPPER = RandomForestModelMapper


class RandomForestRegressor(Trainer):
    TRAIN_OP = T.RandomForestRegTrainBatchOp
    MODEL = "RandomForestRegressionModel"


class RandomForestRegressionModel(MapModel):
    MAPPER = RandomForestModelMapper


class DecisionTreeClassifier(Trainer):
    TRAIN_OP = T.DecisionTreeTrainBatchOp
    MODEL = "DecisionTreeClassificationModel"


class DecisionTreeClassificationModel(MapModel):
    MAPPER = RandomForestModelMapper


class DecisionTreeRegressor(Trainer):
    TRAIN_OP = T.DecisionTreeRegTrainBatchOp
    MODEL = "DecisionTreeRegressionModel"


class DecisionTreeRegressionModel(MapModel):
    MAPPER = RandomForestModelMapper
