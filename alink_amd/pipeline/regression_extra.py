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

    def evaluate(self, data):
        """GLM summary (coefficients, deviance, AIC, ...) of ``data`` under this model (reference
        ``GeneralizedLinearRegressionModel.evaluate``)."""
        from ..operator.base import BatchOperator
        return R.GlmEvaluationBatchOp(self.getParams().clone()).linkFrom(
            BatchOperator.fromTable(self.getModelData()).setMLEnvironmentId(self.getMLEnvironmentId()), data)


class IsotonicRegression(Trainer):
    TRAIN_OP = R.IsotonicRegTrainBatchOp
    MODEL = "IsotonicRegressionModel"


class IsotonicRegressionModel(MapModel):
    MAPPER = IsotonicRegressionModelMapper
