"""Stream predict operators: a batch-trained model applied to every micro-batch.

Reference: ``A/operator/stream/{classification,regression,clustering,...}/*PredictStreamOp.java`` — each is a
``ModelMapStreamOp`` bound to the same ``ModelMapper`` as its batch twin (model pre-collected through
DirectReader, ``ModelMapStreamOp.java:39-56``).
"""
from __future__ import annotations

from ...models.clustering import bisecting as _BKM
from ...models.clustering import gmm as _GMM
from ...models.clustering import lda as _LDA
from ...models.clustering.kmeans import KMeansModelMapper
from ...models.linear.model import AFTModelMapper, LinearModelMapper, SoftmaxModelMapper
from ...models.feature import encoders as _E
from ...models.feature import pca as _PCA
from ...models.feature import scalers as _S
from ...models.classification import mlp as _MLP
from ...models.classification.naive_bayes import NaiveBayesTextModelMapper
from ...models.nlp import text as _T
from ...models.nlp import word2vec as _W
from ...models.recommendation.als import AlsModelMapper
from ...models.recommendation.fm import FmModelMapper
from ...models.tree.model import GbdtModelMapper, RandomForestModelMapper
from ...models.regression.glm import GlmModelMapper
from ...models.regression.isotonic import IsotonicRegressionModelMapper
from .base import MapStreamOp, ModelMapStreamOp

_PREDICTORS = {
    # FM has no stream predictor in the reference; the twins below apply the same FmModelMapper per micro-batch
    "FmClassifierPredictStreamOp": FmModelMapper,
    "FmRegressorPredictStreamOp": FmModelMapper,
    "KMeansPredictStreamOp": KMeansModelMapper,
    "LogisticRegressionPredictStreamOp": LinearModelMapper,
    "LinearSvmPredictStreamOp": LinearModelMapper,
    "LinearRegPredictStreamOp": LinearModelMapper,
    "RidgeRegPredictStreamOp": LinearModelMapper,
    "LassoRegPredictStreamOp": LinearModelMapper,
    "SoftmaxPredictStreamOp": SoftmaxModelMapper,
    "AftSurvivalRegPredictStreamOp": AFTModelMapper,
    "StandardScalerPredictStreamOp": _S.StandardScalerModelMapper,
    "MinMaxScalerPredictStreamOp": _S.MinMaxScalerModelMapper,
    "MaxAbsScalerPredictStreamOp": _S.MaxAbsScalerModelMapper,
    "ImputerPredictStreamOp": _S.ImputerModelMapper,
    "VectorStandardScalerPredictStreamOp": _S.VectorScalerModelMapper,
    "VectorMinMaxScalerPredictStreamOp": _S.VectorScalerModelMapper,
    "VectorMaxAbsScalerPredictStreamOp": _S.VectorScalerModelMapper,
    "VectorImputerPredictStreamOp": _S.VectorImputerModelMapper,
    "StringIndexerPredictStreamOp": _E.StringIndexerModelMapper,
    "MultiStringIndexerPredictStreamOp": _E.MultiStringIndexerModelMapper,
    "IndexToStringPredictStreamOp": _E.IndexToStringModelMapper,
    "OneHotPredictStreamOp": _E.OneHotModelMapper,
    "QuantileDiscretizerPredictStreamOp": _E.QuantileDiscretizerModelMapper,
    "GbdtPredictStreamOp": GbdtModelMapper,
    "GbdtRegPredictStreamOp": GbdtModelMapper,
    "RandomForestPredictStreamOp": RandomForestModelMapper,
    "RandomForestRegPredictStreamOp": RandomForestModelMapper,
    "DecisionTreePredictStreamOp": RandomForestModelMapper,
    "DecisionTreeRegPredictStreamOp": RandomForestModelMapper,
    "AlsPredictStreamOp": AlsModelMapper,
    "DocCountVectorizerPredictStreamOp": _T.DocCountVectorizerModelMapper,
    "DocHashCountVectorizerPredictStreamOp": _T.DocHashCountVectorizerModelMapper,
    "Word2VecPredictStreamOp": _W.Word2VecModelMapper,
    "NaiveBayesTextPredictStreamOp": NaiveBayesTextModelMapper,
    "PcaPredictStreamOp": _PCA.PcaModelMapper,
    "GmmPredictStreamOp": _GMM.GmmModelMapper,
    "BisectingKMeansPredictStreamOp": _BKM.BisectingKMeansModelMapper,
    "LdaPredictStreamOp": _LDA.LdaModelMapper,
    "MultilayerPerceptronPredictStreamOp": _MLP.MlpcModelMapper,
    "GlmPredictStreamOp": GlmModelMapper,
    "IsotonicRegPredictStreamOp": IsotonicRegressionModelMapper,
}

_MAPPERS = {
    "BinarizerStreamOp": _E.BinarizerMapper,
    "BucketizerStreamOp": _E.BucketizerMapper,
    "FeatureHasherStreamOp": _E.FeatureHasherMapper,
    "DCTStreamOp": _E.DCTMapper,
    "TokenizerStreamOp": _T.TokenizerMapper,
    "RegexTokenizerStreamOp": _T.RegexTokenizerMapper,
    "StopWordsRemoverStreamOp": _T.StopWordsRemoverMapper,
    "NGramStreamOp": _T.NGramMapper,
    "SegmentStreamOp": _T.SegmentMapper,
}

__all__ = []


def register_stream_predictor(name: str, mapper):
    cls = type(name, (ModelMapStreamOp,), {"MAPPER": mapper, "__module__": __name__,
                                          "__doc__": f"Stream predict with ``{mapper.__name__}``."})
    globals()[name] = cls
    if name not in __all__:
        __all__.append(name)
    return cls


def register_stream_mapper(name: str, mapper):
    cls = type(name, (MapStreamOp,), {"MAPPER": mapper, "__module__": __name__,
                                     "__doc__": f"Stream transform with ``{mapper.__name__}``."})
    globals()[name] = cls
    if name not in __all__:
        __all__.append(name)
    return cls


for _n, _m in _PREDICTORS.items():
    register_stream_predictor(_n, _m)
for _n, _m in _MAPPERS.items():
    register_stream_mapper(_n, _m)
