"""NLP pipeline stages (reference ``A/pipeline/nlp/*``)."""
from ..models.nlp import text as T
from ..models.nlp import word2vec as W
from ..operator.batch import nlp as N
from .base import MapModel, MapTransformer, Trainer

__all__ = ["Tokenizer", "RegexTokenizer", "StopWordsRemover", "NGram", "Segment", "DocCountVectorizer",
           "DocCountVectorizerModel", "DocHashCountVectorizer", "DocHashCountVectorizerModel", "Word2Vec", "Word2VecModel"]


class Tokenizer(MapTransformer):
    MAPPER = T.TokenizerMapper


class RegexTokenizer(MapTransformer):
    MAPPER = T.RegexTokenizerMapper


class StopWordsRemover(MapTransformer):
    MAPPER = T.StopWordsRemoverMapper


class NGram(MapTransformer):
    MAPPER = T.NGramMapper


class Segment(MapTransformer):
    MAPPER = T.SegmentMapper


class DocCountVectorizer(Trainer):
    TRAIN_OP = N.DocCountVectorizerTrainBatchOp
    MODEL = "DocCountVectorizerModel"


class DocCountVectorizerModel(MapModel):
    MAPPER = T.DocCountVectorizerModelMapper


class DocHashCountVectorizer(Trainer):
    TRAIN_OP = N.DocHashCountVectorizerTrainBatchOp
    MODEL = "DocHashCountVectorizerModel"


class DocHashCountVectorizerModel(MapModel):
    MAPPER = T.DocHashCountVectorizerModelMapper


class Word2Vec(Trainer):
    TRAIN_OP = N.Word2VecTrainBatchOp
    MODEL = "Word2VecModel"


class Word2VecModel(MapModel):
    MAPPER = W.Word2VecModelMapper
