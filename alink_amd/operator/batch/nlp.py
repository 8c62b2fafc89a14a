"""NLP batch operators (reference ``A/operator/batch/nlp/*``); mappers in ``models/nlp/text.py``."""
from __future__ import annotations

from ...common.model.converter import SimpleModelDataConverter
from ...common.table import MTable
from ...models.nlp import text as T
from ...models.nlp import word2vec as W
from ..base import BatchOperator
from .utils import MapBatchOp, ModelMapBatchOp

__all__ = ["TokenizerBatchOp", "RegexTokenizerBatchOp", "StopWordsRemoverBatchOp", "NGramBatchOp", "SegmentBatchOp",
           "DocCountVectorizerTrainBatchOp", "DocCountVectorizerPredictBatchOp",
           "DocHashCountVectorizerTrainBatchOp", "DocHashCountVectorizerPredictBatchOp", "Word2VecTrainBatchOp",
           "Word2VecPredictBatchOp"]


class TokenizerBatchOp(MapBatchOp):
    MAPPER = T.TokenizerMapper


class RegexTokenizerBatchOp(MapBatchOp):
    MAPPER = T.RegexTokenizerMapper


class StopWordsRemoverBatchOp(MapBatchOp):
    MAPPER = T.StopWordsRemoverMapper


class NGramBatchOp(MapBatchOp):
    MAPPER = T.NGramMapper


class SegmentBatchOp(MapBatchOp):
    MAPPER = T.SegmentMapper


class DocCountVectorizerTrainBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        rows = T.train_doc_count_vectorizer(mt, self.getParams())
        self.setOutputTable(MTable.from_rows(rows, SimpleModelDataConverter().getModelSchema(), replicated=True))
        return self


class DocHashCountVectorizerTrainBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        rows = T.train_doc_hash_count_vectorizer(mt, self.getParams())
        self.setOutputTable(MTable.from_rows(rows, SimpleModelDataConverter().getModelSchema(), replicated=True))
        return self


class DocCountVectorizerPredictBatchOp(ModelMapBatchOp):
    MAPPER = T.DocCountVectorizerModelMapper


class DocHashCountVectorizerPredictBatchOp(ModelMapBatchOp):
    MAPPER = T.DocHashCountVectorizerModelMapper


class Word2VecTrainBatchOp(BatchOperator):
    def linkFrom(self, *inputs):
        mt = self.checkAndGetFirst(inputs).getOutputTable()
        rows = W.train_word2vec(mt, self.getParams(), self.env)
        self.setOutputTable(MTable.from_rows(rows, W.MODEL_SCHEMA, replicated=True))
        return self


class Word2VecPredictBatchOp(ModelMapBatchOp):
    MAPPER = W.Word2VecModelMapper
