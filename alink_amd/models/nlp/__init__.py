"""NLP: tokenizers, stop words, n-grams, segmentation, document vectorizers, Word2Vec."""
from .text import *  # noqa: F401,F403
from .word2vec import Word2VecModelMapper, train_word2vec  # noqa: F401
