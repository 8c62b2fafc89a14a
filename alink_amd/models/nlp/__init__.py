"""NLP: tokenizers, stop words, n-grams, segmentation, document vectorizers, Word2Vec."""
from .text import *  # noqa: F401,F403
