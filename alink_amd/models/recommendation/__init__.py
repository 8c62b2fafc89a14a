"""Recommendation: ALS matrix factorisation (explicit / implicit, non-negative, mini-batched)."""
from .als import AlsModelData, AlsModelDataConverter, AlsModelMapper, als_topk, train_als  # noqa: F401
