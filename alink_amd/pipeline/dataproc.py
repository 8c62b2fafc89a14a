"""Data-processing pipeline stages (reference ``A/pipeline/dataproc/**``)."""
from ..models.dataproc import vector as V
from .base import MapTransformer

__all__ = ["VectorAssembler", "VectorNormalizer", "VectorSlicer", "VectorElementwiseProduct", "VectorInteraction",
           "VectorPolynomialExpand", "VectorSizeHint", "VectorToColumns"]


class VectorAssembler(MapTransformer):
    MAPPER = V.VectorAssemblerMapper


class VectorNormalizer(MapTransformer):
    MAPPER = V.VectorNormalizeMapper


class VectorSlicer(MapTransformer):
    MAPPER = V.VectorSliceMapper


class VectorElementwiseProduct(MapTransformer):
    MAPPER = V.VectorElementwiseProductMapper


class VectorInteraction(MapTransformer):
    MAPPER = V.VectorInteractionMapper


class VectorPolynomialExpand(MapTransformer):
    MAPPER = V.VectorPolynomialExpandMapper


class VectorSizeHint(MapTransformer):
    MAPPER = V.VectorSizeHintMapper


class VectorToColumns(MapTransformer):
    MAPPER = V.VectorToColumnsMapper
