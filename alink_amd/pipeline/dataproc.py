"""Data-processing pipeline stages (reference ``A/pipeline/dataproc/**``)."""
from ..common.params import ParamInfo
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
    EXTRA_PARAMS = [ParamInfo("vectorCol", str, "Name of a vector column", default=None),
                    ParamInfo("schemaStr", str, "Formatted schema", default=None),
                    ParamInfo("handleInvalid", str, "Strategy to handle unseen token", default="ERROR")]
