from .vector import DenseVector, SparseVector, Vector, VectorUtil, VectorIterator
from .matrix import DenseMatrix

__all__ = ["DenseVector", "SparseVector", "Vector", "VectorUtil", "VectorIterator", "DenseMatrix"]
