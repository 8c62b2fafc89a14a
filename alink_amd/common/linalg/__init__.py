from .vector import DenseVector, SparseVector, Vector, VectorUtil, VectorIterator
from .matrix import DenseMatrix
from .block import SparseBlock

__all__ = ["DenseVector", "SparseVector", "Vector", "VectorUtil", "VectorIterator", "DenseMatrix", "SparseBlock"]
