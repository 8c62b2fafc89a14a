from .vector import DenseVector, SparseVector, Vector, VectorUtil, VectorIterator
from .matrix import DenseMatrix
from .block import SparseBlock
from .blas import BLAS, MatVecOp, NormalEquation

__all__ = ["DenseVector", "SparseVector", "Vector", "VectorUtil", "VectorIterator", "DenseMatrix", "SparseBlock",
           "BLAS", "MatVecOp", "NormalEquation"]
