from .base import AlgoOperator, BatchOperator  # noqa: F401
