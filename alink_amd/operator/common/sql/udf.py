"""Scalar / table function registry for SQL and ``udf``/``udtf`` ops (reference ``BatchOperator.registerFunction``,
``docs/pyalink/pyalink-udf.md``)."""
from typing import Callable, Dict, List, Optional

_FUNCS: Dict[str, Callable] = {}


class ScalarFunction:
    """A scalar UDF in the reference's (Flink) form: subclass with ``eval(*args)`` and optionally
    ``getResultType(*signature)`` returning the result type (an Alink type or its name)."""

    def getResultType(self, *signature):
        return None

    @property
    def result_type(self):
        return self.getResultType()


class TableFunction:
    """A table UDF in the reference's (Flink) form: ``eval(*args)`` emits any number of rows through
    ``self.collect(row)``; ``getResultType`` may name the output column types."""

    def __init__(self):
        self._rows: List = []

    def collect(self, row):
        self._rows.append(row)

    def getResultType(self, *signature):
        return None

    @property
    def result_types(self):
        return self.getResultType()

    def __call__(self, *args):
        self._rows = []
        self.eval(*args)
        out, self._rows = self._rows, []
        return out


def register_function(name: str, fn: Callable):
    _FUNCS[name.upper()] = getattr(fn, "eval", fn)


def get_registered_function(name: str) -> Callable:
    f = _FUNCS.get(name.upper())
    if f is None:
        raise ValueError(f"No such function: {name}")
    return f


def udf(func: Callable = None, result_type: Optional[str] = None):
    """PyAlink-style ``udf(func, result_type="DOUBLE")`` wrapper."""
    def wrap(f):
        f.result_type = result_type
        return f
    return wrap(func) if func is not None else wrap


def udtf(func: Callable = None, result_types=None):
    def wrap(f):
        f.result_types = result_types
        return f
    return wrap(func) if func is not None else wrap
