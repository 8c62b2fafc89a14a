"""Scalar / table function registry for SQL and ``udf``/``udtf`` ops (reference ``BatchOperator.registerFunction``,
``docs/pyalink/pyalink-udf.md``)."""
from typing import Callable, Dict, Optional

_FUNCS: Dict[str, Callable] = {}


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
