"""Alink parameter catalogue.

``_spec.py`` is generated (tools/gen_param_spec.py) from the reference's ~450 param interfaces
(``A/params/**``).  This module turns that table into ``ParamInfo`` objects and Python ``Enum``
classes, and resolves the interface inheritance so an operator class gets every
``setXxx/getXxx`` its Alink counterpart exposes.
"""
from __future__ import annotations

import enum
from functools import lru_cache
from typing import Dict, List, Optional

from ..common.params import ParamInfo
from . import _spec

__all__ = ["interface_params", "op_params", "get_enum", "param", "ENUM_CACHE"]

ENUM_CACHE: Dict[str, type] = {}

_JTYPE = {
    "String": str, "Integer": int, "int": int, "Long": int, "long": int, "Double": float, "double": float,
    "Float": float, "float": float, "Boolean": bool, "boolean": bool, "Character": str,
    "String[]": [str], "Integer[]": [int], "int[]": [int], "Long[]": [int], "long[]": [int],
    "Double[]": [float], "double[]": [float], "double[][]": object, "DenseVector": object,
    "Object": object,
}


def get_enum(name: str, owner: Optional[str] = None) -> type:
    """Python Enum for a Java enum; ``owner`` is the declaring file (for nested enums)."""
    key = f"{owner}.{name}" if owner and f"{owner}.{name}" in _spec.ENUMS else name
    if key not in _spec.ENUMS:
        raise KeyError(f"unknown enum {name} (owner {owner})")
    if key not in ENUM_CACHE:
        members = _spec.ENUMS[key]
        ENUM_CACHE[key] = enum.Enum(name, [(m, m) for m in members])
    return ENUM_CACHE[key]


def _make_info(entry: dict, owner: str) -> ParamInfo:
    jt = entry["jtype"]
    vt = _JTYPE.get(jt)
    if vt is None:
        try:
            vt = get_enum(jt, owner)
        except KeyError:
            vt = object
    default = entry["default"]
    if isinstance(default, dict) and "__enum__" in default and isinstance(vt, type) and issubclass(vt, enum.Enum):
        default = vt[default["__enum__"]] if default["__enum__"] in vt.__members__ else None
    elif isinstance(default, dict):
        default = None
    if vt is float and isinstance(default, int) and not isinstance(default, bool):
        default = float(default)
    kw = {}
    if entry["has_default"]:
        kw["default"] = default
    return ParamInfo(entry["name"], vt, entry["desc"], optional=not entry["required"],
                     alias=entry["alias"], **kw)


@lru_cache(maxsize=None)
def _iface_own(name: str):
    it = _spec.INTERFACES.get(name)
    if it is None:
        return ()
    return tuple(_make_info(e, it["file"]) for e in it["params"])


def interface_params(name: str, _seen=None) -> List[ParamInfo]:
    """All ``ParamInfo`` of a param interface including the ones it extends (depth-first)."""
    seen = set() if _seen is None else _seen
    if name in seen:
        return []
    seen.add(name)
    out: List[ParamInfo] = []
    it = _spec.INTERFACES.get(name)
    if it is None:
        return out
    for parent in it["extends"]:
        out.extend(interface_params(parent, seen))
    out.extend(_iface_own(name))
    return out


def op_params(op_name: str) -> List[ParamInfo]:
    """Param list of a reference operator / pipeline stage by class name (walks ``extends``).  A stream operator
    the reference does not have (e.g. ``LdaPredictStreamOp``) takes the params of its batch twin."""
    out: Dict[str, ParamInfo] = {}
    if op_name not in _spec.OPS and op_name.endswith("StreamOp") and op_name[:-8] + "BatchOp" in _spec.OPS:
        op_name = op_name[:-8] + "BatchOp"
    cur = op_name
    chain = []
    while cur and cur in _spec.OPS and cur not in chain:
        chain.append(cur)
        cur = _spec.OPS[cur]["extends"]
    for c in reversed(chain):
        for iface in _spec.OPS[c]["implements"]:
            for p in interface_params(iface):
                out.setdefault(p.name, p)
        for p in _iface_own(c):
            out.setdefault(p.name, p)
    return list(out.values())


@lru_cache(maxsize=None)
def _by_name():
    d: Dict[str, ParamInfo] = {}
    for iname in _spec.INTERFACES:
        for p in _iface_own(iname):
            d.setdefault(p.name, p)
    return d


def param(name: str) -> ParamInfo:
    """Look up a ParamInfo by param name (first declaration wins)."""
    return _by_name()[name]
