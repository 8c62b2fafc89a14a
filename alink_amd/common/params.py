"""Params / ParamInfo / WithParams — Alink-compatible configuration system.

Mirrors ``F/api/misc/param/Params.java:19-289`` (a ``HashMap<String,String>`` whose values are Gson
JSON strings, alias lookup on ``get``, defaults), ``ParamInfo.java:46-145`` and the ``WithParams``
mixin (``WithParams.java:8-28``).  Unlike the reference, validators are enforced on ``set``
(SURVEY §2.7 notes the reference never calls them).

Python ergonomics: an operator class lists its ``ParamInfo`` objects in ``PARAMS``; the
``ParamsMeta`` metaclass generates the PyAlink-style ``setXxx`` / ``getXxx`` camel-case accessors.
"""
from __future__ import annotations

import enum
import json
import math
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence

from .javafmt import gson_dumps, java_hashmap_order

__all__ = ["ParamInfo", "Params", "WithParams", "ParamsMeta", "ParamValidationError", "RangeValidator",
           "MinValidator", "InValidator"]

_NO_DEFAULT = object()


class ParamValidationError(ValueError):
    pass


class RangeValidator:
    """Closed/open interval check (reference ``A/params/validators/RangeValidator.java``)."""

    def __init__(self, lo=None, hi=None, left_inclusive=True, right_inclusive=True):
        self.lo, self.hi, self.li, self.ri = lo, hi, left_inclusive, right_inclusive

    def __call__(self, v) -> bool:
        if v is None:
            return True
        if self.lo is not None and (v < self.lo or (v == self.lo and not self.li)):
            return False
        if self.hi is not None and (v > self.hi or (v == self.hi and not self.ri)):
            return False
        return True

    def __repr__(self):
        return f"Range({self.lo}, {self.hi})"


def MinValidator(lo, inclusive=True):
    return RangeValidator(lo, None, inclusive, True)


class InValidator:
    def __init__(self, *vals):
        self.vals = set(vals)

    def __call__(self, v):
        return v is None or v in self.vals


class ParamInfo:
    """Definition of one parameter: name, aliases, value type, default, optional flag, validator.

    ``value_type`` is one of: ``int``, ``float``, ``str``, ``bool``, an ``enum.Enum`` subclass,
    ``list`` forms ``[int]``/``[float]``/``[str]`` (Java arrays), or ``object`` (raw JSON value).
    """

    def __init__(self, name: str, value_type: Any = str, description: str = "", *,
                 optional: bool = True, default: Any = _NO_DEFAULT, alias: Sequence[str] = (),
                 validator: Optional[Callable[[Any], bool]] = None):
        self.name = name
        self.value_type = value_type
        self.description = description
        self.alias = tuple(alias or ())
        self.validator = validator
        self._default = default
        self.optional = optional if default is _NO_DEFAULT else True

    @property
    def has_default(self) -> bool:
        return self._default is not _NO_DEFAULT

    @property
    def default(self):
        return None if self._default is _NO_DEFAULT else self._default

    def names(self):
        return (self.name,) + self.alias

    # --- value coercion ---------------------------------------------------------------------
    def coerce(self, v):
        """Coerce a user-supplied Python value to the declared Java-side type."""
        if v is None:
            return None
        t = self.value_type
        if isinstance(t, type) and issubclass(t, enum.Enum):
            if isinstance(v, t):
                return v
            return search_enum(t, str(v), self.name)
        if t is int:
            if isinstance(v, bool):
                raise ParamValidationError(f"{self.name}: expect int, got bool")
            if isinstance(v, float) and not v.is_integer():
                raise ParamValidationError(f"{self.name}: expect int, got {v}")
            return int(v)
        if t is float:
            return float(v)
        if t is bool:
            if isinstance(v, str):
                return v.strip().lower() == "true"
            return bool(v)
        if t is str:
            return str(v) if not isinstance(v, str) else v
        if isinstance(t, list):
            et = t[0] if t else object
            if isinstance(v, (str, bytes)) or not hasattr(v, "__iter__"):
                v = [v]
            out = []
            for e in v:
                if e is None:
                    out.append(None)
                elif isinstance(et, type) and issubclass(et, enum.Enum):
                    out.append(e if isinstance(e, et) else search_enum(et, str(e), self.name))
                elif et in (int, float, str, bool):
                    out.append(et(e))
                else:
                    out.append(e)
            return out
        return v

    def __repr__(self):
        return f"ParamInfo({self.name!r})"


def search_enum(enum_cls, value: str, param_name: str = ""):
    """Case-insensitive enum lookup (reference ``A/params/ParamUtil.java:41-48``)."""
    if isinstance(value, enum_cls):
        return value
    for m in enum_cls:
        if m.name.upper() == str(value).strip().upper():
            return m
    raise ParamValidationError(
        f"{value} is not member of {param_name or enum_cls.__name__}. "
        f"It maybe {','.join(m.name for m in enum_cls)}.")


def _decode(json_str: Optional[str], info: Optional[ParamInfo]):
    if json_str is None:
        return None
    try:
        v = json.loads(json_str)
    except ValueError:
        v = json_str    # legacy models store some string params unquoted (e.g. "vectorCol":"vec")
    if info is None:
        return v
    t = info.value_type
    if isinstance(t, type) and issubclass(t, enum.Enum):
        return search_enum(t, v, info.name)
    if v is None:
        return None
    if t is int:
        return int(v)
    if t is float:
        return float(v)
    if t is bool:
        return bool(v)
    if isinstance(t, list) and t and isinstance(t[0], type) and issubclass(t[0], enum.Enum):
        return [search_enum(t[0], e, info.name) for e in v]
    if isinstance(t, list) and t and t[0] in (int, float, str):
        return [None if e is None else t[0](e) for e in v]
    return v


class Params:
    """A map ``name -> JSON string`` (Gson semantics).  ``toJson`` emits Java HashMap order."""

    def __init__(self, m: Optional[Dict[str, Optional[str]]] = None):
        self._m: Dict[str, Optional[str]] = dict(m) if m else {}

    # -- construction --
    @staticmethod
    def fromJson(s: str) -> "Params":
        p = Params()
        if s:
            obj = json.loads(s)
            for k, v in obj.items():
                p._m[k] = v if (v is None or isinstance(v, str)) else json.dumps(v)
        return p

    from_json = fromJson

    def toJson(self) -> str:
        return gson_dumps({k: v for k, v in self._m.items()}, java_map_order=True)

    to_json = toJson

    def clone(self) -> "Params":
        return Params(self._m)

    def merge(self, other: Optional["Params"]) -> "Params":
        if other is not None:
            self._m.update(other._m)
        return self

    # -- access --
    def set(self, key, value=None) -> "Params":
        if isinstance(key, ParamInfo):
            value = key.coerce(value)
            if key.validator is not None and value is not None and not key.validator(value):
                raise ParamValidationError(f"value {value!r} of param {key.name} fails validator "
                                           f"{key.validator!r}")
            name = key.name
        else:
            name = key
        self._m[name] = None if value is None else gson_dumps(value)
        return self

    def setIgnoreNull(self, key, value) -> "Params":
        return self if value is None else self.set(key, value)

    def get(self, key, value_type=None):
        if isinstance(key, ParamInfo):
            for n in key.names():
                if n in self._m:
                    return _decode(self._m[n], key)
            if key.optional and key.has_default:
                d = key.default
                return list(d) if isinstance(d, list) else d
            if key.optional:
                raise KeyError(f"Not have defaultValue for parameter: {key.name}")
            raise KeyError(f"Not have parameter: {key.name}")
        if key not in self._m:
            raise KeyError(f"Not have parameter : {key}")
        if value_type is None:
            return _decode(self._m[key], None)
        return _decode(self._m[key], ParamInfo(key, value_type))

    def getOrDefault(self, key, default=None):
        try:
            return self.get(key)
        except KeyError:
            return default

    def contains(self, key) -> bool:
        if isinstance(key, ParamInfo):
            return any(n in self._m for n in key.names())
        if isinstance(key, (list, tuple)):
            return all(k in self._m for k in key)
        return key in self._m

    def remove(self, key):
        name = key.name if isinstance(key, ParamInfo) else key
        self._m.pop(name, None)

    def listParamNames(self):
        return list(self._m.keys())

    def raw(self) -> Dict[str, Optional[str]]:
        return dict(self._m)

    def size(self):
        return len(self._m)

    def isEmpty(self):
        return not self._m

    def __len__(self):
        return len(self._m)

    def __contains__(self, k):
        return self.contains(k)

    def __eq__(self, other):
        return isinstance(other, Params) and other._m == self._m

    def __repr__(self):
        return "Params " + "{" + ", ".join(f"{k}={v}" for k, v in self._m.items()) + "}"


def _camel_suffix(name: str) -> str:
    return name[0].upper() + name[1:]


class ParamsMeta(type):
    """Generates ``setXxx/getXxx`` accessors for every ``ParamInfo`` in the class' ``PARAMS``."""

    def __new__(mcls, cname, bases, ns):
        cls = super().__new__(mcls, cname, bases, ns)
        infos: Dict[str, ParamInfo] = {}
        for b in reversed(cls.__mro__[1:]):
            infos.update(getattr(b, "_param_infos", {}) or {})
        own = ns.get("PARAMS")
        if own is None and not ns.get("_NO_AUTO_PARAMS", False):
            # classes named like a reference operator/stage inherit its param interfaces
            from ..params import op_params
            own = op_params(ns.get("_ALINK_NAME", cname))
        for p in own or ():
            infos[p.name] = p
        for p in ns.get("EXTRA_PARAMS", ()) or ():
            infos[p.name] = p
        cls._param_infos = infos
        for name, info in infos.items():
            suf = _camel_suffix(name)
            if "set" + suf not in ns:
                setattr(cls, "set" + suf, _make_setter(info))
            if "get" + suf not in ns:
                setattr(cls, "get" + suf, _make_getter(info))
        return cls


def _make_setter(info: ParamInfo):
    def setter(self, *values):
        if len(values) == 1:
            v = values[0]
        elif info.name == "cutsArray" and len(values) == 2:
            # BucketizerParams.setCutsArray(double[] flatCuts, int[] lengths): consecutive runs per column
            flat, lens = list(values[0]), [int(x) for x in values[1]]
            if sum(lens) != len(flat):
                raise ValueError("cutsArray lengths do not add up to the number of cuts")
            starts = [sum(lens[:i]) for i in range(len(lens))]
            v = [flat[a:a + n] for a, n in zip(starts, lens)]
        elif isinstance(info.value_type, list):
            v = list(values)
        else:
            raise TypeError(f"set{_camel_suffix(info.name)} takes one value")
        self.getParams().set(info, v)
        return self
    setter.__name__ = "set" + _camel_suffix(info.name)
    setter.__doc__ = info.description
    return setter


def _make_getter(info: ParamInfo):
    def getter(self):
        return self.getParams().get(info)
    getter.__name__ = "get" + _camel_suffix(info.name)
    getter.__doc__ = info.description
    return getter


class WithParams(metaclass=ParamsMeta):
    """Mixin holding a ``Params`` instance."""
    PARAMS: Sequence[ParamInfo] = ()

    def __init__(self, params: Optional[Params] = None, **kwargs):
        self._params = params.clone() if isinstance(params, Params) else Params()
        for k, v in kwargs.items():
            self.set(k, v)

    def getParams(self) -> Params:
        return self._params

    def set(self, key, value):
        if isinstance(key, str):
            info = self._param_infos.get(key)
            if info is None:
                for i in self._param_infos.values():
                    if key in i.alias:
                        info = i
                        break
            if info is not None:
                key = info
        self._params.set(key, value)
        return self

    def get(self, key):
        if isinstance(key, str) and key in self._param_infos:
            key = self._param_infos[key]
        return self._params.get(key)

    def resolvedParams(self) -> "Params":
        """Copy of the params with every declared default filled in (string-keyed ``get`` then works)."""
        out = self._params.clone()
        for name, info in self._param_infos.items():
            if not out.contains(name):
                try:
                    v = self._params.get(info)
                except KeyError:
                    continue
                if v is not None:
                    out.set(info, v)
        return out

    @classmethod
    def paramInfos(cls) -> List[ParamInfo]:
        return list(cls._param_infos.values())
