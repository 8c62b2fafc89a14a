"""Lazy evaluation: ``LazyEvaluation`` (a replay subject with callbacks) and ``LazyObjectsManager``.

Reference: ``A/common/lazy/LazyEvaluation.java:17-73`` (RxJava ``ReplaySubject``) and
``A/common/lazy/LazyObjectsManager.java:22-73``.  Operators here execute eagerly on ``linkFrom``, but
every *observable* lazy behaviour is kept: ``lazyPrint/lazyCollect`` callbacks fire only at the next
``print/collect/execute`` trigger of the environment, in registration order, and lazily-produced
train ops / models / transform results replay to late subscribers.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List

__all__ = ["LazyEvaluation", "LazyObjectsManager"]


class LazyEvaluation:
    def __init__(self):
        self._values: List[Any] = []
        self._callbacks: List[Callable[[Any], None]] = []

    def addValue(self, v):
        self._values.append(v)
        for cb in list(self._callbacks):
            cb(v)

    def addCallback(self, cb: Callable[[Any], None]):
        self._callbacks.append(cb)
        for v in self._values:
            cb(v)

    def getLatestValue(self):
        if not self._values:
            raise RuntimeError("No value available in LazyEvaluation")
        return self._values[-1]

    def hasValue(self):
        return bool(self._values)


class LazyObjectsManager:
    def __init__(self):
        self.lazy_sinks: Dict[int, tuple] = {}  # id(op) -> (op, LazyEvaluation); insertion ordered
        self.lazy_train_ops: Dict[int, LazyEvaluation] = {}
        self.lazy_models: Dict[int, LazyEvaluation] = {}
        self.lazy_transform_results: Dict[int, LazyEvaluation] = {}

    @staticmethod
    def _gen(obj, m: Dict[int, Any], with_obj=False):
        k = id(obj)
        if k not in m:
            m[k] = (obj, LazyEvaluation()) if with_obj else LazyEvaluation()
        return m[k][1] if with_obj else m[k]

    def genLazySink(self, op) -> LazyEvaluation:
        return self._gen(op, self.lazy_sinks, with_obj=True)

    def genLazyTrainOp(self, trainer) -> LazyEvaluation:
        return self._gen(trainer, self.lazy_train_ops)

    def genLazyModel(self, trainer) -> LazyEvaluation:
        return self._gen(trainer, self.lazy_models)

    def genLazyTransformResult(self, transformer) -> LazyEvaluation:
        return self._gen(transformer, self.lazy_transform_results)

    def getLazySinks(self):
        return list(self.lazy_sinks.values())

    def clearVirtualSinks(self):
        self.lazy_sinks.clear()
