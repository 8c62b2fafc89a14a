"""Stream data processing: sampling and splitting (reference ``A/operator/stream/dataproc/{SampleStreamOp,
SplitStreamOp}.java``)."""
from __future__ import annotations

from typing import Optional

import numpy as np

from ...common.params import ParamInfo, Params
from ...parallel import comm
from .base import StreamOperator

__all__ = ["SampleStreamOp", "SplitStreamOp"]


class SampleStreamOp(StreamOperator):
    EXTRA_PARAMS = [ParamInfo("randomSeed", int, "seed", default=0)]

    def linkFrom(self, *inputs):
        (inp,) = self._connect(*inputs)
        self._schema = inp.getSchema()
        self._rng = np.random.default_rng(np.random.SeedSequence([self.getParams().get(
            self._param_infos["randomSeed"]), comm.get_rank()]))
        return self

    def on_batch(self, port, mt):
        self._emit(mt.take(np.nonzero(self._rng.random(mt.num_rows) < self.getRatio())[0]))


class _Side(StreamOperator):
    def linkFrom(self, *inputs):
        return self


class SplitStreamOp(StreamOperator):
    """Rows go to the main output with probability ``fraction``, else to side output 0."""
    EXTRA_PARAMS = [ParamInfo("randomSeed", int, "seed", default=0)]

    def __init__(self, params: Optional[Params] = None, **kw):
        if isinstance(params, float):
            f, params = params, None
            super().__init__(params, **kw)
            self.setFraction(f)
        else:
            super().__init__(params, **kw)

    def linkFrom(self, *inputs):
        (inp,) = self._connect(*inputs)
        self._schema = inp.getSchema()
        side = _Side()
        side._schema = self._schema
        self._side = [side]
        self._rng = np.random.default_rng(np.random.SeedSequence([self.getParams().get(
            self._param_infos["randomSeed"]), comm.get_rank()]))
        return self

    def on_batch(self, port, mt):
        m = self._rng.random(mt.num_rows) < self.getFraction()
        self._emit(mt.take(np.nonzero(m)[0]))
        self._side[0]._emit(mt.take(np.nonzero(~m)[0]))
