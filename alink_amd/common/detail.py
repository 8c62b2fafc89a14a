"""Prediction-detail column kept columnar.

Alink's ``predictionDetailCol`` holds, per row, the Gson JSON of a ``HashMap<String, String>`` label ->
``Double.toString(probability)`` (``LinearModelMapper.java`` / ``SoftmaxModelMapper.java``).  Formatting that string
for every row and parsing it back in a downstream evaluator is the dominant host cost of a scoring pipeline
(the FTRL predict -> evaluate stream of BASELINE config 5).  A ``DetailBlock`` keeps the (labels, probability
matrix) pair instead and materialises the strings only when something reads them (``to_list``, a sink, a row
view): byte-identical to the eager strings, since both come from ``models/linear/model._detail_json``.
Columnar consumers (``EvalBinaryClassStreamOp`` / batch evaluation) read ``probs`` directly.
"""
from __future__ import annotations

from typing import Any, List, Optional, Sequence

import numpy as np

__all__ = ["DetailBlock"]


class DetailBlock:
    """``n`` detail strings as ``labels`` (K label values, the mapper's order) and ``probs`` ([n, K] float64
    numpy, ``probs[i, k]`` = probability of ``labels[k]``).  ``nulls`` (optional bool [n]) marks NULL rows.
    ``quoted``: the map's values are strings (``HashMap<String, String>``, linear / softmax mappers) or, when False,
    JSON numbers (``HashMap<String, Double>``, the tree mappers) — both ``Double.toString`` of the probability."""

    __slots__ = ("labels", "_probs", "_probs_t", "nulls", "quoted", "trusted", "_list")

    def __init__(self, labels: Sequence[Any], probs, nulls: Optional[np.ndarray] = None,
                 quoted: bool = True, trusted: bool = False):
        """``probs``: numpy [n, K], or a (device) torch tensor — then the block stays on the device until something
        reads ``probs`` / the strings (a scoring -> evaluation stream never copies it to the host).  ``trusted``:
        the producer guarantees probabilities in [0, 1] summing to 1 per row (a sigmoid pair), so columnar
        consumers skip the validity scan."""
        self.labels = list(labels)
        if hasattr(probs, "detach"):
            self._probs_t = probs.detach().to(__import__("torch").float64).reshape(-1, len(self.labels))
            self._probs = None
        else:
            self._probs_t = None
            self._probs = np.asarray(probs, dtype=np.float64).reshape(-1, len(self.labels))
        self.nulls = None if nulls is None or not np.any(nulls) else np.asarray(nulls, dtype=bool)
        self.quoted = bool(quoted)
        self.trusted = bool(trusted)
        self._list: Optional[List[Optional[str]]] = None

    @property
    def probs(self) -> np.ndarray:
        if self._probs is None:
            self._probs = self._probs_t.cpu().numpy()
        return self._probs

    def probs_tensor(self):
        """The probabilities as a torch tensor (on the producer's device when it was one), no host copy."""
        import torch
        return self._probs_t if self._probs_t is not None else torch.from_numpy(self._probs)

    def __len__(self) -> int:
        return int((self._probs_t if self._probs_t is not None else self._probs).shape[0])

    def to_list(self) -> List[Optional[str]]:
        if self._list is None:
            from ..models.linear.model import _detail_json
            out = _detail_json(self.labels, self.probs, self.quoted) if len(self) else []
            if self.nulls is not None:
                out = [None if m else s for s, m in zip(out, self.nulls.tolist())]
            self._list = out
        return self._list

    def __iter__(self):
        return iter(self.to_list())

    def __getitem__(self, i):
        if isinstance(i, slice):
            return self.take(i).to_list()
        return self.to_list()[i]

    def take(self, idx) -> "DetailBlock":
        if isinstance(idx, slice):
            sel = idx
        else:
            if hasattr(idx, "detach"):
                idx = idx.detach().cpu().numpy()
            sel = np.asarray(idx)
            if sel.dtype != bool:
                sel = sel.astype(np.int64)
        if self._probs_t is not None and self.nulls is None:
            import torch
            t = self._probs_t[sel] if isinstance(sel, slice) else \
                self._probs_t[torch.as_tensor(sel, device=self._probs_t.device)]
            return DetailBlock(self.labels, t, None, self.quoted, self.trusted)
        return DetailBlock(self.labels, self.probs[sel], None if self.nulls is None else self.nulls[sel], self.quoted,
                           self.trusted)

    @staticmethod
    def concat(blocks: Sequence["DetailBlock"]) -> Optional["DetailBlock"]:
        """One block, or None when the blocks' label sets differ (the caller falls back to strings)."""
        if not blocks or any(b.labels != blocks[0].labels or b.quoted != blocks[0].quoted for b in blocks):
            return None
        nulls = None
        if any(b.nulls is not None for b in blocks):
            nulls = np.concatenate([b.nulls if b.nulls is not None else np.zeros(len(b), bool) for b in blocks])
        return DetailBlock(blocks[0].labels, np.concatenate([b.probs for b in blocks]), nulls, blocks[0].quoted,
                           all(b.trusted for b in blocks))

    def __repr__(self):
        return f"DetailBlock(n={len(self)}, labels={self.labels})"
