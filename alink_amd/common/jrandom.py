"""``java.util.Random`` (48-bit LCG) — reproduces the reference's seeded draws where they shape results
(e.g. the per-node feature shuffles of ``seriestree/DecisionTree.bagging``)."""
from __future__ import annotations

__all__ = ["JavaRandom"]

_MULT = 0x5DEECE66D
_ADD = 0xB
_MASK = (1 << 48) - 1


def _to_int32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


class JavaRandom:
    def __init__(self, seed: int):
        self._seed = (int(seed) ^ _MULT) & _MASK
        self._next_gaussian = None

    def _next(self, bits: int) -> int:
        self._seed = (self._seed * _MULT + _ADD) & _MASK
        return _to_int32(self._seed >> (48 - bits))

    def nextInt(self, bound: int = None) -> int:
        if bound is None:
            return self._next(32)
        if bound <= 0:
            raise ValueError("bound must be positive")
        if (bound & -bound) == bound:
            return _to_int32((bound * self._next(31)) >> 31)
        while True:
            bits = self._next(31)
            val = bits % bound
            if _to_int32(bits - val + (bound - 1)) >= 0:
                return val

    def nextLong(self) -> int:
        v = (self._next(32) << 32) + self._next(32)
        v &= (1 << 64) - 1
        return v - (1 << 64) if v >= (1 << 63) else v

    def nextDouble(self) -> float:
        return ((self._next(26) << 27) + self._next(27)) * (1.0 / (1 << 53))

    def nextFloat(self) -> float:
        return self._next(24) / float(1 << 24)

    def nextGaussian(self) -> float:
        """Marsaglia polar method with the cached second value, as ``Random.nextGaussian``."""
        import math
        if self._next_gaussian is not None:
            v, self._next_gaussian = self._next_gaussian, None
            return v
        while True:
            v1 = 2 * self.nextDouble() - 1
            v2 = 2 * self.nextDouble() - 1
            s = v1 * v1 + v2 * v2
            if 0 < s < 1:
                break
        mul = math.sqrt(-2 * math.log(s) / s)
        self._next_gaussian = v2 * mul
        return v1 * mul

    def nextBoolean(self) -> bool:
        return self._next(1) != 0

    def shuffle_rows(self, rows) -> "np.ndarray":
        """``shuffle`` applied to every row of an int array [m, n] in row order, in place — one host C++ call
        (``_native/csrc/jrandom.cpp``) for a whole tree level; the Python loop without the library."""
        import ctypes
        import numpy as np
        from .. import _native
        a = np.ascontiguousarray(rows, dtype=np.int32)
        L = _native.lib
        if L is not None and hasattr(L, "alink_java_shuffle_rows") and a.ndim == 2 and a.size:
            st = ctypes.c_uint64(self._seed)
            L.alink_java_shuffle_rows(ctypes.byref(st), a.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(a.shape[0]),
                                      ctypes.c_int32(a.shape[1]))
            self._seed = int(st.value)
            return a
        for r in range(a.shape[0]):
            a[r] = self.shuffle(a[r].tolist())
        return a

    def shuffle(self, arr: list) -> list:
        """In-place shuffle as ``DecisionTree.shuffle`` (Fisher-Yates from the end, ``nextInt(i + 1)``)."""
        for i in range(len(arr) - 1, 0, -1):
            idx = self.nextInt(i + 1)
            if idx == i:
                continue
            arr[idx], arr[i] = arr[i], arr[idx]
        return arr
