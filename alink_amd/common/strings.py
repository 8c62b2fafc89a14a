"""Packed string column: UTF-8 bytes + int64 offsets (+ null mask) in tensors, on the host or the device.

Strings in a ``Column`` are Python lists by default; a ``StringBlock`` is the columnar form the data plane
uses where strings move or get hashed in bulk:

* the hash / range shuffle (``parallel/shuffle.py``) exchanges a string column as ONE bytes all-to-all plus
  one lengths all-to-all (RCCL on device tensors, gloo on host tensors) — never pickles per string;
* key hashing runs over the bytes (``ops/strings.py``: murmur3 on the device, the same bits in C++ on the host);
* the Guava murmur3 feature hasher / one-hot path reads the UTF-8 bytes directly (UTF-16 code units are
  decoded inside the HIP kernel), so a device-resident block needs no host packing.

Reference: the reference keeps strings as Java ``String`` inside Flink ``Row`` objects
(``A/common/utils/RowUtil``); its shuffles serialise them per record.  Sequence access (``len``, indexing,
iteration) decodes lazily, so code written against the list form keeps working.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence

import numpy as np
import torch

__all__ = ["StringBlock"]


class StringBlock:
    """``n`` strings: bytes of string i are ``data[offsets[i]:offsets[i+1]]`` (UTF-8); ``nulls[i]`` marks SQL
    NULL (its byte range is empty).  ``data`` / ``offsets`` / ``nulls`` live on one device."""

    __slots__ = ("data", "offsets", "nulls", "_list")

    def __init__(self, data: torch.Tensor, offsets: torch.Tensor, nulls: Optional[torch.Tensor] = None):
        if data.dtype != torch.uint8 or data.dim() != 1:
            raise ValueError("StringBlock data must be a 1-D uint8 tensor")
        if offsets.dtype != torch.int64 or offsets.dim() != 1 or offsets.numel() < 1:
            raise ValueError("StringBlock offsets must be a non-empty 1-D int64 tensor")
        self.data = data
        self.offsets = offsets
        self.nulls = nulls if nulls is None or bool(nulls.any()) else None
        self._list = None

    # -- construction --
    @staticmethod
    def from_list(vals: Iterable[Optional[str]], device=None) -> "StringBlock":
        vals = list(vals)
        enc = [b"" if v is None else (v if isinstance(v, str) else str(v)).encode("utf-8") for v in vals]
        lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=len(enc))
        off = np.zeros(len(enc) + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        data = np.frombuffer(b"".join(enc), dtype=np.uint8) if off[-1] else np.zeros(0, np.uint8)
        nulls = None
        if any(v is None for v in vals):
            nulls = torch.tensor([v is None for v in vals], dtype=torch.bool)
        blk = StringBlock(torch.from_numpy(data.copy()), torch.from_numpy(off), nulls)
        return blk.to(device) if device is not None else blk

    @staticmethod
    def empty(device=None) -> "StringBlock":
        dev = device or "cpu"
        return StringBlock(torch.zeros(0, dtype=torch.uint8, device=dev), torch.zeros(1, dtype=torch.int64,
                                                                                       device=dev))

    # -- properties --
    @property
    def device(self) -> torch.device:
        return self.data.device

    @property
    def nbytes(self) -> int:
        return int(self.data.numel())

    def lengths(self) -> torch.Tensor:
        return self.offsets[1:] - self.offsets[:-1]

    def null_mask(self) -> torch.Tensor:
        if self.nulls is not None:
            return self.nulls
        return torch.zeros(len(self), dtype=torch.bool, device=self.device)

    def to(self, device) -> "StringBlock":
        device = torch.device(device)
        if device == self.device:
            return self
        return StringBlock(self.data.to(device), self.offsets.to(device),
                           None if self.nulls is None else self.nulls.to(device))

    # -- sequence protocol (lazy decode) --
    def __len__(self) -> int:
        return int(self.offsets.numel()) - 1

    def to_list(self) -> List[Optional[str]]:
        if self._list is None:
            raw = self.data.cpu().numpy().tobytes()
            off = self.offsets.cpu().tolist()
            nul = self.nulls.cpu().tolist() if self.nulls is not None else None
            out = [raw[off[i]:off[i + 1]].decode("utf-8") for i in range(len(off) - 1)]
            if nul is not None:
                out = [None if m else s for s, m in zip(out, nul)]
            self._list = out
        return list(self._list)

    def __iter__(self):
        return iter(self.to_list())

    def __getitem__(self, i):
        if isinstance(i, slice):
            return self.take(i)
        if self._list is not None:
            return self._list[i]
        n = len(self)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError(i)
        if self.nulls is not None and bool(self.nulls[i]):
            return None
        a, b = int(self.offsets[i]), int(self.offsets[i + 1])
        return self.data[a:b].cpu().numpy().tobytes().decode("utf-8")

    def __eq__(self, other):
        if isinstance(other, (StringBlock, list, tuple)):
            return list(self) == list(other)
        return NotImplemented

    def __repr__(self):
        return f"StringBlock(n={len(self)}, bytes={self.nbytes}, device={self.device})"

    # -- bulk ops (vectorised, on the block's device) --
    def take(self, idx) -> "StringBlock":
        """Rows by index (tensor / sequence / numpy / boolean mask / slice), as one byte gather."""
        dev = self.device
        n = len(self)
        if isinstance(idx, slice) and idx.step in (None, 1):
            # contiguous rows (MTable.slice): one byte-range view, offsets rebased
            a, b, _ = idx.indices(n)
            b = max(a, b)
            ba, bb = self.offsets[[a, b]].tolist()
            return self.row_range(a, b, ba, bb)
        if isinstance(idx, slice):
            idx = torch.arange(n, device=dev)[idx]
        elif isinstance(idx, torch.Tensor):
            idx = idx.to(dev)
            if idx.dtype == torch.bool:
                idx = torch.nonzero(idx, as_tuple=False).reshape(-1)
        else:
            arr = np.asarray(idx)
            if arr.dtype == bool:
                arr = np.nonzero(arr)[0]
            idx = torch.as_tensor(arr.astype(np.int64), device=dev)
        idx = idx.to(torch.int64)
        if idx.numel() and (int(idx.min()) < -n or int(idx.max()) >= n):
            raise IndexError("StringBlock.take index out of range")
        idx = torch.where(idx < 0, idx + n, idx)
        starts = self.offsets[idx]
        lens = self.offsets[idx + 1] - starts
        off = torch.zeros(idx.numel() + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=off[1:])
        total = int(off[-1]) if idx.numel() else 0
        if total:
            seg = torch.repeat_interleave(torch.arange(idx.numel(), device=dev), lens)
            src = starts[seg] + torch.arange(total, device=dev) - off[:-1][seg]
            data = self.data[src]
        else:
            data = torch.zeros(0, dtype=torch.uint8, device=dev)
        nulls = None if self.nulls is None else self.nulls[idx]
        return StringBlock(data, off, nulls)

    def row_range(self, a: int, b: int, byte_a: int, byte_b: int) -> "StringBlock":
        """Rows [a, b) given their byte range [byte_a, byte_b) = offsets[a], offsets[b] (known to the caller, e.g.
        the micro-batch boundaries of a stream source read in one copy): a view, no device synchronisation."""
        return StringBlock(self.data[byte_a:byte_b], self.offsets[a:b + 1] - byte_a,
                           None if self.nulls is None else self.nulls[a:b])

    @staticmethod
    def concat(blocks: Sequence["StringBlock"]) -> "StringBlock":
        blocks = [b for b in blocks]
        if not blocks:
            return StringBlock.empty()
        dev = blocks[0].device
        blocks = [b.to(dev) for b in blocks]
        data = torch.cat([b.data for b in blocks])
        offs, base = [torch.zeros(1, dtype=torch.int64, device=dev)], 0
        for b in blocks:
            offs.append(b.offsets[1:] + base)
            base += b.nbytes
        nulls = None
        if any(b.nulls is not None for b in blocks):
            nulls = torch.cat([b.null_mask() for b in blocks])
        return StringBlock(data, torch.cat(offs), nulls)

    @staticmethod
    def from_parts(lengths: torch.Tensor, data: torch.Tensor, nulls: Optional[torch.Tensor] = None) -> "StringBlock":
        """From per-string byte lengths (int64) and the concatenated bytes (what a shuffle receives)."""
        off = torch.zeros(lengths.numel() + 1, dtype=torch.int64, device=data.device)
        torch.cumsum(lengths.to(data.device, torch.int64), 0, out=off[1:])
        return StringBlock(data, off, nulls)
