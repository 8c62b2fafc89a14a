"""Feature hot path (kernels K24-K26) — ``csrc/feature.hip``.

* ``murmur3_index(strings, nf, prefix, device)``: ``floorMod(abs(murmur3_32(0).hashUnencodedChars(prefix + s)),
  nf)`` (Guava-exact, reference ``FeatureHasherMapper.java:104-106``) for a batch of strings; on a GPU the hash
  runs on the device over the strings' UTF-16 code units (one lane per string), on the host in C++.
* ``csr_assemble(idx, val, valid, size)``: per-row CSR from ``m`` column-major entry arrays ``[m, n]`` — rows
  sorted by index, duplicate indices summed (the reference's ``TreeMap`` accumulation) — one wave per row on
  the GPU, vectorised torch on the host.  Returns a ``SparseBlock``.

Both fail loudly on a GPU box whose HIP library is missing (``_lib.require``).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from ..common.linalg.block import SparseBlock
from . import _lib

__all__ = ["utf16_units", "murmur3_index", "csr_assemble"]


def utf16_units(strings: Sequence[str]):
    """(code units uint16 [total], offsets int64 [n+1]) of the strings' UTF-16 encoding."""
    joined = "".join(strings)
    if joined.isascii():
        units = np.frombuffer(joined.encode("ascii"), dtype=np.uint8).astype(np.uint16)
        lens = np.fromiter((len(s) for s in strings), dtype=np.int64, count=len(strings))
    else:
        enc = [s.encode("utf-16-le") for s in strings]
        units = np.frombuffer(b"".join(enc), dtype=np.uint16).copy()
        lens = np.fromiter((len(b) // 2 for b in enc), dtype=np.int64, count=len(enc))
    off = np.zeros(len(strings) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    return units, off


def murmur3_index(strings: Sequence[str], nf: int, prefix: str = "", device=None) -> torch.Tensor:
    """int64 feature indices of ``prefix + s`` for every string (see module doc)."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    n = len(strings)
    if device.type != "cuda":
        from ..models.feature.encoders import murmur3_index as host_index
        return torch.from_numpy(np.asarray(host_index([prefix + s for s in strings], nf), dtype=np.int64))
    L = _lib.require()
    out = torch.empty(n, dtype=torch.int32, device=device)
    if n == 0:
        return out.to(torch.int64)
    units, off = utf16_units(strings)
    u = torch.from_numpy(units if units.size else np.zeros(1, np.uint16)).to(device)
    o = torch.from_numpy(off).to(device)
    pu, _ = utf16_units([prefix])
    p = torch.from_numpy(pu if pu.size else np.zeros(1, np.uint16)).to(device)
    rc = L.alink_murmur3_index(u.data_ptr(), o.data_ptr(), n, p.data_ptr(), int(pu.size), 0, int(nf), None,
                               out.data_ptr(), _lib.stream_ptr(device))
    if rc != 0:
        raise RuntimeError(f"alink_murmur3_index failed: {rc}")
    return out.to(torch.int64)


def csr_assemble(idx: torch.Tensor, val: Optional[torch.Tensor], valid: Optional[torch.Tensor], size: int,
                 dense_ratio: Optional[float] = None) -> SparseBlock:
    """Rows ``r`` of ``{(idx[j, r], val[j, r]) : valid[j, r]}`` as sorted, duplicate-summed CSR."""
    m, n = idx.shape
    dev = idx.device
    if dev.type == "cuda" and 1 <= m <= 64:
        L = _lib.require()
        ii = idx.to(torch.int32).contiguous()
        vv = None if val is None else val.to(torch.float64).contiguous()
        ok = None if valid is None else valid.to(torch.uint8).contiguous()
        cnt = torch.empty(n, dtype=torch.int64, device=dev)
        st = _lib.stream_ptr(dev)
        rc = L.alink_csr_assemble(n, m, ii.data_ptr(), None, None if ok is None else ok.data_ptr(), cnt.data_ptr(),
                                  None, None, None, st)
        if rc != 0:
            raise RuntimeError(f"alink_csr_assemble (count) failed: {rc}")
        crow = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(cnt, 0, out=crow[1:])
        nnz = int(crow[-1]) if n else 0
        col = torch.empty(nnz, dtype=torch.int32, device=dev)
        out = torch.empty(nnz, dtype=torch.float64, device=dev)
        if nnz:
            rc = L.alink_csr_assemble(n, m, ii.data_ptr(), None if vv is None else vv.data_ptr(),
                                      None if ok is None else ok.data_ptr(), cnt.data_ptr(), crow.data_ptr(),
                                      col.data_ptr(), out.data_ptr(), st)
            if rc != 0:
                raise RuntimeError(f"alink_csr_assemble (write) failed: {rc}")
        return SparseBlock(crow, col, out, size, dense_ratio)
    # host / fallback: sort (row, index) keys, merge duplicates with index_add
    rows = torch.arange(n, device=dev, dtype=torch.int64).repeat(m)
    ii = idx.reshape(-1).to(torch.int64)
    vv = torch.ones(m * n, dtype=torch.float64, device=dev) if val is None else val.reshape(-1).to(torch.float64)
    if valid is not None:
        keep = valid.reshape(-1).to(torch.bool)
        rows, ii, vv = rows[keep], ii[keep], vv[keep]
    key = rows * (int(size) + 1) + ii
    key, order = torch.sort(key, stable=True)
    uk, inv = torch.unique_consecutive(key, return_inverse=True)
    sums = torch.zeros(uk.shape[0], dtype=torch.float64, device=dev).index_add_(0, inv, vv[order])
    urow = uk // (int(size) + 1)
    crow = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(torch.bincount(urow, minlength=n), 0, out=crow[1:])
    return SparseBlock(crow, (uk % (int(size) + 1)).to(torch.int32), sums, size, dense_ratio)
