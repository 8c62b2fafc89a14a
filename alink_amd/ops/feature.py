"""Feature hot path (kernels K24-K26) — ``csrc/feature.hip``.

* ``murmur3_index(strings, nf, prefix, device)``: ``floorMod(abs(murmur3_32(0).hashUnencodedChars(prefix + s)),
  nf)`` (Guava-exact, reference ``FeatureHasherMapper.java:104-106``) for a list of strings or a packed UTF-8
  ``StringBlock``; on a GPU one lane per string decodes UTF-8 to UTF-16 code units and hashes them on the
  device, on the host the C++ twin does.
* ``csr_mv(crow, col, val, v)``: CSR matrix-vector product (margins of linear / FTRL models), G lanes per row
  with a fixed-order shuffle reduction — deterministic, no atomics.
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

__all__ = ["utf16_units", "murmur3_index", "csr_assemble", "vector_assemble", "csr_mv"]

CSR_MV_CALLS = 0     # HIP SpMV launches (tests check the device path ran)


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


def murmur3_index(strings, nf: int, prefix: str = "", device=None) -> torch.Tensor:
    """int64 feature indices of ``prefix + s`` for every string (see module doc).  ``strings``: a list of str or
    a packed ``StringBlock``; on a GPU the UTF-8 bytes go to the device once and the kernel decodes the UTF-16
    code units Guava hashes (``ops/strings.py``)."""
    from ..common.strings import StringBlock
    from .strings import murmur3_utf8_index
    device = torch.device(device) if device is not None else torch.device("cpu")
    if isinstance(strings, StringBlock):
        block = strings
    else:
        if device.type != "cuda":
            from ..models.feature.encoders import murmur3_index as host_index
            return torch.from_numpy(np.asarray(host_index([prefix + s for s in strings], nf), dtype=np.int64))
        block = StringBlock.from_list(strings)
    if device.type == "cuda":
        _lib.require()
    return murmur3_utf8_index(block.to(device), nf, prefix)


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


_DENSE_KIND = {torch.float64: 0, torch.float32: 1, torch.bfloat16: 2}
# 2: element-parallel VectorAssembler workgroups (coalesced stores), 1: thread per (part, row)
VA_VARIANT = int(__import__("os").environ.get("ALINK_VA_VARIANT", "2"))


def vector_assemble(parts, n: int, skip: Optional[torch.Tensor] = None, dense_ratio: Optional[float] = None,
                    use_kernel: bool = True):
    """K24 VectorAssembler over column blocks: ``parts`` are [n] / [n, d] tensors (numeric or dense-vector
    columns) and ``SparseBlock`` s; row r of the result is their concatenation with every part's entries shifted
    by the running position (``VectorAssemblerMapper.java:50-106``).  ``skip`` [n] bool: rows that become NULL
    (handleInvalid SKIP).  On a GPU one HIP wave per row writes the CSR directly (``csrc/feature.hip``); on the
    host the same layout is built with vectorised torch (``use_kernel=False`` forces that path anywhere, for
    comparison).  Returns (SparseBlock, size)."""
    dev = None
    for p in parts:
        d_ = p.crow.device if isinstance(p, SparseBlock) else p.device
        if d_.type == "cuda":
            dev = d_
            break
    if dev is None:
        dev = parts[0].crow.device if isinstance(parts[0], SparseBlock) else parts[0].device
    norm, lens, size = [], [], 0
    for p in parts:
        if isinstance(p, SparseBlock):
            p = p.to(dev)
            ln = p.crow[1:] - p.crow[:-1]
            norm.append(("csr", p))
            w = int(p.size)
        else:
            t = p.to(dev)
            t = t.reshape(n, -1)
            if t.dtype not in _DENSE_KIND:
                t = t.to(torch.float64)
            t = t.contiguous()
            w = int(t.shape[1])
            ln = torch.full((n,), w, dtype=torch.int64, device=dev)
            norm.append(("dense", t))
        if skip is not None:
            ln = torch.where(skip.to(dev), torch.zeros_like(ln), ln)
        lens.append(ln)
        size += w
    crow = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    if lens:
        torch.cumsum(torch.stack(lens).sum(0), 0, out=crow[1:])
    nnz = int(crow[-1]) if n else 0
    col = torch.empty(nnz, dtype=torch.int32, device=dev)
    val = torch.empty(nnz, dtype=torch.float64, device=dev)
    if dev.type == "cuda" and n and nnz and use_kernel:
        L = _lib.require()
        sk = None if skip is None else skip.to(dev).to(torch.uint8).contiguous()
        desc = torch.zeros((len(norm), 8), dtype=torch.int64)
        pos = 0
        for i, (kind, p) in enumerate(norm):
            desc[i, 6] = pos
            pos += int(p.size) if kind == "csr" else int(p.shape[1])
            if kind == "csr":
                desc[i, 0] = 3
                desc[i, 1] = int(p.size)
                desc[i, 2] = p.val.to(torch.float64).contiguous().data_ptr() if p.val.dtype == torch.float64 \
                    and p.val.is_contiguous() else _keep(p.val.to(torch.float64).contiguous()).data_ptr()
                desc[i, 3] = p.crow.data_ptr()
                cc = p.col if p.col.dtype == torch.int32 and p.col.is_contiguous() else \
                    _keep(p.col.to(torch.int32).contiguous())
                desc[i, 4] = cc.data_ptr()
            else:
                desc[i, 0] = _DENSE_KIND[p.dtype]
                desc[i, 1] = int(p.shape[1])
                desc[i, 2] = p.data_ptr()
            desc[i, 5] = 0 if sk is None else sk.data_ptr()
        ddesc = desc.to(dev)
        tot = crow[1:] - crow[:-1]
        variant = 2 if len(norm) <= 16 and int(tot.max()) < (1 << 22) else 1
        rc = L.alink_vector_assemble(n, len(norm), ddesc.data_ptr(), crow.data_ptr(), col.data_ptr(), val.data_ptr(),
                                     VA_VARIANT if VA_VARIANT in (1, 2) and variant == 2 else variant,
                                     _lib.stream_ptr(dev))
        if rc != 0:
            raise RuntimeError(f"alink_vector_assemble failed: {rc}")
        torch.cuda.current_stream(dev).synchronize()      # the descriptor's raw pointers must outlive the kernel
        _KEEP.clear()
    elif nnz:
        before = torch.zeros(n, dtype=torch.int64, device=dev)
        pos = 0
        for (kind, p), ln in zip(norm, lens):
            m = int(ln.sum())
            if m:
                rid = torch.repeat_interleave(torch.arange(n, device=dev), ln)
                k = torch.arange(m, device=dev) - (torch.cumsum(ln, 0) - ln)[rid]
                dst = crow[:-1][rid] + before[rid] + k
                if kind == "csr":
                    src = p.crow[:-1][rid] + k
                    col[dst] = (p.col[src].to(torch.int64) + pos).to(torch.int32)
                    val[dst] = p.val[src].to(torch.float64)
                else:
                    col[dst] = (k + pos).to(torch.int32)
                    val[dst] = p[rid, k].to(torch.float64)
            before += ln
            pos += int(p.size) if kind == "csr" else int(p.shape[1])
    return SparseBlock(crow, col, val, size, dense_ratio), size


_KEEP = []


def _keep(t):
    _KEEP.append(t)
    return t


def csr_mv(crow: torch.Tensor, col: torch.Tensor, val: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """``out[r] = sum_k val[k] * v[col[k]]`` for the CSR rows (fp64) on the GPU (``alink_csr_mv_f64``)."""
    global CSR_MV_CALLS
    L = _lib.require()
    dev = val.device
    n = int(crow.numel()) - 1
    out = torch.empty(n, dtype=torch.float64, device=dev)
    if n <= 0:
        return out
    crow = crow.to(torch.int64).contiguous()
    col = col.contiguous() if col.dtype in (torch.int32, torch.int64) else col.to(torch.int64).contiguous()
    val = val.to(torch.float64).contiguous()
    v = v.to(torch.float64).contiguous()
    mean_nnz = float(col.numel()) / n
    rc = L.alink_csr_mv_f64(crow.data_ptr(), col.data_ptr(), int(col.dtype == torch.int64), val.data_ptr(), n,
                            v.data_ptr(), out.data_ptr(), mean_nnz, _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_csr_mv_f64 failed: {rc}")
    CSR_MV_CALLS += 1
    return out
