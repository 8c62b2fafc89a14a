"""Bulk hashing of packed string columns (``common/strings.StringBlock``) — ``csrc/feature.hip`` on the device,
the same functions in the C++ runtime on the host (bit-identical, so every rank of a job partitions alike
whichever side hashed).

* ``hash_bytes(block)``: MurmurHash3_x86_32(0) of every string's UTF-8 bytes (Guava ``hashBytes``) — the key
  hash of the relational shuffle (``parallel/shuffle.py``).
* ``murmur3_utf8_index(block, nf, prefix)``: Guava ``hashUnencodedChars(prefix + s)`` (UTF-16 code units,
  decoded from the UTF-8 bytes inside the kernel) -> ``floorMod(abs(h), nf)``: the FeatureHasher / one-hot
  path of ``FeatureHasherMapper.java:104-106`` without any host string handling.
* ``split_tokens(block)``: Java ``String.split(" ")`` of every document into one token block (NLP counting).
* ``unique_ids(block)``: exact dictionary encoding (two-hash 64-bit key + byte comparison with a representative).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np
import torch

from ..common.strings import StringBlock
from . import _lib

__all__ = ["tokenize_ws_lower", "has_strip_space", "join_tokens", "ngram_join", "hash_bytes", "murmur3_utf8_index", "murmur3_bytes_py", "split_tokens", "unique_ids"]


def murmur3_bytes_py(b: bytes, seed: int = 0) -> int:
    """Pure-Python MurmurHash3_x86_32 (test reference / last-resort fallback), signed int32."""
    c1, c2, m = 0xcc9e2d51, 0x1b873593, 0xFFFFFFFF
    h = seed & m
    n = len(b) // 4
    for i in range(n):
        k = int.from_bytes(b[4 * i:4 * i + 4], "little")
        k = (k * c1) & m
        k = ((k << 15) | (k >> 17)) & m
        k = (k * c2) & m
        h ^= k
        h = ((h << 13) | (h >> 19)) & m
        h = (h * 5 + 0xe6546b64) & m
    t = b[4 * n:]
    k = 0
    if len(t) >= 3:
        k ^= t[2] << 16
    if len(t) >= 2:
        k ^= t[1] << 8
    if len(t) >= 1:
        k ^= t[0]
        k = (k * c1) & m
        k = ((k << 15) | (k >> 17)) & m
        k = (k * c2) & m
        h ^= k
    h ^= len(b)
    h ^= h >> 16
    h = (h * 0x85ebca6b) & m
    h ^= h >> 13
    h = (h * 0xc2b2ae35) & m
    h ^= h >> 16
    return h - (1 << 32) if h & 0x80000000 else h


def hash_bytes(block: StringBlock, seed: int = 0) -> torch.Tensor:
    """int32 [n] murmur3 of each string's bytes, on the block's device (nulls hash their empty range)."""
    n = len(block)
    dev = block.device
    if n == 0:
        return torch.zeros(0, dtype=torch.int32, device=dev)
    if dev.type == "cuda":
        L = _lib.require()
        data = block.data if block.nbytes else torch.zeros(1, dtype=torch.uint8, device=dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        rc = L.alink_murmur3_bytes(data.data_ptr(), block.offsets.contiguous().data_ptr(), n, seed & 0xFFFFFFFF,
                                   out.data_ptr(), _lib.stream_ptr(dev))
        if rc != 0:
            raise RuntimeError(f"alink_murmur3_bytes failed: {rc}")
        return out
    from .. import _native
    data, off = block.data.numpy(), block.offsets.numpy()
    h = _native.murmur3_bytes(data, off, seed)
    if h is None:
        raw = data.tobytes()
        h = np.asarray([murmur3_bytes_py(raw[off[i]:off[i + 1]], seed) for i in range(n)], dtype=np.int32)
    return torch.from_numpy(h)


_PREFIX_CACHE: dict = {}


def _device_prefix(pu: np.ndarray, prefix: str, dev) -> torch.Tensor:
    """The UTF-16 prefix on the device, uploaded once per (prefix, device): a stream's FeatureHasher hashes the
    same column prefixes every micro-batch (was one host-to-device copy per column per batch)."""
    key = (prefix, str(dev))
    t = _PREFIX_CACHE.get(key)
    if t is None:
        if len(_PREFIX_CACHE) > 4096:
            _PREFIX_CACHE.clear()
        t = _PREFIX_CACHE[key] = torch.from_numpy(pu).to(dev)
    return t


MH_MAX_COLS, MH_MAX_PREFIX = 32, 1024


class _MultiHashArgs(ctypes.Structure):
    """Mirror of ``MultiHashArgs`` (ops/csrc/feature.hip)."""
    _fields_ = [("data", ctypes.c_void_p * MH_MAX_COLS), ("off", ctypes.c_void_p * MH_MAX_COLS),
                ("nulls", ctypes.c_void_p * MH_MAX_COLS), ("pstart", ctypes.c_int32 * (MH_MAX_COLS + 1)),
                ("prefix", ctypes.c_uint16 * MH_MAX_PREFIX)]


def murmur3_multi_index(blocks, prefixes, nf: int, seed: int = 0):
    """(idx int32 [m, n], valid uint8 [m, n]) of ``murmur3_utf8_index(blocks[j], nf, prefixes[j])`` for m device
    ``StringBlock`` columns of equal length in ONE kernel launch (valid = not NULL; idx 0 there), or None when the
    columns do not fit the launch table (more than 32, prefixes over 1024 UTF-16 units, not on a GPU)."""
    m = len(blocks)
    if m == 0 or m > MH_MAX_COLS or any(b.device.type != "cuda" for b in blocks):
        return None
    units = [np.frombuffer(p.encode("utf-16-le"), dtype=np.uint16) for p in prefixes]
    if sum(u.size for u in units) > MH_MAX_PREFIX:
        return None
    n = len(blocks[0])
    dev = blocks[0].device
    L = _lib.require()
    a = _MultiHashArgs()
    keep = []
    pos = 0
    for j, (b, u) in enumerate(zip(blocks, units)):
        data = b.data if b.nbytes else torch.zeros(1, dtype=torch.uint8, device=dev)
        off = b.offsets.contiguous()
        keep += [data, off]
        a.data[j], a.off[j] = data.data_ptr(), off.data_ptr()
        if b.nulls is not None:
            nl = b.nulls.to(dev, torch.bool).contiguous()
            keep.append(nl)
            a.nulls[j] = nl.data_ptr()
        a.pstart[j] = pos
        for q, c in enumerate(u.tolist()):
            a.prefix[pos + q] = c
        pos += u.size
    a.pstart[m] = pos
    idx = torch.empty((m, n), dtype=torch.int32, device=dev)
    valid = torch.empty((m, n), dtype=torch.uint8, device=dev)
    rc = L.alink_murmur3_multi_index(ctypes.addressof(a), m, n, seed & 0xFFFFFFFF, int(nf), idx.data_ptr(),
                                     valid.data_ptr(), _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_murmur3_multi_index failed: {rc}")
    return idx, valid


def murmur3_utf8_index(block: StringBlock, nf: int, prefix: str = "", seed: int = 0) -> torch.Tensor:
    """int64 [n] ``floorMod(abs(murmur3_32(seed).hashUnencodedChars(prefix + s)), nf)`` on the block's device."""
    n = len(block)
    dev = block.device
    if n == 0:
        return torch.zeros(0, dtype=torch.int64, device=dev)
    pu = np.frombuffer(prefix.encode("utf-16-le"), dtype=np.uint16).copy() if prefix else np.zeros(1, np.uint16)
    plen = len(prefix.encode("utf-16-le")) // 2
    if dev.type == "cuda":
        L = _lib.require()
        data = block.data if block.nbytes else torch.zeros(1, dtype=torch.uint8, device=dev)
        p = _device_prefix(pu, prefix, dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        rc = L.alink_murmur3_utf8_index(data.data_ptr(), block.offsets.contiguous().data_ptr(), n, p.data_ptr(),
                                        plen, seed & 0xFFFFFFFF, int(nf), None, out.data_ptr(), _lib.stream_ptr(dev))
        if rc != 0:
            raise RuntimeError(f"alink_murmur3_utf8_index failed: {rc}")
        return out.to(torch.int64)
    from .. import _native
    h = _native.murmur3_utf8(block.data.numpy(), block.offsets.numpy(), prefix, seed)
    if h is None:
        from ..models.feature.encoders import murmur3_index as host_index
        return torch.from_numpy(np.asarray(host_index([prefix + (s or "") for s in block.to_list()], nf),
                                           dtype=np.int64))
    a = np.abs(h.astype(np.int64))
    a = np.where(h == np.iinfo(np.int32).min, np.int64(np.iinfo(np.int32).min), a)   # Java abs(MIN_VALUE)
    return torch.from_numpy(np.mod(a, int(nf)))


def split_tokens(block: StringBlock, delim: int = 0x20):
    """Java ``String.split(" ")`` of every string of a packed block, on the block's device with no per-string
    Python work: returns ``(tokens, doc)`` — a ``StringBlock`` of the tokens back to back (document order) and the
    int64 document index of each token.  Semantics as ``models/nlp/text.java_split``: leading empty tokens are
    kept, trailing ones dropped, the empty string gives one empty token, a NULL gives none.  UTF-8 never carries
    the delimiter byte inside a multi-byte character, so splitting the bytes is splitting the characters."""
    dev = block.device
    n = len(block)
    data, off = block.data, block.offsets.to(torch.int64)
    nb = int(data.numel())
    is_d = data == delim
    # spaces per document (prefix sum of the delimiter mask at the document boundaries)
    cum = torch.zeros(nb + 1, dtype=torch.int64, device=dev)
    if nb:
        torch.cumsum(is_d.to(torch.int64), 0, out=cum[1:])
    nsp = cum[off[1:]] - cum[off[:-1]]
    ntok = nsp + 1                                            # tokens before the trailing-empty rule
    tok_doc = torch.repeat_interleave(torch.arange(n, device=dev), ntok)
    T = int(tok_doc.numel())
    # token t of document d ends at its k-th delimiter (k = t - first token of d) or at the document end
    first_tok = torch.cumsum(ntok, 0) - ntok
    k = torch.arange(T, device=dev) - first_tok[tok_doc]
    dpos = torch.nonzero(is_d).reshape(-1)                    # delimiter byte positions, ascending
    gk = cum[off[:-1]][tok_doc] + k                           # global index of that delimiter
    is_last = k == nsp[tok_doc]
    end = torch.where(is_last, off[1:][tok_doc], dpos[gk.clamp(max=max(dpos.numel() - 1, 0))] if dpos.numel()
                      else off[1:][tok_doc])
    start = torch.where(k == 0, off[:-1][tok_doc],
                        (dpos[(gk - 1).clamp(min=0)] + 1) if dpos.numel() else off[:-1][tok_doc])
    tlen = end - start
    # trailing empty tokens dropped; "" keeps its single empty token; a NULL document has none
    tid = torch.arange(T, device=dev)
    last_ne = torch.full((n,), -1, dtype=torch.int64, device=dev)
    ne = tlen > 0
    if T:
        last_ne.scatter_reduce_(0, tok_doc[ne], tid[ne], reduce="amax")
    dlen = off[1:] - off[:-1]
    keep = (tid <= last_ne[tok_doc]) | (dlen[tok_doc] == 0)
    if block.nulls is not None:
        keep &= ~block.nulls.to(dev)[tok_doc]
    start, tlen, tok_doc = start[keep], tlen[keep], tok_doc[keep]
    toff = torch.zeros(int(tlen.numel()) + 1, dtype=torch.int64, device=dev)
    torch.cumsum(tlen, 0, out=toff[1:])
    # token bytes back to back: every non-delimiter byte of a kept token, in order
    src = torch.repeat_interleave(start - toff[:-1], tlen) + torch.arange(int(toff[-1]), device=dev)
    tdata = data[src] if src.numel() else torch.zeros(0, dtype=torch.uint8, device=dev)
    return StringBlock(tdata, toff), tok_doc


def unique_ids(block: StringBlock) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """Exact dictionary encoding of a packed block on its device: ``(ids int64 [n], rep int64 [u])`` — equal
    strings get equal ids (0..u-1, in order of the 64-bit key), ``rep[i]`` is the first string with id i.  Keys are
    two 32-bit murmur3 hashes of the bytes; every string is then compared byte for byte with its representative, so
    the result is exact or None (a 64-bit collision: the caller takes its host path)."""
    n = len(block)
    dev = block.device
    if n == 0:
        z = torch.zeros(0, dtype=torch.int64, device=dev)
        return z, z
    h0 = hash_bytes(block, 0).to(torch.int64) & 0xFFFFFFFF
    h1 = hash_bytes(block, 0x5BD1E995).to(torch.int64) & 0xFFFFFFFF
    key = (h0 << 32) | h1
    uk, ids = torch.unique(key, return_inverse=True)
    pos = torch.arange(n, device=dev)
    rep = torch.full((uk.numel(),), n, dtype=torch.int64, device=dev)
    rep.scatter_reduce_(0, ids, pos, reduce="amin")
    off = block.offsets
    lens = off[1:] - off[:-1]
    r = rep[ids]
    if not bool(torch.equal(lens, lens[r])):
        return None
    tot = int(lens.sum())
    if tot:
        seg = torch.repeat_interleave(pos, lens)
        j = torch.arange(tot, device=dev) - torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens)
        if not bool(torch.equal(block.data[off[:-1][seg] + j], block.data[off[:-1][r][seg] + j])):
            return None
    return ids, rep


def tokenize_ws_lower(block: StringBlock) -> Optional[StringBlock]:
    """TokenizerMapper on a packed block, byte-parallel on its device: ASCII lower case, every run of ``\\s``
    (space, \\t \\n \\v \\f \\r) between tokens becomes one space, leading / trailing runs go -- what
    ``" ".join(java_split(s.lower(), "\\s+")).strip()`` gives.  None when a byte is non-ASCII (Unicode lower case)
    or an ASCII separator 0x1c-0x1f (which Python's strip() also treats as whitespace): the caller's row path."""
    d, off = block.data, block.offsets
    n, T = len(block), int(d.numel())
    if T == 0:
        return block
    if bool(((d >= 128) | ((d >= 0x1C) & (d <= 0x1F))).any()):
        return None
    dev = d.device
    ws = (d == 32) | ((d >= 9) & (d <= 13))
    lens = off[1:] - off[:-1]
    seg = torch.repeat_interleave(torch.arange(n, device=dev), lens)
    pos = torch.arange(T, device=dev)
    start, end = off[:-1][seg], off[1:][seg]
    prev_ws = torch.zeros_like(ws)
    prev_ws[1:] = ws[:-1]
    prev_ws &= pos != start
    last_nw = torch.cummax(torch.where(~ws, pos, torch.full_like(pos, -1)), 0).values
    next_nw = torch.flip(torch.cummin(torch.flip(torch.where(~ws, pos, torch.full_like(pos, T)), [0]), 0).values, [0])
    keep = ~ws | (~prev_ws & (last_nw >= start) & (next_nw < end))
    low = torch.where((d >= 65) & (d <= 90), d + 32, d)
    out = torch.where(ws, torch.full_like(d, 32), low)[keep]
    nl = torch.bincount(seg[keep], minlength=n)
    noff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(nl, 0, out=noff[1:])
    return StringBlock(out, noff, block.nulls)


def _gather_bytes(tok: StringBlock, tids: torch.Tensor, starts: torch.Tensor, total: int, fill: int,
                  seps: Optional[torch.Tensor] = None, sep_pos: Optional[torch.Tensor] = None) -> torch.Tensor:
    """An output byte buffer of ``total`` bytes (pre-filled with ``fill``) holding token ``tids[k]`` at ``starts[k]``
    (and the bytes ``seps`` at ``sep_pos``)."""
    dev = tok.data.device
    out = torch.full((total,), fill, dtype=torch.uint8, device=dev)
    toff = tok.offsets.to(dev)
    tl = (toff[1:] - toff[:-1])[tids]
    nb = int(tl.sum()) if tl.numel() else 0
    if nb:
        piece = torch.repeat_interleave(torch.arange(tids.numel(), device=dev), tl)
        local = torch.arange(nb, device=dev) - torch.repeat_interleave(torch.cumsum(tl, 0) - tl, tl)
        out[starts[piece] + local] = tok.data[toff[:-1][tids][piece] + local]
    if seps is not None and sep_pos is not None and sep_pos.numel():
        out[sep_pos] = seps
    return out


def join_tokens(tok: StringBlock, doc: torch.Tensor, keep: torch.Tensor, n: int, nulls=None,
                sep: int = 0x20) -> StringBlock:
    """Per document, its kept tokens (document order) joined by ``sep``: the rebuild half of a token filter
    (``sep.join(t for t in tokens if keep)``), byte-parallel.  ``n`` documents; ``nulls`` carried over."""
    dev = doc.device
    kid = torch.nonzero(keep).reshape(-1)
    kd = doc[kid]
    toff = tok.offsets.to(dev)
    tl = (toff[1:] - toff[:-1])[kid]
    cnt = torch.bincount(kd, minlength=n)
    blen = torch.zeros(n, dtype=torch.int64, device=dev)
    if kid.numel():
        blen.index_add_(0, kd, tl)
    dlen = blen + (cnt - 1).clamp(min=0)
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(dlen, 0, out=off[1:])
    # start of kept token k = its document's offset + the bytes and separators of the kept tokens before it
    cb = torch.cumsum(tl, 0) - tl                              # global exclusive prefix of kept bytes
    first = torch.cumsum(cnt, 0) - cnt                         # first kept token of each document
    rank = torch.arange(kid.numel(), device=dev) - first[kd]
    starts = off[:-1][kd] + (cb - cb[first[kd]]) + rank
    data = _gather_bytes(tok, kid, starts, int(off[-1]), sep)
    return StringBlock(data, off, nulls)


def ngram_join(tok: StringBlock, doc: torch.Tensor, n: int, ngram: int, nulls=None) -> StringBlock:
    """NGramMapper on split tokens: per document with m tokens, the m - ngram + 1 grams (``"_"``-joined runs of
    ``ngram`` consecutive tokens) joined by spaces; fewer than ``ngram`` tokens give "".  ngram >= 2 (a gram always
    holds a "_", so no gram is empty and the row path's strip() has nothing to remove)."""
    dev = doc.device
    m = torch.bincount(doc, minlength=n)
    G = (m - ngram + 1).clamp(min=0)
    Gt = int(G.sum())
    if Gt == 0:
        return StringBlock(torch.zeros(0, dtype=torch.uint8, device=dev),
                           torch.zeros(n + 1, dtype=torch.int64, device=dev), nulls)
    gdoc = torch.repeat_interleave(torch.arange(n, device=dev), G)
    tfirst = torch.cumsum(m, 0) - m                            # first token of each document
    gfirst = torch.cumsum(G, 0) - G                            # first gram of each document
    grank = torch.arange(Gt, device=dev) - gfirst[gdoc]
    pt = (tfirst[gdoc] + grank)[:, None] + torch.arange(ngram, device=dev)[None, :]   # [Gt, ngram] token ids
    toff = tok.offsets.to(dev)
    tl = (toff[1:] - toff[:-1])[pt]                            # [Gt, ngram]
    last_gram = grank == (G[gdoc] - 1)
    sep_len = torch.ones_like(tl)
    sep_len[:, -1] = (~last_gram).to(sep_len.dtype)            # " " after a gram but the document's last
    plen = (tl + sep_len).reshape(-1)
    pstart = torch.cumsum(plen, 0) - plen
    dlen = torch.zeros(n, dtype=torch.int64, device=dev)
    dlen.index_add_(0, gdoc, (tl + sep_len).sum(1))
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(dlen, 0, out=off[1:])
    flat_t = pt.reshape(-1)
    has_sep = sep_len.reshape(-1) > 0
    sep_char = torch.full((Gt, ngram), 0x5F, dtype=torch.uint8, device=dev)     # "_"
    sep_char[:, -1] = 0x20                                                      # " "
    sp = (pstart + tl.reshape(-1))[has_sep]
    data = _gather_bytes(tok, flat_t, pstart, int(off[-1]), 0x20, sep_char.reshape(-1)[has_sep], sp)
    return StringBlock(data, off, nulls)


def has_strip_space(data: torch.Tensor) -> bool:
    """Whether UTF-8 bytes hold a character Python's ``str.strip()`` removes other than the plain space: \\t..\\r,
    0x1c-0x1f, U+0085, U+00A0, U+1680, U+2000-U+200A, U+2028, U+2029, U+202F, U+205F, U+3000."""
    d = data
    if d.numel() == 0:
        return False
    if bool((((d >= 9) & (d <= 13)) | ((d >= 0x1C) & (d <= 0x1F))).any()):
        return True
    if d.numel() >= 2 and bool(((d[:-1] == 0xC2) & ((d[1:] == 0x85) | (d[1:] == 0xA0))).any()):
        return True
    if d.numel() >= 3:
        a, b, c = d[:-2], d[1:-1], d[2:]
        hit = (a == 0xE1) & (b == 0x9A) & (c == 0x80)
        hit |= (a == 0xE2) & (b == 0x80) & (((c >= 0x80) & (c <= 0x8A)) | (c == 0xA8) | (c == 0xA9) | (c == 0xAF))
        hit |= (a == 0xE2) & (b == 0x81) & (c == 0x9F)
        hit |= (a == 0xE3) & (b == 0x80) & (c == 0x80)
        if bool(hit.any()):
            return True
    return False
