"""LDA on the GPU (``csrc/lda.hip``).

* ``gibbs_sweep``: collapsed-Gibbs token sweep from int32 count tables, no [T, K] matrices — by default the
  wave-cooperative kernel (G lanes per token read the document / word count rows coalesced, segmented scan +
  ballot pick); ``variant=0`` is the thread-per-token kernel.
* ``estep``: online-VB E-step, one wave per document running all its fixed-point iterations in registers
  (reference ``OnlineCorpusStep.java``).
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["kernel_supported", "gibbs_sweep", "estep"]

GIBBS_VARIANT = int(__import__("os").environ.get("ALINK_LDA_GIBBS_VARIANT", "1"))


def kernel_supported(dev) -> bool:
    return torch.device(dev).type == "cuda" and (_lib.available() or not _lib.torch_fallback_allowed())


def gibbs_sweep(d_tok, w_tok, z, nd, nw, nk, alpha: float, beta: float, V: int, u,
                variant: int = None) -> torch.Tensor:
    L = _lib.require()
    T = z.numel()
    out = torch.empty_like(z)
    if T == 0:
        return out
    K = nd.shape[1]
    nd = nd.to(torch.int32).contiguous()
    nw = nw.to(torch.int32).contiguous()
    nk = nk.to(torch.float64).contiguous()
    rc = L.alink_lda_gibbs(d_tok.contiguous().data_ptr(), w_tok.contiguous().data_ptr(), z.contiguous().data_ptr(), T,
                           K, nd.data_ptr(), nw.data_ptr(), nk.data_ptr(), float(alpha), float(beta),
                           float(V * beta), u.to(torch.float64).contiguous().data_ptr(), out.data_ptr(),
                           GIBBS_VARIANT if variant is None else int(variant), _lib.stream_ptr(z.device))
    if rc != 0:
        raise RuntimeError(f"alink_lda_gibbs failed: {rc}")
    return out


def estep(doc, word, cts, n_docs: int, expElogbeta_T, alpha, gamma0, max_iter: int = 100, tol: float = 1e-3):
    """Online-VB E-step on the GPU: (gamma [D, K], expElogtheta [D, K], phinorm [T]) for tokens grouped by
    document (``doc`` non-decreasing).  ``expElogbeta_T`` [V, K]; K <= 256."""
    L = _lib.require()
    dev = gamma0.device
    D, K = gamma0.shape
    T = doc.numel()
    order = None
    if T > 1 and bool((doc[1:] < doc[:-1]).any()):
        order = torch.argsort(doc, stable=True)
        doc, word, cts = doc[order], word[order], cts[order]
    off = torch.zeros(D + 1, dtype=torch.int64, device=dev)
    if T:
        torch.cumsum(torch.bincount(doc.to(torch.int64), minlength=D)[:D], 0, out=off[1:])
    word = word.to(torch.int64).contiguous()
    cts = cts.to(torch.float64).contiguous()
    eb = expElogbeta_T.to(torch.float64).contiguous()
    al = alpha.to(device=dev, dtype=torch.float64).contiguous()
    g0 = gamma0.to(torch.float64).contiguous()
    gamma = torch.empty((D, K), dtype=torch.float64, device=dev)
    et = torch.empty((D, K), dtype=torch.float64, device=dev)
    phin = torch.empty(max(T, 1), dtype=torch.float64, device=dev)
    rc = L.alink_lda_estep(off.data_ptr(), word.data_ptr(), cts.data_ptr(), D, K, eb.data_ptr(), al.data_ptr(),
                           g0.data_ptr(), int(max_iter), float(tol), gamma.data_ptr(), et.data_ptr(), phin.data_ptr(),
                           _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_lda_estep failed: {rc}")
    phin = phin[:T]
    if order is not None:
        inv = torch.empty_like(order)
        inv[order] = torch.arange(T, device=dev)
        phin = phin[inv]
    return gamma, et, phin
