"""Collapsed-Gibbs LDA token sweep on the GPU (``csrc/lda.hip``): one thread per token walks
its K topic weights from int32 count tables; no [T, K] matrices."""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["kernel_supported", "gibbs_sweep"]


def kernel_supported(dev) -> bool:
    return torch.device(dev).type == "cuda" and (_lib.available() or not _lib.torch_fallback_allowed())


def gibbs_sweep(d_tok, w_tok, z, nd, nw, nk, alpha: float, beta: float, V: int, u) -> torch.Tensor:
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
                           _lib.stream_ptr(z.device))
    if rc != 0:
        raise RuntimeError(f"alink_lda_gibbs failed: {rc}")
    return out
