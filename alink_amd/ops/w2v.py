"""Word2Vec skip-gram hierarchical-softmax Hogwild kernel (``csrc/w2v.hip``).

``sg_hs_train(docs, shrinks, window, C, P, lens, syn0, syn1, alpha)`` trains every (centre, context) pair of
the documents in place; the window enumeration runs on the device (one wave per centre position).
Reference: ``Word2VecTrainBatchOp.CalcModel`` (``A/operator/batch/nlp/Word2VecTrainBatchOp.java:~425-505``).
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from . import _lib

__all__ = ["kernel_supported", "HuffmanDevice", "sg_hs_train"]


def kernel_supported(dev, d: int) -> bool:
    return torch.device(dev).type == "cuda" and 1 <= d <= 512 and \
        (_lib.available() or not _lib.torch_fallback_allowed())


class HuffmanDevice:
    """Huffman codes (int8) / points (int32) / lengths on the device, padded to a common path length."""

    def __init__(self, C: np.ndarray, P: np.ndarray, lens: np.ndarray, dev):
        self.Lmax = int(C.shape[1])
        self.codes = torch.as_tensor(C.astype(np.int8), device=dev).contiguous()
        self.points = torch.as_tensor(P.astype(np.int32), device=dev).contiguous()
        self.lens = torch.as_tensor(lens.astype(np.int32), device=dev).contiguous()


def sg_hs_train(docs: List[np.ndarray], shrinks: List[np.ndarray], window: int, H: HuffmanDevice,
                syn0: torch.Tensor, syn1: torch.Tensor, alpha: float, max_waves: int = 0) -> None:
    L = _lib.require()
    keep = [(d, b) for d, b in zip(docs, shrinks) if len(d) >= 2]
    if not keep:
        return
    lens = np.array([len(d) for d, _ in keep], np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    tok = np.concatenate([d for d, _ in keep]).astype(np.int32)
    shr = np.concatenate([b for _, b in keep]).astype(np.int32)
    dstart = np.repeat(starts, lens).astype(np.int32)
    dend = np.repeat(starts + lens, lens).astype(np.int32)
    dev = syn0.device
    t = [torch.as_tensor(a, device=dev) for a in (tok, dstart, dend, shr)]
    rc = L.alink_w2v_sg_hs_f32(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), int(tok.size),
                               int(window), H.codes.data_ptr(), H.points.data_ptr(), H.lens.data_ptr(), H.Lmax,
                               syn0.data_ptr(), syn1.data_ptr(), int(syn0.shape[1]), float(alpha), int(max_waves),
                               _lib.stream_ptr(dev))
    if rc != 0:
        raise RuntimeError(f"alink_w2v_sg_hs_f32 failed: {rc}")
