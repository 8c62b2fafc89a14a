"""MLP forward / backward with hipBLASLt GEMMs and fused HIP epilogues.

Hidden layers: ``S = sigmoid(H W + b)`` is one GEMM plus the in-place ``bias_sigmoid`` kernel; the softmax
cross-entropy output layer's ``w * (softmax(z) - onehot(y))`` and loss come from the pivot-free K16 kernel; the
backward pass is ``dW = H^T D``, ``db = sum D``, ``D <- (D W^T) * S (1 - S)`` with the sigmoid derivative fused in
place.  Replaces autograd's recorded graph (which stores more intermediates and launches separate elementwise
kernels).  Reference: ``AffineLayerModel.java:68-84`` (forward / backward), ``SigmoidLayerModel``,
``SoftmaxLayerWithCrossEntropyLoss`` (A/operator/common/classification/ann/).
"""
from __future__ import annotations

from typing import Sequence, Tuple

import torch

from .gemm import tn_matmul
from . import _lib

__all__ = ["mlp_grad", "kernel_supported", "KMAX"]

KMAX = 32


def kernel_supported(X: torch.Tensor, layers: Sequence[int]) -> bool:
    return X.is_cuda and X.dtype == torch.float64 and 0 < int(layers[-1]) <= KMAX and \
        (_lib.available() or not _lib.torch_fallback_allowed())


def _unpack(w: torch.Tensor, layers):
    out, off = [], 0
    for i in range(len(layers) - 1):
        a, b = layers[i], layers[i + 1]
        out.append((w[off:off + a * b].reshape(a, b), w[off + a * b:off + a * b + b]))
        off += a * b + b
    return out


def mlp_grad(X: torch.Tensor, y: torch.Tensor, w: torch.Tensor, coef: torch.Tensor, layers) \
        -> Tuple[torch.Tensor, torch.Tensor]:
    """(flat gradient of sum_i w_i CE_i in the coef layout, weighted loss sum)."""
    L = _lib.require()
    dev = X.device
    st = _lib.stream_ptr(dev)
    params = _unpack(coef, layers)
    X = X.contiguous()
    y = y.to(torch.float64).contiguous()
    w = w.to(torch.float64).contiguous()
    n = X.shape[0]
    hs = [X]
    h = X
    for W, b in params[:-1]:
        z = h @ W
        rc = L.alink_bias_sigmoid_f64(z.data_ptr(), n, z.shape[1], b.contiguous().data_ptr(), st)
        if rc != 0:
            raise RuntimeError(f"alink_bias_sigmoid_f64 failed: {rc}")
        hs.append(z)
        h = z
    Wo, bo = params[-1]
    zo = torch.addmm(bo, h, Wo).contiguous()
    D = torch.empty_like(zo)
    part = torch.zeros(max(1, L.alink_softmax_grid(n)), dtype=torch.float64, device=dev)
    rc = L.alink_softmax_full_grad_f64(zo.data_ptr(), y.data_ptr(), w.data_ptr(), n, zo.shape[1], D.data_ptr(),
                                       part.data_ptr(), st)
    if rc != 0:
        raise RuntimeError(f"alink_softmax_full_grad_f64 failed: {rc}")
    grads = [None] * len(params)
    for i in range(len(params) - 1, -1, -1):
        W, _ = params[i]
        grads[i] = (tn_matmul(hs[i], D).reshape(-1), D.sum(0))
        if i > 0:
            D = (D @ W.T).contiguous()
            rc = L.alink_sigmoid_bwd_f64(D.data_ptr(), hs[i].data_ptr(), D.numel(), st)
            if rc != 0:
                raise RuntimeError(f"alink_sigmoid_bwd_f64 failed: {rc}")
    return torch.cat([t for gw, gb in grads for t in (gw, gb)]), part.sum()
