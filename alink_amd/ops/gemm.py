"""Tall-skinny transposed products ``A^T B`` (A [n, a], B [n, b], n >> a, b) as split-K batched GEMMs.

The library GEMM runs ``A^T B`` with the long n dimension as a single K loop, which leaves most of the 256 CUs idle:
on MI355X an fp64 ``[64 x 2^20] x [2^20 x 128]`` product takes 112 ms (0.2 TFLOP/s).  Cutting n into chunks of
``CHUNK`` rows and running one batched GEMM (one chunk per batch entry) followed by a reduction over the chunks
takes 0.13-0.57 ms (``profiles/gemm_splitk_r2.txt``).  Used by every "statistics over rows" product on the device:
Gram matrices (PCA, GLM IRLS, Newton Hessians, correlation), gradient right-hand sides ``X^T R`` (softmax, MLP
weight gradients) and the GMM / bisecting k-means M-step moments.  CPU tensors use plain ``A.T @ B``.
"""
from __future__ import annotations

import torch

__all__ = ["tn_matmul", "split_k", "CHUNK"]

CHUNK = 2048          # rows per batch entry
_MIN_ROWS = 4 * CHUNK


def tn_matmul(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """``A.T @ B`` for ``A`` [n, a] and ``B`` [n, b] or [n] (same dtype / device)."""
    n = A.shape[0]
    if not A.is_cuda or n < _MIN_ROWS or A.dim() != 2 or B.dim() not in (1, 2):
        return A.T @ B
    if B.dim() == 1:
        return tn_matmul(A, B[:, None])[:, 0]
    return split_k(A, B, CHUNK)


def split_k(A: torch.Tensor, B: torch.Tensor, chunk: int) -> torch.Tensor:
    """``A.T @ B`` as one batched GEMM over ``chunk``-row slices (+ the ragged tail), any device."""
    n = A.shape[0]
    c = n // chunk
    m = c * chunk
    a, b = A.shape[1], B.shape[1]
    A = A.contiguous()
    B = B.contiguous()
    if c == 0:
        return A.T @ B
    out = torch.bmm(A[:m].view(c, chunk, a).transpose(1, 2), B[:m].view(c, chunk, b)).sum(0)
    if m < n:
        out.addmm_(A[m:].T, B[m:])
    return out
