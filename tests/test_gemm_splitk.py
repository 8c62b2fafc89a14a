"""Split-K A^T B chunking logic (ops/gemm.py) on the CPU: exact chunks, ragged tails, fewer rows than a chunk."""
import pytest
import torch

from alink_amd.ops.gemm import split_k, tn_matmul


@pytest.mark.parametrize("n,chunk", [(0, 4), (3, 4), (16, 4), (17, 4), (1001, 64), (4096, 1024)])
def test_split_k_matches_plain(n, chunk):
    g = torch.Generator().manual_seed(n)
    A = torch.randn(n, 5, dtype=torch.float64, generator=g)
    B = torch.randn(n, 3, dtype=torch.float64, generator=g)
    torch.testing.assert_close(split_k(A, B, chunk), A.T @ B, rtol=1e-12, atol=1e-12)


def test_tn_matmul_cpu_is_plain_product():
    A = torch.randn(50, 4, dtype=torch.float64)
    B = torch.randn(50, dtype=torch.float64)
    assert torch.equal(tn_matmul(A, B), A.T @ B)
