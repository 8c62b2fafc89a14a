"""Split-K tall-skinny A^T B (ops/gemm.py) against the plain product, fp64 and fp32, with ragged row counts."""
import pytest
import torch

from alink_amd.ops.gemm import tn_matmul

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [5, 8192, 8193, 100003, 1 << 20])
@pytest.mark.parametrize("a,b", [(1, 1), (64, 128), (10, 3), (129, 1)])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_tn_matmul_matches(n, a, b, dtype):
    g = torch.Generator(device="cuda").manual_seed(n + a + b)
    A = torch.randn(n, a, device="cuda", dtype=dtype, generator=g)
    B = torch.randn(n, b, device="cuda", dtype=dtype, generator=g)
    ref = (A.double().T @ B.double())
    out = tn_matmul(A, B)
    assert out.shape == (a, b) and out.dtype == dtype
    tol = 1e-9 if dtype == torch.float64 else 2e-3
    torch.testing.assert_close(out.double(), ref, rtol=tol, atol=tol * (n ** 0.5))
    v = tn_matmul(A, B[:, 0])
    torch.testing.assert_close(v.double(), ref[:, 0], rtol=tol, atol=tol * (n ** 0.5))
