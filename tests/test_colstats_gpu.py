"""One-pass column statistics HIP kernel (ops/csrc/colstats.hip) against plain fp64 torch."""
import time

import numpy as np
import pytest
import torch

from alink_amd.ops import stats as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d", [(1, 1), (1000, 3), (4097, 100), (2000, 256), (999, 300), (300, 1000), (0, 5)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
def test_colstats_matches_torch(n, d, dtype):
    g = torch.Generator(device="cuda").manual_seed(n * 7 + d)
    X = (torch.randn(n, d, device="cuda", generator=g) * 3).to(dtype)
    if n > 10:
        X[::7, 0] = 0
    a = S.colstats(X, use_kernel=True)
    b = S.colstats_torch(X)
    for k in ("sum", "sum2", "l1"):
        np.testing.assert_allclose(a[k].cpu().numpy(), b[k].cpu().numpy(), rtol=1e-12, atol=1e-9, err_msg=k)
    for k in ("min", "max", "nnz"):
        assert torch.equal(a[k], b[k]), k


def test_colstats_nan_propagates():
    X = torch.ones(500, 4, device="cuda")
    X[123, 2] = float("nan")
    a = S.colstats(X, use_kernel=True)
    assert torch.isnan(a["min"][2]) and torch.isnan(a["max"][2]) and torch.isnan(a["sum"][2])
    assert float(a["min"][1]) == 1.0


def test_colstats_bandwidth_smoke():
    X = torch.randn(4_000_000, 128, device="cuda")
    S.colstats(X, use_kernel=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        S.colstats(X, use_kernel=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(f"colstats 4e6 x 128 fp32: {dt * 1e3:.3f} ms, {X.numel() * 4 / dt / 1e12:.2f} TB/s")
    assert dt < 0.05
