"""Numerics of the fused HIP KMeans assign+accumulate kernel vs a PyTorch fp32/fp64 reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _data(n, k, seed=0, dev="cuda"):
    g = torch.Generator(device="cpu").manual_seed(seed)
    centers = torch.randn(k, 128, generator=g) * 4
    lab = torch.randint(0, k, (n,), generator=g)
    X = (centers[lab] + torch.randn(n, 128, generator=g)).to(dev, torch.bfloat16)
    C = (centers + 0.3 * torch.randn(k, 128, generator=g)).to(dev, torch.float64)
    return X, C


@pytest.mark.parametrize("variant", [1, 3, 4, 5, 6])
@pytest.mark.parametrize("n,k", [(1, 1), (127, 3), (128, 32), (1000, 33), (4097, 100), (50000, 128), (300001, 100)])
def test_assign_accumulate_matches_reference(n, k, variant):
    from alink_amd.ops import kmeans as K
    from alink_amd.ops import _lib
    assert _lib.available(), "HIP library must be built and loadable on the GPU box"
    X, C = _data(n, k)
    got = K.assign_accumulate_hip(X, C, variant=variant)
    ref = K.assign_accumulate_torch(X, C)
    torch.cuda.synchronize()
    # counts: assignments may differ only for near-ties (relative 2^-16 packing); allow a tiny fraction
    dc = (got[:, -1] - ref[:, -1]).abs().sum().item()
    assert dc <= max(2, 1e-4 * n), f"count mismatch {dc}"
    assert abs(got[:, -1].sum().item() - n) < 0.5
    if dc == 0:
        torch.testing.assert_close(got[:, :-1], ref[:, :-1], rtol=1e-5, atol=1e-3 * max(1.0, n / 1000))


@pytest.mark.parametrize("variant,contig", [(1, None), (4, True), (4, False), (5, True), (5, False), (6, True), (6, False)])
@pytest.mark.parametrize("n,k,grid", [(200, 7, 1), (49157, 100, 3), (33333, 64, 7), (640, 100, 2), (70000, 100, 256)])
def test_assign_accumulate_small_grid(n, k, grid, variant, contig):
    """Few workgroups -> long per-workgroup tile loops (pipeline warm-up, steady state and drain)."""
    from alink_amd.ops import kmeans as K
    X, C = _data(n, k, seed=11)
    got = K.assign_accumulate_hip(X, C, grid=grid, variant=variant, contiguous=contig)
    ref = K.assign_accumulate_torch(X, C)
    torch.cuda.synchronize()
    assert (got[:, -1] - ref[:, -1]).abs().sum().item() <= 2
    assert abs(got[:, -1].sum().item() - n) < 0.5


def test_kernel_deterministic():
    from alink_amd.ops import kmeans as K
    X, C = _data(200000, 100, seed=3)
    a = K.assign_accumulate_hip(X, C)
    b = K.assign_accumulate_hip(X, C)
    assert torch.equal(a, b)


@pytest.mark.parametrize("n,k", [(700, 40), (65536, 64), (12345, 17)])
def test_v2_kernel_small_k(n, k):
    from alink_amd.ops import kmeans as K
    X, C = _data(n, k, seed=5)
    got = K.assign_accumulate_hip(X, C, variant=2)
    ref = K.assign_accumulate_torch(X, C)
    assert (got[:, -1] - ref[:, -1]).abs().sum().item() <= 2


@pytest.mark.parametrize("d", [64, 128, 256])
@pytest.mark.parametrize("n,m", [(1, 1), (31, 5), (1000, 33), (4097, 256), (20001, 300), (70000, 700)])
def test_nearest_kernel_matches_fp32_reference(n, m, d):
    """csrc/kmeans_nearest.hip vs a plain fp32 PyTorch argmin of |x - c|^2 (bf16-rounded centroids)."""
    from alink_amd.ops import kmeans as K
    g = torch.Generator(device="cpu").manual_seed(n + m + d)
    X = (torch.randn(n, d, generator=g) * 2).to("cuda", torch.bfloat16)
    C = (torch.randn(m, d, generator=g) * 2).to("cuda", torch.float64)
    idx, d2 = K.nearest_hip(X, C)
    Cb = C.to(torch.bfloat16).float()
    ref = ((X.float()[:, None, :] - Cb[None, :, :]) ** 2).sum(-1) if n * m <= 4_000_000 else torch.cdist(X.float(), Cb) ** 2
    rbest, ridx = ref.min(1)
    torch.cuda.synchronize()
    assert idx.shape == (n,) and d2.shape == (n,)
    assert int(idx.min()) >= 0 and int(idx.max()) < m
    # chosen centroid's true distance equals the optimum up to fp32 rounding of the expanded form
    chosen = ref.gather(1, idx.long()[:, None])[:, 0]
    tol = 1e-4 * (X.float() ** 2).sum(1) + 1e-3
    assert bool(((chosen - rbest) <= tol).all())
    assert bool(((d2 - rbest).abs() <= tol + 1e-3 * rbest).all())
    assert (idx.long() != ridx).float().mean().item() < 0.01


def test_nearest_kernel_exact_candidates():
    """k-means|| candidates are rows of X: distance to itself must come out 0 and the index its own."""
    from alink_amd.ops import kmeans as K
    X = torch.randn(5000, 128, device="cuda").to(torch.bfloat16)
    sel = torch.arange(0, 5000, 17, device="cuda")
    idx, d2 = K.nearest_hip(X, X[sel].double())
    assert torch.equal(idx[sel].long(), torch.arange(sel.numel(), device="cuda"))
    assert float(d2[sel].abs().max()) < 1e-2


@pytest.mark.parametrize("d", [1, 7, 8, 16, 31, 64])
@pytest.mark.parametrize("loss", ["log", "logistic", "square", "hinge", "smooth", "perceptron", "exp", "huber", "svr"])
def test_linear_grad_kernel_matches_fp64_reference(d, loss):
    """csrc/linear.hip fused gradient vs the torch two-GEMV form of the same unary loss (fp64)."""
    from alink_amd.models.linear import objfunc as O
    from alink_amd.ops import linear as lops
    fn = {"log": O.LogLossFunc(), "logistic": O.LogisticLossFunc(), "square": O.SquareLossFunc(),
          "hinge": O.HingeLossFunc(), "smooth": O.SmoothHingeLossFunc(), "perceptron": O.PerceptronLossFunc(),
          "exp": O.ExponentialLossFunc(), "huber": O.HuberLossFunc(0.7), "svr": O.SvrLossFunc(0.2)}[loss]
    g = torch.Generator(device="cpu").manual_seed(d)
    n = 50001
    X = torch.randn(n, d, generator=g, dtype=torch.float64).cuda()
    y = (torch.randint(0, 2, (n,), generator=g) * 2 - 1).double().cuda()
    w = torch.rand(n, generator=g, dtype=torch.float64).cuda()
    coef = (0.3 * torch.randn(d, generator=g, dtype=torch.float64)).cuda()
    code, prm = lops.loss_code(fn)
    got, lsum, wsum = lops.linear_grad_hip(X, y, w, coef, code, prm)
    eta = X @ coef
    ref = X.T @ (w * fn.derivative(eta, y))
    torch.testing.assert_close(got, ref, rtol=1e-10, atol=1e-9)
    torch.testing.assert_close(lsum, (w * fn.loss(eta, y)).sum(), rtol=1e-10, atol=1e-9)
    torch.testing.assert_close(wsum, w.sum(), rtol=1e-12, atol=1e-9)
