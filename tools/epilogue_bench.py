"""Times the fused epilogue kernels (K16 softmax, K22 GMM E-step, K6 GBDT g/h, K27 scaler) against the torch
chains they replace on one GPU.  Prints one line per case."""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from alink_amd.models.clustering.gmm import _root_inv
from alink_amd.ops import elementwise as ew
from alink_amd.ops import gmm as G
from alink_amd.ops import softmax as S


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    n, k1 = 10_000_000, 9
    eta = torch.randn(n, k1, device=dev, dtype=torch.float64, generator=g)
    y = torch.randint(0, k1 + 1, (n,), device=dev, generator=g).double()
    w = torch.ones(n, device=dev, dtype=torch.float64)
    a = timeit(lambda: S.softmax_grad(eta, y, w))
    b = timeit(lambda: S.softmax_grad_torch(eta.clone(), y, w))
    print(f"K16 softmax grad  n={n} k1={k1}: kernel {a:.3f} ms  torch {b:.3f} ms  ({b / a:.1f}x)")
    ed = torch.randn_like(eta)
    a = timeit(lambda: S.softmax_search(eta, ed, y, w, 0.5, 11), 3)
    b = timeit(lambda: S.softmax_search_torch(eta, ed, y, w, 0.5, 11), 3)
    print(f"K16 softmax search n={n} k1={k1} 11 steps: kernel {a:.3f} ms  torch {b:.3f} ms  ({b / a:.1f}x)")
    del eta, ed
    n, k, d = 1_000_000, 16, 32
    X0 = torch.randn(n, d, device=dev, dtype=torch.float64, generator=g)
    mu0 = torch.randn(k, d, device=dev, dtype=torch.float64, generator=g)
    A = torch.randn(k, d, d, device=dev, dtype=torch.float64, generator=g)
    Sg = A @ A.transpose(1, 2) / d + 0.1 * torch.eye(d, device=dev, dtype=torch.float64)
    W, logdet, rank = _root_inv(Sg)
    logw = torch.full((k,), -math.log(k), device=dev, dtype=torch.float64)
    a = timeit(lambda: G.estep(X0, mu0, W, logdet, rank, logw))
    b = timeit(lambda: G.estep_torch(X0, mu0, W, logdet, rank, logw))
    print(f"K22 GMM E-step n={n} k={k} d={d}: kernel+GEMM {a:.3f} ms  torch {b:.3f} ms  ({b / a:.1f}x)")
    n = 50_000_000
    pred = torch.randn(n, device=dev, generator=g)
    yy = (torch.rand(n, device=dev, generator=g) < 0.5).float()
    ww = torch.ones(n, device=dev)
    a = timeit(lambda: ew.gbdt_grad_stats(pred, yy, ww, 1))
    b = timeit(lambda: ew.gbdt_grad_stats_torch(pred, yy, ww, 1))
    print(f"K6 GBDT logistic g/h n={n}: kernel {a:.3f} ms ({n * 28 / a / 1e9:.2f} TB/s)  torch {b:.3f} ms  "
          f"({b / a:.1f}x)")
    X = torch.randn(n // 10, 10, device=dev, dtype=torch.float64, generator=g)
    lo = torch.randn(10, device=dev, dtype=torch.float64)
    hi = lo + 1
    a = timeit(lambda: ew.col_transform(X, "minmax", lo, hi, 0.0, 1.0))
    b = timeit(lambda: ew.col_transform_torch(X, "minmax", lo, hi, 0.0, 1.0))
    print(f"K27 min-max scaler {tuple(X.shape)} fp64: kernel {a:.3f} ms ({X.numel() * 16 / a / 1e9:.2f} TB/s)  "
          f"torch {b:.3f} ms  ({b / a:.1f}x)")
    del X, pred, yy, ww
    from alink_amd.ops import mlp as M
    from alink_amd.models.classification.mlp import mlp_forward, weight_size
    layers = [64, 128, 64, 10]
    n = 1_000_000
    X = torch.randn(n, layers[0], device=dev, dtype=torch.float64, generator=g)
    y = torch.randint(0, layers[-1], (n,), device=dev, generator=g).double()
    w = torch.ones(n, device=dev, dtype=torch.float64)
    coef = torch.randn(weight_size(layers), device=dev, dtype=torch.float64, generator=g) * 0.1

    def autograd_step():
        wt = coef.clone().requires_grad_(True)
        P = mlp_forward(X, wt, layers)
        loss = (-torch.log(P.gather(1, y.long()[:, None])[:, 0].clamp_min(1e-300)) * w).sum()
        return torch.autograd.grad(loss, wt)[0]
    a = timeit(lambda: M.mlp_grad(X, y, w, coef, layers))
    b = timeit(autograd_step)
    print(f"K17 MLP grad {layers} n={n} fp64: explicit+kernels {a:.3f} ms  autograd {b:.3f} ms  ({b / a:.1f}x)")


if __name__ == "__main__":
    main()
