"""fp64 GEMM shapes of the MLP step on one GPU: plain matmul vs row-chunked batched (split-K) for the
tall-skinny weight-gradient products.  Prints ms and TFLOP/s per case."""
import time

import torch


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    n = 1 << 20
    for dt in (torch.float64, torch.float32):
        for a, b in ((64, 128), (128, 64), (64, 10), (10, 64)):
            H = torch.randn(n, a, device="cuda", dtype=dt)
            W = torch.randn(a, b, device="cuda", dtype=dt)
            D = torch.randn(n, b, device="cuda", dtype=dt)
            fl = 2 * n * a * b
            t_f = timeit(lambda: H @ W)
            t_wg = timeit(lambda: H.T @ D)
            res = []
            for c in (64, 256, 1024):
                t = timeit(lambda: torch.bmm(H.view(c, n // c, a).transpose(1, 2), D.view(c, n // c, b)).sum(0))
                res.append(f"splitK{c} {t:.3f}")
            t_bw = timeit(lambda: D @ W.T)
            print(f"{str(dt)[6:]} a={a} b={b}: fwd H@W {t_f:.3f} ms ({fl / t_f / 1e9:.1f} TF)  bwd D@W^T {t_bw:.3f}  "
                  f"wgrad H^T D {t_wg:.3f} ms ({fl / t_wg / 1e9:.1f} TF)  " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
