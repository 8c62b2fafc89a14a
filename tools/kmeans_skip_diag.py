"""Evidence for the round-5 driver failure of ``test_update_convergence_word_and_skipped_assign``.

Re-creates the old slab allocation (``torch.empty``, memory recycled from earlier tests whose inputs held NaN / inf)
and runs the test's skipped-launch sequence, then reports for every slab word that ``torch.equal`` would call
changed: its (slab, row, col), whether the row is >= 16*ceil(k/16) (never written by kmeans_v10), whether it is NaN,
and whether the bit pattern changed.  Run on a GPU box:  python tools/kmeans_skip_diag.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from alink_amd.ops import kmeans as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(9)
    # what the earlier tests leave in the allocator: large bf16 blocks with NaN / inf entries, freed
    junk = []
    for _ in range(4):
        t = torch.randn(300_001, 128, generator=g).to(dev, torch.bfloat16)
        t[::3] = float("nan")
        t[1::3] = float("inf")
        junk.append(t)
    del junk, t
    torch.cuda.synchronize()
    n, k = 100_003, 60
    centers = torch.randn(k, 128, generator=g) * 4
    lab = torch.randint(0, k, (n,), generator=g)
    X = (centers[lab] + torch.randn(n, 128, generator=g)).to(dev, torch.bfloat16)
    C = (centers + 0.3 * torch.randn(k, 128, generator=g)).to(dev, torch.float64)
    grid = int(K._lib.require().alink_kmeans_v10_grid(n, K._num_cus(dev)))
    # the round-5 allocation: uninitialised slabs
    K._BUF.clear()
    K._BUF[(0, grid)] = (torch.empty((grid, K.HIP_KMAX, K.HIP_D), dtype=torch.float32, device=dev),
                         torch.empty((grid, K.HIP_KMAX), dtype=torch.float32, device=dev))
    s, sc = K._BUF[(0, grid)]
    print(f"grid {grid}; NaN words in the fresh slab: {int(torch.isnan(s).sum())} of {s.numel()}; "
          f"in rows >= 64: {int(torch.isnan(s[:, 64:]).sum())}")
    buf = K.assign_accumulate_hip(X, C)
    prev = (buf[:, :128] / buf[:, 128:]) + 1e-3
    Cn, read = K.update_centroids_hip(buf, prev, deferred=True, hysteresis=False, skip_tol=1e9)
    read()
    before = [t.clone() for t in (s, sc)]
    K.assign_accumulate_hip(X, Cn, skip=read.skip)
    torch.cuda.synchronize()
    kb = 16 * ((k + 15) // 16)
    for name, a, b in (("slab", before[0], s), ("slab_cnt", before[1], sc)):
        eq = torch.equal(a, b)
        bits = torch.equal(a.view(torch.int32), b.view(torch.int32))
        ne = (a != b).nonzero()
        nan_ne = int(torch.isnan(a[a != b]).sum()) if ne.numel() else 0
        rows = ne[:, 1] if ne.numel() else ne
        print(f"{name}: torch.equal={eq} bitwise_equal={bits} words a!=b: {ne.shape[0]} "
              f"(NaN: {nan_ne}; in rows >= {kb}: {int((rows >= kb).sum()) if ne.numel() else 0}); "
              f"first: {ne[:3].tolist()}")
    print("verdict:", "test artefact (NaN != NaN in never-written rows)"
          if all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(before, (s, sc)))
          else "the skipped launch WROTE slab words")


if __name__ == "__main__":
    main()
