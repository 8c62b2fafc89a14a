"""Numerics of the fused HIP KMeans assign+accumulate kernel vs a PyTorch fp32/fp64 reference."""
import os

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


def _own_assignment_check(X, C, got, asg, k):
    """The kernel's sums/counts must equal the fp64 sums of X by the kernel's OWN assignment, and every
    assignment must be optimal up to the 2^-17 relative packing of the score (near-ties may go either way)."""
    n = X.shape[0]
    a = asg.long()
    assert int(a.min()) >= 0 and int(a.max()) < k
    ref = torch.zeros((k, 129), dtype=torch.float64, device=X.device)
    ref[:, :128].index_add_(0, a, X.double())
    ref[:, 128].index_add_(0, a, torch.ones(n, dtype=torch.float64, device=X.device))
    assert torch.equal(got[:, 128], ref[:, 128]), "counts differ from the kernel's own assignment"
    cnt = ref[:, 128:129]
    tol = 4e-6 * cnt * float(X.float().abs().max()) + 1e-3
    assert bool(((got[:, :128] - ref[:, :128]).abs() <= tol).all())
    Cb = C.to(torch.bfloat16).float()
    half = 0.5 * (Cb * Cb).sum(1)
    for s in range(0, n, 1 << 20):
        sc = X[s:s + (1 << 20)].float() @ Cb.T - half
        best = sc.max(1).values
        chosen = sc.gather(1, a[s:s + (1 << 20), None])[:, 0]
        assert bool((best - chosen <= 2.0 ** -15 * best.abs() + 1e-4).all()), "non-optimal assignment"


@pytest.fixture(params=["v7", "v10"])
def kernel(request, monkeypatch):
    """Run a test on both fused kernels (v10 serves k <= 112; above that the call falls back to v7)."""
    monkeypatch.setenv("ALINK_KMEANS_KERNEL", request.param)
    return request.param


@pytest.mark.parametrize("n,k", [(1, 1), (63, 3), (64, 16), (65, 17), (129, 100), (1000, 33), (4097, 100),
                                 (50000, 128), (300001, 100), (123457, 112), (70001, 8)])
def test_v7_matches_own_assignment_reference(n, k, kernel):
    from alink_amd.ops import kmeans as K
    from alink_amd.ops import _lib
    assert _lib.available(), "HIP library must be built and loadable on the GPU box"
    X, C = _data(n, k)
    asg = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    got = K.assign_accumulate_hip(X, C, assign_out=asg)
    torch.cuda.synchronize()
    _own_assignment_check(X, C, got, asg, k)
    # and against an independent torch argmax: only near-ties may differ
    ref = K.assign_accumulate_torch(X, C)
    assert (got[:, -1] - ref[:, -1]).abs().sum().item() <= max(2, 1e-4 * n)


@pytest.mark.parametrize("n,k,grid", [(200, 7, 1), (49157, 100, 3), (33333, 64, 7), (640, 100, 2), (70000, 100, 256),
                                      (1000003, 128, 5), (129, 50, 1), (192, 50, 1), (257, 20, 2)])
def test_v7_small_grid_long_loops(n, k, grid, kernel):
    """Few workgroups -> long per-workgroup tile loops (ring warm-up, steady state, one-hot reuse, drain)."""
    from alink_amd.ops import kmeans as K
    X, C = _data(n, k, seed=11)
    asg = torch.empty((n,), dtype=torch.int32, device="cuda")
    got = K.assign_accumulate_hip(X, C, grid=grid, assign_out=asg)
    torch.cuda.synchronize()
    _own_assignment_check(X, C, got, asg, k)


def test_v7_without_assign_output_equals_with(kernel):
    from alink_amd.ops import kmeans as K
    X, C = _data(100003, 100, seed=4)
    a = K.assign_accumulate_hip(X, C)
    asg = torch.empty((X.shape[0],), dtype=torch.int32, device="cuda")
    b = K.assign_accumulate_hip(X, C, assign_out=asg)
    assert torch.equal(a, b)


@pytest.mark.parametrize("flags", [1])
@pytest.mark.parametrize("n,k,grid", [(300001, 100, None), (49157, 97, 3), (4097, 16, None)])
def test_v10_launch_variants_bit_identical(n, k, grid, flags, monkeypatch):
    """The load cache policy (flag 1: default policy instead of non-temporal) changes only the load schedule:
    the sums are bit-identical to the default launch."""
    from alink_amd.ops import kmeans as K
    X, C = _data(n, k, seed=9)
    monkeypatch.setattr(K, "V10_FLAGS", 0)
    a = K.assign_accumulate_hip(X, C, grid=grid)
    monkeypatch.setattr(K, "V10_FLAGS", flags)
    b = K.assign_accumulate_hip(X, C, grid=grid)
    assert K.kernel_version(k) == "v10"
    assert torch.equal(a, b)


def test_v10_and_v7_agree():
    """Same assignments (same distance MFMAs and argmax), sums equal up to fp32 summation order."""
    import os
    from alink_amd.ops import kmeans as K
    X, C = _data(500000, 100, seed=5)
    n = X.shape[0]
    out = {}
    for v in ("v7", "v10"):
        os.environ["ALINK_KMEANS_KERNEL"] = v
        asg = torch.empty((n,), dtype=torch.int32, device="cuda")
        out[v] = (K.assign_accumulate_hip(X, C, assign_out=asg), asg)
    del os.environ["ALINK_KMEANS_KERNEL"]
    assert torch.equal(out["v7"][1], out["v10"][1])
    assert torch.equal(out["v7"][0][:, 128], out["v10"][0][:, 128])
    cnt = out["v7"][0][:, 128:129]
    assert bool(((out["v7"][0][:, :128] - out["v10"][0][:, :128]).abs() <= 4e-6 * cnt * 8 + 1e-3).all())


def test_kernel_deterministic(kernel):
    from alink_amd.ops import kmeans as K
    X, C = _data(200000, 100, seed=3)
    a = K.assign_accumulate_hip(X, C)
    b = K.assign_accumulate_hip(X, C)
    assert torch.equal(a, b)


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


@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("n,m", [(1, 3), (33, 40), (65, 1), (20001, 201), (70001, 401)])
def test_nearest_kernel_two_row_groups_identical(n, m, d, monkeypatch):
    """RG = 2 (two 32-row groups per wave iteration) returns exactly the RG = 1 indices and distances, including
    row counts that leave the last wave iteration half or wholly past N."""
    from alink_amd.ops import kmeans as K
    g = torch.Generator(device="cpu").manual_seed(n * 7 + m + d)
    X = (torch.randn(n, d, generator=g) * 2).to("cuda", torch.bfloat16)
    C = (torch.randn(m, d, generator=g) * 2).to("cuda", torch.float64)
    monkeypatch.setattr(K, "NEAREST_RG", 1)
    i1, d1 = K.nearest_hip(X, C)
    monkeypatch.setattr(K, "NEAREST_RG", 2)
    i2, d2 = K.nearest_hip(X, C)
    assert torch.equal(i1, i2) and torch.equal(d1, d2)
    c1 = K.nearest_counts_hip(X, C)
    for lag in ("0", "1"):        # the lag-1 MFMA / argmax pipeline (A/B) too
        monkeypatch.setenv("ALINK_KMEANS_NEAREST_LAG", lag)
        for rg in ((1, 2, 3, 4) if d == 128 else (1, 2)):     # RG 3 / 4 (no fragment prefetch) at D = 128
            monkeypatch.setattr(K, "NEAREST_RG", rg)
            i3, d3 = K.nearest_hip(X, C)
            assert torch.equal(i1, i3) and torch.equal(d1, d3)
            assert torch.equal(c1, K.nearest_counts_hip(X, C))


@pytest.mark.parametrize("d", [64, 128, 256])
@pytest.mark.parametrize("n,m", [(1, 1), (33, 40), (4097, 256), (70001, 201), (20001, 300)])
def test_nearest_counts_equal_bincount_of_nearest(n, m, d, monkeypatch):
    """Counts mode of the nearest kernel (k-means|| candidate weights in one pass) == bincount of nearest_hip's
    indices, including a NaN row (counted nowhere by the kernel) and m > 256 (two-step fallback): exactly with the
    default exact argmax; with the packed v_max3 argmax (A/B, ALINK_KMEANS_COUNTS_PACKED=1) every row is still
    counted once and only near-ties (scores equal in their top 25 bits) may move between candidates."""
    from alink_amd.ops import kmeans as K
    g = torch.Generator(device="cpu").manual_seed(n + 3 * m + d)
    X = (torch.randn(n, d, generator=g) * 2).to("cuda", torch.bfloat16)
    C = (torch.randn(m, d, generator=g) * 2).to("cuda", torch.float64)
    want = torch.bincount(K.nearest_hip(X, C)[0].long(), minlength=m)
    monkeypatch.setenv("ALINK_KMEANS_COUNTS_PACKED", "0")
    got = K.nearest_counts_hip(X, C)
    assert got.dtype == torch.int64 and torch.equal(got, want)
    monkeypatch.setenv("ALINK_KMEANS_COUNTS_PACKED", "1")
    pk = K.nearest_counts_hip(X, C)
    assert int(pk.sum()) == n and int((pk - want).abs().sum()) <= max(2, n // 5000)
    for flag in ("0", "1"):
        monkeypatch.setenv("ALINK_KMEANS_COUNTS_PACKED", flag)
        if n > 1 and m <= 256:
            Xn = X.clone()
            Xn[n // 2] = float("nan")
            got = K.nearest_counts_hip(Xn, C)
            assert int(got.sum()) == n - 1


@pytest.mark.parametrize("d", [64, 128, 256])
@pytest.mark.parametrize("n", [1, 3, 17, 4099, 300_001])
def test_first_cost_kernel_matches_fp64(n, d):
    """kmeans_cost1_kernel (the first k-means|| cost pass) vs the fp64 distance to the bf16 center; a row equal to
    the center costs exactly 0."""
    from alink_amd.ops import kmeans as K
    g = torch.Generator(device="cpu").manual_seed(n + d)
    X = (torch.randn(n, d, generator=g) * 3).to("cuda", torch.bfloat16)
    c = X[n // 2].double() + 0.0
    got = K.cost1_hip(X, c)
    ref = ((X.double() - c.to(torch.bfloat16).double()[None, :]) ** 2).sum(1).sqrt()
    assert got.dtype == torch.float64 and got.shape == (n,)
    torch.testing.assert_close(got, ref, rtol=2e-6, atol=1e-6)
    assert float(got[n // 2]) == 0.0
    got2, ws = K.cost1_hip(X, c, with_sum=True)        # per-wave sums: the same costs, their total, deterministic
    assert torch.equal(got2, got)
    torch.testing.assert_close(ws.sum(), got.sum(), rtol=1e-12, atol=0.0)
    assert torch.equal(ws, K.cost1_hip(X, c, with_sum=True)[1])
    if n > 2:
        X[0, d - 1] = float("nan")
        X[1, 0] = float("inf")
        got = K.cost1_hip(X, c)
        assert float(got[0]) == 0.0 and float(got[1]) == 0.0


def test_nearest_kernel_exact_candidates():
    """k-means|| candidates are rows of X: distance to itself must come out 0 and the index its own."""
    from alink_amd.ops import kmeans as K
    X = torch.randn(5000, 128, device="cuda").to(torch.bfloat16)
    sel = torch.arange(0, 5000, 17, device="cuda")
    idx, d2 = K.nearest_hip(X, X[sel].double())
    assert torch.equal(idx[sel].long(), torch.arange(sel.numel(), device="cuda"))
    assert float(d2[sel].abs().max()) < 1e-2


@pytest.mark.parametrize("d", [1, 7, 8, 16, 31, 64, 65, 128, 200, 256, 300, 512, 700, 1024])
@pytest.mark.parametrize("loss", ["log", "logistic", "square", "hinge", "smooth", "perceptron", "exp", "huber", "svr"])
def test_linear_grad_kernel_matches_fp64_reference(d, loss):
    """csrc/linear.hip fused gradient vs the torch two-GEMV form of the same unary loss (fp64)."""
    from alink_amd.models.linear import objfunc as O
    from alink_amd.ops import linear as lops
    fn = {"log": O.LogLossFunc(), "logistic": O.LogisticLossFunc(), "square": O.SquareLossFunc(),
          "hinge": O.HingeLossFunc(), "smooth": O.SmoothHingeLossFunc(), "perceptron": O.PerceptronLossFunc(),
          "exp": O.ExponentialLossFunc(), "huber": O.HuberLossFunc(0.7), "svr": O.SvrLossFunc(0.2)}[loss]
    g = torch.Generator(device="cpu").manual_seed(d)
    n = 50001 if d <= 256 else 20011
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


@pytest.mark.parametrize("d", [3, 32, 64, 100, 256, 700])
@pytest.mark.parametrize("loss", ["log", "square", "smooth", "huber", "svr"])
def test_linear_search_losses_kernel_matches_fp64(d, loss):
    """K14 fused line-search losses (csrc/linear.hip) vs the torch [n,d]x[d,2] GEMM + elementwise form."""
    from alink_amd.models.linear import objfunc as O
    from alink_amd.ops import linear as lops
    fn = {"log": O.LogLossFunc(), "square": O.SquareLossFunc(), "smooth": O.SmoothHingeLossFunc(),
          "huber": O.HuberLossFunc(0.7), "svr": O.SvrLossFunc(0.2)}[loss]
    g = torch.Generator(device="cpu").manual_seed(d + 7)
    n = 40007
    X = torch.randn(n, d, generator=g, dtype=torch.float64).cuda()
    y = (torch.randint(0, 2, (n,), generator=g) * 2 - 1).double().cuda()
    w = torch.rand(n, generator=g, dtype=torch.float64).cuda()
    coef = (0.3 * torch.randn(d, generator=g, dtype=torch.float64)).cuda()
    dirv = (0.1 * torch.randn(d, generator=g, dtype=torch.float64)).cuda()
    code, prm = lops.loss_code(fn)
    for nsteps, beta in [(5, 0.25), (16, 0.1), (1, 1.0)]:
        got = lops.search_losses_hip(X, y, w, coef, dirv, code, prm, beta, nsteps)
        E = X @ torch.stack([coef, dirv], 1)
        steps = torch.arange(nsteps, dtype=torch.float64, device="cuda")
        etas = E[:, :1] - steps[None, :] * (E[:, 1:2] * beta)
        ref = (fn.loss(etas, y[:, None]) * w[:, None]).sum(0)
        torch.testing.assert_close(got, ref, rtol=1e-10, atol=1e-8)


@pytest.mark.parametrize("k", [1, 37, 100, 128])
def test_fused_centroid_update_matches_torch(k):
    """csrc/kmeans_common.hip kmeans_update: C = sums / counts, max shift vs prev (fp64), empty flag, and the next
    superstep's bf16 operands identical to a fresh prep launch."""
    from alink_amd.ops import kmeans as K
    g = torch.Generator(device="cuda").manual_seed(k)
    buf = torch.randn(k, 129, device="cuda", dtype=torch.float64, generator=g) * 100
    buf[:, 128] = torch.randint(1, 1000, (k,), device="cuda", generator=g).double()
    prev = torch.randn(k, 128, device="cuda", dtype=torch.float64, generator=g)
    C, shift, empty = K.update_centroids_hip(buf, prev, hysteresis=False)
    ref = buf[:, :128] / buf[:, 128:]
    torch.testing.assert_close(C, ref, rtol=0, atol=0)
    assert not empty
    assert abs(shift - float((ref - prev).norm(dim=1).max())) <= 1e-12 * max(1.0, shift)
    cpad, ninit = K.prepare_centroids(C, C.device)            # cached: no launch
    cpad2, ninit2 = [t.clone() for t in (cpad, ninit)]
    K._PREPARED.clear()
    cpad3, ninit3 = K.prepare_centroids(C, C.device)          # fresh prep launch
    assert torch.equal(cpad2, cpad3) and torch.equal(ninit2, ninit3)
    buf[k // 2, 128] = 0.0
    _, _, empty = K.update_centroids_hip(buf, None, hysteresis=False)
    assert empty


def test_update_operand_hysteresis():
    """With hysteresis the next-step bf16 operand is held while the fp64 centroid stays within one bf16 ulp of the
    row's largest coordinate,
    and re-rounded otherwise; ninit always matches the operands actually written."""
    from alink_amd.ops import kmeans as K
    k = 50
    g = torch.Generator(device="cuda").manual_seed(3)
    buf = torch.randn(k, 129, device="cuda", dtype=torch.float64, generator=g) * 100
    buf[:, 128] = torch.randint(1, 1000, (k,), device="cuda", generator=g).double()
    C0, _, _ = K.update_centroids_hip(buf, None, hysteresis=False)
    cpad, ninit = K._PREP[C0.device.index]
    held = cpad[:k].clone()
    # nudge every centroid by a quarter ulp of its row's largest operand (within the one-ulp band -> held), and
    # row 0 by 3 such ulps (outside -> re-rounded)
    m = C0.abs().amax(1, keepdim=True).float()
    ulp = torch.ldexp(torch.ones_like(m), torch.frexp(m)[1] - 8).double()
    C1 = C0 + 0.25 * ulp
    C1[0] = C0[0] + 3.0 * ulp[0]
    buf2 = buf.clone()
    buf2[:, :128] = C1 * buf[:, 128:]
    C, _, _ = K.update_centroids_hip(buf2, C0, hysteresis=True)
    cpad, ninit = K._PREP[C.device.index]
    assert torch.equal(cpad[1:k], held[1:])
    assert torch.equal(cpad[0], C[0].float().to(torch.bfloat16))
    f = cpad[:k].float()
    torch.testing.assert_close(ninit[:k], -0.5 * (f * f).sum(1), rtol=1e-6, atol=1e-3)


def test_update_convergence_word_and_skipped_assign():
    """kmeans_update's skip word (an empty cluster, or max shift < tol with prev given) is exactly the host's drop
    test on the returned stats; an assign launch reading a set word leaves the slabs untouched, one reading a
    cleared word equals a plain launch."""
    from alink_amd.ops import kmeans as K
    X, C = _data(100_003, 60, seed=9)
    buf = K.assign_accumulate_hip(X, C)
    prev = (buf[:, :128] / buf[:, 128:]) + 1e-3
    for tol, want in ((1.0, 1), (1e-9, 0)):
        Cn, read = K.update_centroids_hip(buf, prev, deferred=True, hysteresis=False, skip_tol=tol)
        assert read.skip is not None
        shift, empty = read()
        assert not empty and (shift < tol) == bool(want)
        assert int(read.skip.item()) == want
    Cn, read = K.update_centroids_hip(buf, prev, deferred=True, hysteresis=False, skip_tol=1e-9)
    read()
    plain = K.assign_accumulate_hip(X, Cn)
    assert torch.equal(K.assign_accumulate_hip(X, Cn, skip=read.skip), plain)
    bad = buf.clone()
    bad[3, 128] = 0.0
    _, read = K.update_centroids_hip(bad, prev, deferred=True, hysteresis=False, skip_tol=-1.0)
    _, empty = read()
    assert empty and int(read.skip.item()) == 1
    _, read = K.update_centroids_hip(bad, None, deferred=True, hysteresis=False, skip_tol=-1.0)
    _, empty = read()
    assert empty and int(read.skip.item()) == 1
    _, read = K.update_centroids_hip(buf, prev, deferred=True, hysteresis=False, skip_tol=1e9)
    read()
    # bitwise comparison (int32 views): a slab row the kernel never writes (rows >= 16*ceil(k/16)) may hold a NaN
    # pattern, and torch.equal(NaN, NaN) is False even when nothing changed -- the round-5 driver failure
    # (profiles/kmeans_skip_r6.txt).  The slabs are zeroed at allocation now, but the check must not rest on that.
    slab = [t.view(torch.int32).clone() for pair in K._BUF.values() for t in pair]
    out = K.assign_accumulate_hip(X, Cn, skip=read.skip)
    torch.cuda.synchronize()
    after = [t.view(torch.int32) for pair in K._BUF.values() for t in pair]
    for a, b in zip(slab, after):
        diff = (a != b).nonzero()
        assert diff.numel() == 0, f"skipped launch wrote {diff.shape[0]} slab words, first at {diff[0].tolist()}"
    # the reduction reads the same word: a poisoned output buffer stays poisoned
    poison = torch.full((60, 129), 7.0, dtype=torch.float64, device="cuda")
    L = K._lib.require()
    key = next(iter(K._BUF))
    s, sc = K._BUF[key]
    assert L.alink_kmeans_reduce_slabs2(s.data_ptr(), sc.data_ptr(), key[1], 60, poison.data_ptr(),
                                        read.skip.data_ptr(), K._lib.stream_ptr(poison.device)) == 0
    torch.cuda.synchronize()
    assert bool((poison == 7.0).all()) and out.shape == (60, 129)


def test_slab_tail_nan_garbage_is_not_a_write():
    """The round-5 failure mode, reproduced deliberately: NaN bits in the never-written tail of a slab make
    torch.equal report a change although no word changed; the bitwise view does not."""
    from alink_amd.ops import kmeans as K
    X, C = _data(20_011, 60, seed=4)
    K.assign_accumulate_hip(X, C)
    grid = K._GRID[(K.kernel_version(60), X.shape[0], None, X.device.index)]
    s, _ = K._BUF[(X.device.index, grid)]
    s[:, 64:].fill_(float("nan"))           # rows >= 16*ceil(60/16) = 64 are never written by v10 for k = 60
    before = s.clone()
    K.assign_accumulate_hip(X, C)
    torch.cuda.synchronize()
    assert not torch.equal(before, s)        # NaN != NaN
    assert torch.equal(before[:, 64:].view(torch.int32), s[:, 64:].view(torch.int32))
    s[:, 64:].zero_()


def test_fused_update_host_compaction_equals_generic_path(monkeypatch):
    """An empty cluster (a far-away initial centroid) is compacted by the fused update path on the host; the model
    and the superstep count equal the generic torch update path's on the same assign kernels."""
    from alink_amd import useLocalEnv
    from alink_amd.models.clustering.kmeans import train_kmeans
    from alink_amd.ops import kmeans as K
    env = useLocalEnv(1, device="cuda:0")
    g = torch.Generator(device="cuda").manual_seed(11)
    k = 24
    centers = torch.randn(k, 128, device="cuda", generator=g) * 4
    lab = torch.randint(0, k, (200_000,), device="cuda", generator=g)
    X = (centers[lab] + torch.randn(lab.numel(), 128, device="cuda", generator=g)).to(torch.bfloat16)
    init = (centers + 0.5 * torch.randn(k, 128, device="cuda", generator=g)).double()
    init[5] = 1e4                       # attracts no row: emptied at the first update
    monkeypatch.setenv("ALINK_KMEANS_HYSTERESIS", "0")     # the generic path re-quantises every step
    a, qa = train_kmeans(X, k, 15, 1e-4, "EUCLIDEAN", "RANDOM", 2, "v", env, init_centroids=init)
    monkeypatch.setattr(K, "update_supported", lambda buf: False)
    b, qb = train_kmeans(X, k, 15, 1e-4, "EUCLIDEAN", "RANDOM", 2, "v", env, init_centroids=init)
    assert len(qa.stats) == len(qb.stats)
    assert [list(r) for r in a] == [list(r) for r in b]
    assert int(qa.final_contexts[0].getObj("k")) == k - 1


def test_speculative_next_step_launch_gives_identical_model():
    """KMeansUpdateCentroids queues the next superstep's assign kernel before reading the update stats; the
    trained model must be bit-identical to a run without speculation (sync after every step), incl. a run that
    converges early (the queued kernel of the step after convergence is dropped)."""
    from alink_amd import useLocalEnv
    from alink_amd.models.clustering.kmeans import train_kmeans
    env = useLocalEnv(1, device="cuda:0")
    g = torch.Generator(device="cuda").manual_seed(5)
    k = 40
    centers = torch.randn(k, 128, device="cuda", generator=g) * 4
    lab = torch.randint(0, k, (400_000,), device="cuda", generator=g)
    X = (centers[lab] + torch.randn(lab.numel(), 128, device="cuda", generator=g)).to(torch.bfloat16)
    init = (centers + 0.5 * torch.randn(k, 128, device="cuda", generator=g)).double()
    for tol in (-1.0, 1e-4):
        a, qa = train_kmeans(X, k, 12, tol, "EUCLIDEAN", "RANDOM", 2, "v", env, init_centroids=init)
        b, qb = train_kmeans(X, k, 12, tol, "EUCLIDEAN", "RANDOM", 2, "v", env, init_centroids=init,
                             sync_steps=range(100))
        assert len(qa.stats) == len(qb.stats)
        assert [list(r) for r in a] == [list(r) for r in b]


@pytest.mark.parametrize("n,k,grid", [(300001, 100, None), (49157, 97, 3), (4097, 16, None), (129, 50, 1),
                                      (70001, 112, 5)])
def test_v10_serpentine_reverse_order(n, k, grid):
    """The serpentine (reverse) walk visits the same rows: identical assignments and counts, sums equal up to the
    fp32 summation order; and the reverse launch is itself deterministic."""
    from alink_amd.ops import kmeans as K
    X, C = _data(n, k, seed=21)
    fa = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    ra = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    f = K.assign_accumulate_hip(X, C, grid=grid, assign_out=fa)
    r = K.assign_accumulate_hip(X, C, grid=grid, assign_out=ra, reverse=True)
    r2 = K.assign_accumulate_hip(X, C, grid=grid, reverse=True)
    assert K.kernel_version(k) == "v10"
    assert torch.equal(fa, ra)
    assert torch.equal(f[:, 128], r[:, 128])
    assert torch.equal(r, r2)
    _own_assignment_check(X, C, r, ra, k)


@pytest.mark.parametrize("n,first_row,rnd", [(1, 0, 0), (1000, 0, 0), (300001, 12345, 1), (2_000_003, 10**9, 3)])
def test_par_pick_kernel_equals_torch_draw(n, first_row, rnd):
    """k-means|| oversampling picks of the HIP kernel are bit-for-bit the torch expression's (same splitmix64
    uniforms of the global row index, same fp64 threshold compare), including more picks than the first cap."""
    from alink_amd.models.clustering import kmeans as km
    from alink_amd.ops import kmeans as K
    g = torch.Generator(device="cpu").manual_seed(n)
    cost = (torch.rand(n, generator=g, dtype=torch.float64) * 3).cuda()
    for thre in (200.0 / float(cost.sum()), 9000.0 / float(cost.sum())):
        got = K.par_pick_hip(cost, first_row, km._round_key(7, rnd), thre)
        u = km._row_uniform(first_row, n, 7, rnd, cost.device)
        ref = torch.nonzero(u < cost * thre).reshape(-1)
        assert torch.equal(got, ref)


def test_local_kmeans_device_resident_equals_host_loop_on_gpu():
    """The device-resident k-means++ seeding + Lloyd on the GPU agrees with the host loop and is deterministic."""
    import numpy as np  # noqa: F401
    from alink_amd.models.clustering import kmeans as km
    from tests.test_kmeans import _host_loop_local_kmeans
    g = torch.Generator(device="cpu").manual_seed(5)
    X = torch.randn(230, 128, generator=g, dtype=torch.float64).cuda()
    w = torch.randint(1, 50, (230,), generator=g).to(torch.float64).cuda()
    got = km._local_kmeans(X, w, 100, "EUCLIDEAN", seed=1)
    # the host loop's device index_add_ sums in atomic order: equal up to fp64 rounding
    assert torch.allclose(got, _host_loop_local_kmeans(X, w, 100, "EUCLIDEAN", seed=1), rtol=1e-12, atol=1e-12)
    assert torch.equal(got, km._local_kmeans(X, w, 100, "EUCLIDEAN", seed=1))          # deterministic


@pytest.mark.parametrize("n,k", [(2, 2), (230, 100), (1000, 300), (4096, 50)])
def test_seed_ref_kernel_equals_torch_loop(n, k):
    """The one-workgroup seeding kernel picks the same candidates as the per-pick torch loop (run on the host)."""
    import numpy as np
    from alink_amd.models.clustering import kmeans as km
    g = torch.Generator(device="cpu").manual_seed(n)
    S = torch.randn(n, 16, generator=g, dtype=torch.float64)
    D = km.pairwise_distance(S, S, "EUCLIDEAN")
    w = torch.randint(1, 30, (n,), generator=g).to(torch.float64)
    a = km._seed_reference_device(D.cuda(), w.cuda(), k, np.random.default_rng(4), 0)
    b = km._seed_reference_device(D, w, k, np.random.default_rng(4), 0)
    assert a is not None and b is not None
    assert torch.equal(a.cpu(), b)


@pytest.mark.parametrize("n,k", [(64, 30), (700, 120), (4096, 40)])
def test_seed_ref_kernel_equals_host_on_ties_and_wide_weights(n, k):
    """Tied distances (integer grid points), zero weights (flat cumulative runs) and weights over 18 decades (sums
    whose rounding depends on the order): the kernel's sequential prefix picks exactly the host torch.cumsum's."""
    import numpy as np
    from alink_amd.models.clustering import kmeans as km
    g = torch.Generator(device="cpu").manual_seed(n + k)
    S = torch.randint(0, 3, (n, 4), generator=g).to(torch.float64)
    D = km.pairwise_distance(S, S, "EUCLIDEAN")
    w = torch.pow(10.0, torch.randint(-3, 16, (n,), generator=g).to(torch.float64))
    w[torch.rand(n, generator=g) < 0.3] = 0.0
    for seed in range(3):
        a = km._seed_reference_device(D.cuda(), w.cuda(), k, np.random.default_rng(seed), 0)
        b = km._seed_reference_device(D, w, k, np.random.default_rng(seed), 0)
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a.cpu(), b)


@pytest.mark.parametrize("n,k", [(1, 1), (201, 100), (700, 120), (4096, 40)])
def test_seed_ref_kernel_first_pick(n, k):
    """idx0 < 0: the kernel also makes the first pick, as the host does (searchsorted over the SEQUENTIAL cumulative
    weights, side left), then the same picks as with that index given."""
    import numpy as np
    from alink_amd.models.clustering import kmeans as km
    from alink_amd.ops import kmeans as K
    g = torch.Generator(device="cpu").manual_seed(n + 7)
    S = torch.randint(0, 4, (n, 5), generator=g).to(torch.float64)
    D = km.pairwise_distance(S, S, "EUCLIDEAN").cuda()
    w = torch.pow(10.0, torch.randint(-3, 16, (n,), generator=g).to(torch.float64))
    w[torch.rand(n, generator=g) < 0.2] = 0.0
    w[0] = 1.0
    for seed in range(4):
        rng = np.random.default_rng(seed)
        r0 = float(rng.random())
        U = torch.as_tensor(rng.random(max(k - 1, 0)), dtype=torch.float64)
        cum = np.cumsum(w.numpy())
        idx = int(min(np.searchsorted(cum, r0 * cum[-1], side="left"), n - 1))
        a, ma = K.seed_ref_hip(D, w.cuda(), U.cuda(), k, idx0=-1, r0=r0)
        b, mb = K.seed_ref_hip(D, w.cuda(), U.cuda(), k, idx0=idx)
        assert int(a[0]) == idx
        assert torch.equal(a, b) and torch.equal(ma, mb)


def _lloyd_case(n, d, k, seed, dup=False):
    g = torch.Generator(device="cpu").manual_seed(seed)
    X = torch.randn(n, d, generator=g, dtype=torch.float64) * 3
    if dup:
        X = torch.cat([X[: n // 2]] * 2 + [X[: n - 2 * (n // 2)]])
    # weights >= 1 (k-means|| candidate counts): zero weights plus refills make exact-copy centroids whose
    # distances tie at the rounding level, which two summation orders may break differently
    w = torch.randint(1, 40, (n,), generator=g).to(torch.float64)
    return X.cuda(), w.cuda()


@pytest.mark.parametrize("n,d,k,dup", [(201, 128, 100, False), (230, 128, 100, True), (600, 16, 150, False),
                                       (4096, 8, 64, False), (65, 3, 64, False), (129, 256, 20, True)])
def test_local_kmeans_kernels_equal_torch_path(n, d, k, dup, monkeypatch):
    """The one-workgroup seeding + Lloyd kernels (ALINK_KMEANS_LOCAL_KERNEL, default on) return the torch device
    path's centroids: the same picks (fallback to the torch path when a pick meets an all-zero total), the same
    assignments each iteration, sums equal up to fp64 summation order; empty clusters (zero weights, duplicated
    rows) refilled from the same generator draws; run-to-run deterministic."""
    from alink_amd.models.clustering import kmeans as km
    from alink_amd.ops import kmeans as K
    monkeypatch.delenv("ALINK_KMEANS_SEEDING", raising=False)
    X, w = _lloyd_case(n, d, k, seed=n + k, dup=dup)
    assert K.local_lloyd_ok(X, k)
    monkeypatch.setenv("ALINK_KMEANS_LOCAL_KERNEL", "0")
    ref = km._local_kmeans(X, w, k, "EUCLIDEAN", seed=2)
    monkeypatch.setenv("ALINK_KMEANS_LOCAL_KERNEL", "1")
    got = km._local_kmeans(X, w, k, "EUCLIDEAN", seed=2)
    assert torch.allclose(got, ref, rtol=1e-11, atol=1e-11)
    assert torch.equal(got, km._local_kmeans(X, w, k, "EUCLIDEAN", seed=2))


def test_local_lloyd_kernel_iterations_and_empty_exit():
    """The Lloyd kernel stops at the first empty cluster (live flags mark it, centroid kept), and max_iter = 1
    runs exactly one iteration whose assignment is the torch argmin of the start centroids."""
    from alink_amd.models.clustering import kmeans as km
    from alink_amd.ops import kmeans as K
    X, w = _lloyd_case(300, 32, 40, seed=5)
    C0 = X[:40].clone()
    C0[7] = 1e3                                   # far away: nobody's nearest -> empty in iteration 1
    C, a, st, live = K.local_lloyd_hip(X, w, 40, C=C0.clone(), max_iter=30)
    st = st.cpu().tolist()
    assert st[0] == 1 and st[1] == 1 and st[2] == 1 and st[3] == 0
    assert int(live[7]) == 0 and int(live.sum()) == 39
    assert torch.equal(C[7], C0[7])
    assert torch.equal(a, km.pairwise_distance(X, C0, "EUCLIDEAN").argmin(1))
    C1, a1, st1, _ = K.local_lloyd_hip(X, w, 40, C=X[:40].clone(), max_iter=1)
    assert st1.cpu().tolist()[0] == 1
    assert torch.equal(a1, km.pairwise_distance(X, X[:40], "EUCLIDEAN").argmin(1))


def test_local_lloyd_kernel_non_finite_falls_back(monkeypatch):
    """A non-finite candidate: the kernel writes nothing and flags it; _local_kmeans takes the torch path with the
    generator untouched (same result as the kernel switched off)."""
    from alink_amd.models.clustering import kmeans as km
    from alink_amd.ops import kmeans as K
    X, w = _lloyd_case(120, 16, 10, seed=9)
    X[17, 3] = float("nan")
    _, _, st, _ = K.local_lloyd_hip(X, w, 10, C=X[20:30].clone(), max_iter=5)
    assert st.cpu().tolist()[3] == 1
    monkeypatch.setenv("ALINK_KMEANS_LOCAL_KERNEL", "0")
    ref = km._local_kmeans(X, w, 10, "EUCLIDEAN", seed=1)
    monkeypatch.setenv("ALINK_KMEANS_LOCAL_KERNEL", "1")
    got = km._local_kmeans(X, w, 10, "EUCLIDEAN", seed=1)
    assert torch.equal(torch.nan_to_num(got, nan=7.0), torch.nan_to_num(ref, nan=7.0))


@pytest.mark.parametrize("pool", [0.0, 0.1, 0.5, 1.0])
@pytest.mark.parametrize("n,k,grid", [(300001, 100, None), (49157, 97, 3), (4097, 16, None), (129, 50, 1),
                                      (1000003, 112, 7), (70, 8, 2)])
def test_v10_work_stealing_tail(n, k, grid, pool, monkeypatch):
    """DYN: static chunks plus a pool of 16-tile chunks claimed from a device counter — every tile exactly once
    (identical assignments and counts to the static split, sums to fp32 order), in both walk directions, and the
    two alternating counters reset themselves across launches."""
    from alink_amd.ops import kmeans as K
    X, C = _data(n, k, seed=31)
    monkeypatch.setattr(K, "V10_POOL", 0.0)
    sa = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    ref = K.assign_accumulate_hip(X, C, grid=grid, assign_out=sa)
    monkeypatch.setattr(K, "V10_POOL", pool)
    for rev in (False, True, False, True):
        da = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        got = K.assign_accumulate_hip(X, C, grid=grid, assign_out=da, reverse=rev)
        assert torch.equal(da, sa)
        assert torch.equal(got[:, 128], ref[:, 128])
        _own_assignment_check(X, C, got, da, k)


_PFD_CASES = [(300001, 100, None), (49157, 97, 3), (4097, 16, None), (129, 50, 1), (70001, 112, 5)]


def _pfd_identity_check():
    """Runs in a child process on the KM10_PFD=1 variant library (ALINK_HIP_LIB): every prefetch distance returns
    bit-identical sums, counts and ids to distance 0, forward and serpentine."""
    from alink_amd.ops import kmeans as K
    for n, k, grid in _PFD_CASES:
        X, C = _data(n, k, seed=31)
        out = {}
        for v in ("0", "1", "4", "12"):
            os.environ["ALINK_KMEANS_V10_PFD"] = v
            ids = torch.full((n,), -1, dtype=torch.int32, device="cuda")
            f = K.assign_accumulate_hip(X, C, grid=grid, assign_out=ids)
            r = K.assign_accumulate_hip(X, C, grid=grid, reverse=True)
            torch.cuda.synchronize()
            out[v] = (f.view(torch.int64).clone(), r.view(torch.int64).clone(), ids.clone())
        for v in ("1", "4", "12"):
            assert all(torch.equal(a, b) for a, b in zip(out["0"], out[v])), (n, k, grid, v)
    print("PFD_IDENTICAL_OK")


def test_v10_l2_prefetch_identical():
    """ALINK_KMEANS_V10_PFD (the L2 prefetch A/B, compiled only into variants/libalink_hip_pfd.so by
    tools/build_kmeans_variants.sh pfd -- the default build compiles it out): the prefetch loads (LDS-DMA into a
    sink, 5 loads per staged tile in the vmcnt arithmetic) change no result.  Run in a child process because the
    kernel library is loaded once per process."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "variants", "libalink_hip_pfd.so")
    if not os.path.exists(lib):
        pytest.skip("variants/libalink_hip_pfd.so not built (tools/build_kmeans_variants.sh pfd)")
    env = dict(os.environ, ALINK_HIP_LIB=lib, PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", "import tests.test_kmeans_kernel_gpu as t; t._pfd_identity_check()"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "PFD_IDENTICAL_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
