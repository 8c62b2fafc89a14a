"""Fused score + top-K HIP kernel (ops/csrc/topk.hip) against a plain fp32 torch reference."""
import numpy as np
import pytest
import torch

from alink_amd.ops import topk as T

pytestmark = pytest.mark.gpu


def _ref(Q, I, K):
    S = (Q.double() @ I.double().T)
    v, i = torch.topk(S, min(K, I.shape[0]), dim=1)
    return v, i


@pytest.mark.parametrize("m,n,r,K", [(1, 5, 3, 4), (130, 1000, 10, 7), (257, 3001, 64, 100), (64, 200, 33, 128),
                                     (300, 70, 16, 128)])
def test_topk_kernel_matches_torch(m, n, r, K):
    g = torch.Generator(device="cuda").manual_seed(m + n)
    Q = torch.randn(m, r, device="cuda", generator=g)
    I = torch.randn(n, r, device="cuda", generator=g)
    st = T.TopKState(m, K, "cuda")
    # two blocks with an id offset: the state carries over between launches
    h = n // 3
    T.merge(st, Q, I[:h], 0, use_kernel=True)
    T.merge(st, Q, I[h:], h, use_kernel=True)
    v, i = T.finish(st)
    torch.cuda.synchronize()
    kk = min(K, n)
    rv, ri = _ref(Q, I, K)
    np.testing.assert_allclose(v[:, :kk].cpu().numpy(), rv.cpu().numpy(), rtol=1e-5, atol=1e-4)
    # ids: the scores the kernel reports must be the true scores of the ids it returns
    S = (Q.double() @ I.double().T)
    got = torch.gather(S, 1, i[:, :kk].long())
    np.testing.assert_allclose(got.cpu().numpy(), rv.cpu().numpy(), rtol=1e-5, atol=1e-4)
    assert bool((i[:, :kk] >= 0).all()) and bool((i[:, kk:] == -1).all())
    for row in i[:, :kk].cpu().numpy():
        assert len(set(row.tolist())) == kk


def test_topk_kernel_equals_fallback_with_ties():
    Q = torch.ones(20, 8, device="cuda")
    I = torch.cat([torch.ones(50, 8), 2 * torch.ones(3, 8)]).cuda()     # 3 winners then 50-way ties
    a = T.TopKState(20, 10, "cuda")
    T.merge(a, Q, I, 0, use_kernel=True)
    b = T.TopKState(20, 10, "cuda")
    T.merge(b, Q, I, 0, use_kernel=False)
    va, ia = T.finish(a)
    vb, ib = T.finish(b)
    assert torch.equal(va, vb)
    assert set(ia[0, :3].tolist()) == {50, 51, 52}


def test_blockwise_topk_single_rank_cuda():
    from alink_amd.parallel.cross import blockwise_topk
    Q = torch.randn(100, 20, device="cuda")
    I = torch.randn(900, 20, device="cuda")
    v, i = blockwise_topk(Q, I, 12, descending=False)
    rv, _ = torch.topk(-(Q @ I.T), 12, dim=1)
    np.testing.assert_allclose(v.cpu().numpy(), (-rv).cpu().numpy(), rtol=1e-5, atol=1e-4)
