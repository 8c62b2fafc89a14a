"""Collapsed-Gibbs LDA sweep HIP kernel (ops/csrc/lda.hip) against the torch [T, K] formula with the same uniforms."""
import numpy as np
import pandas as pd
import pytest
import torch

from alink_amd.ops import lda as L

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("K", [1, 7, 100, 300])
def test_gibbs_kernel_matches_torch_formula(K, variant):
    g = torch.Generator(device="cuda").manual_seed(K)
    D, V, T = 50, 80, 5000
    d_tok = torch.randint(0, D, (T,), device="cuda", generator=g)
    w_tok = torch.randint(0, V, (T,), device="cuda", generator=g)
    z = torch.randint(0, K, (T,), device="cuda", generator=g)
    nd = torch.bincount(d_tok * K + z, minlength=D * K).reshape(D, K)
    nw = torch.bincount(w_tok * K + z, minlength=V * K).reshape(V, K)
    nk = nw.sum(0).double()
    alpha, beta = 50.0 / K + 1, 1.01
    u = torch.rand(T, device="cuda", generator=g, dtype=torch.float64)
    got = L.gibbs_sweep(d_tok, w_tok, z, nd, nw, nk, alpha, beta, V, u, variant=variant)
    own = torch.nn.functional.one_hot(z, K).double()
    p = (nd.double()[d_tok] - own + alpha) * (nw.double()[w_tok] - own + beta) / (nk[None, :] - own + V * beta)
    cum = torch.cumsum(p, 1)
    ref = torch.searchsorted(cum, (u * cum[:, -1])[:, None]).squeeze(1).clamp(max=K - 1)
    agree = (got == ref).double().mean().item()
    assert agree > 0.999, agree


def test_lda_em_trains_on_cuda():
    from alink_amd import BatchOperator, LdaTrainBatchOp, useLocalEnv
    rng = np.random.default_rng(1)
    a = [f"a{i}" for i in range(10)]
    b = [f"b{i}" for i in range(10)]
    docs = [" ".join(rng.choice(a if i % 2 else b, 20)) for i in range(200)]
    useLocalEnv(1, device="cuda:0")
    src = BatchOperator.fromDataframe(pd.DataFrame({"doc": docs}), schemaStr="doc string")
    m = LdaTrainBatchOp().setSelectedCol("doc").setTopicNum(2).setMethod("em").setNumIter(30) \
        .linkFrom(src)
    rows = m.collect()
    assert len(rows) > 0


@pytest.mark.parametrize("K", [5, 64, 100, 256])
def test_online_estep_kernel_matches_torch(K):
    """HIP online-VB E-step (one wave per document, all iterations in registers) == the torch loop (on the
    host) for gamma, expElogtheta and per-token phinorm."""
    from alink_amd.models.clustering import lda as M
    g = torch.Generator().manual_seed(K)
    D, V = 300, 400
    lens = torch.randint(1, 40, (D,), generator=g)
    doc = torch.repeat_interleave(torch.arange(D), lens)
    word = torch.randint(0, V, (doc.numel(),), generator=g)
    cts = torch.randint(1, 4, (doc.numel(),), generator=g).double()
    lam = torch.distributions.Gamma(100.0, 100.0).sample((K, V)).double()
    ebT = torch.exp(M._dir_exp(lam)).T.contiguous()
    alpha = torch.full((K,), 1.0 / K, dtype=torch.float64)
    g0 = torch.distributions.Gamma(100.0, 100.0).sample((D, K)).double()
    ref = M.e_step(doc, word, cts, D, ebT, alpha, g0)
    got = M.e_step(doc.cuda(), word.cuda(), cts.cuda(), D, ebT.cuda(), alpha.cuda(), g0.cuda())
    # a document whose mean gamma change sits on the convergence threshold may stop one iteration apart on
    # the two paths (different fp64 summation order): that moves its values by ~1e-7 relative
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a.cpu().numpy(), b.numpy(), rtol=2e-6, atol=1e-10)
