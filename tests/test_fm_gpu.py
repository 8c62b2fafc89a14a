"""FM micro-batch HIP kernels (ops/csrc/fm.hip) against the fp64 torch formulas, and FM training on cuda vs CPU."""
import numpy as np
import pandas as pd
import pytest
import torch

from alink_amd.models.common.features import FeatureMatrix
from alink_amd.ops import fm as F

pytestmark = pytest.mark.gpu


def _sparse(n, d, nnz_per_row, seed):
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(0, nnz_per_row + 1, (n,), generator=g)
    crow = torch.zeros(n + 1, dtype=torch.int64)
    crow[1:] = torch.cumsum(lens, 0)
    col = torch.cat([torch.randperm(d, generator=g)[:int(k)] for k in lens]).to(torch.int64)
    val = torch.randn(int(crow[-1]), generator=g, dtype=torch.float64)
    return FeatureMatrix(crow=crow.cuda(), col=col.cuda(), val=val.cuda(), ncols=d)


@pytest.mark.parametrize("k", [1, 10, 64])
def test_fm_forward_and_update_match_torch(k):
    d, n = 300, 257
    fm = _sparse(n, d, 12, k)
    g = torch.Generator(device="cuda").manual_seed(1)
    w = torch.randn(d, dtype=torch.float64, device="cuda", generator=g)
    V = torch.randn(d, k, dtype=torch.float64, device="cuda", generator=g) * 0.1
    y, vx = F.fm_forward(fm, w, V, 0.25)
    rows = fm.row_ids()
    vx_ref = torch.zeros(n, k, dtype=torch.float64, device="cuda").index_add_(0, rows, fm.val[:, None] * V[fm.col])
    v2 = torch.zeros(n, k, dtype=torch.float64, device="cuda").index_add_(0, rows, (fm.val ** 2)[:, None] * V[fm.col] ** 2)
    lin = torch.zeros(n, dtype=torch.float64, device="cuda").index_add_(0, rows, fm.val * w[fm.col])
    y_ref = 0.25 + lin + 0.5 * (vx_ref ** 2 - v2).sum(1)
    torch.testing.assert_close(vx, vx_ref, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(y, y_ref, rtol=1e-12, atol=1e-12)

    gr = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    sw = torch.rand(n, dtype=torch.float64, device="cuda", generator=g)
    sg_w, sg_V = torch.rand_like(w), torch.rand_like(V)
    use = torch.zeros(d, dtype=torch.float64, device="cuda")
    lr, l1, l2 = 0.05, 0.01, 0.02
    # torch reference of one micro-batch update
    cols, vals = fm.col, fm.val
    Vc = V[cols]
    gv = (gr[rows] * vals)[:, None] * (vx_ref[rows] - vals[:, None] * Vc) + l2 * Vc
    sgV_ref = sg_V.clone().index_add_(0, cols, gv * gv)
    V_ref = V - lr * torch.zeros_like(V).index_add_(0, cols, gv) / torch.sqrt(sgV_ref + F.EPS)
    gl = gr[rows] * vals + l1 * w[cols]
    sgw_ref = sg_w.clone().index_add_(0, cols, gl * gl)
    w_ref = w - lr * torch.zeros_like(w).index_add_(0, cols, gl) / torch.sqrt(sgw_ref + F.EPS)
    use_ref = torch.zeros_like(use).index_add_(0, cols, sw[rows])
    F.fm_coord_update(fm, gr, vx, sw, w, sg_w, V, sg_V, use, lr, l1, l2)
    for a, b in ((V, V_ref), (sg_V, sgV_ref), (w, w_ref), (sg_w, sgw_ref), (use, use_ref)):
        torch.testing.assert_close(a, b, rtol=1e-11, atol=1e-12)


def test_fm_train_sparse_cuda_equals_cpu():
    from alink_amd import BatchOperator, FmClassifierTrainBatchOp, useLocalEnv
    rng = np.random.default_rng(3)
    rows = []
    for i in range(400):
        idx = np.sort(rng.choice(50, 5, replace=False))
        rows.append(("$50$" + " ".join(f"{j}:{rng.normal():.4f}" for j in idx), int(rng.random() < 0.5)))
    df = pd.DataFrame(rows, columns=["vec", "label"])
    out = {}
    for dev in ("cpu", "cuda:0"):
        useLocalEnv(1, device=dev)
        src = BatchOperator.fromDataframe(df, schemaStr="vec string, label int")
        m = FmClassifierTrainBatchOp().setVectorCol("vec").setLabelCol("label").setNumEpochs(3).setNumFactor(8) \
            .setLearnRate(0.05).linkFrom(src)
        out[dev] = [list(r) for r in m.collect()]
    assert len(out["cpu"]) == len(out["cuda:0"])
    for a, b in zip(out["cpu"], out["cuda:0"]):
        if isinstance(a[1], str) and a[1].startswith("{") and '"factors"' in a[1]:
            import json
            fa, fb = json.loads(a[1]), json.loads(b[1])
            np.testing.assert_allclose(np.array(fa["factors"]), np.array(fb["factors"]), rtol=1e-8, atol=1e-10)
