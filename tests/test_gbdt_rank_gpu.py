"""GBDT ranking gradients on the GPU (``ops/csrc/gbdt_rank.hip``) against the host C++ transcription of the
reference loop, and a ranking model trained on the GPU against the CPU-trained one."""
import numpy as np
import pytest
import torch

from tests.test_gbdt_rank import _queries, _rank_frame, _reference_grad

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("algo", [2, 3, 4])
@pytest.mark.parametrize("nq,max_len", [(300, 12), (7, 700), (1, 1), (2, 3000)])
def test_rank_kernel_matches_host(algo, nq, max_len):
    from alink_amd.ops import elementwise as ew
    pred, gain, offsets = _queries(nq=nq, seed=nq + max_len, max_len=max_len)
    args = (torch.from_numpy(gain), None, torch.from_numpy(offsets), algo)
    host = ew.gbdt_rank_stats(torch.from_numpy(pred), *args)
    dev = ew.gbdt_rank_stats(torch.from_numpy(pred).cuda(), torch.from_numpy(gain).cuda(), None,
                             torch.from_numpy(offsets).cuda(), algo).cpu()
    assert torch.allclose(dev[:, 1], host[:, 1], rtol=1e-5, atol=1e-6)
    assert torch.allclose(dev[:, 2], host[:, 2], rtol=1e-5, atol=1e-6)
    if max_len <= 12:
        g_ref, _ = _reference_grad(pred, gain, offsets, algo)
        np.testing.assert_allclose(dev[:, 1].numpy(), g_ref, rtol=2e-6, atol=1e-7)


def test_rank_kernel_weights_and_deterministic():
    from alink_amd.ops import elementwise as ew
    pred, gain, offsets = _queries(nq=50, seed=9)
    w = torch.rand(len(pred)).cuda()
    a = ew.gbdt_rank_stats(torch.from_numpy(pred).cuda(), torch.from_numpy(gain).cuda(), w,
                           torch.from_numpy(offsets).cuda(), 2)
    b = ew.gbdt_rank_stats(torch.from_numpy(pred).cuda(), torch.from_numpy(gain).cuda(), None,
                           torch.from_numpy(offsets).cuda(), 2)
    assert torch.equal(a[:, 1], b[:, 1] * w)
    assert torch.equal(a, ew.gbdt_rank_stats(torch.from_numpy(pred).cuda(), torch.from_numpy(gain).cuda(), w,
                                             torch.from_numpy(offsets).cuda(), 2))


@pytest.mark.parametrize("algo", [2, 4])
def test_rank_training_gpu_equals_cpu(algo):
    from alink_amd import BatchOperator, GbdtRegTrainBatchOp, GbdtRegPredictBatchOp, useLocalEnv
    df = _rank_frame(nq=40)
    out = {}
    for dev in ("cpu", "cuda:0"):
        useLocalEnv(1, device=dev)
        src = BatchOperator.fromDataframe(df, schemaStr="f0 double, f1 double, f2 double, qid int, rel double")
        model = GbdtRegTrainBatchOp(algoType=algo).setFeatureCols(["f0", "f1", "f2"]).setLabelCol("rel") \
            .setGroupCol("qid").setNumTrees(6).setMaxDepth(3).setMinSamplesPerLeaf(5).linkFrom(src)
        out[dev] = GbdtRegPredictBatchOp().setPredictionCol("s").linkFrom(model, src).collectToDataframe()["s"].values
    useLocalEnv(1)
    np.testing.assert_allclose(out["cuda:0"], out["cpu"], rtol=1e-4, atol=1e-4)
