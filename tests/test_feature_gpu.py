"""Feature hot-path kernels (ops/csrc/feature.hip: murmur3 K26, CSR assembler K24/K25) vs the host paths, and
the FeatureHasher / OneHot / VectorAssembler operators end to end in a GPU environment."""
import numpy as np
import pandas as pd
import pytest
import torch

pytestmark = pytest.mark.gpu


def _strings(rng, n):
    alpha = list("abcXYZ019_=-") + ["é", "中", "文", "\U0001F600"]
    return ["".join(rng.choice(alpha, size=int(rng.integers(0, 41)))) for _ in range(n)]


@pytest.mark.parametrize("prefix", ["", "c", "col=", "ab=", "中="])
@pytest.mark.parametrize("nf", [200, 262144, 2 ** 30 + 7])
def test_murmur3_gpu_bitexact_with_host(prefix, nf):
    from alink_amd.ops import _lib
    from alink_amd.ops.feature import murmur3_index
    from alink_amd.models.feature.encoders import murmur3_index as host
    assert _lib.available()
    rng = np.random.default_rng(len(prefix) + nf % 97)
    s = _strings(rng, 20000) + ["", "a", "ab", "abc"]
    got = murmur3_index(s, nf, prefix=prefix, device="cuda").cpu().numpy()
    ref = np.asarray(host([prefix + x for x in s], nf), dtype=np.int64)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("m", [1, 5, 33, 64])
def test_csr_assemble_gpu_matches_host(m):
    from alink_amd.ops.feature import csr_assemble
    rng = np.random.default_rng(m)
    n, size = 20000, 50                       # small index range -> many duplicate indices per row
    idx = torch.from_numpy(rng.integers(0, size, size=(m, n)))
    val = torch.from_numpy(rng.normal(size=(m, n)))
    valid = torch.from_numpy(rng.random((m, n)) < 0.8)
    ref = csr_assemble(idx, val, valid, size)
    got = csr_assemble(idx.cuda(), val.cuda(), valid.cuda(), size)
    assert torch.equal(got.crow.cpu(), ref.crow)
    assert torch.equal(got.col.cpu(), ref.col)
    np.testing.assert_allclose(got.val.cpu().numpy(), ref.val.numpy(), rtol=1e-12, atol=1e-12)
    cols = got.col.cpu().numpy()
    crow = got.crow.cpu().numpy()
    for r in range(0, n, 997):
        seg = cols[crow[r]:crow[r + 1]]
        assert np.all(np.diff(seg) > 0)       # sorted, unique


def _d4():
    from alink_amd import BatchOperator
    D4 = [(1.1, True, 2, "A"), (1.1, False, 2, "B"), (1.1, True, 1, "B"), (2.2, True, 1, "A")]
    df = pd.DataFrame({"double": [r[0] for r in D4], "bool": [r[1] for r in D4], "number": [r[2] for r in D4],
                       "str": [r[3] for r in D4]})
    return BatchOperator.fromDataframe(df, schemaStr="double double, bool boolean, number int, str string")


def test_feature_hasher_doc_on_gpu_env():
    from alink_amd import useLocalEnv, FeatureHasherBatchOp
    from alink_amd.common.linalg import SparseBlock, VectorUtil
    useLocalEnv(1, device="cuda:0")
    op = FeatureHasherBatchOp().setSelectedCols(["double", "bool", "number", "str"]).setOutputCol("output") \
        .setNumFeatures(200).linkFrom(_d4())
    col = op.getOutputTable().col("output").values
    assert isinstance(col, SparseBlock) and col.device.type == "cuda"
    got = [VectorUtil.toString(r[4]) for r in op.collect()]
    assert got == ["$200$13:2.0 38:1.1 45:1.0 195:1.0", "$200$13:2.0 30:1.0 38:1.1 76:1.0",
                   "$200$13:1.0 38:1.1 76:1.0 195:1.0", "$200$13:1.0 38:2.2 45:1.0 195:1.0"]


def test_one_hot_doc_on_gpu_env():
    from alink_amd import useLocalEnv, OneHotTrainBatchOp, OneHotPredictBatchOp
    from alink_amd.common.linalg import VectorUtil
    useLocalEnv(1, device="cuda:0")
    src = _d4()
    onehot = OneHotTrainBatchOp().setSelectedCols(["double", "bool", "number", "str"]).setDiscreteThresholds(2)
    pred = OneHotPredictBatchOp().setSelectedCols(["double", "bool"]).setEncode("ASSEMBLED_VECTOR") \
        .setOutputCols(["pred"]).setDropLast(False)
    out = pred.linkFrom(onehot.linkFrom(src), src).collect()
    assert [VectorUtil.toString(r[4]) for r in out] == ["$6$0:1.0 3:1.0", "$6$0:1.0 5:1.0", "$6$0:1.0 3:1.0",
                                                         "$6$2:1.0 3:1.0"]


def test_hashed_features_into_vector_assembler_and_lr_on_gpu():
    """FeatureHasher (GPU SparseBlock) -> VectorAssembler with a numeric column -> LR train: the whole chain
    stays columnar on the device and matches the CPU environment."""
    from alink_amd import (useLocalEnv, BatchOperator, FeatureHasherBatchOp, VectorAssemblerBatchOp,
                           LogisticRegressionTrainBatchOp)
    from alink_amd.common.mlenv import resetEnv
    rng = np.random.default_rng(0)
    n = 4000
    df = pd.DataFrame({"a": rng.choice(["x", "y", "z", "w"], n), "b": rng.choice([str(i) for i in range(50)], n),
                       "c": rng.normal(size=n)})
    df["label"] = ((df["a"] == "x") ^ (df["c"] > 0.3)).astype(int)
    out = {}
    for dev in ("cpu", "cuda:0"):
        resetEnv()
        useLocalEnv(1, device=dev)
        src = BatchOperator.fromDataframe(df, schemaStr="a string, b string, c double, label int")
        h = FeatureHasherBatchOp().setSelectedCols(["a", "b"]).setOutputCol("h").setNumFeatures(4096).linkFrom(src)
        va = VectorAssemblerBatchOp().setSelectedCols(["c", "h"]).setOutputCol("v").linkFrom(h)
        m = LogisticRegressionTrainBatchOp().setVectorCol("v").setLabelCol("label").setMaxIter(20).linkFrom(va)
        out[dev] = [r for r in m.collect()]
    import json
    a = json.loads([r for r in out["cpu"] if r[0] == 1048576][0][1])["coefVector"]["data"]
    b = json.loads([r for r in out["cuda:0"] if r[0] == 1048576][0][1])["coefVector"]["data"]
    np.testing.assert_allclose(b, a, rtol=1e-6, atol=1e-8)


@pytest.mark.parametrize("mean_len,idx_dtype", [(3, torch.int32), (21, torch.int64), (40, torch.int32),
                                                (150, torch.int64)])
def test_csr_mv_matches_fp64_reference(mean_len, idx_dtype):
    """HIP CSR SpMV (FeatureMatrix.mv on the GPU) == the fp64 segment sum, rows of length 0..3x the mean."""
    from alink_amd.models.common.features import FeatureMatrix
    from alink_amd.ops import feature as F
    g = torch.Generator().manual_seed(mean_len)
    n, d = 5000, 100_000
    lens = torch.randint(0, 3 * mean_len + 1, (n,), generator=g)
    lens[::97] = 0
    crow = torch.zeros(n + 1, dtype=torch.int64)
    crow[1:] = torch.cumsum(lens, 0)
    nnz = int(crow[-1])
    col = torch.randint(0, d, (nnz,), generator=g).to(idx_dtype)
    val = torch.randn(nnz, generator=g, dtype=torch.float64)
    v = torch.randn(d, generator=g, dtype=torch.float64)
    rows = torch.repeat_interleave(torch.arange(n), lens)
    ref = torch.zeros(n, dtype=torch.float64).index_add_(0, rows, val * v[col.long()])
    calls = F.CSR_MV_CALLS
    fm = FeatureMatrix(crow=crow.cuda(), col=col.cuda(), val=val.cuda(), ncols=d)
    got = fm.mv(v.cuda())
    assert F.CSR_MV_CALLS == calls + 1
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-12, atol=1e-12)
    assert torch.equal(fm.mv(v.cuda()), got)                 # deterministic
