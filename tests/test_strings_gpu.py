"""HIP string kernels (csrc/feature.hip): byte murmur3 for shuffle keys, UTF-8 -> UTF-16 Guava feature hash."""
import numpy as np
import pytest
import torch

from alink_amd.common.strings import StringBlock
from alink_amd.ops import strings as S

pytestmark = pytest.mark.gpu


def _words(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        L = int(rng.integers(0, 40))
        pool = rng.choice([0x41, 0xE9, 0x4E2D, 0x1F600], size=L)
        out.append("".join(chr(int(c) + int(rng.integers(0, 20))) for c in pool))
    return out


def test_device_block_take_and_concat_match_host():
    w = _words(5000, 1)
    host = StringBlock.from_list(w)
    dev = host.to("cuda")
    idx = np.random.default_rng(2).integers(0, 5000, 7000)
    assert dev.take(torch.as_tensor(idx).cuda()).to_list() == [w[i] for i in idx]
    assert StringBlock.concat([dev, dev.take([3])]).to_list() == w + [w[3]]


def test_hip_murmur3_bytes_matches_host():
    w = _words(20000, 3) + ["", "hello"]
    blk = StringBlock.from_list(w)
    assert torch.equal(S.hash_bytes(blk.to("cuda")).cpu(), S.hash_bytes(blk))


def test_hip_utf8_feature_hash_matches_guava_host():
    from alink_amd.models.feature.encoders import murmur3_index as host_index
    w = _words(8000, 4)
    got = S.murmur3_utf8_index(StringBlock.from_list(w).to("cuda"), 262144, prefix="cat=").cpu().numpy()
    ref = np.asarray(host_index(["cat=" + x for x in w], 262144), dtype=np.int64)
    np.testing.assert_array_equal(got, ref)


def test_feature_hasher_on_device_string_block_equals_list_column():
    """FeatureHasher over a device-resident StringBlock column == over the same strings as a Python list."""
    import pandas as pd
    from alink_amd import useLocalEnv, BatchOperator, FeatureHasherBatchOp
    from alink_amd.common.mlenv import resetEnv
    from alink_amd.common.table import Column, MTable
    from alink_amd.operator.batch.source import TableSourceBatchOp
    w = _words(3000, 5)
    resetEnv()
    useLocalEnv(1, device="cuda:0")
    df = pd.DataFrame({"c": w, "x": np.arange(3000.0)})
    a = FeatureHasherBatchOp().setSelectedCols(["c", "x"]).setCategoricalCols(["c"]).setOutputCol("f") \
        .setNumFeatures(1 << 16).linkFrom(BatchOperator.fromDataframe(df, schemaStr="c string, x double")).collect()
    src = BatchOperator.fromDataframe(df, schemaStr="c string, x double")
    mt = src.getOutputTable()
    mt2 = MTable(mt.schema, [Column(StringBlock.from_list(w).to("cuda")), mt.cols[1]])
    b = FeatureHasherBatchOp().setSelectedCols(["c", "x"]).setCategoricalCols(["c"]).setOutputCol("f") \
        .setNumFeatures(1 << 16).linkFrom(TableSourceBatchOp(mt2)).collect()
    assert [str(r[-1]) for r in a] == [str(r[-1]) for r in b]
