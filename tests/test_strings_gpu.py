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


def test_hip_multi_column_feature_hash_equals_per_column():
    """murmur3_multi_index: m string columns (different prefixes, NULLs, empty strings, non-ASCII) in one launch ==
    murmur3_utf8_index per column; and an all-categorical FeatureHasher over device StringBlocks (the one-launch
    path) == the same strings as Python lists (the per-column path)."""
    cols = [_words(4000, 10 + j) for j in range(5)]
    nulls = [None, torch.as_tensor(np.random.default_rng(1).random(4000) < 0.1), None, None, None]
    blocks = []
    for w, nl in zip(cols, nulls):
        b = StringBlock.from_list([None if (nl is not None and bool(nl[i])) else s for i, s in enumerate(w)])
        blocks.append(b.to("cuda"))
    prefixes = [f"C{j}=" for j in range(4)] + ["中="]
    idx, valid = S.murmur3_multi_index(blocks, prefixes, 1 << 20)
    for j, b in enumerate(blocks):
        ref = S.murmur3_utf8_index(b, 1 << 20, prefix=prefixes[j])
        ok = ~b.null_mask()
        assert torch.equal(valid[j].bool(), ok)
        assert torch.equal(idx[j].long()[ok], ref[ok])
    import pandas as pd
    from alink_amd import useLocalEnv, BatchOperator, FeatureHasherBatchOp
    from alink_amd.common.mlenv import resetEnv
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    resetEnv()
    useLocalEnv(1, device="cuda:0")
    names = [f"c{j}" for j in range(5)]
    lists = [[None if (nl is not None and bool(nl[i])) else s for i, s in enumerate(w)] for w, nl in zip(cols, nulls)]
    df = pd.DataFrame({nm: col for nm, col in zip(names, lists)})
    op = lambda: FeatureHasherBatchOp().setSelectedCols(names).setCategoricalCols(names).setOutputCol("f") \
        .setNumFeatures(1 << 18)
    a = op().linkFrom(BatchOperator.fromDataframe(df, schemaStr=", ".join(f"{c} string" for c in names))).collect()
    mt = MTable(TableSchema(names, [Types.STRING] * 5), [Column(b) for b in blocks])
    b = op().linkFrom(TableSourceBatchOp(mt)).collect()
    assert [str(r[-1]) for r in a] == [str(r[-1]) for r in b]


def test_split_tokens_unique_ids_device_equal_host():
    """ops/strings.split_tokens / unique_ids on the GPU return exactly the host results (the NLP count trainers)."""
    import random
    from alink_amd.common.strings import StringBlock
    from alink_amd.ops.strings import split_tokens, unique_ids
    random.seed(11)
    docs = ["", " ", " a  b ", "中文 分词", None] + [
        " ".join(random.choice(["a", "", "é", "w%d" % random.randint(0, 300)]) for _ in range(random.randint(0, 12)))
        for _ in range(20000)]
    h = StringBlock.from_list(docs)
    th, dh = split_tokens(h)
    td, dd = split_tokens(h.to("cuda"))
    assert torch.equal(td.data.cpu(), th.data) and torch.equal(td.offsets.cpu(), th.offsets)
    assert torch.equal(dd.cpu(), dh)
    ih, rh = unique_ids(th)
    idd, rd = unique_ids(td)
    assert torch.equal(idd.cpu(), ih) and torch.equal(rd.cpu(), rh)


def test_doc_count_and_hash_vectorizers_gpu_equal_cpu():
    import pandas as pd
    from alink_amd import BatchOperator, DocCountVectorizerTrainBatchOp, DocHashCountVectorizerTrainBatchOp, \
        useLocalEnv
    import random
    random.seed(12)
    docs = [" ".join(random.choice(["a", "b", "", "dé", "w%d" % random.randint(0, 80)])
                     for _ in range(random.randint(0, 9))) for _ in range(3000)] + [None, ""]
    out = {}
    for dev in ("cpu", "cuda:0"):
        useLocalEnv(1, device=dev)
        src = BatchOperator.fromDataframe(pd.DataFrame({"t": docs}), schemaStr="t string")
        out[dev] = (DocCountVectorizerTrainBatchOp().setSelectedCol("t").setMinDF(2.0).linkFrom(src).collect(),
                    DocHashCountVectorizerTrainBatchOp().setSelectedCol("t").setNumFeatures(512).linkFrom(src)
                    .collect())
    useLocalEnv(1)
    assert out["cpu"] == out["cuda:0"]
