"""Feature engineering / statistics vs the reference docs (docs/en/*.md script examples)."""
import numpy as np
import pandas as pd
import pytest

from alink_amd import *  # noqa: F401,F403
from alink_amd.common.linalg import VectorUtil

SC = [["a", 10.0, 100], ["b", -2.5, 9], ["c", 100.2, 1], ["d", -99.9, 100], ["a", 1.4, 1], ["b", -2.2, 9],
      ["c", 100.9, 1]]


def _scaler_in(extra_null=False):
    rows = SC + ([[None, None, None]] if extra_null else [])
    df = pd.DataFrame({"col1": [r[0] for r in rows], "col2": [r[1] for r in rows], "col3": [r[2] for r in rows]})
    return BatchOperator.fromDataframe(df, schemaStr="col1 string, col2 double, col3 long"), df


@pytest.mark.parametrize("stage,ref2,ref3", [
    (StandardScaler, [-0.078352, -0.259243, 1.226961, -1.668749, -0.202805, -0.254902, 1.237091],
     [1.459581, -0.481449, -0.652089, 1.459581, -0.652089, -0.481449, -0.652089]),
    (MinMaxScaler, [0.547311, 0.485060, 0.996514, 0.0, 0.504482, 0.486554, 1.0],
     [1.0, 0.080808, 0.0, 1.0, 0.0, 0.080808, 0.0]),
    (MaxAbsScaler, [0.099108, -0.024777, 0.993062, -0.990089, 0.013875, -0.021804, 1.0],
     [1.0, 0.09, 0.01, 1.0, 0.01, 0.09, 0.01])])
def test_scalers_doc(stage, ref2, ref3):
    op, df = _scaler_in()
    out = stage().setSelectedCols(["col2", "col3"]).fit(op).transform(op).collectToDataframe()
    np.testing.assert_allclose(out["col2"].values, ref2, atol=1e-6)
    np.testing.assert_allclose(out["col3"].values, ref3, atol=1e-6)
    # stream path with the same model
    box = []
    m = stage().setSelectedCols(["col2", "col3"]).fit(op)
    m.transform(StreamOperator.fromDataframe(df, schemaStr="col1 string, col2 double, col3 long")) \
        .link(CollectStreamOp(box))
    StreamOperator.execute()
    np.testing.assert_allclose([r[1] for r in box], ref2, atol=1e-6)


def test_imputer_doc():
    op, _ = _scaler_in(extra_null=True)
    out = Imputer().setSelectedCols(["col2", "col3"]).fit(op).transform(op).collect()
    assert out[-1][1] == pytest.approx(15.414286, abs=1e-6) and out[-1][2] == 31


def test_string_indexer_doc():
    df = pd.DataFrame({"f0": ["football"] * 3 + ["basketball"] * 2 + ["tennis"]})
    op = BatchOperator.fromDataframe(df, schemaStr="f0 string")
    out = StringIndexer().setSelectedCol("f0").setOutputCol("f0_indexed").setStringOrderType("frequency_asc") \
        .fit(op).transform(op).collectToDataframe()
    assert list(out["f0_indexed"]) == [2, 2, 2, 1, 1, 0]


D4 = [[1.1, True, 2, "A"], [1.1, False, 2, "B"], [1.1, True, 1, "B"], [2.2, True, 1, "A"]]


def _d4():
    df = pd.DataFrame({"double": [r[0] for r in D4], "bool": [r[1] for r in D4], "number": [r[2] for r in D4],
                       "str": [r[3] for r in D4]})
    return BatchOperator.fromDataframe(df, schemaStr="double double, bool boolean, number int, str string")


def test_feature_hasher_doc_bitexact():
    out = FeatureHasher().setSelectedCols(["double", "bool", "number", "str"]).setOutputCol("output") \
        .setNumFeatures(200).transform(_d4()).collect()
    got = [VectorUtil.toString(r[4]) for r in out]
    assert got == ["$200$13:2.0 38:1.1 45:1.0 195:1.0", "$200$13:2.0 30:1.0 38:1.1 76:1.0",
                   "$200$13:1.0 38:1.1 76:1.0 195:1.0", "$200$13:1.0 38:2.2 45:1.0 195:1.0"]


def test_one_hot_doc():
    src = _d4()
    onehot = OneHotTrainBatchOp().setSelectedCols(["double", "bool", "number", "str"]).setDiscreteThresholds(2)
    pred = OneHotPredictBatchOp().setSelectedCols(["double", "bool"]).setEncode("ASSEMBLED_VECTOR") \
        .setOutputCols(["pred"]).setDropLast(False)
    onehot.linkFrom(src)
    out = pred.linkFrom(onehot, src).collect()
    assert [VectorUtil.toString(r[4]) for r in out] == ["$6$0:1.0 3:1.0", "$6$0:1.0 5:1.0", "$6$0:1.0 3:1.0",
                                                         "$6$2:1.0 3:1.0"]


def test_bucketizer_binarizer_doc():
    out = Bucketizer().setSelectedCols(["double"]).setCutsArray([[2.0]]).transform(_d4()).collect()
    assert [r[0] for r in out] == [0, 0, 0, 1]
    out = Binarizer().setSelectedCol("double").setThreshold(2.0).transform(_d4()).collect()
    assert [r[0] for r in out] == [0.0, 0.0, 0.0, 1.0]


def test_dct_doc():
    df = pd.DataFrame({"features": ["-0.6264538 0.1836433", "11.1249309 9.9550664"]})
    out = DCT().setSelectedCol("features").setOutputCol("result").transform(
        BatchOperator.fromDataframe(df, schemaStr="features string")).collect()
    np.testing.assert_allclose(out[0][1].data, [-0.31311430733060563, -0.5728251528295567], rtol=1e-12)
    np.testing.assert_allclose(out[1][1].data, [14.905809038224113, 0.8272191210194105], rtol=1e-12)


def test_quantile_discretizer_and_summarizer():
    rng = np.random.default_rng(0)
    df = pd.DataFrame({"x": rng.normal(size=1000), "y": rng.integers(0, 10, 1000)})
    op = BatchOperator.fromDataframe(df, schemaStr="x double, y long")
    out = QuantileDiscretizer().setSelectedCols(["x"]).setNumBuckets(4).fit(op).transform(op).collectToDataframe()
    counts = np.bincount(out["x"].values.astype(int))
    assert len(counts) == 4 and counts.min() > 200
    s = SummarizerBatchOp().setSelectedCols(["x", "y"]).linkFrom(op).collectSummary()
    assert s.mean("x") == pytest.approx(df["x"].mean()) and s.standardDeviation("y") == pytest.approx(df["y"].std())
    c = CorrelationBatchOp().setSelectedCols(["x", "y"]).linkFrom(op).collectCorrelation().getCorrelation()
    assert c[0, 1] == pytest.approx(np.corrcoef(df["x"], df["y"])[0, 1])


def test_correlation_pairwise_complete_and_spearman():
    """TableSummarizerTest (reference operator/common/statistics/basicstatistic): with NULLs, every column pair
    uses the rows where both are present (long/int vs double -> -1.0 on the two shared rows); the reference's
    method enum spells Spearman ``SPEAMAN``."""
    from alink_amd import CorrelationBatchOp, SummarizerBatchOp
    from alink_amd.operator.batch.source import MemSourceBatchOp
    rows = [(1, 1, 2.0), (2, 2, -3.0), (None, None, 2.0), (0, 0, None)]
    src = MemSourceBatchOp(rows, "f_long long, f_int int, f_double double")
    cols = ["f_long", "f_int", "f_double"]
    c = CorrelationBatchOp().setSelectedCols(cols).linkFrom(src).collectCorrelation().getCorrelationMatrix()
    np.testing.assert_allclose(c.getArrayCopy2D(), [[1, 1, -1], [1, 1, -1], [-1, -1, 1]], atol=1e-12)
    s = SummarizerBatchOp().setSelectedCols(cols).linkFrom(src).collectSummary()
    assert [s.sum(x) for x in cols] == [3.0, 3.0, 1.0]
    assert [s.normL2(x) ** 2 for x in cols] == pytest.approx([5.0, 5.0, 17.0])
    assert [s.min(x) for x in cols] == [0.0, 0.0, -3.0] and [s.max(x) for x in cols] == [2.0, 2.0, 2.0]
    assert s.variance("f_double") == pytest.approx(8.333333333333334)
    src2 = MemSourceBatchOp([(1.0, 3.0), (2.0, 1.0), (3.0, 2.0), (4.0, 10.0)], "a double, b double")
    sp = CorrelationBatchOp().setSelectedCols(["a", "b"]).setMethod("SPEAMAN").linkFrom(src2) \
        .collectCorrelation().getCorrelationMatrix()
    assert sp.get(0, 1) == pytest.approx(0.4)                 # 1 - 6 * 6 / (4 * 15)


def _mapper_table(rows, names, types):
    from alink_amd.common.types import TableSchema
    return rows, TableSchema(names, types)


def test_scaler_and_imputer_mappers_on_reference_model_rows():
    """{Imputer,StandardScaler,MinMaxScaler,MaxAbsScaler}MapperTest (reference operator/common/dataproc): the
    reference's model tables (no scalerKind key) load and transform in place, arrays in model-column order."""
    from alink_amd.common.params import Params
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.feature import scalers as S
    T = Types
    ms = TableSchema(["model_id", "model_info", "f_double", "f_long", "f_int"], [T.LONG, T.STRING, T.DOUBLE, T.LONG,
                                                                                   T.INT])
    ds = TableSchema(["f_string", "f_long", "f_int", "f_double", "f_boolean"],
                     [T.STRING, T.LONG, T.INT, T.DOUBLE, T.BOOLEAN])
    for strat, vals, expect in (("mean", "[0.3333333333333333,1.0,1.0]", (1, 1, 0.3333333333333333)),
                                ("min", "[-3.0,0.0,0.0]", (0, 0, -3.0)), ("min", "[2.0, 2.0, 2.0]", (2, 2, 2.0))):
        m = S.ImputerModelMapper(ms, ds, Params())
        m.loadModel([(0, '{"selectedCols":"[\\"f_double\\",\\"f_long\\",\\"f_int\\"]","strategy":"\\"%s\\""}' % strat,
                      None, None, None), (1048576, vals, None, None, None)])
        r = m.map(("a", None, None, None, True))
        assert (r[1], r[2]) == expect[:2] and type(r[1]) is int and r[3] == pytest.approx(expect[2])
    msb = TableSchema(["model_id", "model_info", "f_double", "f_long", "f_int", "f_boolean"],
                      [T.LONG, T.STRING, T.DOUBLE, T.LONG, T.INT, T.BOOLEAN])
    m = S.ImputerModelMapper(msb, ds, Params())
    m.loadModel([(0, '{"selectedCols":"[\\"f_double\\",\\"f_long\\",\\"f_int\\",\\"f_boolean\\"]","fillValue":"\\"0\\"",'
                     '"strategy":"\\"VALUE\\""}', None, None, None, None)])
    assert tuple(m.map(("a", None, None, None, None))[1:]) == (0, 0, 0.0, False)
    m = S.StandardScalerModelMapper(ms, ds, Params())
    m.loadModel([(0, '{"withMean":"true","withStd":"true"}', None, None, None),
                 (1048576, "[1.0,1.0,0.2]", None, None, None), (2097152, "[1.0,1.0,1.0]", None, None, None)])
    assert tuple(m.map(("a", 1, 1, 2.0, True))[1:4]) == pytest.approx((0.0, 0.8, 1.0))
    m = S.MinMaxScalerModelMapper(ms, ds, Params())
    m.loadModel([(0, '{"min":"0.0","max":"1.0","selectedCols":"[\\"f_long\\",\\"f_int\\",\\"f_double\\"]"}', None, None,
                  None), (1048576, "[0.0,0.0,-3.0]", None, None, None), (2097152, "[2.0, 2.0, 2.0]", None, None, None)])
    assert tuple(m.map(("d", 1, 1, 2.0, True))[1:4]) == pytest.approx((0.5, 0.8, 1.0))
    m = S.MaxAbsScalerModelMapper(TableSchema(["model_id", "model_info", "f0", "f1"], [T.LONG, T.STRING, T.DOUBLE,
                                                                                     T.DOUBLE]),
                                  TableSchema(["f0", "f1"], [T.DOUBLE, T.DOUBLE]), Params())
    m.loadModel([(0, '{"selectedCols":"[\\"f0\\",\\"f1\\"]"}', None, None), (1048576, "[4.0,3.0]", None, None)])
    assert tuple(m.map((1.0, 2.0))) == pytest.approx((0.25, 0.6666666666666666))


@pytest.mark.parametrize("selector,expect", [("NumTopFeatures", [0, 2]), ("PERCENTILE", [0, 2]),
                                             ("FPR", [0, 1, 2, 3]), ("FDR", [0, 1, 2, 3, 4]), ("FWE", [0])])
def test_chisq_selector_rules_reference(selector, expect):
    """ChiSquareTestTest.testChiSqSelector*: five features with p-values 0.1, 0.3, 0.2, 0.4, 0.5; numTopFeatures 2,
    percentile / fpr / fdr / fwe 0.5."""
    from types import SimpleNamespace
    from alink_amd.common.params import Params
    from alink_amd.operator.batch.feature import _chisq_select
    results = [SimpleNamespace(p=v) for v in (0.1, 0.3, 0.2, 0.4, 0.5)]
    p = Params().set("selectorType", selector).set("numTopFeatures", 2).set("percentile", 0.5).set("fpr", 0.5) \
        .set("fdr", 0.5).set("fwe", 0.5)
    got = _chisq_select(results, p)
    assert len(got) == len(expect) and got[:2] == expect[:2]


def test_table_summary_reference():
    """TableSummaryTest: 4 rows, 5 columns, f_double = 2, -3, 2, NULL."""
    import alink_amd as A
    from alink_amd.operator.batch.source import MemSourceBatchOp
    d = MemSourceBatchOp([("a", 1, 1, 2.0, True), (None, 2, 2, -3.0, True), ("c", None, None, 2.0, False),
                          ("a", 0, 0, None, None)],
                         "f_string string, f_long bigint, f_int int, f_double double, f_boolean boolean")
    s = A.SummarizerBatchOp().linkFrom(d).collectSummary()
    assert len(s.colNames) == 5 and s.count() == 4 and s.count == 4
    assert s.numMissingValue("f_double") == 1 and s.numValidValue("f_double") == 3
    assert s.max("f_double") == 2.0 and s.min("f_int") == 0.0
    assert s.mean("f_double") == pytest.approx(0.3333333333333333, abs=1e-3)
    assert s.variance("f_double") == pytest.approx(8.333333333333334, abs=1e-3)
    assert s.standardDeviation("f_double") == pytest.approx(2.886751345948129, abs=1e-3)
    assert s.normL1("f_double") == pytest.approx(7.0) and s.normL2("f_double") == pytest.approx(4.123105625617661)


def _vector_summary(rows):
    import alink_amd as A
    from alink_amd.operator.batch.source import MemSourceBatchOp
    return A.VectorSummarizerBatchOp().setSelectedCol("v").linkFrom(MemSourceBatchOp([(r,) for r in rows], ["v"])) \
        .collectVectorSummary()


def _dense(v):
    return list(v.toDenseVector().data) if hasattr(v, "toDenseVector") else list(v.data)


def test_sparse_vector_summary_reference():
    """SparseVectorSummaryTest: implicit zeros count in min / max / variance; numNonZero is dense."""
    s = _vector_summary(["$5$0:1.0 1:-1.0 2:3.0", "$5$1:2.0 2:-2.0 3:3.0", "$5$2:3.0 3:-3.0 4:3.0",
                         "$5$0:4.0 2:-4.0 3:3.0", "$5$0:5.0 1:-5.0 4:3.0"])
    assert s.colNum == 5 and s.vectorSize() == 5
    got = [s.max(1), s.min(1), s.sum(1), s.mean(1), s.variance(1), s.standardDeviation(1), s.normL1(1), s.normL2(1),
           s.numNonZero(1)]
    assert got == pytest.approx([2.0, -5.0, -4.0, -0.8, 6.7, 2.588436, 8.0, 5.477226, 3], abs=1e-3)
    from alink_amd.common.linalg import DenseVector, SparseVector
    assert isinstance(s.numNonZero(), DenseVector) and list(s.numNonZero().data) == [3.0, 3.0, 4.0, 3.0, 2.0]
    assert isinstance(s.max(), SparseVector)
    expect = {"max": [5.0, 2.0, 3.0, 3.0, 3.0], "min": [0.0, -5.0, -4.0, -3.0, 0.0], "sum": [10.0, -4.0, 0.0, 3.0, 6.0],
              "mean": [2.0, -0.8, 0.0, 0.6, 1.2], "variance": [5.5, 6.7, 9.5, 6.3, 2.7],
              "standardDeviation": [2.345208, 2.588436, 3.082207, 2.509980, 1.643168],
              "normL1": [10, 8.0, 12.0, 9.0, 6.0], "normL2": [6.480741, 5.477226, 6.164414, 5.196152, 4.242641]}
    for name, e in expect.items():
        assert _dense(getattr(s, name)()) == pytest.approx(e, abs=1e-3), name


def test_dense_vector_summary_reference():
    """DenseVectorSummaryTest."""
    s = _vector_summary(["1.0 -1.0 3.0", "2.0 -2.0 3.0", "3.0 -3.0 3.0", "4.0 -4.0 3.0", "5.0 -5.0 3.0"])
    assert s.vectorSize() == 3 and s.count() == 5
    got = [s.max(1), s.min(1), s.sum(1), s.mean(1), s.variance(1), s.standardDeviation(1), s.normL1(1), s.normL2(1)]
    assert got == pytest.approx([-1.0, -5.0, -15.0, -3.0, 2.5, 1.5811, 15.0, 7.416198], abs=1e-3)
    expect = {"max": [5.0, -1.0, 3.0], "min": [1.0, -5.0, 3.0], "sum": [15.0, -15.0, 15.0], "mean": [3.0, -3.0, 3.0],
              "variance": [2.5, 2.5, 0.0], "standardDeviation": [1.5811, 1.5811, 0.0], "normL1": [15, 15, 15],
              "normL2": [7.416198, 7.416198, 6.7082]}
    for name, e in expect.items():
        assert _dense(getattr(s, name)()) == pytest.approx(e, abs=1e-3), name


@pytest.mark.parametrize("invalid", ["KEEP", "SKIP", "ERROR"])
def test_string_indexer_packed_column_paths_equal_row_path(invalid):
    """StringIndexer train / predict on a packed string column (device dictionary encoding, one lookup per
    distinct token) equal the per-value paths: nulls, empty strings, unseen tokens under KEEP / SKIP / ERROR,
    and the INDEX bucket output of the quantile discretizer stays int64 with its null mask."""
    import torch
    from alink_amd.common.params import Params
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.feature import encoders as E
    vals = ["b", "a", None, "", "c", "a", "b", "", None, "zz"] * 7
    blk = StringBlock.from_list(vals)
    mt_blk = MTable(TableSchema(["c"], [Types.STRING]), [Column(blk)])
    mt_lst = MTable(TableSchema(["c"], [Types.STRING]), [Column(list(vals))])
    assert E._column_token_counts(mt_blk.col("c")) == E._column_token_counts(mt_lst.col("c"))
    model = E.train_string_indexer(MTable(TableSchema(["c"], [Types.STRING]),
                                          [Column([v for v in vals if v != "zz"])]),
                                   Params().set("selectedCol", "c").set("stringOrderType", "ALPHABET_ASC"))
    p = Params().set("selectedCol", "c").set("outputCol", "i").set("handleInvalid", invalid)
    m = E.StringIndexerModelMapper(model.schema, mt_blk.schema, p)
    m.loadModel(list(model.rows()))
    if invalid == "ERROR":
        with pytest.raises(RuntimeError):
            m._map_columns(mt_blk)
        return
    got = m._map_columns(mt_blk)[0].to_list()
    ref = [m.mapColumn(v) for v in vals]
    assert got == ref


@pytest.mark.parametrize("invalid", ["KEEP", "SKIP"])
@pytest.mark.parametrize("left_open", [True, False])
def test_bucket_index_tensor_path_equals_numpy_path(invalid, left_open):
    """INDEX bucketing of tensor columns (torch.searchsorted where the column lives) equals the numpy path:
    values on the split points (both interval sides), NaN / null cells, +-inf."""
    import numpy as np
    import torch
    from alink_amd.common.params import Params
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.feature.encoders import BucketizerMapper
    x = torch.tensor([-5.0, 0.0, 1.0, 1.5, 2.0, 3.0, float("nan"), float("inf"), -float("inf"), 2.0, 0.5],
                     dtype=torch.float64)
    nulls = torch.zeros(11, dtype=torch.bool)
    nulls[9] = True
    mt = MTable(TableSchema(["a"], [Types.DOUBLE]), [Column(x, nulls)])
    p = Params().set("selectedCols", ["a"]).set("cutsArray", [[0.0, 1.0, 2.0]]).set("leftOpen", left_open) \
        .set("handleInvalid", invalid).set("encode", "INDEX")
    m = BucketizerMapper(mt.schema, p)
    got = m._map_columns(mt)[0]
    vals = [None if (nulls[i] or np.isnan(x[i].item())) else x[i].item() for i in range(11)]
    mt2 = MTable(TableSchema(["a"], [Types.DOUBLE]), [Column(vals)])
    ref = m._map_columns(mt2)[0]
    assert got.to_list() == ref.to_list()


@pytest.mark.parametrize("invalid,enable_else", [("KEEP", False), ("SKIP", False), ("KEEP", True), ("SKIP", True)])
def test_onehot_packed_column_equals_list_column(invalid, enable_else):
    """OneHot predict on a packed string column (device dictionary encoding) equals the list-column path:
    nulls, empty strings, unseen tokens, every invalid / else strategy."""
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    import alink_amd as A
    train_vals = ["b", "a", "", "c", "a", "b"] * 5
    vals = ["b", "a", None, "", "c", "zz", "a", None] * 4
    tr = MTable(TableSchema(["c"], [Types.STRING]), [Column(list(train_vals))])
    op = A.OneHotTrainBatchOp().setSelectedCols(["c"])
    if enable_else:
        op = op.setDiscreteThresholds(6)              # rare tokens go to the 'else' slot
    model = op.linkFrom(TableSourceBatchOp(tr))
    outs = []
    for col in (Column(StringBlock.from_list(vals)), Column(list(vals))):
        mt = MTable(TableSchema(["c"], [Types.STRING]), [col])
        op = A.OneHotPredictBatchOp().setSelectedCols(["c"]).setOutputCols(["oh"]).setHandleInvalid(invalid) \
            .setReservedCols([]).linkFrom(model, TableSourceBatchOp(mt))
        outs.append([str(v) for v in op.getOutputTable().col("oh").to_list()])
    assert outs[0] == outs[1]


def test_imputer_tensor_columns_equal_list_columns():
    """Imputer on tensor columns (nulls and NaN replaced on the tensor) equals the list path, int and double."""
    import torch
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    import alink_amd as A
    x = torch.tensor([1.0, float("nan"), 3.0, 4.0, 0.5], dtype=torch.float64)
    xn = torch.tensor([False, False, False, True, False])
    k = torch.tensor([1, 2, 3, 4, 5], dtype=torch.int64)
    kn = torch.tensor([False, True, False, False, False])
    schema = TableSchema(["x", "k"], [Types.DOUBLE, Types.LONG])
    t_mt = MTable(schema, [Column(x, xn), Column(k, kn)])
    l_mt = MTable(schema, [Column([1.0, float("nan"), 3.0, None, 0.5]), Column([1, None, 3, 4, 5])])
    for strategy in ("MEAN", "MIN", "VALUE"):
        op = A.ImputerTrainBatchOp().setSelectedCols(["x", "k"]).setStrategy(strategy)
        if strategy == "VALUE":
            op = op.setFillValue("7")
        model = op.linkFrom(TableSourceBatchOp(l_mt))
        outs = [A.ImputerPredictBatchOp().linkFrom(model, TableSourceBatchOp(m)).collect() for m in (t_mt, l_mt)]
        assert [tuple(r) for r in outs[0]] == [tuple(r) for r in outs[1]], strategy


@pytest.mark.parametrize("invalid", ["KEEP", "SKIP", "ERROR"])
def test_multi_string_indexer_columnar(invalid):
    """MultiStringIndexer predict over packed string columns (device dictionary codes, one lookup per distinct
    token) equals the row path: unseen tokens, nulls and the handleInvalid rules."""
    from alink_amd import MultiStringIndexerPredictBatchOp, MultiStringIndexerTrainBatchOp
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.feature.encoders import MultiStringIndexerModelMapper
    from alink_amd.operator.batch.source import TableSourceBatchOp
    schema = TableSchema(["c", "d"], [Types.STRING, Types.STRING])
    train = MTable(schema, [Column(StringBlock.from_list(["a", "b", "a", "c"])),
                            Column(StringBlock.from_list(["x", "y", "y", "z"]))])
    model = MultiStringIndexerTrainBatchOp().setSelectedCols(["c", "d"]).linkFrom(TableSourceBatchOp(train))
    cs = ["a", "b", "c", "a"] * 5 if invalid == "ERROR" else ["a", "q", None, "b", "", "c"] * 4
    ds = ["y", "x", "z", "y"] * 5 if invalid == "ERROR" else ["z", None, "w", "x", "y", "y"] * 4
    test = MTable(schema, [Column(StringBlock.from_list(cs)), Column(StringBlock.from_list(ds))])
    op = MultiStringIndexerPredictBatchOp().setSelectedCols(["c", "d"]).setOutputCols(["ci", "di"]) \
        .setHandleInvalid(invalid).setReservedCols([])
    fast = op.linkFrom(model, TableSourceBatchOp(test)).collect()
    mapper = MultiStringIndexerModelMapper(model.getOutputTable().schema, schema,
                                           op.getParams().set("handleInvalid", invalid))
    mapper.loadModel(model.getOutputTable().rows())
    slow = [tuple(mapper._map_row_values(r)) for r in test.rows()]
    assert [tuple(r) for r in fast] == slow
    if invalid == "ERROR":
        bad = MTable(schema, [Column(StringBlock.from_list(["a", "zz"])), Column(StringBlock.from_list(["x", "y"]))])
        with pytest.raises(RuntimeError, match="Unseen token"):
            op.linkFrom(model, TableSourceBatchOp(bad)).collect()
