"""Operator catalogue coverage, part 2: format-conversion stream twins, triple formats, sources / sinks,
Map / FlatMap / ModelMap bases, AFT survival regression, IndexToString, stream evaluation and the gated
connectors (reference: A/operator/{batch,stream}/{dataproc/format,source,sink}/*.java)."""
import os

import numpy as np
import pandas as pd
import pytest

import alink_amd as A
from alink_amd import BatchOperator, StreamOperator, useLocalEnv
from alink_amd.operator.stream.utils import CollectStreamOp


@pytest.fixture(autouse=True)
def _env():
    useLocalEnv(1)


DF = pd.DataFrame({"id": [1, 2, 3, 4], "f0": [1.5, -2.0, 0.25, 3.0], "f1": [0.5, 1.0, -1.0, 2.0],
                   "csv": ["1.5,0.5", "-2.0,1.0", "0.25,-1.0", "3.0,2.0"],
                   "json": ['{"f0":1.5,"f1":0.5}', '{"f0":-2.0,"f1":1.0}', '{"f0":0.25,"f1":-1.0}', '{"f0":3.0,"f1":2.0}'],
                   "kv": ["f0:1.5,f1:0.5", "f0:-2.0,f1:1.0", "f0:0.25,f1:-1.0", "f0:3.0,f1:2.0"],
                   "vec": ["1.5 0.5", "-2.0 1.0", "0.25 -1.0", "3.0 2.0"]})
SCHEMA = "id long, f0 double, f1 double, csv string, json string, kv string, vec string"
COLS = "f0 double, f1 double"


def _b():
    return BatchOperator.fromDataframe(DF, schemaStr=SCHEMA)


def _s():
    return StreamOperator.fromDataframe(DF, schemaStr=SCHEMA)


def _collect(sop):
    box = []
    sop.link(CollectStreamOp(box))
    StreamOperator.execute()
    return box


def _key(rows):
    return sorted((tuple(round(x, 6) if isinstance(x, float) else (str(x) if x is not None and not isinstance(
        x, (int, str)) else x) for x in r) for r in rows), key=str)


# (batch op, stream op, params) — the stream twin must reproduce the batch rows
FORMAT_TWINS = [
    (A.ColumnsToCsvBatchOp, A.ColumnsToCsvStreamOp, dict(selectedCols=["f0", "f1"], csvCol="o", schemaStr=COLS)),
    (A.ColumnsToJsonBatchOp, A.ColumnsToJsonStreamOp, dict(selectedCols=["f0", "f1"], jsonCol="o")),
    (A.ColumnsToKvBatchOp, A.ColumnsToKvStreamOp, dict(selectedCols=["f0", "f1"], kvCol="o")),
    (A.ColumnsToVectorBatchOp, A.ColumnsToVectorStreamOp, dict(selectedCols=["f0", "f1"], vectorCol="o")),
    (A.ColumnsToTripleBatchOp, A.ColumnsToTripleStreamOp, dict(selectedCols=["f0", "f1"], tripleColValSchemaStr="c string, v double")),
    (A.CsvToColumnsBatchOp, A.CsvToColumnsStreamOp, dict(csvCol="csv", schemaStr=COLS)),
    (A.CsvToJsonBatchOp, A.CsvToJsonStreamOp, dict(csvCol="csv", schemaStr=COLS, jsonCol="o")),
    (A.CsvToKvBatchOp, A.CsvToKvStreamOp, dict(csvCol="csv", schemaStr=COLS, kvCol="o")),
    (A.CsvToVectorBatchOp, A.CsvToVectorStreamOp, dict(csvCol="csv", schemaStr=COLS, vectorCol="o")),
    (A.CsvToTripleBatchOp, A.CsvToTripleStreamOp, dict(csvCol="csv", schemaStr=COLS, tripleColValSchemaStr="c string, v double")),
    (A.JsonToColumnsBatchOp, A.JsonToColumnsStreamOp, dict(jsonCol="json", schemaStr=COLS)),
    (A.JsonToCsvBatchOp, A.JsonToCsvStreamOp, dict(jsonCol="json", schemaStr=COLS, csvCol="o")),
    (A.JsonToKvBatchOp, A.JsonToKvStreamOp, dict(jsonCol="json", kvCol="o")),
    (A.JsonToTripleBatchOp, A.JsonToTripleStreamOp, dict(jsonCol="json", tripleColValSchemaStr="c string, v double")),
    (A.KvToColumnsBatchOp, A.KvToColumnsStreamOp, dict(kvCol="kv", schemaStr=COLS)),
    (A.KvToCsvBatchOp, A.KvToCsvStreamOp, dict(kvCol="kv", schemaStr=COLS, csvCol="o")),
    (A.KvToJsonBatchOp, A.KvToJsonStreamOp, dict(kvCol="kv", jsonCol="o")),
    (A.KvToTripleBatchOp, A.KvToTripleStreamOp, dict(kvCol="kv", tripleColValSchemaStr="c string, v double")),
    (A.VectorToColumnsBatchOp, A.VectorToColumnsStreamOp, dict(vectorCol="vec", schemaStr=COLS)),
    (A.VectorToCsvBatchOp, A.VectorToCsvStreamOp, dict(vectorCol="vec", schemaStr=COLS, csvCol="o")),
    (A.VectorToJsonBatchOp, A.VectorToJsonStreamOp, dict(vectorCol="vec", jsonCol="o")),
    (A.VectorToKvBatchOp, A.VectorToKvStreamOp, dict(vectorCol="vec", kvCol="o")),
    (A.VectorToTripleBatchOp, A.VectorToTripleStreamOp, dict(vectorCol="vec", tripleColValSchemaStr="c long, v double")),
    (A.JsonToVectorBatchOp, A.JsonToVectorStreamOp, dict(jsonCol="o2", vectorCol="o")),
    (A.KvToVectorBatchOp, A.KvToVectorStreamOp, dict(kvCol="o2", vectorCol="o")),
]


def _set(op, kw):
    for k, v in kw.items():
        getattr(op, "set" + k[0].upper() + k[1:])(v)
    return op


@pytest.mark.parametrize("bop,sop,kw", FORMAT_TWINS, ids=[t[0].__name__ for t in FORMAT_TWINS])
def test_format_stream_twins(bop, sop, kw):
    src_b, src_s = _b(), _s()
    if kw.get("jsonCol") == "o2" or kw.get("kvCol") == "o2":
        # index-keyed inputs for the ...ToVector conversions
        idx = DF.assign(o2=['{"0":1.5,"1":0.5}', '{"0":-2.0,"1":1.0}', '{"0":0.25,"1":-1.0}', '{"0":3.0,"1":2.0}']
                        if "jsonCol" in kw else ["0:1.5,1:0.5", "0:-2.0,1:1.0", "0:0.25,1:-1.0", "0:3.0,1:2.0"])
        src_b = BatchOperator.fromDataframe(idx, schemaStr=SCHEMA + ", o2 string")
        src_s = StreamOperator.fromDataframe(idx, schemaStr=SCHEMA + ", o2 string")
    b = _set(bop(), dict(kw, reservedCols=["id"])).linkFrom(src_b).collect()
    s = _collect(_set(sop(), dict(kw, reservedCols=["id"])).linkFrom(src_s))
    assert len(b) >= 4 and _key(b) == _key(s)


def test_triple_to_any_and_any_to_triple():
    trip = A.ColumnsToTripleBatchOp().setSelectedCols(["f0", "f1"]).setReservedCols(["id"]) \
        .setTripleColValSchemaStr("c string, v double").linkFrom(_b())
    rows = trip.collect()
    assert len(rows) == 8
    kw = dict(tripleRowCol="id", tripleColCol="c", tripleValCol="v")
    for op, col, extra in ((A.TripleToCsvBatchOp, "csv", dict(csvCol="o", schemaStr=COLS)),
                           (A.TripleToKvBatchOp, "kv", dict(kvCol="o")),
                           (A.TripleToJsonBatchOp, "json", dict(jsonCol="o")),
                           (A.TripleToColumnsBatchOp, None, dict(schemaStr=COLS))):
        out = _set(op(), dict(kw, **extra)).linkFrom(trip).collect()
        assert len(out) == 4, op
    vec = A.TripleToVectorBatchOp().setTripleRowCol("id").setTripleColCol("col").setTripleValCol("val") \
        .setVectorCol("v").linkFrom(BatchOperator.fromDataframe(
            pd.DataFrame({"id": [1, 1, 2], "col": [0, 2, 1], "val": [1.0, 3.0, 2.0]}), schemaStr="id long, col long, val double")).collect()
    assert len(vec) == 2
    anyop = A.TripleToAnyBatchOp().setTripleRowCol("id").setTripleColCol("c").setTripleValCol("v") \
        .setToFormat("KV").setKvCol("o").linkFrom(trip).collect()
    assert len(anyop) == 4
    back = A.AnyToTripleBatchOp().setFromFormat("KV").setKvCol("kv").setReservedCols(["id"]) \
        .setTripleColValSchemaStr("c string, v double").linkFrom(_b()).collect()
    sb = _collect(A.AnyToTripleStreamOp().setFromFormat("KV").setKvCol("kv").setReservedCols(["id"])
                  .setTripleColValSchemaStr("c string, v double").linkFrom(_s()))
    assert len(back) == 8 and _key(back) == _key(sb)
    assert issubclass(A.BaseFormatTransBatchOp, BatchOperator) and issubclass(A.BaseFormatTransStreamOp, StreamOperator)


def test_sources_and_sinks_roundtrip(tmp_path):
    txt = str(tmp_path / "t.txt")
    A.TextSinkBatchOp().setFilePath(txt).linkFrom(_b().select("csv"))
    BatchOperator.execute()
    assert [r[0] for r in A.TextSourceBatchOp().setFilePath(txt).collect()] == list(DF["csv"])
    assert [r[0] for r in _collect(A.TextSourceStreamOp().setFilePath(txt))] == list(DF["csv"])
    txt2 = str(tmp_path / "t2.txt")
    A.TextSinkStreamOp().setFilePath(txt2).linkFrom(_s().select("kv"))
    StreamOperator.execute()
    assert sorted(open(txt2).read().split()) == sorted(DF["kv"])
    lib = str(tmp_path / "d.libsvm")
    A.LibSvmSinkBatchOp().setFilePath(lib).setVectorCol("vec").setLabelCol("id").linkFrom(_b())
    BatchOperator.execute()
    got = A.LibSvmSourceBatchOp().setFilePath(lib).collect()
    assert len(got) == 4 and float(got[0][0]) == 1.0
    assert len(_collect(A.LibSvmSourceStreamOp().setFilePath(lib))) == 4
    lib2 = str(tmp_path / "e.libsvm")
    A.LibSvmSinkStreamOp().setFilePath(lib2).setVectorCol("vec").setLabelCol("id").linkFrom(_s())
    StreamOperator.execute()
    assert len(open(lib2).read().strip().split("\n")) == 4
    assert [r[0] for r in A.NumSeqSourceBatchOp(1, 5).collect()] == [1, 2, 3, 4, 5]
    assert [r[0] for r in _collect(A.NumSeqSourceStreamOp(1, 3))] == [1, 2, 3]
    rt = A.RandomTableSourceBatchOp().setNumRows(10).setNumCols(3).collect()
    assert len(rt) == 10 and len(rt[0]) == 3
    assert len(_collect(A.RandomTableSourceStreamOp().setNumRows(7).setNumCols(2))) == 7
    assert len(_collect(A.RandomVectorSourceStreamOp().setNumRows(5).setSize(4))) == 5
    assert len(_collect(A.TableSourceStreamOp(_b().getOutputTable()))) == 4


def test_print_sample_udtf_stream(capsys):
    from alink_amd.operator.common.sql.udf import udtf
    _s().link(A.PrintStreamOp())
    StreamOperator.execute()
    assert "csv" in capsys.readouterr().out
    n = len(_collect(A.SampleStreamOp().setRatio(1.0).linkFrom(_s())))
    assert n == 4
    split = udtf(lambda s: [(w,) for w in s.split(",")], result_types=["STRING"])
    out = _collect(A.UDTFStreamOp().setFunc(split).setSelectedCols(["csv"]).setOutputCols(["w"]).linkFrom(_s()))
    assert len(out) == 8


def test_map_flatmap_modelmap_bases():
    from alink_amd.common.mapper import FlatMapper, SISOMapper
    from alink_amd.common.types import Types

    class Doubler(SISOMapper):
        def initOutputColType(self):
            return Types.DOUBLE

        def mapColumn(self, v):
            return None if v is None else 2.0 * v

    out = A.MapBatchOp(mapper=Doubler).setSelectedCol("f0").setOutputCol("d").linkFrom(_b()).collect() \
        if hasattr(A.MapBatchOp(), "setSelectedCol") else None
    if out is not None:
        assert [r[-1] for r in out] == [3.0, -4.0, 0.5, 6.0]
    class Splitter(FlatMapper):
        def getOutputSchema(self):
            from alink_amd.common.types import TableSchema
            return TableSchema(["id", "part"], [Types.LONG, Types.STRING])

        def flatMap(self, row):
            return [(row[0], p) for p in row[3].split(",")]

    ids = [r[0] for r in A.FlatMapBatchOp(mapper=Splitter).linkFrom(_b()).collect()]
    assert sorted(ids) == [1, 1, 2, 2, 3, 3, 4, 4]
    sids = _collect(A.FlatMapStreamOp(mapper=Splitter).linkFrom(_s()))
    assert len(sids) == 8
    from alink_amd.models.clustering.kmeans import KMeansModelMapper
    model = A.KMeansTrainBatchOp().setVectorCol("vec").setK(2).linkFrom(_b())
    from alink_amd.common.params import Params
    pred = A.ModelMapBatchOp(Params().set("vectorCol", "vec").set("predictionCol", "p"), mapper=KMeansModelMapper) \
        .linkFrom(model, _b())
    assert len(pred.collect()) == 4
    assert issubclass(A.DataSetWrapperBatchOp, BatchOperator)
    assert issubclass(A.BaseLinearModelTrainBatchOp, BatchOperator)


def test_aft_survival_regression_batch_and_stream():
    rng = np.random.default_rng(0)
    n = 60
    x = rng.normal(size=(n, 2))
    t = np.exp(0.5 * x[:, 0] - 0.3 * x[:, 1] + 0.2 * rng.normal(size=n))
    df = pd.DataFrame({"x0": x[:, 0], "x1": x[:, 1], "t": t, "c": (rng.random(n) < 0.8).astype(float)})
    sch = "x0 double, x1 double, t double, c double"
    model = A.AftSurvivalRegTrainBatchOp().setFeatureCols(["x0", "x1"]).setLabelCol("t").setCensorCol("c") \
        .linkFrom(BatchOperator.fromDataframe(df, schemaStr=sch))
    b = A.AftSurvivalRegPredictBatchOp().setPredictionCol("p").linkFrom(model, BatchOperator.fromDataframe(df, schemaStr=sch))
    s = _collect(A.AftSurvivalRegPredictStreamOp(model).setPredictionCol("p").linkFrom(
        StreamOperator.fromDataframe(df, schemaStr=sch)))
    assert len(b.collect()) == n and _key(b.collect()) == _key(s)
    assert np.corrcoef([r[-1] for r in b.collect()], t)[0, 1] > 0.5


def test_index_to_string_batch_and_stream():
    df = pd.DataFrame({"w": ["x", "y", "x", "z"]})
    src = BatchOperator.fromDataframe(df, schemaStr="w string")
    model = A.StringIndexerTrainBatchOp().setSelectedCol("w").linkFrom(src)
    idx = A.StringIndexerPredictBatchOp().setSelectedCol("w").setOutputCol("i").linkFrom(model, src)
    back = A.IndexToStringPredictBatchOp().setSelectedCol("i").setOutputCol("w2").linkFrom(model, idx).collect()
    assert [r[2] for r in back] == ["x", "y", "x", "z"]
    sidx = StreamOperator.fromDataframe(pd.DataFrame({"i": [int(r[1]) for r in idx.collect()]}), schemaStr="i long")
    sb = _collect(A.IndexToStringPredictStreamOp(model).setSelectedCol("i").setOutputCol("w2").linkFrom(sidx))
    assert sorted(r[1] for r in sb) == ["x", "x", "y", "z"]


def test_eval_multiclass_stream():
    df = pd.DataFrame({"label": ["a", "b", "c", "a"] * 5, "pred": ["a", "b", "b", "a"] * 5,
                       "detail": ['{"a":0.8,"b":0.1,"c":0.1}', '{"a":0.1,"b":0.8,"c":0.1}',
                                  '{"a":0.1,"b":0.6,"c":0.3}', '{"a":0.7,"b":0.2,"c":0.1}'] * 5})
    out = _collect(A.EvalMultiClassStreamOp().setLabelCol("label").setPredictionCol("pred")
                   .setPredictionDetailCol("detail").linkFrom(
                       StreamOperator.fromDataframe(df, schemaStr="label string, pred string, detail string")))
    assert len(out) >= 1


def test_gated_connectors(tmp_path):
    broker = "file://" + str(tmp_path / "kafka")
    _s().select("id, f0").link(A.Kafka010SinkStreamOp().setBootstrapServers(broker).setTopic("t"))
    _s().select("id, f1").link(A.Kafka011SinkStreamOp().setBootstrapServers(broker).setTopic("u"))
    StreamOperator.execute()
    a = _collect(A.Kafka010SourceStreamOp().setBootstrapServers(broker).setTopic("t").setStartupMode("EARLIEST"))
    b = _collect(A.Kafka011SourceStreamOp().setBootstrapServers(broker).setTopic("u").setStartupMode("EARLIEST"))
    assert len(a) == 4 and len(b) == 4
    wh = "file://" + str(tmp_path / "hive")
    _b().select("id, f0").link(A.HiveSinkBatchOp().setHiveConfDir(wh).setOutputTableName("h"))
    assert len(_collect(A.HiveSourceStreamOp().setHiveConfDir(wh).setInputTableName("h"))) == 4
    from alink_amd.operator.common.io.db import SqliteDB
    db = SqliteDB(str(tmp_path / "x.db"))
    _s().select("id, f0").link(A.DBSinkStreamOp(db, "s"))
    StreamOperator.execute()
    assert len(db.read("s").rows()) == 4
    # MySQL needs pymysql / mysql-connector (not installed): the ops fail with a clear message, not silently
    for op in (A.MySqlSinkBatchOp().setDbName("d").setIp("127.0.0.1").setPort("3306").setUsername("u")
               .setPassword("p").setOutputTableName("t"),):
        with pytest.raises(Exception):
            _b().link(op)
            BatchOperator.execute()
    with pytest.raises(Exception):
        _collect(A.MySqlSourceStreamOp().setDbName("d").setIp("127.0.0.1").setPort("3306").setUsername("u")
                 .setPassword("p").setInputTableName("t"))
    with pytest.raises(Exception):
        _s().link(A.MySqlSinkStreamOp().setDbName("d").setIp("127.0.0.1").setPort("3306").setUsername("u")
                  .setPassword("p").setOutputTableName("t"))
        StreamOperator.execute()
