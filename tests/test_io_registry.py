"""IO registry (reference @IoOpAnnotation / AnnotationUtils / Base*Op.of(params))."""
import os

import pandas as pd

from alink_amd import *  # noqa: F401,F403
from alink_amd.common.io_registry import IO_NAME, IO_TYPE, AnnotationUtils, IOType
from alink_amd.operator.batch.sink import BaseSinkBatchOp
from alink_amd.operator.batch.source import BaseSourceBatchOp
from alink_amd.operator.stream.base import StreamSourceOp


def test_annotated_names_match_reference():
    assert AnnotationUtils.annotatedName(CsvSourceBatchOp) == "csv"
    assert AnnotationUtils.annotatedIoType(CsvSourceBatchOp) == IOType.SourceBatch
    assert AnnotationUtils.annotatedName(CsvSinkStreamOp) == "csv"
    assert AnnotationUtils.annotatedName(PrintBatchOp) == "print"
    assert AnnotationUtils.annotatedName(MySqlSourceBatchOp) == "my_sql_batch_source"
    assert {"csv", "text", "libsvm", "db", "print", "sqlite", "mysql"} <= set(AnnotationUtils.allDBAndOpNames())


def test_source_and_sink_of_params_round_trip(tmp_path):
    path = os.path.join(tmp_path, "a.csv")
    with open(path, "w") as f:
        f.write("1,a\n2,b\n3,c\n")
    p = Params().set(IO_NAME, "csv").set(IO_TYPE, "SourceBatch").set("filePath", path) \
        .set("schemaStr", "id long, s string")
    src = BaseSourceBatchOp.of(p)
    assert isinstance(src, CsvSourceBatchOp)
    assert [list(r) for r in src.collect()] == [[1, "a"], [2, "b"], [3, "c"]]
    out = os.path.join(tmp_path, "b.csv")
    sink = BaseSinkBatchOp.of(Params().set(IO_NAME, "csv").set(IO_TYPE, "SinkBatch").set("filePath", out)
                              .set("overwriteSink", True))
    assert isinstance(sink, CsvSinkBatchOp)
    src.link(sink)
    BatchOperator.execute()
    assert open(out).read().split() == ["1,a", "2,b", "3,c"]
    ss = StreamSourceOp.of(p.clone().set(IO_TYPE, "SourceStream"))
    assert isinstance(ss, CsvSourceStreamOp)


def test_db_source_from_params(tmp_path):
    db = SqliteDB(os.path.join(tmp_path, "x.db"))
    df = pd.DataFrame({"k": [1, 2], "v": ["x", "y"]})
    BatchOperator.fromDataframe(df, schemaStr="k long, v string").link(
        DBSinkBatchOp(db, "t1"))
    BatchOperator.execute()
    p = Params().set(IO_NAME, "sqlite").set(IO_TYPE, "SourceBatch").set("dbName", os.path.join(tmp_path, "x.db")) \
        .set("inputTableName", "t1")
    src = BaseSourceBatchOp.of(p)
    assert isinstance(src, DBSourceBatchOp)
    assert sorted(list(r) for r in src.collect()) == [[1, "x"], [2, "y"]]
