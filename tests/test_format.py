"""Format conversion ops (Columns/CSV/JSON/KV/Vector/Triple), JsonValue and the string-to-columns parsers,
checked against the reference docs (docs/en/columnstokvbatchop.md, jsonvaluebatchop.md,
tripletojsonbatchop.md, jsontovectorbatchop.md) and Java HashMap iteration order."""
import json

import numpy as np

import pytest

from alink_amd import *  # noqa: F401,F403
from alink_amd.common.javafmt import java_hashmap_order
from alink_amd.models.dataproc.format import json_path_read, lenient_json_loads

ROWS = [('1', '{"f1":"1.0","f2":"2.0"}', '$3$1:1.0 2:2.0', '1:1.0,2:2.0', '1.0,2.0', 1.0, 2.0),
        ('2', '{"f2":"4.0","f4":"8.0"}', '$3$1:4.0 2:8.0', '1:4.0,2:8.0', '4.0,8.0', 4.0, 8.0)]
SCHEMA = "row string, json string, vec string, kv string, csv string, f0 double, f1 double"


def _data():
    return MemSourceBatchOp(ROWS, SCHEMA)


def test_columns_to_kv_doc():
    out = ColumnsToKvBatchOp().setSelectedCols(["f0", "f1"]).setReservedCols(["row"]).setKvCol("kv") \
        .linkFrom(_data()).collect()
    assert [tuple(r) for r in out] == [("1", "f0:1.0,f1:2.0"), ("2", "f0:4.0,f1:8.0")]


def test_columns_to_json_and_back():
    js = ColumnsToJsonBatchOp().setSelectedCols(["f0", "f1"]).setReservedCols(["row"]).setJsonCol("j") \
        .linkFrom(_data())
    assert [r[1] for r in js.collect()] == ['{"f0":"1.0","f1":"2.0"}', '{"f0":"4.0","f1":"8.0"}']
    back = JsonToColumnsBatchOp().setJsonCol("j").setSchemaStr("f0 double, f1 double").setReservedCols(["row"]) \
        .linkFrom(js).collect()
    assert [tuple(r) for r in back] == [("1", 1.0, 2.0), ("2", 4.0, 8.0)]


def test_json_to_vector_doc():
    src = MemSourceBatchOp([('1', '{"1":"1.0","2":"2.0"}'), ('2', '{"2":"4.0","4":"8.0"}')], "row string, json string")
    out = JsonToVectorBatchOp().setJsonCol("json").setReservedCols(["row"]).setVectorCol("vec").setVectorSize(5) \
        .linkFrom(src).collect()
    assert [r[1] for r in out] == ["$5$1:1.0 2:2.0", "$5$2:4.0 4:8.0"]


def test_columns_to_vector_and_csv():
    out = ColumnsToVectorBatchOp().setSelectedCols(["f0", "f1"]).setVectorCol("v").setReservedCols(["row"]) \
        .linkFrom(_data()).collect()
    assert [r[1] for r in out] == ["1.0 2.0", "4.0 8.0"]
    out = ColumnsToCsvBatchOp().setSelectedCols(["f0", "f1"]).setSchemaStr("f0 double, f1 double").setCsvCol("c") \
        .setReservedCols(["row"]).linkFrom(_data()).collect()
    assert [r[1] for r in out] == ["1.0,2.0", "4.0,8.0"]


def test_vector_to_columns_format_flavour():
    out = VectorToColumnsBatchOp().setVectorCol("vec").setSchemaStr("f0 double, f1 double, f2 double") \
        .setReservedCols(["row"]).linkFrom(_data()).collect()
    assert [tuple(r) for r in out] == [("1", 0.0, 1.0, 2.0), ("2", 0.0, 4.0, 8.0)]


def test_csv_kv_to_columns():
    out = CsvToColumnsBatchOp().setCsvCol("csv").setSchemaStr("a double, b double").setReservedCols(["row"]) \
        .linkFrom(_data()).collect()
    assert [tuple(r) for r in out] == [("1", 1.0, 2.0), ("2", 4.0, 8.0)]
    out = KvToColumnsBatchOp().setKvCol("kv").setSchemaStr("1 double, 2 double").setReservedCols(["row"]) \
        .linkFrom(_data()).collect()
    assert [tuple(r) for r in out] == [("1", 1.0, 2.0), ("2", 4.0, 8.0)]


def test_triple_round_trip():
    t = MemSourceBatchOp([(1.0, 'f1', 1.0), (1.0, 'f2', 2.0), (2.0, 'f1', 4.0), (2.0, 'f2', 8.0)],
                         "row double, col string, val double")
    out = TripleToJsonBatchOp().setTripleRowCol("row").setTripleColCol("col").setTripleValCol("val") \
        .setJsonCol("json").linkFrom(t).collect()
    assert [tuple(r) for r in out] == [(1.0, '{"f1":"1.0","f2":"2.0"}'), (2.0, '{"f1":"4.0","f2":"8.0"}')]
    cols = TripleToColumnsBatchOp().setTripleRowCol("row").setTripleColCol("col").setTripleValCol("val") \
        .setSchemaStr("f1 double, f2 double").linkFrom(t).collect()
    assert [tuple(r) for r in cols] == [(1.0, 1.0, 2.0), (2.0, 4.0, 8.0)]
    trip = ColumnsToTripleBatchOp().setSelectedCols(["f0", "f1"]).setReservedCols(["row"]) \
        .setTripleColValSchemaStr("col string, val double").linkFrom(_data()).collect()
    assert [tuple(r) for r in trip] == [("1", "f0", 1.0), ("1", "f1", 2.0), ("2", "f0", 4.0), ("2", "f1", 8.0)]


def test_json_value_doc_lenient_json():
    j = MemSourceBatchOp([("{a:boy,b:{b1:1,b2:2}}",), ("{a:girl,b:{b1:1,b2:2}}",)], "str string")
    out = JsonValueBatchOp().setJsonPath(["$.a", "$.b.b1"]).setSelectedCol("str").setOutputCols(["f0", "f1"]) \
        .linkFrom(j).collect()
    assert [tuple(r) for r in out] == [("{a:boy,b:{b1:1,b2:2}}", "boy", "1"), ("{a:girl,b:{b1:1,b2:2}}", "girl", "1")]
    assert json_path_read(lenient_json_loads('{"a":[1,{"x":"y"}]}'), "$.a[1].x") == "y"
    assert json_path_read({"a": [1, 2]}, "$.a[*]") == [1, 2]


def test_hashmap_order_in_kv_writer():
    # 17 keys forces a resize (cap 32); order must follow java.util.HashMap bucket order, not insertion
    keys = [f"k{i}" for i in range(17)]
    row = tuple(float(i) for i in range(17))
    src = MemSourceBatchOp([row], ", ".join(f"{k} double" for k in keys))
    kv = ColumnsToKvBatchOp().setSelectedCols(keys).setKvCol("kv").setReservedCols([]).linkFrom(src).collect()[0][0]
    assert [p.split(":")[0] for p in kv.split(",")] == java_hashmap_order(keys)


def test_stream_and_pipeline_twins():
    s = MemSourceStreamOp(ROWS, SCHEMA)
    box = []
    ColumnsToKvStreamOp().setSelectedCols(["f0", "f1"]).setReservedCols(["row"]).setKvCol("kv").linkFrom(s) \
        .link(CollectStreamOp(box))
    StreamOperator.execute()
    assert [tuple(r) for r in box] == [("1", "f0:1.0,f1:2.0"), ("2", "f0:4.0,f1:8.0")]
    p = Pipeline(ColumnsToKv().setSelectedCols(["f0", "f1"]).setKvCol("kv2"), Select("row, kv2"))
    assert [tuple(r) for r in p.fit(_data()).transform(_data()).collect()] == \
        [("1", "f0:1.0,f1:2.0"), ("2", "f0:4.0,f1:8.0")]


def test_polynomial_expansion_reference_order():
    """PolynomialExpansionMapperTest (reference operator/common/dataproc/vector): Spark's monomial order, dense in
    -> dense out, sparse in -> sparse out, sizes C(n + d, d) - 1."""
    from alink_amd import VectorPolynomialExpandBatchOp
    from alink_amd.common.linalg import DenseVector, SparseVector
    from alink_amd.models.dataproc.vector import poly_size
    from alink_amd.operator.batch.source import MemSourceBatchOp
    src = MemSourceBatchOp([(DenseVector([3.0, 4.0]),), (SparseVector(3, [0, 2], [2.0, 3.0]),)], "vec vector")
    out = VectorPolynomialExpandBatchOp().setSelectedCol("vec").setOutputCol("res").setDegree(2).linkFrom(src) \
        .collect()
    assert out[0][1] == DenseVector([3.0, 9.0, 4.0, 12.0, 16.0])
    assert out[1][1] == SparseVector(9, [0, 1, 5, 6, 8], [2.0, 4.0, 3.0, 6.0, 9.0])
    assert poly_size(4, 4) == 70 and poly_size(65, 2) == 2211
    d3 = VectorPolynomialExpandBatchOp().setSelectedCol("vec").setDegree(3).linkFrom(
        MemSourceBatchOp([(DenseVector([2.0, 0.0, 1.5]),)], "vec vector")).collect()[0][0]
    sp3 = VectorPolynomialExpandBatchOp().setSelectedCol("vec").setDegree(3).linkFrom(
        MemSourceBatchOp([(SparseVector(3, [0, 2], [2.0, 1.5]),)], "vec vector")).collect()[0][0]
    np.testing.assert_array_equal(sp3.toDenseVector().getData(), d3.getData())   # same monomials either way


def test_string_parsers_reference_cases():
    """StringParsersTest (reference operator/common/dataproc): JSON with numbers of every form, KV with date /
    time / timestamp columns, CSV with a multi-character separator."""
    import datetime
    from alink_amd.operator.batch.source import MemSourceBatchOp
    kv = "f1=1,f2=2.0,f3=false,f4=val,f5=2018-09-10,f6=14:22:20,f7=2018-09-10 14:22:20"
    out = KvToColumnsBatchOp().setKvCol("kv").setKvValDelimiter("=").setSchemaStr(
        "f1 bigint, f2 double, f3 boolean, f4 string, f5 date, f6 time, f7 timestamp").linkFrom(
        MemSourceBatchOp([(kv,)], "kv string")).collect()[0]
    assert tuple(out[1:]) == (1, 2.0, False, "val", datetime.date(2018, 9, 10), datetime.time(14, 22, 20),
                              datetime.datetime(2018, 9, 10, 14, 22, 20))
    js = ('{\n  "media_name": "Titanic",\n  "title": "Titanic",\n  "compare_point": 0.0001,\n  "spider_point": 0.0000,'
          '\n  "search_point": 0.6,\n  "collection_id": 123456,\n  "media_id": 3214\n}')
    out = JsonToColumnsBatchOp().setJsonCol("j").setSchemaStr(
        "media_name string, title string, compare_point double, spider_point double, search_point double, "
        "collection_id bigint, media_id bigint").linkFrom(MemSourceBatchOp([(js,)], "j string")).collect()[0]
    assert tuple(out[1:]) == ("Titanic", "Titanic", 0.0001, 0.0, 0.6, 123456, 3214)
    out = CsvToColumnsBatchOp().setCsvCol("c").setFieldDelimiter("____").setSchemaStr(
        "a string, b string, c2 string").linkFrom(MemSourceBatchOp([("hello_____world____",)], "c string")).collect()
    assert tuple(out[0][1:]) == ("hello", "_world", None)


def test_vector_mappers_reference_values():
    """Vector{Interaction,ElementwiseProduct,Normalize,Slice}MapperTest (reference operator/common/dataproc/vector)."""
    from alink_amd.common.linalg import DenseVector, SparseVector
    from alink_amd.operator.batch.source import MemSourceBatchOp

    def run(op, *vals, schema="vec vector"):
        return op.linkFrom(MemSourceBatchOp([tuple(vals)], schema)).collect()[0][-1]
    d34 = DenseVector([3.0, 4.0])
    assert run(VectorInteractionBatchOp().setSelectedCols(["a", "b"]).setOutputCol("o"), d34, d34,
               schema="a vector, b vector") == DenseVector([9.0, 12.0, 12.0, 16.0])
    assert run(VectorInteractionBatchOp().setSelectedCols(["a", "b"]).setOutputCol("o"), d34,
               DenseVector([1.0, 2.0, 5.0]), schema="a vector, b vector") == \
        DenseVector([3.0, 6.0, 15.0, 4.0, 8.0, 20.0])                       # a_i * b_j at i * |b| + j
    s = SparseVector(10, [0, 9], [1.0, 4.0])
    assert run(VectorInteractionBatchOp().setSelectedCols(["a", "b"]).setOutputCol("o"), s, s,
               schema="a vector, b vector") == SparseVector(100, [0, 9, 90, 99], [1.0, 4.0, 4.0, 16.0])
    assert run(VectorElementwiseProductBatchOp().setSelectedCol("vec").setScalingVector("3.0 4.5"), d34) == \
        DenseVector([9.0, 18.0])
    assert run(VectorElementwiseProductBatchOp().setSelectedCol("vec").setOutputCol("res")
               .setScalingVector("$10$1:3.0 2:10.0 9:4.5"), SparseVector(10, [1, 5, 9], [2.0, 4.0, 3.0])) == \
        SparseVector(10, [1, 5, 9], [6.0, 0.0, 13.5])
    assert run(VectorNormalizeBatchOp().setSelectedCol("vec").setP(2.0), d34) == DenseVector([0.6, 0.8])
    assert run(VectorNormalizeBatchOp().setSelectedCol("vec").setOutputCol("res").setP(1.0),
               DenseVector([2.0, 3.0])) == DenseVector([0.4, 0.6])
    assert run(VectorSliceBatchOp().setSelectedCol("vec").setIndices([0, 1]), DenseVector([3.0, 4.0, 3.0])) == d34


def test_triple_to_any_reference_constructor():
    """TripleToAnyBatchOpTest: the reference's (FormatType, Params) constructor; 8 triples over 4 row ids give 4
    KV rows and 4 vector rows."""
    import alink_amd as A
    from alink_amd.common.params import Params
    from alink_amd.operator.batch.source import MemSourceBatchOp
    rows = [(1, 1, 1.0), (1, 2, 1.0), (2, 3, 1.0), (3, 4, 1.0), (4, 2, 1.0), (3, 1, 1.0), (2, 4, 1.0), (4, 1, 1.0)]
    data = MemSourceBatchOp(rows, ["start", "dest", "weight"])
    base = Params().set("tripleRowCol", "start").set("tripleColCol", "dest").set("tripleValCol", "weight")
    kv = A.TripleToAnyBatchOp("KV", base.clone().set("kvCol", "kv")).linkFrom(data).collect()
    assert sorted(tuple(r) for r in kv) == [(1, "1:1.0,2:1.0"), (2, "3:1.0,4:1.0"), (3, "1:1.0,4:1.0"),
                                            (4, "1:1.0,2:1.0")]
    vec = A.TripleToAnyBatchOp("VECTOR", base.clone().set("vectorCol", "vec")).linkFrom(data).collect()
    assert len(vec) == 4
    trans = A.BaseFormatTransBatchOp("KV", "COLUMNS", Params().set("kvCol", "kv").set("schemaStr", "1 double"))
    assert trans.getParams().get("fromFormat") == "KV" and trans.getParams().get("toFormat") == "COLUMNS"


def test_vector_size_hint_slice_to_columns_mappers_reference():
    """VectorSizeHintMapperTest / VectorSliceMapperTest / VectorToColumnsMapperTest."""
    from alink_amd.common.linalg import DenseVector, SparseVector
    from alink_amd.common.params import Params
    from alink_amd.common.types import schema_str_to_schema
    from alink_amd.models.dataproc import vector as V
    s = schema_str_to_schema("vec string")
    m = V.VectorSizeHintMapper(s, Params().set("selectedCol", "vec").set("size", 3))
    assert m.getOutputSchema().getFieldNames() == ["vec"]
    m = V.VectorSizeHintMapper(s, Params().set("selectedCol", "vec").set("outputCol", "res")
                               .set("handleInvalid", "SKIP").set("size", 2))
    assert m.getOutputSchema().getFieldNames() == ["vec", "res"]
    m = V.VectorSliceMapper(s, Params().set("selectedCol", "vec").set("indices", [0, 1]))
    assert str(m.map((DenseVector([3.0, 4.0, 3.0]),))[0]) == "3.0 4.0"
    m = V.VectorSliceMapper(s, Params().set("selectedCol", "vec").set("outputCol", "res").set("reservedCols", [])
                            .set("indices", [0, 2, 4]))
    assert str(m.map((SparseVector(5, [0, 2, 4], [3.0, 4.0, 3.0]),))[0]) == "$3$0:3.0 1:4.0 2:3.0"
    m = V.VectorToColumnsMapper(s, Params().set("selectedCol", "vec").set("outputCols", ["f0", "f1"]))
    assert tuple(m.map((DenseVector([3.0, 4.0]),)))[1:] == (3.0, 4.0)
    assert m.getOutputSchema().getFieldNames() == ["vec", "f0", "f1"]
    m = V.VectorToColumnsMapper(s, Params().set("selectedCol", "vec").set("outputCols", ["f0", "f1", "f2"])
                                .set("reservedCols", []))
    assert tuple(m.map((SparseVector(3, [1, 2], [3.0, 4.0]),))) == (0.0, 3.0, 4.0)
