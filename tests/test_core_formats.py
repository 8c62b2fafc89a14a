"""Params / vector / model-table formats against the reference's golden strings."""
import numpy as np
import pytest

from alink_amd.common.javafmt import java_double_str, java_hashmap_order
from alink_amd.common.linalg import DenseVector, SparseVector, VectorUtil
from alink_amd.common.params import Params, ParamInfo
from alink_amd.common.model import get_model_id, extract_meta_and_data, SEGMENT_SIZE
from alink_amd.common.types import schema_str_to_schema, schema_to_schema_str, Types

KMEANS_META = ('{"vectorCol":"\\"Y\\"","latitudeCol":null,"longitudeCol":null,'
               '"distanceType":"\\"EUCLIDEAN\\"","k":"2","vectorSize":"3"}')
KMEANS_ROWS = [
    (0, KMEANS_META),
    (1048576, '{"clusterId":0,"weight":3.0,"vec":{"data":[9.1,9.1,9.1]}}'),
    (2097152, '{"clusterId":1,"weight":3.0,"vec":{"data":[0.1,0.1,0.1]}}'),
]


def test_java_double_format():
    assert java_double_str(3.0) == "3.0"
    assert java_double_str(1e-4) == "1.0E-4"
    assert java_double_str(1e7) == "1.0E7"
    assert java_double_str(0.010869565217391353) == "0.010869565217391353"
    assert java_double_str(-0.0) == "-0.0"
    assert java_double_str(float("nan")) == "NaN"


def test_params_json_matches_java_hashmap_order():
    # golden meta row from KMeansModelMapperTest.java:21-24
    from alink_amd.models.clustering.kmeans import KMeansTrainModelData
    md = KMeansTrainModelData([], 2, 3, "EUCLIDEAN", "Y")
    assert md.to_params().toJson() == KMEANS_META


def test_params_alias_default_and_roundtrip():
    p = Params()
    info = ParamInfo("maxIter", int, "", default=20, alias=["numIter"])
    assert p.get(info) == 20
    p.set("numIter", 7)
    assert p.get(info) == 7
    q = Params.fromJson(p.toJson())
    assert q.get(info) == 7


def test_params_validator_enforced():
    from alink_amd.common.params import RangeValidator, ParamValidationError
    info = ParamInfo("k", int, "", default=2, validator=RangeValidator(1, None))
    with pytest.raises(ParamValidationError):
        Params().set(info, 0)


def test_vector_formats():
    v = VectorUtil.parse("$5$1:2.0 3:4.5")
    assert isinstance(v, SparseVector) and v.size() == 5
    assert VectorUtil.toString(v) == "$5$1:2.0 3:4.5"
    d = VectorUtil.parse("1 2 3")
    assert isinstance(d, DenseVector) and VectorUtil.toString(d) == "1.0 2.0 3.0"
    assert VectorUtil.parse("1,2,3").size() == 3
    assert VectorUtil.toString(SparseVector(-1, [0, 2], [1.0, 0.5])) == "0:1.0 2:0.5"
    assert abs(d.dot(v.toDenseVector()) if d.size() == 5 else 1.0) >= 0


def test_model_table_roundtrip_and_slicing():
    from alink_amd.common.model import SimpleModelDataConverter

    class C(SimpleModelDataConverter):
        def serializeModel(self, m):
            p = Params().set("n", len(m))
            return p, m

        def deserializeModel(self, meta, data):
            return list(data)

    big = "x" * (SEGMENT_SIZE * 2 + 5)
    rows = C().save(["a", big, "c"])
    ids = [r[0] for r in rows]
    assert ids[0] == 0 and get_model_id(2, 2) in ids
    rows = list(reversed(rows))  # loading must sort by model_id
    assert C().load(rows) == ["a", big, "c"]


def test_kmeans_model_converter_golden():
    from alink_amd.models.clustering.kmeans import KMeansModelDataConverter
    m = KMeansModelDataConverter().load(KMEANS_ROWS)
    assert m.k == 2 and m.centroids.shape == (2, 3)
    assert np.allclose(m.centroids[0], 9.1)


def test_schema_strings():
    s = schema_str_to_schema("f0 int, f1 bigint,f2 string, v VEC_TYPES_VECTOR")
    assert s.types == [Types.INT, Types.LONG, Types.STRING, Types.VECTOR]
    assert schema_to_schema_str(s) == "f0 INT,f1 BIGINT,f2 VARCHAR,v VEC_TYPES_VECTOR"


def test_hashmap_order_examples():
    assert java_hashmap_order(["distanceType", "k", "vectorSize", "vectorCol", "latitudeCol", "longitudeCol"]) == \
        ["vectorCol", "latitudeCol", "longitudeCol", "distanceType", "k", "vectorSize"]


def test_native_java_double_join_matches_python_formatter():
    """The C++ Double.toString formatter used for large model vectors (snapshots) gives the same strings as the
    Python reference formatter, edge cases included."""
    import numpy as np
    from alink_amd import _native
    from alink_amd.common.javafmt import java_double_str, gson_dumps
    if _native.lib is None or getattr(_native.lib, "alink_java_double_join", None) is None:
        import pytest
        pytest.skip("native runtime not built")
    rng = np.random.default_rng(3)
    xs = np.concatenate([rng.normal(size=5000) * 10.0 ** rng.integers(-15, 15, size=5000),
                         [0.0, -0.0, 1e-3, 9.99e-4, 1e7, 9999999.999999998, 1.0, -100.0, float("nan"), float("inf"),
                          -float("inf"), 5e-324, 1.7976931348623157e308, 0.1 + 0.2, 1e21, 1e-5, 123456789.0]])
    assert _native.java_double_join(xs).split(",") == [java_double_str(float(v)) for v in xs]
    assert gson_dumps(xs) == "[" + ",".join(java_double_str(float(v)) for v in xs) + "]"
