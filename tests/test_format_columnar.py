"""Columnar fast paths of the format conversions (``models/dataproc/format.py``: COLUMNS<->VECTOR, COLUMNS->CSV,
CSV->COLUMNS, ``CsvToColumnsMapper``): on every input — including the ones outside the fast path's conditions,
which fall back — the output equals the reader -> map -> writer row path cell for cell (repr, so NaN / -0.0 /
integer-vs-float differences count)."""
import numpy as np
import pytest
import torch

from alink_amd.common.mapper import Mapper
from alink_amd.common.params import Params
from alink_amd.common.table import Column, MTable
from alink_amd.common.types import TableSchema, Types
from alink_amd.models.dataproc import format as F


def _doubles(n, rng):
    x = rng.normal(size=n) * 10.0 ** rng.integers(-12, 12, size=n)
    x[rng.random(n) < 0.05] = 0.0
    x[rng.random(n) < 0.03] = -0.0
    x[rng.random(n) < 0.02] = np.nan
    x[rng.random(n) < 0.02] = np.inf
    x[rng.random(n) < 0.02] = 1e300
    x[rng.random(n) < 0.02] = 5e-324
    return x


def _both(m, mt):
    fast = m.map_table(mt)
    slow = m.helper.result_table(mt, Mapper._map_columns(m, mt))   # the per-row reader -> writer path
    rf = [[repr(v) for v in r] for r in fast.rows()]
    rs = [[repr(v) for v in r] for r in slow.rows()]
    assert rf == rs
    return fast


def _num_table(k, n, rng, nulls=False):
    names = [f"c{i}" for i in range(k)]
    cols = []
    for _ in range(k):
        nm = torch.from_numpy(rng.random(n) < 0.1) if nulls else None
        cols.append(Column(torch.from_numpy(_doubles(n, rng)), nm))
    return MTable(TableSchema(names, [Types.DOUBLE] * k), cols), names


@pytest.mark.parametrize("size", [-1, 3, 9])
def test_columns_to_vector_fast_equals_rows(size):
    rng = np.random.default_rng(size + 5)
    mt, names = _num_table(5, 400, rng)
    p = Params().set("fromFormat", "COLUMNS").set("toFormat", "VECTOR").set("selectedCols", names) \
        .set("vectorCol", "vec").set("vectorSize", size)
    m = F.FormatTransMapper(mt.schema, p)
    assert m._fast(m, mt) is not None
    _both(m, mt)
    mtn, _ = _num_table(5, 200, rng, nulls=True)                 # nulls: row path ("null" cells)
    assert m._fast(m, mtn) is None
    _both(m, mtn)


@pytest.mark.parametrize("delim", [",", "\t", "|"])
def test_columns_to_csv_fast_equals_rows(delim):
    rng = np.random.default_rng(len(delim) + ord(delim))
    mt, names = _num_table(4, 300, rng)
    p = Params().set("fromFormat", "COLUMNS").set("toFormat", "CSV").set("selectedCols", names) \
        .set("csvCol", "csv").set("schemaStr", ", ".join(f"{c} double" for c in names)) \
        .set("csvFieldDelimiter", delim)
    m = F.FormatTransMapper(mt.schema, p)
    assert m._fast(m, mt) is not None
    _both(m, mt)
    p2 = p.clone().set("csvFieldDelimiter", ".")                 # separator inside the numbers: row path quotes
    m2 = F.FormatTransMapper(mt.schema, p2)
    assert m2._fast(m2, mt) is None
    _both(m2, mt)


def _vec_strings(n, d, rng):
    out = []
    for i in range(n):
        k = int(rng.integers(0, d + 1))
        v = _doubles(k, rng)
        v[~np.isfinite(v)] = 1.5
        sep = ", " if i % 3 == 0 else " "
        out.append(sep.join(repr(float(x)) for x in v))
    return out


def test_vector_to_columns_fast_equals_rows():
    rng = np.random.default_rng(11)
    strs = _vec_strings(300, 6, rng)
    mt = MTable(TableSchema(["id", "vec"], [Types.LONG, Types.STRING]),
                [Column(torch.arange(300)), Column(strs)])
    p = Params().set("fromFormat", "VECTOR").set("toFormat", "COLUMNS").set("vectorCol", "vec") \
        .set("schemaStr", "f0 double, f1 double, f2 double, f3 double, f4 double, f5 double") \
        .set("reservedCols", ["id"])
    m = F.FormatTransMapper(mt.schema, p)
    assert m._fast(m, mt) is not None
    _both(m, mt)
    # NaN / sparse / over-long vectors -> row path
    for bad in ("NaN 1.0", "$6$0:1.0 3:2.0", "1 2 3 4 5 6 7"):
        mt2 = MTable(mt.schema, [Column(torch.arange(3)), Column(["1.0 2.0", bad, "3.0"])])
        assert m._fast(m, mt2) is None
        _both(m, mt2)
    # a dense 2-D tensor vector column
    X = torch.from_numpy(rng.normal(size=(50, 4)))
    mt3 = MTable(TableSchema(["id", "vec"], [Types.LONG, Types.DENSE_VECTOR]), [Column(torch.arange(50)), Column(X)])
    m3 = F.FormatTransMapper(mt3.schema, p)
    assert m3._fast(m3, mt3) is not None
    _both(m3, mt3)


def _csv_lines(n, rng, full=False):
    out = []
    for i in range(n):
        s = ["plain", "", 'with "q"', "a,b", "x"][i % 5]
        q = '"' + s.replace('"', '""') + '"' if ("," in s or '"' in s) else s
        d = "" if i % 7 == 0 and not full else repr(float(rng.normal()))
        li = "" if i % 11 == 0 and not full else str(int(rng.integers(-10 ** 12, 10 ** 12)))
        b = ["true", "false", "" if not full else "true"][i % 3]
        out.append(",".join([d, li, q, b, str(int(rng.integers(-100, 100)))]))
    return out


@pytest.mark.parametrize("how", ["ERROR", "SKIP"])
def test_csv_to_columns_fast_equals_rows(how):
    rng = np.random.default_rng(3)
    schema_str = "d double, l long, s string, b boolean, i int"
    lines = _csv_lines(200, rng)
    mt = MTable(TableSchema(["csv"], [Types.STRING]), [Column(lines)])
    p = Params().set("fromFormat", "CSV").set("toFormat", "COLUMNS").set("csvCol", "csv") \
        .set("schemaStr", schema_str).set("handleInvalid", how)
    m = F.FormatTransMapper(mt.schema, p)
    assert m._fast(m, mt) is None                          # empty typed fields: ColumnsWriter's row path
    if how == "SKIP":
        _both(m, mt)
    full = _csv_lines(200, rng, full=True)
    mtf = MTable(mt.schema, [Column(full)])
    assert m._fast(m, mtf) is not None
    _both(m, mtf)
    m2 = F.CsvToColumnsMapper(mt.schema, Params().set("selectedCol", "csv").set("schemaStr", schema_str)
                              .set("handleInvalid", how))
    assert F.csv_columns_fast(lines, m2.types, m2.parser.delim, m2.parser.quote) is not None
    _both(m2, mt)
    if how == "SKIP":                                          # an unparsable number / int overflow: row path
        for extra in ("1.0,notanumber,s,true,1", "1.0,1,s,true,99999999999"):
            mt2 = MTable(mt.schema, [Column(lines[:5] + [extra])])
            assert F.csv_columns_fast(lines[:5] + [extra], m2.types, ",", '"') is None
            _both(m2, mt2)
            _both(m, mt2)


def _kv_lines(n, rng, keys, holes=False, dup=False):
    out = []
    for i in range(n):
        ks = list(keys) + ["extra"]
        rng.shuffle(ks)
        if holes and i % 5 == 0:
            ks = ks[1:]
        if dup and i == n // 2:
            ks.append(ks[0])
        out.append(",".join(f"{k}:{repr(float(rng.normal() * 10.0 ** int(rng.integers(-5, 5))))}" for k in ks))
    return out


@pytest.mark.parametrize("holes", [False, True])
@pytest.mark.parametrize("how", ["ERROR", "SKIP"])
def test_kv_to_columns_fast_equals_rows(holes, how):
    rng = np.random.default_rng(13)
    keys = ["k0", "k1", "k2", "k3"]
    schema_str = ", ".join(f"{k} double" for k in keys)
    lines = _kv_lines(300, rng, keys, holes=holes)
    mt = MTable(TableSchema(["kv"], [Types.STRING]), [Column(lines)])
    m = F.FormatTransMapper(mt.schema, Params().set("fromFormat", "KV").set("toFormat", "COLUMNS")
                            .set("kvCol", "kv").set("schemaStr", schema_str).set("handleInvalid", how))
    assert m._fast(m, mt) is not None                      # missing keys are NULL cells for FormatTrans
    _both(m, mt)
    m2 = F.KvToColumnsMapper(mt.schema, Params().set("selectedCol", "kv").set("schemaStr", schema_str)
                             .set("handleInvalid", how))
    fast = F.kv_columns_fast(mt.cols[0], m2.names, m2.types, ",", ":", need_all=m2.err, allow_dup=False)
    assert (fast is None) == (holes and how == "ERROR")
    if not (holes and how == "ERROR"):
        _both(m2, mt)
    # outside the plain form -> row path (whitespace, empty field, duplicate key for KvToColumns)
    for bad in ("k0: 1.0,k1:2,k2:3,k3:4", "k0:1,,k1:2,k2:3,k3:4", "k0:1,k0:2,k1:2,k2:3,k3:4"):
        mt2 = MTable(mt.schema, [Column(lines[:3] + [bad])])
        assert F.kv_columns_fast(mt2.cols[0], m2.names, m2.types, ",", ":", need_all=False, allow_dup=False) is None
        if how == "SKIP":
            _both(m2, mt2)


def _json_lines(n, rng, keys, holes=False):
    import json as _json
    out = []
    for i in range(n):
        d = {}
        for k in keys + ["note"]:
            if holes and i % 4 == 0 and k == keys[0]:
                continue
            if k == "note":
                d[k] = "x"
            elif i % 7 == 0:
                d[k] = int(rng.integers(-5, 5))                # integers, -0 written by hand below
            else:
                d[k] = float(rng.normal() * 10.0 ** int(rng.integers(-8, 8)))
        s = _json.dumps(d, separators=(",", ":") if i % 2 else (", ", ": "))
        out.append(s.replace('": 0,', '": -0,') if i % 9 == 0 else s)
    return out


@pytest.mark.parametrize("holes", [False, True])
@pytest.mark.parametrize("how", ["ERROR", "SKIP"])
def test_json_to_columns_fast_equals_rows(holes, how):
    rng = np.random.default_rng(17)
    keys = ["a", "b_2", "c"]
    schema_str = ", ".join(f"{k} double" for k in keys)
    lines = _json_lines(300, rng, keys, holes=holes)
    mt = MTable(TableSchema(["js"], [Types.STRING]), [Column(lines)])
    m = F.FormatTransMapper(mt.schema, Params().set("fromFormat", "JSON").set("toFormat", "COLUMNS")
                            .set("jsonCol", "js").set("schemaStr", schema_str).set("handleInvalid", how))
    assert m._fast(m, mt) is not None
    _both(m, mt)
    m2 = F.JsonToColumnsMapper(mt.schema, Params().set("selectedCol", "js").set("schemaStr", schema_str)
                               .set("handleInvalid", how))
    fast = F.json_columns_fast(mt.cols[0], m2.names, m2.types, need_all=m2.err)
    assert (fast is None) == (holes and how == "ERROR")
    if not (holes and how == "ERROR"):
        _both(m2, mt)
    # outside the plain form -> the JSON reader (null / string / nested values, lenient syntax, escapes)
    for bad in ('{"a":null,"b_2":1,"c":2}', '{"a":"1.5","b_2":1,"c":2}', "{a:1,b_2:2,c:3}",
                '{"a":[1],"b_2":1,"c":2}', '{"a\\u0041":1,"a":1,"b_2":1,"c":2}'):
        mt2 = MTable(mt.schema, [Column(lines[:3] + [bad])])
        assert F.json_columns_fast(mt2.cols[0], m2.names, m2.types, need_all=False) is None
        if how == "SKIP":
            _both(m2, mt2)


@pytest.mark.parametrize("to", ["KV", "JSON"])
def test_columns_to_kv_json_fast_equals_rows(to):
    rng = np.random.default_rng(23)
    mt, names = _num_table(6, 300, rng)
    p = Params().set("fromFormat", "COLUMNS").set("toFormat", to).set("selectedCols", names) \
        .set("kvCol", "out").set("jsonCol", "out")
    m = F.FormatTransMapper(mt.schema, p)
    assert m._fast(m, mt) is not None
    _both(m, mt)
    mtn, _ = _num_table(6, 100, rng, nulls=True)            # nulls drop keys row by row: row path
    assert m._fast(m, mtn) is None
    _both(m, mtn)


@pytest.mark.parametrize("to", ["VECTOR", "CSV", "KV", "JSON"])
def test_csv_to_writers_fast_equals_rows(to):
    """CSV (all-DOUBLE schema) into the VECTOR / CSV / KV / JSON writers: one C++ parse, one C++ format pass."""
    rng = np.random.default_rng(29)
    names = ["x0", "x1", "x2", "x3"]
    X = _doubles(4 * 200, rng).reshape(200, 4)
    X[~np.isfinite(X)] = 2.5
    lines = [",".join(repr(float(v)) for v in row) for row in X]
    mt = MTable(TableSchema(["csv"], [Types.STRING]), [Column(lines)])
    p = Params().set("fromFormat", "CSV").set("toFormat", to).set("csvCol", "csv") \
        .set("schemaStr", ", ".join(f"{c} double" for c in names)).set("vectorCol", "o").set("kvCol", "o") \
        .set("jsonCol", "o")
    if to == "CSV":
        p = p.set("csvFieldDelimiter", ",")
    m = F.FormatTransMapper(mt.schema, p)
    assert m._fast(m, mt) is not None
    _both(m, mt)
    mt2 = MTable(mt.schema, [Column(lines[:5] + ["1.0,,2.0,3.0"])])   # an empty field: the row path
    assert m._fast(m, mt2) is None


@pytest.mark.parametrize("to", ["CSV", "KV", "JSON"])
@pytest.mark.parametrize("named", [False, True])
def test_vector_to_writers_fast_equals_rows(to, named):
    """Dense VECTOR (all rows of the reader's width; with or without a schema) into the CSV / KV / JSON writers."""
    rng = np.random.default_rng(31)
    X = _doubles(5 * 150, rng).reshape(150, 5)
    X[~np.isfinite(X)] = -3.25
    strs = [" ".join(repr(float(v)) for v in row) for row in X]
    mt = MTable(TableSchema(["vec"], [Types.STRING]), [Column(strs)])
    p = Params().set("fromFormat", "VECTOR").set("toFormat", to).set("vectorCol", "vec").set("kvCol", "o") \
        .set("jsonCol", "o").set("csvCol", "o")
    if named or to == "CSV":
        p = p.set("schemaStr", "a double, b double, c double, d double, e double")
    m = F.FormatTransMapper(mt.schema, p)
    fast_ok = not (to == "JSON" and not (named or to == "CSV"))   # digit keys are not plain JSON names
    assert (m._fast(m, mt) is not None) == fast_ok
    _both(m, mt)
    mt2 = MTable(mt.schema, [Column(strs[:4] + ["1.0 2.0"])])       # a shorter row: the row path
    assert m._fast(m, mt2) is None
    _both(m, mt2)


@pytest.mark.parametrize("flavour", ["outputCols", "schemaStr"])
def test_vector_to_columns_columnar_equals_rows(flavour):
    """VectorToColumns on a dense tensor vector column (both flavours) equals the per-row mapping (schema columns
    past the vector's width: 0.0)."""
    import torch
    from alink_amd.common.params import Params
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.dataproc.vector import VectorToColumnsMapper
    V = torch.randn(9, 3, dtype=torch.float64)
    mt = MTable(TableSchema(["v"], [Types.DENSE_VECTOR]), [Column(V)])
    p = Params().set("selectedCol", "v").set("reservedCols", [])
    p = p.set("outputCols", ["a", "b", "c"]) if flavour == "outputCols" else \
        p.set("schemaStr", "a double, b double, c double, d double")
    m = VectorToColumnsMapper(mt.schema, p)
    got = [c.to_list() for c in m._map_columns(mt)]
    rows = [m._map_row_values(r) for r in mt.rows()]
    ref = [[r[j] for r in rows] for j in range(len(got))]
    assert got == ref


@pytest.mark.parametrize("target", ["DOUBLE", "INT", "BIGINT"])
def test_numerical_type_cast_tensor_equals_list(target):
    """NumericalTypeCast over tensor columns equals the per-value path: truncation toward zero, nulls kept."""
    import torch
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    import alink_amd as A
    x = torch.tensor([1.7, -1.7, 0.0, -0.0, 2.5, 1e9, -3.999], dtype=torch.float64)
    xn = torch.tensor([False, False, True, False, False, False, False])
    k = torch.tensor([3, -4, 5, 2 ** 40, 0, 7, 9], dtype=torch.int64)
    schema = TableSchema(["x", "k"], [Types.DOUBLE, Types.LONG])
    tm = MTable(schema, [Column(x, xn), Column(k)])
    lm = MTable(schema, [Column([None if xn[i] else float(x[i]) for i in range(7)]), Column(k.tolist())])
    cols = ["x"] if target == "INT" else ["x", "k"]
    outs = [A.NumericalTypeCastBatchOp().setSelectedCols(cols).setTargetType(target)
            .linkFrom(TableSourceBatchOp(m)).collect() for m in (tm, lm)]
    assert [tuple(r) for r in outs[0]] == [tuple(r) for r in outs[1]]


@pytest.mark.parametrize("p", [1.0, 2.0, 3.0, float("inf")])
def test_vector_normalize_columnar(p):
    """VectorNormalize over a dense 2-D tensor column equals the per-vector row path (to rounding)."""
    import numpy as np
    import torch
    from alink_amd.common.linalg import DenseVector
    from alink_amd.common.params import Params
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.dataproc.vector import VectorNormalizeMapper
    X = torch.randn(50, 7, dtype=torch.float64)
    X[3] = 0
    mt = MTable(TableSchema(["v"], [Types.DENSE_VECTOR]), [Column(X)])
    m = VectorNormalizeMapper(mt.schema, Params().set("selectedCol", "v").set("p", p))
    out = m._map_columns(mt)[0].values
    for i in range(50):
        ref = m.mapColumn(DenseVector(X[i].numpy().copy())).getData()
        np.testing.assert_allclose(out[i].numpy(), ref, rtol=1e-15, atol=0)


def test_pca_predict_packed_strings():
    import numpy as np
    import pandas as pd
    from alink_amd import BatchOperator, PcaPredictBatchOp, PcaTrainBatchOp
    from alink_amd.common.linalg import DenseVector, VectorUtil
    rng = np.random.default_rng(2)
    df = pd.DataFrame(rng.standard_normal((80, 4)), columns=["a", "b", "c", "d"])
    src = BatchOperator.fromDataframe(df, schemaStr="a double, b double, c double, d double")
    model = PcaTrainBatchOp().setSelectedCols(["a", "b", "c", "d"]).setK(2).linkFrom(src)
    rows = PcaPredictBatchOp().setPredictionCol("p").linkFrom(model, src).collect()
    for r in rows:
        s = r[-1]
        assert s == VectorUtil.toString(DenseVector(np.array([float(x) for x in s.split(" ")])))
        assert len(s.split(" ")) == 2


@pytest.mark.gpu
@pytest.mark.parametrize("p", [1.0, 2.0, float("inf")])
def test_vector_normalize_device(p):
    """VectorNormalize on a cuda 2-D column stays on the device and equals the host path to rounding."""
    import torch
    from alink_amd.common.params import Params
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.dataproc.vector import VectorNormalizeMapper
    X = torch.randn(1000, 33, dtype=torch.float64)
    X[7] = 0
    schema = TableSchema(["v"], [Types.DENSE_VECTOR])
    m = VectorNormalizeMapper(schema, Params().set("selectedCol", "v").set("p", p))
    host = m._map_columns(MTable(schema, [Column(X)]))[0].values
    dev = m._map_columns(MTable(schema, [Column(X.cuda())]))[0].values
    assert dev.is_cuda and dev.dtype == torch.float64
    torch.testing.assert_close(dev.cpu(), host, rtol=1e-14, atol=0)


@pytest.mark.parametrize("skip", [True, False])
def test_json_value_columnar_matches_row_path(skip):
    from alink_amd.common.params import Params
    from alink_amd.common.table import MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.dataproc.format import JsonPathMapper
    docs = ['{"a": 1, "b": {"c": "x", "d": [1, 2.5]}}', '{"a": 1.5e3, "b": {"c": {"z": true}}}',
            '{"a": "s", "b": {}}', None, "  ", "{bad", '{"a": null, "b": {"c": null}}']
    if not skip:
        docs = [docs[0], docs[1], docs[6]]
    schema = TableSchema(["j"], [Types.STRING])
    mt = MTable.from_rows([(d,) for d in docs], schema)
    paths = ["$.a", "$.b.c", "b.d"] if skip else ["$.a", "$.b.c"]
    m = JsonPathMapper(schema, Params().set("selectedCol", "j").set("jsonPath", paths)
                       .set("outputCols", [f"o{i}" for i in range(len(paths))]).set("skipFailed", skip))
    cols = m._map_columns(mt)
    fast = [tuple(c.to_list()[i] for c in cols) for i in range(len(docs))]
    slow = [tuple(m._map_row_values((d,))) for d in docs]
    assert fast == slow


def test_json_value_columnar_raises_like_row_path():
    from alink_amd.common.params import Params
    from alink_amd.common.table import MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.dataproc.format import JsonPathMapper
    schema = TableSchema(["j"], [Types.STRING])
    m = JsonPathMapper(schema, Params().set("selectedCol", "j").set("jsonPath", ["$.q"]).set("outputCols", ["o"]))
    with pytest.raises(RuntimeError, match="No results for path"):
        m._map_columns(MTable.from_rows([('{"a": 1}',)], schema))
    with pytest.raises(RuntimeError, match="No results for path"):
        m._map_row_values(('{"a": 1}',))


@pytest.mark.gpu
@pytest.mark.parametrize("calc,transform", [("COV_SAMPLE", "SIMPLE"), ("CORR", "NORMALIZATION"),
                                            ("COVAR_POP", "SUBMEAN")])
def test_pca_predict_device_matches_host(calc, transform):
    """PCA projection on a cuda table equals the host projection to rounding."""
    import numpy as np
    import torch
    from alink_amd import PcaPredictBatchOp, PcaTrainBatchOp
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    g = torch.Generator().manual_seed(3)
    X = torch.randn(500, 6, generator=g, dtype=torch.float64) * torch.arange(1, 7, dtype=torch.float64)
    names = [f"x{i}" for i in range(6)]
    schema = TableSchema(names, [Types.DOUBLE] * 6)
    host = TableSourceBatchOp(MTable(schema, [Column(X[:, j].clone()) for j in range(6)]))
    dev = TableSourceBatchOp(MTable(schema, [Column(X[:, j].cuda()) for j in range(6)]))
    model = PcaTrainBatchOp().setSelectedCols(names).setK(3).setCalculationType(calc).linkFrom(host)
    outs = []
    for src in (host, dev):
        rows = PcaPredictBatchOp().setPredictionCol("p").setTransformType(transform).setReservedCols([]) \
            .linkFrom(model, src).collect()
        outs.append(np.array([[float(v) for v in r[0].split(" ")] for r in rows]))
    np.testing.assert_allclose(outs[1], outs[0], rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("skip", [True, False])
@pytest.mark.parametrize("packed", [True, False])
def test_json_value_native_top_members(skip, packed):
    """Top-level ``$.key`` paths through the C++ member scanner equal the JSON-reader row path: strings (UTF-8,
    escaped), integers (big, negative, -0), doubles (exponents, 1.0, 1e400), booleans, null, nested values,
    duplicates, missing members, blank and malformed documents."""
    from alink_amd.common.params import Params
    from alink_amd.common.strings import StringBlock
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.dataproc.format import JsonPathMapper
    docs = ['{"a": 1, "b": "héllo wörld"}', '{"a": -2.5e3, "b": "q\\"x"}', '{"a":-0,"b":true}',
            '{"a": 123456789012345678901234567890, "b": false}', '{"a": 1.0, "b": null}',
            '{"a": 1e400, "b": [1, {"x": "]"}]}', '{"a": 0.1, "b": {"c": 1}, "a": 7}', ' { "a" : 3 , "b" : "t\\u00e9" } ',
            '{"a": 5E-7, "b": "tab\\tx"}', '{"a": 2, "b": ""}']
    if skip:
        docs += ['{"b": "only b"}', None, "   ", "{bad", '{"a":1,}', '{"a":01, "b": 1}', '{"a":"x"} trailing']
    schema = TableSchema(["j"], [Types.STRING])
    col = Column(StringBlock.from_list(docs)) if packed else Column(list(docs))
    mt = MTable(schema, [col])
    m = JsonPathMapper(schema, Params().set("selectedCol", "j").set("jsonPath", ["$.a", "b"])
                       .set("outputCols", ["oa", "ob"]).set("skipFailed", skip))
    cols = m._map_columns(mt)
    assert all(isinstance(c.values, StringBlock) for c in cols)
    fast = [tuple(c.to_list()[i] for c in cols) for i in range(len(docs))]
    slow = [tuple(m._map_row_values((d,))) for d in docs]
    assert fast == slow


def _row_vs_columnar(mapper, mt):
    import numpy as np
    cols = mapper._map_columns(mt)
    fast = [v.getData() if hasattr(v, "getData") else v for v in cols[0].to_list()]
    slow = [mapper._map_row_values(r)[0] for r in mt.rows()]
    slow = [v.getData() if hasattr(v, "getData") else v for v in slow]
    assert len(fast) == len(slow)
    for a, b in zip(fast, slow):
        a, b = np.asarray(a), np.asarray(b)
        assert a.shape == b.shape and a.tobytes() == b.tobytes()      # bit for bit, signed zeros included


def test_vector_mappers_columnar_bitwise():
    """Slice / elementwise product / interaction / polynomial expansion / size hint over dense 2-D tensor
    columns equal the per-vector row path bit for bit (zeros, negatives, inf, NaN)."""
    import torch
    from alink_amd.common.params import Params
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.dataproc import vector as V
    g = torch.Generator().manual_seed(9)
    X = torch.randn(40, 4, generator=g, dtype=torch.float64)
    X[0] = torch.tensor([0.0, -3.0, float("inf"), 2.0])
    X[1] = torch.tensor([float("nan"), 0.0, -0.0, 1e-200])
    X[2] = torch.tensor([1e-200, 1e-200, -1e-200, 5.0])
    Y = torch.randn(40, 3, generator=g, dtype=torch.float64)
    schema = TableSchema(["x", "y"], [Types.DENSE_VECTOR, Types.DENSE_VECTOR])
    mt = MTable(schema, [Column(X), Column(Y)])
    P = lambda **kw: Params().set("selectedCol", "x").set("outputCol", "o") if not kw else \
        Params().set("outputCol", "o").set(*next(iter(kw.items())))  # noqa: E731
    _row_vs_columnar(V.VectorSliceMapper(schema, P().set("indices", [3, 0, -1])), mt)
    _row_vs_columnar(V.VectorElementwiseProductMapper(schema, P().set("scalingVector", "2 -1 0.5 3 9")), mt)
    _row_vs_columnar(V.VectorInteractionMapper(schema, P(selectedCols=["x", "y"])), mt)
    for deg in (1, 2, 3):
        _row_vs_columnar(V.VectorPolynomialExpandMapper(schema, P().set("degree", deg)), mt)
    m = V.VectorSizeHintMapper(schema, P().set("size", 4))
    assert m._map_columns(mt)[0].values is X


def test_vector_serialize_and_index_to_string_columnar():
    """VectorSerialize of a dense tensor column (C++ Double.toString rows) and IndexToString over an integer
    tensor column (one lookup per distinct index) equal their row paths, NULLs and unknown indices included."""
    import torch
    from alink_amd.common.params import Params
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.dataproc.vector import VectorSerializeMapper
    from alink_amd.models.feature.encoders import IndexToStringModelMapper
    X = torch.tensor([[1.0, -0.0, 1e-7], [float("nan"), 3.5, 1e21]], dtype=torch.float64)
    schema = TableSchema(["v", "i"], [Types.DENSE_VECTOR, Types.LONG])
    mt = MTable(schema, [Column(X), Column(torch.tensor([0, 5]))])
    m = VectorSerializeMapper(schema, Params())
    assert m._map_columns(mt)[0].to_list() == [m._map_row_values(r)[0] for r in mt.rows()]
    ischema = TableSchema(["i"], [Types.LONG])
    idx = torch.tensor([2, 0, 7, 2, 1, 0])
    nm = torch.tensor([False, False, False, True, False, False])
    imt = MTable(ischema, [Column(idx, nm)])
    mm = IndexToStringModelMapper(TableSchema(["token", "token_index"], [Types.STRING, Types.LONG]), ischema,
                                  Params().set("selectedCol", "i").set("outputCol", "s"))
    mm.loadModel([("a", 0), ("bé", 1), ("c", 2)])
    assert mm._map_columns(imt)[0].to_list() == [mm.mapColumn(v) for v in imt.col("i").to_list()]


@pytest.mark.parametrize("inverse", [False, True])
def test_dct_columnar(inverse):
    import numpy as np
    import torch
    from alink_amd.common.linalg import DenseVector
    from alink_amd.common.params import Params
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.feature.encoders import DCTMapper
    X = torch.randn(64, 17, dtype=torch.float64)
    schema = TableSchema(["v"], [Types.DENSE_VECTOR])
    m = DCTMapper(schema, Params().set("selectedCol", "v").set("inverse", inverse))
    out = m._map_columns(MTable(schema, [Column(X)]))[0].values.numpy()
    for i in range(64):
        ref = m.mapColumn(DenseVector(X[i].numpy().copy())).getData()
        np.testing.assert_allclose(out[i], ref, rtol=1e-13, atol=1e-15)
