"""BatchOperator.sqlQuery: joins, subqueries, grouping/HAVING, set operations, ordering (query.py executor)."""
import math

import pandas as pd
import pytest

from alink_amd import BatchOperator, useLocalEnv
from alink_amd.operator.common.sql.query import parse_query


@pytest.fixture
def tables():
    useLocalEnv(1)
    a = BatchOperator.fromDataframe(pd.DataFrame({"id": [1, 2, 3, 4], "name": ["a", "b", "c", "d"],
                                                  "v": [1.0, 2.5, None, 4.0]}), schemaStr="id int, name string, v double")
    b = BatchOperator.fromDataframe(pd.DataFrame({"id": [2, 3, 5], "score": [10, 20, 30]}),
                                    schemaStr="id int, score int")
    a.registerTableName("ta")
    b.registerTableName("tb")


def q(text):
    return [tuple(r) for r in BatchOperator.sqlQuery(text).collect()]


def test_where_order(tables):
    assert q("select * from ta where v > 1 order by v desc") == [(4, "d", 4.0), (2, "b", 2.5)]


def test_inner_left_full_joins(tables):
    assert q("select ta.id, name, score from ta join tb on ta.id = tb.id") == [(2, "b", 10), (3, "c", 20)]
    assert q("select x.id, y.score from ta x left outer join tb y on x.id = y.id order by x.id") == \
        [(1, None), (2, 10), (3, 20), (4, None)]
    assert q("select x.id, y.id, y.score from ta x right join tb y on x.id = y.id order by y.id") == \
        [(2, 2, 10), (3, 3, 20), (None, 5, 30)]
    full = q("select x.id, y.score from ta x full outer join tb y on x.id = y.id order by 1")
    assert full == [(None, 30), (1, None), (2, 10), (3, 20), (4, None)]
    # comma join + qualified star
    assert q("select a.*, b.score from ta a, tb b where a.id = b.id") == [(2, "b", 2.5, 10), (3, "c", None, 20)]
    # non-equi join condition
    assert len(q("select x.id from ta x join tb y on x.id < y.id")) == 3 + 2 + 1 + 1


def test_aggregates_group_having(tables):
    assert q("select count(*) as n, sum(score) s from tb") == [(3, 60)]
    assert q("select id % 2 as k, count(*) c, max(v) from ta group by id % 2 having count(*) > 1") == \
        [(1, 2, 1.0), (0, 2, 4.0)]
    assert q("select count(*) from ta where id > 100") == [(0,)]


def test_subqueries(tables):
    assert q("select name from ta where id in (select id from tb)") == [("b",), ("c",)]
    assert q("select name from ta where id not in (select id from tb) order by name desc") == [("d",), ("a",)]
    assert q("select name, v from ta where v > (select avg(v) from ta)") == [("d", 4.0)]
    assert q("select id, cnt from (select id, count(*) cnt from ta group by id) t where cnt >= 1 "
             "order by id desc limit 2") == [(4, 1), (3, 1)]


def test_set_operations(tables):
    assert q("select id from ta union select id from tb order by id") == [(i,) for i in (1, 2, 3, 4, 5)]
    assert len(q("select id from ta union all select id from tb")) == 7
    assert q("select id from ta except select id from tb") == [(1,), (4,)]
    assert q("select id from ta intersect select id from tb order by id") == [(2,), (3,)]
    assert q("(select id from ta where id < 3) union (select id from tb) order by id limit 3 offset 1") == \
        [(2,), (3,), (5,)]


def test_distinct_and_expressions(tables):
    assert q("select distinct id % 2 from ta order by 1") == [(0,), (1,)]
    rows = q("select upper(name) u, case when v is null then -1 else v * 2 end w from ta order by u")
    assert rows[0] == ("A", 2.0) and rows[2] == ("C", -1)


def test_parse_errors():
    with pytest.raises(ValueError):
        parse_query("select from")
    with pytest.raises(ValueError):
        parse_query("select a from t join u")
    assert math.isfinite(len(parse_query("select a from t;").body.items))


def test_reference_scalar_functions():
    """MathFunctionsTest / StringFunctionsTest (reference common/sql/functions) through select."""
    import hashlib
    import math
    import re
    from alink_amd.operator.batch.source import MemSourceBatchOp
    src = MemSourceBatchOp([(10.0, "HelloWorld", "hello,world", 100, "foobar", "foothebar", "hi", "SGVsbG9Xb3JsZA==")],
                           "v double, s string, h string, n long, f string, g string, t string, b string")

    def q(e):
        return src.select(e + " AS r").collect()[0][0]
    assert q("LOG2(v)") == pytest.approx(math.log(10) / math.log(2))
    assert q("LOG(v)") == pytest.approx(math.log(10))
    assert q("LOG(3, v)") == pytest.approx(math.log(10) / math.log(3))
    assert (q("SINH(v)"), q("COSH(v)"), q("TANH(v)")) == pytest.approx((math.sinh(10), math.cosh(10), math.tanh(10)))
    assert q("BIN(n)") == "1100100" and q("HEX(n)") == "64" and q("HEX(h)") == "68656C6C6F2C776F726C64"
    assert q("FROM_BASE64(b)") == "HelloWorld" and q("TO_BASE64(s)") == "SGVsbG9Xb3JsZA=="
    assert q("LPAD(t, 4, '??')") == "??hi" and q("RPAD(t, 4, '??')") == "hi??"
    assert q("REGEXP_REPLACE(f, 'oo|ar', '')") == "fb"
    assert q("REGEXP_EXTRACT(g, 'foo(.*?)(bar)', 2)") == "bar"
    assert q("MD5(s)") == hashlib.md5(b"HelloWorld").hexdigest()
    assert q("SHA1(s)") == hashlib.sha1(b"HelloWorld").hexdigest()
    for bits in (224, 256, 384, 512):
        assert q(f"SHA{bits}(s)") == getattr(hashlib, f"sha{bits}")(b"HelloWorld").hexdigest()
    assert q("SHA2(s, 384)") == hashlib.sha384(b"HelloWorld").hexdigest()
    assert re.fullmatch("[0-9a-f]{8}-[0-9a-f]{4}-[1-5][0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12}", q("UUID()"))
