"""CSV parser / formatter against the reference's unit tests (``core/src/test/java/com/alibaba/alink/operator/
common/io/csv/{CsvParserTest,CsvFormatterTest}.java``)."""
import datetime
import math
import random
import sys

from alink_amd.common.types import Types
from alink_amd.operator.common.io.csv import CsvFormatter, CsvParser, format_timestamp, parse_timestamp


def test_quoted_and_empty_strings():
    p = CsvParser([Types.STRING], ",", '"')
    assert p.parse('"hello, world"')[1][0] == "hello, world"
    assert p.parse("")[1][0] is None
    assert p.parse('""')[1][0] == ""
    assert p.parse('""""""')[1][0] == '""'


def test_long_field_separator():
    p = CsvParser([Types.STRING] * 3, "____", '"')
    assert p.parse("hello_____world____")[1] == ["hello", "_world", None]
    assert p.parse('"hello_____world____"')[1] == ["hello_____world____", None, None]


def test_malformed_quotes():
    p = CsvParser([Types.STRING, Types.LONG], ",", '"')
    assert p.parse('"hello" world,1')[0]
    assert not p.parse('"hello world,1')[0]


def test_format_parse_round_trip_with_timestamp():
    types = [Types.STRING, Types.DOUBLE, Types.LONG, Types.BOOLEAN, Types.TIMESTAMP]
    row = ("string", 1.0, 1, True, datetime.datetime(2024, 5, 6, 7, 8, 9, 123000))
    text = CsvFormatter(types, ",", '"').format(row)
    assert text == "string,1.0,1,true,2024-05-06 07:08:09.123"
    ok, parsed = CsvParser(types, ",", '"').parse(text)
    assert ok and tuple(parsed) == row
    assert format_timestamp(datetime.datetime(2020, 1, 2, 3, 4, 5)) == "2020-01-02 03:04:05.0"
    assert parse_timestamp("2020-1-2 3:04:05.000000001") == datetime.datetime(2020, 1, 2, 3, 4, 5)


def test_double_precision_round_trip():
    f, p = CsvFormatter([Types.DOUBLE], ",", '"'), CsvParser([Types.DOUBLE], ",", '"')
    for v in (sys.float_info.max, 5e-324, -math.inf, math.inf, random.random()):
        assert p.parse(f.format((v,)))[1][0] == v
