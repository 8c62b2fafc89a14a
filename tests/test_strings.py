"""Packed string columns (common/strings.StringBlock) and bulk string hashing (ops/strings.py), host side."""
import numpy as np
import pytest
import torch

from alink_amd.common.strings import StringBlock
from alink_amd.common.table import Column, MTable
from alink_amd.common.types import TableSchema, Types
from alink_amd.ops import strings as S

VALS = ["ab", None, "héllo", "", "z", "x\U0001F600y", "中文"]


def test_string_block_roundtrip_take_concat():
    b = StringBlock.from_list(VALS)
    assert len(b) == len(VALS) and b.to_list() == VALS and list(b) == VALS
    assert b[2] == "héllo" and b[1] is None and b[-1] == VALS[-1]
    assert b.take([6, 0, 0, 1]).to_list() == [VALS[6], "ab", "ab", None]
    assert b.take(np.array([True] + [False] * 6)).to_list() == ["ab"]
    assert b[1:4].to_list() == VALS[1:4]
    assert StringBlock.concat([b, b.take([5])]).to_list() == VALS + [VALS[5]]
    assert b.nbytes == sum(len(v.encode()) for v in VALS if v)


def test_column_and_table_accept_string_blocks():
    mt = MTable(TableSchema(["s", "x"], [Types.STRING, Types.LONG]),
                [Column(StringBlock.from_list(VALS)), Column(torch.arange(len(VALS)))])
    assert [r[0] for r in mt.rows()] == VALS
    t = mt.take([3, 2])
    assert isinstance(t.cols[0].values, StringBlock) and t.cols[0].to_list() == ["", "héllo"]
    c = MTable.concat([mt, mt.slice(0, 2)])
    assert c.cols[0].to_list() == VALS + VALS[:2]


def test_murmur3_bytes_standard_vectors_and_native_equals_python():
    b = StringBlock.from_list(["", "hello", "The quick brown fox jumps over the lazy dog"])
    got = [int(x) & 0xFFFFFFFF for x in S.hash_bytes(b)]
    assert got == [0, 0x248bfa47, 0x2e4ff723]
    rng = np.random.default_rng(0)
    words = ["".join(chr(int(c)) for c in rng.integers(32, 0x2FFF, rng.integers(0, 17))) for _ in range(300)]
    blk = StringBlock.from_list(words)
    ref = [S.murmur3_bytes_py(w.encode()) for w in words]
    assert S.hash_bytes(blk).tolist() == ref


def test_utf8_feature_hash_equals_guava_utf16():
    from alink_amd.models.feature.encoders import murmur3_index as host_index
    words = [w for w in VALS if w is not None] + ["col", "a" * 33]
    got = S.murmur3_utf8_index(StringBlock.from_list(words), 1 << 18, prefix="c=").tolist()
    assert got == list(host_index(["c=" + w for w in words], 1 << 18))
