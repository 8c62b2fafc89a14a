"""Binary evaluation summary: the host C++ bulk parser of two-entry detail strings (_native.parse_binary_detail)
gives the same bins, log-loss and count as the per-row JSON loop; malformed strings fall back to that loop."""
import numpy as np
import pytest

from alink_amd import _native
from alink_amd.models.evaluation import metrics as M


def _data(n, seed):
    rng = np.random.default_rng(seed)
    p = rng.random(n)
    labs = ["a" if v else "b" for v in rng.random(n) < 0.4]
    dets = ['{"a":%r,"b":%r}' % (float(x), float(1 - x)) if i % 3 else '{"b": %r, "a": %r}' % (float(1 - x), float(x))
            for i, x in enumerate(p)]
    labs[5], dets[7] = None, None
    return labs, dets


@pytest.mark.skipif(_native.lib is None, reason="native runtime not built")
def test_native_detail_summary_equals_json_loop(monkeypatch):
    labs, dets = _data(5000, 0)
    fast = M.binary_summary(labs, dets, ["a", "b"])
    assert M._binary_detail_native(labs, dets, ["a", "b"]) is not None
    monkeypatch.setattr(M, "_binary_detail_native", lambda *a: None)
    slow = M.binary_summary(labs, dets, ["a", "b"])
    assert np.array_equal(fast[0], slow[0]) and np.array_equal(fast[1], slow[1]) and fast[3] == slow[3]
    assert fast[2] == pytest.approx(slow[2], rel=1e-14)


@pytest.mark.skipif(_native.lib is None, reason="native runtime not built")
def test_native_detail_rejects_other_forms():
    assert _native.parse_binary_detail(['{"a":0.5,"b":0.5,"c":0.0}'], "a", "b") is None
    assert _native.parse_binary_detail(['{"a\\u0041":0.5,"b":0.5}'], "a", "b") is None
    assert _native.parse_binary_detail(['{"a":0.5,"c":0.5}'], "a", "b") is None
    assert _native.parse_binary_detail(['{"a":x,"b":0.5}'], "a", "b") is None
    p0, p1 = _native.parse_binary_detail(['{"a":0.25,"b":0.75}', ' { "b" : 1e-3 , "a" : 0.999 } '], "a", "b")
    assert list(p0) == [0.25, 0.999] and list(p1) == [0.75, 1e-3]


@pytest.mark.skipif(_native.lib is None, reason="native runtime not built")
def test_native_and_json_paths_reject_the_same_rows(monkeypatch):
    """A malformed detail on a row whose label is NOT one of the two still fails (the JSON loop parses every
    non-null row), whichever path runs."""
    labs, dets = _data(200, 1)
    labs[3], dets[3] = "zzz", '{"a":0.5,"b":0.25,"c":0.25}'
    with pytest.raises(ValueError):
        M.binary_summary(labs, dets, ["a", "b"])
    monkeypatch.setattr(M, "_binary_detail_native", lambda *a: None)
    with pytest.raises(ValueError):
        M.binary_summary(labs, dets, ["a", "b"])
