"""P-rank vs 1-rank correctness matrix on the CPU (gloo): every distributed algorithm family of
``tests/matrix_helpers.py`` runs in ONE launch of P processes (P = 8, and P = 3 for an odd split) and must
agree across ranks and with the single-rank run — exactly where the algorithm is order-free (vocabularies,
patterns, trees, assignments), to fp64 summation-order tolerance where ranks sum partial moments."""
import json
import math
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import matrix_helpers as MH  # noqa: E402

NAMES = list(MH.SCENARIOS)
# results that must be bit-identical across world sizes (integer / combinatorial / order-free outputs)
EXACT = {"bisecting", "gmm", "softmax", "onehot_indexer", "doccount", "word2vec", "lda", "fpgrowth", "prefixspan",
         "lsh_join", "gbdt_fshard", "gbdt_rank", "als", "ftrl", "quantile", "mlp"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(world, outdir):
    port = _free_port()
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "matrix_helpers.py"), str(r), str(world), str(port),
                               outdir, ",".join(NAMES)], env=env) for r in range(world)]
    for p in procs:
        p.wait(timeout=900)
    res = {}
    for name in NAMES:
        per = []
        for r in range(world):
            with open(os.path.join(outdir, f"{name}_{world}_{r}.json")) as f:
                per.append(json.load(f))
        res[name] = per
    return res


@pytest.fixture(scope="module")
def runs(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("matrix"))
    return {w: _launch(w, d) for w in (1, 3, 8)}


def _close(a, b, path=""):
    """Equal structure; numbers (also inside JSON strings) within 1e-9 relative."""
    if isinstance(a, str) and isinstance(b, str) and a != b:
        try:
            return _close(json.loads(a), json.loads(b), path)
        except (ValueError, TypeError):
            pass
        try:                                            # dense vector strings "v0 v1 ..." / "v0,v1,..."
            return _close([float(x) for x in a.replace(",", " ").split()],
                          [float(x) for x in b.replace(",", " ").split()], path)
        except ValueError:
            return f"{path}: {a[:120]!r} != {b[:120]!r}"
    if isinstance(a, dict) and isinstance(b, dict):
        if a.keys() != b.keys():
            return f"{path}: keys {sorted(a)} != {sorted(b)}"
        for k in a:
            r = _close(a[k], b[k], f"{path}/{k}")
            if r:
                return r
        return None
    if isinstance(a, list) and isinstance(b, list):
        if len(a) != len(b):
            return f"{path}: len {len(a)} != {len(b)}"
        for i, (x, y) in enumerate(zip(a, b)):
            r = _close(x, y, f"{path}[{i}]")
            if r:
                return r
        return None
    if isinstance(a, (int, float)) and isinstance(b, (int, float)) and not isinstance(a, bool):
        if math.isnan(a) and math.isnan(b):
            return None
        if abs(a - b) <= 1e-9 * max(1.0, abs(a), abs(b)):
            return None
        return f"{path}: {a!r} vs {b!r}"
    return None if a == b else f"{path}: {a!r} vs {b!r}"


@pytest.mark.parametrize("world", [3, 8])
@pytest.mark.parametrize("name", NAMES)
def test_multirank_equals_single(runs, name, world):
    one = runs[1][name][0]
    many = runs[world][name]
    assert "error" not in one, one.get("error")
    for r, o in enumerate(many):
        assert "error" not in o, f"rank {r}: {o.get('error')}"
    assert all(o == many[0] for o in many), "ranks disagree"
    if name in EXACT:
        assert many[0] == one, _close(one, many[0]) or "differs"
    else:
        msg = _close(one, many[0])
        assert msg is None, msg
