"""The generated operator reference (docs/operators, tools/gen_docs.py) covers every exported operator and stage
and is in sync with the code."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_exported_op_documented():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_docs
    ops = gen_docs.collect()
    text = open(os.path.join(ROOT, "docs", "operators", "README.md"), encoding="utf-8").read()
    missing = [n for n in ops if f"[{n}]" not in text]
    assert not missing, missing[:20]
    assert len(ops) >= 450


@pytest.mark.skipif(not os.path.isdir("/root/reference/docs/en"), reason="reference docs not present")
def test_docs_in_sync():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_docs.py"), "--check"], capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
