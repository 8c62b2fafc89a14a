"""Host C++ runtime under AddressSanitizer + UBSan (tools/asan_host.py)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_runtime_clean_under_asan_ubsan():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asan_host.py")], capture_output=True,
                       text=True, timeout=900)
    if p.returncode == 77:
        pytest.skip("sanitizer runtimes not installed")
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-6000:]
    assert "ASAN_EXERCISE_OK" in p.stdout
