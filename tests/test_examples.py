"""The four reference examples (examples/*_example.py, mirroring examples/src/main/java/com/alibaba/alink/*Example.java)
run end to end on small synthetic data; the GPU variants run the same scripts in a cuda:0 environment."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(name, device, rows, tmp_path, extra=()):
    cmd = [sys.executable, os.path.join(ROOT, "examples", f"{name}_example.py"), "--device", device, "--rows",
           str(rows), "--workdir", str(tmp_path)] + list(extra)
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=os.path.join(ROOT, "examples"))
    assert out.returncode == 0, out.stderr[-3000:]
    return out.stdout


@pytest.mark.parametrize("name,rows,check", [("kmeans", 150, "purity:"), ("gbdt", 3000, "AUC:"),
                                             ("als", 20000, "RMSE:"), ("ftrl", 3000, "final window: AUC"),
                                             ("observability", 5000, "stream predictions: 5000")])
def test_example_cpu(name, rows, check, tmp_path):
    out = _run(name, "cpu", rows, tmp_path)
    assert check in out


@pytest.mark.gpu
@pytest.mark.parametrize("name,rows,check,extra", [("kmeans", 150, "purity:", ()), ("gbdt", 20000, "AUC:", ()),
                                                   ("als", 100000, "RMSE:", ()),
                                                   ("ftrl", 20000, "final window: AUC", ("--mode", "SHARDED")),
                                                   ("observability", 20000, "stream predictions: 20000", ())])
def test_example_gpu(name, rows, check, extra, tmp_path):
    out = _run(name, "cuda:0", rows, tmp_path, extra)
    assert check in out
