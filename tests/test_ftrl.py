"""FTRL online learning vs the reference docs (docs/en/ftrltrainstreamop.md) + update-rule checks."""
import json

import numpy as np
import pandas as pd
import pytest

from alink_amd import *  # noqa: F401,F403
from alink_amd import _native
from alink_amd.operator.stream.onlinelearning import _ftrl_python

DATA = np.array([[2, 1, 1], [3, 2, 1], [4, 3, 2], [2, 4, 1], [2, 2, 1], [4, 3, 2], [1, 2, 1], [5, 3, 2]])
DETAILS = ['{"1":"0.9999917437501057","2":"8.256249894311729E-6"}',
           '{"1":"0.9659178381854678","2":"0.034082161814532164"}',
           '{"1":"0.00658782416074899","2":"0.993412175839251"}']


def _run(interval=1):
    df = pd.DataFrame({"f0": DATA[:, 0], "f1": DATA[:, 1], "label": DATA[:, 2]})
    batch = BatchOperator.fromDataframe(df, schemaStr="f0 int, f1 int, label int")
    stream = StreamOperator.fromDataframe(df, schemaStr="f0 int, f1 int, label int")
    model = LogisticRegressionTrainBatchOp().setFeatureCols(["f0", "f1"]).setLabelCol("label").setMaxIter(5) \
        .linkFrom(batch)
    models = FtrlTrainStreamOp(model).setFeatureCols(["f0", "f1"]).setLabelCol("label").setTimeInterval(interval) \
        .setAlpha(0.1).setBeta(0.1).setL1(0.1).setL2(0.1).setVectorSize(2).setWithIntercept(True) \
        .linkFrom(stream)
    preds, snaps = [], []
    models.link(CollectStreamOp(snaps))
    FtrlPredictStreamOp(model).setPredictionCol("pred").setReservedCols(["label"]) \
        .setPredictionDetailCol("details").linkFrom(models, stream).link(CollectStreamOp(preds))
    StreamOperator.execute()
    return preds, snaps


def test_ftrl_doc_example():
    preds, snaps = _run()
    assert [r[1] for r in preds] == [r[0] for r in preds] == [1, 1, 2, 1, 1, 2, 1, 2]
    for r, ref in zip(preds[:3], DETAILS):   # the warm-start LR model is trained on the device: ~1e-12 apart
        got, exp = json.loads(r[2]), json.loads(ref)
        assert got.keys() == exp.keys() and all(abs(float(got[k]) - float(exp[k])) < 1e-9 for k in exp)
    # snapshot framing: bid, ntab, then the linear-model table rows
    bids = sorted({r[0] for r in snaps})
    assert bids[0] == 0 and all(r[1] == 4 for r in snaps)
    assert snaps[1][3].startswith('{"featureColNames":["f0","f1"]')


def test_ftrl_native_matches_python_rule():
    rng = np.random.default_rng(0)
    n, d = 50, 6
    X = rng.normal(size=(n, d))
    X[rng.random((n, d)) < 0.5] = 0.0
    y = (rng.random(n) < 0.5).astype(float)
    indptr = np.zeros(n + 1, np.int64)
    idx, val = [], []
    for i in range(n):
        nz = np.nonzero(X[i])[0]
        idx.extend(nz)
        val.extend(X[i, nz])
        indptr[i + 1] = len(idx)
    idx, val = np.asarray(idx, np.int32), np.asarray(val)
    w0 = rng.normal(size=d)
    a = [w0.copy(), np.zeros(d), np.zeros(d)]
    b = [w0.copy(), np.zeros(d), np.zeros(d)]
    if not _native.ftrl_update_csr(indptr, idx, val, y, *a, 0.1, 1.0, 0.05, 0.1):
        pytest.skip("native library not built")
    _ftrl_python(indptr, idx, val, y, *b, 0.1, 1.0, 0.05, 0.1)
    for u, v in zip(a, b):
        np.testing.assert_allclose(u, v, rtol=1e-12, atol=1e-14)
