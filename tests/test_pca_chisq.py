"""PCA and chi-square selection vs the reference docs (docs/en/pcatrainbatchop.md, chisqselectorbatchop.md)."""
import numpy as np
import pandas as pd

from alink_amd import *  # noqa: F401,F403

PCA_DATA = np.array([[0.0, 0.0, 0.0], [0.1, 0.2, 0.1], [0.2, 0.2, 0.8], [9.0, 9.5, 9.7], [9.1, 9.1, 9.6],
                     [9.2, 9.3, 9.9]])
PCA_REF = {(9.0, 9.5, 9.7): [3.2280384305400736, 1.1516225426477789E-4],
           (0.2, 0.2, 0.8): [0.13565076707329407, 0.09003329494282108],
           (9.2, 9.3, 9.9): [3.250783163664603, 0.0456526246528135],
           (9.1, 9.1, 9.6): [3.182618319978973, 0.027469531992220464],
           (0.1, 0.2, 0.1): [0.045855205015063565, -0.012182917696915518],
           (0.0, 0.0, 0.0): [0.0, 0.0]}


def test_pca_doc_example_batch_stream_pipeline():
    df = pd.DataFrame({"x1": PCA_DATA[:, 0], "x2": PCA_DATA[:, 1], "x3": PCA_DATA[:, 2]})
    src = BatchOperator.fromDataframe(df, schemaStr="x1 double, x2 double, x3 double")
    train = PcaTrainBatchOp().setK(2).setSelectedCols(["x1", "x2", "x3"]).linkFrom(src)
    out = PcaPredictBatchOp().setPredictionCol("pred").linkFrom(train, src).collect()
    for r in out:
        np.testing.assert_allclose([float(x) for x in r[3].split(" ")], PCA_REF[tuple(r[:3])], atol=1e-9)
    box = []
    PcaPredictStreamOp(train).setPredictionCol("pred").linkFrom(
        StreamOperator.fromDataframe(df, schemaStr="x1 double, x2 double, x3 double")).link(CollectStreamOp(box))
    StreamOperator.execute()
    assert len(box) == 6
    m = PCA().setK(2).setSelectedCols(["x1", "x2", "x3"]).setPredictionCol("pred").fit(src)
    assert len(m.transform(src).collect()) == 6
    # SUBMEAN transform centres the scores
    sub = PcaPredictBatchOp().setPredictionCol("pred").setTransformType("SUBMEAN").linkFrom(train, src).collect()
    S = np.array([[float(x) for x in r[3].split(" ")] for r in sub])
    np.testing.assert_allclose(S.mean(0), 0.0, atol=1e-9)


def test_chisq_selector_doc():
    data = [["a", 1, 1, 2.0, True], ["c", 1, 2, -3.0, True], ["a", 2, 2, 2.0, False], ["c", 0, 0, 0.0, False]]
    df = pd.DataFrame(data, columns=["f_string", "f_long", "f_int", "f_double", "f_boolean"])
    src = BatchOperator.fromDataframe(
        df, schemaStr="f_string string, f_long long, f_int int, f_double double, f_boolean boolean")
    sel = ChiSqSelectorBatchOp().setSelectedCols(["f_string", "f_long", "f_int", "f_double"]) \
        .setLabelCol("f_boolean").setNumTopFeatures(2)
    sel.linkFrom(src)
    assert sel.collectResult() == ["f_string", "f_long"]
    assert sel.selectedIndices() == [1, 2]     # f_long (p=0.135), then f_int (tie with f_double, lower index)
