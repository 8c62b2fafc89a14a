"""Pipeline-level reference tests (``core/src/test/java/com/alibaba/alink/pipeline/classification/*Test.java``):
three copies of one estimator over feature columns, a dense vector and a sparse vector column predict the training
labels in batch and stream; OneVsRest over LR (direct and behind VectorAssembler, with a LocalPredictor) and over
GBDT exceeds 0.9 accuracy on iris."""
import pytest

import alink_amd as A
from alink_amd.operator.batch.source import MemSourceBatchOp
from alink_amd.operator.stream.source import MemSourceStreamOp

from test_mlp import FEATS, _iris

BIN_ROWS = [("$31$0:1.0 1:1.0 2:1.0 30:1.0", "1.0  1.0  1.0  1.0", 1.0, 1.0, 1.0, 1.0, 1),
            ("$31$0:1.0 1:1.0 2:0.0 30:1.0", "1.0  1.0  0.0  1.0", 1.0, 1.0, 0.0, 1.0, 1),
            ("$31$0:1.0 1:0.0 2:1.0 30:1.0", "1.0  0.0  1.0  1.0", 1.0, 0.0, 1.0, 1.0, 1),
            ("$31$0:1.0 1:0.0 2:1.0 30:1.0", "1.0  0.0  1.0  1.0", 1.0, 0.0, 1.0, 1.0, 1)] + \
           [("$31$0:0.0 1:1.0 2:1.0 30:0.0", "0.0  1.0  1.0  0.0", 0.0, 1.0, 1.0, 0.0, 0)] * 4
BIN_COLS = ["svec", "vec", "f0", "f1", "f2", "f3", "labels"]


def _assert_labels(rows):
    for r in rows:
        assert r[1] == r[0] and r[2] == r[0] and r[3] == r[0], r


@pytest.mark.parametrize("est", ["LogisticRegression", "LinearSvm"])
def test_binary_linear_pipeline_predicts_labels(est):
    """LogisticRegTest.pipelineTestBatch / SvmTest.pipelineTest."""
    C = getattr(A, est)
    pl = A.Pipeline().add(C().setLabelCol("labels").setFeatureCols(["f0", "f1", "f2", "f3"]).setPredictionCol("p1")) \
        .add(C().setLabelCol("labels").setVectorCol("vec").setPredictionCol("p2")) \
        .add(C().setLabelCol("labels").setVectorCol("svec").setPredictionCol("p3").setPredictionDetailCol("detail"))
    data = MemSourceBatchOp(BIN_ROWS, BIN_COLS)
    model = pl.fit(data)
    _assert_labels(model.transform(data).select(["labels", "p1", "p2", "p3"]).collect())
    out = model.transform(MemSourceStreamOp(BIN_ROWS, BIN_COLS)).select(["labels", "p1", "p2", "p3"])
    rows = []
    out.collect_to(rows)
    A.StreamOperator.execute()
    assert len(rows) == len(BIN_ROWS)
    _assert_labels(rows)


def test_softmax_pipeline_predicts_labels():
    """SoftmaxTest.pipelineTest: standardised softmax with intercept, epsilon 1e-20, 10000 iterations."""
    rows = [("0:1.0 2:7.0 4:9.0", "1.0 7.0 9.0", 1.0, 7.0, 9.0, 2), ("0:1.0 2:3.0 4:3.0", "1.0 3.0 3.0", 1.0, 3.0, 3.0, 3),
            ("0:1.0 2:2.0 4:4.0", "1.0 2.0 4.0", 1.0, 2.0, 4.0, 1), ("0:1.0 2:2.0 4:4.0", "1.0 2.0 4.0", 1.0, 2.0, 4.0, 1)]
    cols = ["svec", "vec", "f0", "f1", "f2", "label"]

    def sm():
        return A.Softmax().setStandardization(True).setWithIntercept(True).setEpsilon(1.0e-20).setLabelCol("label") \
            .setMaxIter(10000)
    pl = A.Pipeline().add(sm().setFeatureCols(["f0", "f1", "f2"]).setPredictionCol("predLr")) \
        .add(sm().setVectorCol("vec").setPredictionCol("vpredLr")) \
        .add(sm().setVectorCol("svec").setPredictionCol("svpredLr").setPredictionDetailCol("svpredDetail"))
    data = MemSourceBatchOp(rows, cols)
    model = pl.fit(data)
    _assert_labels(model.transform(data).select(["label", "predLr", "vpredLr", "svpredLr"]).collect())
    got = []
    model.transform(MemSourceStreamOp(rows, cols)).select(["label", "predLr", "vpredLr", "svpredLr"]).collect_to(got)
    A.StreamOperator.execute()
    assert len(got) == len(rows)
    _assert_labels(got)


def test_naive_bayes_text_pipeline_predicts_labels():
    """NaiveBayesTextTest.testPipelineBatch: Bernoulli, smoothing 0.5, dense and sparse vectors."""
    rows = [(r[0], r[1], r[6]) for r in BIN_ROWS[:7]]

    def nb():
        return A.NaiveBayesTextClassifier().setModelType("Bernoulli").setLabelCol("labels").setSmoothing(0.5)
    pl = A.Pipeline().add(nb().setVectorCol("vec").setPredictionCol("pv").setPredictionDetailCol("pvd")) \
        .add(nb().setVectorCol("svec").setPredictionCol("psv").setPredictionDetailCol("psvd"))
    data = MemSourceBatchOp(rows, ["svec", "vec", "labels"])
    for r in pl.fit(data).transform(data).select(["labels", "pv", "psv"]).collect():
        assert r[1] == r[0] and r[2] == r[0]


def _accuracy(pred):
    return A.EvalMultiClassBatchOp().setPredictionDetailCol("pred_detail").setLabelCol("category").linkFrom(pred) \
        .collectMetrics().getAccuracy()


def test_one_vs_rest_iris():
    """OneVsRestTest.lr / pipeline / gbdtTriCls."""
    src, _ = _iris()
    lr = A.LogisticRegression().setFeatureCols(FEATS).setLabelCol("category").setMaxIter(100)
    model = A.OneVsRest().setClassifier(lr).setNumClass(3).fit(src)
    model.setPredictionCol("pred_result").setPredictionDetailCol("pred_detail")
    assert _accuracy(model.transform(src)) > 0.9

    va = A.VectorAssembler().setSelectedCols(FEATS).setOutputCol("features").setReservedCols(["category"])
    lr = A.LogisticRegression().setVectorCol("features").setLabelCol("category").setPredictionDetailCol("pred_detail") \
        .setMaxIter(100)
    model = A.Pipeline().add(va).add(A.OneVsRest().setClassifier(lr).setNumClass(3).setPredictionCol("pred_label")) \
        .fit(src)
    assert _accuracy(model.transform(src)) > 0.9
    row = model.getLocalPredictor(src.getSchema()).map((1.0, 1.0, 1.0, 1.0, "Iris-versicolor"))
    assert row[-2] in ("Iris-setosa", "Iris-versicolor", "Iris-virginica")

    gbdt = A.GbdtClassifier().setFeatureCols(FEATS).setLabelCol("category").setCategoricalCols([]).setMaxBins(128) \
        .setMaxDepth(5).setNumTrees(10).setMinSamplesPerLeaf(1).setLearningRate(0.3).setMinInfoGain(0.0) \
        .setSubsamplingRatio(1.0).setFeatureSubsamplingRatio(1.0)
    model = A.OneVsRest().setClassifier(gbdt).setNumClass(3).fit(src)
    model.setPredictionCol("pred_result").setPredictionDetailCol("pred_detail")
    assert _accuracy(model.transform(src)) > 0.9
