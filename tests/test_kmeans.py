"""KMeans end to end (reference T/pipeline/clustering/KMeansTest.java, KMeansModelMapperTest.java)."""
import numpy as np
import pytest

from alink_amd import *
from alink_amd.common.types import TableSchema, Types
from tests.test_core_formats import KMEANS_ROWS

ROWS = [["0 0 0"], ["0.1 0.1 0.1"], ["0.2 0.2 0.2"], ["9 9 9"], ["9.1 9.1 9.1"], ["9.2 9.2 9.2"]]


def test_kmeans_pipeline_distances():
    data = MemSourceBatchOp(ROWS, ["vector"])
    km = KMeans().setVectorCol("vector").setPredictionCol("pred").setPredictionDistanceCol("distance").setK(2)
    model = Pipeline().add(km).fit(data)
    res = model.transform(data).select("distance").collect()
    expect = [0.173, 0, 0.173, 0.173, 0, 0.173]
    for r, e in zip(res, expect):
        assert abs(r[0] - e) < 0.01


def test_kmeans_model_mapper_detail():
    from alink_amd.models.clustering.kmeans import KMeansModelMapper, KMeansModelDataConverter
    from alink_amd.common.params import Params
    ds = TableSchema(["Y"], [Types.STRING])
    p = Params().set("predictionCol", "pred").set("predictionDetailCol", "detail").set("predictionDistanceCol",
                                                                                         "distance")
    m = KMeansModelMapper(KMeansModelDataConverter().getModelSchema(), ds, p)
    m.loadModel(KMEANS_ROWS)
    r = m.map(("0 0 0",))
    assert r[1] == 1
    assert r[2] == "0.010869565217391353 0.9891304347826086"
    assert abs(r[3] - 0.173) < 0.001
    assert m.getOutputSchema() == TableSchema(["Y", "pred", "detail", "distance"],
                                              [Types.STRING, Types.LONG, Types.STRING, Types.DOUBLE])


def test_kmeans_train_op_model_rows_format():
    data = MemSourceBatchOp(ROWS, ["vector"])
    model = KMeansTrainBatchOp().setVectorCol("vector").setK(2).linkFrom(data)
    rows = model.collect()
    assert rows[0][0] == 0 and rows[1][0] == 1048576
    meta = rows[0][1]
    assert meta.startswith('{"vectorCol":"\\"vector\\"","latitudeCol":null')
    pred = KMeansPredictBatchOp().setPredictionCol("p").linkFrom(model, data).collect()
    assert len({r[1] for r in pred[:3]}) == 1 and pred[0][1] != pred[5][1]


def test_kmeans_blobs_converges_and_recovers_centers():
    rng = np.random.default_rng(0)
    centers = rng.normal(size=(5, 4)) * 10
    lab = rng.integers(0, 5, 2000)
    X = centers[lab] + rng.normal(size=(2000, 4)) * 0.3
    rows = [[" ".join(map(str, x))] for x in X]
    op = KMeansTrainBatchOp().setVectorCol("v").setK(5).setMaxIter(50).setInitSteps(5).linkFrom(MemSourceBatchOp(rows, ["v"]))
    from alink_amd.models.clustering.kmeans import KMeansModelDataConverter
    m = KMeansModelDataConverter().load(op.collect())
    got = m.centroids
    d = np.linalg.norm(got[:, None, :] - centers[None, :, :], axis=2).min(0)
    assert d.max() < 0.2
    assert op.getTrainInfo()["iterations"] < 50


@pytest.mark.parametrize("init", ["RANDOM", "K_MEANS_PARALLEL"])
def test_kmeans_init_modes_and_cosine(init):
    rng = np.random.default_rng(1)
    X = np.abs(rng.normal(size=(300, 3)))
    rows = [[" ".join(map(str, x))] for x in X]
    data = MemSourceBatchOp(rows, ["v"])
    for dt in ["EUCLIDEAN", "COSINE"]:
        op = KMeansTrainBatchOp().setVectorCol("v").setK(3).setInitMode(init).setDistanceType(dt).linkFrom(data)
        out = KMeansPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d").linkFrom(op, data).collect()
        assert len(out) == 300 and all(0 <= r[1] < 3 for r in out)


def test_reference_seeding_rule_flag(monkeypatch):
    """Default (reference) rule: one sampled candidate per pick (LocalKmeansFunc); greedy opt-in; both give k
    distinct centroids from the candidate set."""
    import torch
    from alink_amd.models.clustering.kmeans import _local_kmeans
    g = torch.Generator().manual_seed(0)
    pts = torch.cat([torch.randn(50, 4, generator=g, dtype=torch.float64) + 10 * i for i in range(5)])
    w = torch.ones(pts.shape[0], dtype=torch.float64)
    for rule in ("greedy", "reference"):
        monkeypatch.setenv("ALINK_KMEANS_SEEDING", rule)
        C = _local_kmeans(pts, w, 5, "EUCLIDEAN", seed=3)
        assert C.shape == (5, 4)
        assert len({tuple(torch.round(c / 10).tolist()) for c in C}) >= 4
