"""GMM and bisecting k-means vs the reference docs (docs/en/gmm*.md, bisectingkmeans*.md)."""
import json

import numpy as np
import pandas as pd
import pytest

from alink_amd import *  # noqa: F401,F403
from alink_amd.models.clustering.gmm import pack_cov, unpack_cov

GMM_DATA = ["-0.6264538 0.1836433", "-0.8356286 1.5952808", "0.3295078 -0.8204684", "0.4874291 0.7383247",
            "0.5757814 -0.3053884", "1.5117812 0.3898432", "-0.6212406 -2.2146999", "11.1249309 9.9550664",
            "9.9838097 10.9438362", "10.8212212 10.5939013", "10.9189774 10.7821363", "10.0745650 8.0106483",
            "10.6198257 9.9438713", "9.8442045 8.5292476", "9.5218499 10.4179416"]


def test_gmm_doc_example():
    src = BatchOperator.fromDataframe(pd.DataFrame({"features": GMM_DATA}), schemaStr="features string")
    model = GmmTrainBatchOp().setVectorCol("features").setTol(0.).linkFrom(src)
    rows = model.collect()
    meta = json.loads(rows[0][1])
    assert meta["numFeatures"] == "2" and meta["k"] == "2"
    c0 = json.loads(rows[1][1])
    assert set(c0) == {"clusterId", "weight", "mean", "cov"} and len(c0["cov"]["data"]) == 3
    out = GmmPredictBatchOp().setVectorCol("features").setPredictionCol("cluster_id") \
        .setPredictionDetailCol("cluster_detail").linkFrom(model, src).collect()
    # EM reaches the same local optimum as the reference's documented model (component order differs)
    weights = sorted(json.loads(r[1])["weight"] for r in rows[1:])
    np.testing.assert_allclose(weights, [0.26455102514508383, 0.7354489748549162], atol=1e-9)
    for r in out:
        p = [float(x) for x in r[2].split(" ")]
        assert abs(sum(p) - 1) < 1e-9
    m = GaussianMixture().setVectorCol("features").setPredictionCol("c").fit(src)
    assert len(m.transform(src).collect()) == 15


def test_gmm_cov_packing():
    S = np.array([[1.0, 2.0, 3.0], [2.0, 5.0, 6.0], [3.0, 6.0, 9.0]])
    v = pack_cov(S)
    assert v.tolist() == [1.0, 2.0, 5.0, 3.0, 6.0, 9.0]
    np.testing.assert_array_equal(unpack_cov(v, 3), S)


def test_bisecting_kmeans_doc_example():
    df = pd.DataFrame({"id": [0, 1, 2, 3, 4, 5],
                       "vec": ["0 0 0", "0.1,0.1,0.1", "0.2,0.2,0.2", "9 9 9", "9.1 9.1 9.1", "9.2 9.2 9.2"]})
    src = BatchOperator.fromDataframe(df, schemaStr="id int, vec string")
    model = BisectingKMeansTrainBatchOp().setVectorCol("vec").setK(2).linkFrom(src)
    rows = model.collect()
    nodes = [json.loads(r[1]) for r in rows[1:]]
    assert [(n["clusterId"], n["size"]) for n in nodes] == [(1, 6), (2, 3), (3, 3)]
    np.testing.assert_allclose(nodes[0]["center"]["data"], [4.6] * 3)
    np.testing.assert_allclose(nodes[1]["center"]["data"], [0.1] * 3)
    np.testing.assert_allclose(nodes[2]["center"]["data"], [9.1] * 3)
    pred = BisectingKMeansPredictBatchOp().setPredictionCol("pred").linkFrom(model, src).collect()
    assert [r[2] for r in pred] == [0, 0, 0, 1, 1, 1]
    box = []
    BisectingKMeansPredictStreamOp(model).setPredictionCol("pred").linkFrom(
        StreamOperator.fromDataframe(df, schemaStr="id int, vec string")).link(CollectStreamOp(box))
    StreamOperator.execute()
    assert sorted((r[0], r[2]) for r in box) == [(0, 0), (1, 0), (2, 0), (3, 1), (4, 1), (5, 1)]


def test_bisecting_kmeans_k4():
    rng = np.random.default_rng(0)
    centers = np.array([[0, 0], [10, 0], [0, 10], [10, 10]], dtype=float)
    X = np.concatenate([c + rng.normal(scale=0.5, size=(30, 2)) for c in centers])
    df = pd.DataFrame({"v": [f"{a} {b}" for a, b in X]})
    src = BatchOperator.fromDataframe(df, schemaStr="v string")
    m = BisectingKMeans().setVectorCol("v").setK(4).setPredictionCol("p").setPredictionDetailCol("d").fit(src)
    out = m.transform(src).collect()
    labels = np.array([r[1] for r in out]).reshape(4, 30)
    assert all(len(set(row)) == 1 for row in labels) and len({row[0] for row in labels}) == 4
    p = [float(x) for x in out[0][2].split(" ")]
    assert abs(sum(p) - 1.0) < 1e-12


BISECT_ROWS = [
    (0, '{"vectorCol":"\\"Y\\"","distanceType":"\\"EUCLIDEAN\\"","k":"3","vectorSize":"3"}'),
    (1048576, '{"clusterId":1,"size":6,"center":{"data":[4.6,4.6,4.6]},"cost":364.61999999999995}'),
    (2097152, '{"clusterId":2,"size":3,"center":{"data":[0.1,0.1,0.1]},"cost":0.06}'),
    (3145728, '{"clusterId":3,"size":3,"center":{"data":[9.1,9.1,9.1]},"cost":0.06000000000005912}'),
    (4194304, '{"clusterId":6,"size":1,"center":{"data":[9.0,9.0,9.0]},"cost":0.0}'),
    (5242880, '{"clusterId":7,"size":2,"center":{"data":[9.149999999999999,9.149999999999999,9.149999999999999]},'
              '"cost":0.015000000000100044}')]


@pytest.mark.parametrize("detail", [False, True])
def test_bisecting_model_mapper_reference_rows(detail):
    """BisectingKMeansModelMapperTest (reference operator/common/clustering/kmeans): the tree of cluster ids
    1 -> (2, 3), 3 -> (6, 7); "0 0 0" lands in leaf cluster 2 = prediction 0, detail "0.5 0.25 0.25"."""
    from alink_amd.common.params import Params
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.models.clustering import bisecting as B
    conv = [c for n, c in vars(B).items() if n.endswith("ModelDataConverter") and isinstance(c, type)][0]
    p = Params().set("predictionCol", "pred")
    if detail:
        p.set("predictionDetailCol", "detail")
    m = B.BisectingKMeansModelMapper(conv().getModelSchema(), TableSchema(["Y"], [Types.STRING]), p)
    m.loadModel(BISECT_ROWS)
    out = m.map(("0 0 0",))
    assert out[1] == 0
    if detail:
        assert out[2] == "0.5 0.25 0.25"
        assert m.getOutputSchema() == TableSchema(["Y", "pred", "detail"], [Types.STRING, Types.LONG, Types.STRING])
    else:
        assert m.getOutputSchema() == TableSchema(["Y", "pred"], [Types.STRING, Types.LONG])


def test_multivariate_gaussian_reference_values():
    """MultivariateGaussianTest (reference operator/common/statistics/basicstatistic), degenerate covariance
    included (pseudo-inverse / pseudo-determinant)."""
    from alink_amd.common.linalg import DenseMatrix, DenseVector
    from alink_amd.models.clustering.gmm import MultivariateGaussian
    tol = 1e-5
    mu1 = DenseVector.zeros(1)
    g1 = MultivariateGaussian(mu1, DenseMatrix.ones(1, 1))
    assert g1.pdf(DenseVector([0.0])) == pytest.approx(0.39894, abs=tol)
    assert g1.pdf(DenseVector([1.5])) == pytest.approx(0.12952, abs=tol)
    g2 = MultivariateGaussian(mu1, DenseMatrix.ones(1, 1).scale(4.0))
    assert g2.pdf(DenseVector([0.0])) == pytest.approx(0.19947, abs=tol)
    assert g2.pdf(DenseVector([1.5])) == pytest.approx(0.15057, abs=tol)
    mu = DenseVector.zeros(2)
    m1 = MultivariateGaussian(mu, DenseMatrix.eye(2))
    assert m1.pdf(DenseVector.zeros(2)) == pytest.approx(0.15915, abs=tol)
    assert m1.pdf(DenseVector.ones(2)) == pytest.approx(0.05855, abs=tol)
    m2 = MultivariateGaussian(mu, DenseMatrix(2, 2, [4.0, -1.0, -1.0, 2.0]))
    assert m2.pdf(DenseVector.zeros(2)) == pytest.approx(0.060155, abs=tol)
    assert m2.pdf(DenseVector.ones(2)) == pytest.approx(0.033971, abs=tol)
    deg = MultivariateGaussian(mu, DenseMatrix(2, 2, [1.0, 1.0, 1.0, 1.0]))
    assert deg.pdf(DenseVector.zeros(2)) == pytest.approx(0.11254, abs=tol)
    assert deg.pdf(DenseVector.ones(2)) == pytest.approx(0.068259, abs=tol)


def test_gmm_predict_detail_packed():
    """GMM prediction detail strings (Double.toString of the posteriors, space separated) formatted in C++ equal
    VectorUtil.toString of the same DenseVector; predictions are an int64 column."""
    import numpy as np
    import pandas as pd
    from alink_amd import BatchOperator, GmmPredictBatchOp, GmmTrainBatchOp
    from alink_amd.common.linalg import DenseVector, VectorUtil
    rng = np.random.default_rng(0)
    X = np.concatenate([rng.standard_normal((100, 3)), rng.standard_normal((100, 3)) + 5])
    df = pd.DataFrame({"v": [" ".join(map(str, r)) for r in X]})
    b = BatchOperator.fromDataframe(df, schemaStr="v string")
    m = GmmTrainBatchOp().setVectorCol("v").setK(2).setMaxIter(20).linkFrom(b)
    out = GmmPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d").linkFrom(m, b)
    mt = out.getOutputTable()
    rows = out.collect()
    assert {r[1] for r in rows} == {0, 1}
    for r in rows[:20]:
        probs = [float(x) for x in r[2].split(" ")]
        assert r[2] == VectorUtil.toString(DenseVector(np.array(probs)))
        assert abs(sum(probs) - 1) < 1e-12
    assert mt.col("p").values.dtype.is_floating_point is False


@pytest.mark.parametrize("distance", ["EUCLIDEAN", "COSINE"])
def test_bisecting_predict_columnar_matches_rows(distance):
    """Level-by-level leaf descent over the whole matrix gives the per-row descent's clusters."""
    import numpy as np
    import pandas as pd
    from alink_amd import BatchOperator, BisectingKMeansPredictBatchOp, BisectingKMeansTrainBatchOp
    rng = np.random.default_rng(4)
    X = np.concatenate([rng.standard_normal((60, 3)) + c for c in ([0, 0, 0], [6, 0, 0], [0, 6, 0], [0, 0, 6])])
    df = pd.DataFrame({"v": [" ".join(map(str, r)) for r in X]})
    b = BatchOperator.fromDataframe(df, schemaStr="v string")
    m = BisectingKMeansTrainBatchOp().setVectorCol("v").setK(4).setDistanceType(distance).linkFrom(b)
    fast = [r[-1] for r in BisectingKMeansPredictBatchOp().setPredictionCol("p").linkFrom(m, b).collect()]
    slow = [r[-2] for r in BisectingKMeansPredictBatchOp().setPredictionCol("p").setPredictionDetailCol("d")
            .linkFrom(m, b).collect()]
    assert fast == slow and len(set(fast)) == 4


@pytest.mark.gpu
@pytest.mark.parametrize("distance", ["EUCLIDEAN", "COSINE"])
def test_bisecting_predict_device(distance):
    """Bisecting k-means predict on a cuda vector column descends on the device to the host's clusters."""
    import numpy as np
    import torch
    from alink_amd import BisectingKMeansPredictBatchOp, BisectingKMeansTrainBatchOp
    from alink_amd.common.table import Column, MTable
    from alink_amd.common.types import TableSchema, Types
    from alink_amd.operator.batch.source import TableSourceBatchOp
    rng = np.random.default_rng(4)
    X = np.concatenate([rng.standard_normal((200, 3)) + c for c in ([0, 0, 0], [6, 0, 0], [0, 6, 0], [0, 0, 6])])
    schema = TableSchema(["v"], [Types.DENSE_VECTOR])
    host = TableSourceBatchOp(MTable(schema, [Column(torch.from_numpy(X))]))
    dev = TableSourceBatchOp(MTable(schema, [Column(torch.from_numpy(X).cuda())]))
    m = BisectingKMeansTrainBatchOp().setVectorCol("v").setK(4).setDistanceType(distance).linkFrom(host)
    op = lambda: BisectingKMeansPredictBatchOp().setPredictionCol("p").setReservedCols([])  # noqa: E731
    a = op().linkFrom(m, host).getOutputTable().col("p").values
    b = op().linkFrom(m, dev).getOutputTable().col("p").values
    assert torch.equal(a.cpu(), b.cpu())
