"""Distance measures against the reference's unit tests (``core/src/test/java/com/alibaba/alink/operator/common/
distance/{Euclidean,Cosine,ManHattan,Jaccard,Haversine}DistanceTest.java``): pair values for dense / sparse /
array inputs, and the block form equal to the pair form."""
import numpy as np
import pytest
import torch

from alink_amd.common.distance import (CosineDistance, EuclideanDistance, HaversineDistance, JaccardDistance,
                                       LevenshteinDistance, LevenshteinSimilarity, ManHattanDistance, distance_of)
from alink_amd.common.linalg import DenseVector, SparseVector

D1, D2 = DenseVector([1, 2, 4, 1, 3]), DenseVector([4, 6, 1, 2, 4])
S1, S2 = SparseVector(5, [1, 3], [0.1, 0.4]), SparseVector(5, [2, 3], [0.4, 0.1])


@pytest.mark.parametrize("dist,expect", [
    (EuclideanDistance(), [6.0, 5.47, 0.50, 8.38]),
    (CosineDistance(), [0.2852, 0.73, 0.76, 0.60]),
    (ManHattanDistance(), [12.0, 10.5, 0.8, 16.5])])
def test_continuous_pairs(dist, expect):
    got = [dist.calc(D1, D2), dist.calc(D1, S1), dist.calc(S1, S2), dist.calc(S1, D2)]
    np.testing.assert_allclose(got, expect, atol=0.01)
    assert dist.calc(D1.getData(), D2.getData()) == pytest.approx(got[0])
    block = dist.pairwise([D1, S1], [D2, S1, S2]).numpy()
    pairs = [[dist.calc(a, b) for b in (D2, S1, S2)] for a in (D1, S1)]
    np.testing.assert_allclose(block, pairs, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(dist.pairwise([D1, D2], [D1, D2]).numpy().diagonal(), [0, 0], atol=1e-7)


def test_jaccard():
    j = JaccardDistance()
    v1, v2 = DenseVector([1, 0, 4, 0, 3]), DenseVector([0, 6, 1, 0, 4])
    assert j.calc(v1, v2) == pytest.approx(0.5)
    assert j.calc(v1.getData(), v2.getData()) == pytest.approx(0.5)
    assert j.calc(v1, S1) == pytest.approx(1.0) and j.calc(S1, v1) == pytest.approx(1.0)
    assert j.calc(S1, S2) == pytest.approx(2 / 3)
    np.testing.assert_allclose(j.pairwise([v1, S1], [v2, S2]).numpy(), [[0.5, 0.75], [0.75, 2 / 3]], atol=1e-12)


def test_haversine():
    h = HaversineDistance()
    a, b = DenseVector([40, 20]), DenseVector([10, 60])
    assert h.calc(a, b) == pytest.approx(5160.251, abs=0.01)
    assert h.calc(a.getData(), b.getData()) == pytest.approx(5160.251, abs=0.01)
    assert h.calc(40, 20, 10, 60) == pytest.approx(5160.251, abs=0.01)
    np.testing.assert_allclose(h.pairwise([a, b], [a, b]).numpy(), [[0, 5160.251], [5160.251, 0]], atol=0.01)


def test_levenshtein_and_distance_type_enum():
    assert LevenshteinDistance.calcDistance("kitten", "sitting") == 3
    assert LevenshteinDistance().calc(["a", "b", "c"], ["a", "c"]) == 1
    assert LevenshteinDistance.calcDistance("", "abc") == 3
    assert LevenshteinSimilarity().similarity("abcd", "abce") == pytest.approx(0.75)
    assert isinstance(distance_of("CITYBLOCK"), ManHattanDistance)
    assert isinstance(distance_of("jaccard"), JaccardDistance)
    with pytest.raises(ValueError):
        distance_of("MAHALANOBIS")


def test_pairwise_on_torch_rows_matches_cdist():
    g = torch.Generator().manual_seed(0)
    X, Y = torch.randn(50, 8, generator=g, dtype=torch.float64), torch.randn(30, 8, generator=g, dtype=torch.float64)
    torch.testing.assert_close(EuclideanDistance().pairwise(X, Y), torch.cdist(X, Y), rtol=1e-9, atol=1e-9)
    torch.testing.assert_close(ManHattanDistance().pairwise(X, Y), torch.cdist(X, Y, p=1.0))


def test_lsh_hash_functions_reference_values():
    """MinHashLSHTest / BucketRandomProjectionLSHTest (reference operator/common/feature): table hashes of seed 0,
    2 projections x 2 tables (BRP: width 1 over 5 dims), and the key distances."""
    from alink_amd.models.similarity.lsh import BucketRandomProjectionLSH, MinHashLSH, _Rows
    rows = _Rows([DenseVector([1, 2, 3, 4, 5]), SparseVector(5, [0, 4], [1.0, 4.0])])
    assert MinHashLSH(0, 2, 2).hash(rows).tolist() == [[478212008, -1798305157], [-967745172, -594675602]]
    brp = BucketRandomProjectionLSH(0, 5, 2, 2, 1.0)
    assert brp.hash(rows, torch.device("cpu")).tolist() == [[-348137008, 1394862530], [-802232505, 1759100286]]
    a = _Rows([DenseVector([1, 0, 0, 2, 0]), SparseVector(10, [0, 4, 5, 7, 9], [1.0] * 5)])
    b = _Rows([DenseVector([0, 1, 0, 2, 1]), SparseVector(10, [0, 1, 3, 5, 9], [1.0] * 5)])
    ij = np.array([0, 1])
    np.testing.assert_allclose(MinHashLSH.distance(a, ij, b, ij), [0.75, 0.5714], atol=1e-3)
    np.testing.assert_allclose(brp.distance_fn(torch.device("cpu"))(a, ij, b, ij), [1.732, 2.0], atol=1e-3)
