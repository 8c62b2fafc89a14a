"""Objective functions against the reference's golden values (``core/src/test/java/com/alibaba/alink/operator/
common/linear/objFunc/{UnaryObjFuncTest,SoftmaxObjFuncTest}.java``): line-search losses, constrained (OWL-QN)
search losses, objective value, gradient and Hessian diagonal of L1 = L2 = 0.1 log loss and 3-class softmax.

The reference asserts with an absolute 1e-16; its sums run in Java's sample order, ours as tensor reductions,
so the values are checked to 1e-12 relative (the last binary digits of a 100-term sum)."""
import numpy as np
import pytest
import torch

from alink_amd.models.common.features import FeatureMatrix
from alink_amd.models.linear.objfunc import LabeledData, LogLossFunc, SoftmaxObjFunc, UnaryLossObjFunc

D = 10
REL = 1e-12


def _data(rows, labels, weights, ncols=D):
    X = torch.tensor(rows, dtype=torch.float64)[:, :ncols].contiguous()
    return LabeledData(FeatureMatrix(X), torch.tensor(labels, dtype=torch.float64),
                       torch.tensor(weights, dtype=torch.float64))


def _search_data():
    rows = [[j + 0.1 * i for j in range(D)] for i in range(100)]
    return _data(rows, [1.0 - i % 2 for i in range(100)], [1.0] * 100)


def _grad_data():
    rows = [[1.0 + 0.1 * i for _ in range(D)] for i in range(100)]
    return _data(rows, [1.0 * (i % 2) for i in range(100)], [i * 0.1 for i in range(100)])


def _lr():
    return UnaryLossObjFunc(LogLossFunc(), l1=0.1, l2=0.1)


def test_unary_search_values():
    coef = torch.tensor([1.0 + 0.5 * i for i in range(D)], dtype=torch.float64)
    dirv = torch.tensor([i + 0.5 for i in range(D)], dtype=torch.float64)
    got = _lr().calc_search_values(_search_data(), coef, dirv, 1.0, 10)
    expect = [34.65735902799723, 10322.157359028002, 37947.15735902796, 65572.15735902794, 93197.15735902794,
              120822.15735902793, 148447.157359028, 176072.15735902806, 203697.15735902812, 231322.15735902818]
    np.testing.assert_allclose(got[:D].numpy(), expect, rtol=REL)


def test_unary_constraint_search_values():
    coef = torch.tensor([1.0 + 0.5 * i for i in range(D)], dtype=torch.float64)
    dirv = torch.tensor([i + 0.1 for i in range(D)], dtype=torch.float64)
    got = _lr().constraint_calc_search_values(_search_data(), coef, dirv, 0.5, 10)
    expect = [34.65735902799723, 34.65735902799723, 37.163138901642334, 39.847755908478675, 40.14874960561338,
              40.48932608213041, 40.87755215903219, 41.323690786508514, 41.84091851878743, 42.44629788093937]
    np.testing.assert_allclose(got[:D].numpy(), expect, rtol=REL)


def test_unary_obj_value():
    coef = torch.tensor([1.0 + 0.5 * i for i in range(D)], dtype=torch.float64)
    f, _ = _lr().calc_obj_value(_search_data(), coef)
    assert f == pytest.approx(16.221573590279974, rel=REL)


def test_unary_gradient():
    coef = torch.tensor([1.0 + 0.01 * i for i in range(D)], dtype=torch.float64)
    g, _ = _lr().calc_gradient(_grad_data(), coef)
    expect = [0.29999999645330994 + 0.002 * i for i in range(D)]
    np.testing.assert_allclose(g.numpy(), expect, rtol=REL)


def test_unary_hessian_diagonal():
    coef = torch.tensor([1.0 + 0.01 * i for i in range(D)], dtype=torch.float64)
    H, _, _, _ = _lr().calc_hessian_gradient_loss(_grad_data(), coef)
    np.testing.assert_allclose(torch.diagonal(H).numpy(), [99.0000020939605] * D, rtol=REL)


# ---- softmax, 3 classes: coef = 2 blocks x 5 features (the reference reads the first coef.size / (k-1) entries
# of every 10-entry sample vector) ----
def _softmax_data():
    rows = [[j + 0.1 * i for j in range(D)] for i in range(100)]
    return _data(rows, [1.0] * 100, [1.0] * 100, ncols=D // 2)


def _softmax():
    return SoftmaxObjFunc(3, l1=0.1, l2=0.1)


COEF_S = torch.tensor([1.0 + 0.1 * i for i in range(D)], dtype=torch.float64)


def test_softmax_search_values():
    got = _softmax().calc_search_values(_softmax_data(), COEF_S, torch.full((D,), 0.5, dtype=torch.float64), 0.5,
                                        10)
    expect = [0.030403516448075152, 0.03040384780510408, 0.03040847327743279, 0.030475957193068837,
              0.03153435656977166, 0.05059162113327886, 0.5457886921018531, 118.42109132310769,
              943.4408732404858, 1811.2962418211239]
    np.testing.assert_allclose(got[:D].numpy(), expect, rtol=1e-10)


def test_softmax_obj_value():
    f, _ = _softmax().calc_obj_value(_softmax_data(), COEF_S)
    assert f == pytest.approx(3.6353040351644808, rel=REL)


def test_softmax_gradient():
    g, _ = _softmax().calc_gradient(_softmax_data(), COEF_S)
    expect = [0.3001070700605414, 0.32041053188156643, 0.34071399370259137, 0.3610174555236164,
              0.38132091734464146, 0.3998929299196802, 0.4195894678341977, 0.43928600574871535,
              0.4589825436632329, 0.4786790815777505]
    np.testing.assert_allclose(g.numpy(), expect, rtol=1e-10)


def test_softmax_hessian_diagonal():
    H, _, _, _ = _softmax().calc_hessian_gradient_loss(_softmax_data(), COEF_S)
    expect = [20.008609951451433, 20.060220545670703, 20.172295036435074, 20.34483342374455, 20.577835707599135,
              20.008609951941853, 20.060220576228186, 20.172295149343217, 20.344833671286942, 20.57783614205936]
    np.testing.assert_allclose(torch.diagonal(H).numpy(), expect, rtol=1e-10)


def test_unary_loss_function_properties():
    """UnaryLossFuncTest (reference operator/common/linear/unarylossfunc): margin losses decrease in the margin,
    are symmetric in (eta, y) -> (-eta, -y), convex; regression losses vanish and are flat at the target."""
    from alink_amd.models.linear import objfunc as O
    t = lambda v: torch.tensor(v, dtype=torch.float64)     # noqa: E731

    def f(fn, eta, y):
        return float(fn(t(eta), t(y)))
    for lf in (O.ExponentialLossFunc(), O.HingeLossFunc(), O.LogisticLossFunc(), O.LogLossFunc(),
               O.PerceptronLossFunc(), O.ZeroOneLossFunc()):
        name = type(lf).__name__
        assert f(lf.loss, -1.0, 1.0) > 1.0 - 1e-10, name
        assert f(lf.loss, 1.0, 1.0) < 0.5, name
        assert f(lf.loss, -0.5, 1.0) - f(lf.loss, 0.5, 1.0) > 0.49, name
        assert f(lf.loss, -0.5, 1.0) == f(lf.loss, 0.5, -1.0), name
        assert f(lf.derivative, -0.5, 1.0) <= f(lf.derivative, 0.5, 1.0), name
        assert f(lf.second_derivative, -0.5, 1.0) >= f(lf.second_derivative, 0.5, 1.0), name
    for lf in (O.SquareLossFunc(), O.SvrLossFunc(1.0), O.HuberLossFunc(1.0)):
        name = type(lf).__name__
        assert abs(f(lf.loss, 0.0, 0.0)) < 1e-10 and abs(f(lf.derivative, 0.0, 0.0)) < 1e-10, name
        assert f(lf.derivative, -0.5, 0.0) == -f(lf.derivative, 0.5, 0.0), name
        assert f(lf.second_derivative, -0.5, 0.0) == f(lf.second_derivative, 0.5, 0.0), name


# ---- AftObjFuncTest: 100 samples of 10 entries (x_j = j + 0.01 i), censor 1, label 1; the vectors are as long
# as the coefficients, so the dot product covers log(sigma) too (AftRegObjFunc.getDotProduct) ----
def _aft_data():
    rows = [[j + 0.01 * i for j in range(D)] for i in range(100)]
    return _data(rows, [1.0] * 100, [1.0] * 100)


def _aft(l1=0.1, l2=0.1):
    from alink_amd.models.linear.objfunc import AftRegObjFunc
    return AftRegObjFunc(l1=l1, l2=l2)


AFT_COEF = torch.tensor([1.0 + 0.01 * i for i in range(D)], dtype=torch.float64)
AFT_SEARCH = [1858.0906639, 1854.4931528, 1846.4415772, 1833.475521, 1815.0990642, 1790.7783532, 1759.9390144,
              1721.9634027, 1676.1876744, 1621.8986742]


def test_aft_search_values():
    dirv = torch.full((D,), 0.1, dtype=torch.float64)
    got = _aft().calc_search_values(_aft_data(), AFT_COEF, dirv, 0.5, 10)
    np.testing.assert_allclose(np.round(got[:D].numpy(), 7), AFT_SEARCH, atol=1e-9)
    got = _aft().constraint_calc_search_values(_aft_data(), AFT_COEF, dirv, 0.5, 10)
    np.testing.assert_allclose(np.round(got[:D].numpy(), 7), AFT_SEARCH, atol=1e-9)


def test_aft_objective_and_gradient():
    f, _ = _aft().calc_obj_value(_aft_data(), AFT_COEF)
    assert round(float(f), 7) == 20.7187566
    g, _ = _aft().calc_gradient(_aft_data(), AFT_COEF)
    expect = [0.4664272, 0.8046436, 1.1428601, 1.4810766, 1.8192931, 2.1575096, 2.495726, 2.8339425, 3.172159,
              -12.9805304]
    np.testing.assert_allclose(np.round(g.numpy(), 7), expect, atol=1e-9)


def test_aft_hessian_diagonal():
    H, _, _, _ = _aft(1e-2, 1e-2).calc_hessian_gradient_loss(_aft_data(), AFT_COEF)
    expect = [2.0000000510094984, 2.000000737376146, 2.000002340193193, 2.00000485946064, 2.000008295178487,
              2.0000126473467335, 2.0000179159653797, 2.000024101034426, 2.000031202553872, 1751.091754655224]
    np.testing.assert_allclose(torch.diagonal(H).numpy(), expect, rtol=1e-12)
