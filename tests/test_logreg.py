"""logistic_regression_test.go equivalents: coefficient vectors vs per-record
cartesian loops, packing, gradient vs numerical derivative, training works."""
import itertools
import math

import pytest
import torch

from drynx_amd.crypto import elgamal as eg
from drynx_amd.models import logistic_regression as lr
from drynx_amd.query import LogisticRegressionParameters


def _per_record(X, y, k):
    """ComputeAllApproxCoefficients + AggregateApproxCoefficients, literally."""
    d1 = X.shape[1]
    out = [[0.0] * (d1 ** (j + 1)) for j in range(k)]
    for xi, yi in zip(X.tolist(), y.tolist()):
        for s in range(d1):
            out[0][s] += xi[s] * (2 * yi - 1)
        for j in range(2, k + 1):
            ypart = yi - yi * ((-1) ** j) - 1
            for ri, comb in enumerate(itertools.product(range(d1), repeat=j)):
                p = 1.0
                for c in comb:
                    p *= xi[c]
                out[j - 1][ri] += ypart * p
    return out


@pytest.mark.parametrize("k", [1, 2, 3])
def test_approx_coefficients_match_reference_loops(k):
    g = torch.Generator().manual_seed(3)
    X = lr.augment(torch.randn(30, 3, generator=g, dtype=torch.float64))
    y = torch.randint(0, 2, (30,), generator=g)
    got = lr.approx_coefficients(X, y, k)
    exp = _per_record(X, y, k)
    for a, b in zip(got, exp):
        assert torch.allclose(a, torch.tensor(b, dtype=torch.float64), atol=1e-9)


def test_round_precision_go_semantics():
    v = torch.tensor([0.5, -0.5, 1.49, -2.5], dtype=torch.float64)
    assert lr.round_precision(v, 1.0).tolist() == [1, -1, 1, -3]


def test_gradient_matches_numerical_derivative_of_loss():
    g = torch.Generator().manual_seed(5)
    X = lr.augment(torch.randn(50, 2, generator=g, dtype=torch.float64))
    y = torch.randint(0, 2, (50,), generator=g)
    approx = lr.approx_coefficients(X, y, 2)
    w = torch.tensor([0.1, -0.2, 0.3], dtype=torch.float64)
    c = lr.POLY_APPROX_COEFFICIENTS

    def loss(w):  # the approximated log-loss the gradient belongs to
        A2 = approx[1].reshape(3, 3)
        return float((c[1] * (w * approx[0]).sum() + c[2] * (w @ A2 @ w)) / 50 + 0.5 / 50 * (w[1:] ** 2).sum())

    num = []
    for i in range(3):
        e = torch.zeros(3, dtype=torch.float64)
        e[i] = 1e-6
        num.append((loss(w + e) - loss(w - e)) / 2e-6)
    got = lr.gradient(w, approx, 50, 1.0)
    assert torch.allclose(got, torch.tensor(num, dtype=torch.float64), atol=1e-6)


def test_cost_reference_quirk():
    approx = [torch.tensor([1.0, 2.0]), torch.tensor([1.0, 0.0, 0.0, 1.0])]
    w = torch.tensor([1.0, 1.0])
    c = lr.POLY_APPROX_COEFFICIENTS
    # cost accumulates level 1, multiplies by c1, adds level 2, multiplies by c2
    exp = ((3.0 * c[1]) + 2.0) * c[2] / 10 - c[0] + (0.5 / (2 * 10)) * 1.0
    assert math.isclose(lr.cost(w, approx, 10, 0.5), exp, rel_tol=1e-12)


def test_encrypted_training_recovers_signal():
    g = torch.Generator().manual_seed(9)
    n, d = 2000, 3
    X = torch.randn(n, d, generator=g, dtype=torch.float64)
    w_true = torch.tensor([0.5, 2.0, -1.0, 0.5], dtype=torch.float64)
    y = (torch.sigmoid(lr.augment(X) @ w_true) > torch.rand(n, generator=g, dtype=torch.float64)).long()
    params = LogisticRegressionParameters(NbrRecords=n, NbrFeatures=d, Lambda=1.0, Step=0.1, MaxIterations=300,
                                          InitialWeights=[0.0] * (d + 1), K=2, PrecisionApproxCoefficients=1e3)
    kp = eg.KeyPair.generate()
    res = lr.encode_logistic_regression(X, y, params, eg.pk_table(kp.public))
    vals = eg.decrypt_auto(kp.secret, res.cv, 10000).tolist()
    assert vals == res.clear
    w = lr.decode_logistic_regression_values(vals, params)
    m, s = lr.compute_means_sds(X)
    pred = lr.predict(X, w, m, s)
    met = lr.metrics(pred, y)
    assert met["accuracy"] > 0.7 and met["auc"] > 0.75


def test_predict_homomorphic_close_to_clear():
    X = torch.tensor([[0.5, -1.0], [1.5, 0.25]], dtype=torch.float64)
    w = [0.2, -0.7, 1.1]
    kp = eg.KeyPair.generate()
    he = lr.predict_homomorphic(X, w, eg.pk_table(kp.public), kp.secret, precision=100.0)
    assert torch.allclose(he, lr.predict(X, w), atol=0.01)


# literal vectors of lib/encoding/logistic_regression_test.go:20-72 (TestComputeApproxCoefficients)
_X5 = [0, 1, 2, 3, 4]
_L2 = [0, 0, 0, 0, 0, 1, 2, 3, 4, 4, 6, 8, 9, 12, 16]
_L3 = [0] * 15 + [1, 2, 3, 4, 4, 6, 8, 9, 12, 16, 8, 12, 16, 18, 24, 32, 27, 36, 48, 64]


@pytest.mark.parametrize("y,k,expected", [
    (1, 1, [[0, 1, 2, 3, 4]]),
    (0, 1, [[0, -1, -2, -3, -4]]),
    (1, 2, [[0, 1, 2, 3, 4], [-v for v in _L2]]),
    (0, 2, [[0, -1, -2, -3, -4], _L2]),
    (1, 3, [[0, 1, 2, 3, 4], [-v for v in _L2], [-v for v in _L3]]),
    (0, 3, [[0, -1, -2, -3, -4], _L2, [-v for v in _L3]]),
])
def test_distinct_approx_coefficients_reference_vectors(y, k, expected):
    from drynx_amd.models.logistic_regression import distinct_approx_coefficients

    assert distinct_approx_coefficients(_X5, y, k) == [[float(v) for v in lvl] for lvl in expected]


@pytest.mark.parametrize("y", [0, 1])
def test_cartesian_coefficients_expand_distinct(y):
    """The encoder's cartesian layout (approx_coefficients = the reference's
    ComputeAllApproxCoefficients, one record) holds the multiset product of
    every ordering.  The two reference functions sign levels >= 2 differently
    (ComputeAll: ypart_j; Distinct: the running product of the ypart factors,
    logistic_regression.go:338-361 vs :382-399), so magnitudes are compared."""
    import itertools

    from drynx_amd.models.logistic_regression import approx_coefficients, distinct_approx_coefficients

    x = [1.0, 0.5, -2.0, 3.0]
    cart = approx_coefficients(torch.tensor([x], dtype=torch.float64), torch.tensor([y]), 3)
    dist = distinct_approx_coefficients(x, y, 3)
    n = len(x)
    for j in (1, 2, 3):
        lookup = dict(zip(itertools.combinations_with_replacement(range(n), j), dist[j - 1]))
        flat = cart[j - 1].tolist()
        for pos, idx in enumerate(itertools.product(range(n), repeat=j)):
            assert abs(flat[pos]) == pytest.approx(abs(lookup[tuple(sorted(idx))]))


def test_lr_evaluation_helpers():
    """FindMinimumWeightsWithEncryption, Predict on an encrypted record,
    StandardiseWithTrain / NormalizeWith and PartitionDataset
    (lib/encoding/logistic_regression.go:746, :820, :943-1012, :1389)."""
    import torch

    from drynx_amd.crypto import elgamal as eg
    from drynx_amd.models import logistic_regression as lr

    g = torch.Generator().manual_seed(5)
    X = torch.rand((60, 3), generator=g, dtype=torch.float64) * 4
    y = (X[:, 0] + 0.5 * X[:, 1] > 2.5).to(torch.int64)
    Xtr, ytr, Xte, yte = lr.partition_dataset(X, y, 0.75, shuffle=False)
    assert Xtr.shape[0] == 45 and Xte.shape[0] == 15 and torch.equal(Xtr, X[:45]) and torch.equal(yte, y[45:])
    a = lr.partition_dataset(X, y, 0.8, shuffle=True, seed=7)
    b = lr.partition_dataset(X, y, 0.8, shuffle=True, seed=7)
    assert torch.equal(a[0], b[0]) and a[0].shape[0] == 48 and not torch.equal(a[0], X[:48])
    st = lr.standardise_with_train(Xte, Xtr)
    m, s = lr.compute_means_sds(Xtr)
    assert torch.allclose(st, (Xte - m) / s)
    nw = lr.normalize_with(Xte, Xtr)
    assert torch.allclose(nw, (Xte - Xtr.min(0).values) / (Xtr.max(0).values - Xtr.min(0).values))
    assert torch.allclose(lr.normalize(Xtr).min(0).values, torch.zeros(3, dtype=torch.float64))
    # training on encrypted coefficients == training on the clear ones
    from drynx_amd.query import LogisticRegressionParameters

    p = LogisticRegressionParameters(NbrRecords=45, NbrFeatures=3, Lambda=1.0, Step=0.1, MaxIterations=50,
                                     InitialWeights=[0.1] * 4, K=2, PrecisionApproxCoefficients=100.0)
    vals = lr.encode_coefficients_int(Xtr, ytr, p)
    kp = eg.KeyPair.generate()
    pk = eg.pk_table(kp.public)
    lv1, lv2 = vals[:4], vals[4:]
    enc = [eg.encrypt_ints(pk, lv1)[0], eg.encrypt_ints(pk, lv2)[0]]
    w, approx = lr.find_minimum_weights_with_encryption(enc, kp.secret, p.InitialWeights, 45, 1.0, 0.1, 50, 100.0)
    assert w == lr.decode_logistic_regression_values(vals.tolist(), p)
    assert approx[0] == [v / 100.0 for v in lv1.tolist()]
    # Predict on one encrypted record vs PredictInClear
    x = [1.5, 0.25, 3.0]
    cv, _ = eg.encrypt_ints(pk, [round(v * 100) for v in x])
    pe = lr.predict_encrypted(cv, w, kp.secret, 100.0, 100.0)
    assert abs(pe - lr.predict_in_clear(x, w)) < 1e-2
    c = lr.logistic_regression_cost(w, lr.augment(Xtr), ytr, 45, 1.0)
    assert c > 0 and len(lr.logistic_regression_gradient(w, lr.augment(Xtr), ytr, 45, 1.0)) == 4
