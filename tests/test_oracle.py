"""CPU: the oracle itself, pinned to the reference's own known-answer tests, and the three
restatements (pure-Python loop, vectorised numpy, OpenMP C) against each other."""

import math

import numpy as np
import pytest

from oracle import fm_ref as R


def kat_model():
    # FactorizationMachinesSuite.scala:30-53
    m = R.Model.empty(4, 3, w0=5.0)
    m.load([0, 1, 2, 3], [0.1, 0.2, 0.3, 0.4],
           [[1.0, 2.0, 3.0], [3.0, 2.0, 1.0], [-0.1, -0.1, -0.2], [-0.5, 0.3, 0.0]])
    return m


def kat_rows():
    # FactorizationMachinesSuite.scala:34-39: dense, sparse, sparse with unlearned index 4, empty
    return R.explode([0, 0, 0, 0], [R.dense(1.0, 2.0, 1.5, -1.0), R.sparse(4, [(0, 0.5), (2, -1.5)]),
                                   R.sparse(5, [(0, 2.0), (4, 1.5)]), R.sparse(4, [])])


def test_predict_kat_unclamped():
    """FactorizationMachinesSuite.scala:64-68 at its own 1e-8 tolerance (pre-clamp)."""
    p = R.predict(kat_model(), kat_rows(), -math.inf, math.inf)
    for got, want in zip(p, [23.77, 5.275, 5.2, 5.0]):
        assert abs(got - want) <= 1e-8


def test_predict_kat_default_clamp():
    # default [minLabel, maxLabel] = [0, 1] (Model.scala:54-61); empty row -> na.fill(w0) (:86)
    assert R.predict(kat_model(), kat_rows(), 0.0, 1.0).tolist() == [1.0, 1.0, 1.0, 5.0]


def test_vector_sum_kat():
    """VectorSumSuite, FactorizationMachinesSuite.scala:83-100: exact equality."""
    vecs = [R.dense(0.01, 0.02, 0.03), R.sparse(3, [(0, 0.1), (1, 0.2), (2, 0.3)]), R.dense(1.0, 2.0, 3.0),
            R.sparse(3, [(0, 10.0), (1, 20.0), (2, 30.0)]), R.dense(100.0, 200.0, 300.0)]
    assert R.vector_sum(vecs).tolist() == [111.11, 222.22, 333.33]


def test_active_entries_rules():
    # udfVecToMap (Model.scala:244-250): dense -> every index incl. zeros; sparse -> stored
    # entries incl. explicit zeros
    assert R.active_entries(R.dense(0.0, 2.0)) == {0: 0.0, 1: 2.0}
    assert R.active_entries(R.sparse(5, [(1, 0.0), (3, 4.0)])) == {1: 0.0, 3: 4.0}
    assert R.active_entries(R.sparse(5, [])) == {}


def test_zero_entry_w_gradient_is_minus_label():
    """SURVEY P1 + P5: an explicit zero entry still moves w by +y * eta / m."""
    m = R.Model.empty(2, 2)
    m.load([0, 1], [0.0, 0.0], [[0.0, 0.0], [0.0, 0.0]])
    csr = R.explode([3.0], [R.sparse(2, [(0, 0.0), (1, 0.0)])])
    R.sgd_step(m, csr, 1, 1.0, 0.0)
    # w -= ((0*yhat - 3) / 1) * 1  ->  w = 3
    assert m.w.tolist() == [3.0, 3.0]


def test_soft_threshold_composes():
    rng = np.random.default_rng(0)
    z = rng.normal(size=1000)
    a, b = 0.3, 0.45
    np.testing.assert_allclose(R.soft_threshold(R.soft_threshold(z, a), b), R.soft_threshold(z, a + b), atol=1e-15)


def _problem(seed, B=300, F=80, k=5, hot=None):
    from problems import make_problem

    return make_problem(seed, B, F, k, 7, hot=hot)


@pytest.mark.parametrize("reg", [0.0, 1e-3])
def test_three_restatements_agree(reg):
    from oracle import oracle_c

    csr, ids, w, V = _problem(1, hot=3)
    a = R.Model.empty(80, 5)
    a.load(ids, w, V)
    b = a.copy()
    lib = oracle_c.load()
    h = oracle_c.create(lib, 80, 5)
    try:
        oracle_c.load_tables(lib, h, ids, w, V)
        for t in range(1, 4):
            ra = R.sgd_step(a, csr, t, 0.3, reg)
            rb = R.sgd_step_fast(b, csr, t, 0.3, reg)
            rc, loss, nl, nu = oracle_c.step(lib, h, csr, t, 0.3, reg)
            assert ra.loss_sum == pytest.approx(rb.loss_sum, rel=1e-13)
            assert ra.loss_sum == pytest.approx(loss, rel=1e-13)
            assert (ra.n_loss_rows, ra.n_unique) == (nl, nu)
        cw, cV, cp = oracle_c.tables(lib, h, 80, 5)
    finally:
        lib.oracle_destroy(h)
    np.testing.assert_allclose(a.w, b.w, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(a.V, b.V, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(a.w, cw, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(a.V, cV, rtol=1e-12, atol=1e-15)


def test_empty_batch_leaves_model():
    m = R.Model.empty(3, 2)
    m.load([0, 1, 2], [1.0, 2.0, 3.0], np.ones((3, 2)))
    before = m.copy()
    r = R.sgd_step(m, R.CSR(np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0), np.zeros(0)), 1, 1.0, 0.5)
    assert not r.executed
    assert np.array_equal(m.w, before.w) and np.array_equal(m.V, before.V)


def test_rows_without_entries_count_in_m_and_l1_applies():
    """m includes rows with no active entry; the L1 still runs on every row."""
    m = R.Model.empty(2, 1)
    m.load([0, 1], [1.0, -1.0], [[0.5], [0.05]])
    csr = R.explode([1.0, 0.0], [R.sparse(2, [(0, 1.0)]), R.sparse(2, [])])
    r = R.sgd_step(m, csr, 1, 1.0, 0.1)
    assert r.n_rows == 2 and r.n_loss_rows == 1
    # untouched row 1: S_0.1(-1) = -0.9, S_0.1(0.05) = 0
    assert m.w[1] == pytest.approx(-0.9) and m.V[1, 0] == 0.0


def test_init_draw_statistics():
    w, V = R.init_draw(np.arange(20000), 8, 7, 0.01)
    allv = np.concatenate([w, V.ravel()])
    assert abs(allv.mean()) < 2e-4 and abs(allv.std() - 0.01) < 2e-4
