"""GPU: the fused step (fm_config.fuse_single, on by default for prepared single-table batches with
k <= 16).

fm_batch_prepare sorts the batch; the step's split (k_split_count / scan / scatter) keeps only the
runs of two or more entries and tags those rows' headers with the step's epoch as it finds them,
the forward updates every untagged row -- a feature with one entry in the batch -- in place, and
the segmented update walks the multi runs only.  The
forward uses the update's arithmetic on the same fp32-rounded S, r and yhat; the multi runs are
summed in the same entry order, but their pieces meet at other wave boundaries of the compacted
view, so the fp64 run sums may differ in the last bits: the fused step must give the unfused step's
counts exactly, its loss to 1e-9 and its table within the north_star tolerance (rtol 1e-5,
atol 1e-8 where a strong L1 leaves values next to zero), match the fp64
oracle, and be bitwise reproducible run to run.  Cases: every kp the fused forward serves (4, 8, 12, 16) and one it does not (32, where
the switch changes nothing); rows absent from the model and an L1 that zeroes values; empty, short
and long rows (beyond the 40 entries a sample keeps in LDS: the re-read path); a feature in every
row; split chunks of 1024 sorted entries crossed by long runs; a batch that is not prepared (the
unfused path) between prepared ones.
"""

import numpy as np
import pytest

from oracle import fm_ref as R
from problems import make_problem
from test_gpu_parity import assert_tables, to_host

pytestmark = pytest.mark.gpu


def _steps(fuse, csrs, F, k, ids, w, V, steps, step_size=0.3, reg=1e-4, prepare=lambda t: True):
    from fm_spark_amd.engine import FMContext

    ctx = FMContext(F, k, fuse=fuse)
    ctx.load_tables(ids, w, V)
    dbs = [ctx.batch(to_host(c)) for c in csrs]
    losses = []
    for t in range(1, steps + 1):
        b = dbs[(t - 1) % len(dbs)]
        if prepare(t):
            b.prepare()
        o = ctx.step_batch(b, t, step_size, reg)
        losses.append((o.loss_sum, o.n_unique, o.n_loss_rows))
    out = ctx.export_tables()
    ctx.close()
    return losses, out


def _assert_same(a, b):
    (la, ta), (lb, tb) = a, b
    for (l1, u1, n1), (l2, u2, n2) in zip(la, lb):
        assert (u1, n1) == (u2, n2)
        assert l1 == pytest.approx(l2, rel=1e-9)
    np.testing.assert_array_equal(ta[0], tb[0])
    np.testing.assert_allclose(ta[1], tb[1], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(ta[2], tb[2], rtol=1e-5, atol=1e-8)


def _assert_bitwise(a, b):
    (la, ta), (lb, tb) = a, b
    assert la == lb
    for x, y in zip(ta, tb):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("k", [3, 8, 12, 16, 32])
def test_fused_matches_unfused_and_oracle(gpu, k):
    """Fused against unfused within the north_star tolerance (not bit for bit: the multi runs' fp64
    pieces meet at other wave boundaries), against the fp64 oracle, and bitwise reproducible."""
    F = 20000
    csrs = [make_problem(700 + i, 1500, F, k, 12, hot=5 + i)[0] for i in range(3)]
    _, ids, w, V = make_problem(71, 1, F, k, 1)
    fused = _steps(True, csrs, F, k, ids, w, V, 4)
    unfused = _steps(False, csrs, F, k, ids, w, V, 4)
    _assert_same(fused, unfused)
    _assert_bitwise(fused, _steps(True, csrs, F, k, ids, w, V, 4))  # reproducible
    model = R.Model.empty(F, k)
    model.load(ids, w, V)
    for t in range(1, 5):
        ro = R.sgd_step_fast(model, csrs[(t - 1) % 3], t, 0.3, 1e-4)
        np.testing.assert_allclose(fused[0][t - 1][0], ro.loss_sum, rtol=1e-6)
        assert fused[0][t - 1][1] == ro.n_unique
    assert_tables(model, fused[1])


def test_fused_absent_rows_and_l1(gpu):
    """Rows absent from the model (singletons and multi rows made present by their update) and a
    regParam whose soft-threshold zeroes values: fused and unfused agree."""
    F, k = 5000, 16
    csrs = [make_problem(760 + i, 800, F, k, 10)[0] for i in range(2)]
    _, ids, w, V = make_problem(72, 1, F, k, 1)
    keep = ids[::3]  # two thirds of the rows absent
    res = [_steps(f, csrs, F, k, keep, w[keep], V[keep], 3, step_size=0.5, reg=0.05) for f in (True, False)]
    _assert_same(res[0], res[1])


def test_fused_short_empty_long_rows_and_unprepared(gpu):
    """Rows shorter than a team's entry slots, empty rows, rows longer than the 40 entries a sample
    keeps in LDS (119 at most: the re-read path), and every third step on a batch that is not
    prepared (the unfused path, sorted inside its step) between fused ones."""
    F, k = 30000, 16
    csrs = [make_problem(780 + i, 1200, F, k, 3, empty_frac=0.3)[0] for i in range(2)]
    csrs += [make_problem(790, 300, F, k, 60)[0]]
    _, ids, w, V = make_problem(73, 1, F, k, 1)
    prep = lambda t: t % 3 != 0  # noqa: E731
    fused = _steps(True, csrs, F, k, ids, w, V, 7, prepare=prep)
    unfused = _steps(False, csrs, F, k, ids, w, V, 7, prepare=prep)
    _assert_same(fused, unfused)


def test_fused_feature_in_every_row_and_long_runs(gpu):
    """A feature present in every row (one run of n_rows entries) and hot features whose runs cross
    many 1024-entry split chunks and 256-entry update waves; the split keeps them whole and in order."""
    F, k = 200000, 8
    csrs = []
    for i in range(2):
        c, _, _, _ = make_problem(800 + i, 6000, F - 8, k, 20, hot=17 + i, empty_frac=0.0)
        col = c.col + 8
        col[c.row_ptr[:-1]] = 3  # each row's first (smallest) id becomes id 3: rows stay sorted and distinct
        csrs.append(R.CSR(c.row_ptr, col.astype(np.int32), c.val, c.label))
    _, ids, w, V = make_problem(74, 1, F, k, 1)
    fused = _steps(True, csrs, F, k, ids, w, V, 4)
    unfused = _steps(False, csrs, F, k, ids, w, V, 4)
    _assert_same(fused, unfused)
    model = R.Model.empty(F, k)
    model.load(ids, w, V)
    for t in range(1, 5):
        ro = R.sgd_step_fast(model, csrs[(t - 1) % 2], t, 0.3, 1e-4)
        assert fused[0][t - 1][1] == ro.n_unique
    assert_tables(model, fused[1])


def test_fused_all_singletons_and_all_multi(gpu):
    """Batches whose features are all singletons (nothing left for the segmented update) and all
    repeated (nothing for the fused forward)."""
    F, k = 100000, 16
    rng = np.random.default_rng(5)
    B, z = 500, 8
    ids_all = rng.permutation(F)[: B * z].astype(np.int32)
    rp = np.arange(0, B * z + 1, z, dtype=np.int64)
    single = R.CSR(rp, np.sort(ids_all.reshape(B, z), axis=1).ravel(), rng.normal(size=B * z), rng.random(B))
    pool = rng.permutation(F)[:40].astype(np.int32)
    cols = np.concatenate([np.sort(rng.choice(pool, size=z, replace=False)) for _ in range(B)]).astype(np.int32)
    multi = R.CSR(rp, cols, rng.normal(size=B * z), rng.random(B))
    _, ids, w, V = make_problem(75, 1, F, k, 1)
    fused = _steps(True, [single, multi], F, k, ids, w, V, 4)
    unfused = _steps(False, [single, multi], F, k, ids, w, V, 4)
    _assert_same(fused, unfused)


@pytest.mark.parametrize("k", [8, 16])
def test_fused_teams_take_many_samples_of_mixed_lengths(gpu, k):
    """40,000 rows, more than the forward's 2048 blocks x 8 teams, so every team walks several
    samples, of 1..19 entries (odd lengths below the 8 / 16 entry slots of a pass included).  A lane
    group with no entry in a sample flushes the previous sample's singleton rows before the entry
    loop while its neighbour flushes inside it; each must still write the other's row headers (the
    paired stores), or w misses its update and V is shrunk twice.  Three steps, the fused table
    against the unfused one and the fp64 oracle, with an L1 strong enough to show a double shrink."""
    F = 400_000
    csrs = [make_problem(900 + i + k, 40_000, F, k, 10, empty_frac=0.05)[0] for i in range(2)]
    _, ids, w, V = make_problem(76, 1, F, k, 1)
    fused = _steps(True, csrs, F, k, ids, w, V, 3, reg=1e-2)
    unfused = _steps(False, csrs, F, k, ids, w, V, 3, reg=1e-2)
    _assert_same(fused, unfused)
    model = R.Model.empty(F, k)
    model.load(ids, w, V)
    for t in range(1, 4):
        ro = R.sgd_step_fast(model, csrs[(t - 1) % 2], t, 0.3, 1e-2)
        np.testing.assert_allclose(fused[0][t - 1][0], ro.loss_sum, rtol=1e-6)
        assert fused[0][t - 1][1] == ro.n_unique
    assert_tables(model, fused[1])
