"""GPU parity: the HIP path (through the C-ABI) against the fp64 oracle on the same inputs.

Inputs that cross the boundary are rounded to fp32 first (the device keeps fp32 tables and
values), so the comparison measures the device arithmetic only.  Tolerance: north_star's
1e-5 relative, with an absolute floor of 1e-8 for values that the L1 soft-threshold drives
to (near) zero.
"""

import math

import numpy as np
import pytest

from oracle import fm_ref as R

pytestmark = pytest.mark.gpu

RTOL = 1e-5
ATOL = 1e-8


from problems import f32, make_problem  # noqa: E402


def to_host(csr):
    from fm_spark_amd._native import CSRHost

    return CSRHost(csr.row_ptr, csr.col, csr.val, csr.label)


def run_both(csr_list, F, k, ids, w, V, step_size, reg_param, t0=1):
    from fm_spark_amd.engine import FMContext

    model = R.Model.empty(F, k)
    model.load(ids, w, V)
    ctx = FMContext(F, k)
    ctx.load_tables(ids, w, V)
    losses = []
    for i, csr in enumerate(csr_list):
        t = t0 + i
        ro = R.sgd_step_fast(model, csr, t, step_size, reg_param)
        go = ctx.step(to_host(csr), t, step_size, reg_param)
        assert go.executed == ro.executed
        if ro.executed:
            losses.append((go.loss_sum, ro.loss_sum))
            assert go.n_loss_rows == ro.n_loss_rows
            assert go.n_unique == ro.n_unique
            assert go.n_rows == ro.n_rows
    gids, gw, gV = ctx.export_tables()
    ctx.close()
    return model, (gids, gw, gV), losses


def assert_tables(model, g):
    gids, gw, gV = g
    pids = np.nonzero(model.present)[0]
    np.testing.assert_array_equal(gids, pids)
    np.testing.assert_allclose(gw, model.w[pids], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(gV, model.V[pids], rtol=RTOL, atol=ATOL)


def test_predict_kat(gpu):
    """FactorizationMachinesSuite.scala:30-68 (pinned KAT), unclamped."""
    from fm_spark_amd.engine import FMContext

    csr = R.explode([0, 0, 0, 0], [R.dense(1.0, 2.0, 1.5, -1.0), R.sparse(4, [(0, 0.5), (2, -1.5)]),
                                   R.sparse(5, [(0, 2.0), (4, 1.5)]), R.sparse(4, [])])
    ctx = FMContext(4, 3, w0=5.0)
    ctx.load_tables([0, 1, 2, 3], [0.1, 0.2, 0.3, 0.4],
                    [[1.0, 2.0, 3.0], [3.0, 2.0, 1.0], [-0.1, -0.1, -0.2], [-0.5, 0.3, 0.0]])
    p = ctx.predict(to_host(csr), -math.inf, math.inf)
    np.testing.assert_allclose(p, [23.77, 5.275, 5.2, 5.0], rtol=1e-6)
    # default [minLabel, maxLabel] = [0, 1] clamp (Model.scala:54-61,129-132); the empty row
    # is na.fill(globalBias) unclamped (:86)
    p = ctx.predict(to_host(csr), 0.0, 1.0)
    np.testing.assert_allclose(p, [1.0, 1.0, 1.0, 5.0], rtol=1e-6)


def test_vector_sum_kat(gpu):
    """FactorizationMachinesSuite.scala:77-100 (pinned KAT): exact (111.11, 222.22, 333.33)."""
    from fm_spark_amd.engine import FMContext

    ctx = FMContext(4, 3)
    vecs = np.array([[0.01, 0.02, 0.03], [0.1, 0.2, 0.3], [1.0, 2.0, 3.0], [10.0, 20.0, 30.0],
                     [100.0, 200.0, 300.0]])
    keys, sums = ctx.vector_sum_by_key([1, 1, 1, 1, 1], vecs)
    np.testing.assert_array_equal(keys, [1])
    assert sums[0].tolist() == [111.11, 222.22, 333.33]


def test_vector_sum_by_key_many(gpu):
    from fm_spark_amd.engine import FMContext

    rng = np.random.default_rng(3)
    keys = rng.integers(0, 3000, 20000).astype(np.int32)
    vecs = rng.normal(size=(20000, 5))
    ctx = FMContext(4, 3)
    gk, gs = ctx.vector_sum_by_key(keys, vecs)
    rk, rs = R.vector_sum_by_key(keys, vecs)
    np.testing.assert_array_equal(gk, rk)
    assert np.array_equal(gs, rs)  # same sequential order -> bitwise


@pytest.mark.parametrize("k", [5, 16, 80])
def test_loss_grad_matches_oracle(gpu, k):
    """calcLossGrad on the team forward kernel (loss-grad mode; k = 80 beyond the old kernel's 64)."""
    from fm_spark_amd.engine import FMContext

    csr, ids, w, V = make_problem(5, 300, 60, k, 6)
    model = R.Model.empty(60, k)
    model.load(ids, w, V)
    ctx = FMContext(60, k)
    ctx.load_tables(ids, w, V)
    gp, gl, gdw, gdv = ctx.loss_grad(to_host(csr))
    rp, rl, rdw, rdv = R.loss_grad(model, csr)
    np.testing.assert_allclose(gp, rp, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(gl, rl, rtol=1e-5, atol=1e-9)
    np.testing.assert_array_equal(gdw, rdw)
    np.testing.assert_allclose(gdv, rdv, rtol=1e-5, atol=1e-9)


def _gauss_draw(seed, e, f, sd):
    """numpy restatement of the device's keyed N(0, sd^2) draw (fm_kernels.hip gauss_draw)."""
    u64 = np.uint64
    e = np.asarray(e, dtype=np.uint64)

    def splitmix64(x):
        x = x + u64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> u64(30))) * u64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> u64(27))) * u64(0x94D049BB133111EB)
        return x ^ (x >> u64(31))

    with np.errstate(over="ignore"):
        c = (e << u64(10)) ^ u64(f + 1)
        h1 = splitmix64(u64(seed) ^ splitmix64(c))
        h2 = splitmix64(h1 ^ u64(0x632BE59BD9B4E019))
    u1 = ((h1 >> u64(11)) + u64(1)).astype(np.float64) * 2.0**-53
    u2 = (h2 >> u64(11)).astype(np.float64) * 2.0**-53
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2) * sd).astype(np.float32)


def test_calc_loss_grad_fills_absent_ids(gpu):
    """calcLossGrad(df, initialSd) (Model.scala:135-234): entries whose id the model lacks --
    absent rows and ids >= numFeatures alike (the left outer joins, :155-164) -- get their own
    N(0, initialSd^2) strength and vector (coalesce with randn / udfInitVec, :144-146, 170-171),
    keyed here by (seed, entry).  Checked against the oracle with every such entry relabelled as a
    feature of its own holding the drawn row; fm_loss_grad without the fill still refuses them."""
    from fm_spark_amd.engine import FMContext

    F, k, sd, seed = 200, 5, 0.05, 7
    csr, ids, w, V = make_problem(41, 250, F + 20, k, 7, hot=3)  # ids up to F + 19
    keep = ids[(ids % 4 != 1) & (ids < F)]
    ctx = FMContext(F, k)
    ctx.load_tables(keep, w[keep], V[keep])
    got = ctx.loss_grad(to_host(csr), initial_sd=sd, seed=seed)
    with pytest.raises(Exception, match="absent from the model|>= num_features"):
        ctx.loss_grad(to_host(csr))
    e_abs = np.nonzero(~np.isin(csr.col, keep))[0]
    assert len(e_abs) > 0 and (csr.col[e_abs] >= F).any()
    col = csr.col.astype(np.int64).copy()
    col[e_abs] = F + 20 + np.arange(len(e_abs))
    model = R.Model.empty(F + 20 + len(e_abs), k)
    model.load(keep, w[keep], V[keep])
    wd = _gauss_draw(seed, e_abs, -1, sd).astype(np.float64)
    Vd = np.stack([_gauss_draw(seed, e_abs, f, sd) for f in range(k)], axis=1).astype(np.float64)
    model.load(col[e_abs], wd, Vd)
    ref = R.loss_grad(model, R.CSR(csr.row_ptr, col.astype(np.int32), csr.val, csr.label))
    for g, r in zip(got, ref):
        np.testing.assert_allclose(g, r, rtol=1e-5, atol=1e-9)
    again = ctx.loss_grad(to_host(csr), initial_sd=sd, seed=seed)
    other = ctx.loss_grad(to_host(csr), initial_sd=sd, seed=seed + 1)
    assert all(np.array_equal(a, b) for a, b in zip(got, again))
    assert not np.array_equal(got[3], other[3])
    ctx.close()


def test_upload_unit_values_elided(gpu):
    """The host upload sends only the values that do not round to 1.0f (bit 31 of the id marks
    them) and the device rebuilds every entry's x: calcLossGrad's deltaWi = x (Model.scala:200)
    returns the device's x of every entry, which must be the fp32 rounding of the input exactly --
    unit, near-unit, negative, explicit-zero and large values, rows of only unit or only valued
    entries, empty rows, and rows longer than the 16-lane team."""
    from fm_spark_amd.engine import FMContext

    rng = np.random.default_rng(31)
    F, k = 3000, 4
    lens = [0, 1, 5, 16, 17, 40, 0, 33, 3, 64]
    row_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    nnz = int(row_ptr[-1])
    col = np.concatenate([rng.choice(F, size=n, replace=False) for n in lens]).astype(np.int32)
    pool = np.array([1.0, 1.0 + 1e-12, 1.0 - 1e-10, 1.0000001, 2.5, -1.0, 0.0, 1e6, np.nextafter(1.0, 2.0)])
    val = rng.choice(pool, size=nnz)
    val[row_ptr[2]:row_ptr[3]] = 1.0  # a row of unit values only
    val[row_ptr[3]:row_ptr[4]] = 2.5  # a row of valued entries only
    label = rng.normal(size=len(lens))
    ctx = FMContext(F, k)
    ctx.load_tables(np.arange(F, dtype=np.int32), rng.normal(0, 0.1, F), rng.normal(0, 0.1, (F, k)))
    _, _, dw, _ = ctx.loss_grad(to_host(R.CSR(row_ptr, col, val, label)))
    np.testing.assert_array_equal(dw, val.astype(np.float32).astype(np.float64))
    ctx.close()


@pytest.mark.parametrize("k", [1, 2, 3, 4, 8, 10, 16, 32, 48, 72, 136, 256])
def test_step_parity_k(gpu, k):
    F = 97
    batches = []
    for i in range(3):
        csr, ids, w, V = make_problem(100 + i, 400, F, k, 8)
        batches.append(csr)
    _, ids, w, V = make_problem(7, 1, F, k, 1)
    model, g, losses = run_both(batches, F, k, ids, w, V, step_size=0.5, reg_param=1e-4)
    assert_tables(model, g)
    for gl, rl in losses:
        assert gl == pytest.approx(rl, rel=RTOL)


@pytest.mark.parametrize("reg", [0.0, 1e-6, 3e-3])
def test_step_parity_l1(gpu, reg):
    """L1 on every present row (SGD.scala:177-181) incl. rows the batches never touch."""
    F, k = 400, 8
    batches = [make_problem(200 + i, 150, 120, k, 5)[0] for i in range(4)]  # ids < 120: rows 120..399 untouched
    _, ids, w, V = make_problem(9, 1, F, k, 1)
    model, g, losses = run_both(batches, F, k, ids, w, V, step_size=1.0, reg_param=reg)
    assert_tables(model, g)


def test_step_parity_hot_row(gpu):
    """One id in ~90% of 5000 rows: its run crosses many 256-entry update waves (combine path)."""
    F, k = 2000, 16
    csr, ids, w, V = make_problem(11, 5000, F, k, 10, hot=17)
    model, g, losses = run_both([csr], F, k, ids, w, V, step_size=0.1, reg_param=1e-6)
    assert_tables(model, g)
    assert losses[0][0] == pytest.approx(losses[0][1], rel=RTOL)


def test_empty_batch_and_empty_rows(gpu):
    from fm_spark_amd.engine import FMContext

    F, k = 10, 4
    _, ids, w, V = make_problem(1, 1, F, k, 1)
    ctx = FMContext(F, k)
    ctx.load_tables(ids, w, V)
    empty = R.CSR(row_ptr=np.zeros(1, np.int64), col=np.zeros(0, np.int32), val=np.zeros(0), label=np.zeros(0))
    assert not ctx.step(to_host(empty), 1, 1.0, 0.1).executed  # SGD.scala:126-128
    assert ctx.epoch == 0
    # rows but no entries: m = 3, no gradient, L1 still applies (SGD.scala:124, :157-181)
    noent = R.CSR(row_ptr=np.zeros(4, np.int64), col=np.zeros(0, np.int32), val=np.zeros(0), label=np.ones(3))
    model = R.Model.empty(F, k)
    model.load(ids, w, V)
    ro = R.sgd_step_fast(model, noent, 2, 1.0, 0.05)
    go = ctx.step(to_host(noent), 2, 1.0, 0.05)
    assert go.executed and go.n_rows == 3 and go.n_loss_rows == 0 and go.loss_sum == 0.0
    assert_tables(model, ctx.export_tables())


def test_determinism_bitwise(gpu):
    from fm_spark_amd.engine import FMContext

    F, k = 5000, 16
    csr, ids, w, V = make_problem(21, 3000, F, k, 20, hot=3)
    outs = []
    for _ in range(2):
        ctx = FMContext(F, k)
        ctx.load_tables(ids, w, V)
        for t in range(1, 4):
            ctx.step(to_host(csr), t, 0.3, 1e-5)
        outs.append(ctx.export_tables())
        ctx.close()
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)


def test_device_batch_async(gpu):
    from fm_spark_amd.engine import FMContext

    F, k = 300, 8
    csrs = [make_problem(300 + i, 200, F, k, 6)[0] for i in range(3)]
    _, ids, w, V = make_problem(8, 1, F, k, 1)
    model = R.Model.empty(F, k)
    model.load(ids, w, V)
    ctx = FMContext(F, k)
    ctx.load_tables(ids, w, V)
    dbs = [ctx.batch(to_host(c)) for c in csrs]
    ref_losses = []
    for i, (c, b) in enumerate(zip(csrs, dbs)):
        ref_losses.append(R.sgd_step_fast(model, c, i + 1, 0.2, 1e-4).loss_sum)
        ctx.step_batch(b, i + 1, 0.2, 1e-4, sync=False)
    ctx.sync()
    np.testing.assert_allclose(ctx.loss_history(), ref_losses, rtol=RTOL)
    assert_tables(model, ctx.export_tables())


def test_init_random_matches_oracle_draw(gpu):
    from fm_spark_amd.engine import FMContext

    ctx = FMContext(1000, 5, seed=1234, init_sd=0.01)
    ids = np.array([0, 7, 999, 500], dtype=np.int32)
    ctx.init_random(ids)
    gids, gw, gV = ctx.export_tables()
    rw, rV = R.init_draw(ids, 5, 1234, 0.01)
    np.testing.assert_array_equal(gids, np.sort(ids))
    order = np.argsort(ids)
    np.testing.assert_allclose(gw, rw[order], rtol=1e-6)
    np.testing.assert_allclose(gV, rV[order], rtol=1e-6)


@pytest.mark.parametrize("fuse", [False, True])
def test_prepared_batches_match_inline_sort(gpu, fuse):
    """fm_batch_prepare (sort ahead on the side stream) changes scheduling only: bit for bit the
    inline-sorted step without the fused step; with it (the singleton rows updated by the forward,
    the multi runs summed from a compacted view, test_gpu_fuse.py) the same counts, the loss to 1e-9
    and the tables within rtol 1e-5."""
    from fm_spark_amd.engine import FMContext

    F, k = 3000, 16
    csrs = [make_problem(400 + i, 1500, F, k, 12, hot=5)[0] for i in range(3)]
    _, ids, w, V = make_problem(10, 1, F, k, 1)
    outs = []
    for prep in (False, True):
        ctx = FMContext(F, k, fuse=fuse)
        ctx.load_tables(ids, w, V)
        dbs = [ctx.batch(to_host(c)) for c in csrs]
        if prep:
            dbs[0].prepare()
        for i in range(6):
            if prep and i + 1 < 6:
                dbs[(i + 1) % 3].prepare()
            ctx.step_batch(dbs[i % 3], i + 1, 0.2, 1e-5, sync=False)
        ctx.sync()
        outs.append((ctx.export_tables(), ctx.loss_history()))
        ctx.close()
    (a, la), (b, lb) = outs
    if not fuse:
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
        assert np.array_equal(la, lb)
        return
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_allclose(a[1], b[1], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(a[2], b[2], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(la, lb, rtol=1e-9)


@pytest.mark.parametrize("k", [3, 16, 80])
def test_predict_matches_oracle(gpu, k):
    """transform/predict (Model.scala:69-133) on the team forward kernel: ids the model does not
    hold (absent rows, ids >= num_features) are dropped, rows left empty score w0 unclamped, the
    rest are clamped; host CSR (fm_predict) and device batch (fm_predict_batch) agree bitwise.
    k = 80 exercises the wide-row path (the old thread-per-sample kernel stopped at 64)."""
    from fm_spark_amd.engine import FMContext

    F = 700
    csr, ids, w, V = make_problem(71 + k, 400, F + 50, k, 9, hot=4)  # ids up to F + 49
    keep = ids[(ids % 3 != 0) & (ids < F)]  # every third id absent from the model
    ctx = FMContext(F, k, w0=0.25)
    ctx.load_tables(keep, w[keep], V[keep])
    model = R.Model.empty(F, k)
    model.load(keep, w[keep], V[keep])
    model.w0 = 0.25
    ref = R.predict(model, csr, -0.5, 1.5, num_features=F)
    got = ctx.predict(to_host(csr), -0.5, 1.5)
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL)
    inrange = csr.col < F
    sub = R.CSR(np.concatenate([[0], np.cumsum([inrange[a:b].sum() for a, b in zip(csr.row_ptr[:-1], csr.row_ptr[1:])])]).astype(np.int64),
                csr.col[inrange], csr.val[inrange], csr.label)
    db = ctx.batch(to_host(sub))  # device batches only hold ids < num_features
    got_b = ctx.predict_batch(db, -0.5, 1.5)
    np.testing.assert_array_equal(got_b, ctx.predict(to_host(sub), -0.5, 1.5))
    np.testing.assert_allclose(got_b, ref, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("shards", [1, 3])
def test_init_from_batch_equals_distinct_init(gpu, shards):
    """createInitialModel on the device over the data's entries (fm_init_from_batch) equals
    fm_init_random over np.unique of the ids, bitwise, per shard; present rows are kept."""
    from fm_spark_amd.engine import FMContext

    F, k = 5000, 12
    csr = make_problem(91, 800, F, k, 15, hot=17)[0]
    for r in range(shards):
        a = FMContext(F, k, seed=77, init_sd=0.02, shard_index=r, shard_count=shards)
        b = FMContext(F, k, seed=77, init_sd=0.02, shard_index=r, shard_count=shards)
        n = a.init_from_batch(a.batch(to_host(csr)))
        u = np.unique(csr.col)
        mine = u[u % shards == r]
        b.init_random(mine)
        assert n == len(mine)
        for x, y in zip(a.export_tables(), b.export_tables()):
            assert np.array_equal(x, y)
        # a second pass over other data keeps the rows already present
        before = a.export_tables()
        csr2 = make_problem(92, 300, F, k, 15)[0]
        a.init_from_batch(a.batch(to_host(csr2)))
        gi, gw, gV = a.export_tables()
        pos = np.searchsorted(gi, before[0])
        assert np.array_equal(gw[pos], before[1]) and np.array_equal(gV[pos], before[2])


def test_int_max_feature_ids(gpu):
    """Config c4's id range: numFeatures = Int.MaxValue, so slot * stride exceeds
    2^31 floats and the sort keys are 31 bits wide.  One table of 2^31 - 1 rows at k = 4 (64-B
    records, 137 GB of HBM).  The step is invariant under relabelling ids, so the device run on
    ids spread up to Int.MaxValue - 1 is compared with the oracle on the compact labels 0..n-1."""
    from fm_spark_amd.engine import FMContext

    F, k, n = 2**31 - 1, 4, 300
    big = np.unique(np.concatenate([[0, 1, 2**30, 2**31 - 2, 2**31 - 3], 
                                    np.random.default_rng(5).integers(2**31 - 10**6, 2**31 - 1, n)]))[:n]
    n = len(big)
    csrs = [make_problem(500 + i, 300, n, k, 9, hot=3)[0] for i in range(2)]
    _, ids, w, V = make_problem(501, 1, n, k, 1)
    model = R.Model.empty(n, k)
    model.load(ids, w, V)
    ctx = FMContext(F, k)
    ctx.load_tables(big[ids], w, V)
    losses = []
    for t, c in enumerate(csrs, start=1):
        ref = R.sgd_step_fast(model, c, t, 0.3, 1e-4)
        bc = R.CSR(c.row_ptr, big[c.col].astype(np.int32), c.val, c.label)
        out = ctx.step(to_host(bc), t, 0.3, 1e-4)
        assert out.loss_sum == pytest.approx(ref.loss_sum, rel=RTOL)
        assert out.n_unique == len(np.unique(c.col))
    gi, gw, gV = ctx.export_tables()
    ctx.close()
    np.testing.assert_array_equal(gi, big[np.nonzero(model.present)[0]])
    np.testing.assert_allclose(gw, model.w[model.present], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(gV, model.V[model.present], rtol=RTOL, atol=ATOL)


def test_host_step_async_matches_sync(gpu):
    """fm_step from host CSRs without host synchronisation (two upload slots in turn) gives the
    same tables and losses, bit for bit, as synchronous calls; the host buffers are free on
    return (overwritten right after each call here)."""
    from fm_spark_amd.engine import FMContext

    F, k = 2000, 16
    csrs = [make_problem(610 + i, 700 + 50 * i, F, k, 12, hot=5)[0] for i in range(5)]
    _, ids, w, V = make_problem(611, 1, F, k, 1)
    outs = []
    for sync in (True, False):
        ctx = FMContext(F, k)
        ctx.load_tables(ids, w, V)
        for t, c in enumerate(csrs, start=1):
            h = to_host(R.CSR(c.row_ptr.copy(), c.col.copy(), c.val.copy(), c.label.copy()))
            ctx.step(h, t, 0.2, 1e-5, sync=sync)
            h.col[:] = 0  # the call borrowed the buffers only for its duration
            h.val[:] = 1e9
        ctx.sync()
        outs.append((ctx.export_tables(), ctx.loss_history()))
        ctx.close()
    (a, la), (b, lb) = outs
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert np.array_equal(la, lb) and len(la) == len(csrs)


def test_prepared_pipeline_at_c2_scale_bitwise(gpu):
    """The bench's pipeline at c2's shape (1M features, k = 8, 64K rows of 39 entries, four batches
    cycled, each prepared -- sorted on the side stream -- right after the step before it is enqueued,
    no host synchronisation): bit for bit the steps whose sorts run inline.  A step that started its
    segmented update before its batch's sort had finished would read a partly written view."""
    from oracle.fm_ref import CSR
    from fm_spark_amd.engine import FMContext

    F, k, B, z, steps = 1_000_000, 8, 65_536, 39, 40
    rng = np.random.default_rng(2028)
    csrs = []
    for _ in range(4):
        col = np.minimum((F * rng.random((B, z)) ** 3).astype(np.int64), F - 1)
        col.sort(axis=1)
        val = np.where(rng.random((B, z)) < 0.6, 1.0, f32(rng.random((B, z))))
        csrs.append(CSR(row_ptr=np.arange(0, B * z + 1, z, dtype=np.int64), col=col.ravel().astype(np.int32),
                        val=val.ravel(), label=(rng.random(B) < 0.25).astype(np.float64)))
    outs = []
    for prep in (True, False):
        ctx = FMContext(F, k, fuse=False, seed=5)
        ctx.init_random_range(0, F)
        dbs = [ctx.batch(to_host(c)) for c in csrs]
        if prep:
            dbs[0].prepare()
        for i in range(steps):
            ctx.step_batch(dbs[i % 4], i + 1, 0.1, 1e-6, sync=False)
            if prep:
                dbs[(i + 1) % 4].prepare()
        ctx.sync()
        outs.append((ctx.export_tables(), ctx.loss_history()))
        ctx.close()
    (a, la), (b, lb) = outs
    assert np.array_equal(la, lb)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
