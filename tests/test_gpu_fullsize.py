"""GPU parity at BASELINE.json's full sizes.

c2 (1M features, k = 8, 64K rows): the whole table is compared with the fp64 oracle after three
steps (the dense oracle fits in host memory at this size).

c3 (100M hashed features, k = 16, 256K rows, Zipf(1.05)): the oracle cannot hold a 100M-row
table, so the step is checked through properties that do not depend on size:
  * the batch statistics (rows, loss rows, distinct ids) equal host counts;
  * the loss equals the fp64 forward of the whole batch over the exported pre-step table;
  * a feature's update depends only on the samples that hold it, so for a chosen set of
    features (the three hottest ids — runs of thousands of entries that cross many update
    waves —, twenty ids with 200..2000 entries and a thousand random ids) the oracle step
    over just those samples (padded with empty rows to the full miniBatchSize, which only
    count in m) must give the device's rows for them;
  * rows present but absent from the next batch only receive that step's L1 shrink;
  * two contexts running the same sequence end bitwise identical.
The synthetic data is the bench's generator (fm_spark_amd.data.synthetic_batch).
"""

import math

import numpy as np
import pytest

from oracle import fm_ref as R

pytestmark = pytest.mark.gpu

RTOL = 1e-5
ATOL = 1e-8
STEP, REG = 0.1, 1e-6


def _host(b):
    from fm_spark_amd._native import CSRHost

    return CSRHost(b.row_ptr, b.col, b.val, b.label)


def _rows_of(b):
    return np.repeat(np.arange(b.n_rows), np.diff(b.row_ptr))


def _lookup(ids, table_ids):
    pos = np.searchsorted(table_ids, ids)
    assert np.all(table_ids[np.minimum(pos, len(table_ids) - 1)] == ids), "id missing from the exported table"
    return pos


def _forward_loss(b, ids, w, V):
    """fp64 forward of the whole batch (Model.scala:173-230) over an exported table; every row
    of the synthetic batches holds 39 entries, so CSR segments are never empty."""
    rp = b.row_ptr
    assert np.all(np.diff(rp) > 0)
    p = _lookup(b.col.astype(np.int64), ids)
    x = b.val
    Vp = V[p]
    S = np.add.reduceat(Vp * x[:, None], rp[:-1], axis=0)
    vv = np.add.reduceat(np.sum(Vp * Vp, axis=1) * x * x, rp[:-1])
    wx = np.add.reduceat(w[p] * x, rp[:-1])
    yhat = 0.5 * (np.sum(S * S, axis=1) - vv) + wx
    d = yhat - b.label
    return float(np.sum(d * d))


def _sub_problem(b, chosen):
    """The samples holding any chosen id, all their entries, padded with empty rows to b's
    row count (empty rows count in miniBatchSize, SGD.scala:124, and nowhere else)."""
    rows = _rows_of(b)
    samples = np.unique(rows[np.isin(b.col, chosen)])
    lens = np.diff(b.row_ptr)[samples]
    starts = b.row_ptr[samples]
    tot = int(lens.sum())
    first = np.concatenate([[0], np.cumsum(lens)[:-1]])
    idx = np.arange(tot) + np.repeat(starts - first, lens)
    pad = b.n_rows - len(samples)
    row_ptr = np.concatenate([[0], np.cumsum(lens), np.full(pad, tot)]).astype(np.int64)
    label = np.concatenate([b.label[samples], np.zeros(pad)])
    return row_ptr, b.col[idx].astype(np.int64), b.val[idx], label, len(samples)


def _check_chosen(b, before, after, chosen, t):
    ids0, w0, V0 = before
    ids1, w1, V1 = after
    row_ptr, col, val, label, ns = _sub_problem(b, chosen)
    uniq, inv = np.unique(col, return_inverse=True)
    k = V0.shape[1]
    model = R.Model.empty(len(uniq), k)
    p0 = _lookup(uniq, ids0)
    model.load(np.arange(len(uniq)), w0[p0], V0[p0])
    R.sgd_step_fast(model, R.CSR(row_ptr, inv.astype(np.int32), val, label), t, STEP, REG)
    c = np.searchsorted(uniq, chosen)
    p1 = _lookup(chosen, ids1)
    np.testing.assert_allclose(w1[p1], model.w[c], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(V1[p1], model.V[c], rtol=RTOL, atol=ATOL)
    return ns


def _choose(b, rng):
    ids, cnt = np.unique(b.col.astype(np.int64), return_counts=True)
    order = np.argsort(-cnt, kind="stable")
    hot = ids[order[:3]]
    mid_pool = ids[(cnt >= 200) & (cnt <= 2000)]
    mid = rng.choice(mid_pool, size=min(20, len(mid_pool)), replace=False)
    cold = rng.choice(ids, size=1000, replace=False)
    chosen = np.unique(np.concatenate([hot, mid, cold]))
    return chosen, int(cnt[order[0]]), len(ids)


def test_c3_full_size_step_properties(gpu):
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.engine import FMContext

    F, k, B = 100_000_000, 16, 262144
    hb = [synthetic_batch(B, F, batch_index=i) for i in range(2)]
    rng = np.random.default_rng(11)

    def run():
        ctx = FMContext(F, k, seed=20261015, init_sd=0.01)
        b1 = ctx.batch(_host(hb[0]))
        ctx.init_from_batch(b1)  # createInitialModel over the data's ids (SGD.scala:218-252)
        t0 = ctx.export_tables()
        o1 = ctx.step_batch(b1, 1, STEP, REG, sync=True)
        t1 = ctx.export_tables()
        b2 = ctx.batch(_host(hb[1]))
        ctx.init_from_batch(b2)
        t1b = ctx.export_tables()
        o2 = ctx.step_batch(b2, 2, STEP, REG, sync=True)
        t2 = ctx.export_tables()
        out = (t0, o1, t1, t1b, o2, t2)
        b1.close()
        b2.close()
        ctx.close()
        return out

    t0, o1, t1, t1b, o2, t2 = run()

    # batch statistics
    for o, b in ((o1, hb[0]), (o2, hb[1])):
        assert o.n_rows == B
        assert o.n_loss_rows == int(np.count_nonzero(np.diff(b.row_ptr)))
        assert o.n_unique == len(np.unique(b.col))
    np.testing.assert_array_equal(t1[0], t0[0])  # every id of batch 1 was present before its step

    # whole-batch loss against the fp64 forward over the pre-step tables
    assert o1.loss_sum == pytest.approx(_forward_loss(hb[0], *t0), rel=1e-9)
    assert o2.loss_sum == pytest.approx(_forward_loss(hb[1], *t1b), rel=1e-9)

    # per-feature update parity on the samples that hold the chosen ids
    chosen, top, U = _choose(hb[0], rng)
    assert top > 1000 and U > 5_000_000  # the workload's skew reaches the long-run paths
    _check_chosen(hb[0], t0, t1, chosen, 1)
    chosen2, _, _ = _choose(hb[1], rng)
    _check_chosen(hb[1], t1b, t2, chosen2, 2)

    # rows present after step 1 but absent from batch 2 only shrink by step 2's lambda
    only1 = np.setdiff1d(t1[0], hb[1].col.astype(np.int64))
    probe = rng.choice(only1, size=5000, replace=False)
    lam2 = STEP / math.sqrt(2) * REG
    pa, pb = _lookup(probe, t1[0]), _lookup(probe, t2[0])
    np.testing.assert_allclose(t2[1][pb], R.soft_threshold(t1[1][pa], lam2), rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(t2[2][pb], R.soft_threshold(t1[2][pa], lam2), rtol=1e-6, atol=1e-9)

    # determinism: a second context on the same sequence ends bitwise identical
    _, q1, _, _, q2, u2 = run()  # the same calls: exports flush the lazy L1
    assert (q1.loss_sum, q2.loss_sum) == (o1.loss_sum, o2.loss_sum)
    for x, y in zip(t2, u2):
        assert np.array_equal(x, y)


def test_c2_full_size_table_parity(gpu):
    """c2: 1M features, k = 8, 64K rows per mini-batch, Zipf(1.05): three steps over the whole
    table against the fp64 oracle (every row, losses, counts)."""
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.engine import FMContext

    F, k, B = 1_000_000, 8, 65536
    hb = [synthetic_batch(B, F, batch_index=10 + i) for i in range(3)]
    ctx = FMContext(F, k, seed=7, init_sd=0.01)
    ctx.init_random_range(0, F)
    ids, w, V = ctx.export_tables()
    assert len(ids) == F
    model = R.Model.empty(F, k)
    model.load(ids, w, V)
    for t, b in enumerate(hb, start=1):
        ref = R.sgd_step_fast(model, R.CSR(b.row_ptr, b.col, b.val, b.label), t, STEP, REG)
        out = ctx.step(_host(b), t, STEP, REG)
        assert out.n_unique == ref.n_unique and out.n_loss_rows == ref.n_loss_rows
        assert out.loss_sum == pytest.approx(ref.loss_sum, rel=RTOL)
    gi, gw, gV = ctx.export_tables()
    ctx.close()
    np.testing.assert_array_equal(gi, np.arange(F))
    np.testing.assert_allclose(gw, model.w, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(gV, model.V, rtol=RTOL, atol=ATOL)


def test_c2_replicated_r8_full_table_parity(gpu):
    """c2's whole table replicated over R = 8 ranks of one context (COPY transport, every replica on
    this GPU): each rank steps its eighth of the 64K-row mini-batch, the per-slot gradient sums cross
    ranks as fp32 (the all-reduce of fm_repl_grad's buffer, include/fm_hip.h) and every replica
    applies the same update.  Five steps against the fp64 oracle over the whole table: the fp32
    cross-rank sums stay within the north_star tolerance (rtol 1e-5; the largest relative error
    over values >= 1e-6 is printed)."""
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.engine import FMContext

    F, k, B, NR = 1_000_000, 8, 65536, 8
    hb = [synthetic_batch(B, F, batch_index=60 + i) for i in range(5)]
    ctx = FMContext(F, k, seed=7, init_sd=0.01, parallel="replicated", n_gpus=NR, devices=[0] * NR, transport="copy")
    ctx.init_random_range(0, F)
    ids, w, V = ctx.export_tables()
    assert len(ids) == F
    model = R.Model.empty(F, k)
    model.load(ids, w, V)
    for t, b in enumerate(hb, start=1):
        ref = R.sgd_step_fast(model, R.CSR(b.row_ptr, b.col, b.val, b.label), t, STEP, REG)
        out = ctx.step(_host(b), t, STEP, REG)
        assert out.n_unique == ref.n_unique and out.n_loss_rows == ref.n_loss_rows
        assert out.loss_sum == pytest.approx(ref.loss_sum, rel=RTOL)
    gi, gw, gV = ctx.export_tables()
    ctx.close()
    np.testing.assert_array_equal(gi, np.arange(F))
    np.testing.assert_allclose(gw, model.w, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(gV, model.V, rtol=RTOL, atol=ATOL)
    big = np.abs(model.V) >= 1e-6
    print(f"c2 replicated x{NR}: max relative V error {np.max(np.abs(gV[big] - model.V[big]) / np.abs(model.V[big])):.3e}")


def test_c3_whole_table_parity_against_c_oracle(gpu):
    """c3 at full size, every row: the whole 100M x k = 16 table, initialised with the device's
    seeded draw on both sides (oracle_init_device_draw replicates it), stepped twice -- the device
    through prepared batches (the fused step: singleton rows updated by the forward, the rest by the
    segmented update, lazy L1 for the untouched rows) and the fp64 C oracle (oracle/fm_oracle.c,
    eager L1 over every row as SGD.scala:157-181) -- then every row compared in id-range chunks
    through fm_export_rows at rtol 1e-5 (atol 1e-8 for values the L1 leaves next to zero)."""
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.engine import FMContext
    from oracle import oracle_c

    F, k, B, seed, sd = 100_000_000, 16, 262144, 20261015, 0.01
    hb = [synthetic_batch(B, F, batch_index=40 + i) for i in range(2)]
    lib = oracle_c.load()
    m = oracle_c.create(lib, F, k)
    try:
        lib.oracle_init_device_draw(m, seed, sd, 0, F)
        ctx = FMContext(F, k, seed=seed, init_sd=sd)
        ctx.init_random_range(0, F)
        dbs = [ctx.batch(_host(b)) for b in hb]
        for t, (b, db) in enumerate(zip(hb, dbs), start=1):
            db.prepare()
            go = ctx.step_batch(db, t, STEP, REG, sync=True)
            rc, loss, nl, nu = oracle_c.step(lib, m, b, t, STEP, REG)
            assert rc == 0
            assert (go.n_loss_rows, go.n_unique) == (nl, nu)
            assert go.loss_sum == pytest.approx(loss, rel=1e-9)
        ow, oV, opres = (np.ctypeslib.as_array(lib.oracle_w(m), shape=(F,)),
                         np.ctypeslib.as_array(lib.oracle_V(m), shape=(F * k,)).reshape(F, k),
                         np.ctypeslib.as_array(lib.oracle_present(m), shape=(F,)))
        worst = 0.0
        chunk = 1 << 23
        for a in range(0, F, chunk):
            ids = np.arange(a, min(F, a + chunk), dtype=np.int32)
            w, V, pres = ctx.export_rows(ids)
            assert pres.all() and opres[a:a + len(ids)].all()
            np.testing.assert_allclose(w, ow[a:a + len(ids)], rtol=RTOL, atol=ATOL)
            np.testing.assert_allclose(V, oV[a:a + len(ids)], rtol=RTOL, atol=ATOL)
            ref = oV[a:a + len(ids)]
            big = np.abs(ref) >= 1e-6
            worst = max(worst, float(np.max(np.abs(V[big] - ref[big]) / np.abs(ref[big]))))
        print(f"c3 whole table: {F} rows x {k} compared after 2 steps, max relative error {worst:.3e}")
        ctx.close()
    finally:
        lib.oracle_destroy(m)


def test_c3_split_views_bitwise_equal_host_batches(gpu):
    """c3 at full size through the estimator's loop: three 256K-row mini-batches laid out as one
    split-ordered resident dataset (fm_batch_create_splits) and stepped in place through two views
    re-pointed in turn, sorted on the side stream one iteration ahead, every step only enqueued
    (ml.run_minibatch_sgd_splits, the fit path), against a second context stepping the same rows
    uploaded as host batches, prepared and stepped synchronously: the loss sums and every one of the
    100M rows (fm_export_rows in id-range chunks) bitwise equal."""
    import bench
    from fm_spark_amd import ml
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.engine import FMContext

    F, k, B, n, seed, sd = 100_000_000, 16, 262144, 3, 20261015, 0.01
    hb = [synthetic_batch(B, F, batch_index=50 + i) for i in range(n)]
    lay = bench.concat_batches(hb)
    split_rows = np.arange(n + 1, dtype=np.int64) * B

    a = FMContext(F, k, seed=seed, init_sd=sd)
    a.init_random_range(0, F)
    data = a.batch_splits(_host(lay), split_rows)
    la = ml.run_minibatch_sgd_splits(a, data, STEP, REG)
    a.sync()

    b = FMContext(F, k, seed=seed, init_sd=sd)
    b.init_random_range(0, F)
    lb = []
    for t, h in enumerate(hb, start=1):
        db = b.batch(_host(h))
        db.prepare()
        lb.append(b.step_batch(db, t, STEP, REG, sync=True).loss_sum)
        db.close()
    assert list(la) == lb

    chunk = 1 << 23
    for s in range(0, F, chunk):
        ids = np.arange(s, min(F, s + chunk), dtype=np.int32)
        wa, Va, pa = a.export_rows(ids)
        wb, Vb, pb = b.export_rows(ids)
        assert pa.all() and pb.all()
        assert np.array_equal(wa, wb) and np.array_equal(Va, Vb)
    data.close()
    a.close()
    b.close()
