"""GPU: the dataset kept on the device (dfData.cache(), FactorizationMachinesSGD.scala:93) and each
randomSplit split (:111-112) taken from it: laid out split after split and stepped in place
(fm_batch_create_splits / fm_batch_split_view), or gathered there from its row list
(fm_batch_from_rows); then the pipelined fit (the next split sorted on the side stream while the
current one steps).

A split view and fm_batch_from_rows must give the batch a host CSR of the same rows gives -- the same
rows, labels and entries in the same order, so every step on it is bitwise the host batch's step --
and the pipelined fit the synchronous fit's model and loss log."""

import logging

import numpy as np
import pytest

from fm_spark_amd.linalg import SparseVector
from problems import make_problem
from test_gpu_parity import to_host

pytestmark = pytest.mark.gpu


def _select(csr, rows):
    from oracle import fm_ref as R

    rows = np.asarray(rows, dtype=np.int64)
    lens = csr.row_ptr[rows + 1] - csr.row_ptr[rows]
    rp = np.zeros(len(rows) + 1, dtype=np.int64)
    np.cumsum(lens, out=rp[1:])
    idx = np.repeat(csr.row_ptr[rows] - rp[:-1], lens) + np.arange(rp[-1], dtype=np.int64)
    return R.CSR(rp, csr.col[idx], csr.val[idx], csr.label[rows])


def _run(fuse, F, k, ids, w, V, batches, prepare):
    """Steps over a list of ('host', csr) / ('rows', data_csr, rows) batches; returns losses + table."""
    from fm_spark_amd.engine import FMContext

    ctx = FMContext(F, k, fuse=fuse)
    ctx.load_tables(ids, w, V)
    data = {}
    into = None
    out = []
    for t, b in enumerate(batches, start=1):
        if b[0] == "host":
            db = ctx.batch(to_host(b[1]))
        else:
            key = id(b[1])
            if key not in data:
                data[key] = ctx.batch(to_host(b[1]))
            into = ctx.batch_from_rows(data[key], b[2], into=into)  # one batch refilled in turn
            db = into
        if prepare:
            db.prepare()
        o = ctx.step_batch(db, t, 0.3, 1e-3)
        out.append((o.loss_sum, o.n_rows, o.n_loss_rows, o.n_unique, o.executed))
    tab = ctx.export_tables()
    ctx.close()
    return out, tab


@pytest.mark.parametrize("fuse,prepare", [(False, False), (False, True), (True, True)])
def test_from_rows_bitwise_equal_host_batch(gpu, fuse, prepare):
    """Rows out of order, repeated rows, empty rows, a selection that grows the refilled batch, an
    empty selection (nothing to do): every step bitwise the one on the host CSR of the same rows."""
    F, k = 50_000, 16
    data, ids, w, V = make_problem(1201, 6000, F, k, 12, empty_frac=0.1, hot=7)
    rng = np.random.default_rng(3)
    sels = [rng.permutation(6000)[:1500], np.sort(rng.choice(6000, 4000, replace=True)), np.arange(0),
            rng.permutation(6000), np.arange(5990, 6000)]
    a = _run(fuse, F, k, ids, w, V, [("rows", data, s) for s in sels], prepare)
    b = _run(fuse, F, k, ids, w, V, [("host", _select(data, s)) for s in sels], prepare)
    assert a[0] == b[0]
    assert a[0][2][4] is False  # the empty selection: FM_NOTHING_TO_DO
    for x, y in zip(a[1], b[1]):
        assert np.array_equal(x, y)


def test_from_rows_predict_and_errors(gpu):
    from fm_spark_amd._native import FMError
    from fm_spark_amd.engine import FMContext

    F, k = 3000, 8
    data, ids, w, V = make_problem(1202, 800, F, k, 6)
    ctx = FMContext(F, k)
    ctx.load_tables(ids, w, V)
    d = ctx.batch(to_host(data))
    rows = np.arange(799, -1, -3)
    b = ctx.batch_from_rows(d, rows)
    p_rows = ctx.predict_batch(b, 0.0, 1.0)
    p_all = ctx.predict_batch(d, 0.0, 1.0)
    np.testing.assert_array_equal(p_rows, p_all[rows])
    with pytest.raises(FMError, match="row index"):
        ctx.batch_from_rows(d, [0, 800])
    with pytest.raises(FMError, match="other than data"):
        ctx.batch_from_rows(d, [1, 2], into=d)
    other = FMContext(F, k)
    with pytest.raises(FMError, match="another context"):
        other.batch_from_rows(d, [1, 2])
    other.close()
    ctx.close()


def _dataset(n_rows, F, seed, parts):
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.ml import DataFrame

    b = synthetic_batch(n_rows, F, batch_index=seed)
    vecs = [SparseVector(F, b.col[b.row_ptr[i]:b.row_ptr[i + 1]], b.val[b.row_ptr[i]:b.row_ptr[i + 1]])
            for i in range(b.n_rows)]
    sizes = [n_rows * (i + 1) // parts - n_rows * i // parts for i in range(parts)]
    return DataFrame({"label": [float(y) for y in b.label], "features": vecs}, sizes)


def test_pipelined_fit_matches_synchronous_fit(gpu, caplog):
    """The pipelined fit (resident dataset, device-gathered splits, side-stream sorts, enqueue-only
    steps) against the synchronous one (a host CSR per split, each step read back): the same model
    (rtol 1e-5; bitwise here, both unfused) and the same loss log lines (rel 1e-9), in order,
    including a zero-size split's warning (maxIter 30 over 20 rows leaves most
    splits empty)."""
    from fm_spark_amd.ml import FactorizationMachinesSGD

    def est(it, frac):
        return (FactorizationMachinesSGD().setDimFactorization(8).setMaxIter(it).setMiniBatchFraction(frac)
                .setStepSize(0.5).setRegParam(1e-4).setNumFeatures(20_000).setSeed(5))

    for n_rows, it, frac in ((4000, 6, 0.15), (20, 30, 0.05)):
        df = _dataset(n_rows, 20_000, 31 + n_rows, 4)
        logs = []
        tabs = []
        for pipe in (True, False):
            caplog.clear()
            with caplog.at_level(logging.INFO, logger="org.apache.spark.ml.fm"):
                m = est(it, frac).fit(df, pipelined=pipe)
            logs.append([(r.levelname, r.getMessage()) for r in caplog.records])
            tabs.append(m._ctx.export_tables())
        assert len(logs[0]) == it and len(logs[1]) == it
        for (l1, m1), (l2, m2) in zip(*logs):
            assert l1 == l2
            h1, v1 = m1.rsplit(" ", 1)
            h2, v2 = m2.rsplit(" ", 1)
            assert h1 == h2
            if l1 == "INFO":
                assert float(v1) == pytest.approx(float(v2), rel=1e-9)
        if n_rows == 20:
            assert any(lv == "WARNING" for lv, _ in logs[0]), "expected a zero-size split"
        np.testing.assert_array_equal(tabs[0][0], tabs[1][0])
        np.testing.assert_allclose(tabs[0][1], tabs[1][1], rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(tabs[0][2], tabs[1][2], rtol=1e-5, atol=1e-8)


def test_resident_loop_fused_matches_host_steps(gpu):
    """run_minibatch_sgd_resident on a fused context (fuse on, k = 16: singleton rows updated by the
    forward) against the synchronous host-CSR steps of the same splits on a fused context: the
    fused step of a prepared batch against the unprepared (unfused) step, so within the north_star
    tolerance."""
    from fm_spark_amd.engine import FMContext
    from fm_spark_amd.ml import _select_csr, run_minibatch_sgd_resident

    F, k = 60_000, 16
    data, ids, w, V = make_problem(1203, 9000, F, k, 14, hot=11)
    rng = np.random.default_rng(8)
    split_of = rng.integers(-1, 5, size=data.n_rows)
    splits = [np.flatnonzero(split_of == i) for i in range(5)]
    ctx = FMContext(F, k, fuse=True)
    ctx.load_tables(ids, w, V)
    assert ctx.fuse_active
    d = ctx.batch(to_host(data))
    losses = run_minibatch_sgd_resident(ctx, d, splits, 0.3, 1e-4)
    ref = FMContext(F, k, fuse=True)
    ref.load_tables(ids, w, V)
    rl = []
    for i, rows in enumerate(splits):
        rl.append(ref.step(_select_csr(data.row_ptr, data.col, data.val, data.label, rows), i + 1, 0.3, 1e-4).loss_sum)
    np.testing.assert_allclose(losses, rl, rtol=1e-9)
    a, b = ctx.export_tables(), ref.export_tables()
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_allclose(a[1], b[1], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(a[2], b[2], rtol=1e-5, atol=1e-8)
    ctx.close()
    ref.close()


@pytest.mark.parametrize("mode", ["sharded", "replicated"])
def test_from_rows_on_a_multi_gpu_context(gpu, mode):
    """fm_batch_from_rows on a 3-rank context (COPY transport on this GPU): each rank gathers its
    contiguous share of the selection from its own copy of the dataset; the steps are the steps of
    the host CSR of the same rows, bitwise (the same rows reach the same ranks in the same order)."""
    from fm_spark_amd.engine import FMContext

    F, k, R = 3000, 8, 3
    data, ids, w, V = make_problem(1205, 2500, F, k, 9, hot=4)
    rng = np.random.default_rng(12)
    sels = [rng.permutation(2500)[:900], np.sort(rng.choice(2500, 1300)), rng.permutation(2500)[:2]]

    def run(use_rows):
        ctx = FMContext(F, k, parallel=mode, n_gpus=R, devices=[0] * R, transport="copy")
        ctx.load_tables(ids, w, V)
        d = ctx.batch(to_host(data))
        into, out = None, []
        for t, s in enumerate(sels, start=1):
            if use_rows:
                into = ctx.batch_from_rows(d, s, into=into)
                b = into
            else:
                b = ctx.batch(to_host(_select(data, s)))
            b.prepare()
            o = ctx.step_batch(b, t, 0.3, 1e-3)
            out.append((o.loss_sum, o.n_rows, o.n_loss_rows, o.n_unique))
        tab = ctx.export_tables()
        ctx.close()
        return out, tab

    a, b = run(True), run(False)
    assert a[0] == b[0]
    for x, y in zip(a[1], b[1]):
        assert np.array_equal(x, y)


def _layout(data, sels):
    """The rows of the selections concatenated (the split-ordered dataset) and their split offsets."""
    lay = np.concatenate([np.asarray(x, dtype=np.int64) for x in sels]) if sels else np.zeros(0, np.int64)
    return _select(data, lay), np.concatenate([[0], np.cumsum([len(x) for x in sels])]).astype(np.int64)


@pytest.mark.parametrize("fuse,prepare", [(False, False), (False, True), (True, True)])
def test_split_views_bitwise_equal_host_batch(gpu, fuse, prepare):
    """A dataset laid out split by split, each split stepped in place through a view re-pointed in
    turn (ragged splits, an empty one, repeated rows, a last split never stepped): every step bitwise
    the one on the host CSR of the same rows, and the view's predictions those of the host rows."""
    from fm_spark_amd.engine import FMContext

    F, k = 50_000, 16
    data, ids, w, V = make_problem(1211, 6000, F, k, 12, empty_frac=0.1, hot=7)
    rng = np.random.default_rng(4)
    sels = [rng.permutation(6000)[:1500], np.sort(rng.choice(6000, 2000, replace=True)), np.arange(0),
            rng.permutation(6000)[:700], np.arange(5990, 6000), np.arange(3000)]
    steps = sels[:-1]
    lay, split_rows = _layout(data, sels)

    def run(views):
        ctx = FMContext(F, k, fuse=fuse)
        ctx.load_tables(ids, w, V)
        d = ctx.batch_splits(to_host(lay), split_rows) if views else None
        out, preds, into = [], [], None
        for t, sel in enumerate(steps, start=1):
            if views:
                into = ctx.split_view(d, t - 1, into=into)
                b = into
            else:
                b = ctx.batch(to_host(_select(data, sel)))
            assert b.n_rows == len(sel)
            preds.append(ctx.predict_batch(b, 0.0, 1.0) if len(sel) else None)
            if prepare:
                b.prepare()
            o = ctx.step_batch(b, t, 0.3, 1e-3)
            out.append((o.loss_sum, o.n_rows, o.n_loss_rows, o.n_unique, o.executed))
        tab = ctx.export_tables()
        ctx.close()
        return out, preds, tab

    a, b = run(True), run(False)
    assert a[0] == b[0]
    assert a[0][2][4] is False  # the empty split: FM_NOTHING_TO_DO
    for x, y in zip(a[1], b[1]):
        assert (x is None and y is None) or np.array_equal(x, y)
    for x, y in zip(a[2], b[2]):
        assert np.array_equal(x, y)


def test_split_dataset_rules(gpu):
    """The dataset itself is not stepped or prepared; a view's split index is checked; a view refilled
    by fm_batch_from_rows (and a gathered batch turned into a view) steps as the host rows do;
    createInitialModel over the split dataset draws exactly the rows a plain dataset draws."""
    from fm_spark_amd._native import FMError
    from fm_spark_amd.engine import FMContext

    F, k = 3000, 8
    data, ids, w, V = make_problem(1212, 900, F, k, 6)
    sels = [np.arange(0, 300), np.arange(300, 900)[::-1]]
    lay, split_rows = _layout(data, sels)
    ctx = FMContext(F, k, seed=9)
    d = ctx.batch_splits(to_host(lay), split_rows)
    with pytest.raises(FMError, match="split views"):
        ctx.step_batch(d, 1, 0.3, 1e-3)
    with pytest.raises(FMError, match="split views"):
        d.prepare()
    with pytest.raises(FMError, match="split index"):
        ctx.split_view(d, 2)
    plain = ctx.batch(to_host(data))
    with pytest.raises(FMError, match="fm_batch_create_splits"):
        ctx.split_view(plain, 0)
    # createInitialModel over either layout: the same rows, the same draws
    n1 = ctx.init_from_batch(d)
    ref = FMContext(F, k, seed=9)
    n2 = ref.init_from_batch(ref.batch(to_host(data)))
    assert n1 == n2
    for x, y in zip(ctx.export_tables(), ref.export_tables()):
        assert np.array_equal(x, y)
    # view -> gathered batch -> view, stepped against the host rows
    b = ctx.split_view(d, 1)
    o1 = ctx.step_batch(b, 1, 0.3, 1e-3)
    b = ctx.batch_from_rows(plain, sels[0], into=b)
    o2 = ctx.step_batch(b, 2, 0.3, 1e-3)
    b = ctx.split_view(d, 0, into=b)
    o3 = ctx.step_batch(b, 3, 0.3, 1e-3)
    r1 = ref.step(to_host(_select(data, sels[1])), 1, 0.3, 1e-3)
    r2 = ref.step(to_host(_select(data, sels[0])), 2, 0.3, 1e-3)
    r3 = ref.step(to_host(_select(data, sels[0])), 3, 0.3, 1e-3)
    assert [(o.loss_sum, o.n_unique) for o in (o1, o2, o3)] == [(o.loss_sum, o.n_unique) for o in (r1, r2, r3)]
    for x, y in zip(ctx.export_tables(), ref.export_tables()):
        assert np.array_equal(x, y)
    ctx.close()
    ref.close()


@pytest.mark.parametrize("mode", ["sharded", "replicated"])
def test_from_rows_of_a_split_dataset_on_a_multi_gpu_context(gpu, mode):
    """fm_batch_from_rows over a split dataset on a 3-rank context (COPY): rank l holds its share of
    every split, so its copy of the dataset is assembled split by split, rank by rank -- row i of the
    copy is row i of the CSR the dataset was made from.  Row lists over that CSR step bitwise as the
    host CSR of the same rows; a split dataset is refused as the batch to refill."""
    from fm_spark_amd._native import FMError
    from fm_spark_amd.engine import FMContext

    F, k, R = 3000, 8, 3
    data, ids, w, V = make_problem(1216, 2000, F, k, 9, hot=4)
    rng = np.random.default_rng(14)
    lay, split_rows = _layout(data, [rng.permutation(2000)[:700], np.arange(0), rng.permutation(2000)[:1100],
                                     np.arange(1990, 2000)])
    n_lay = len(lay.row_ptr) - 1
    sels = [rng.permutation(n_lay)[:800], np.sort(rng.choice(n_lay, 1000)), np.arange(n_lay)[::-1]]

    def run(use_rows):
        ctx = FMContext(F, k, parallel=mode, n_gpus=R, devices=[0] * R, transport="copy")
        ctx.load_tables(ids, w, V)
        d = ctx.batch_splits(to_host(lay), split_rows)
        if use_rows:
            with pytest.raises(FMError, match="other than data"):
                ctx.batch_from_rows(d, [0, 1], into=ctx.batch_splits(to_host(lay), split_rows))
        into, out = None, []
        for t, s in enumerate(sels, start=1):
            if use_rows:
                into = ctx.batch_from_rows(d, s, into=into)
                b = into
            else:
                b = ctx.batch(to_host(_select(lay, s)))
            b.prepare()
            o = ctx.step_batch(b, t, 0.3, 1e-3)
            out.append((o.loss_sum, o.n_rows, o.n_loss_rows, o.n_unique))
        tab = ctx.export_tables()
        ctx.close()
        return out, tab

    a, b = run(True), run(False)
    assert a[0] == b[0]
    for x, y in zip(a[1], b[1]):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("mode", ["sharded", "replicated"])
def test_split_views_on_a_multi_gpu_context(gpu, mode):
    """fm_batch_create_splits on a 3-rank context (COPY transport on this GPU): every rank holds its
    contiguous share of every split; each split view steps bitwise as the host CSR of the same rows;
    createInitialModel over the split dataset (split by split through the owners, sharded) draws the
    plain dataset's rows."""
    from fm_spark_amd.engine import FMContext

    F, k, R = 3000, 8, 3
    data, ids, w, V = make_problem(1215, 2500, F, k, 9, hot=4)
    rng = np.random.default_rng(13)
    sels = [rng.permutation(2500)[:900], np.sort(rng.choice(2500, 1300)), rng.permutation(2500)[:2], np.arange(0)]
    lay, split_rows = _layout(data, sels)

    def run(views):
        ctx = FMContext(F, k, parallel=mode, n_gpus=R, devices=[0] * R, transport="copy", seed=3)
        d = ctx.batch_splits(to_host(lay), split_rows) if views else ctx.batch(to_host(lay))
        ctx.init_from_batch(d)
        into, out = None, []
        for t, s in enumerate(sels[:3], start=1):
            if views:
                into = ctx.split_view(d, t - 1, into=into)
                b = into
            else:
                b = ctx.batch(to_host(_select(data, s)))
            b.prepare()
            o = ctx.step_batch(b, t, 0.3, 1e-3)
            out.append((o.loss_sum, o.n_rows, o.n_loss_rows, o.n_unique))
        tab = ctx.export_tables()
        ctx.close()
        return out, tab

    a, b = run(True), run(False)
    assert a[0] == b[0]
    for x, y in zip(a[1], b[1]):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("mode", ["sharded", "replicated"])
def test_pipelined_resident_loop_on_a_multi_gpu_context(gpu, mode):
    """run_minibatch_sgd_resident (enqueue-only steps; each batch refilled by fm_batch_from_rows two
    iterations ahead while earlier steps may still be queued) on a 3-rank context (COPY transport):
    the losses and the table bitwise those of synchronous steps on the host CSRs of the same rows.
    A refill must wait for the sharded iteration that last read the batch (its combine reads the
    labels, its route the entries)."""
    from fm_spark_amd.engine import FMContext
    from fm_spark_amd.ml import run_minibatch_sgd_resident

    F, k, R = 3000, 8, 3
    data, ids, w, V = make_problem(1216, 2400, F, k, 9, hot=4)
    rng = np.random.default_rng(14)
    splits = [rng.permutation(2400)[: 300 + 40 * i] for i in range(7)]

    def ctx_():
        c = FMContext(F, k, parallel=mode, n_gpus=R, devices=[0] * R, transport="copy")
        c.load_tables(ids, w, V)
        return c

    a = ctx_()
    d = a.batch(to_host(data))
    la = run_minibatch_sgd_resident(a, d, splits, 0.3, 1e-3)
    ta = a.export_tables()
    b = ctx_()
    lb = [b.step(to_host(_select(data, s)), i + 1, 0.3, 1e-3).loss_sum for i, s in enumerate(splits)]
    tb = b.export_tables()
    assert la == lb
    for x, y in zip(ta, tb):
        assert np.array_equal(x, y)
    a.close()
    b.close()
