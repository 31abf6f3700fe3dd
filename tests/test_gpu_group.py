"""GPU: multi-GPU inside one fm_ctx (fm_config.parallel; csrc/fm_group.hip), driven through the
C entry points alone -- no Python exchange code.

The COPY transport lets R ranks share this box's one MI355X (RCCL refuses two ranks on one
device), so the sharded and replicated jobs run at R = 1..8 in one process; the RCCL transport
runs at R = 1 (the same grouped send/recv, all-gather and all-reduce calls, one rank).  Every
job is compared with the fp64 oracle step over the concatenated mini-batch (the reference's one
global mini-batch: SGD.scala:116-211), and the sharded transform with oracle.predict
(Model.scala:69-133: ids outside or absent from the model dropped, w0 for rows left without a
learned feature, clamp)."""

import math

import numpy as np
import pytest

from oracle import fm_ref as R_
from problems import make_problem

pytestmark = pytest.mark.gpu


def _host(c):
    from fm_spark_amd._native import CSRHost

    return CSRHost(c.row_ptr, c.col, c.val, c.label)


def _ctx(F, k, R, mode="sharded", transport="copy", **kw):
    from fm_spark_amd.engine import FMContext

    devs = [0] * R if transport == "copy" else list(range(R))
    return FMContext(F, k, parallel=mode, n_gpus=R, devices=devs, transport=transport, **kw)


def _check_tables(ctx, model):
    gi, gw, gV = ctx.export_tables()
    np.testing.assert_array_equal(gi, np.nonzero(model.present)[0])
    np.testing.assert_allclose(gw, model.w[gi], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(gV, model.V[gi], rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("R,k,F,hot,transport", [
    (1, 8, 503, 11, "copy"), (2, 16, 503, 11, "copy"), (3, 5, 401, 7, "copy"), (4, 32, 513, 512, "copy"),
    (8, 16, 1031, 1030, "copy"), (12, 8, 1031, 1030, "copy"), (1, 16, 300, 2, "rccl"),
])
def test_group_sharded_step_matches_oracle(gpu, R, k, F, hot, transport):
    _, ids, w, V = make_problem(3, 1, F, k, 1)
    ctx = _ctx(F, k, R, transport=transport)
    ctx.load_tables(ids, w, V)
    model = R_.Model.empty(F, k)
    model.load(ids, w, V)
    # steps 1-2 from host CSRs (fm_step), 3-4 from device batches with the next one prepared
    probs = [make_problem(40 + t, 150 + 13 * t, F, k, 9, hot=hot)[0] for t in range(1, 5)]
    for t in (1, 2):
        o = ctx.step(_host(probs[t - 1]), t, 0.3, 1e-4)
        ref = R_.sgd_step_fast(model, probs[t - 1], t, 0.3, 1e-4)
        assert o.loss_sum == pytest.approx(ref.loss_sum, rel=1e-5)
        assert (o.n_rows, o.n_loss_rows, o.n_unique) == (ref.n_rows, ref.n_loss_rows, ref.n_unique)
    bs = [ctx.batch(_host(p)) for p in probs[2:]]
    bs[0].prepare()
    for t in (3, 4):
        o = ctx.step_batch(bs[t - 3], t, 0.3, 1e-4, sync=True)
        if t == 3:
            bs[1].prepare()  # routed, exchanged and slot-sorted behind step 3
        ref = R_.sgd_step_fast(model, probs[t - 1], t, 0.3, 1e-4)
        assert o.loss_sum == pytest.approx(ref.loss_sum, rel=1e-5)
        assert o.n_unique == ref.n_unique
    assert ctx.epoch == 4
    hist = ctx.loss_history()
    assert len(hist) == 4 and hist[-1] == pytest.approx(o.loss_sum, rel=1e-12)
    _check_tables(ctx, model)
    # rows by id through the owners
    q = np.array([0, hot, F - 1, F // 2], dtype=np.int32)
    rw, rV, rp = ctx.export_rows(q)
    assert rp.all()
    np.testing.assert_allclose(rw, model.w[q], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(rV, model.V[q], rtol=1e-5, atol=1e-8)
    ctx.close()


@pytest.mark.parametrize("R,k,transport", [(1, 16, "copy"), (2, 8, "copy"), (3, 16, "copy"), (8, 16, "copy"),
                                           (1, 16, "rccl")])
def test_group_sharded_step_ignores_fuse(gpu, R, k, transport):
    """A sharded group never fuses (fm_fuse_active 0 whatever fm_config.fuse_single says: the fused
    owner step measured slower at R = 8 and at world 1 and was removed): with fuse on
    and off the steps are bitwise the same and match the fp64 oracle, from host CSRs and from prepared
    device batches, with a hot feature and rows absent from the model."""
    F = 4001
    _, ids, w, V = make_problem(33, 1, F, k, 1)
    keep = ids[ids % 5 != 0]  # a fifth of the rows absent: singletons and multi runs create them
    probs = [make_problem(140 + t, 400 + 37 * t, F, k, 9, hot=17)[0] for t in range(1, 5)]
    model = R_.Model.empty(F, k)
    model.load(keep, w[keep], V[keep])
    out = {}
    for fuse in (True, False):
        ctx = _ctx(F, k, R, transport=transport, fuse=fuse)
        assert not ctx.fuse_active
        ctx.load_tables(keep, w[keep], V[keep])
        res = []
        for t in (1, 2):
            res.append(ctx.step(_host(probs[t - 1]), t, 0.3, 1e-3))
        bs = [ctx.batch(_host(p)) for p in probs[2:]]
        bs[0].prepare()
        for t in (3, 4):
            res.append(ctx.step_batch(bs[t - 3], t, 0.3, 1e-3, sync=True))
            if t == 3:
                bs[1].prepare()
        out[fuse] = ([(o.loss_sum, o.n_rows, o.n_loss_rows, o.n_unique) for o in res], ctx.export_tables())
        for b in bs:
            b.close()
        ctx.close()
    for t in range(1, 5):
        ref = R_.sgd_step_fast(model, probs[t - 1], t, 0.3, 1e-3)
        got = out[True][0][t - 1]
        assert got[0] == pytest.approx(ref.loss_sum, rel=1e-5)
        assert got[1:] == (ref.n_rows, ref.n_loss_rows, ref.n_unique)
    assert out[True][0] == out[False][0]
    for a, b in zip(out[True][1], out[False][1]):
        assert np.array_equal(a, b)
    gi, gw, gV = out[True][1]
    np.testing.assert_array_equal(gi, np.nonzero(model.present)[0])
    np.testing.assert_allclose(gw, model.w[gi], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(gV, model.V[gi], rtol=1e-5, atol=1e-8)
    np.testing.assert_array_equal(gi, out[False][1][0])
    np.testing.assert_allclose(gw, out[False][1][1], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(gV, out[False][1][2], rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("R,transport", [(3, "copy"), (1, "rccl")])
def test_group_sharded_prepare_two_ahead(gpu, R, transport):
    """fm_batch_prepare on a sharded group is two-phase: it enqueues the batch's route and count
    gather, and completes the batch prepared before it.  Batches prepared two steps ahead, a batch
    prepared twice, a pending batch predicted (its plan completed, then re-routed for the transform)
    and a pending batch destroyed before its step all leave the oracle steps."""
    F, k = 600, 8
    _, ids, w, V = make_problem(5, 1, F, k, 1)
    ctx = _ctx(F, k, R, transport=transport)
    ctx.load_tables(ids, w, V)
    model = R_.Model.empty(F, k)
    model.load(ids, w, V)
    probs = [make_problem(90 + i, 120 + 17 * i, F, k, 8, hot=13)[0] for i in range(3)]
    bs = [ctx.batch(_host(p)) for p in probs]
    gone = ctx.batch(_host(probs[0]))
    gone.prepare()
    gone.close()  # pending when destroyed
    bs[0].prepare()
    bs[1].prepare()  # completes bs[0]'s plan, routes bs[1]
    bs[1].prepare()  # already routed: nothing new
    refs = []
    for i in range(6):
        t = i + 1
        ctx.step_batch(bs[i % 3], t, 0.3, 1e-4, sync=False)
        refs.append(R_.sgd_step_fast(model, probs[i % 3], t, 0.3, 1e-4).loss_sum)
        if i == 3:  # bs[1] is pending here (routed after step 3): a transform completes and redoes it
            got = ctx.predict_batch(bs[1], 0.0, 1.0)
            np.testing.assert_allclose(got, R_.predict(model, probs[1], 0.0, 1.0, num_features=F), rtol=1e-5, atol=1e-7)
        if i + 2 < 6:
            bs[(i + 2) % 3].prepare()
    ctx.sync()
    np.testing.assert_allclose(ctx.loss_history(), refs, rtol=1e-5)
    _check_tables(ctx, model)
    ctx.close()


@pytest.mark.parametrize("chunks", [1, 3, 16])
def test_group_sharded_exchange_chunks(gpu, chunks):
    """The owners' partial pass in C chunks whose exchange overlaps the next chunk's compute
    (fm_config.xchg_chunks; default 4): any C gives the oracle step, including chunks with no pairs."""
    F, k, R = 257, 8, 4
    _, ids, w, V = make_problem(21, 1, F, k, 1)
    ctx = _ctx(F, k, R, xchg_chunks=chunks)
    ctx.load_tables(ids, w, V)
    model = R_.Model.empty(F, k)
    model.load(ids, w, V)
    for t, rows in ((1, 90), (2, 7), (3, 140)):  # 7 rows: most (owner, requester) blocks hold < 16 pairs
        p = make_problem(60 + t, rows, F, k, 6, hot=3)[0]
        o = ctx.step(_host(p), t, 0.3, 1e-4)
        ref = R_.sgd_step_fast(model, p, t, 0.3, 1e-4)
        assert o.loss_sum == pytest.approx(ref.loss_sum, rel=1e-5)
        assert o.n_unique == ref.n_unique
    _check_tables(ctx, model)
    ctx.close()


@pytest.mark.parametrize("R,k,transport", [(1, 8, "copy"), (3, 16, "copy"), (1, 16, "rccl")])
def test_group_replicated_step_matches_oracle(gpu, R, k, transport):
    F = 401
    _, ids, w, V = make_problem(12, 1, F, k, 1)
    ctx = _ctx(F, k, R, mode="replicated", transport=transport)
    ctx.load_tables(ids, w, V)
    model = R_.Model.empty(F, k)
    model.load(ids, w, V)
    for t in range(1, 4):
        p = make_problem(300 * t, 200 + 11 * t, F, k, 7, hot=5)[0]
        o = ctx.step(_host(p), t, 0.3, 1e-4)
        ref = R_.sgd_step_fast(model, p, t, 0.3, 1e-4)
        assert o.loss_sum == pytest.approx(ref.loss_sum, rel=1e-5)
        assert (o.n_rows, o.n_loss_rows, o.n_unique) == (ref.n_rows, ref.n_loss_rows, ref.n_unique)
    _check_tables(ctx, model)
    ctx.close()


def test_group_empty_batch_and_empty_rows(gpu):
    """An empty global mini-batch is skipped by every rank (SGD.scala:126-128); rows without
    entries count in miniBatchSize only; a part may hold no row at all."""
    F, k, R = 97, 4, 3
    _, ids, w, V = make_problem(8, 1, F, k, 1)
    ctx = _ctx(F, k, R)
    ctx.load_tables(ids, w, V)
    model = R_.Model.empty(F, k)
    model.load(ids, w, V)
    empty = R_.CSR(np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0), np.zeros(0))
    o = ctx.step(_host(empty), 1, 0.3, 1e-4)
    assert not o.executed and ctx.epoch == 0
    two = make_problem(9, 2, F, k, 5, empty_frac=0.0)[0]  # 2 rows over 3 ranks: one part is empty
    o = ctx.step(_host(two), 1, 0.3, 1e-4)
    ref = R_.sgd_step_fast(model, two, 1, 0.3, 1e-4)
    assert o.loss_sum == pytest.approx(ref.loss_sum, rel=1e-5)
    p = make_problem(10, 60, F, k, 5, hot=3, empty_frac=0.3)[0]
    o = ctx.step(_host(p), 2, 0.3, 1e-4)
    ref = R_.sgd_step_fast(model, p, 2, 0.3, 1e-4)
    assert o.loss_sum == pytest.approx(ref.loss_sum, rel=1e-5) and o.n_rows == p.n_rows
    _check_tables(ctx, model)
    ctx.close()


@pytest.mark.parametrize("R,transport", [(1, "copy"), (2, "copy"), (3, "copy"), (4, "copy"), (1, "rccl")])
def test_group_sharded_predict_matches_oracle(gpu, R, transport):
    """transform on a sharded table: ids >= F and ids absent from the model drop out, rows left
    without a learned feature score w0 unclamped, the rest are clamped."""
    F, k, w0 = 211, 8, 0.25
    _, _, w, V = make_problem(5, 1, F, k, 1)
    present = np.sort(np.random.default_rng(1).choice(F, size=150, replace=False)).astype(np.int32)
    ctx = _ctx(F, k, R, transport=transport, w0=w0)
    ctx.load_tables(present, w[present], V[present])
    model = R_.Model.empty(F, k, w0=w0)
    model.load(present, w[present], V[present])
    p = make_problem(6, 300, F + 40, k, 6, empty_frac=0.15)[0]  # ids up to F + 39: some outside
    lone = np.nonzero(~np.isin(np.arange(F), present))[0][:3]  # a row holding only absent ids
    rp = np.concatenate([p.row_ptr, [p.row_ptr[-1] + len(lone)]]).astype(np.int64)
    csr = R_.CSR(rp, np.concatenate([p.col, lone]).astype(np.int32), np.concatenate([p.val, np.ones(len(lone))]),
                 np.concatenate([p.label, [0.0]]))
    for lo, hi in ((0.0, 1.0), (-math.inf, math.inf)):
        got = ctx.predict(_host(csr), lo, hi)
        ref = R_.predict(model, csr, lo, hi, num_features=F)
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-7)
    assert got[-1] == w0
    ctx.close()


def test_group_c3_r8_matches_single_table(gpu):
    """Config c3's table (100M hashed features, k = 16) sharded over R = 8 ranks of one context
    (COPY transport, every rank on this GPU): two iterations of 8 x 32K rows against the
    single-table HIP step over the same global mini-batch; then transform of a third batch on both."""
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.engine import FMContext

    F, k, R, B = 100_000_000, 16, 8, 8 * 32768
    ref = FMContext(F, k, seed=5, init_sd=0.01)
    grp = _ctx(F, k, R, seed=5, init_sd=0.01)
    for t in (1, 2):
        b = synthetic_batch(B, F, batch_index=500 + t)
        rb = ref.batch(_host(b))
        gb = grp.batch(_host(b))
        n1 = ref.init_from_batch(rb)
        n2 = grp.init_from_batch(gb)  # createInitialModel through the owners: the same seeded draw
        assert n1 == n2
        o = ref.step_batch(rb, t, 0.1, 1e-6, sync=True)
        q = grp.step_batch(gb, t, 0.1, 1e-6, sync=True)
        assert q.n_unique == o.n_unique == len(np.unique(b.col))
        assert q.loss_sum == pytest.approx(o.loss_sum, rel=1e-9)
    gi, gw, gV = ref.export_tables()
    si, sw, sV = grp.export_tables()
    np.testing.assert_array_equal(si, gi)
    np.testing.assert_allclose(sw, gw, rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(sV, gV, rtol=1e-5, atol=1e-8)
    b3 = synthetic_batch(65536, F, batch_index=777)
    pr = ref.predict(_host(b3), 0.0, 1.0)
    pg = grp.predict(_host(b3), 0.0, 1.0)
    np.testing.assert_allclose(pg, pr, rtol=1e-5, atol=1e-7)
    ref.close()
    grp.close()


@pytest.mark.parametrize("mode", ["sharded", "replicated"])
def test_rccl_two_devices_matches_copy(gpu, mode):
    """The first lease with two GPUs checks RCCL with R > 1 -- grouped ncclSend / ncclRecv on
    three communicators, the device-side all-gather of the route counts, the chunked partial
    exchange, the in-place stats all-reduce -- against the COPY transport and the oracle on the
    same job.  Skipped on a one-GPU box (every box of rounds 1-3 had one MI355X)."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs: RCCL refuses two ranks on one device")
    F, k = 513, 8
    _, ids, w, V = make_problem(31, 1, F, k, 1)
    model = R_.Model.empty(F, k)
    model.load(ids, w, V)
    from fm_spark_amd.engine import FMContext

    ctxs = {"rccl": FMContext(F, k, parallel=mode, n_gpus=2, devices=[0, 1], transport="rccl"),
            "copy": FMContext(F, k, parallel=mode, n_gpus=2, devices=[0, 0], transport="copy")}
    for c in ctxs.values():
        c.load_tables(ids, w, V)
    for t in range(1, 4):
        p = make_problem(500 + t, 300, F, k, 9, hot=4)[0]
        outs = {tr: c.step(_host(p), t, 0.3, 1e-4) for tr, c in ctxs.items()}
        ref = R_.sgd_step_fast(model, p, t, 0.3, 1e-4)
        for o in outs.values():
            assert o.loss_sum == pytest.approx(ref.loss_sum, rel=1e-5)
            assert (o.n_loss_rows, o.n_unique) == (ref.n_loss_rows, ref.n_unique)
        assert outs["rccl"].loss_sum == pytest.approx(outs["copy"].loss_sum, rel=1e-12)
    tabs = {tr: c.export_tables() for tr, c in ctxs.items()}
    for a, b in zip(tabs["rccl"], tabs["copy"]):
        assert np.array_equal(a, b)  # the same ranks, the same fixed orders: bitwise
    _check_tables(ctxs["rccl"], model)
    for c in ctxs.values():
        c.close()


def test_group_loss_grad_refused_when_sharded_answered_when_replicated(gpu):
    """calcLossGrad's per-entry rows need the whole table: a sharded group refuses it (FM_ERR_ARG,
    include/fm_hip.h fm_create), a replicated group answers it as a single-table context does."""
    from fm_spark_amd._native import FMError
    from fm_spark_amd.engine import FMContext

    F, k = 300, 4
    _, ids, w, V = make_problem(14, 1, F, k, 1)
    p = make_problem(15, 40, F, k, 6)[0]
    sh = _ctx(F, k, 2)
    sh.load_tables(ids, w, V)
    with pytest.raises(FMError, match="whole table"):
        sh.loss_grad(_host(p))
    sh.close()
    rep = _ctx(F, k, 2, mode="replicated")
    one = FMContext(F, k)
    for c in (rep, one):
        c.load_tables(ids, w, V)
    got, ref = rep.loss_grad(_host(p)), one.loss_grad(_host(p))
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
    rep.close()
    one.close()
