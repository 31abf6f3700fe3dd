"""GPU parity over seeded random problems: the step against the fp64 oracle on configurations
drawn at random -- k from 1 to 40, 5 to 60000 features, 0 to 3000 rows of 1 to 50 entries (empty
rows and explicit zeros included), with or without a hot feature, binary or regression labels,
step sizes and L1 strengths across their ranges -- through each way the library runs a step (and
then transform / predict on the trained model): the
host CSR (fm_step), a prepared device batch with the fused step on and off, and the three-rank
sharded and replicated contexts (COPY transport on this GPU).  Tolerance: north_star's 1e-5
relative, the counts exact; the absolute floor for values the L1 drives to (near) zero is 1e-8 on
one table, and on the three-rank paths 4 fp32 ulps of the table's largest value: their wire
carries each owner's partial sums (sharded) or each rank's gradient sums (replicated) in fp32
(DESIGN.md §6), so a value left near zero by the L1 keeps a few ulps of the value it was shrunk
from (case 39, sharded: 2.1e-8 at a value of 3.9e-5, the table's largest 0.68).  The cases are
fixed by their seeds, so a failure reproduces."""

import numpy as np
import pytest

from oracle import fm_ref as R
from problems import make_problem
from test_gpu_parity import ATOL, RTOL, to_host

pytestmark = pytest.mark.gpu

N_CASES = 40
PATHS = ["host", "fused", "unfused", "sharded3", "replicated3"]


def draw(seed):
    rng = np.random.default_rng(seed)
    k = int(rng.integers(1, 41))
    F = int(np.exp(rng.uniform(np.log(5), np.log(60000))))
    rows = int(rng.integers(0, 3001))
    nnz = int(rng.integers(1, 51))
    hot = int(rng.integers(0, F)) if rng.random() < 0.5 else None
    labels = "binary" if rng.random() < 0.5 else "regression"
    step = float(rng.uniform(0.05, 1.0))
    reg = float(rng.choice([0.0, 1e-6, 1e-4, 1e-3]))
    batches = [make_problem(seed * 10 + i, rows, F, k, nnz, hot=hot, labels=labels,
                            empty_frac=float(rng.uniform(0, 0.3)))[0] for i in range(3)]
    _, ids, w, V = make_problem(seed * 10 + 9, 1, F, k, 1)
    return dict(k=k, F=F, rows=rows, nnz=nnz, hot=hot, labels=labels, step=step, reg=reg), batches, ids, w, V


def score_terms(model, csr):
    """Per row, the magnitude of the terms a score sums: |w x| over the entries, and per factor the
    square of the |v x| sum and the v^2 x^2 sum (Model.scala:173-221)."""
    n = csr.n_rows
    row = np.repeat(np.arange(n), np.diff(csr.row_ptr))
    ok = csr.col < len(model.w)
    row, col, x = row[ok], csr.col[ok], csr.val[ok]
    aw = np.zeros(n)
    np.add.at(aw, row, np.abs(model.w[col] * x))
    vx = np.abs(model.V[col] * x[:, None])
    s1 = np.zeros((n, model.k))
    np.add.at(s1, row, vx)
    s2 = np.zeros(n)
    np.add.at(s2, row, (vx * vx).sum(axis=1))
    return aw + 0.5 * ((s1 * s1).sum(axis=1) + s2)


def run_path(path, cfg, batches, ids, w, V):
    from fm_spark_amd.engine import FMContext

    F, k = cfg["F"], cfg["k"]
    if path in ("sharded3", "replicated3"):
        ctx = FMContext(F, k, parallel=path[:-1], n_gpus=3, devices=[0] * 3, transport="copy")
    else:
        ctx = FMContext(F, k, fuse={"fused": True, "unfused": False}.get(path))
    ctx.load_tables(ids, w, V)
    outs = []
    dbs = [ctx.batch(to_host(c)) for c in batches] if path != "host" else None
    for t, c in enumerate(batches, start=1):
        if path == "host":
            o = ctx.step(to_host(c), t, cfg["step"], cfg["reg"])
        else:
            dbs[t - 1].prepare()
            o = ctx.step_batch(dbs[t - 1], t, cfg["step"], cfg["reg"])
        outs.append(o)
    tabs = ctx.export_tables()
    pred = ctx.predict(to_host(batches[0]), -2.0, 3.0)  # transform of the first batch with the trained model
    ctx.close()
    return outs, tabs, pred


@pytest.mark.parametrize("case", range(N_CASES))
def test_random_problems_every_path(gpu, case):
    cfg, batches, ids, w, V = draw(2027 + case)
    model = R.Model.empty(cfg["F"], cfg["k"])
    model.load(ids, w, V)
    ref = [R.sgd_step_fast(model, c, t, cfg["step"], cfg["reg"]) for t, c in enumerate(batches, start=1)]
    pids = np.nonzero(model.present)[0]
    ulp4 = 4 * 2.0 ** -24 * max(float(np.max(np.abs(model.V[pids]), initial=0.0)),
                                float(np.max(np.abs(model.w[pids]), initial=0.0)))
    for path in PATHS:
        atol = ATOL if path in ("host", "fused", "unfused") else max(ATOL, ulp4)
        outs, (gids, gw, gV), pred = run_path(path, cfg, batches, ids, w, V)
        for o, r in zip(outs, ref):
            assert o.executed == r.executed, (path, cfg)
            if r.executed:
                assert (o.n_rows, o.n_loss_rows, o.n_unique) == (r.n_rows, r.n_loss_rows, r.n_unique), (path, cfg)
                assert o.loss_sum == pytest.approx(r.loss_sum, rel=RTOL, abs=1e-9), (path, cfg)
        np.testing.assert_array_equal(gids, pids, err_msg=f"{path} {cfg}")
        np.testing.assert_allclose(gw, model.w[pids], rtol=RTOL, atol=atol, err_msg=f"{path} {cfg}")
        np.testing.assert_allclose(gV, model.V[pids], rtol=RTOL, atol=atol, err_msg=f"{path} {cfg}")
        # the transform's arithmetic against the oracle's on the tables this path trained (the tables
        # themselves are checked above; a score near zero is a cancellation of terms that carry the
        # tables' fp32 rounding, so the trained oracle model is not the reference for it)
        trained = R.Model.empty(cfg["F"], cfg["k"])
        trained.load(gids, gw, gV)
        ref_pred = R.predict(trained, batches[0], -2.0, 3.0, num_features=cfg["F"])
        if path in ("host", "fused", "unfused"):
            np.testing.assert_allclose(pred, ref_pred, rtol=RTOL, atol=1e-7, err_msg=f"predict {path} {cfg}")
        else:
            # the three-rank transform sums each owner's fp32 partial sums: a score that cancels keeps
            # a few fp32 ulps of the terms it cancels (8 ulps of their magnitude per row)
            bound = RTOL * np.abs(ref_pred) + np.maximum(1e-7, 8 * 2.0 ** -24 * score_terms(trained, batches[0]))
            assert np.all(np.abs(pred - ref_pred) <= bound), (path, cfg, float(np.max(np.abs(pred - ref_pred) - bound)))


@pytest.mark.parametrize("case", range(10))
def test_random_create_initial_model_every_path(gpu, case):
    """createInitialModel over a random batch (SGD.scala:218-252): the rows present afterwards are
    the batch's distinct ids, and the seeded draw is the same table on one GPU and on the
    three-rank sharded and replicated contexts, bit for bit."""
    from fm_spark_amd.engine import FMContext

    cfg, batches, _, _, _ = draw(4051 + case)
    F, k = cfg["F"], cfg["k"]
    csr = batches[0]
    tabs = []
    for path in ("single", "sharded3", "replicated3"):
        if path == "single":
            ctx = FMContext(F, k, seed=77)
        else:
            ctx = FMContext(F, k, seed=77, parallel=path[:-1], n_gpus=3, devices=[0] * 3, transport="copy")
        n = ctx.init_from_batch(ctx.batch(to_host(csr)))
        tabs.append((n, ctx.export_tables()))
        ctx.close()
    distinct = np.unique(csr.col)
    for n, (gids, gw, gV) in tabs:
        assert n == len(distinct), cfg
        np.testing.assert_array_equal(gids, distinct)
    for n, t in tabs[1:]:
        for x, y in zip(t, tabs[0][1]):
            assert np.array_equal(x, y), cfg


@pytest.mark.parametrize("case", range(8))
def test_random_resident_splits_every_path(gpu, case):
    """fit()'s resident dataset on random data: laid out split by split (ragged, empty and
    repeated-row splits), every split stepped through its in-place view and, on the same context, a
    random row list gathered from the dataset by fm_batch_from_rows -- bitwise the steps on the host
    CSRs of the same rows, on one GPU (fused and unfused) and on three sharded or replicated ranks."""
    from fm_spark_amd.engine import FMContext
    from test_gpu_resident_fit import _layout, _select

    cfg, batches, ids, w, V = draw(6073 + case)
    F, k = cfg["F"], cfg["k"]
    data = batches[0]
    n = data.n_rows
    rng = np.random.default_rng(case)
    sels = [rng.permutation(n)[: int(rng.integers(0, n + 1))] for _ in range(int(rng.integers(1, 5)))]
    sels.append(np.sort(rng.choice(n, int(rng.integers(0, n + 1)), replace=True)) if n else np.arange(0))
    lay, split_rows = _layout(data, sels)
    picks = np.sort(rng.choice(max(n, 1), int(rng.integers(0, n + 1)), replace=True)) if n else np.arange(0)

    def run(path, views):
        kw = dict(fuse={"fused": True, "unfused": False}[path]) if path in ("fused", "unfused") else dict(
            parallel=path[:-1], n_gpus=3, devices=[0] * 3, transport="copy")
        ctx = FMContext(F, k, **kw)
        ctx.load_tables(ids, w, V)
        d = ctx.batch_splits(to_host(lay), split_rows) if views else None
        plain = ctx.batch(to_host(data)) if views else None
        out, into = [], None
        for t, s in enumerate(sels, start=1):
            b = ctx.split_view(d, t - 1, into=into) if views else ctx.batch(to_host(_select(lay, np.arange(split_rows[t - 1], split_rows[t]))))
            into = b if views else None
            b.prepare()
            o = ctx.step_batch(b, t, cfg["step"], cfg["reg"])
            out.append((o.executed, o.loss_sum, o.n_rows, o.n_loss_rows, o.n_unique))
        t = len(sels) + 1
        g = ctx.batch_from_rows(plain, picks) if views else ctx.batch(to_host(_select(data, picks)))
        g.prepare()
        o = ctx.step_batch(g, t, cfg["step"], cfg["reg"])
        out.append((o.executed, o.loss_sum, o.n_rows, o.n_loss_rows, o.n_unique))
        tab = ctx.export_tables()
        ctx.close()
        return out, tab

    for path in ("fused", "unfused", "sharded3", "replicated3"):
        a, b = run(path, True), run(path, False)
        assert a[0] == b[0], (path, cfg)
        for x, y in zip(a[1], b[1]):
            assert np.array_equal(x, y), (path, cfg)


@pytest.mark.parametrize("case", range(10))
def test_random_loss_grad_and_vector_sum(gpu, case):
    """calcLossGrad (Model.scala:135-234) per entry on random problems against the oracle, and
    VectorSum by key (FactorizationMachines.scala:45-81) on random keys and widths, bitwise the
    oracle's sequential sums."""
    from fm_spark_amd.engine import FMContext

    cfg, batches, ids, w, V = draw(8089 + case)
    F, k = cfg["F"], cfg["k"]
    model = R.Model.empty(F, k)
    model.load(ids, w, V)
    ctx = FMContext(F, k)
    ctx.load_tables(ids, w, V)
    csr = batches[1]
    if csr.nnz:
        gp, gl, gdw, gdv = ctx.loss_grad(to_host(csr))
        rp, rl, rdw, rdv = R.loss_grad(model, csr)
        np.testing.assert_allclose(gp, rp, rtol=1e-6, atol=1e-9, err_msg=str(cfg))
        np.testing.assert_allclose(gl, rl, rtol=1e-5, atol=1e-9, err_msg=str(cfg))
        np.testing.assert_array_equal(gdw, rdw)
        np.testing.assert_allclose(gdv, rdv, rtol=1e-5, atol=1e-9, err_msg=str(cfg))
    rng = np.random.default_rng(case)
    n, width = int(rng.integers(1, 50000)), int(rng.integers(1, 40))
    keys = rng.integers(0, int(rng.integers(1, 5000)), n).astype(np.int32)
    vecs = rng.normal(size=(n, width)) * 10.0 ** rng.uniform(-3, 3, size=(n, 1))
    gk, gs = ctx.vector_sum_by_key(keys, vecs)
    rk, rs = R.vector_sum_by_key(keys, vecs)
    np.testing.assert_array_equal(gk, rk)
    assert np.array_equal(gs, rs)
    ctx.close()
