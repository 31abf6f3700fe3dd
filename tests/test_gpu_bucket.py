"""GPU: the two-phase bucket sort (fm_config.sort_algo = FM_SORT_BUCKET; fm_sort.hip "bucket sort")
against the three-pass LSD sort.  Both are stable sorts by feature slot, so every step -- unfused
(the whole sorted view) or fused (the multi view the bucket sort keeps as it orders each bucket,
against the LSD view reduced by the split pass) -- must be bitwise the same: losses, counts and
tables.  Cases: random batches, Zipf-skewed ids, a feature in every row (its bucket larger than the
LDS image and mixed: the global-scratch passes and the in-place compaction), a bucket holding one
hot id alone (larger than the image, all one key: copied as is), prepared and unprepared batches,
k = 8 and 16."""

import numpy as np
import pytest

from oracle import fm_ref as R
from problems import make_problem
from test_gpu_parity import to_host

pytestmark = pytest.mark.gpu


def _csr_from_rows(rows, rng, F):
    rp = np.zeros(len(rows) + 1, dtype=np.int64)
    np.cumsum([len(r) for r in rows], out=rp[1:])
    col = np.concatenate(rows).astype(np.int32) if rows else np.zeros(0, np.int32)
    val = np.float32(rng.normal(size=len(col))).astype(np.float64)
    val[rng.random(len(col)) < 0.3] = 1.0
    return R.CSR(rp, col, val, (rng.random(len(rows)) < 0.3).astype(np.float64))


def _hot_batch(seed, n_rows, F, hot, avoid=None, per_row=8):
    """Every row holds `hot`; its other ids are uniform over [0, F) minus the range `avoid`."""
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(n_rows):
        z = int(rng.integers(1, 2 * per_row))
        ids = rng.choice(F, size=z + 4, replace=False)
        if avoid is not None:
            ids = ids[(ids < avoid[0]) | (ids >= avoid[1])]
        ids = ids[ids != hot][:z]
        rows.append(np.sort(np.append(ids, hot)))
    return _csr_from_rows(rows, rng, F)


def _zipf_batch(seed, n_rows, F, s=1.2, per_row=10):
    rng = np.random.default_rng(seed)
    rows = []
    perm = rng.permutation(F)
    for _ in range(n_rows):
        z = int(rng.integers(1, 2 * per_row))
        ids = np.unique(perm[np.minimum(rng.zipf(s, size=z) - 1, F - 1)])
        rows.append(ids)
    return _csr_from_rows(rows, rng, F)


def _run(sort, fuse, F, k, csrs, steps, prepare):
    from fm_spark_amd.engine import FMContext

    _, ids, w, V = make_problem(91, 1, F, k, 1)
    ctx = FMContext(F, k, fuse=fuse, sort=sort)
    ctx.load_tables(ids, w, V)
    dbs = [ctx.batch(to_host(c)) for c in csrs]
    out = []
    for t in range(1, steps + 1):
        b = dbs[(t - 1) % len(dbs)]
        if prepare(t):
            b.prepare()
        o = ctx.step_batch(b, t, 0.3, 1e-3)
        out.append((o.loss_sum, o.n_loss_rows, o.n_unique))
    tab = ctx.export_tables()
    ctx.close()
    return out, tab


def _same(a, b):
    assert a[0] == b[0]
    for x, y in zip(a[1], b[1]):
        assert np.array_equal(x, y)


CASES = {
    "random": lambda F: [make_problem(1301 + i, 4000, F, 16, 12, hot=9)[0] for i in range(2)],
    "zipf": lambda F: [_zipf_batch(1310 + i, 6000, F) for i in range(2)],
    # 40,000 rows all holding id 3: its bucket (ids 0 .. 2^L - 1) far beyond the 30,720-entry image,
    # mixed with the other ids of that range
    "every_row_mixed": lambda F: [_hot_batch(1320, 40_000, F, 3), make_problem(1321, 3000, F, 16, 12)[0]],
    # id 5000 in every row and no other id of its bucket: one key, copied
    "every_row_alone": lambda F: [_hot_batch(1330, 40_000, F, 5000, avoid=(4096, 6144)),
                                  make_problem(1331, 3000, F, 16, 12)[0]],
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("k,fuse", [(16, True), (16, False), (8, True)])
def test_bucket_sort_step_bitwise_equal_lsd(gpu, case, k, fuse):
    F = 1 << 20
    csrs = CASES[case](F)
    prep = (lambda t: t % 3 != 0)  # noqa: E731  (every third step unprepared: the inline sort)
    a = _run("bucket", fuse, F, k, csrs, 4, prep)
    b = _run("lsd", fuse, F, k, csrs, 4, prep)
    _same(a, b)


def test_bucket_sort_against_oracle_and_c3_key_width(gpu):
    """27-bit feature slots (c3's 100M-row table: ten top bits per bucket, 17 low bits ordered in
    two in-LDS passes) on a small table-sized problem: the fused bucket-sorted step against the fp64
    oracle, and bitwise against the LSD step."""
    F = 100_000_000
    rng = np.random.default_rng(7)
    rows = [np.unique(rng.integers(0, F, size=int(rng.integers(1, 30)))) for _ in range(20_000)]
    hot = rng.integers(0, F, size=20)
    rows = [np.unique(np.append(r, hot[rng.integers(0, 20, size=3)])) for r in rows]
    csr = _csr_from_rows(rows, rng, F)
    ids = np.unique(csr.col)
    k = 16
    w = np.float32(rng.normal(0, 0.1, len(ids))).astype(np.float64)
    V = np.float32(rng.normal(0, 0.1, (len(ids), k))).astype(np.float64)
    from fm_spark_amd.engine import FMContext

    res = []
    for sort in ("bucket", "lsd"):
        ctx = FMContext(F, k, fuse=True, sort=sort)
        ctx.load_tables(ids, w, V)
        b = ctx.batch(to_host(csr))
        ls = []
        for t in (1, 2):
            b.prepare()
            o = ctx.step_batch(b, t, 0.3, 1e-4)
            ls.append((o.loss_sum, o.n_unique))
        res.append((ls, ctx.export_rows(ids)))
        ctx.close()
    assert res[0][0] == res[1][0]
    for x, y in zip(res[0][1], res[1][1]):
        assert np.array_equal(x, y)
    # the oracle over the present rows (a dense model of F rows is too large here: relabel the ids)
    remap = {int(v): i for i, v in enumerate(ids)}
    rc = R.CSR(csr.row_ptr, np.asarray([remap[int(c)] for c in csr.col], np.int32), csr.val, csr.label)
    model = R.Model.empty(len(ids), k)
    model.load(np.arange(len(ids), dtype=np.int32), w, V)
    for t in (1, 2):
        ro = R.sgd_step_fast(model, rc, t, 0.3, 1e-4)
        assert res[0][0][t - 1][0] == pytest.approx(ro.loss_sum, rel=1e-6)
        assert res[0][0][t - 1][1] == ro.n_unique
    gw, gV, _ = res[0][1]
    np.testing.assert_allclose(gw, model.w, rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(gV, model.V, rtol=1e-5, atol=1e-8)


def test_bucket_sort_oversized_bucket_at_c3_key_width(gpu):
    """27-bit slots with a feature in every one of 60,000 rows: its bucket (18 low bits, a 16K-entry
    LDS image) goes through the global-scratch passes (9 + 9 bits) and, fused, the in-place
    compaction; another feature alone in its bucket in every row (copied as one run).  Fused and
    unfused, bucket-sorted steps bitwise equal to the LSD-sorted ones over the touched rows."""
    from fm_spark_amd.engine import FMContext

    F, k = 100_000_000, 16
    rng = np.random.default_rng(17)
    hot_mixed, hot_alone = 12_345, 50_000_000  # bucket 0 (ids < 2^18) is full of other ids too
    rows = []
    for _ in range(60_000):
        z = int(rng.integers(2, 20))
        ids = rng.integers(0, F, size=z)
        ids = ids[(ids >> 18) != (hot_alone >> 18)]
        ids = np.concatenate([ids, rng.integers(0, 1 << 18, size=2), [hot_mixed, hot_alone]])
        rows.append(np.unique(ids))
    csr = _csr_from_rows(rows, rng, F)
    touched = np.unique(csr.col).astype(np.int32)
    for fuse in (True, False):
        res = []
        for sort in ("bucket", "lsd"):
            ctx = FMContext(F, k, fuse=fuse, sort=sort, seed=3, init_sd=0.01)
            ctx.init_from_batch(ctx.batch(to_host(csr)))
            b = ctx.batch(to_host(csr))
            ls = []
            for t in (1, 2):
                b.prepare()
                o = ctx.step_batch(b, t, 0.3, 1e-4)
                ls.append((o.loss_sum, o.n_unique))
            res.append((ls, ctx.export_rows(touched)))
            b.close()
            ctx.close()
        assert res[0][0] == res[1][0]
        for x, y in zip(res[0][1], res[1][1]):
            assert np.array_equal(x, y)
