"""GPU: the bucket sort (fm_sort.hip, MSD pass on the top bits + one block per bucket) gives the
step exactly what the LSD passes give it.

Both sorts are stable by feature slot, so the step that consumes them must come out bit for bit
the same; each case also runs against the fp64 oracle.  FM_SORT_BUCKET_MIN=0 forces the bucket
path at test sizes (it normally starts at 1M entries); FM_SORT_BUCKET=0 selects the LSD passes.
Cases cover one in-bucket pass (slots of <= 9 + 9 bits), two passes, and a hot feature whose
bucket outgrows the LDS image (30720 entries) and takes the global-scratch route.
"""

import numpy as np
import pytest

from oracle import fm_ref as R
from problems import make_problem
from test_gpu_parity import assert_tables, run_both, to_host

pytestmark = pytest.mark.gpu


def _run(monkeypatch, bucket, csrs, F, k, ids, w, V):
    monkeypatch.setenv("FM_SORT_BUCKET", "1" if bucket else "0")
    monkeypatch.setenv("FM_SORT_BUCKET_MIN", "0")
    return run_both(csrs, F, k, ids, w, V, 0.2, 1e-5)


@pytest.mark.parametrize(
    "F,n_rows,mean_nnz,hot",
    [
        (5000, 1500, 12, None),       # 13-bit slots: one in-bucket pass of 4 bits
        (300000, 3000, 20, 7),        # 19-bit slots: two in-bucket passes (5 + 5 bits)
        ((1 << 21) + 5, 2500, 16, 123),  # 22-bit slots
        (70000, 20000, 6, 4242),      # hot id in ~90 % of rows: an 18K-entry bucket
        (70000, 40000, 4, 4243),      # hot id in ~90 % of 40K rows: a 36K-entry bucket (global scratch)
    ],
)
def test_bucket_sort_step_matches_lsd_bitwise(monkeypatch, gpu, F, n_rows, mean_nnz, hot):
    k = 8
    csrs = [make_problem(900 + i, n_rows, F, k, mean_nnz, hot=hot)[0] for i in range(2)]
    _, ids, w, V = make_problem(77, 1, F, k, 1)
    model, g_b, losses_b = _run(monkeypatch, True, csrs, F, k, ids, w, V)
    _, g_l, losses_l = _run(monkeypatch, False, csrs, F, k, ids, w, V)
    assert_tables(model, g_b)
    for (gb, rb), (gl, _) in zip(losses_b, losses_l):
        assert gb == gl
        np.testing.assert_allclose(gb, rb, rtol=1e-6)
    for a, b in zip(g_b, g_l):
        assert np.array_equal(a, b)


def test_bucket_sort_prepared_batch(monkeypatch, gpu):
    """fm_batch_prepare (the sorted view written into the batch's own buffers) through the bucket path."""
    from fm_spark_amd.engine import FMContext

    monkeypatch.setenv("FM_SORT_BUCKET_MIN", "0")
    F, k = 40000, 16
    csrs = [make_problem(950 + i, 4000, F, k, 25, hot=11)[0] for i in range(3)]
    _, ids, w, V = make_problem(78, 1, F, k, 1)
    model = R.Model.empty(F, k)
    model.load(ids, w, V)
    ctx = FMContext(F, k)
    ctx.load_tables(ids, w, V)
    dbs = [ctx.batch(to_host(c)) for c in csrs]
    for b in dbs:
        b.prepare()
    for i, (c, b) in enumerate(zip(csrs, dbs)):
        ro = R.sgd_step_fast(model, c, i + 1, 0.2, 1e-5)
        go = ctx.step_batch(b, i + 1, 0.2, 1e-5)
        np.testing.assert_allclose(go.loss_sum, ro.loss_sum, rtol=1e-6)
        assert go.n_unique == ro.n_unique
    assert_tables(model, ctx.export_tables())
    ctx.close()
