"""GPU parity on fp64 inputs that are NOT pre-rounded to fp32 (VERDICT r01 "What's weak" 1).

Every other full-size fixture rounds x, the labels and M0 to fp32 first, so the device starts
from exactly the oracle's values.  Here nothing is rounded: x = log1p(Poisson(3)) and the
regression labels y = <w*, x> + N(0, 0.1) stay fp64 (Spark's Double columns), M0 is an fp64
Gaussian draw.  The device rounds x and the tables to fp32 on upload and keeps the labels, yhat
and the residual yhat - y in fp64 (FactorizationMachinesSGD.scala:145-146 forms pred - label in
Double).  Five steps per config against the fp64 oracle over the whole table; the largest
relative errors on w, V and the per-step loss are printed (run with -s) and asserted <= 1e-5.

Configs (BASELINE.json): c2 = 1M features, k = 8, 64K rows, Zipf(1.05); c5 shape = 1M features,
Zipf(1.2) hot rows, regression loss, k = 16 (a point of the CrossValidator grid), 64K rows."""

import numpy as np
import pytest

from oracle import fm_ref as R

pytestmark = pytest.mark.gpu

RTOL = 1e-5
ATOL = 1e-12  # fp64 Gaussians: no table value is 0, the bound is relative everywhere
STEP, STEPS = 0.1, 5


def _rel(a, b):
    """(largest relative error over values with |ref| >= 1e-6, largest absolute error below that:
    values the L1 shrink leaves next to zero carry no relative meaning)."""
    big = np.abs(b) >= 1e-6
    rel = float(np.max(np.abs(a - b)[big] / np.abs(b[big]))) if big.any() else 0.0
    ab = float(np.max(np.abs(a - b)[~big])) if (~big).any() else 0.0
    return rel, ab


@pytest.mark.parametrize("name,F,k,B,zipf_s,reg", [
    ("c2", 1_000_000, 8, 65536, 1.05, 1e-6),
    ("c5", 1_000_000, 16, 65536, 1.2, 1e-5),
])
def test_fp64_inputs_full_table_parity(gpu, name, F, k, B, zipf_s, reg):
    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.engine import FMContext

    rng = np.random.default_rng(2026 + k)
    w_star = rng.normal(0.0, 0.1, F)
    hb = [synthetic_batch(B, F, batch_index=40 + i, zipf_s=zipf_s, labels="regression", w_star=w_star, exact=True)
          for i in range(STEPS)]
    # the fixtures really are fp64: neither x nor y survive a round trip through fp32
    assert np.any(hb[0].val != hb[0].val.astype(np.float32))
    assert np.all(hb[0].label != hb[0].label.astype(np.float32))
    ids = np.arange(F, dtype=np.int32)
    w0 = rng.normal(0.0, 0.01, F)
    V0 = rng.normal(0.0, 0.01, (F, k))
    model = R.Model.empty(F, k)
    model.load(ids, w0, V0)
    ctx = FMContext(F, k, seed=3)
    ctx.load_tables(ids, w0, V0)
    loss_err = 0.0
    for t, b in enumerate(hb, start=1):
        ref = R.sgd_step_fast(model, R.CSR(b.row_ptr, b.col, b.val, b.label), t, STEP, reg)
        out = ctx.step(CSRHost(b.row_ptr, b.col, b.val, b.label), t, STEP, reg)
        assert out.n_unique == ref.n_unique and out.n_loss_rows == ref.n_loss_rows
        loss_err = max(loss_err, abs(out.loss_sum - ref.loss_sum) / abs(ref.loss_sum))
    gi, gw, gV = ctx.export_tables()
    ctx.close()
    np.testing.assert_array_equal(gi, ids)
    (ew, aw), (eV, aV) = _rel(gw, model.w), _rel(gV, model.V)
    print(f"\n{name} fp64 inputs, {STEPS} steps: max rel err w {ew:.3g}, V {eV:.3g} (|ref| >= 1e-6), max abs err "
          f"below it w {aw:.3g}, V {aV:.3g}; loss rel err {loss_err:.3g}")
    assert loss_err <= RTOL
    np.testing.assert_allclose(gw, model.w, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(gV, model.V, rtol=RTOL, atol=ATOL)
