"""GPU: the two-level grouping (fm_msd.hip, fm_config.sort_algo = FM_SORT_DEFAULT) against the LSD
radix passes (FM_SORT_LSD), bit for bit.

Both are stable sorts by feature slot -- the reference's groupBy featureId with the CSR order kept
inside each feature (FactorizationMachinesSGD.scala:148-155) -- so the sorted view, the fused step's
multi view and every table after every step must be the same bits, fused and unfused.  The shapes
cover each branch of the plan (msd_plan) and of the kernels:
  * one bucket (n <= 32K entries, slots of <= 17 bits): no level-1 pass;
  * level-1 buckets with one or two LDS passes, 20- and 27-bit slots;
  * oversized buckets (a hot feature in > 32K entries: k_msd_presort) with two passes, one pass (the
    split's copy back) and none (a bucket of one slot);
  * one bucket holding every entry and 63 empty ones (the look-back over empty buckets);
  * ragged and empty rows; steps on unprepared batches (the inline LSD sort) in between.
"""

import numpy as np
import pytest

from problems import f32
from test_gpu_parity import to_host

pytestmark = pytest.mark.gpu


def field_batch(seed, B, F, z, *, zipf=1.15, hot=None, hot_frac=0.0, id_hi=None, empty_frac=0.05):
    """Criteo-shaped rows: field j draws Zipf ranks hashed into its own id range (distinct ids per
    row); ragged lengths, some rows empty; `hot` replaces field 0 in a fraction of the rows."""
    from oracle import fm_ref as R

    rng = np.random.default_rng(seed)
    hi = F if id_hi is None else id_hi
    span = max(hi // z, 1)
    r = rng.zipf(zipf, size=(B, z)).astype(np.int64) - 1
    ids = np.arange(z, dtype=np.int64)[None, :] * span + (r * 2654435761) % span
    if hot is not None:
        ids[rng.random(B) < hot_frac, 0] = hot
    lens = rng.integers(1, z + 1, size=B)
    lens[rng.random(B) < empty_frac] = 0
    keep = np.arange(z)[None, :] < lens[:, None]
    col = ids[keep].astype(np.int32)
    row_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    val = f32(rng.normal(size=col.size))
    y = (rng.random(B) < 0.3).astype(np.float64)
    return R.CSR(row_ptr=row_ptr, col=col, val=val, label=y)


def run(sort, fuse, csrs, F, k, init_ids, steps, prepare=lambda t: True):
    from fm_spark_amd.engine import FMContext

    ctx = FMContext(F, k, fuse=fuse, sort=sort, seed=5, init_sd=0.05)
    ctx.init_random(init_ids)
    dbs = [ctx.batch(to_host(c)) for c in csrs]
    out = []
    for t in range(1, steps + 1):
        b = dbs[(t - 1) % len(dbs)]
        if prepare(t):
            b.prepare()
        o = ctx.step_batch(b, t, 0.2, 1e-4)
        out.append((o.loss_sum, o.n_unique, o.n_loss_rows))
    present = np.unique(np.concatenate([c.col for c in csrs] + [init_ids]))
    w, V, pres = ctx.export_rows(present.astype(np.int32))
    ctx.close()
    return out, w, V, pres


def assert_bitwise(a, b):
    assert a[0] == b[0]  # losses, distinct counts, loss rows: the same bits
    for x, y in zip(a[1:], b[1:]):
        assert np.array_equal(x, y)


CASES = {
    # name: (F, k, batches [(B, z, kwargs)])
    "one_bucket": (20000, 8, [(2000, 10, {}), (1800, 12, {"hot": 3, "hot_frac": 0.5})]),
    "buckets_20bit": (1 << 20, 8, [(60000, 10, {}), (50000, 12, {"zipf": 1.3})]),
    "oversized_two_passes": (1 << 20, 16, [(50000, 10, {"hot": 5, "hot_frac": 0.9})]),
    "oversized_one_pass": (1 << 15, 4, [(40000, 5, {"hot": 3, "hot_frac": 0.9})]),
    "oversized_one_slot": (64, 4, [(40000, 5, {"hot": 1, "hot_frac": 0.9})]),
    "one_full_bucket": (1 << 20, 8, [(10000, 10, {"id_hi": 2000})]),
    "buckets_27bit": (100_000_000, 4, [(100000, 10, {"zipf": 1.05})]),
}


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("fuse", [True, False])
def test_two_level_grouping_bitwise_lsd(gpu, name, fuse):
    F, k, specs = CASES[name]
    csrs = [field_batch(900 + i, B, F, z, **kw) for i, (B, z, kw) in enumerate(specs)]
    used = np.unique(np.concatenate([c.col for c in csrs]))
    init_ids = used[::2].astype(np.int32)  # half the touched rows present, the rest absent
    steps = 3
    a = run("default", fuse, csrs, F, k, init_ids, steps)
    b = run("lsd", fuse, csrs, F, k, init_ids, steps)
    assert_bitwise(a, b)
    assert a[0][0][1] > 0


def test_two_level_with_unprepared_steps(gpu):
    """Unprepared steps (sorted inline by the LSD passes) between prepared ones: the same bits."""
    F, k = 1 << 20, 16
    csrs = [field_batch(950 + i, 40000, F, 12, hot=7, hot_frac=0.3) for i in range(3)]
    init_ids = np.arange(0, F, 3, dtype=np.int32)
    prep = lambda t: t % 3 != 0  # noqa: E731
    a = run("default", True, csrs, F, k, init_ids, 6, prepare=prep)
    b = run("lsd", True, csrs, F, k, init_ids, 6, prepare=prep)
    assert_bitwise(a, b)
