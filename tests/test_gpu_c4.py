"""GPU: BASELINE config c4 at its own shape -- F = Int.MaxValue (2^31 - 1), k = 32, the table
row-sharded over 8 ranks -- on the HIP path, seen from one rank (tests/c4_emul.py).

One MI355X holds rank 0's eighth of the table: 268,435,456 rows of a real fm_ctx (shard 0 of 8,
every row present after the seeded range init), 69 GB of HBM.  Rank 0 routes and combines its
own 256K-row batch on the device and runs the owner phases over the entries that all eight
ranks' 256K-row batches route to it (about 10.2M entries, 2.1M pairs); the seven other ranks are
emulated.  Checked (README.md:7-8 "feature dimension up to Int.MaxValue"; Model.scala:281,289
Int ids; SGD.scala:116-211):
  * the device route of rank 0's batch equals the emulated routing (counts and wire entries);
  * rank 0's loss equals the fp64 forward of its batch over the pre-step rows (rel 1e-5);
  * distinct ids the owner updated = distinct owner-0 ids of the eight batches;
  * per-feature update parity against the fp64 oracle step over the samples that hold chosen
    owner-0 ids (hot runs spanning many 256-entry update waves, mid, cold), padded with empty
    rows to the global miniBatchSize 8 x 256K (as test_gpu_fullsize does for c3);
  * owned rows absent from every batch only take the step's L1 shrink.
"""

import math

import numpy as np
import pytest

from oracle import fm_ref as R_

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-5, 1e-8
STEP, REG = 0.1, 1e-6


class _Cat:
    """The eight batches concatenated in rank order (the global mini-batch)."""

    def __init__(self, hb):
        off = np.concatenate([[0], np.cumsum([b.nnz for b in hb])])
        self.row_ptr = np.concatenate([[0]] + [b.row_ptr[1:] + off[i] for i, b in enumerate(hb)]).astype(np.int64)
        self.col = np.concatenate([b.col for b in hb])
        self.val = np.concatenate([b.val for b in hb])
        self.label = np.concatenate([b.label for b in hb])
        self.n_rows = len(self.label)


def _sub_problem(b, chosen):
    rows = np.repeat(np.arange(b.n_rows), np.diff(b.row_ptr))
    samples = np.unique(rows[np.isin(b.col, chosen)])
    lens = np.diff(b.row_ptr)[samples]
    starts = b.row_ptr[samples]
    tot = int(lens.sum())
    first = np.concatenate([[0], np.cumsum(lens)[:-1]])
    idx = np.arange(tot) + np.repeat(starts - first, lens)
    pad = b.n_rows - len(samples)
    row_ptr = np.concatenate([[0], np.cumsum(lens), np.full(pad, tot)]).astype(np.int64)
    label = np.concatenate([b.label[samples], np.zeros(pad)])
    return row_ptr, b.col[idx].astype(np.int64), b.val[idx], label


@pytest.mark.timeout(900)
def test_c4_rank_full_size_step(gpu):
    import torch

    from c4_emul import B_C4, F_C4, K_C4, R_C4, TBatch, other_rows_np, run_iteration
    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.distributed import HipShardEngine

    eng = HipShardEngine(F_C4, K_C4, 0, R_C4, seed=20261015, init_sd=0.01)
    assert eng.ctx.num_features == 2**31 - 1
    eng.init_random_range(0, F_C4)  # all 268,435,456 rows of this rank present
    hb = [synthetic_batch(B_C4, F_C4, batch_index=700 + r) for r in range(R_C4)]
    cat = _Cat(hb)
    ids64 = cat.col.astype(np.int64)
    assert ids64.max() > 2**30  # the id range reaches past 2^30 (slots past 2^27)
    own_ids, own_cnt = np.unique(ids64[ids64 % R_C4 == 0], return_counts=True)

    # chosen owner-0 ids: runs of 2,000-30,000 entries (8-117 update waves), 200-2,000, and cold
    rng = np.random.default_rng(4)
    hot_pool = own_ids[(own_cnt >= 2000) & (own_cnt <= 30000)]
    hot = hot_pool[np.argsort(-own_cnt[np.isin(own_ids, hot_pool)], kind="stable")[:3]]
    mid_pool = own_ids[(own_cnt >= 200) & (own_cnt < 2000)]
    mid = rng.choice(mid_pool, size=min(20, len(mid_pool)), replace=False)
    cold = rng.choice(own_ids, size=500, replace=False)
    chosen = np.unique(np.concatenate([hot, mid, cold]))
    assert len(hot) == 3 and own_cnt[np.searchsorted(own_ids, hot)].min() >= 2000

    # the oracle sub-problem and the pre-step rows it needs (owner-0 rows from the device)
    row_ptr, col, val, label = _sub_problem(cat, chosen)
    uniq, inv = np.unique(col, return_inverse=True)
    mine = uniq % R_C4 == 0
    w_pre = np.zeros(len(uniq))
    V_pre = np.zeros((len(uniq), K_C4))
    wd, Vd, pres = eng.ctx.export_rows(uniq[mine])
    assert pres.all()
    w_pre[mine], V_pre[mine] = wd, Vd
    w_pre[~mine], V_pre[~mine] = other_rows_np(uniq[~mine], K_C4)
    # rank 0's whole batch for the loss check, and a probe of owned rows no batch touches
    b0_ids = np.unique(hb[0].col.astype(np.int64))
    b0_own = b0_ids[b0_ids % R_C4 == 0]
    w0_own, V0_own, _ = eng.ctx.export_rows(b0_own)
    probe = rng.integers(0, (F_C4 + R_C4 - 1) // R_C4, size=20000) * R_C4
    probe = np.setdiff1d(probe[probe < F_C4], own_ids)
    wp0, Vp0, _ = eng.ctx.export_rows(probe)

    b0 = eng.batch(CSRHost(hb[0].row_ptr, hb[0].col, hb[0].val, hb[0].label))
    tbs = [TBatch(b, eng.device) for b in hb]
    info = run_iteration(eng, b0, tbs, 1, STEP, REG)
    assert info["route_counts_ok"] and info["route_entries_ok"]
    assert info["n_entries_in"] == int(np.sum(ids64 % R_C4 == 0))
    loss, n_loss, n_uniq = eng.last_stats()
    assert n_uniq == len(own_ids)
    assert n_loss == B_C4

    # rank 0's loss: the fp64 forward of its batch over the pre-step rows
    b0i = hb[0].col.astype(np.int64)
    own_m = b0i % R_C4 == 0
    Wt = np.zeros(len(b0i))
    Vt = np.zeros((len(b0i), K_C4))
    p = np.searchsorted(b0_own, b0i[own_m])
    Wt[own_m], Vt[own_m] = w0_own[p], V0_own[p]
    Wt[~own_m], Vt[~own_m] = other_rows_np(b0i[~own_m], K_C4)
    x = hb[0].val
    rp = hb[0].row_ptr
    S = np.add.reduceat(Vt * x[:, None], rp[:-1], axis=0)
    vv = np.add.reduceat(np.sum(Vt * Vt, axis=1) * x * x, rp[:-1])
    wx = np.add.reduceat(Wt * x, rp[:-1])
    ref_loss = float(np.sum((0.5 * (np.sum(S * S, axis=1) - vv) + wx - hb[0].label) ** 2))
    assert loss == pytest.approx(ref_loss, rel=RTOL)
    assert loss == pytest.approx(info["own_loss_emul"], rel=1e-9)

    # per-feature update parity on the chosen owner-0 ids
    model = R_.Model.empty(len(uniq), K_C4)
    model.load(np.arange(len(uniq)), w_pre, V_pre)
    R_.sgd_step_fast(model, R_.CSR(row_ptr, inv.astype(np.int32), val, label), 1, STEP, REG)
    c = np.searchsorted(uniq, chosen)
    w1, V1, pres1 = eng.ctx.export_rows(chosen)
    assert pres1.all()
    np.testing.assert_allclose(w1, model.w[c], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(V1, model.V[c], rtol=RTOL, atol=ATOL)

    # untouched owned rows: the step's L1 shrink only (lazy composition, SGD.scala:177-181)
    lam = STEP / math.sqrt(1) * REG
    wp1, Vp1, _ = eng.ctx.export_rows(probe)
    np.testing.assert_allclose(wp1, R_.soft_threshold(wp0, lam), rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(Vp1, R_.soft_threshold(Vp0, lam), rtol=1e-6, atol=1e-9)
    print(f"\nc4 rank 0: {info['n_entries_in']} entries / {info['n_pairs_in']} pairs in, {n_uniq} rows updated, "
          f"hot runs {own_cnt[np.searchsorted(own_ids, hot)].tolist()}, sub-problem {len(uniq)} rows")
    del tbs
    b0.close()
    eng.ctx.close()
    torch.cuda.empty_cache()
