"""GPU: the HIP sharded phase kernels (fm_shard_* of include/fm_hip.h: route, owner_forward,
combine, owner_update).  R ranks are simulated in one process on one GPU (one fm_ctx per
rank, all-to-all done by tensor slicing), compared with the single-table oracle step over
the concatenated batches."""

import numpy as np
import pytest

from oracle import fm_ref as R_
from problems import make_problem

pytestmark = pytest.mark.gpu


def _concat(parts):
    row_ptr = [np.zeros(1, np.int64)]
    off = 0
    for p in parts:
        row_ptr.append(p.row_ptr[1:] + off)
        off += p.nnz
    return R_.CSR(np.concatenate(row_ptr), np.concatenate([p.col for p in parts]),
                  np.concatenate([p.val for p in parts]), np.concatenate([p.label for p in parts]))


def split_pairs(buf, counts, kp):
    """A pair buffer in the wire layout ([P][kp] vectors, then [P][2] scalars) cut per peer."""
    import torch

    counts = [int(c) for c in counts]
    P = sum(counts)
    vec = torch.split(buf[: P * kp], [c * kp for c in counts])
    sc = torch.split(buf[P * kp:], [c * 2 for c in counts])
    return list(zip(vec, sc))


def cat_pairs(parts):
    """Concatenate per-peer pieces back into the wire layout (what an all-to-all delivers)."""
    import torch

    return torch.cat([v for v, _ in parts] + [s for _, s in parts])


def _simulated_step(engines, batches, t, step_size, reg):
    """One iteration of the ShardedTrainer protocol with the all-to-alls done by slicing."""
    import torch

    R = len(engines)
    W = engines[0].width
    kp = engines[0].kp
    routed = [e.route(b) for e, b in zip(engines, batches)]
    ent_cnt = [c[:R] for _, _, c in routed]   # [src][owner]
    pair_cnt = [c[R:] for _, _, c in routed]
    keep = []
    torch.cuda.synchronize()  # the slicing below runs on the main stream, owner_prepare on the side streams
    for o in range(R):
        slots = torch.cat([torch.split(routed[r][0], ent_cnt[r].tolist())[o] for r in range(R)])
        ents = torch.cat([torch.split(routed[r][1], (2 * ent_cnt[r]).tolist())[o] for r in range(R)])
        src_e = np.array([ent_cnt[r][o] for r in range(R)])
        src_p = np.array([pair_cnt[r][o] for r in range(R)])
        engines[o].owner_prepare(batches[o], slots, ents, src_e, src_p)
        keep.append((slots, ents, src_p))
    torch.cuda.synchronize()  # route / prepare ran on the engines' side streams
    partials = []
    for o in range(R):
        out = engines[o].owner_forward(batches[o], int(keep[o][2].sum()))
        partials.append(split_pairs(out, keep[o][2], kp))
    s_rows = []
    for r in range(R):
        pin = cat_pairs([partials[o][r] for o in range(R)])
        s = engines[r].combine(batches[r], pin, int(pair_cnt[r].sum()))
        s_rows.append(split_pairs(s, pair_cnt[r], kp))
    gm = sum(int(b.n_rows) for b in batches)
    for o in range(R):
        engines[o].owner_update(batches[o], cat_pairs([s_rows[r][o] for r in range(R)]), t, step_size, reg, gm)
    torch.cuda.synchronize()
    return sum(e.last_stats()[0] for e in engines), sum(e.last_stats()[2] for e in engines)


# F = R * 2^s + 1 (513 at R = 2 and R = 4): owner 0 holds one slot more than the others, and that
# slot (id F - 1, made hot) needs one more key bit than a rank with fewer rows would give it
@pytest.mark.parametrize("R,k,F,hot", [(1, 8, 503, 11), (2, 16, 503, 11), (3, 5, 503, 11), (4, 32, 503, 11),
                                       (2, 8, 513, 512), (4, 4, 513, 512), (1, 16, 503, 11), (3, 8, 503, 11),
                                       (8, 16, 1031, 7), (12, 16, 1031, 7)])
def test_hip_shard_phases_match_single_table(gpu, R, k, F, hot):
    """The fm_shard_* phases driven one by one (the all-to-alls done by slicing) against the fp64
    oracle step over the concatenated batches (R = 12: the combine's any-R path; R <= 8 keeps each
    sample's pair slots in registers)."""
    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.distributed import HipShardEngine

    _, ids, w, V = make_problem(3, 1, F, k, 1)
    engines = [HipShardEngine(F, k, r, R) for r in range(R)]
    for e in engines:
        e.load_tables(ids, w, V)
    model = R_.Model.empty(F, k)
    model.load(ids, w, V)
    for t in range(1, 4):
        parts = [make_problem(100 * t + r, 120 + 17 * r, F, k, 9, hot=hot)[0] for r in range(R)]
        bs = [e.batch(CSRHost(p.row_ptr, p.col, p.val, p.label)) for e, p in zip(engines, parts)]
        loss, nu = _simulated_step(engines, bs, t, 0.3, 1e-4)
        cat = _concat(parts)
        ref = R_.sgd_step_fast(model, cat, t, 0.3, 1e-4)
        assert loss == pytest.approx(ref.loss_sum, rel=1e-5), f"step {t}"
        assert nu == len(np.unique(cat.col))
    gi, gw, gV = zip(*[e.export_tables() for e in engines])
    gi = np.concatenate(gi)
    order = np.argsort(gi)
    np.testing.assert_array_equal(gi[order], np.nonzero(model.present)[0])
    np.testing.assert_allclose(np.concatenate(gw)[order], model.w[gi[order]], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(np.concatenate(gV)[order], model.V[gi[order]], rtol=1e-5, atol=1e-8)


def test_hip_shard_c3_r8_matches_single_table(gpu):
    """Config c3's table at R = 8 (100M hashed features, k = 16, owner = id % 8), eight ranks of
    32K synthetic rows each (the bench's generator), two iterations of the sharded phases
    against one single-table HIP step over the concatenated batches: losses, distinct counts
    and every touched row (the two paths differ only in fp summation order)."""
    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.distributed import HipShardEngine
    from fm_spark_amd.engine import FMContext

    F, k, R, B = 100_000_000, 16, 8, 32768
    ref = FMContext(F, k, seed=5, init_sd=0.01)
    engines = [HipShardEngine(F, k, r, R) for r in range(R)]
    for t in (1, 2):
        parts = [synthetic_batch(B, F, batch_index=100 * t + r) for r in range(R)]
        cat = _concat([R_.CSR(p.row_ptr, p.col, p.val, p.label) for p in parts])
        cb = ref.batch(CSRHost(cat.row_ptr, cat.col, cat.val, cat.label))
        before = np.zeros(0, np.int32) if t == 1 else ids
        ref.init_from_batch(cb)  # createInitialModel's rows for the new ids, loaded on every owner
        ids, w, V = ref.export_tables()
        new = ~np.isin(ids, before)
        for e in engines:
            e.load_tables(ids[new], w[new], V[new])
        o = ref.step_batch(cb, t, 0.1, 1e-6, sync=True)
        bs = [e.batch(CSRHost(p.row_ptr, p.col, p.val, p.label)) for e, p in zip(engines, parts)]
        loss, nu = _simulated_step(engines, bs, t, 0.1, 1e-6)
        assert nu == o.n_unique == len(np.unique(cat.col))
        assert loss == pytest.approx(o.loss_sum, rel=1e-9), f"step {t}"
    gi, gw, gV = ref.export_tables()
    si, sw, sV = (np.concatenate(x) for x in zip(*[e.export_tables() for e in engines]))
    order = np.argsort(si)
    np.testing.assert_array_equal(si[order], gi)
    np.testing.assert_allclose(sw[order], gw, rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(sV[order], gV, rtol=1e-5, atol=1e-8)


def test_sharded_trainer_world1_rccl(gpu):
    """The full ShardedTrainer over torch.distributed (nccl = RCCL) with one rank."""
    import os

    import torch
    import torch.distributed as dist

    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.distributed import ShardedTrainer

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        F, k = 300, 16
        _, ids, w, V = make_problem(4, 1, F, k, 1)
        tr = ShardedTrainer(F, k, rank=0, world=1)
        tr.load_tables(ids, w, V)
        model = R_.Model.empty(F, k)
        model.load(ids, w, V)
        probs = [make_problem(50 + t, 200, F, k, 8, hot=2)[0] for t in range(1, 6)]
        bs = [tr.batch(CSRHost(p.row_ptr, p.col, p.val, p.label)) for p in probs]
        # steps 1-2 plain, steps 3-5 with the next batch prefetched behind each update
        for t in range(1, 6):
            nxt = bs[t] if 3 <= t < 5 else None
            o = tr.step(bs[t - 1], t, 0.2, 1e-5, prefetch=nxt)
            ref = R_.sgd_step_fast(model, probs[t - 1], t, 0.2, 1e-5)
            assert o.loss_sum == pytest.approx(ref.loss_sum, rel=1e-5)
            assert o.n_unique == len(np.unique(probs[t - 1].col))
        gi, gw, gV = tr.export_tables()
        np.testing.assert_array_equal(gi, np.nonzero(model.present)[0])
        np.testing.assert_allclose(gw, model.w[gi], rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(gV, model.V[gi], rtol=1e-5, atol=1e-8)
    finally:
        dist.destroy_process_group()


def test_hip_shard_empty_rank_and_empty_rows(gpu):
    """One rank steps an empty batch, the other one with empty rows; the global step still
    equals the single-table step over the concatenation (m counts every row)."""
    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.distributed import HipShardEngine

    F, k, R = 97, 4, 2
    _, ids, w, V = make_problem(8, 1, F, k, 1)
    engines = [HipShardEngine(F, k, r, R) for r in range(R)]
    for e in engines:
        e.load_tables(ids, w, V)
    model = R_.Model.empty(F, k)
    model.load(ids, w, V)
    empty = R_.CSR(np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0), np.zeros(0))
    p = make_problem(9, 40, F, k, 5, hot=3)[0]
    # make rows 3 and 7 empty
    lens = np.diff(p.row_ptr)
    keep = np.ones(p.nnz, bool)
    for r_ in (3, 7):
        keep[p.row_ptr[r_]:p.row_ptr[r_ + 1]] = False
    lens[[3, 7]] = 0
    q = R_.CSR(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64), p.col[keep], p.val[keep], p.label)
    parts = [empty, q]
    bs = [e.batch(CSRHost(c.row_ptr, c.col, c.val, c.label)) for e, c in zip(engines, parts)]
    loss, nu = _simulated_step(engines, bs, 1, 0.3, 1e-4)
    ref = R_.sgd_step_fast(model, _concat(parts), 1, 0.3, 1e-4)
    assert loss == pytest.approx(ref.loss_sum, rel=1e-5)
    gi, gw, gV = zip(*[e.export_tables() for e in engines])
    gi = np.concatenate(gi)
    order = np.argsort(gi)
    np.testing.assert_allclose(np.concatenate(gw)[order], model.w[gi[order]], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(np.concatenate(gV)[order], model.V[gi[order]], rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("R,k", [(1, 8), (3, 16)])
def test_hip_replicated_matches_single_table(gpu, R, k):
    """fm_repl_grad / fm_repl_apply with R replicas in one process (the all-reduce is a tensor
    sum), against the single-table oracle step over the concatenated batches; the replicas
    stay bitwise identical."""
    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.distributed import HipReplEngine

    F = 401
    _, ids, w, V = make_problem(12, 1, F, k, 1)
    engines = [HipReplEngine(F, k) for _ in range(R)]
    for e in engines:
        e.load_tables(ids, w, V)
    model = R_.Model.empty(F, k)
    model.load(ids, w, V)
    for t in range(1, 4):
        parts = [make_problem(300 * t + r, 90 + 11 * r, F, k, 7, hot=5)[0] for r in range(R)]
        bs = [e.batch(CSRHost(p.row_ptr, p.col, p.val, p.label)) for e, p in zip(engines, parts)]
        grads = [e.grad_phase(b).clone() for e, b in zip(engines, bs)]
        total = grads[0]
        for g in grads[1:]:
            total = total + g
        gm = sum(p.n_rows for p in parts)
        for e in engines:
            e.apply(total, t, 0.3, 1e-4, gm)
        cat = _concat(parts)
        ref = R_.sgd_step_fast(model, cat, t, 0.3, 1e-4)
        # each engine's loss covers its own rows
        assert sum(engines[r].last_stats()[0] for r in range(R)) == pytest.approx(ref.loss_sum, rel=1e-5)
        assert engines[0].last_stats()[2] == len(np.unique(cat.col))
    exports = [e.export_tables() for e in engines]
    gi, gw, gV = exports[0]
    np.testing.assert_array_equal(gi, np.nonzero(model.present)[0])
    np.testing.assert_allclose(gw, model.w[gi], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(gV, model.V[gi], rtol=1e-5, atol=1e-8)
    for oi, ow, oV in exports[1:]:
        np.testing.assert_array_equal(oi, gi)
        np.testing.assert_array_equal(ow, gw)
        np.testing.assert_array_equal(oV, gV)
