"""GPU: the HIP sharded phase kernels (fm_shard_* of include/fm_hip.h).  R ranks are
simulated in one process on one GPU (one fm_ctx per rank, all-to-all done by tensor
slicing), compared with the single-table oracle step over the concatenated batches."""

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


def _simulated_step(engines, batches, t, step_size, reg):
    import torch

    R = len(engines)
    W = engines[0].width
    dev = engines[0].device
    sends = [e.plan(b) for e, b in zip(engines, batches)]
    reqs = []
    for e, s in zip(engines, sends):
        q = torch.empty(int(s.sum()), dtype=torch.int32, device=dev)
        e.request_copy(q)
        reqs.append(torch.split(q, s.tolist()))
    recv_req = [torch.cat([reqs[r][o] for r in range(R)]) for o in range(R)]
    rows_out = []
    for o in range(R):
        n = recv_req[o].numel()
        out = torch.empty(n * W, dtype=torch.float32, device=dev)
        engines[o].serve(recv_req[o], n, out)
        rows_out.append(torch.split(out, [int(sends[r][o]) * W for r in range(R)]))
    grads = []
    for r in range(R):
        rows_in = torch.cat([rows_out[o][r] for o in range(R)])
        g = torch.empty(int(sends[r].sum()) * W, dtype=torch.float32, device=dev)
        engines[r].local_grad(batches[r], rows_in, g)
        grads.append(torch.split(g, [int(c) * W for c in sends[r]]))
    gm = sum(int(b.n_rows) for b in batches)
    for o in range(R):
        gin = torch.cat([grads[r][o] for r in range(R)])
        engines[o].apply(recv_req[o], gin, recv_req[o].numel(), t, step_size, reg, gm)
    torch.cuda.synchronize()
    return sum(e.last_loss()[0] for e in engines)


@pytest.mark.parametrize("R,k", [(1, 8), (2, 16), (3, 5), (4, 32)])
def test_hip_shard_phases_match_single_table(gpu, R, k):
    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.distributed import HipShardEngine

    F = 503
    _, ids, w, V = make_problem(3, 1, F, k, 1)
    engines = [HipShardEngine(F, k, r, R) for r in range(R)]
    for e in engines:
        e.load_tables(ids, w, V)
    model = R_.Model.empty(F, k)
    model.load(ids, w, V)
    for t in range(1, 4):
        parts = [make_problem(100 * t + r, 120 + 17 * r, F, k, 9, hot=11)[0] for r in range(R)]
        bs = [e.batch(CSRHost(p.row_ptr, p.col, p.val, p.label)) for e, p in zip(engines, parts)]
        loss = _simulated_step(engines, bs, t, 0.3, 1e-4)
        ref = R_.sgd_step_fast(model, _concat(parts), t, 0.3, 1e-4)
        assert loss == pytest.approx(ref.loss_sum, rel=1e-5)
    gi, gw, gV = zip(*[e.export_tables() for e in engines])
    gi = np.concatenate(gi)
    order = np.argsort(gi)
    np.testing.assert_array_equal(gi[order], np.nonzero(model.present)[0])
    np.testing.assert_allclose(np.concatenate(gw)[order], model.w[gi[order]], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(np.concatenate(gV)[order], model.V[gi[order]], rtol=1e-5, atol=1e-8)


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
        for t in range(1, 4):
            p = make_problem(50 + t, 200, F, k, 8, hot=2)[0]
            o = tr.step(tr.batch(CSRHost(p.row_ptr, p.col, p.val, p.label)), t, 0.2, 1e-5)
            ref = R_.sgd_step_fast(model, p, t, 0.2, 1e-5)
            assert o.loss_sum == pytest.approx(ref.loss_sum, rel=1e-5)
        gi, gw, gV = tr.export_tables()
        np.testing.assert_array_equal(gi, np.nonzero(model.present)[0])
        np.testing.assert_allclose(gw, model.w[gi], rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(gV, model.V[gi], rtol=1e-5, atol=1e-8)
    finally:
        dist.destroy_process_group()
