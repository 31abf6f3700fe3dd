"""CPU, world_size 2 over gloo: the replicated step (grad -> all-reduce -> apply) and the
sharded step's exchange protocol
(fm_spark_amd.distributed.ShardedTrainer: route -> a2a entries -> owner_forward -> a2a partials ->
combine -> a2a S -> owner_update) with the NumPy phase engine equals one single-table oracle step over the ranks'
batches concatenated in rank order."""

import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
F, K, WORLD = 211, 5, 2
STEPS = 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem_for(rank, step):
    from problems import make_problem

    return make_problem(1000 * rank + step, 60 + 13 * rank, F, K, 6, hot=7)[0]


def _worker(rank, world, port, outdir, mode="sharded"):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from fm_spark_amd.distributed import ReplicatedTrainer, ShardedTrainer
    from problems import make_problem
    from shard_ref_engine import NumpyReplEngine, NumpyShardEngine

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, ids, w, V = make_problem(5, 1, F, K, 1)
        if mode == "sharded":
            tr = ShardedTrainer(F, K, rank=rank, world=world, engine=NumpyShardEngine(F, K, rank, world))
        else:
            tr = ReplicatedTrainer(F, K, rank=rank, world=world, engine=NumpyReplEngine(F, K))
        tr.load_tables(ids, w, V)
        losses = []
        bs = [tr.batch(_problem_for(rank, t)) for t in range(1, STEPS + 1)]
        for t in range(1, STEPS + 1):
            # sharded: from step 2 on, the next batch's route / entry exchange / owner preparation
            # is prefetched behind the current update (the bench's schedule)
            kw = {"prefetch": bs[t]} if mode == "sharded" and 2 <= t < STEPS else {}
            o = tr.step(bs[t - 1], t, 0.4, 1e-3, **kw)
            losses.append(o.loss_sum)
        gi, gw, gV = tr.export_tables()
        np.savez(os.path.join(outdir, f"r{rank}.npz"), ids=gi, w=gw, V=gV, losses=np.array(losses))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["sharded", "replicated"])
def test_two_ranks_match_single_table(tmp_path, mode):
    from oracle import fm_ref as R
    from problems import make_problem

    port = _free_port()
    mp.spawn(_worker, args=(WORLD, port, str(tmp_path), mode), nprocs=WORLD, join=True)
    _, ids, w, V = make_problem(5, 1, F, K, 1)
    model = R.Model.empty(F, K)
    model.load(ids, w, V)
    ref_losses = []
    for t in range(1, STEPS + 1):
        parts = [_problem_for(r, t) for r in range(WORLD)]
        row_ptr = [np.zeros(1, np.int64)]
        off = 0
        for p in parts:
            row_ptr.append(p.row_ptr[1:] + off)
            off += p.nnz
        cat = R.CSR(np.concatenate(row_ptr), np.concatenate([p.col for p in parts]),
                    np.concatenate([p.val for p in parts]), np.concatenate([p.label for p in parts]))
        ref_losses.append(R.sgd_step_fast(model, cat, t, 0.4, 1e-3).loss_sum)
    gids, gw, gV = [], [], []
    if mode == "replicated":  # every rank holds the whole table: compare rank 0's, then rank 1 == rank 0
        d0, d1 = (np.load(tmp_path / f"r{r}.npz") for r in range(WORLD))
        np.testing.assert_array_equal(d0["ids"], d1["ids"])
        np.testing.assert_array_equal(d0["w"], d1["w"])
        np.testing.assert_array_equal(d0["V"], d1["V"])
        np.testing.assert_allclose(d0["losses"], ref_losses, rtol=1e-6)
        np.testing.assert_array_equal(d0["ids"], np.nonzero(model.present)[0])
        np.testing.assert_allclose(d0["w"], model.w[d0["ids"]], rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(d0["V"], model.V[d0["ids"]], rtol=1e-6, atol=1e-9)
        return
    for r in range(WORLD):
        d = np.load(tmp_path / f"r{r}.npz")
        gids.append(d["ids"])
        gw.append(d["w"])
        gV.append(d["V"])
        np.testing.assert_allclose(d["losses"], ref_losses, rtol=1e-6)
    gids = np.concatenate(gids)
    order = np.argsort(gids)
    np.testing.assert_array_equal(gids[order], np.nonzero(model.present)[0])
    # fp32 wire for rows and gradients: 1e-6 relative
    np.testing.assert_allclose(np.concatenate(gw)[order], model.w[gids[order]], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(np.concatenate(gV)[order], model.V[gids[order]], rtol=1e-6, atol=1e-9)
