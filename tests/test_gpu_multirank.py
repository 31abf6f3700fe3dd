"""GPU, two processes on the one GPU of the box: the sharded and replicated trainers with their
real HIP engines (one fm_ctx per process, side-stream prefetch of the next batch), the collectives
staged through host memory over gloo (RCCL cannot put two ranks on one device).  The result equals
the single-table oracle step over the ranks' batches concatenated in rank order."""

import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
F, K, WORLD, STEPS = 401, 16, 2, 4


class HostStagedComm:
    """all_to_all_single / all_reduce on device tensors through gloo: device -> host on the
    current stream, the gloo collective, host -> device on the current stream."""

    def __init__(self, dist):
        self.dist = dist

    def all_to_all_single(self, out, inp, output_split_sizes=None, input_split_sizes=None, group=None):
        o = out.cpu()
        self.dist.all_to_all_single(o, inp.cpu(), output_split_sizes=output_split_sizes,
                                    input_split_sizes=input_split_sizes, group=group)
        out.copy_(o)

    def all_reduce(self, t, group=None, op=None):
        h = t.cpu()
        self.dist.all_reduce(h, group=group)
        t.copy_(h)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem(rank, step):
    from problems import make_problem

    return make_problem(700 * rank + step, 150 + 31 * rank, F, K, 10, hot=9)[0]


def _worker(rank, world, port, outdir, mode):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.distributed import ReplicatedTrainer, ShardedTrainer
    from problems import make_problem

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, ids, w, V = make_problem(77, 1, F, K, 1)
        cls = ShardedTrainer if mode == "sharded" else ReplicatedTrainer
        tr = cls(F, K, rank=rank, world=world, comm=HostStagedComm(dist))
        tr.load_tables(ids, w, V)
        bs = []
        for t in range(1, STEPS + 1):
            p = _problem(rank, t)
            bs.append(tr.batch(CSRHost(p.row_ptr, p.col, p.val, p.label)))
        losses = []
        for t in range(1, STEPS + 1):
            kw = {"prefetch": bs[t]} if mode == "sharded" and t < STEPS else {}
            losses.append(tr.step(bs[t - 1], t, 0.3, 1e-4, **kw).loss_sum)
        gi, gw, gV = tr.export_tables()
        np.savez(os.path.join(outdir, f"r{rank}.npz"), ids=gi, w=gw, V=gV, losses=np.array(losses))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["sharded", "replicated"])
def test_two_processes_hip_engines(gpu, tmp_path, mode):
    from oracle import fm_ref as R
    from problems import make_problem

    mp.spawn(_worker, args=(WORLD, _free_port(), str(tmp_path), mode), nprocs=WORLD, join=True)
    _, ids, w, V = make_problem(77, 1, F, K, 1)
    model = R.Model.empty(F, K)
    model.load(ids, w, V)
    ref = []
    for t in range(1, STEPS + 1):
        parts = [_problem(r, t) for r in range(WORLD)]
        rp, off = [np.zeros(1, np.int64)], 0
        for p in parts:
            rp.append(p.row_ptr[1:] + off)
            off += p.nnz
        cat = R.CSR(np.concatenate(rp), np.concatenate([p.col for p in parts]),
                    np.concatenate([p.val for p in parts]), np.concatenate([p.label for p in parts]))
        ref.append(R.sgd_step_fast(model, cat, t, 0.3, 1e-4).loss_sum)
    outs = [np.load(tmp_path / f"r{r}.npz") for r in range(WORLD)]
    for d in outs:
        np.testing.assert_allclose(d["losses"], ref, rtol=1e-5)
    if mode == "replicated":
        gi, gw, gV = outs[0]["ids"], outs[0]["w"], outs[0]["V"]
        for d in outs[1:]:  # replicas stay bitwise identical
            assert np.array_equal(d["w"], gw) and np.array_equal(d["V"], gV)
    else:
        gi = np.concatenate([d["ids"] for d in outs])
        order = np.argsort(gi)
        gi = gi[order]
        gw = np.concatenate([d["w"] for d in outs])[order]
        gV = np.concatenate([d["V"] for d in outs])[order]
    np.testing.assert_array_equal(gi, np.nonzero(model.present)[0])
    np.testing.assert_allclose(gw, model.w[gi], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(gV, model.V[gi], rtol=1e-5, atol=1e-8)
