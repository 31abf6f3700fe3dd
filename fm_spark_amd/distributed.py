"""Row-sharded multi-GPU FM SGD step, owner-computes: one process per GPU, RCCL all-to-all
over xGMI.

The reference shards its model implicitly: every join / groupBy on featureId shuffles the
exploded entries and the model Datasets by feature hash (SURVEY §2b, S1/S2/S5/S6:
FactorizationMachinesModel.scala:155-164, FactorizationMachinesSGD.scala:148-166).  Here the
table is row-sharded by ``owner = id % R`` (slot ``id // R``) across R ranks and the work
moves to the rows instead of the rows to the work.  One SGD iteration is five phases of the
C-ABI (include/fm_hip.h, fm_shard_*) joined by three all-to-alls:

    route (requester: entries by owner) -> a2a entries -> owner_prepare (pair table, slot
    sort)  ||  owner_forward (partial sums per (sample, owner) pair) -> a2a partials back ->
    combine (requester: S, yhat, loss) -> a2a S to the owners -> owner_update (per-slot
    gradient sums, update + L1)

The first two phases depend on the batch alone: ``ShardedTrainer.step(b, ..., prefetch=next)``
issues them for the next batch right after the current iteration's update, on the side stream,
so the next routing, entry exchange and slot sort overlap the current update.

Every rank steps its own mini-batch; the iteration's miniBatchSize is the sum over ranks
(weak scaling: the global batch grows with R).  The result equals one single-table step over
the ranks' batches concatenated in rank order, up to fp summation order (deterministic for a
given R).  Only entries (12 B) and twice kp + 2 words per (sample, owner) pair cross xGMI
-- no table row or per-id gradient does.
"""

from __future__ import annotations

import contextlib
import ctypes as C

import numpy as np

from . import _native as N
from .engine import FMContext, StepOut


class HipShardEngine:
    """The HIP phase functions of one rank (its own fm_ctx with shard_index = rank)."""

    def __init__(self, num_features: int, k: int, rank: int, world: int, *, device: int = 0, seed: int = 0,
                 init_sd: float = 0.01, w0: float = 0.0):
        import torch

        self.torch = torch
        self.device = torch.device("cuda", device)
        self.R = world
        self.ctx = FMContext(num_features, k, device=device, seed=seed, init_sd=init_sd, w0=w0, shard_index=rank,
                             shard_count=world)
        # launch on torch's streams so the C-ABI kernels and the collectives are stream-ordered:
        # the iteration on the current stream, batch-only preparation on a side stream
        self.main_stream = torch.cuda.current_stream(self.device)
        self.side_stream = torch.cuda.Stream(self.device)
        self.ctx.set_stream(self.main_stream.cuda_stream)
        self._lib = N.load()
        N.check(self._lib.fm_set_side_stream(self.ctx.handle, C.c_void_p(self.side_stream.cuda_stream)),
                "fm_set_side_stream")
        self.kp = (k + 3) // 4 * 4
        self.width = self.kp + 2  # fp32 words per pair on the wire: [P][kp] vectors, then [P][2] scalars

    def _empty(self, n, dtype):
        return self.torch.empty(max(int(n), 1), dtype=dtype, device=self.device)[: int(n)]

    @staticmethod
    def _ptr(t):
        return C.c_void_p(t.data_ptr() if t.numel() else 0)

    def side(self):
        """Context for the batch-only phases and their exchange (torch's current stream = side)."""
        return self.torch.cuda.stream(self.side_stream)

    def batch(self, csr: N.CSRHost):
        return self.ctx.batch(csr)

    def route(self, b):
        torch = self.torch
        n = int(b.nnz)
        send_slot = self._empty(n, torch.int32)
        send_ent = self._empty(2 * n, torch.int32)
        counts = np.zeros(2 * self.R, dtype=np.int64)
        N.check(self._lib.fm_shard_route(self.ctx.handle, b.handle, self._ptr(send_slot), self._ptr(send_ent),
                                         N.ptr(counts, C.c_int64)), "fm_shard_route")
        return send_slot, send_ent, counts

    def owner_prepare(self, b, recv_slot, recv_ent, src_entries, src_pairs):
        se = np.ascontiguousarray(src_entries, dtype=np.int64)
        sp = np.ascontiguousarray(src_pairs, dtype=np.int64)
        N.check(self._lib.fm_shard_owner_prepare(self.ctx.handle, b.handle, self._ptr(recv_slot), self._ptr(recv_ent),
                                                 int(recv_slot.numel()), N.ptr(se, C.c_int64), N.ptr(sp, C.c_int64)),
                "fm_shard_owner_prepare")

    def owner_forward(self, b, n_pairs_in: int):
        out = self._empty(int(n_pairs_in) * self.width, self.torch.float32)
        N.check(self._lib.fm_shard_owner_forward(self.ctx.handle, b.handle, self._ptr(out)), "fm_shard_owner_forward")
        return out

    def combine(self, b, partials_in, n_pairs_out: int):
        s_send = self._empty(int(n_pairs_out) * self.width, self.torch.float32)
        N.check(self._lib.fm_shard_combine(self.ctx.handle, b.handle, self._ptr(partials_in), self._ptr(s_send)),
                "fm_shard_combine")
        return s_send

    def owner_update(self, b, s_recv, t: int, step_size: float, reg_param: float, global_rows: int) -> int:
        return N.check(self._lib.fm_shard_owner_update(self.ctx.handle, b.handle, self._ptr(s_recv), int(t),
                                                       float(step_size), float(reg_param), int(global_rows)),
                       "fm_shard_owner_update")

    def retire(self, tensors):
        """Tensors allocated on the side stream and read by the main stream: keep their memory
        from being reused before the main stream's reads are done."""
        for t in tensors:
            if t.numel():
                t.record_stream(self.main_stream)

    def last_stats(self):
        """(loss_sum, n_loss_rows) of this rank's samples, distinct ids this rank owns."""
        loss, nl, nu = C.c_double(), C.c_int64(), C.c_int64()
        N.check(self._lib.fm_last_stats(self.ctx.handle, C.byref(loss), C.byref(nl), C.byref(nu)), "fm_last_stats")
        return loss.value, nl.value, nu.value

    def init_random_range(self, begin: int, end: int):
        self.ctx.init_random_range(begin, end)

    def load_tables(self, ids, w, V):
        self.ctx.load_tables(ids, w, V)

    def export_tables(self):
        return self.ctx.export_tables()


def _global_rows(trainer, b) -> int:
    """The all-reduced row count of b's iteration, kept on b until its step consumes it."""
    gm = getattr(b, "_fm_global_rows", None)
    if gm is None:
        t = trainer.torch.tensor([int(b.n_rows)], dtype=trainer.torch.int64, device=trainer.device)
        trainer.dist.all_reduce(t, group=trainer.group)
        gm = int(t.item())
        b._fm_global_rows = gm
    return gm


class _Plan:
    """One batch's exchange plan: what the batch-only phases produced (counts per peer and the
    received entries, which the owner phases read until the iteration's forward is done)."""

    __slots__ = ("ent_in", "ent_out", "pair_in", "pair_out", "keep")

    def __init__(self, ent_in, ent_out, pair_in, pair_out, keep):
        self.ent_in, self.ent_out, self.pair_in, self.pair_out, self.keep = ent_in, ent_out, pair_in, pair_out, keep


class ShardedTrainer:
    """Drives one rank of the sharded step.  ``engine`` supplies the phase functions (HIP on a
    GPU); ``group`` is the torch.distributed process group (nccl = RCCL on ROCm); ``comm`` the
    module the collectives go through (torch.distributed unless a test stages them)."""

    def __init__(self, num_features: int, k: int, *, rank: int, world: int, device: int = 0, seed: int = 0,
                 init_sd: float = 0.01, w0: float = 0.0, group=None, engine=None, comm=None):
        import torch
        import torch.distributed as dist

        self.torch = torch
        self.dist = comm if comm is not None else dist
        self.rank, self.world = rank, world
        self.group = group
        self.engine = engine if engine is not None else HipShardEngine(
            num_features, k, rank, world, device=device, seed=seed, init_sd=init_sd, w0=w0)
        self.device = self.engine.device

    # convenience passthroughs -------------------------------------------------------
    @property
    def ctx(self):
        return getattr(self.engine, "ctx", None)

    def batch(self, csr):
        return self.engine.batch(csr)

    def init_random_range(self, begin, end):
        self.engine.init_random_range(begin, end)

    def load_tables(self, ids, w, V):
        self.engine.load_tables(ids, w, V)

    def export_tables(self):
        return self.engine.export_tables()

    # ------------------------------------------------------------------------------
    def global_rows(self, b) -> int:
        """miniBatchSize of the iteration: the sum of every rank's rows.  Cached on the batch object
        itself until its step consumes it (a cache keyed by id(b) could hand a recycled id a stale
        count, and the ranks would then disagree on whether to enter the collective)."""
        return _global_rows(self, b)

    def _a2a(self, out, inp, out_splits, in_splits):
        self.dist.all_to_all_single(out, inp, output_split_sizes=[int(x) for x in out_splits],
                                    input_split_sizes=[int(x) for x in in_splits], group=self.group)

    def _empty(self, n, dtype):
        return self.torch.empty(max(int(n), 1), dtype=dtype, device=self.device)[: int(n)]

    def _a2a_pairs(self, out, inp, out_pairs, in_pairs):
        """All-to-all of a pair buffer in the wire layout (include/fm_hip.h): the [P][kp] vector section,
        then the [P][2] scalar section, each exchanged with its own splits."""
        kp = self.engine.kp
        po, pi = int(np.sum(out_pairs)), int(np.sum(in_pairs))
        self._a2a(out[: po * kp], inp[: pi * kp], out_pairs * kp, in_pairs * kp)
        self._a2a(out[po * kp:], inp[pi * kp:], out_pairs * 2, in_pairs * 2)

    def _side(self):
        side = getattr(self.engine, "side", None)
        return side() if side is not None else contextlib.nullcontext()

    def prefetch(self, b) -> None:
        """The batch-only phases of b's iteration (route, entry exchange, owner pair table and slot
        sort), enqueued on the side stream.  Every rank must prefetch the same iterations in the
        same order (the exchange is collective).  Idempotent until b's step consumes it."""
        if getattr(b, "_fm_plan", None) is not None:
            return
        torch, R = self.torch, self.world
        with self._side():
            send_slot, send_ent, counts = self.engine.route(b)
            ent_out, pair_out = counts[:R], counts[R:]
            cnt = torch.tensor(np.stack([ent_out, pair_out], axis=1).reshape(-1), dtype=torch.int64,
                               device=self.device)
            rcnt = torch.empty_like(cnt)
            self.dist.all_to_all_single(rcnt, cnt, group=self.group)
            rc = rcnt.cpu().numpy().reshape(R, 2)
            ent_in, pair_in = rc[:, 0], rc[:, 1]
            recv_slot = self._empty(ent_in.sum(), torch.int32)
            self._a2a(recv_slot, send_slot, ent_in, ent_out)
            recv_ent = self._empty(2 * ent_in.sum(), torch.int32)
            self._a2a(recv_ent, send_ent, 2 * ent_in, 2 * ent_out)
            self.engine.owner_prepare(b, recv_slot, recv_ent, ent_in, pair_in)
        b._fm_plan = _Plan(ent_in, ent_out, pair_in, pair_out, (recv_slot, recv_ent))

    def step(self, b, t: int, step_size: float, reg_param: float, sync: bool = True, prefetch=None) -> StepOut | None:
        """One iteration on this rank's batch b.  ``prefetch``: the batch of the next iteration,
        whose batch-only phases are then enqueued behind this iteration's update (collective:
        pass the same schedule on every rank)."""
        W = self.engine.width
        gm = self.global_rows(b)
        b._fm_global_rows = None  # consumed: a later step of the same batch re-counts
        if gm == 0:  # SGD.scala:126-128: every rank skips together
            self._drop_plan(b)
            if prefetch is not None:
                self.prefetch(prefetch)
            return StepOut(0.0, 0, 0, 0, executed=False)
        self.prefetch(b)  # no-op when an earlier step already did
        plan, b._fm_plan = b._fm_plan, None
        partials = self.engine.owner_forward(b, int(plan.pair_in.sum()))
        part_in = self._empty(plan.pair_out.sum() * W, self.torch.float32)
        self._a2a_pairs(part_in, partials, plan.pair_out, plan.pair_in)
        s_send = self.engine.combine(b, part_in, int(plan.pair_out.sum()))
        s_recv = self._empty(plan.pair_in.sum() * W, self.torch.float32)
        self._a2a_pairs(s_recv, s_send, plan.pair_in, plan.pair_out)
        self.engine.owner_update(b, s_recv, t, step_size, reg_param, gm)
        self._retire(plan)
        if prefetch is not None:
            self.prefetch(prefetch)
        if not sync:
            return None
        loss, nl, U = self.engine.last_stats()
        tot = self.torch.tensor([loss, float(nl), float(U)], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(tot, group=self.group)
        return StepOut(float(tot[0]), gm, int(tot[1]), int(tot[2]))

    def _retire(self, plan):
        retire = getattr(self.engine, "retire", None)
        if retire is not None:
            retire(plan.keep)
        plan.keep = None

    def _drop_plan(self, b):
        plan = getattr(b, "_fm_plan", None)
        b._fm_plan = None
        if plan is not None:
            self._retire(plan)


# ------------------------------------------------------------------------------ replicated
class HipReplEngine:
    """The whole table on every rank (small feature spaces, BASELINE config c2): the phase
    functions fm_repl_grad / fm_repl_apply of include/fm_hip.h."""

    def __init__(self, num_features: int, k: int, *, device: int = 0, seed: int = 0, init_sd: float = 0.01,
                 w0: float = 0.0):
        import torch

        self.torch = torch
        self.device = torch.device("cuda", device)
        self.ctx = FMContext(num_features, k, device=device, seed=seed, init_sd=init_sd, w0=w0)
        self.ctx.set_stream(torch.cuda.current_stream(self.device).cuda_stream)
        self.kp = (k + 3) // 4 * 4
        self.width = self.kp + 4
        self.grad = torch.empty(num_features * self.width, dtype=torch.float32, device=self.device)
        self._lib = N.load()

    def batch(self, csr: N.CSRHost):
        return self.ctx.batch(csr)

    def grad_phase(self, b):
        N.check(self._lib.fm_repl_grad(self.ctx.handle, b.handle, C.c_void_p(self.grad.data_ptr())), "fm_repl_grad")
        return self.grad

    def apply(self, grad, t: int, step_size: float, reg_param: float, global_rows: int) -> int:
        return N.check(self._lib.fm_repl_apply(self.ctx.handle, C.c_void_p(grad.data_ptr()), int(t),
                                               float(step_size), float(reg_param), int(global_rows)),
                       "fm_repl_apply")

    def last_stats(self):
        loss, nl, nu = C.c_double(), C.c_int64(), C.c_int64()
        N.check(self._lib.fm_last_stats(self.ctx.handle, C.byref(loss), C.byref(nl), C.byref(nu)), "fm_last_stats")
        return loss.value, nl.value, nu.value

    def init_random_range(self, begin: int, end: int):
        self.ctx.init_random_range(begin, end)

    def load_tables(self, ids, w, V):
        self.ctx.load_tables(ids, w, V)

    def export_tables(self):
        return self.ctx.export_tables()


class ReplicatedTrainer:
    """Data-parallel step with the table replicated on every rank: local gradient sums into a
    dense [F][kp + 4] fp32 buffer, one RCCL all-reduce (sum), the identical update everywhere.
    For small tables (c2: 1M features x k = 8 -> 48 MB per all-reduce); larger feature spaces
    use ShardedTrainer.  Equals the single-table step over the ranks' batches concatenated,
    up to fp summation order."""

    def __init__(self, num_features: int, k: int, *, rank: int, world: int, device: int = 0, seed: int = 0,
                 init_sd: float = 0.01, w0: float = 0.0, group=None, engine=None, comm=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, comm if comm is not None else dist
        self.rank, self.world, self.group = rank, world, group
        self.engine = engine if engine is not None else HipReplEngine(
            num_features, k, device=device, seed=seed, init_sd=init_sd, w0=w0)
        self.device = self.engine.device

    @property
    def ctx(self):
        return getattr(self.engine, "ctx", None)

    def batch(self, csr):
        return self.engine.batch(csr)

    def init_random_range(self, begin, end):
        self.engine.init_random_range(begin, end)

    def load_tables(self, ids, w, V):
        self.engine.load_tables(ids, w, V)

    def export_tables(self):
        return self.engine.export_tables()

    def global_rows(self, b) -> int:
        return _global_rows(self, b)

    def step(self, b, t: int, step_size: float, reg_param: float, sync: bool = True) -> StepOut | None:
        gm = self.global_rows(b)
        b._fm_global_rows = None
        if gm == 0:  # SGD.scala:126-128
            return StepOut(0.0, 0, 0, 0, executed=False)
        g = self.engine.grad_phase(b)
        self.dist.all_reduce(g, group=self.group)
        self.engine.apply(g, t, step_size, reg_param, gm)
        if not sync:
            return None
        loss, nl, U = self.engine.last_stats()
        tot = self.torch.tensor([loss, float(nl)], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(tot, group=self.group)
        return StepOut(float(tot[0]), gm, int(tot[1]), int(U))
