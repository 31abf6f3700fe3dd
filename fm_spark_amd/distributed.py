"""Row-sharded multi-GPU FM SGD step: one process per GPU, RCCL all-to-all over xGMI.

The reference shards its model implicitly: every join / groupBy on featureId shuffles the
exploded entries and the model Datasets by feature hash (SURVEY §2b, S1/S2/S5/S6:
FactorizationMachinesModel.scala:155-164, FactorizationMachinesSGD.scala:148-166).  Here the
table is row-sharded by ``owner = id % R`` (slot ``id // R``) across R ranks and one SGD
iteration is four phases of the C-ABI (include/fm_hip.h, fm_shard_*) joined by three
all-to-alls:

    plan (requester)  -> a2a request ids -> serve (owner) -> a2a rows back ->
    local_grad (requester) -> a2a gradients -> apply (owner: rank-ordered sums, update, L1)

Every rank steps its own mini-batch; the iteration's miniBatchSize is the sum over ranks
(weak scaling: the global batch grows with R).  The result equals one single-table step over
the ranks' batches concatenated in rank order, up to fp summation order (owners sum the <= R
partials per feature in rank order, so the result is deterministic for a given R).
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N
from .engine import DeviceBatch, FMContext, StepOut


class HipShardEngine:
    """The HIP phase functions of one rank (its own fm_ctx with shard_index = rank)."""

    def __init__(self, num_features: int, k: int, rank: int, world: int, *, device: int = 0, seed: int = 0,
                 init_sd: float = 0.01, w0: float = 0.0):
        import torch

        self.torch = torch
        self.device = torch.device("cuda", device)
        self.ctx = FMContext(num_features, k, device=device, seed=seed, init_sd=init_sd, w0=w0, shard_index=rank,
                             shard_count=world)
        # launch on torch's stream so the C-ABI kernels and the collectives are stream-ordered
        self.ctx.set_stream(torch.cuda.current_stream(self.device).cuda_stream)
        self.kp = (k + 3) // 4 * 4
        self.width = self.kp + 4
        self._lib = N.load()

    def batch(self, csr: N.CSRHost) -> DeviceBatch:
        return self.ctx.batch(csr)

    def plan(self, b: DeviceBatch) -> np.ndarray:
        R = self.ctx.shard_count
        counts = np.zeros(R, dtype=np.int64)
        N.check(self._lib.fm_shard_plan(self.ctx.handle, b.handle, N.ptr(counts, C.c_int64)), "fm_shard_plan")
        return counts

    def request_copy(self, dst):
        N.check(self._lib.fm_shard_request_copy(self.ctx.handle, C.c_void_p(dst.data_ptr())), "fm_shard_request_copy")

    def serve(self, req, n: int, rows_out):
        N.check(self._lib.fm_shard_serve_device(self.ctx.handle, C.c_void_p(req.data_ptr()), int(n),
                                                C.c_void_p(rows_out.data_ptr())), "fm_shard_serve_device")

    def local_grad(self, b: DeviceBatch, rows_in, grads_out):
        N.check(self._lib.fm_shard_local_grad_device(self.ctx.handle, b.handle, C.c_void_p(rows_in.data_ptr()),
                                                     C.c_void_p(grads_out.data_ptr())), "fm_shard_local_grad_device")

    def apply(self, req, grads, n: int, t: int, step_size: float, reg_param: float, global_rows: int) -> int:
        return N.check(self._lib.fm_shard_apply_device(self.ctx.handle, C.c_void_p(req.data_ptr()),
                                                       C.c_void_p(grads.data_ptr()), int(n), int(t),
                                                       float(step_size), float(reg_param), int(global_rows)),
                       "fm_shard_apply_device")

    def last_loss(self):
        loss = C.c_double()
        nl = C.c_int64()
        N.check(self._lib.fm_shard_last_loss(self.ctx.handle, C.byref(loss), C.byref(nl)), "fm_shard_last_loss")
        return loss.value, nl.value

    def init_random_range(self, begin: int, end: int):
        self.ctx.init_random_range(begin, end)

    def load_tables(self, ids, w, V):
        self.ctx.load_tables(ids, w, V)

    def export_tables(self):
        return self.ctx.export_tables()


class ShardedTrainer:
    """Drives one rank of the sharded step.  ``engine`` supplies the phase functions (HIP on a
    GPU); ``group`` is the torch.distributed process group (nccl = RCCL on ROCm)."""

    def __init__(self, num_features: int, k: int, *, rank: int, world: int, device: int = 0, seed: int = 0,
                 init_sd: float = 0.01, w0: float = 0.0, group=None, engine=None):
        import torch
        import torch.distributed as dist

        self.torch = torch
        self.dist = dist
        self.rank, self.world = rank, world
        self.group = group
        self.engine = engine if engine is not None else HipShardEngine(
            num_features, k, rank, world, device=device, seed=seed, init_sd=init_sd, w0=w0)
        self.device = self.engine.device
        self._global_rows = {}

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
        """miniBatchSize of the iteration: the sum of every rank's rows (cached per batch)."""
        key = id(b)
        if key not in self._global_rows:
            t = self.torch.tensor([int(b.n_rows)], dtype=self.torch.int64, device=self.device)
            self.dist.all_reduce(t, group=self.group)
            self._global_rows[key] = int(t.item())
        return self._global_rows[key]

    def _a2a(self, out, inp, out_splits, in_splits):
        self.dist.all_to_all_single(out, inp, output_split_sizes=[int(x) for x in out_splits],
                                    input_split_sizes=[int(x) for x in in_splits], group=self.group)

    def step(self, b, t: int, step_size: float, reg_param: float, sync: bool = True) -> StepOut | None:
        torch = self.torch
        gm = self.global_rows(b)
        if gm == 0:  # SGD.scala:126-128: every rank skips together
            return StepOut(0.0, 0, 0, 0, executed=False)
        W = self.engine.width
        send = self.engine.plan(b)
        send_t = torch.tensor(send, dtype=torch.int64, device=self.device)
        recv_t = torch.empty_like(send_t)
        self.dist.all_to_all_single(recv_t, send_t, group=self.group)
        recv = recv_t.cpu().numpy()
        U, n_recv = int(send.sum()), int(recv.sum())
        req_send = torch.empty(max(U, 1), dtype=torch.int32, device=self.device)[:U]
        self.engine.request_copy(req_send)
        req_recv = torch.empty(max(n_recv, 1), dtype=torch.int32, device=self.device)[:n_recv]
        self._a2a(req_recv, req_send, recv, send)
        rows_out = torch.empty(max(n_recv, 1) * W, dtype=torch.float32, device=self.device)[: n_recv * W]
        self.engine.serve(req_recv, n_recv, rows_out)
        rows_in = torch.empty(max(U, 1) * W, dtype=torch.float32, device=self.device)[: U * W]
        self._a2a(rows_in, rows_out, send * W, recv * W)
        grads_out = torch.empty(max(U, 1) * W, dtype=torch.float32, device=self.device)[: U * W]
        self.engine.local_grad(b, rows_in, grads_out)
        grads_in = torch.empty(max(n_recv, 1) * W, dtype=torch.float32, device=self.device)[: n_recv * W]
        self._a2a(grads_in, grads_out, recv * W, send * W)
        self.engine.apply(req_recv, grads_in, n_recv, t, step_size, reg_param, gm)
        if not sync:
            return None
        loss, nl = self.engine.last_loss()
        tot = torch.tensor([loss, float(nl), float(U)], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(tot, group=self.group)
        return StepOut(float(tot[0]), gm, int(tot[1]), U)
