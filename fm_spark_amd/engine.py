"""Pythonic handle over one fm_ctx (one device's FM tables) — thin, no arithmetic.

Every method calls straight through the C-ABI of include/fm_hip.h; errors raise FMError.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native as N


@dataclass
class StepOut:
    loss_sum: float
    n_rows: int
    n_loss_rows: int
    n_unique: int
    executed: bool = True


class DeviceBatch:
    """A CSR mini-batch resident in HBM (fm_batch_create)."""

    def __init__(self, ctx: "FMContext", csr: N.CSRHost | None):
        self._lib = N.load()
        self.ctx = ctx
        h = C.c_void_p()
        self.handle = h
        self.n_rows = self.nnz = 0
        if csr is not None:
            N.check(self._lib.fm_batch_create(ctx.handle, C.byref(csr.c), C.byref(h)), "fm_batch_create")
            self.n_rows = csr.n_rows
            self.nnz = csr.nnz

    def select_rows(self, data: "DeviceBatch", rows):
        """Refill this batch with rows[i] of the resident dataset `data`, on the device
        (fm_batch_from_rows); returns self."""
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        h = self.handle if self.handle else C.c_void_p()
        N.check(self._lib.fm_batch_from_rows(self.ctx.handle, data.handle, N.ptr(rows, C.c_int64), len(rows),
                                             C.byref(h)), "fm_batch_from_rows")
        self.handle = h
        self.n_rows = len(rows)
        self.nnz = int(self._lib.fm_batch_nnz(h))
        self._data = data  # the dataset stays alive while this batch's gather may be queued
        return self

    def view_split(self, data: "DeviceBatch", split: int):
        """Re-point this batch at split `split` of the split-ordered dataset `data`
        (fm_batch_split_view: no copy, no device work); returns self."""
        h = self.handle if self.handle else C.c_void_p()
        N.check(self._lib.fm_batch_split_view(self.ctx.handle, data.handle, int(split), C.byref(h)),
                "fm_batch_split_view")
        self.handle = h
        self.n_rows = int(self._lib.fm_batch_rows(h))
        self.nnz = int(self._lib.fm_batch_nnz(h))
        self._data = data  # the dataset outlives the view (its rows are borrowed)
        return self

    def prepare(self):
        """Sort this batch by feature on the side stream ahead of its step (fm_batch_prepare)."""
        N.check(self._lib.fm_batch_prepare(self.ctx.handle, self.handle), "fm_batch_prepare")

    def close(self):
        if self.handle:
            self._lib.fm_batch_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id() -> bytes:
    """RCCL unique id (128 bytes) that process 0 of a multi-process job hands to the others
    (fm_comm_unique_id)."""
    lib = N.load()
    buf = (C.c_uint8 * 128)()
    N.check(lib.fm_comm_unique_id(buf), "fm_comm_unique_id")
    return bytes(buf)


class FMContext:
    """One fm_ctx.  ``parallel`` = "sharded" / "replicated": the context drives ``n_gpus`` local
    ranks on ``devices`` (default device, device + 1, ...) of a job of ``n_procs`` processes and runs
    the multi-GPU step itself (include/fm_hip.h); ``transport`` "auto" | "rccl" | "copy".
    ``fuse`` None (the library's default: on) | True | False: the fused step for prepared batches
    (fm_config.fuse_single); ``xchg_chunks``: 0 = default (fm_config.xchg_chunks)."""

    _PAR = {None: N.FM_PARALLEL_NONE, "none": N.FM_PARALLEL_NONE, "sharded": N.FM_PARALLEL_SHARDED,
            "replicated": N.FM_PARALLEL_REPLICATED}
    _TR = {"auto": N.FM_TRANSPORT_AUTO, "rccl": N.FM_TRANSPORT_RCCL, "copy": N.FM_TRANSPORT_COPY}

    def __init__(self, num_features: int, k: int, *, device: int = 0, seed: int = 0, init_sd: float = 0.01,
                 w0: float = 0.0, shard_index: int = 0, shard_count: int = 1, parallel: str | None = None,
                 n_gpus: int = 1, devices=None, transport: str = "auto", n_procs: int = 1, proc_rank: int = 0,
                 comm_id: bytes | None = None, fuse: bool | None = None, xchg_chunks: int = 0):
        self._lib = N.load()
        cfg = N.fm_config(num_features=int(num_features), k=int(k), device=int(device), seed=int(seed) & (2**64 - 1),
                          init_sd=float(init_sd), w0=float(w0), shard_index=int(shard_index),
                          shard_count=int(shard_count))
        cfg.parallel = self._PAR[parallel]
        cfg.n_gpus = int(n_gpus)
        devs = list(devices) if devices is not None else [int(device) + i for i in range(int(n_gpus))]
        if cfg.parallel != N.FM_PARALLEL_NONE and len(devs) != n_gpus:
            raise ValueError("devices must list n_gpus devices")
        for i, d in enumerate(devs[: N.FM_MAX_LOCAL]):
            cfg.devices[i] = int(d)
        if cfg.parallel != N.FM_PARALLEL_NONE:
            cfg.device = int(devs[0])
        cfg.transport = self._TR[transport]
        cfg.fuse_single = N.FM_FUSE_DEFAULT if fuse is None else (N.FM_FUSE_ON if fuse else N.FM_FUSE_OFF)
        cfg.xchg_chunks = int(xchg_chunks)
        cfg.n_procs = int(n_procs)
        cfg.proc_rank = int(proc_rank)
        if comm_id is not None:
            if len(comm_id) != 128:
                raise ValueError("comm_id must be 128 bytes")
            for i, b in enumerate(comm_id):
                cfg.comm_id[i] = b
        self.parallel = parallel if parallel not in (None, "none") else None
        self.n_gpus = int(n_gpus)
        h = C.c_void_p()
        N.check(self._lib.fm_create(C.byref(cfg), C.byref(h)), "fm_create")
        self.handle = h
        self.num_features = int(num_features)
        self.k = int(k)
        self.w0 = float(w0)
        self.shard_index = int(shard_index)
        self.shard_count = int(shard_count)

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "handle", None):
            self._lib.fm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr: int | None):
        """Launch on this hipStream_t (an int handle, e.g. torch.cuda.current_stream().cuda_stream);
        0 / None = the device's default (null) stream."""
        N.check(self._lib.fm_set_stream(self.handle, C.c_void_p(stream_ptr or None)), "fm_set_stream")

    def sync(self):
        N.check(self._lib.fm_sync(self.handle), "fm_sync")

    def reserve(self, max_rows: int, max_nnz: int):
        N.check(self._lib.fm_reserve(self.handle, int(max_rows), int(max_nnz)), "fm_reserve")

    # --------------------------------------------------------------------- tables
    def load_tables(self, ids, w, V):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        w = np.ascontiguousarray(w, dtype=np.float64)
        V = np.ascontiguousarray(V, dtype=np.float64).reshape(len(ids), self.k)
        N.check(self._lib.fm_load_tables(self.handle, N.ptr(ids, C.c_int32), len(ids), N.ptr(w, C.c_double),
                                         N.ptr(V, C.c_double)), "fm_load_tables")

    def init_random(self, ids):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        N.check(self._lib.fm_init_random(self.handle, N.ptr(ids, C.c_int32), len(ids)), "fm_init_random")

    def init_random_range(self, begin: int, end: int):
        N.check(self._lib.fm_init_random_range(self.handle, int(begin), int(end)), "fm_init_random_range")

    def init_from_batch(self, b: "DeviceBatch") -> int:
        """createInitialModel over a device-resident dataset (SGD.scala:224-241): the seeded draw for
        every absent id of b's entries, on the device; returns the number of present rows."""
        n = C.c_int64()
        N.check(self._lib.fm_init_from_batch(self.handle, b.handle, C.byref(n)), "fm_init_from_batch")
        return n.value

    def export_tables(self):
        n = C.c_int64()
        N.check(self._lib.fm_export_tables(self.handle, None, None, None, 0, C.byref(n)), "fm_export_tables")
        cnt = n.value
        ids = np.zeros(max(cnt, 1), dtype=np.int32)
        w = np.zeros(max(cnt, 1))
        V = np.zeros((max(cnt, 1), self.k))
        if cnt:
            N.check(self._lib.fm_export_tables(self.handle, N.ptr(ids, C.c_int32), N.ptr(w, C.c_double),
                                               N.ptr(V, C.c_double), cnt, C.byref(n)), "fm_export_tables")
        return ids[:cnt], w[:cnt], V[:cnt]

    def export_rows(self, ids):
        """(w, V, present) of the given ids as they stand now (pending L1 applied), without a
        whole-table export (fm_export_rows)."""
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        n = len(ids)
        w = np.zeros(max(n, 1))
        V = np.zeros((max(n, 1), self.k))
        pres = np.zeros(max(n, 1), dtype=np.int8)
        N.check(self._lib.fm_export_rows(self.handle, N.ptr(ids, C.c_int32), n, N.ptr(w, C.c_double),
                                         N.ptr(V, C.c_double), N.ptr(pres, C.c_int8)), "fm_export_rows")
        return w[:n], V[:n], pres[:n].astype(bool)

    def num_present(self) -> int:
        return N.check(self._lib.fm_num_present(self.handle), "fm_num_present")

    @property
    def epoch(self) -> int:
        return int(self._lib.fm_epoch(self.handle))

    # ------------------------------------------------------------------- stepping
    def batch(self, csr: N.CSRHost) -> DeviceBatch:
        return DeviceBatch(self, csr)

    def batch_splits(self, csr: N.CSRHost, split_rows) -> DeviceBatch:
        """A dataset laid out split after split (fm_batch_create_splits): split s = rows
        [split_rows[s], split_rows[s + 1]) of csr; each split is then stepped in place through
        split_view."""
        sr = np.ascontiguousarray(split_rows, dtype=np.int64)
        b = DeviceBatch(self, None)
        h = C.c_void_p()
        N.check(self._lib.fm_batch_create_splits(self.handle, C.byref(csr.c), len(sr) - 1, N.ptr(sr, C.c_int64),
                                                 C.byref(h)), "fm_batch_create_splits")
        b.handle = h
        b.n_rows, b.nnz = csr.n_rows, csr.nnz
        b.split_rows = sr
        return b

    def split_view(self, data: DeviceBatch, split: int, into: DeviceBatch | None = None) -> DeviceBatch:
        """Split `split` of a dataset made by batch_splits as a mini-batch, in place (fm_batch_split_view);
        `into` (a view of this context) is re-pointed instead of creating one."""
        b = into if into is not None else DeviceBatch(self, None)
        return b.view_split(data, split)

    def batch_from_rows(self, data: DeviceBatch, rows, into: DeviceBatch | None = None) -> DeviceBatch:
        """The mini-batch of rows `rows` of the resident dataset `data`, gathered on the device
        (fm_batch_from_rows); `into` (a batch of this context) is refilled in place instead of
        creating one."""
        b = into if into is not None else DeviceBatch(self, None)
        return b.select_rows(data, rows)

    @property
    def fuse_active(self) -> bool:
        """Whether prepared batches of this context take the fused step (fm_fuse_active)."""
        return int(self._lib.fm_fuse_active(self.handle)) == 1

    def step(self, csr: N.CSRHost, t: int, step_size: float, reg_param: float, sync: bool = True):
        """One iteration from a host CSR.  sync=False only enqueues (the host buffers are free on
        return; losses via loss_history), so consecutive calls overlap upload and compute."""
        if not sync:
            N.check(self._lib.fm_step(self.handle, C.byref(csr.c), int(t), float(step_size), float(reg_param), None),
                    "fm_step")
            return None
        out = N.fm_step_out()
        rc = N.check(self._lib.fm_step(self.handle, C.byref(csr.c), int(t), float(step_size), float(reg_param),
                                       C.byref(out)), "fm_step")
        if rc == N.FM_NOTHING_TO_DO:
            return StepOut(0.0, 0, 0, 0, executed=False)
        return StepOut(out.loss_sum, out.n_rows, out.n_loss_rows, out.n_unique)

    def step_batch(self, b: DeviceBatch, t: int, step_size: float, reg_param: float, sync: bool = True):
        if sync:
            out = N.fm_step_out()
            rc = N.check(self._lib.fm_step_batch(self.handle, b.handle, int(t), float(step_size), float(reg_param),
                                                 C.byref(out)), "fm_step_batch")
            if rc == N.FM_NOTHING_TO_DO:
                return StepOut(0.0, 0, 0, 0, executed=False)
            return StepOut(out.loss_sum, out.n_rows, out.n_loss_rows, out.n_unique)
        N.check(self._lib.fm_step_batch(self.handle, b.handle, int(t), float(step_size), float(reg_param), None),
                "fm_step_batch")
        return None

    def loss_history(self) -> np.ndarray:
        n = C.c_int64()
        N.check(self._lib.fm_loss_history(self.handle, None, 0, C.byref(n)), "fm_loss_history")
        out = np.zeros(max(n.value, 1))
        if n.value:
            N.check(self._lib.fm_loss_history(self.handle, N.ptr(out, C.c_double), n.value, C.byref(n)),
                    "fm_loss_history")
        return out[: n.value]

    # ------------------------------------------------------------------- inference
    def predict(self, csr: N.CSRHost, min_label: float, max_label: float) -> np.ndarray:
        out = np.zeros(max(csr.n_rows, 1))
        N.check(self._lib.fm_predict(self.handle, C.byref(csr.c), float(min_label), float(max_label),
                                     N.ptr(out, C.c_double)), "fm_predict")
        return out[: csr.n_rows]

    def predict_batch(self, b: DeviceBatch, min_label: float, max_label: float) -> np.ndarray:
        out = np.zeros(max(b.n_rows, 1))
        N.check(self._lib.fm_predict_batch(self.handle, b.handle, float(min_label), float(max_label),
                                           N.ptr(out, C.c_double)), "fm_predict_batch")
        return out[: b.n_rows]

    def loss_grad(self, csr: N.CSRHost, initial_sd: float | None = None, seed: int = 0):
        """calcLossGrad per entry (pred, loss, deltaWi, deltaVi).  initial_sd: ids the model lacks
        get their own N(0, initial_sd^2) draws per entry (fm_calc_loss_grad, keyed by seed); None:
        such ids are an error (fm_loss_grad)."""
        n = max(csr.nnz, 1)
        pred, loss, dw = np.zeros(n), np.zeros(n), np.zeros(n)
        dv = np.zeros((n, self.k))
        outs = (N.ptr(pred, C.c_double), N.ptr(loss, C.c_double), N.ptr(dw, C.c_double), N.ptr(dv, C.c_double))
        if initial_sd is None:
            N.check(self._lib.fm_loss_grad(self.handle, C.byref(csr.c), *outs), "fm_loss_grad")
        else:
            N.check(self._lib.fm_calc_loss_grad(self.handle, C.byref(csr.c), float(initial_sd), int(seed) & (2**64 - 1),
                                                *outs), "fm_calc_loss_grad")
        m = csr.nnz
        return pred[:m], loss[:m], dw[:m], dv[:m]

    def vector_sum_by_key(self, keys, vecs):
        keys = np.ascontiguousarray(keys, dtype=np.int32)
        vecs = np.ascontiguousarray(vecs, dtype=np.float64)
        n, k = vecs.shape
        ok = np.zeros(max(n, 1), dtype=np.int32)
        os_ = np.zeros((max(n, 1), k))
        nout = C.c_int64()
        N.check(self._lib.fm_vector_sum_by_key(self.handle, N.ptr(keys, C.c_int32), n, N.ptr(vecs, C.c_double), k,
                                               N.ptr(ok, C.c_int32), N.ptr(os_, C.c_double), C.byref(nout)),
                "fm_vector_sum_by_key")
        return ok[: nout.value], os_[: nout.value]

    # ------------------------------------------------------------------ profiling
    def profile_enable(self, on: bool = True):
        N.check(self._lib.fm_profile_enable(self.handle, 1 if on else 0), "fm_profile_enable")

    def profile_reset(self):
        N.check(self._lib.fm_profile_reset(self.handle), "fm_profile_reset")

    def profile_read(self) -> dict:
        n = C.c_int64()
        cap = 64
        names = C.create_string_buffer(4096)
        ms = np.zeros(cap)
        cnt = np.zeros(cap, dtype=np.int64)
        N.check(self._lib.fm_profile_read(self.handle, names, 4096, N.ptr(ms, C.c_double), N.ptr(cnt, C.c_int64),
                                          cap, C.byref(n)), "fm_profile_read")
        keys = names.value.decode().split("\n") if n.value else []
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(keys)}
