"""TEST INFRASTRUCTURE: a NumPy implementation of the sharded phase functions (plan / serve /
local_grad / apply, include/fm_hip.h fm_shard_*) with the oracle's fp64 math, so the
exchange protocol of fm_spark_amd.distributed.ShardedTrainer can run on CPU under gloo."""

import math

import numpy as np
import torch


class NpBatch:
    def __init__(self, csr):
        self.csr = csr
        self.n_rows = csr.n_rows
        self.nnz = csr.nnz
        self.uidx = None


class NumpyShardEngine:
    def __init__(self, num_features, k, rank, world, w0=0.0):
        self.device = torch.device("cpu")
        self.F, self.k, self.R, self.rank, self.w0 = num_features, k, world, rank, w0
        self.kp = (k + 3) // 4 * 4
        self.width = self.kp + 4
        self.rows = (num_features - rank + world - 1) // world
        self.rpsh = (num_features + world - 1) // world
        self.w = np.zeros(self.rows)
        self.V = np.zeros((self.rows, k))
        self.present = np.zeros(self.rows, dtype=bool)
        self.req = np.zeros(0, dtype=np.int32)
        self.loss = (0.0, 0)

    def batch(self, csr):
        return NpBatch(csr)

    def load_tables(self, ids, w, V):
        ids = np.asarray(ids, dtype=np.int64)
        mine = ids % self.R == self.rank
        slots = ids[mine] // self.R
        self.w[slots] = np.asarray(w)[mine]
        self.V[slots] = np.asarray(V).reshape(len(ids), self.k)[mine]
        self.present[slots] = True

    def export_tables(self):
        slots = np.nonzero(self.present)[0]
        return (slots * self.R + self.rank).astype(np.int32), self.w[slots], self.V[slots]

    def plan(self, b):
        ids = b.csr.col.astype(np.int64)
        ck = (ids % self.R) * self.rpsh + ids // self.R
        uk, inv = np.unique(ck, return_inverse=True)
        b.uidx = inv
        self.req = (uk % self.rpsh).astype(np.int32)
        return np.bincount(uk // self.rpsh, minlength=self.R).astype(np.int64)

    def request_copy(self, dst):
        dst.copy_(torch.from_numpy(self.req))

    def serve(self, req, n, rows_out):
        slots = req.numpy().astype(np.int64)
        out = np.zeros((n, self.width), dtype=np.float32)
        out[:, : self.k] = self.V[slots]
        out[:, self.kp] = self.w[slots]
        rows_out.copy_(torch.from_numpy(out.reshape(-1)))

    def local_grad(self, b, rows_in, grads_out):
        csr = b.csr
        U = len(self.req)
        rows = rows_in.numpy().reshape(U, self.width).astype(np.float64)
        m = csr.n_rows
        srow = np.repeat(np.arange(m), np.diff(csr.row_ptr))
        x = csr.val
        V = rows[b.uidx, : self.k]
        w = rows[b.uidx, self.kp]
        vfxi = V * x[:, None]
        S = np.zeros((m, self.k))
        np.add.at(S, srow, vfxi)
        wsum = np.zeros(m)
        np.add.at(wsum, srow, w * x)
        vv = np.zeros(m)
        np.add.at(vv, srow, np.sum(V * V, axis=1) * x * x)
        yhat = 0.5 * (np.sum(S * S, axis=1) - vv) + wsum + self.w0
        has = np.diff(csr.row_ptr) > 0
        d = (yhat - csr.label)[has]
        self.loss = (float(np.sum(d * d)), int(has.sum()))
        r = (yhat - csr.label)[srow]
        gw = x * yhat[srow] - csr.label[srow]
        gv = (S[srow] * x[:, None] - vfxi * x[:, None]) * r[:, None]
        GW = np.zeros(U)
        np.add.at(GW, b.uidx, gw)
        GV = np.zeros((U, self.k))
        np.add.at(GV, b.uidx, gv)
        out = np.zeros((U, self.width), dtype=np.float32)
        out[:, : self.k] = GV
        out[:, self.kp] = GW
        grads_out.copy_(torch.from_numpy(out.reshape(-1)))

    def apply(self, req, grads, n, t, step_size, reg_param, global_rows):
        if global_rows == 0:
            return 1
        eta = step_size / math.sqrt(t)
        lam = eta * reg_param
        slots = req.numpy().astype(np.int64)
        G = grads.numpy().reshape(n, self.width).astype(np.float64)
        GW = np.zeros(self.rows)
        GV = np.zeros((self.rows, self.k))
        np.add.at(GW, slots, G[:, self.kp])
        np.add.at(GV, slots, G[:, : self.k])
        touched = np.unique(slots)
        w_new, V_new = self.w.copy(), self.V.copy()
        w_new[touched] = self.w[touched] - (GW[touched] / global_rows) * eta
        V_new[touched] = self.V[touched] - GV[touched] * (eta / global_rows)
        pres = self.present.copy()
        pres[touched] = True
        self.w[pres] = np.sign(w_new[pres]) * np.maximum(0.0, np.abs(w_new[pres]) - lam)
        self.V[pres] = np.sign(V_new[pres]) * np.maximum(0.0, np.abs(V_new[pres]) - lam)
        self.present = pres
        return 0

    def last_loss(self):
        return self.loss
