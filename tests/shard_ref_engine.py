"""TEST INFRASTRUCTURE: a NumPy implementation of the sharded phase functions (route /
owner_forward / combine / owner_update, include/fm_hip.h fm_shard_*) with the oracle's fp64
math and the same fp32 wire formats, so the exchange protocol of
fm_spark_amd.distributed.ShardedTrainer can run on CPU under gloo."""

import math

import numpy as np
import torch


def rows_to_soa(rows, kp):
    """[P][kp + 2] rows -> the fp32 wire layout: [P][kp] vectors, then [P][2] scalars (flat)."""
    rows = np.asarray(rows, dtype=np.float32)
    return np.ascontiguousarray(np.concatenate([rows[:, :kp].reshape(-1), rows[:, kp:kp + 2].reshape(-1)]))


def soa_to_rows(flat, kp):
    P = len(flat) // (kp + 2)
    return np.concatenate([flat[: P * kp].reshape(P, kp), flat[P * kp:].reshape(P, 2)], axis=1).astype(np.float64)


class NpBatch:
    def __init__(self, csr):
        self.csr = csr
        self.n_rows = csr.n_rows
        self.nnz = csr.nnz


class NumpyShardEngine:
    def __init__(self, num_features, k, rank, world, w0=0.0):
        self.device = torch.device("cpu")
        self.F, self.k, self.R, self.rank, self.w0 = num_features, k, world, rank, w0
        self.kp = (k + 3) // 4 * 4
        self.width = self.kp + 2  # wire: [P][kp] vectors, then [P][2] scalars
        self.rows = (num_features - rank + world - 1) // world
        self.w = np.zeros(self.rows)
        self.V = np.zeros((self.rows, k))
        self.present = np.zeros(self.rows, dtype=bool)
        self.stats = (0.0, 0, 0)

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

    # requester -------------------------------------------------------------------
    def route(self, b):
        csr = b.csr
        ids = csr.col.astype(np.int64)
        owner = ids % self.R
        sample = np.repeat(np.arange(csr.n_rows), np.diff(csr.row_ptr))
        order = np.argsort(owner, kind="stable")
        send_slot = (ids[order] // self.R).astype(np.int32)
        ents = np.bincount(owner, minlength=self.R)
        has = np.zeros((csr.n_rows, self.R), dtype=bool)
        has[sample, owner] = True
        pairs = has.sum(axis=0)
        b.pairidx = np.where(has, np.cumsum(has, axis=0) - 1, -1)  # [B][R]
        b.pairs_out = pairs
        # wire entry = {index of its (sample, owner) pair within this rank's pairs to the owner, x}
        local = b.pairidx[sample[order], owner[order]].astype(np.uint32)
        ent = np.stack([local, csr.val[order].astype(np.float32).view(np.uint32)], axis=1)
        counts = np.concatenate([ents, pairs]).astype(np.int64)
        return torch.from_numpy(send_slot), torch.from_numpy(ent.view(np.int32).reshape(-1).copy()), counts

    def combine(self, b, partials_in, n_pairs_out):
        csr = b.csr
        kp = self.kp
        part = soa_to_rows(partials_in.numpy(), kp).astype(np.float64)
        poff = np.concatenate([[0], np.cumsum(b.pairs_out)])
        B = csr.n_rows
        S = np.zeros((B, kp))
        vv = np.zeros(B)
        wx = np.zeros(B)
        for o in range(self.R):  # owner order
            ix = b.pairidx[:, o]
            m = ix >= 0
            rows = part[poff[o] + ix[m]]
            S[m] += rows[:, :kp]
            vv[m] += rows[:, kp]
            wx[m] += rows[:, kp + 1]
        yhat = 0.5 * (np.sum(S * S, axis=1) - vv) + wx + self.w0
        has = np.diff(csr.row_ptr) > 0
        d = (yhat - csr.label)[has]
        b.loss = (float(np.sum(d * d)), int(has.sum()))
        out = np.zeros((int(n_pairs_out), kp + 2), dtype=np.float64)
        for o in range(self.R):
            ix = b.pairidx[:, o]
            m = ix >= 0
            out[poff[o] + ix[m], :kp] = S[m]
            out[poff[o] + ix[m], kp] = yhat[m] - csr.label[m]  # r, formed in fp64
            out[poff[o] + ix[m], kp + 1] = yhat[m]
        return torch.from_numpy(rows_to_soa(out, kp))

    # owner -----------------------------------------------------------------------
    def owner_prepare(self, b, recv_slot, recv_ent, src_entries, src_pairs):
        b.recv_in = (recv_slot.clone(), recv_ent.clone(), np.asarray(src_entries), np.asarray(src_pairs))

    def owner_forward(self, b, n_pairs_in):
        recv_slot, recv_ent, src_entries, src_pairs = b.recv_in
        slots = recv_slot.numpy().astype(np.int64)
        ent = recv_ent.numpy().view(np.uint32).reshape(-1, 2)
        s, x = ent[:, 0].astype(np.int64), ent[:, 1].view(np.float32).astype(np.float64)
        n = len(slots)
        src = np.repeat(np.arange(self.R), src_entries)
        head = np.ones(n, dtype=bool)
        head[1:] = (s[1:] != s[:-1]) | (src[1:] != src[:-1])
        pair = np.cumsum(head) - 1
        P = int(head.sum())
        assert P == int(np.sum(src_pairs)) == n_pairs_in
        V, w = self.V[slots], self.w[slots]
        part = np.zeros((P, self.kp + 2))
        np.add.at(part[:, : self.k], pair, V * x[:, None])
        np.add.at(part[:, self.kp], pair, np.sum(V * V, axis=1) * x * x)
        np.add.at(part[:, self.kp + 1], pair, w * x)
        b.recv = (slots, x, pair)
        return torch.from_numpy(rows_to_soa(part, self.kp))

    def owner_update(self, b, s_recv, t, step_size, reg_param, global_rows):
        if global_rows == 0:
            return 1
        slots, x, pair = b.recv
        Srow = soa_to_rows(s_recv.numpy(), self.kp).astype(np.float64)
        S, r, yhat = Srow[pair, : self.k], Srow[pair, self.kp], Srow[pair, self.kp + 1]
        eta = step_size / math.sqrt(t)
        lam = eta * reg_param
        V = self.V[slots]
        gw = (x - 1.0) * yhat + r  # x * yhat - y with y = yhat - r (SGD.scala:145)
        gv = (S * x[:, None] - V * x[:, None] * x[:, None]) * r[:, None]
        GW = np.zeros(self.rows)
        GV = np.zeros((self.rows, self.k))
        np.add.at(GW, slots, gw)
        np.add.at(GV, slots, gv)
        touched = np.unique(slots)
        w_new, V_new = self.w.copy(), self.V.copy()
        w_new[touched] = self.w[touched] - (GW[touched] / global_rows) * eta
        V_new[touched] = self.V[touched] - GV[touched] * (eta / global_rows)
        pres = self.present.copy()
        pres[touched] = True
        self.w[pres] = np.sign(w_new[pres]) * np.maximum(0.0, np.abs(w_new[pres]) - lam)
        self.V[pres] = np.sign(V_new[pres]) * np.maximum(0.0, np.abs(V_new[pres]) - lam)
        self.present = pres
        self.stats = (b.loss[0], b.loss[1], len(touched))
        return 0

    def last_stats(self):
        return self.stats


class NumpyReplEngine:
    """TEST INFRASTRUCTURE: the replicated phase functions (fm_repl_grad / fm_repl_apply) in
    NumPy with the same fp32 gradient buffer layout [F][kp + 4]."""

    def __init__(self, num_features, k, w0=0.0):
        self.device = torch.device("cpu")
        self.F, self.k, self.w0 = num_features, k, w0
        self.kp = (k + 3) // 4 * 4
        self.width = self.kp + 4
        self.w = np.zeros(num_features)
        self.V = np.zeros((num_features, k))
        self.present = np.zeros(num_features, dtype=bool)
        self.stats = (0.0, 0, 0)

    def batch(self, csr):
        return NpBatch(csr)

    def load_tables(self, ids, w, V):
        ids = np.asarray(ids, dtype=np.int64)
        self.w[ids] = w
        self.V[ids] = np.asarray(V).reshape(len(ids), self.k)
        self.present[ids] = True

    def export_tables(self):
        ids = np.nonzero(self.present)[0]
        return ids.astype(np.int32), self.w[ids], self.V[ids]

    def grad_phase(self, b):
        csr = b.csr
        g = np.zeros((self.F, self.width))
        self.loss = (0.0, 0)
        if csr.n_rows:
            ids = csr.col.astype(np.int64)
            x = csr.val
            srow = np.repeat(np.arange(csr.n_rows), np.diff(csr.row_ptr))
            V, w = self.V[ids], self.w[ids]
            S = np.zeros((csr.n_rows, self.k))
            np.add.at(S, srow, V * x[:, None])
            vv = np.zeros(csr.n_rows)
            np.add.at(vv, srow, np.sum(V * V, axis=1) * x * x)
            wx = np.zeros(csr.n_rows)
            np.add.at(wx, srow, w * x)
            yhat = 0.5 * (np.sum(S * S, axis=1) - vv) + wx + self.w0
            has = np.diff(csr.row_ptr) > 0
            d = (yhat - csr.label)[has]
            self.loss = (float(np.sum(d * d)), int(has.sum()))
            r = (yhat - csr.label)[srow]
            np.add.at(g[:, : self.k], ids, (S[srow] * x[:, None] - V * x[:, None] * x[:, None]) * r[:, None])
            np.add.at(g[:, self.kp], ids, x * yhat[srow] - csr.label[srow])
            g[ids, self.kp + 1] = 1.0
        self.grad = torch.from_numpy(g.astype(np.float32).reshape(-1))
        return self.grad

    def apply(self, grad, t, step_size, reg_param, global_rows):
        if global_rows == 0:
            return 1
        G = grad.numpy().reshape(self.F, self.width).astype(np.float64)
        touched = np.nonzero(G[:, self.kp + 1] > 0)[0]
        eta = step_size / math.sqrt(t)
        lam = eta * reg_param
        w_new, V_new = self.w.copy(), self.V.copy()
        w_new[touched] -= (G[touched, self.kp] / global_rows) * eta
        V_new[touched] -= G[touched, : self.k] * (eta / global_rows)
        pres = self.present.copy()
        pres[touched] = True
        self.w[pres] = np.sign(w_new[pres]) * np.maximum(0.0, np.abs(w_new[pres]) - lam)
        self.V[pres] = np.sign(V_new[pres]) * np.maximum(0.0, np.abs(V_new[pres]) - lam)
        self.present = pres
        self.stats = (self.loss[0], self.loss[1], len(touched))
        return 0

    def last_stats(self):
        return self.stats
