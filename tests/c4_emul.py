"""TEST INFRASTRUCTURE (never imported by the product): BASELINE config c4 seen from ONE rank.

c4 = F = Int.MaxValue (2^31 - 1) features, k = 32, the table row-sharded over 8 ranks (owner =
id % 8, slot = id / 8; include/fm_hip.h fm_shard_*; README.md:7-8, Model.scala:281,289).  One
MI355X holds ONE rank's eighth of the table -- 268,435,456 rows, a real fm_ctx with shard_index 0
and shard_count 8 -- and runs that rank's phases on the HIP path: the requester phases (route,
combine) of its own 256K-row batch and the owner phases (owner_prepare, owner_forward,
owner_update) over the entries that all eight ranks' 256K-row batches route to it.

The seven other ranks exist only as data.  Their routing, their owners' partial sums and their
combine are emulated here in fp64 with torch on the same GPU, with the wire's rounding (fp32
vectors, fp64 scalars) and the device combine's summation order (owners 0..7).  Their rows are a
closed form of the id (`other_rows_np` / `other_rows_t`, identical in numpy and torch), so the
oracle can rebuild any sample's forward without holding 2^31 rows.
"""

from __future__ import annotations

import numpy as np
import torch

F_C4 = 2**31 - 1
K_C4 = 32
R_C4 = 8
B_C4 = 262144
OWNER = 0


# ------------------------------------------------------------------ rows of the other ranks
def _hash_cols(ids, f):
    """int64 mixing without overflow: every product stays below 2^63 (ids < 2^31)."""
    h1 = (ids * 2654435761) & 0x7FFFFFFF
    h2 = ((h1 + (f + 1) * 40503) * 1103515245 + 12345) & 0x7FFFFFFF
    h3 = (h2 * 1103515245 + 12345) & 0x7FFFFFFF
    return h3


def other_rows_np(ids: np.ndarray, k: int):
    """(w [n], V [n, k]) fp64 values in [-2^-7, 2^-7), multiples of 2^-30: exact in fp32."""
    ids = np.asarray(ids, dtype=np.int64)[:, None]
    f = np.arange(-1, k, dtype=np.int64)[None, :]
    h = _hash_cols(ids, f)
    vals = ((h >> 7) - (1 << 23)).astype(np.float64) * 2.0**-30
    return vals[:, 0].copy(), vals[:, 1:].copy()


def other_rows_t(ids: torch.Tensor, k: int):
    f = torch.arange(-1, k, dtype=torch.int64, device=ids.device)[None, :]
    h = _hash_cols(ids.to(torch.int64)[:, None], f)
    vals = ((h >> 7) - (1 << 23)).to(torch.float64) * 2.0**-30
    return vals[:, 0].contiguous(), vals[:, 1:].contiguous()


# ------------------------------------------------------------------ one requester batch on the GPU
class TBatch:
    """A host batch as torch tensors on the GPU: ids, x (fp64), sample of each entry, labels."""

    def __init__(self, b, device):
        self.B = b.n_rows
        self.ids = torch.from_numpy(b.col.astype(np.int64)).to(device)
        self.x = torch.from_numpy(b.val).to(device)
        self.x32 = self.x.to(torch.float32)  # the device's x (fm_step rounds x to fp32 on upload)
        self.sample = torch.repeat_interleave(torch.arange(self.B, device=device),
                                              torch.from_numpy(np.diff(b.row_ptr)).to(device))
        self.label = torch.from_numpy(b.label).to(device)
        self.owner = self.ids % R_C4


def route_to(tb: TBatch, o: int):
    """The entries of tb that owner o holds, in CSR order, as the wire carries them: slot (int32) and
    {pair index within tb's pairs to o, x fp32 bits} (int32 x 2); has[s] = sample s has such an
    entry, pair_of[s] = its pair index (pairs numbered in sample order)."""
    m = tb.owner == o
    s = tb.sample[m]
    has = torch.zeros(tb.B, dtype=torch.bool, device=tb.ids.device)
    has[s] = True
    pair_of = torch.cumsum(has.to(torch.int64), 0) - 1
    slot = (tb.ids[m] // R_C4).to(torch.int32)
    ent = torch.stack([pair_of[s].to(torch.int32), tb.x32[m].view(torch.int32)], dim=1).reshape(-1)
    return slot, ent, has, pair_of, m


def owner_partial_emul(tb: TBatch, o: int, k: int, kp: int):
    """Owner o's partial forward sums (as fm_shard_owner_forward writes them) over the rows of
    `other_rows_t`: vec [P][kp] = sum v x, sc [P][2] = {sum v^2 x^2, sum w x}, fp32 on the wire."""
    _, _, has, pair_of, m = route_to(tb, o)
    P = int(has.sum())
    ids, x, s = tb.ids[m], tb.x32[m].to(torch.float64), tb.sample[m]
    w, V = other_rows_t(ids, k)
    V = V.to(torch.float32).to(torch.float64)
    w = w.to(torch.float32).to(torch.float64)
    pidx = pair_of[s]
    vec = torch.zeros(P, kp, dtype=torch.float64, device=ids.device)
    vec[:, :k].index_add_(0, pidx, V * x[:, None])
    sc = torch.zeros(P, 2, dtype=torch.float64, device=ids.device)
    sc[:, 0].index_add_(0, pidx, (V * V).sum(1) * x * x)
    sc[:, 1].index_add_(0, pidx, w * x)
    return vec.to(torch.float32), sc.to(torch.float32), has, pair_of


def wire(vec: torch.Tensor, sc: torch.Tensor) -> torch.Tensor:
    """[P][kp] + [P][2] -> the flat fp32 wire layout (include/fm_hip.h)."""
    return torch.cat([vec.reshape(-1), sc.to(torch.float32).contiguous().reshape(-1)])


def unwire(buf: torch.Tensor, kp: int):
    P = buf.numel() // (kp + 2)
    return buf[: P * kp].reshape(P, kp), buf[P * kp:].reshape(P, 2)


def combine_emul(tb: TBatch, parts, kp: int, w0: float = 0.0):
    """fm_shard_combine for an emulated requester: parts[o] = (vec, sc, has, pair_of) of owner o.
    Sums in owner order in fp64 as k_shard_combine does; returns S [B][kp] fp64, yhat [B]."""
    dev = tb.ids.device
    S = torch.zeros(tb.B, kp, dtype=torch.float64, device=dev)
    vv = torch.zeros(tb.B, dtype=torch.float64, device=dev)
    wx = torch.zeros(tb.B, dtype=torch.float64, device=dev)
    for vec, sc, has, pair_of in parts:
        idx = pair_of[has]
        S[has] += vec[idx].to(torch.float64)
        vv[has] += sc[idx, 0].to(torch.float64)
        wx[has] += sc[idx, 1].to(torch.float64)
    yhat = 0.5 * ((S * S).sum(1) - vv) + wx + w0
    return S, yhat


def run_iteration(eng, b0_dev, tbs, t, step_size, reg_param, check_route=True):
    """One c4 iteration seen from rank 0 (module docstring).  Returns a dict of what the checks need."""
    k, kp, R = eng.ctx.k, eng.kp, R_C4
    # requester phase of rank 0's own batch, on the device
    send_slot0, send_ent0, counts0 = eng.route(b0_dev)
    routes = [route_to(tb, OWNER) for tb in tbs]
    info = {}
    if check_route:
        torch.cuda.synchronize()
        ent_cnt = [int((tbs[0].owner == o).sum()) for o in range(R)]
        pair_cnt = [int(route_to(tbs[0], o)[2].sum()) for o in range(R)]
        info["route_counts_ok"] = list(counts0[:R]) == ent_cnt and list(counts0[R:]) == pair_cnt
        n0 = ent_cnt[0]
        info["route_entries_ok"] = (torch.equal(send_slot0[:n0], routes[0][0]) and
                                    torch.equal(send_ent0[: 2 * n0], routes[0][1]))
    src_e = np.array([int(r[0].numel()) for r in routes], dtype=np.int64)
    src_p = np.array([int(r[2].sum()) for r in routes], dtype=np.int64)
    recv_slot = torch.cat([r[0] for r in routes])
    recv_ent = torch.cat([r[1] for r in routes])
    torch.cuda.synchronize()  # owner_prepare runs on the context's side stream; the buffers came from this one
    eng.owner_prepare(b0_dev, recv_slot, recv_ent, src_e, src_p)
    P = int(src_p.sum())
    part0 = eng.owner_forward(b0_dev, P)
    vec0, sc0 = unwire(part0, kp)
    pbase = np.concatenate([[0], np.cumsum(src_p)])
    s_vec, s_sc = [], []
    for r, tb in enumerate(tbs):
        mine = (vec0[pbase[r]: pbase[r + 1]], sc0[pbase[r]: pbase[r + 1]], routes[r][2], routes[r][3])
        parts = [mine] + [owner_partial_emul(tb, o, k, kp) for o in range(1, R)]
        if r == 0:  # rank 0 combines its own batch on the device
            pin = torch.cat([torch.cat([p[0].reshape(-1) for p in parts]),
                             torch.cat([p[1].contiguous().reshape(-1) for p in parts])])
            s_send = eng.combine(b0_dev, pin, int(sum(int(p[2].sum()) for p in parts)))
            v_all, c_all = unwire(s_send, kp)
            p0 = int(routes[0][2].sum())
            s_vec.append(v_all[:p0])
            s_sc.append(c_all[:p0])
            S, yhat = combine_emul(tb, parts, kp)
            info["own_loss_emul"] = float(((yhat - tb.label) ** 2).sum())
        else:
            S, yhat = combine_emul(tb, parts, kp)
            has = routes[r][2]
            s_vec.append(S[has].to(torch.float32))
            s_sc.append(torch.stack([yhat[has] - tb.label[has], yhat[has]], dim=1).to(torch.float32))
    s_recv = wire(torch.cat(s_vec), torch.cat(s_sc))
    gm = sum(tb.B for tb in tbs)
    eng.owner_update(b0_dev, s_recv, t, step_size, reg_param, gm)
    torch.cuda.synchronize()
    info["n_entries_in"] = int(src_e.sum())
    info["n_pairs_in"] = P
    info["global_rows"] = gm
    return info
