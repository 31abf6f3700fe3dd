"""Measurement tool (not product): the per-rank kernel times of the sharded step at R ranks,
simulated in one process on one GPU (R fm_ctx shards of the c3 table, all-to-alls done by
tensor slicing, as in tests/test_gpu_shard.py).  Shows the R = 8 shapes (about z / R entries per
(sample, owner) pair) that a world-1 run cannot.

  python tools/shard_sim_bench.py [--ranks 8] [--rows 262144] [--features 100000000] [--k 16] [--steps 5]
                                  [--reps 3]

--reps: repeated runs on the same host batches, each with fresh shard contexts.  (Round 5 timed the
fused owner step here against the unfused one, alternating, at R = 8: 1.23-1.24 against 0.92-0.93 ms
per rank-step, profiles/r05_a/sim8.log; the fused owner step was removed.)
"""

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--rows", type=int, default=262144)
    ap.add_argument("--features", type=int, default=100_000_000)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    from fm_spark_amd.data import synthetic_batch

    hb = [synthetic_batch(a.rows, a.features, batch_index=r) for r in range(a.ranks)]
    for rep in range(a.reps):
        run(a, hb, rep)


def run(a, hb, rep):
    import torch

    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.distributed import HipShardEngine

    R, F, k, B = a.ranks, a.features, a.k, a.rows
    engines = [HipShardEngine(F, k, r, R, seed=20261015) for r in range(R)]
    for e in engines:
        e.init_random_range(0, F)
    bs = [e.batch(CSRHost(b.row_ptr, b.col, b.val, b.label)) for e, b in zip(engines, hb)]
    W = engines[0].width
    kp = engines[0].kp
    for e in engines:
        e.ctx.profile_enable(True)
    for t in range(1, a.steps + 2):
        if t == 2:
            for e in engines:
                e.ctx.profile_reset()
        routed = [e.route(b) for e, b in zip(engines, bs)]
        ent_cnt = [c[:R] for _, _, c in routed]
        pair_cnt = [c[R:] for _, _, c in routed]
        keep = []
        torch.cuda.synchronize()
        for o in range(R):
            slots = torch.cat([torch.split(routed[r][0], ent_cnt[r].tolist())[o] for r in range(R)])
            ents = torch.cat([torch.split(routed[r][1], (2 * ent_cnt[r]).tolist())[o] for r in range(R)])
            src_e = np.array([ent_cnt[r][o] for r in range(R)])
            src_p = np.array([pair_cnt[r][o] for r in range(R)])
            torch.cuda.synchronize()
            engines[o].owner_prepare(bs[o], slots, ents, src_e, src_p)
            keep.append((slots, ents, src_p))
        torch.cuda.synchronize()
        partials = []
        for o in range(R):
            out = engines[o].owner_forward(bs[o], int(keep[o][2].sum()))
            partials.append(split_pairs(out, keep[o][2], kp))
        s_rows = []
        for r in range(R):
            pin = cat_pairs([partials[o][r] for o in range(R)])
            s = engines[r].combine(bs[r], pin, int(pair_cnt[r].sum()))
            s_rows.append(split_pairs(s, pair_cnt[r], kp))
        for o in range(R):
            engines[o].owner_update(bs[o], cat_pairs([s_rows[r][o] for r in range(R)]), t, 0.1, 1e-6, B * R)
        torch.cuda.synchronize()
    tot = {}
    for e in engines:
        for name, (ms, n) in e.ctx.profile_read().items():
            x = tot.setdefault(name, [0.0, 0])
            x[0] += ms
            x[1] += n
    P = [int(sum(pair_cnt[r])) for r in range(R)]
    print(f"R={R} rep={rep} rows/rank={B} pairs/rank={np.mean(P):.0f} "
          f"entries/pair={B * 39 / np.mean(P):.2f} wire MB/rank/direction={np.mean(P) * W * 4 / 1e6:.1f}")
    owner = 0.0
    for name, (ms, n) in tot.items():
        print(f"  {name:14s} {ms / n:.3f} ms per rank-step")
        if name.startswith("owner_") and name != "owner_prepare":
            owner += ms / n
    print(f"  owner phases (forward + update, critical path) {owner:.3f} ms per rank-step", flush=True)
    for e in engines:
        e.ctx.close()
    del engines, bs
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
