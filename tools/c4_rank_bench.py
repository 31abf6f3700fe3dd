#!/usr/bin/env python3
"""Config c4 (F = Int.MaxValue, k = 32, 8 row shards) timed on ONE rank at full size.

Rank 0's eighth of the table (268M rows x 256 B = 69 GB, every row present) lives on this GPU;
each iteration it routes and combines its own 256K-row batch and runs the owner phases over the
entries that all eight ranks' 256K-row batches route to it (tests/c4_emul.py emulates the seven
other ranks between the phases).  The phases' device times come from fm_profile (HIP events on
the launch streams); run under rocprofv3 --kernel-trace --stats for the per-kernel view.

  python tools/c4_rank_bench.py [--iters 5]
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    import torch

    from c4_emul import B_C4, F_C4, K_C4, R_C4, TBatch, run_iteration
    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.distributed import HipShardEngine

    t0 = time.perf_counter()
    eng = HipShardEngine(F_C4, K_C4, 0, R_C4, seed=20261015, init_sd=0.01)
    eng.init_random_range(0, F_C4)
    eng.ctx.sync()
    t_init = time.perf_counter() - t0
    hb = [synthetic_batch(B_C4, F_C4, batch_index=700 + r) for r in range(R_C4)]
    b0 = eng.batch(CSRHost(hb[0].row_ptr, hb[0].col, hb[0].val, hb[0].label))
    tbs = [TBatch(b, eng.device) for b in hb]
    print(f"[c4] table init {t_init:.1f}s, batches ready", file=sys.stderr, flush=True)
    t = 0
    for _ in range(args.warmup):
        t += 1
        run_iteration(eng, b0, tbs, t, 0.1, 1e-6, check_route=False)
    eng.ctx.profile_reset()
    eng.ctx.profile_enable(True)
    infos = []
    for _ in range(args.iters):
        t += 1
        infos.append(run_iteration(eng, b0, tbs, t, 0.1, 1e-6, check_route=False))
        print(f"[c4] iteration {t} done", file=sys.stderr, flush=True)
    prof = eng.ctx.profile_read()
    eng.ctx.profile_enable(False)
    _, _, n_upd = eng.last_stats()
    k = K_C4
    kp = (k + 3) // 4 * 4
    n_in, P = infos[-1]["n_entries_in"], infos[-1]["n_pairs_in"]
    phases = {n: {"avg_ms": ms / max(c, 1), "launches": c} for n, (ms, c) in prof.items()}
    # algorithmic bytes (SURVEY §8(d) restated per owner): the update reads + writes every row it
    # updates, 8 (k + 1) B; the owner forward reads each received entry (slot 4 B + {pair, x} 8 B) and
    # gathers its row 4 (k + 1) B, and writes a partial row per pair ((kp + 4) 4-B words)
    algo = {"owner_update": 8 * (k + 1) * n_upd, "owner_forward": n_in * (12 + 4 * (k + 1)) + P * (kp + 4) * 4}
    # counted HBM traffic per launch from the committed PMC passes of this command (profiles/pmc_c4.json,
    # tools/pmc.sh + tools/pmc_to_json.py), when present
    pmc = {}
    try:
        pmc = json.load(open(os.path.join(ROOT, "profiles", "pmc_c4.json"))).get("kernels", {})
    except (OSError, ValueError):
        pass
    kern_of = {"owner_update": ["k_segment_update", "k_segment_combine"], "owner_forward": ["k_forward"]}
    roof = {}
    for name, bytes_ in algo.items():
        if name in phases:
            ach = bytes_ / (phases[name]["avg_ms"] * 1e-3) / 1e9
            roof[name] = {"algorithmic_bytes": bytes_, "achieved_GBs": ach, "frac": ach / HBM_PEAK_GBS}
            if all("traffic_bytes" in pmc.get(kn, {}) for kn in kern_of[name]):
                roof[name]["traffic"] = sum(pmc[kn]["traffic_bytes"] for kn in kern_of[name])
                roof[name]["traffic_source"] = "profiles/pmc_c4.json"
    crit = sum(phases[n]["avg_ms"] for n in ("owner_forward", "combine", "owner_update") if n in phases)
    line = {
        "workload": "c4 per rank: F = 2^31 - 1, k = 32, rank 0 of 8 (268,435,456 rows x 256 B resident), "
                    "eight 256K-row batches routed to it per iteration",
        "iters": args.iters, "entries_in": n_in, "pairs_in": P, "rows_updated": n_upd,
        "table_bytes": int(eng.ctx.num_features // R_C4 + 1) * 256,
        "phases": phases, "roofline": roof,
        "critical_path_kernels_ms": crit,
        "note": "route / owner_prepare run on the side stream one iteration ahead in the real protocol; "
                "the all-to-all exchanges are not included (one GPU)",
    }
    print(json.dumps(line), flush=True)
    del tbs
    b0.close()
    eng.ctx.close()
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
