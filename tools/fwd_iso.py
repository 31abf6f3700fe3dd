#!/usr/bin/env python3
"""Per-kernel times of the c3 step with nothing else on the GPU: every batch is prepared (sorted,
split) and the device drained before its step, so the step's kernels run alone.  Prints one JSON
line per variant (fused / unfused) with the average ms of each profiled phase."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fm_spark_amd._native import CSRHost  # noqa: E402
from fm_spark_amd.data import synthetic_batch  # noqa: E402
from fm_spark_amd.engine import FMContext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--features", type=int, default=100_000_000)
ap.add_argument("--k", type=int, default=16)
ap.add_argument("--rows", type=int, default=262144)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--variants", default="on,off")
a = ap.parse_args()
hb = [synthetic_batch(a.rows, a.features, batch_index=i) for i in range(2)]
for v in a.variants.split(","):
    ctx = FMContext(a.features, a.k, seed=1, init_sd=0.01, fuse=(v == "on"))
    ctx.init_random_range(0, a.features)
    dbs = [ctx.batch(CSRHost(b.row_ptr, b.col, b.val, b.label)) for b in hb]
    for t in range(1, 3):
        dbs[t % 2].prepare()
        ctx.step_batch(dbs[t % 2], t, 0.1, 1e-6, sync=True)
    torch.cuda.synchronize()
    ctx.profile_reset()
    ctx.profile_enable(True)
    for t in range(3, 3 + a.steps):
        dbs[t % 2].prepare()
        torch.cuda.synchronize()  # the sort and split are done: the step runs alone
        ctx.step_batch(dbs[t % 2], t, 0.1, 1e-6, sync=True)
    prof = ctx.profile_read()
    ctx.profile_enable(False)
    print(json.dumps({"fuse": v, "phases_ms": {k: ms / n for k, (ms, n) in prof.items()}}), flush=True)
    ctx.close()
