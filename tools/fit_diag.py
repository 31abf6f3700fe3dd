"""Measurement tool (not product): where the resident fit loop's time goes at c3.  Builds bench.py's
fit_leg dataset, then times (host clock) the loop as run_minibatch_sgd_resident runs it, with each
API call's host time accumulated; the same loop with a device sync after every step (GPU time per
iteration); fm_batch_from_rows alone; prepare + step on pre-gathered batches.
  python tools/fit_diag.py [iters]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fm_spark_amd._native import CSRHost  # noqa: E402
from fm_spark_amd.data import synthetic_batch  # noqa: E402
from fm_spark_amd.engine import FMContext  # noqa: E402
from fm_spark_amd.sampler import random_split_csr  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 8
F, k, B, zs, _ = bench.CONFIGS["c3"]
ctx = FMContext(F, k, seed=20261015, init_sd=bench.INIT_SD)
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
ctx.set_stream(st.cuda_stream)
ctx.init_random_range(0, F)
ds = bench.concat_batches([synthetic_batch(B, F, batch_index=7000 + i, zipf_s=zs) for i in range(iters)])
n = ds.n_rows
sizes = [n * (i + 1) // 16 - n * i // 16 for i in range(16)]
split_of, _, order = random_split_csr(sizes, ds.label, ds.row_ptr, ds.col, ds.val, F, [0.1] * iters, 1234)
splits = [order[split_of[order] == i] for i in range(iters)]
data = ctx.batch(CSRHost(ds.row_ptr, ds.col, ds.val, ds.label))
ctx.sync()
res = {"iters": iters, "rows": [len(s) for s in splits]}


def loop(sync_each=False, acc=None, bufs=None):
    own = bufs is None
    if own:
        bufs = [None, None, None]

    def timed(name, f):
        t0 = time.perf_counter()
        r = f()
        if acc is not None:
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
        return r

    nb = len(bufs)

    def gather(j):
        bufs[j % nb] = timed("from_rows", lambda: ctx.batch_from_rows(data, splits[j], into=bufs[j % nb]))

    t0 = time.perf_counter()
    gather(0)
    timed("prepare", bufs[0].prepare)
    gather(1)
    for j in range(iters):
        timed("step", lambda: ctx.step_batch(bufs[j % nb], j + 1, bench.STEP_SIZE, bench.REG_PARAM, sync=False))
        if sync_each:
            timed("sync", ctx.sync)
        if j + 1 < iters:
            timed("prepare", bufs[(j + 1) % nb].prepare)
        if j + 2 < iters:
            gather(j + 2)
    timed("sync", ctx.sync)
    dt = time.perf_counter() - t0
    if own:
        for b in bufs:
            b.close()
    return dt


keep = [None, None, None]
loop(bufs=keep)  # buffers grown
for rep in range(2):
    acc = {}
    dt = loop(acc=acc, bufs=keep)
    res[f"pipelined_{rep}"] = {"ms_per_iter": 1e3 * dt / iters, "host_ms_per_iter": {k: 1e3 * v / iters for k, v in acc.items()}}
acc = {}
dt = loop(acc=acc)
res["pipelined_fresh_batches"] = {"ms_per_iter": 1e3 * dt / iters, "host_ms_per_iter": {k: 1e3 * v / iters for k, v in acc.items()}}
acc = {}
dt = loop(sync_each=True, acc=acc, bufs=keep)
res["synced"] = {"ms_per_iter": 1e3 * dt / iters, "host_ms_per_iter": {k: 1e3 * v / iters for k, v in acc.items()}}
# fm_batch_from_rows alone, into one batch
b = None
t0 = time.perf_counter()
for j in range(iters):
    b = ctx.batch_from_rows(data, splits[j], into=b)
ctx.sync()
res["from_rows_only_ms"] = 1e3 * (time.perf_counter() - t0) / iters
# prepare + step on pre-gathered batches (the bench's own loop shape)
pre = [ctx.batch_from_rows(data, s) for s in splits]
ctx.sync()
pre[0].prepare()
t0 = time.perf_counter()
for j in range(iters):
    ctx.step_batch(pre[j], j + 1, bench.STEP_SIZE, bench.REG_PARAM, sync=False)
    if j + 1 < iters:
        pre[j + 1].prepare()
ctx.sync()
res["pregathered_ms_per_iter"] = 1e3 * (time.perf_counter() - t0) / iters
print(json.dumps(res, indent=1))
