"""Measurement tool (not product): fm_random_split on the bench's fit-leg dataset (16 x 262,144 c3 rows in
16 partitions, weights 16 x 0.1, seed 1234).  Times the C call as fit makes it (partitions on the
library's host pool) against the same partitions split one call at a time on one thread (partition p
sorted and sampled alone with seed 1234 + p -- what the pooled call does for p), checks the two equal,
and times the Python wrapper's array preparation (sampler.random_split_csr) separately.

  python tools/sampler_bench.py [--iters 16] [--rows 262144]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from fm_spark_amd import _native as N  # noqa: E402
from fm_spark_amd.data import synthetic_batch  # noqa: E402
from fm_spark_amd.sampler import random_split_csr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=16)
ap.add_argument("--rows", type=int, default=262144)
ap.add_argument("--features", type=int, default=100_000_000)
a = ap.parse_args()
t0 = time.perf_counter()
ds = bench.concat_batches([synthetic_batch(a.rows, a.features, batch_index=7000 + i, zipf_s=1.05)
                           for i in range(a.iters)])
t_gen = time.perf_counter() - t0
n, parts = ds.n_rows, 16
sizes = [n * (i + 1) // parts - n * i // parts for i in range(parts)]
t0 = time.perf_counter()
ref_split, _, ref_order = random_split_csr(sizes, ds.label, ds.row_ptr, ds.col, ds.val, a.features, [0.1] * a.iters, 1234)
t_wrapper = time.perf_counter() - t0

lib = N.load()
lab = np.ascontiguousarray(ds.label, dtype=np.float64)
rp = np.ascontiguousarray(ds.row_ptr, dtype=np.int64)
col = np.ascontiguousarray(ds.col, dtype=np.int32)
val = np.ascontiguousarray(ds.val, dtype=np.float64)
vtype = np.zeros(n, np.int8)
vsize = np.full(n, a.features, np.int32)
ex = np.zeros(1, np.int64)
w = np.full(a.iters, 0.1)
pp = np.zeros(parts + 1, np.int64)
pp[1:] = np.cumsum(sizes)


def call(np_, pptr, r0, seed, so, sid, od):
    e0 = int(rp[r0])
    N.check(lib.fm_random_split(np_, N.ptr(pptr, C.c_int64), b"LF", N.ptr(lab[r0:], C.c_double),
                                N.ptr(vtype[r0:], C.c_int8), N.ptr(vsize[r0:], C.c_int32),
                                N.ptr(np.ascontiguousarray(rp[r0:] - e0), C.c_int64), N.ptr(col[e0:], C.c_int32),
                                N.ptr(val[e0:], C.c_double), N.ptr(ex, C.c_int64), len(w), N.ptr(w, C.c_double),
                                int(seed), N.ptr(so, C.c_int32), N.ptr(sid, C.c_int64), N.ptr(od, C.c_int64)),
            "fm_random_split")


so, sid, od = np.zeros(n, np.int32), np.zeros(n, np.int64), np.zeros(n, np.int64)
t_pool = []
for _ in range(3):
    t0 = time.perf_counter()
    call(parts, pp, 0, 1234, so, sid, od)
    t_pool.append(time.perf_counter() - t0)
assert np.array_equal(so, ref_split) and np.array_equal(od, ref_order)
so1, sid1, od1 = np.zeros(n, np.int32), np.zeros(n, np.int64), np.zeros(n, np.int64)
t0 = time.perf_counter()
for p in range(parts):
    r0, r1 = int(pp[p]), int(pp[p + 1])
    one = np.asarray([0, r1 - r0], np.int64)
    call(1, one, r0, 1234 + p, so1[r0:], sid1[r0:], od1[r0:])
    od1[r0:r1] += r0
t_one = time.perf_counter() - t0
assert np.array_equal(so1, so) and np.array_equal(od1, od)
print(json.dumps({"rows": n, "partitions": parts, "host_cpus": os.cpu_count(), "pool_threads": min(16, os.cpu_count()),
                  "generate_s": t_gen, "wrapper_s": t_wrapper, "call_pool_s": t_pool,
                  "call_one_thread_s": t_one, "speedup": t_one / min(t_pool)}))
