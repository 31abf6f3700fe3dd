"""Seeded test problems shared by the CPU and GPU suites (inputs rounded to fp32 so the
device's fp32 tables start from exactly the oracle's values)."""

import numpy as np

from oracle import fm_ref as R


def f32(a):
    return np.asarray(a, dtype=np.float32).astype(np.float64)


def make_problem(seed, n_rows, F, k, mean_nnz, *, empty_frac=0.1, zero_frac=0.05, hot=None, labels="binary"):
    rng = np.random.default_rng(seed)
    row_ptr = [0]
    cols, vals = [], []
    for _ in range(n_rows):
        if rng.random() < empty_frac:
            row_ptr.append(len(cols))
            continue
        z = int(rng.integers(1, 2 * mean_nnz))
        z = min(z, F)
        ids = rng.choice(F, size=z, replace=False)
        if hot is not None and rng.random() < 0.9 and hot not in ids:
            ids[0] = hot
        ids = np.sort(ids)
        v = f32(rng.normal(0.0, 1.0, size=z))
        v[rng.random(z) < zero_frac] = 0.0  # explicit zeros stay active
        cols.extend(ids.tolist())
        vals.extend(v.tolist())
        row_ptr.append(len(cols))
    if labels == "binary":
        y = (rng.random(n_rows) < 0.25).astype(np.float64)
    else:
        y = f32(rng.normal(0.0, 1.0, n_rows))
    csr = R.CSR(row_ptr=np.asarray(row_ptr, np.int64), col=np.asarray(cols, np.int32),
                val=np.asarray(vals, np.float64), label=y)
    ids = np.arange(F, dtype=np.int32)
    w = f32(rng.normal(0.0, 0.1, F))
    V = f32(rng.normal(0.0, 0.1, (F, k)))
    return csr, ids, w, V
