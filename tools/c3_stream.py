"""Measurement tool (not product): write one c3 batch's forward address stream for
tools/gather_ceiling.hip -- int64 {B, N}, row_ptr [B + 1] int64, feature ids [N] uint32 in CSR order
with bit 31 set on ids that have one entry in the batch (the rows the fused forward writes back),
x [N] fp32.  The batch is bench.py's first c3 batch (synthetic_batch(262144, 100M, batch_index=0)).

  python tools/c3_stream.py <out.bin> [--features 100000000] [--rows 262144] [--batch-index 0]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fm_spark_amd.data import synthetic_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--features", type=int, default=100_000_000)
ap.add_argument("--rows", type=int, default=262144)
ap.add_argument("--batch-index", type=int, default=0)
a = ap.parse_args()
b = synthetic_batch(a.rows, a.features, batch_index=a.batch_index)
_, inv, cnt = np.unique(b.col, return_inverse=True, return_counts=True)
ids = b.col.astype(np.uint32) | (np.uint32(1 << 31) * (cnt[inv] == 1).astype(np.uint32))
with open(a.out, "wb") as f:
    f.write(np.asarray([b.n_rows, b.nnz], dtype=np.int64).tobytes())
    f.write(b.row_ptr.astype(np.int64).tobytes())
    f.write(ids.astype(np.uint32).tobytes())
    f.write(b.val.astype(np.float32).tobytes())
print(f"wrote {a.out}: rows={b.n_rows} entries={b.nnz} distinct={len(cnt)} singleton_ids={int((cnt == 1).sum())}")
