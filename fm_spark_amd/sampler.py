"""Mini-batch sampler: Spark 2.1.0 ``randomSplit`` replay through the C-ABI
(fm_random_split, fm_spark_amd/csrc/fm_sampler.cpp).  Replaces
``dfData.randomSplit(Array.fill(maxIter)(miniBatchFraction), 1234L)``
(FactorizationMachinesSGD.scala:111-112) over rows tagged by monotonically_increasing_id
(FactorizationMachinesModel.scala:268-272)."""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N
from .linalg import DenseVector, Vector


def encode_rows(labels, vectors):
    """Flatten (label, Vector) rows into the column arrays fm_random_split sorts on."""
    n = len(vectors)
    vtype = np.zeros(n, dtype=np.int8)
    vsize = np.zeros(n, dtype=np.int32)
    ptr = np.zeros(n + 1, dtype=np.int64)
    idx, val = [], []
    for r, v in enumerate(vectors):
        if isinstance(v, DenseVector):
            vtype[r] = 1
            vals = v.values
            idx.extend([0] * len(vals))
        else:
            vtype[r] = 0
            vals = v.values
            idx.extend(v.indices.tolist())
        vsize[r] = v.size
        val.extend(vals.tolist())
        ptr[r + 1] = ptr[r] + len(vals)
    lab = np.ascontiguousarray(labels, dtype=np.float64) if labels is not None else np.zeros(n)
    return lab, vtype, vsize, ptr, np.asarray(idx, dtype=np.int32), np.asarray(val, dtype=np.float64)


def random_split(part_sizes, labels, vectors, weights, seed: int, column_order: str = "LF", extra=None):
    """Returns (split_of[n], sample_id[n], order[n]) for rows laid out partition after
    partition (part_sizes[p] rows in partition p)."""
    lib = N.load()
    n = len(vectors)
    part_ptr = np.zeros(len(part_sizes) + 1, dtype=np.int64)
    part_ptr[1:] = np.cumsum(part_sizes)
    if part_ptr[-1] != n:
        raise ValueError("partition sizes do not add up to the row count")
    lab, vtype, vsize, ptr, idx, val = encode_rows(labels, vectors)
    w = np.ascontiguousarray(weights, dtype=np.float64)
    ex = np.ascontiguousarray(extra if extra is not None else np.zeros(n), dtype=np.int64)
    split_of = np.zeros(max(n, 1), dtype=np.int32)
    sid = np.zeros(max(n, 1), dtype=np.int64)
    order = np.zeros(max(n, 1), dtype=np.int64)
    if len(idx) == 0:
        idx = np.zeros(1, dtype=np.int32)
        val = np.zeros(1)
    N.check(lib.fm_random_split(len(part_sizes), N.ptr(part_ptr, C.c_int64), column_order.encode(),
                                N.ptr(lab, C.c_double), N.ptr(vtype, C.c_int8), N.ptr(vsize, C.c_int32),
                                N.ptr(ptr, C.c_int64), N.ptr(idx, C.c_int32), N.ptr(val, C.c_double),
                                N.ptr(ex, C.c_int64), len(w), N.ptr(w, C.c_double), int(seed),
                                N.ptr(split_of, C.c_int32), N.ptr(sid, C.c_int64), N.ptr(order, C.c_int64)),
            "fm_random_split")
    return split_of[:n], sid[:n], order[:n]


def random_split_csr(part_sizes, labels, row_ptr, col, val, num_features: int, weights, seed: int):
    """random_split over rows given as a CSR of sparse vectors of size num_features (columns
    label, features; what a DataFrame of (label, SparseVector) rows sorts on), without Vector
    objects: the bench's resident-fit leg splits a multi-million-row synthetic dataset this way."""
    lib = N.load()
    n = len(labels)
    part_ptr = np.zeros(len(part_sizes) + 1, dtype=np.int64)
    part_ptr[1:] = np.cumsum(part_sizes)
    if part_ptr[-1] != n:
        raise ValueError("partition sizes do not add up to the row count")
    lab = np.ascontiguousarray(labels, dtype=np.float64)
    vtype = np.zeros(max(n, 1), dtype=np.int8)
    vsize = np.full(max(n, 1), int(num_features), dtype=np.int32)
    ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
    idx = np.ascontiguousarray(col, dtype=np.int32) if len(col) else np.zeros(1, dtype=np.int32)
    vv = np.ascontiguousarray(val, dtype=np.float64) if len(val) else np.zeros(1)
    w = np.ascontiguousarray(weights, dtype=np.float64)
    ex = np.zeros(max(n, 1), dtype=np.int64)
    split_of = np.zeros(max(n, 1), dtype=np.int32)
    sid = np.zeros(max(n, 1), dtype=np.int64)
    order = np.zeros(max(n, 1), dtype=np.int64)
    N.check(lib.fm_random_split(len(part_sizes), N.ptr(part_ptr, C.c_int64), b"LF", N.ptr(lab, C.c_double),
                                N.ptr(vtype, C.c_int8), N.ptr(vsize, C.c_int32), N.ptr(ptr, C.c_int64),
                                N.ptr(idx, C.c_int32), N.ptr(vv, C.c_double), N.ptr(ex, C.c_int64), len(w),
                                N.ptr(w, C.c_double), int(seed), N.ptr(split_of, C.c_int32), N.ptr(sid, C.c_int64),
                                N.ptr(order, C.c_int64)), "fm_random_split")
    return split_of[:n], sid[:n], order[:n]


def hash_seed(seed: int) -> int:
    return int(N.load().fm_xorshift_hash_seed(int(seed)))


def next_doubles(seed: int, n: int) -> np.ndarray:
    out = np.zeros(max(n, 1))
    N.check(N.load().fm_xorshift_next_doubles(int(seed), int(n), N.ptr(out, C.c_double)), "fm_xorshift_next_doubles")
    return out[:n]


def murmur3(data: bytes, seed: int) -> int:
    buf = (C.c_uint8 * max(len(data), 1)).from_buffer_copy(data if data else b"\0")
    return int(N.load().fm_murmur3_bytes_hash(buf, len(data), int(seed))) & 0xFFFFFFFF
