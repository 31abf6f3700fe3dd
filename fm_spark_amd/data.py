"""Input formats either side of the hot path.

* ``synthetic_batch`` — the Criteo-shaped synthetic workload of BASELINE.md / SURVEY.md §8(d):
  39 fields per sample (13 numeric with x = log1p(Poisson(3)) rounded to fp32, 26
  categorical with x = 1.0; ``exact=True`` keeps x and the regression labels in fp64, as Spark's
  Double columns hold them).  Field f's feature id is splitmix64(f * 2^32 + rank) mod F
  with rank ~ Zipf(s) (s = 1.05, or 1.2 for the c5 skew); ids that collide inside a row are
  re-drawn, so every row holds 39 distinct ids in ascending order.  Labels are
  Bernoulli(0.25) ("binary") or <w*, x> + N(0, 0.1) ("regression", c5).
* ``read_libsvm`` — Spark's ``libsvm`` data source as used for data/sample.txt (config c1):
  1-based indices -> 0-based, every listed pair kept (explicit zeros stay active entries,
  SURVEY P5), features sized by the largest index.
"""

from __future__ import annotations

from dataclasses import dataclass

import os

import numpy as np

N_NUMERIC = 13
N_CATEGORICAL = 26
N_FIELDS = N_NUMERIC + N_CATEGORICAL
DEFAULT_SEED = 20261015

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


@dataclass
class Batch:
    row_ptr: np.ndarray  # int64 [B+1]
    col: np.ndarray  # int32 [N]
    val: np.ndarray  # float64 [N] (fp32-representable)
    label: np.ndarray  # float64 [B]

    @property
    def n_rows(self) -> int:
        return len(self.label)

    @property
    def nnz(self) -> int:
        return len(self.col)


def _field_ids(field: int, ranks: np.ndarray, F: int) -> np.ndarray:
    key = (np.uint64(field) << np.uint64(32)) + (ranks.astype(np.uint64) & np.uint64(0xFFFFFFFF))
    return (splitmix64(key) % np.uint64(F)).astype(np.int64)


def synthetic_batch(n_rows: int, num_features: int, *, seed: int = DEFAULT_SEED, batch_index: int = 0,
                    zipf_s: float = 1.05, labels: str = "binary", w_star: np.ndarray | None = None,
                    exact: bool = False) -> Batch:
    """One mini-batch of the synthetic workload (deterministic in (seed, batch_index)).  exact:
    numeric values and regression labels are not rounded to fp32 (the device rounds x to fp32 on
    upload and keeps labels in fp64; parity tests of that rounding use this)."""
    F = int(num_features)
    if F < N_FIELDS:
        raise ValueError("num_features must be >= 39")
    rng = np.random.default_rng([seed, batch_index])
    B = int(n_rows)
    ranks = rng.zipf(zipf_s, size=(B, N_FIELDS))
    ids = np.empty((B, N_FIELDS), dtype=np.int64)
    for f in range(N_FIELDS):
        ids[:, f] = _field_ids(f, ranks[:, f], F)
    vals = np.ones((B, N_FIELDS), dtype=np.float64)
    pois = rng.poisson(3.0, size=(B, N_NUMERIC))
    vals[:, :N_NUMERIC] = np.log1p(pois) if exact else np.log1p(pois).astype(np.float32).astype(np.float64)
    # re-draw colliding ids (rare: hash collisions mod F)
    srt = np.sort(ids, axis=1)
    bad = np.nonzero((srt[:, 1:] == srt[:, :-1]).any(axis=1))[0]
    for r in bad:
        seen = set()
        for f in range(N_FIELDS):
            while int(ids[r, f]) in seen:
                ids[r, f] = int(_field_ids(f, rng.zipf(zipf_s, size=1), F)[0])
            seen.add(int(ids[r, f]))
    order = np.argsort(ids, axis=1, kind="stable")
    ids = np.take_along_axis(ids, order, axis=1)
    vals = np.take_along_axis(vals, order, axis=1)
    if labels == "binary":
        y = (rng.random(B) < 0.25).astype(np.float64)
    elif labels == "regression":
        if w_star is None:
            raise ValueError("regression labels need w_star")
        y = (w_star[ids] * vals).sum(axis=1) + rng.normal(0.0, 0.1, B)
        if not exact:
            y = y.astype(np.float32).astype(np.float64)
    else:
        raise ValueError(labels)
    row_ptr = np.arange(B + 1, dtype=np.int64) * N_FIELDS
    return Batch(row_ptr=row_ptr, col=ids.reshape(-1).astype(np.int32), val=vals.reshape(-1), label=y)


def read_libsvm_csr(path: str):
    """Spark 2.1 ``libsvm`` data source for one file (MLUtils.parseLibSVMFile), parsed natively
    (fm_read_libsvm in libfm_hip.so).  Returns (labels, row_ptr, col, val, num_features)."""
    import ctypes as C

    from . import _native as N

    lib = N.load()
    b, nnz, nf = C.c_int64(), C.c_int64(), C.c_int64()
    bp = os.fsencode(path)
    N.check(lib.fm_read_libsvm(bp, 0, 0, None, None, None, None, C.byref(b), C.byref(nnz), C.byref(nf)),
            "fm_read_libsvm")
    labels = np.zeros(max(b.value, 1))
    row_ptr = np.zeros(b.value + 1, dtype=np.int64)
    col = np.zeros(max(nnz.value, 1), dtype=np.int32)
    val = np.zeros(max(nnz.value, 1))
    N.check(lib.fm_read_libsvm(bp, max(b.value, 1), max(nnz.value, 1), N.ptr(labels, C.c_double),
                               N.ptr(row_ptr, C.c_int64), N.ptr(col, C.c_int32), N.ptr(val, C.c_double),
                               C.byref(b), C.byref(nnz), C.byref(nf)), "fm_read_libsvm")
    return labels[: b.value], row_ptr, col[: nnz.value], val[: nnz.value], nf.value


def read_libsvm(path: str):
    """The same as (labels, rows, num_features) with rows as lists of (index, value) pairs."""
    labels, row_ptr, col, val, nf = read_libsvm_csr(path)
    rows = [list(zip(col[a:b].tolist(), val[a:b].tolist())) for a, b in zip(row_ptr[:-1], row_ptr[1:])]
    return labels, rows, nf


# ------------------------------------------------------------------ MovieLens features (demo)
MAX_USER_ID = 671       # FactorizationMachinesSample.scala:13
MAX_MOVIE_ID = 164979   # FactorizationMachinesSample.scala:14


def read_ratings_csv(path: str):
    """ratings.csv of ml-latest-small (header userId,movieId,rating,timestamp), the input of
    FactorizationMachinesSample.scala:97-102.  Returns (user_id, movie_id, rating) arrays."""
    users, movies, ratings = [], [], []
    with open(path) as fh:
        header = fh.readline().strip().split(",")
        iu, im, ir = header.index("userId"), header.index("movieId"), header.index("rating")
        for line in fh:
            if not line.strip():
                continue
            f = line.rstrip("\n").split(",")
            users.append(int(f[iu]))
            movies.append(int(f[im]))
            ratings.append(float(f[ir]))
    return np.asarray(users, np.int64), np.asarray(movies, np.int64), np.asarray(ratings, np.float64)


def movielens_features(user_id, movie_id, rating):
    """createRatingDataFrame (FactorizationMachinesSample.scala:75-128) as CSR rows.

    Per user, the set of distinct "movieId:rating" strings (collect_set); one row per element
    (explode) with label = rating and the sparse features of udfCrateFeatureVec (:76-95):
    userId -> 1.0, MaxUserId + movieId -> 1.0, and, when the user's set has at least two
    elements, every OTHER movie m of the set at MaxUserId + MaxMovieId + m with weight
    1 / (|set| - 1).  Vector size MaxUserId + 2 * MaxMovieId.  Spark leaves the row order of the
    groupBy unspecified; here users ascend and each user's rows follow (movieId, rating).
    Returns (labels, row_ptr, col, val, num_features)."""
    size = MAX_USER_ID + MAX_MOVIE_ID + MAX_MOVIE_ID
    by_user = {}
    for u, m, r in zip(np.asarray(user_id).tolist(), np.asarray(movie_id).tolist(), np.asarray(rating).tolist()):
        by_user.setdefault(int(u), set()).add((int(m), float(r)))  # collect_set of "movieId:rating"
    labels, row_ptr, cols, vals = [], [0], [], []
    for u in sorted(by_user):
        mr = sorted(by_user[u])
        for cur_m, cur_r in mr:  # explode(movieRatings)
            feat = {}
            if len(mr) >= 2:
                wgt = 1.0 / (len(mr) - 1.0)
                for m, _ in mr:
                    if m != cur_m:
                        feat[MAX_USER_ID + MAX_MOVIE_ID + m] = wgt
            feat[u] = 1.0
            feat[MAX_USER_ID + cur_m] = 1.0
            for i in sorted(feat):  # Vectors.sparse sorts by index
                if not 0 <= i < size:
                    raise ValueError(f"feature index {i} outside the vector size {size}")
                cols.append(i)
                vals.append(feat[i])
            labels.append(cur_r)
            row_ptr.append(len(cols))
    return (np.asarray(labels, np.float64), np.asarray(row_ptr, np.int64), np.asarray(cols, np.int32),
            np.asarray(vals, np.float64), size)
