"""Input formats either side of the hot path.

* ``synthetic_batch`` — the Criteo-shaped synthetic workload of BASELINE.md / SURVEY.md §8(d):
  39 fields per sample (13 numeric with x = log1p(Poisson(3)) rounded to fp32, 26
  categorical with x = 1.0).  Field f's feature id is splitmix64(f * 2^32 + rank) mod F
  with rank ~ Zipf(s) (s = 1.05, or 1.2 for the c5 skew); ids that collide inside a row are
  re-drawn, so every row holds 39 distinct ids in ascending order.  Labels are
  Bernoulli(0.25) ("binary") or <w*, x> + N(0, 0.1) ("regression", c5).
* ``read_libsvm`` — Spark's ``libsvm`` data source as used for data/sample.txt (config c1):
  1-based indices -> 0-based, every listed pair kept (explicit zeros stay active entries,
  SURVEY P5), features sized by the largest index.
"""

from __future__ import annotations

from dataclasses import dataclass

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
                    zipf_s: float = 1.05, labels: str = "binary", w_star: np.ndarray | None = None) -> Batch:
    """One mini-batch of the synthetic workload (deterministic in (seed, batch_index))."""
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
    vals[:, :N_NUMERIC] = np.log1p(pois).astype(np.float32).astype(np.float64)
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
        y = y.astype(np.float32).astype(np.float64)
    else:
        raise ValueError(labels)
    row_ptr = np.arange(B + 1, dtype=np.int64) * N_FIELDS
    return Batch(row_ptr=row_ptr, col=ids.reshape(-1).astype(np.int32), val=vals.reshape(-1), label=y)


def read_libsvm(path: str):
    """Spark 2.1 ``libsvm`` source semantics for one file (labels, 0-based sparse rows).
    Returns (labels, rows, num_features) with rows as lists of (index, value) pairs."""
    labels, rows = [], []
    max_idx = -1
    with open(path) as fh:
        for line in fh:
            line = line.split("#", 1)[0].strip()
            if not line:
                continue
            items = line.split()
            labels.append(float(items[0]))
            pairs = []
            prev = -1
            for it in items[1:]:
                i, v = it.split(":")
                idx = int(i) - 1
                if idx < 0 or idx <= prev:
                    raise ValueError(f"indices must be one-based and ascending: {line!r}")
                prev = idx
                pairs.append((idx, float(v)))
                max_idx = max(max_idx, idx)
            rows.append(pairs)
    return np.asarray(labels), rows, max_idx + 1
