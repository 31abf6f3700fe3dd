"""CPU: the randomSplit replay.  The C++ implementation behind the C-ABI (fm_random_split)
against the pure-Python restatement (oracle/spark_sampler.py) — bit-exact split assignment,
sampleIds and per-partition order.  MurmurHash3 is pinned to the SMHasher verification
value; agreement with a live Spark 2.1.0 is unverifiable offline (no JVM in this image)."""

import numpy as np
import pytest

from fm_spark_amd import sampler as S
from fm_spark_amd.linalg import DenseVector, SparseVector, Vectors
from oracle import spark_sampler as O


def smhasher_verification(h):
    key = bytes(range(256))
    out = b""
    for i in range(256):
        out += h(key[:i], 256 - i).to_bytes(4, "little")
    return h(out, 0)


def test_murmur3_smhasher_vector():
    assert smhasher_verification(O.murmur3_bytes_hash) == 0xB0F57EE3
    assert smhasher_verification(S.murmur3) == 0xB0F57EE3


@pytest.mark.parametrize("seed", [0, 1, 1234, 1235, -7, 2**62 + 11])
def test_hash_seed_and_stream(seed):
    assert S.hash_seed(seed) == O.hash_seed(seed)
    r = O.XORShiftRandom(seed)
    want = [r.next_double() for _ in range(257)]
    got = S.next_doubles(seed, 257)
    assert got.tolist() == want
    assert all(0.0 <= x < 1.0 for x in want)


def test_normalized_weights_match_scanleft():
    w = [0.1] * 10
    cum = O.normalized_cum_weights(w)
    assert cum[0] == 0.0 and len(cum) == 11
    with pytest.raises(ValueError):
        O.normalized_cum_weights([0.0, 0.0])
    with pytest.raises(ValueError):
        O.normalized_cum_weights([0.5, -0.1])


def _rows(rng, n, kinds=("dense", "sparse"), ties=True):
    labels, vecs = [], []
    for i in range(n):
        y = float(rng.integers(0, 3)) if ties else float(rng.normal())
        if rng.random() < 0.5 and "dense" in kinds:
            v = Vectors.dense(np.round(rng.normal(size=3), 1) if ties else rng.normal(size=3))
        else:
            z = int(rng.integers(0, 4))
            idx = np.sort(rng.choice(6, size=z, replace=False))
            v = SparseVector(6, idx, np.round(rng.normal(size=z), 1))
        labels.append(y)
        vecs.append(v)
    return labels, vecs


def _oracle_rows(labels, vecs, extra=None):
    out = []
    for i, (y, v) in enumerate(zip(labels, vecs)):
        if isinstance(v, DenseVector):
            ov = O_vec(v.size, v.values, None)
        else:
            ov = O_vec(v.size, v.values, v.indices)
        out.append({"label": y, "features": ov, "extra": extra[i] if extra is not None else 0})
    return out


class O_vec:
    def __init__(self, size, values, indices):
        self.size, self.values, self.indices = size, values, indices


@pytest.mark.parametrize("order", ["LF", "FL", "IF", "ILF"])
@pytest.mark.parametrize("parts", [[40], [10, 17, 0, 13]])
def test_random_split_matches_restatement(order, parts):
    rng = np.random.default_rng(len(order) * 7 + len(parts))
    n = sum(parts)
    labels, vecs = _rows(rng, n)
    extra = rng.integers(0, 5, n)
    weights = [0.2] * 5
    split_of, sid, ordr = S.random_split(parts, labels, vecs, weights, 1234, order, extra=extra)
    # oracle
    rows = _oracle_rows(labels, vecs, extra)
    partitions, off = [], 0
    for p in parts:
        partitions.append(rows[off:off + p])
        off += p
    splits, sample_id = O.random_split(partitions, weights, 1234, order)
    want_split = np.full(n, -1)
    want_order = []
    off = 0
    starts = np.concatenate([[0], np.cumsum(parts)])
    for i, sp in enumerate(splits):
        for (p, r) in sp:
            want_split[starts[p] + r] = i
    assert split_of.tolist() == want_split.tolist()
    for p in range(len(parts)):
        for r in range(parts[p]):
            assert sid[starts[p] + r] == sample_id[(p, r)] == (p << 33) + r
    # the splits are disjoint and (up to the last cumulative bound's rounding) cover every row
    assert (split_of >= 0).sum() >= n - 1


def test_random_split_row_order_is_spark_ordering():
    labels = [1.0, 0.0, 1.0, 0.0]
    vecs = [Vectors.dense(1.0, 0.0), Vectors.sparse(2, [(1, 5.0)]), Vectors.sparse(2, [(0, 1.0)]),
            Vectors.dense(0.5, 0.5)]
    _, _, order = S.random_split([4], labels, vecs, [1.0], 1234, "LF")
    # label asc; for ties the struct: sparse (type 0) before dense (type 1)
    assert order.tolist() == [1, 3, 2, 0]


def test_random_split_rejects_bad_weights():
    from fm_spark_amd._native import FMError

    with pytest.raises(FMError):
        S.random_split([1], [0.0], [Vectors.dense(1.0)], [0.0, 0.0], 1, "LF")


def test_random_split_csr_matches_vector_rows():
    """The CSR entry point (no Vector objects: the bench's multi-million-row resident-fit dataset)
    gives the split, sampleId and order of the same rows as SparseVectors."""
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.linalg import SparseVector

    b = synthetic_batch(3000, 5000, batch_index=3)
    vecs = [SparseVector(5000, b.col[b.row_ptr[i]:b.row_ptr[i + 1]], b.val[b.row_ptr[i]:b.row_ptr[i + 1]])
            for i in range(b.n_rows)]
    parts = [700, 800, 0, 1500]
    want = S.random_split(parts, b.label, vecs, [0.1] * 8, 1234, "LF")
    got = S.random_split_csr(parts, b.label, b.row_ptr, b.col, b.val, 5000, [0.1] * 8, 1234)
    for x, y in zip(got, want):
        assert np.array_equal(x, y)
