"""CPU oracle — TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the mini-batch sampler the reference relies on:
``dfData.randomSplit(Array.fill(maxIter)(miniBatchFraction), 1234L)``
(FactorizationMachinesSGD.scala:111-112) plus ``monotonically_increasing_id``
(FactorizationMachinesModel.scala:268-272).

The algorithm lives in third-party code that is NOT vendored in /root/reference:
spark-core_2.11 / spark-sql_2.11 **2.1.0** (build.sbt:7-12) and scala-library 2.11.8
(MurmurHash3).  Restated from the published sources of those versions:

  Dataset.randomSplit(weights, seed)                      [spark-sql 2.1.0]
      require(weights.forall(_ >= 0)); require(weights.sum > 0)
      sorted = Sort(all output columns, Ascending, global = false)   (per partition)
      normalizedCumWeights = weights.map(_ / sum).scanLeft(0.0d)(_ + _)
      split i = Sample(lb_i, ub_i, withReplacement = false, seed, sorted)
  SampleExec -> RDD.randomSampleWithRange(lb, ub, seed)   [spark-core 2.1.0]
      mapPartitionsWithIndex: BernoulliCellSampler(lb, ub).setSeed(seed + index)
  BernoulliCellSampler.sample: keep item iff lb <= rng.nextDouble() < ub
      (ub - lb <= 0 keeps nothing)
  XORShiftRandom(init): seed = hashSeed(init); next(bits):
      s ^= s << 21; s ^= s >>> 35; s ^= s << 4; return (s & ((1L << bits) - 1)).toInt
  XORShiftRandom.hashSeed(seed):
      bytes = ByteBuffer.allocate(java.lang.Long.SIZE /* = 64 */).putLong(seed).array()
      lo = MurmurHash3.bytesHash(bytes)          (seed = arraySeed 0x3c074a61)
      hi = MurmurHash3.bytesHash(bytes, lo)
      (hi.toLong << 32) | (lo.toLong & 0xFFFFFFFFL)
  java.util.Random.nextDouble = ((next(26).toLong << 27) + next(27)) * 2^-53
  monotonically_increasing_id = (partitionIndex << 33) + rowIndexInPartition

Sort order of the row ``(columns..., sampleId)``: Spark's ascending ordering with nulls
first; doubles by nanSafeCompare (NaN largest, -0.0 == 0.0); the VectorUDT column is the
struct (type: byte, size: int, indices: array<int>, values: array<double>) with
sparse = 0 / dense = 1 (dense: size and indices null); arrays compare element-wise then
shorter-first.

Parity status: bit-exactness against a live Spark 2.1.0 is UNVERIFIABLE offline (no JVM in
this image).  MurmurHash3 is pinned to the SMHasher verification value (tests).
"""

from __future__ import annotations

import math

M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF
ARRAY_SEED = 0x3C074A61


def _rotl32(x: int, r: int) -> int:
    return ((x << r) | (x >> (32 - r))) & M32


def _mix_last(h: int, k: int) -> int:
    k = (k * 0xCC9E2D51) & M32
    k = _rotl32(k, 15)
    k = (k * 0x1B873593) & M32
    return h ^ k


def _mix(h: int, k: int) -> int:
    h = _mix_last(h, k)
    h = _rotl32(h, 13)
    return (h * 5 + 0xE6546B64) & M32


def _finalize(h: int, length: int) -> int:
    h ^= length & M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def murmur3_bytes_hash(data: bytes, seed: int = ARRAY_SEED) -> int:
    """scala.util.hashing.MurmurHash3.bytesHash (scala-library 2.11.8): MurmurHash3_x86_32.
    Returns the value as an unsigned 32-bit int."""
    h = seed & M32
    n = len(data)
    i = 0
    while n - i >= 4:
        k = data[i] | (data[i + 1] << 8) | (data[i + 2] << 16) | (data[i + 3] << 24)
        h = _mix(h, k)
        i += 4
    rem = n - i
    if rem:
        k = 0
        if rem == 3:
            k ^= data[i + 2] << 16
        if rem >= 2:
            k ^= data[i + 1] << 8
        k ^= data[i]
        h = _mix_last(h, k)
    return _finalize(h, n)


def _to_signed32(x: int) -> int:
    return x - (1 << 32) if x & 0x80000000 else x


def _to_signed64(x: int) -> int:
    x &= M64
    return x - (1 << 64) if x & (1 << 63) else x


def hash_seed(seed: int) -> int:
    """XORShiftRandom.hashSeed (spark-core 2.1.0) as a signed 64-bit value."""
    b = (seed & M64).to_bytes(8, "big") + bytes(56)  # ByteBuffer.allocate(Long.SIZE = 64)
    lo = murmur3_bytes_hash(b, ARRAY_SEED)
    hi = murmur3_bytes_hash(b, lo)  # bytesHash(bytes, lowBits): seed is the signed int
    val = ((_to_signed32(hi) << 32) | lo) & M64  # lowBits & 0xFFFFFFFFL
    return _to_signed64(val)


class XORShiftRandom:
    """org.apache.spark.util.random.XORShiftRandom (spark-core 2.1.0)."""

    def __init__(self, seed: int):
        self.s = hash_seed(seed) & M64

    def next_bits(self, bits: int) -> int:
        s = self.s
        s ^= (s << 21) & M64
        s ^= s >> 35  # >>> on the 64-bit pattern
        s ^= (s << 4) & M64
        self.s = s
        return s & ((1 << bits) - 1)  # then .toInt; bits <= 27 so always non-negative

    def next_double(self) -> float:
        return ((self.next_bits(26) << 27) + self.next_bits(27)) * (1.0 / (1 << 53))


# ------------------------------------------------------------------ Spark row ordering
def _double_key(x: float):
    if math.isnan(x):
        return (1, 0.0)
    return (0, x + 0.0)


def _vector_key(vec):
    """VectorUDT.sqlType struct, nulls first: (type, size, indices, values)."""
    if vec.indices is None:  # dense: type 1, size null, indices null
        return (1, (0,), (0,), (1, tuple(_double_key(float(v)) for v in vec.values)))
    return (0, (1, int(vec.size)), (1, tuple(int(i) for i in vec.indices)),
            (1, tuple(_double_key(float(v)) for v in vec.values)))


def row_sort_key(row, column_order: str, sample_id: int):
    key = []
    for c in column_order:
        if c == "L":
            key.append(_double_key(float(row["label"])))
        elif c == "F":
            key.append(_vector_key(row["features"]))
        elif c == "I":
            key.append(int(row["extra"]))
        else:
            raise ValueError(c)
    key.append(sample_id)
    return tuple(key)


def normalized_cum_weights(weights) -> list[float]:
    """weights.map(_ / sum).scanLeft(0.0d)(_ + _) with sum = weights.sum (sequential)."""
    if any(w < 0 for w in weights):
        raise ValueError("Weights must be nonnegative")
    total = 0.0
    for w in weights:
        total += w
    if not total > 0:
        raise ValueError("Sum of weights must be positive")
    out = [0.0]
    acc = 0.0
    for w in weights:
        acc = acc + w / total
        out.append(acc)
    return out


def random_split(partitions, weights, seed: int, column_order: str = "LF"):
    """Returns (splits, sample_id) where splits[i] is the list of (partition, row) pairs of
    split i in sorted per-partition order and sample_id[(p, r)] = (p << 33) + r."""
    cum = normalized_cum_weights(weights)
    sample_id = {}
    splits = [[] for _ in weights]
    for p, rows in enumerate(partitions):
        ids = [(p << 33) + r for r in range(len(rows))]
        for r, sid in enumerate(ids):
            sample_id[(p, r)] = sid
        order = sorted(range(len(rows)), key=lambda r: row_sort_key(rows[r], column_order, ids[r]))
        for i in range(len(weights)):
            lb, ub = cum[i], cum[i + 1]
            if ub - lb <= 0.0:
                continue
            rng = XORShiftRandom(seed + p)
            for r in order:
                x = rng.next_double()
                if lb <= x < ub:
                    splits[i].append((p, r))
    return splits, sample_id


def parallelize_slices(n: int, num_slices: int):
    """ParallelCollectionRDD.slice positions (spark-core 2.1.0): slice i covers
    [i*n/numSlices, (i+1)*n/numSlices) in Long arithmetic — the partitioning of
    spark.createDataFrame(localSeq) on local[numSlices]."""
    return [((i * n) // num_slices, ((i + 1) * n) // num_slices) for i in range(num_slices)]
