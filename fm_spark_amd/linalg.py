"""org.apache.spark.ml.linalg.{Vector, Vectors, DenseVector, SparseVector} as used by the
reference (FactorizationMachinesModel.scala:5, FactorizationMachinesSuite.scala:34-53)."""

from __future__ import annotations

import numpy as np


class Vector:
    size: int

    def foreach_active(self):
        """Vector.foreachActive: every index of a DenseVector, every stored entry of a
        SparseVector (explicit zeros included)."""
        raise NotImplementedError

    def to_array(self) -> np.ndarray:
        raise NotImplementedError

    def __len__(self):
        return self.size


class DenseVector(Vector):
    def __init__(self, values):
        self.values = np.asarray(values, dtype=np.float64).reshape(-1)
        self.size = len(self.values)

    def foreach_active(self):
        return zip(range(self.size), self.values.tolist())

    def to_array(self):
        return self.values.copy()

    def to_sparse(self) -> "SparseVector":
        nz = np.nonzero(self.values)[0]
        return SparseVector(self.size, nz, self.values[nz])

    toSparse = to_sparse

    def __eq__(self, other):
        return isinstance(other, Vector) and self.size == other.size and np.array_equal(self.to_array(),
                                                                                     other.to_array())

    def __repr__(self):
        return f"DenseVector({self.values.tolist()})"


class SparseVector(Vector):
    def __init__(self, size, indices, values):
        self.size = int(size)
        self.indices = np.asarray(indices, dtype=np.int32).reshape(-1)
        self.values = np.asarray(values, dtype=np.float64).reshape(-1)
        if len(self.indices) != len(self.values):
            raise ValueError("indices and values must have the same length")

    def foreach_active(self):
        return zip(self.indices.tolist(), self.values.tolist())

    def to_array(self):
        out = np.zeros(self.size)
        out[self.indices] = self.values
        return out

    def to_dense(self) -> DenseVector:
        return DenseVector(self.to_array())

    toDense = to_dense

    def __eq__(self, other):
        return isinstance(other, Vector) and self.size == other.size and np.array_equal(self.to_array(),
                                                                                     other.to_array())

    def __repr__(self):
        return f"SparseVector({self.size}, {self.indices.tolist()}, {self.values.tolist()})"


class Vectors:
    @staticmethod
    def dense(*values) -> DenseVector:
        if len(values) == 1 and not np.isscalar(values[0]):
            return DenseVector(values[0])
        return DenseVector(values)

    @staticmethod
    def sparse(size, *args) -> SparseVector:
        """Vectors.sparse(size, Seq[(Int, Double)]) or Vectors.sparse(size, indices, values).
        Pairs are sorted by index and duplicate indices rejected, as Spark does."""
        if len(args) == 1:
            pairs = sorted(((int(i), float(v)) for i, v in args[0]), key=lambda p: p[0])
            for a, b in zip(pairs, pairs[1:]):
                if a[0] == b[0]:
                    raise ValueError(f"Found duplicate indices: {a[0]}.")
            return SparseVector(size, [p[0] for p in pairs], [p[1] for p in pairs])
        return SparseVector(size, args[0], args[1])

    @staticmethod
    def zeros(size) -> DenseVector:
        return DenseVector(np.zeros(size))


def active_map(vec: Vector) -> dict:
    """udfVecToMap (FactorizationMachinesModel.scala:244-250): index -> value over the
    active entries, last value per index."""
    m = {}
    for i, v in vec.foreach_active():
        m[int(i)] = float(v)
    return m
