"""pyspark.ml.linalg-compatible vectors (DenseVector / SparseVector / Vectors factory).

Spark's libsvm reader yields SparseVector features; the reference converts them with
``x.toArray()`` (distributed_multilayer_perceptron.py:69-71).  These classes give the same
surface so reference-style code runs unchanged on sparkmi frames.
"""
import numpy as np


class Vector:
    def toArray(self):
        raise NotImplementedError

    def __len__(self):
        return self.size

    def __eq__(self, other):
        return isinstance(other, Vector) and self.size == other.size and np.array_equal(self.toArray(),
                                                                                        other.toArray())

    def __hash__(self):
        return hash(self.toArray().tobytes())


class DenseVector(Vector):
    def __init__(self, values):
        self.values = np.asarray(values, dtype=np.float64).reshape(-1)

    @property
    def size(self):
        return int(self.values.shape[0])

    def toArray(self):
        return self.values

    def __getitem__(self, i):
        return float(self.values[i])

    def dot(self, other):
        return float(np.dot(self.values, other.toArray() if isinstance(other, Vector) else np.asarray(other)))

    def norm(self, p=2):
        return float(np.linalg.norm(self.values, p))

    def numNonzeros(self):
        return int(np.count_nonzero(self.values))

    def __repr__(self):
        return f"DenseVector({self.values.tolist()})"


class SparseVector(Vector):
    def __init__(self, size, indices, values=None):
        self._size = int(size)
        if values is None and isinstance(indices, dict):
            items = sorted(indices.items())
            indices = [k for k, _ in items]
            values = [v for _, v in items]
        self.indices = np.asarray(indices, dtype=np.int32).reshape(-1)
        self.values = np.asarray(values, dtype=np.float64).reshape(-1)

    @property
    def size(self):
        return self._size

    def toArray(self):
        a = np.zeros(self._size, dtype=np.float64)
        a[self.indices] = self.values
        return a

    def __getitem__(self, i):
        j = np.searchsorted(self.indices, i)
        if j < len(self.indices) and self.indices[j] == i:
            return float(self.values[j])
        return 0.0

    def numNonzeros(self):
        return int(np.count_nonzero(self.values))

    def __repr__(self):
        return f"SparseVector({self._size}, {dict(zip(self.indices.tolist(), self.values.tolist()))})"


class Vectors:
    @staticmethod
    def dense(*values):
        if len(values) == 1 and not isinstance(values[0], (int, float)):
            return DenseVector(values[0])
        return DenseVector(values)

    @staticmethod
    def sparse(size, *args):
        if len(args) == 1:
            return SparseVector(size, args[0])
        return SparseVector(size, args[0], args[1])

    @staticmethod
    def zeros(size):
        return DenseVector(np.zeros(size))


class VectorColumn:
    """Columnar storage of a vector column: dense float64 matrix or CSR (libsvm reads)."""

    def __init__(self, dense=None, csr=None, size=None):
        self.dense = dense
        self.csr = csr  # (indptr, indices, values)
        if dense is not None:
            self.size = dense.shape[1]
            self.n = dense.shape[0]
        else:
            self.size = int(size)
            self.n = len(csr[0]) - 1

    def __len__(self):
        return self.n

    def to_dense(self):
        if self.dense is not None:
            return self.dense
        indptr, idx, val = self.csr
        out = np.zeros((self.n, self.size), dtype=np.float64)
        rows = np.repeat(np.arange(self.n), np.diff(indptr))
        out[rows, idx] = val
        return out

    def take(self, rows):
        rows = np.asarray(rows, dtype=np.int64)
        if self.dense is not None:
            return VectorColumn(dense=self.dense[rows])
        indptr, idx, val = self.csr
        counts = np.diff(indptr)[rows]
        new_ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        sel = np.concatenate([np.arange(indptr[r], indptr[r + 1]) for r in rows]) if len(rows) else np.zeros(0, np.int64)
        return VectorColumn(csr=(new_ptr, idx[sel], val[sel]), size=self.size)

    def row(self, i):
        if self.dense is not None:
            return DenseVector(self.dense[i])
        indptr, idx, val = self.csr
        return SparseVector(self.size, idx[indptr[i]:indptr[i + 1]], val[indptr[i]:indptr[i + 1]])

    def to_objects(self):
        return [self.row(i) for i in range(self.n)]

    @staticmethod
    def from_objects(vs):
        vs = list(vs)
        if not vs:
            return VectorColumn(dense=np.zeros((0, 0)))
        return VectorColumn(dense=np.stack([v.toArray() if isinstance(v, Vector) else np.asarray(v, np.float64)
                                            for v in vs]))
