"""Frame: a DataFrame-lite (columnar, in-memory, partition-aware) with the pyspark.sql surface
the reference uses: ``spark.read.format("libsvm").load`` -> ``randomSplit`` ->
``toPandas`` / ``select`` / ``transform`` (mllib_multilayer_perceptron_classifier.py:22-48,
distributed_multilayer_perceptron.py:62-66).

Columns are numpy arrays (scalars) or :class:`VectorColumn` (features).  A frame carries a
partition count; ``partition(i, n)`` yields executor ``i``'s disjoint shard (what Spark's
partitions + a *correct* DistributedSampler would give).
"""
from collections import OrderedDict, namedtuple

import numpy as np

from ..ml.linalg import Vector, VectorColumn


class Row(tuple):
    """pyspark.sql.Row-like: attribute and key access."""

    def __new__(cls, fields, values):
        r = super().__new__(cls, values)
        r._fields = tuple(fields)
        return r

    def __getattr__(self, k):
        try:
            return self[self._fields.index(k)]
        except ValueError:
            raise AttributeError(k)

    def __getitem__(self, k):
        if isinstance(k, str):
            return tuple.__getitem__(self, self._fields.index(k))
        return tuple.__getitem__(self, k)

    def asDict(self):
        return dict(zip(self._fields, self))

    def __repr__(self):
        return "Row(" + ", ".join(f"{k}={v!r}" for k, v in zip(self._fields, self)) + ")"


class Frame:
    def __init__(self, columns, num_partitions=1, session=None):
        self._cols = OrderedDict()
        n = None
        for k, v in columns.items():
            if not isinstance(v, VectorColumn):
                v = np.asarray(v)
            ln = len(v)
            if n is None:
                n = ln
            elif ln != n:
                raise ValueError(f"column {k} has {ln} rows, expected {n}")
            self._cols[k] = v
        self._n = n or 0
        self.num_partitions = max(1, int(num_partitions))
        self.session = session

    # -- schema ---------------------------------------------------------------------------
    @property
    def columns(self):
        return list(self._cols.keys())

    @property
    def dtypes(self):
        out = []
        for k, v in self._cols.items():
            out.append((k, "vector" if isinstance(v, VectorColumn) else str(v.dtype)))
        return out

    def printSchema(self):
        print("root")
        for k, t in self.dtypes:
            print(f" |-- {k}: {t}")

    def count(self):
        return self._n

    def __len__(self):
        return self._n

    def column(self, name):
        return self._cols[name]

    # -- relational ops -------------------------------------------------------------------
    def select(self, *cols):
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = cols[0]
        return Frame(OrderedDict((c, self._cols[c]) for c in cols), self.num_partitions, self.session)

    def withColumn(self, name, values):
        cols = OrderedDict(self._cols)
        cols[name] = values
        return Frame(cols, self.num_partitions, self.session)

    def drop(self, *cols):
        return Frame(OrderedDict((k, v) for k, v in self._cols.items() if k not in cols), self.num_partitions,
                     self.session)

    def take_rows(self, rows):
        cols = OrderedDict()
        for k, v in self._cols.items():
            cols[k] = v.take(rows) if isinstance(v, VectorColumn) else v[np.asarray(rows, dtype=np.int64)]
        return Frame(cols, self.num_partitions, self.session)

    def filter(self, mask):
        return self.take_rows(np.nonzero(np.asarray(mask))[0])

    def limit(self, n):
        return self.take_rows(np.arange(min(n, self._n)))

    def union(self, other):
        cols = OrderedDict()
        for k in self.columns:
            a, b = self._cols[k], other._cols[k]
            if isinstance(a, VectorColumn):
                cols[k] = VectorColumn(dense=np.concatenate([a.to_dense(), b.to_dense()]))
            else:
                cols[k] = np.concatenate([a, b])
        return Frame(cols, self.num_partitions, self.session)

    def randomSplit(self, weights, seed=None):
        """Seeded Bernoulli split (Spark semantics: each row falls into the bucket of a uniform draw
        against the normalised cumulative weights).  Spark draws per partition with XORShiftRandom
        after a local sort; sparkmi draws one PCG64 stream over the rows — splits are deterministic
        in ``seed`` but not bit-identical to Spark's."""
        w = np.asarray(weights, dtype=np.float64)
        if (w < 0).any() or w.sum() <= 0:
            raise ValueError("weights must be non-negative with a positive sum")
        cum = np.cumsum(w / w.sum())
        rng = np.random.default_rng(seed if seed is not None else np.random.SeedSequence().entropy)
        u = rng.random(self._n)
        bucket = np.searchsorted(cum, u, side="right")
        return [self.take_rows(np.nonzero(bucket == i)[0]) for i in range(len(w))]

    def repartition(self, n):
        return Frame(OrderedDict(self._cols), n, self.session)

    def coalesce(self, n):
        return self.repartition(min(n, self.num_partitions))

    def cache(self):
        return self

    persist = cache

    def partition(self, index, num=None):
        """Rows of partition ``index`` of ``num`` (default: this frame's partitions): contiguous
        near-equal ranges, disjoint and covering."""
        num = num or self.num_partitions
        if not 0 <= index < num:
            raise IndexError(index)
        bounds = np.linspace(0, self._n, num + 1).astype(np.int64)
        return self.take_rows(np.arange(bounds[index], bounds[index + 1]))

    # -- materialisation -------------------------------------------------------------------
    def collect(self):
        names = self.columns
        cols = [self._cols[k] for k in names]
        out = []
        for i in range(self._n):
            vals = []
            for c in cols:
                if isinstance(c, VectorColumn):
                    vals.append(c.row(i))
                else:
                    v = c[i]
                    vals.append(v.item() if hasattr(v, "item") and np.ndim(v) == 0 else v)
            out.append(Row(names, vals))
        return out

    def head(self, n=1):
        return self.limit(n).collect()

    def first(self):
        r = self.head(1)
        return r[0] if r else None

    def show(self, n=20, truncate=True):
        rows = self.head(n)
        print(" | ".join(self.columns))
        for r in rows:
            print(" | ".join(str(v)[:20] if truncate else str(v) for v in r))

    def toPandas(self):
        import pandas as pd
        data = OrderedDict()
        for k, v in self._cols.items():
            data[k] = v.to_objects() if isinstance(v, VectorColumn) else v
        return pd.DataFrame(data)

    def to_numpy(self, features_col="features", label_col="label"):
        """(X float64 [n,F], y float64 [n]) — the fast path the trainers use (no per-row objects)."""
        X = self._cols[features_col].to_dense() if isinstance(self._cols[features_col], VectorColumn) else \
            np.asarray(self._cols[features_col], np.float64)
        y = np.asarray(self._cols[label_col], np.float64) if label_col in self._cols else None
        return X, y

    def to_torch(self, features_col="features", label_col="label", device="cpu"):
        import torch
        X, y = self.to_numpy(features_col, label_col)
        xt = torch.as_tensor(X, dtype=torch.float32, device=device)
        yt = torch.as_tensor(y, dtype=torch.int64, device=device) if y is not None else None
        return xt, yt

    @staticmethod
    def from_rows(rows, schema=None, session=None):
        rows = list(rows)
        if not rows:
            return Frame({}, session=session)
        if schema is None:
            if hasattr(rows[0], "asDict"):
                schema = list(rows[0].asDict().keys())
            elif isinstance(rows[0], dict):
                schema = list(rows[0].keys())
            else:
                schema = [f"_{i + 1}" for i in range(len(rows[0]))]
        cols = OrderedDict()
        for j, name in enumerate(schema):
            vals = [r[name] if isinstance(r, dict) else r[j] for r in rows]
            if isinstance(vals[0], Vector):
                cols[name] = VectorColumn.from_objects(vals)
            else:
                cols[name] = np.asarray(vals)
        return Frame(cols, session=session)

    @staticmethod
    def from_pandas(df, session=None):
        cols = OrderedDict()
        for k in df.columns:
            vals = df[k].values
            if len(vals) and isinstance(vals[0], Vector):
                cols[k] = VectorColumn.from_objects(vals)
            else:
                cols[k] = np.asarray(vals)
        return Frame(cols, session=session)

    def __repr__(self):
        return f"Frame[{', '.join(f'{k}: {t}' for k, t in self.dtypes)}] ({self._n} rows, {self.num_partitions} partitions)"
