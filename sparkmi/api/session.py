"""Session: a SparkSession-lite for MI355X executors.

Reference usage (re-provided without a JVM):
  * ``SparkSession.builder.appName(..).config("spark.executor.instances", ..).getOrCreate()``
    (mllib_multilayer_perceptron_classifier.py:12-19) and the empty-SparkConf +
    spark-submit form (distributed_cnn.py:41-43);
  * ``spark.sparkContext.getConf().get('spark.executor.instances')`` (distributed_cnn.py:43) —
    here defaulting to the visible MI355X count instead of crashing on ``int(None)`` (Q13);
  * ``spark.read.format("libsvm").load(path)`` (mllib_multilayer_perceptron_classifier.py:22-23);
  * ``spark.stop()``.
One executor = one process pinned to one MI355X (launched by :class:`Distributor`).
If a real pyspark is importable and ``SPARKMI_USE_PYSPARK=1``, ``getOrCreate`` returns a real
SparkSession instead (optional pass-through).
"""
import os
import threading

import numpy as np

from ..ml.linalg import VectorColumn
from .frame import Frame


class Conf:
    """SparkConf-lite."""

    def __init__(self, loadDefaults=True):
        self._conf = {}
        if loadDefaults:
            for k, v in os.environ.items():
                if k.startswith("SPARKMI_CONF_"):
                    self._conf[k[len("SPARKMI_CONF_"):].lower().replace("_", ".")] = v

    def set(self, key, value):
        self._conf[key] = str(value)
        return self

    def setAppName(self, name):
        return self.set("spark.app.name", name)

    def setMaster(self, master):
        return self.set("spark.master", master)

    def get(self, key, defaultValue=None):
        return self._conf.get(key, defaultValue)

    def getAll(self):
        return list(self._conf.items())

    def contains(self, key):
        return key in self._conf


def visible_gpus():
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


class _Context:
    def __init__(self, conf):
        self._conf = conf

    def getConf(self):
        return self._conf

    @property
    def defaultParallelism(self):
        return int(self._conf.get("spark.executor.instances", 1))

    def setLogLevel(self, level):
        self._conf.set("spark.log.level", level)


class DataFrameReader:
    def __init__(self, session):
        self._session = session
        self._format = None
        self._options = {}

    def format(self, fmt):
        self._format = fmt.lower()
        return self

    def option(self, key, value):
        self._options[key] = value
        return self

    def options(self, **kw):
        self._options.update(kw)
        return self

    def load(self, path=None, format=None, **options):
        fmt = (format or self._format or "libsvm").lower()
        self._options.update(options)
        if fmt == "libsvm":
            return self.libsvm(path, **self._options)
        if fmt == "parquet":
            return self.parquet(path)
        if fmt == "csv":
            return self.csv(path, **self._options)
        raise ValueError(f"unsupported format {fmt}")

    def libsvm(self, path_or_text, numFeatures=None, vectorType="sparse", text=False, **_):
        """libsvm -> Frame[label: double, features: vector] via the C++ parser (csrc/runtime/libsvm.cpp)."""
        from .. import _native
        RT = _native.RT()
        if text or (isinstance(path_or_text, str) and "\n" in path_or_text):
            labels, indptr, indices, values, maxi = RT.parse_libsvm_buffer(path_or_text, 4)
        else:
            labels, indptr, indices, values, maxi = RT.parse_libsvm_file(str(path_or_text), 4)
        nf = int(numFeatures) if numFeatures else int(maxi)
        if indices.size and indices.max() >= nf:
            raise ValueError(f"feature index {indices.max() + 1} exceeds numFeatures={nf}")
        col = VectorColumn(csr=(indptr, indices, values), size=nf)
        if vectorType == "dense":
            col = VectorColumn(dense=col.to_dense())
        n_parts = int(self._session.conf.get("spark.default.parallelism", self._session.num_executors))
        return Frame({"label": labels, "features": col}, num_partitions=n_parts, session=self._session)

    def parquet(self, path):
        import pyarrow.parquet as pq
        t = pq.read_table(path)
        return Frame({c: np.asarray(t.column(c).to_pylist()) for c in t.column_names}, session=self._session)

    def csv(self, path, header=True, inferSchema=True, sep=",", **_):
        import pandas as pd
        return Frame.from_pandas(pd.read_csv(path, sep=sep, header=0 if header else None), session=self._session)


class Session:
    _active = None
    _lock = threading.Lock()

    class Builder:
        def __init__(self):
            self._conf = Conf()

        def appName(self, name):
            self._conf.set("spark.app.name", name)
            return self

        def master(self, m):
            self._conf.set("spark.master", m)
            return self

        def config(self, key=None, value=None, conf=None):
            if conf is not None:
                for k, v in conf.getAll():
                    self._conf.set(k, v)
            if key is not None:
                self._conf.set(key, value)
            return self

        def getOrCreate(self):
            if os.environ.get("SPARKMI_USE_PYSPARK") == "1":
                try:  # optional pass-through to a real Spark
                    from pyspark.sql import SparkSession
                    b = SparkSession.builder
                    for k, v in self._conf.getAll():
                        b = b.config(k, v)
                    return b.getOrCreate()
                except ImportError:
                    pass
            with Session._lock:
                if Session._active is None:
                    Session._active = Session(self._conf)
                else:
                    for k, v in self._conf.getAll():
                        Session._active.conf.set(k, v)
                return Session._active

    builder = None  # set below (class attribute like SparkSession.builder)

    def __init__(self, conf=None):
        self.conf = conf or Conf()
        if not self.conf.contains("spark.executor.instances"):
            # Q13: default to one executor per visible MI355X (at least one)
            self.conf.set("spark.executor.instances", max(1, visible_gpus()))
        self.sparkContext = _Context(self.conf)
        self.read = DataFrameReader(self)
        self._stopped = False

    @property
    def num_executors(self):
        return int(self.conf.get("spark.executor.instances", 1))

    @property
    def version(self):
        return "3.5.0-sparkmi"

    def createDataFrame(self, data, schema=None):
        try:
            import pandas as pd
            if isinstance(data, pd.DataFrame):
                return Frame.from_pandas(data, session=self)
        except ImportError:  # pragma: no cover
            pass
        if isinstance(data, dict):
            return Frame(data, session=self)
        return Frame.from_rows(data, schema, session=self)

    def range(self, n):
        return Frame({"id": np.arange(n)}, session=self)

    def stop(self):
        self._stopped = True
        with Session._lock:
            if Session._active is self:
                Session._active = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()


class _BuilderDescriptor:
    def __get__(self, obj, cls):
        return Session.Builder()


Session.builder = _BuilderDescriptor()
SparkSession = Session
SparkConf = Conf
