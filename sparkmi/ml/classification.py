"""MultilayerPerceptronClassifier / MultilayerPerceptronClassificationModel — the Spark MLlib
estimator of mllib_multilayer_perceptron_classifier.py:32-48, re-provided GPU-natively.

Semantics:
  * topology = affine + sigmoid hidden layers, affine + softmax-CE output (same model as the
    reference's PyTorch MLP, R03);
  * weights = ONE flat vector, per layer W as a column-major numOut x numIn matrix (element
    (o,i) at i*numOut+o) followed by b — identical to Spark, so saved models are
    interchangeable in structure;
  * rows are stacked into blocks of ``blockSize``; the objective is the mean over blocks of the
    per-block mean CE (per-row weights 1/(|block| * nblocks));
  * solver "l-bfgs" (memory 10, tol, maxIter) or "gd" (full-batch, step stepSize/sqrt(t));
  * default init (rand * 4.8 - 2.4)/sqrt(numIn) per layer from ``seed``.
Compute: the objective and gradient come from the fused HIP MLP kernels (sparkmi/ops/mlp.py)
on the executor's GPU when one is visible (the whole dataset resident in HBM), CPU torch
otherwise.  ``transform`` appends rawPrediction / probability / prediction columns.
Persistence: ``write().overwrite().save(path)`` / ``load(path)`` in Spark's on-disk layout
(metadata/part-00000 JSON + data/part-00000-*.parquet with a VectorUDT ``weights`` struct).
"""
import json
import os
import shutil
import time
import uuid

import numpy as np
import torch

from .base import Estimator, Model
from .linalg import DenseVector, VectorColumn
from .param import (HasBlockSize, HasFeaturesCol, HasLabelCol, HasMaxIter, HasPredictionCol, HasProbabilityCol,
                    HasRawPredictionCol, HasSeed, HasSolver, HasStepSize, HasTol, Param, TypeConverters,
                    apply_mixin_defaults)

SPARK_VERSION = "3.5.0"


# ---------------- weight layout helpers (Spark flat vector <-> torch tensors) -------------
def num_weights(layers):
    return sum(layers[i + 1] * (layers[i] + 1) for i in range(len(layers) - 1))


def unpack_weights(flat, layers):
    """Spark flat weights -> lists of torch-layout W [out,in] and b [out] (views)."""
    Ws, bs = [], []
    off = 0
    for i in range(len(layers) - 1):
        nin, nout = layers[i], layers[i + 1]
        Wcm = flat[off:off + nin * nout].reshape(nin, nout)  # column-major (o,i) at i*nout+o
        Ws.append(Wcm.t())
        off += nin * nout
        bs.append(flat[off:off + nout])
        off += nout
    return Ws, bs


def pack_weights(Ws, bs):
    parts = []
    for W, b in zip(Ws, bs):
        parts.append(W.t().reshape(-1))
        parts.append(b.reshape(-1))
    return torch.cat(parts)


def init_weights(layers, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(len(layers) - 1):
        nin, nout = layers[i], layers[i + 1]
        out.append((rng.random(nout * (nin + 1)) * 4.8 - 2.4) / np.sqrt(nin))
    return np.concatenate(out)


def block_row_weights(n, block_size):
    """Per-row weights realising Spark's block-averaged objective: mean over blocks of block means."""
    nb = max(1, (n + block_size - 1) // block_size)
    w = np.empty(n, dtype=np.float64)
    for b in range(nb):
        s, e = b * block_size, min(n, (b + 1) * block_size)
        w[s:e] = 1.0 / ((e - s) * nb)
    return w


def _device():
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


class _MLPParams(HasFeaturesCol, HasLabelCol, HasPredictionCol, HasMaxIter, HasTol, HasSeed, HasStepSize, HasSolver,
                 HasBlockSize, HasProbabilityCol, HasRawPredictionCol):
    layers = Param("undefined", "layers", "Sizes of layers from input layer to output layer E.g., Array(780, 100, "
                   "10) means 780 inputs, one hidden layer with 100 neurons and output layer of 10 neurons.",
                   TypeConverters.toListInt)
    initialWeights = Param("undefined", "initialWeights", "The initial weights of the model.",
                           TypeConverters.toVector)

    def getLayers(self):
        return self.getOrDefault("layers")

    def getInitialWeights(self):
        return self.getOrDefault("initialWeights")


class MultilayerPerceptronClassifier(Estimator, _MLPParams):
    def __init__(self, featuresCol="features", labelCol="label", predictionCol="prediction", maxIter=100, tol=1e-6,
                 seed=None, layers=None, blockSize=128, stepSize=0.03, solver="l-bfgs", initialWeights=None,
                 probabilityCol="probability", rawPredictionCol="rawPrediction", device=None):
        super().__init__()
        apply_mixin_defaults(self)
        self._setDefault(maxIter=100, tol=1e-6, blockSize=128, stepSize=0.03, solver="l-bfgs")
        kw = dict(featuresCol=featuresCol, labelCol=labelCol, predictionCol=predictionCol, maxIter=maxIter, tol=tol,
                  seed=seed, layers=layers, blockSize=blockSize, stepSize=stepSize, solver=solver,
                  initialWeights=initialWeights, probabilityCol=probabilityCol, rawPredictionCol=rawPredictionCol)
        self._set(**{k: v for k, v in kw.items() if v is not None})
        self.device = torch.device(device) if device else _device()

    def setLayers(self, v):
        return self._set(layers=v)

    def setInitialWeights(self, v):
        return self._set(initialWeights=v)

    def _fit(self, dataset):
        from ..optim.lbfgs import LBFGS
        from ..ops.mlp import mlp_loss
        layers = self.getLayers()
        if not layers or len(layers) < 2:
            raise ValueError("layers must be set, e.g. [4, 5, 4, 3]")
        solver = self.getSolver()
        if solver not in ("l-bfgs", "gd"):
            raise ValueError(f"solver must be l-bfgs or gd, got {solver}")
        X, y = dataset.to_numpy(self.getFeaturesCol(), self.getLabelCol())
        if X.shape[1] != layers[0]:
            raise ValueError(f"input layer size {layers[0]} != numFeatures {X.shape[1]}")
        if y.max() >= layers[-1] or y.min() < 0 or (y != np.round(y)).any():
            raise ValueError("labels must be integers in [0, numClasses)")
        dev = self.device
        xt = torch.as_tensor(X, dtype=torch.float32, device=dev)
        yt = torch.as_tensor(y, dtype=torch.int64, device=dev)
        rw = torch.as_tensor(block_row_weights(len(y), self.getBlockSize()), dtype=torch.float32, device=dev)
        if self.isDefined("initialWeights") and self.getOrDefault("initialWeights") is not None:
            w0 = np.asarray(self.getOrDefault("initialWeights").toArray(), dtype=np.float64)
            if w0.shape[0] != num_weights(layers):
                raise ValueError("initialWeights has the wrong size")
        else:
            w0 = init_weights(layers, self.getSeed())
        theta0 = torch.as_tensor(w0, dtype=torch.float32, device=dev)

        def fg(theta):
            Ws, bs = unpack_weights(theta, layers)
            Ws = [W.contiguous().detach().requires_grad_() for W in Ws]
            bs = [b.contiguous().detach().requires_grad_() for b in bs]
            for p in Ws + bs:
                p.grad = None
            loss = mlp_loss(xt, yt, Ws, bs, "sigmoid", rw)
            loss.backward()
            g = pack_weights([W.grad for W in Ws], [b.grad for b in bs])
            return float(loss.detach()), g

        t0 = time.time()
        if solver == "l-bfgs":
            opt = LBFGS(max_iter=self.getMaxIter(), m=10, tol=self.getTol())
            theta = opt.minimize(fg, theta0)
            history, iters = opt.objective_history, opt.iterations
        else:
            theta = theta0.clone()
            f, g = fg(theta)
            history = [f]
            iters = 0
            for it in range(1, self.getMaxIter() + 1):
                step = self.getStepSize() / np.sqrt(it)
                new = theta - step * g
                diff = float((new - theta).norm())
                theta = new
                f, g = fg(theta)
                history.append(f)
                iters = it
                if diff < self.getTol() * max(float(theta.norm()), 1.0):
                    break
        model = MultilayerPerceptronClassificationModel(layers, theta.detach().double().cpu().numpy(), device=dev)
        self._copyValues(model)
        model._summary = TrainingSummary(history, iters, time.time() - t0)
        return model


class TrainingSummary:
    def __init__(self, objective_history, total_iterations, train_time_s):
        self.objectiveHistory = list(objective_history)
        self.totalIterations = int(total_iterations)
        self.trainTimeSeconds = float(train_time_s)


class MultilayerPerceptronClassificationModel(Model, _MLPParams):
    def __init__(self, layers=None, weights=None, device=None):
        super().__init__()
        apply_mixin_defaults(self)
        self._setDefault(maxIter=100, tol=1e-6, blockSize=128, stepSize=0.03, solver="l-bfgs")
        if layers is not None:
            self._set(layers=layers)
        self._weights = np.asarray(weights, dtype=np.float64) if weights is not None else None
        self.device = torch.device(device) if device else _device()
        self._summary = None

    @property
    def weights(self):
        return DenseVector(self._weights)

    @property
    def numFeatures(self):
        return self.getLayers()[0]

    @property
    def numClasses(self):
        return self.getLayers()[-1]

    @property
    def summary(self):
        if self._summary is None:
            raise RuntimeError("No training summary available for this model")
        return self._summary

    @property
    def hasSummary(self):
        return self._summary is not None

    def _torch_params(self):
        theta = torch.as_tensor(self._weights, dtype=torch.float32, device=self.device)
        Ws, bs = unpack_weights(theta, self.getLayers())
        return [W.contiguous() for W in Ws], [b.contiguous() for b in bs]

    def predictRaw_batch(self, X):
        from ..ops.mlp import mlp_logits
        Ws, bs = self._torch_params()
        xt = torch.as_tensor(np.asarray(X), dtype=torch.float32, device=self.device)
        return mlp_logits(xt, Ws, bs, "sigmoid").double().cpu().numpy()

    def predictRaw(self, value):
        return DenseVector(self.predictRaw_batch(np.asarray(value.toArray() if hasattr(value, "toArray") else value)
                                                 [None, :])[0])

    def predictProbability(self, value):
        z = self.predictRaw(value).toArray()
        e = np.exp(z - z.max())
        return DenseVector(e / e.sum())

    def predict(self, value):
        return float(np.argmax(self.predictRaw(value).toArray()))

    def _transform(self, dataset):
        X, _ = dataset.to_numpy(self.getFeaturesCol(), label_col="__none__")
        raw = self.predictRaw_batch(X)
        z = raw - raw.max(1, keepdims=True)
        prob = np.exp(z)
        prob /= prob.sum(1, keepdims=True)
        pred = raw.argmax(1).astype(np.float64)
        out = dataset
        if self.getRawPredictionCol():
            out = out.withColumn(self.getRawPredictionCol(), VectorColumn(dense=raw))
        if self.getProbabilityCol():
            out = out.withColumn(self.getProbabilityCol(), VectorColumn(dense=prob))
        return out.withColumn(self.getPredictionCol(), pred)

    def evaluate(self, dataset):
        from .evaluation import MulticlassMetrics
        res = self.transform(dataset)
        return MulticlassMetrics(res.column(self.getPredictionCol()), res.column(self.getLabelCol()))

    # ---------------- persistence (Spark layout) ----------------
    def write(self):
        return MLPModelWriter(self)

    def save(self, path):
        self.write().save(path)

    @classmethod
    def read(cls):
        return MLPModelReader()

    @classmethod
    def load(cls, path):
        return MLPModelReader().load(path)

    def to_torch_module(self):
        """The equivalent sparkmi/torch MLP (reference R03 layout) with these weights."""
        from ..models.mlp import MultilayerPerceptron
        m = MultilayerPerceptron(self.getLayers())
        Ws, bs = self._torch_params()
        with torch.no_grad():
            for lin, W, b in zip(m.linears(), Ws, bs):
                lin.weight.copy_(W.cpu())
                lin.bias.copy_(b.cpu())
        return m

    @classmethod
    def from_torch_module(cls, module, layers=None):
        lins = module.linears() if hasattr(module, "linears") else [m for m in module.modules()
                                                                     if isinstance(m, torch.nn.Linear)]
        layers = layers or [lins[0].in_features] + [l.out_features for l in lins]
        flat = pack_weights([l.weight.detach().float().cpu() for l in lins], [l.bias.detach().float().cpu() for l in lins])
        return cls(layers, flat.double().numpy())


class MLPModelWriter:
    CLASS = "org.apache.spark.ml.classification.MultilayerPerceptronClassificationModel"

    def __init__(self, model):
        self.model = model
        self._overwrite = False

    def overwrite(self):
        self._overwrite = True
        return self

    def save(self, path):
        import pyarrow as pa
        import pyarrow.parquet as pq
        if os.path.exists(path):
            if not self._overwrite:
                raise FileExistsError(f"Path {path} already exists. Use write().overwrite().save(path).")
            shutil.rmtree(path)
        m = self.model
        os.makedirs(os.path.join(path, "metadata"))
        os.makedirs(os.path.join(path, "data"))
        meta = {"class": self.CLASS, "timestamp": int(time.time() * 1000), "sparkVersion": SPARK_VERSION,
                "uid": m.uid, "paramMap": m._param_json("set"), "defaultParamMap": m._param_json("default")}
        meta["paramMap"].setdefault("layers", list(m.getLayers()))
        with open(os.path.join(path, "metadata", "part-00000"), "w") as f:
            f.write(json.dumps(meta, separators=(",", ":")) + "\n")
        open(os.path.join(path, "metadata", "_SUCCESS"), "w").close()
        vec_type = pa.struct([("type", pa.int8()), ("size", pa.int32()), ("indices", pa.list_(pa.int32())),
                              ("values", pa.list_(pa.float64()))])
        arr = pa.array([{"type": 1, "size": None, "indices": None, "values": m._weights.tolist()}], type=vec_type)
        table = pa.table({"weights": arr})
        pq.write_table(table, os.path.join(path, "data", f"part-00000-{uuid.uuid4()}-c000.snappy.parquet"),
                       compression="snappy")
        open(os.path.join(path, "data", "_SUCCESS"), "w").close()


class MLPModelReader:
    def load(self, path):
        import pyarrow.parquet as pq
        with open(os.path.join(path, "metadata", "part-00000")) as f:
            meta = json.loads(f.readline())
        if meta.get("class") != MLPModelWriter.CLASS:
            raise ValueError(f"not a MultilayerPerceptronClassificationModel: {meta.get('class')}")
        files = sorted(p for p in os.listdir(os.path.join(path, "data")) if p.endswith(".parquet"))
        t = pq.read_table(os.path.join(path, "data", files[0]))
        w = t.column("weights").to_pylist()[0]
        values = np.asarray(w["values"], dtype=np.float64)
        if w.get("type") == 0:  # sparse vector
            dense = np.zeros(w["size"])
            dense[np.asarray(w["indices"])] = values
            values = dense
        layers = meta["paramMap"].get("layers") or meta["defaultParamMap"].get("layers")
        if layers is None and "layers" in t.column_names:  # Spark < 3.0 data layout
            layers = t.column("layers").to_pylist()[0]
        model = MultilayerPerceptronClassificationModel(layers, values)
        model.uid = meta["uid"]
        for k, v in meta.get("defaultParamMap", {}).items():
            if model.hasParam(k) and k not in ("layers", "initialWeights"):
                model._setDefault(**{k: v})
        for k, v in meta.get("paramMap", {}).items():
            if model.hasParam(k) and k not in ("initialWeights",):
                model._set(**{k: v})
        return model
