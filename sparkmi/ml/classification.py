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
Compute: ``fit`` runs on the session's executors (spark.executor.instances, or ``numExecutors``):
one process per executor (Distributor), each holding its contiguous row partition resident on
its device; every objective evaluation is the fused HIP MLP loss+gradient (sparkmi/ops/mlp.py)
on the partition followed by ONE all-reduce of [gradient, loss] — Spark's treeAggregate — and
every executor runs the identical device L-BFGS (sparkmi/optim/lbfgs.py, csrc/kernels/lbfgs.hip).
CPU executors use float64 torch.  The objective is fixed on the global row order and reduced
over fixed slabs of whole blocks in slab order (``reduction_slabs``), so a fit on N executors
is bit-identical to the single-executor fit.  ``transform`` appends rawPrediction / probability / prediction columns.
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
                 probabilityCol="probability", rawPredictionCol="rawPrediction", device=None, numExecutors=None,
                 fitTimeout=600):
        super().__init__()
        apply_mixin_defaults(self)
        self._setDefault(maxIter=100, tol=1e-6, blockSize=128, stepSize=0.03, solver="l-bfgs")
        kw = dict(featuresCol=featuresCol, labelCol=labelCol, predictionCol=predictionCol, maxIter=maxIter, tol=tol,
                  seed=seed, layers=layers, blockSize=blockSize, stepSize=stepSize, solver=solver,
                  initialWeights=initialWeights, probabilityCol=probabilityCol, rawPredictionCol=rawPredictionCol)
        self._set(**{k: v for k, v in kw.items() if v is not None})
        self.device = torch.device(device) if device else _device()
        self.num_executors = numExecutors  # None: the dataset session's spark.executor.instances
        self.fit_timeout = fitTimeout

    def setLayers(self, v):
        return self._set(layers=v)

    def setInitialWeights(self, v):
        return self._set(initialWeights=v)

    def _fit(self, dataset):
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
        if self.isDefined("initialWeights") and self.getOrDefault("initialWeights") is not None:
            w0 = np.asarray(self.getOrDefault("initialWeights").toArray(), dtype=np.float64)
            if w0.shape[0] != num_weights(layers):
                raise ValueError("initialWeights has the wrong size")
        else:
            w0 = init_weights(layers, self.getSeed())
        # Spark's block-averaged objective, fixed on the GLOBAL row order: each executor's rows
        # carry their global weights, so the executors' partial sums add up to the same
        # objective whatever the partitioning
        rw = block_row_weights(len(y), self.getBlockSize())
        opts = dict(layers=list(layers), solver=solver, max_iter=self.getMaxIter(), tol=self.getTol(),
                    step_size=self.getStepSize())
        slabs = reduction_slabs(len(y), self.getBlockSize())
        n_exec = self._executors(dataset, len(slabs) - 1)
        t0 = time.time()
        if n_exec <= 1:
            theta, history, iters = _fit_arrays(X, y, rw, w0, opts, self.device, slabs)
        else:
            from ..api.distributor import Distributor
            gpu = self.device.type == "cuda"
            env = {}
            if gpu and torch.cuda.device_count() < n_exec:
                env["SPARKMI_DIST_BACKEND"] = "gloo"  # several executors share a device: no RCCL
            theta, history, iters = Distributor(num_processes=n_exec, use_gpu=gpu, share_gpus=True, env=env,
                                                log_sink=None, timeout=self.fit_timeout).run(
                _fit_executor, X, y, rw, w0, opts, slabs)
        model = MultilayerPerceptronClassificationModel(layers, np.asarray(theta, dtype=np.float64), device=self.device)
        self._copyValues(model)
        model._summary = TrainingSummary(history, iters, time.time() - t0)
        model._num_executors = n_exec
        return model

    def _executors(self, dataset, n_slabs):
        """Executors the fit runs on: ``numExecutors`` if given, else the dataset's session
        (spark.executor.instances, mllib_multilayer_perceptron_classifier.py:12-19), at most one
        per reduction slab."""
        n = self.num_executors
        if n is None:
            sess = getattr(dataset, "session", None)
            n = sess.num_executors if sess is not None else 1
        return max(1, min(int(n), n_slabs))


def _objective(X, y, rw, layers, device):
    """fg(theta) -> (weighted CE sum over these rows [0-d tensor], flat gradient [new tensor]).
    GPU: the fused HIP MLP kernels (fp32, sparkmi/ops/mlp.py); CPU: float64 torch."""
    from ..ops.mlp import mlp_loss
    if device.type == "cuda":
        xt = torch.as_tensor(X, dtype=torch.float32, device=device)
        yt = torch.as_tensor(y, dtype=torch.int64, device=device)
        wt = torch.as_tensor(rw, dtype=torch.float32, device=device)

        def fg(theta):
            Ws, bs = unpack_weights(theta, layers)
            Ws = [W.contiguous().detach().requires_grad_() for W in Ws]
            bs = [b.contiguous().detach().requires_grad_() for b in bs]
            loss = mlp_loss(xt, yt, Ws, bs, "sigmoid", wt)
            loss.backward()
            return loss.detach(), pack_weights([W.grad for W in Ws], [b.grad for b in bs])
        return fg
    xt = torch.as_tensor(X, dtype=torch.float64)
    yt = torch.as_tensor(y, dtype=torch.int64)
    wt = torch.as_tensor(rw, dtype=torch.float64)

    def fg(theta):
        th = theta.detach().requires_grad_()
        Ws, bs = unpack_weights(th, layers)
        h = xt
        for i, (W, b) in enumerate(zip(Ws, bs)):
            h = h @ W.t() + b
            if i < len(Ws) - 1:
                h = torch.sigmoid(h)
        rl = torch.logsumexp(h, 1) - h.gather(1, yt[:, None]).squeeze(1)
        loss = (rl * wt).sum()
        (g,) = torch.autograd.grad(loss, th)
        return loss.detach(), g
    return fg


MAX_SLABS = 64


def reduction_slabs(n_rows, block_size, max_slabs=MAX_SLABS):
    """Row boundaries of the objective's reduction slabs: whole Spark blocks grouped into at most
    ``max_slabs`` contiguous slabs.  Each slab's loss/gradient is computed on its own and the
    slabs are summed in slab order, so the result does not depend on how slabs are spread over
    executors (floating-point sums are not associative; a plain all-reduce of per-executor
    partial sums would make an N-executor fit differ from the 1-executor fit)."""
    nb = max(1, (n_rows + block_size - 1) // block_size)
    ns = min(nb, max_slabs)
    return [min(n_rows, (s * nb // ns) * block_size) for s in range(ns)] + [n_rows]


def _fit_arrays(X, y, rw, w0, opts, device, slabs, mine=None, reduce=None):
    """Solve with the objective summed over reduction slabs.  ``slabs``: global row boundaries;
    ``mine``: the slab indices whose rows are in X/y/rw (all of them by default, rows given
    from the first of them on).  ``reduce(buf)`` sums the [slabs, n+1] partials over executors
    in place — each slab is non-zero on exactly one executor, so that sum is exact (this is
    Spark's treeAggregate, made order-independent) — and every executor then adds the slabs in
    slab order and follows the identical trajectory."""
    from ..optim.lbfgs import LBFGS
    layers = opts["layers"]
    dtype = torch.float32 if device.type == "cuda" else torch.float64
    ns = len(slabs) - 1
    mine = list(range(ns)) if mine is None else list(mine)
    base = slabs[mine[0]] if mine else 0
    objs = [(s, _objective(X[slabs[s] - base:slabs[s + 1] - base], y[slabs[s] - base:slabs[s + 1] - base],
                           rw[slabs[s] - base:slabs[s + 1] - base], layers, device)) for s in mine]
    n = num_weights(layers)

    def fg(theta):
        part = torch.zeros(ns, n + 1, dtype=dtype, device=device)
        for s, obj in objs:
            f, g = obj(theta)
            part[s, :n] = g.reshape(-1)
            part[s, n] = f
        if reduce is not None:
            reduce(part)
        tot = part.sum(0)
        return tot[n], tot[:n].clone()

    theta0 = torch.as_tensor(w0, dtype=dtype, device=device)
    if opts["solver"] == "l-bfgs":
        opt = LBFGS(max_iter=opts["max_iter"], m=10, tol=opts["tol"])
        theta = opt.minimize(fg, theta0)
        history, iters = opt.objective_history, opt.iterations
    else:
        theta = theta0.clone()
        f, g = fg(theta)
        history = [float(f)]
        iters = 0
        for it in range(1, opts["max_iter"] + 1):
            step = opts["step_size"] / np.sqrt(it)
            new = theta - step * g
            diff = float((new - theta).norm())
            theta = new
            f, g = fg(theta)
            history.append(float(f))
            iters = it
            if diff < opts["tol"] * max(float(theta.norm()), 1.0):
                break
    return theta.detach().double().cpu().numpy(), history, iters


def _fit_executor(X, y, rw, w0, opts, slabs):
    """One executor of a distributed fit (run by Distributor): its contiguous run of reduction
    slabs stays resident on its device; the slab partials are all-reduced every evaluation."""
    import torch.distributed as dist
    from ..parallel import init_distributed
    rank, world, device = init_distributed()
    ns = len(slabs) - 1
    cut = np.linspace(0, ns, world + 1).round().astype(int)
    mine = list(range(cut[rank], cut[rank + 1]))
    lo, hi = (slabs[mine[0]], slabs[mine[-1] + 1]) if mine else (0, 0)
    host = dist.get_backend() == "gloo" and device.type == "cuda"

    def reduce(buf):
        if host:  # gloo on shared devices: reduce through host memory
            t = buf.cpu()
            dist.all_reduce(t)
            buf.copy_(t)
        else:
            dist.all_reduce(buf)

    out = _fit_arrays(X[lo:hi], y[lo:hi], rw[lo:hi], w0, opts, device, slabs, mine, reduce=reduce)
    dist.barrier()
    return out


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
