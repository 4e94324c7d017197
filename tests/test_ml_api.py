"""Spark-API layer (T1): Session/Frame/libsvm reader, the MLlib-compatible
MultilayerPerceptronClassifier (fit/transform/evaluate, l-bfgs and gd), the evaluator's metrics
against scikit-learn, and the Spark on-disk model format round trip."""
import json
import os

import numpy as np
import pytest
import torch

from sparkmi.api import Session
from sparkmi.data.synthetic import iris_libsvm_text, iris_like
from sparkmi.ml import (MulticlassClassificationEvaluator, MultilayerPerceptronClassificationModel,
                        MultilayerPerceptronClassifier, Vectors)
from sparkmi.ml.classification import block_row_weights, num_weights, pack_weights, unpack_weights


@pytest.fixture()
def spark():
    s = Session.builder.appName("test").config("spark.executor.instances", "2").getOrCreate()
    yield s
    s.stop()


@pytest.fixture()
def iris(tmp_path, spark):
    p = tmp_path / "sample.txt"
    p.write_text(iris_libsvm_text(150, seed=3))
    return spark.read.format("libsvm").load(str(p))


def test_session_conf(spark):
    assert int(spark.sparkContext.getConf().get("spark.executor.instances")) == 2
    s2 = Session.builder.getOrCreate()
    assert s2 is spark


def test_libsvm_reader(iris):
    assert iris.count() == 150
    assert iris.columns == ["label", "features"]
    r = iris.first()
    assert r.features.size == 4
    pdf = iris.toPandas()
    X = np.stack(pdf["features"].apply(lambda v: v.toArray()).tolist())
    _, ref = iris_like(150, seed=3)
    np.testing.assert_allclose(np.where(np.abs(ref) < 0.02, 0.0, ref), X, atol=1e-6)


def test_libsvm_errors(spark):
    with pytest.raises(RuntimeError):
        spark.read.libsvm("1 2:0.5 1:0.3\n", text=True)  # not ascending
    f = spark.read.libsvm("0 1:1.0 3:2.0\n1 2:5\n", text=True, numFeatures=4)
    X, y = f.to_numpy()
    np.testing.assert_array_equal(X, [[1, 0, 2, 0], [0, 5, 0, 0]])
    np.testing.assert_array_equal(y, [0, 1])


def test_random_split_disjoint_covering(iris):
    a, b = iris.randomSplit([0.6, 0.4], 1234)
    assert a.count() + b.count() == 150
    assert 60 < a.count() < 120
    a2, _ = iris.randomSplit([0.6, 0.4], 1234)
    np.testing.assert_array_equal(a.to_numpy()[0], a2.to_numpy()[0])


def test_partitions_disjoint_covering(iris):
    parts = [iris.partition(i, 4) for i in range(4)]
    assert sum(p.count() for p in parts) == 150
    X = np.concatenate([p.to_numpy()[0] for p in parts])
    np.testing.assert_array_equal(X, iris.to_numpy()[0])


def test_weight_layout_roundtrip():
    layers = [4, 5, 4, 3]
    assert num_weights(layers) == 64
    flat = torch.arange(64, dtype=torch.float32)
    Ws, bs = unpack_weights(flat, layers)
    assert Ws[0].shape == (5, 4) and bs[0].shape == (5,)
    # Spark column-major: element (o, i) at i * numOut + o
    assert float(Ws[0][2, 1]) == 1 * 5 + 2
    torch.testing.assert_close(pack_weights(Ws, bs), flat)


def test_block_weights_sum_to_one():
    w = block_row_weights(90, 30)
    assert abs(w.sum() - 1.0) < 1e-12
    w = block_row_weights(95, 30)
    assert abs(w.sum() - 1.0) < 1e-12 and w[-1] > w[0]


@pytest.mark.parametrize("solver", ["l-bfgs", "gd"])
def test_mlp_classifier_fit_transform_evaluate(iris, solver):
    train, test = iris.randomSplit([0.6, 0.4], 1234)
    trainer = MultilayerPerceptronClassifier(maxIter=100 if solver == "l-bfgs" else 400, layers=[4, 5, 4, 3],
                                             blockSize=30, seed=1234, solver=solver,
                                             stepSize=0.03 if solver == "l-bfgs" else 5.0, device="cpu")
    model = trainer.fit(train)
    assert model.numFeatures == 4 and model.numClasses == 3
    assert len(model.weights) == 64
    hist = model.summary.objectiveHistory
    assert hist[-1] < hist[0]
    result = model.transform(test)
    assert {"rawPrediction", "probability", "prediction"} <= set(result.columns)
    acc = MulticlassClassificationEvaluator(metricName="accuracy").evaluate(result.select("prediction", "label"))
    assert acc > (0.85 if solver == "l-bfgs" else 0.6), acc
    p = model.predictProbability(test.first().features).toArray()
    assert abs(p.sum() - 1) < 1e-6


def test_evaluator_matches_sklearn():
    from sklearn import metrics as skm
    rng = np.random.default_rng(0)
    y = rng.integers(0, 4, 200).astype(float)
    pred = np.where(rng.random(200) < 0.7, y, rng.integers(0, 4, 200)).astype(float)
    prob = rng.random((200, 4))
    prob /= prob.sum(1, keepdims=True)
    from sparkmi.api import Frame
    from sparkmi.ml.linalg import VectorColumn
    df = Frame({"prediction": pred, "label": y, "probability": VectorColumn(dense=prob)})
    ev = lambda m: MulticlassClassificationEvaluator(metricName=m).evaluate(df)  # noqa: E731
    assert abs(ev("accuracy") - skm.accuracy_score(y, pred)) < 1e-12
    assert abs(ev("f1") - skm.f1_score(y, pred, average="weighted")) < 1e-12
    assert abs(ev("weightedPrecision") - skm.precision_score(y, pred, average="weighted")) < 1e-12
    assert abs(ev("weightedRecall") - skm.recall_score(y, pred, average="weighted")) < 1e-12
    assert abs(ev("logLoss") - skm.log_loss(y, prob, labels=[0, 1, 2, 3])) < 1e-9
    assert abs(ev("hammingLoss") - skm.hamming_loss(y, pred)) < 1e-12
    e = MulticlassClassificationEvaluator(metricName="precisionByLabel", metricLabel=2.0)
    assert abs(e.evaluate(df) - skm.precision_score(y, pred, labels=[2], average=None)[0]) < 1e-12


def test_model_save_load_spark_layout(iris, tmp_path):
    model = MultilayerPerceptronClassifier(maxIter=20, layers=[4, 5, 4, 3], blockSize=30, seed=7,
                                           device="cpu").fit(iris)
    path = str(tmp_path / "mlp_model")
    model.write().overwrite().save(path)
    meta = json.loads(open(os.path.join(path, "metadata", "part-00000")).read())
    assert meta["class"] == "org.apache.spark.ml.classification.MultilayerPerceptronClassificationModel"
    assert meta["paramMap"]["layers"] == [4, 5, 4, 3]
    import pyarrow.parquet as pq
    data = [f for f in os.listdir(os.path.join(path, "data")) if f.endswith(".parquet")]
    t = pq.read_table(os.path.join(path, "data", data[0]))
    ty = t.schema.field("weights").type
    assert [ty.field(i).name for i in range(ty.num_fields)] == ["type", "size", "indices", "values"]
    assert str(ty.field(0).type) == "int8" and str(ty.field(3).type.value_type) == "double"
    with pytest.raises(FileExistsError):
        model.write().save(path)
    m2 = MultilayerPerceptronClassificationModel.load(path)
    np.testing.assert_array_equal(m2.weights.toArray(), model.weights.toArray())
    assert m2.getBlockSize() == 30
    r1 = model.transform(iris).column("prediction")
    r2 = m2.transform(iris).column("prediction")
    np.testing.assert_array_equal(r1, r2)


def test_torch_module_conversion(iris):
    model = MultilayerPerceptronClassifier(maxIter=10, layers=[4, 5, 4, 3], seed=1, device="cpu").fit(iris)
    tm = model.to_torch_module()
    X, _ = iris.to_numpy()
    z = tm(torch.as_tensor(X, dtype=torch.float32)).detach().numpy()
    np.testing.assert_allclose(z, model.predictRaw_batch(X), atol=1e-5)
    back = MultilayerPerceptronClassificationModel.from_torch_module(tm)
    np.testing.assert_allclose(back.weights.toArray(), model.weights.toArray(), atol=1e-6)


def test_params_api():
    t = MultilayerPerceptronClassifier(layers=[4, 5, 3], blockSize=30)
    assert t.getBlockSize() == 30 and t.getMaxIter() == 100 and t.getSolver() == "l-bfgs"
    assert "blockSize" in t.explainParams()
    t2 = t.copy({t.maxIter: 5})
    assert t2.getMaxIter() == 5 and t.getMaxIter() == 100
    v = Vectors.dense([1.0, 2.0])
    assert v.toArray().tolist() == [1.0, 2.0]
    sv = Vectors.sparse(4, [1, 3], [1.0, 2.0])
    assert sv.toArray().tolist() == [0.0, 1.0, 0.0, 2.0]


@pytest.mark.parametrize("solver", ["l-bfgs", "gd"])
def test_distributed_fit_equals_single_executor(iris, tmp_path, solver):
    """Executor-parallel fit (2 processes, partitions resident per executor, [grad, loss]
    all-reduced each evaluation = Spark's treeAggregate) lands on the single-executor weights."""
    train, _ = iris.randomSplit([0.6, 0.4], 1234)
    kw = dict(maxIter=60, layers=[4, 5, 4, 3], blockSize=30, seed=1234, solver=solver, device="cpu",
              stepSize=0.03 if solver == "l-bfgs" else 5.0)
    m2 = MultilayerPerceptronClassifier(numExecutors=2, **kw).fit(train)
    m1 = MultilayerPerceptronClassifier(numExecutors=1, **kw).fit(train)
    assert m2._num_executors == 2 and m1._num_executors == 1
    assert m1.summary.totalIterations == m2.summary.totalIterations
    np.testing.assert_allclose(m2.weights.toArray(), m1.weights.toArray(), atol=1e-6, rtol=0)
    np.testing.assert_allclose(m2.summary.objectiveHistory, m1.summary.objectiveHistory, rtol=1e-9)
    path = str(tmp_path / "dist_model")
    m2.write().overwrite().save(path)
    back = MultilayerPerceptronClassificationModel.load(path)
    np.testing.assert_array_equal(back.weights.toArray(), m2.weights.toArray())
    np.testing.assert_array_equal(back.transform(iris).column("prediction"), m2.transform(iris).column("prediction"))


def test_lbfgs_minimises_quadratic_cpu():
    """Device-memory L-BFGS (ring buffers + two-loop) on an ill-conditioned quadratic."""
    from sparkmi.optim.lbfgs import LBFGS
    torch.manual_seed(0)
    n = 40
    Q = torch.randn(n, n, dtype=torch.float64)
    A = Q @ Q.t() / n + 0.05 * torch.eye(n, dtype=torch.float64)  # condition number ~100
    b = torch.randn(n, dtype=torch.float64)

    def fg(x):
        return 0.5 * x @ A @ x - b @ x, A @ x - b
    opt = LBFGS(max_iter=1000, m=10, tol=1e-15)
    x = opt.minimize(fg, torch.zeros(n, dtype=torch.float64))
    torch.testing.assert_close(x, torch.linalg.solve(A, b), atol=1e-5, rtol=1e-5)
    assert 10 < opt.iterations < 1000
