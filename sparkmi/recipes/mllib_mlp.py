"""Spark-MLlib-style MultilayerPerceptronClassifier flow — mllib_multilayer_perceptron_classifier.py (R01).

Session (3 executors x 1 core x 8g in the reference, :12-19) -> libsvm reader (:22-23) ->
randomSplit([0.6, 0.4], 1234) (:27) -> MultilayerPerceptronClassifier(maxIter=100,
layers=[4,5,4,3], blockSize=30, solver='l-bfgs', stepSize=0.03, seed=1234) (:32-35) -> timed fit
(:37-42) -> transform -> select("prediction", "label") -> accuracy evaluator (:45-48); optionally
``--save-path`` writes the model in Spark's on-disk layout.  The estimator runs full-batch
L-BFGS with the fused MLP gradient kernel on the GPU (sparkmi.ml.classification).
"""
import argparse
import os
import time

from ..api.session import Session
from ..data.synthetic import iris_libsvm_text
from ..ml.classification import MultilayerPerceptronClassifier
from ..ml.evaluation import MulticlassClassificationEvaluator


def run(data_path=None, max_iter=100, layers=(4, 5, 4, 3), block_size=30, solver="l-bfgs", step_size=0.03, seed=1234,
        save_path=None, verbose=True):
    spark = (Session.builder.appName("Multilayer_perceptron").config("spark.executor.instances", "3")
             .config("spark.executor.cores", "1").config("spark.executor.memory", "8g")
             .config("spark.driver.cores", "4").config("spark.driver.memory", "8g").getOrCreate())
    if data_path and os.path.exists(data_path):
        data = spark.read.format("libsvm").load(data_path)
    else:
        data = spark.read.libsvm(iris_libsvm_text(150, seed=seed), text=True)
    train, test = data.randomSplit([0.6, 0.4], seed)
    trainer = MultilayerPerceptronClassifier(maxIter=max_iter, layers=list(layers), blockSize=block_size,
                                             solver=solver, stepSize=step_size, seed=seed)
    t0 = time.time()
    model = trainer.fit(train)
    fit_s = time.time() - t0
    result = model.transform(test)
    prediction_and_labels = result.select("prediction", "label")
    evaluator = MulticlassClassificationEvaluator(metricName="accuracy")
    acc = evaluator.evaluate(prediction_and_labels)
    if save_path:
        model.write().overwrite().save(save_path)
    out = {"fit_time_s": fit_s, "test_accuracy": acc, "n_train": train.count(), "n_test": test.count(),
           "iterations": getattr(getattr(model, "summary", None), "totalIterations", None)}
    if verbose:
        print(f"Training time: {fit_s:.3f}s")
        print("Test set accuracy = " + str(acc))
    return out


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--data-path", default=None)
    p.add_argument("--max-iter", type=int, default=100)
    p.add_argument("--layers", default="4,5,4,3")
    p.add_argument("--block-size", type=int, default=30)
    p.add_argument("--solver", default="l-bfgs")
    p.add_argument("--step-size", type=float, default=0.03)
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--save-path", default=None)
    a = p.parse_args(argv)
    return run(a.data_path, a.max_iter, [int(v) for v in a.layers.split(",")], a.block_size, a.solver, a.step_size,
               a.seed, a.save_path)


if __name__ == "__main__":
    main()
