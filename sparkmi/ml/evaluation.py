"""MulticlassClassificationEvaluator (pyspark.ml.evaluation) — Spark MulticlassMetrics
definitions, computed from a (weighted) confusion matrix.

Reference: MulticlassClassificationEvaluator(metricName="accuracy")
(mllib_multilayer_perceptron_classifier.py:47-48).  Supported metricName: f1 (default),
accuracy, weightedPrecision, weightedRecall, weightedTruePositiveRate,
weightedFalsePositiveRate, weightedFMeasure, truePositiveRateByLabel,
falsePositiveRateByLabel, precisionByLabel, recallByLabel, fMeasureByLabel, logLoss,
hammingLoss.  Also used by the trainers for full-split accuracy (fixes Q18: the reference
reports the last batch only).
"""
import numpy as np

from .base import Evaluator
from .param import HasLabelCol, HasPredictionCol, HasProbabilityCol, HasWeightCol, Param, TypeConverters, \
    apply_mixin_defaults

METRICS = {"f1", "accuracy", "weightedPrecision", "weightedRecall", "weightedTruePositiveRate",
           "weightedFalsePositiveRate", "weightedFMeasure", "truePositiveRateByLabel", "falsePositiveRateByLabel",
           "precisionByLabel", "recallByLabel", "fMeasureByLabel", "logLoss", "hammingLoss"}


class MulticlassMetrics:
    def __init__(self, pred, label, weight=None, probability=None):
        pred = np.asarray(pred, dtype=np.float64)
        label = np.asarray(label, dtype=np.float64)
        w = np.ones_like(label) if weight is None else np.asarray(weight, dtype=np.float64)
        self.labels = np.unique(np.concatenate([label, pred]))
        idx = {v: i for i, v in enumerate(self.labels)}
        L = len(self.labels)
        cm = np.zeros((L, L))
        for p, l, ww in zip(pred, label, w):
            cm[idx[l], idx[p]] += ww
        self.cm = cm  # rows: true label, cols: prediction
        self.total = w.sum()
        self.label_count = cm.sum(1)
        self.tp = np.diag(cm)
        self.fp = cm.sum(0) - self.tp
        self._probability = probability
        self._label = label
        self._w = w
        self._idx = idx

    def _li(self, label):
        return self._idx.get(float(label))

    def precision(self, label):
        i = self._li(label)
        d = self.tp[i] + self.fp[i]
        return 0.0 if d == 0 else self.tp[i] / d

    def recall(self, label):
        i = self._li(label)
        return 0.0 if self.label_count[i] == 0 else self.tp[i] / self.label_count[i]

    def truePositiveRate(self, label):
        return self.recall(label)

    def falsePositiveRate(self, label):
        i = self._li(label)
        d = self.total - self.label_count[i]
        return 0.0 if d == 0 else self.fp[i] / d

    def fMeasure(self, label, beta=1.0):
        p, r = self.precision(label), self.recall(label)
        b2 = beta * beta
        return 0.0 if p + r == 0 else (1 + b2) * p * r / (b2 * p + r)

    def _weighted(self, fn):
        freq = self.label_count / self.total
        return float(sum(fn(l) * f for l, f in zip(self.labels, freq)))

    @property
    def accuracy(self):
        return float(self.tp.sum() / self.total) if self.total else 0.0

    @property
    def weightedPrecision(self):
        return self._weighted(self.precision)

    @property
    def weightedRecall(self):
        return self._weighted(self.recall)

    @property
    def weightedTruePositiveRate(self):
        return self.weightedRecall

    @property
    def weightedFalsePositiveRate(self):
        return self._weighted(self.falsePositiveRate)

    def weightedFMeasure(self, beta=1.0):
        return self._weighted(lambda l: self.fMeasure(l, beta))

    @property
    def hammingLoss(self):
        return 1.0 - self.accuracy

    def logLoss(self, eps=1e-15):
        if self._probability is None:
            raise ValueError("logLoss needs a probability column")
        P = np.asarray(self._probability, dtype=np.float64)
        p = np.clip(P[np.arange(len(self._label)), self._label.astype(np.int64)], eps, 1.0)
        return float(-(self._w * np.log(p)).sum() / self._w.sum())


class MulticlassClassificationEvaluator(Evaluator, HasLabelCol, HasPredictionCol, HasWeightCol, HasProbabilityCol):
    metricName = Param("undefined", "metricName", "metric name in evaluation " + "|".join(sorted(METRICS)),
                       TypeConverters.toString)
    metricLabel = Param("undefined", "metricLabel", "The class whose metric will be computed in *ByLabel metrics.",
                        TypeConverters.toFloat)
    beta = Param("undefined", "beta", "The beta value used in weightedFMeasure|fMeasureByLabel.",
                 TypeConverters.toFloat)
    eps = Param("undefined", "eps", "log-loss clipping epsilon", TypeConverters.toFloat)

    def __init__(self, predictionCol="prediction", labelCol="label", metricName="f1", weightCol=None,
                 metricLabel=0.0, beta=1.0, probabilityCol="probability", eps=1e-15):
        super().__init__()
        apply_mixin_defaults(self)
        self._setDefault(metricName="f1", metricLabel=0.0, beta=1.0, eps=1e-15)
        if metricName not in METRICS:
            raise ValueError(f"unknown metricName {metricName}")
        self._set(predictionCol=predictionCol, labelCol=labelCol, metricName=metricName, metricLabel=metricLabel,
                  beta=beta, probabilityCol=probabilityCol, eps=eps)
        if weightCol:
            self._set(weightCol=weightCol)

    def setMetricName(self, v):
        return self._set(metricName=v)

    def getMetricName(self):
        return self.getOrDefault("metricName")

    def metrics(self, dataset):
        pred = np.asarray(dataset.column(self.getPredictionCol()), dtype=np.float64)
        label = np.asarray(dataset.column(self.getLabelCol()), dtype=np.float64)
        w = None
        if self.isDefined("weightCol") and self.getOrDefault("weightCol"):
            w = np.asarray(dataset.column(self.getOrDefault("weightCol")), dtype=np.float64)
        prob = None
        pc = self.getOrDefault("probabilityCol")
        if pc in dataset.columns:
            col = dataset.column(pc)
            prob = col.to_dense() if hasattr(col, "to_dense") else np.asarray(col)
        return MulticlassMetrics(pred, label, w, prob)

    def _evaluate(self, dataset):
        m = self.metrics(dataset)
        name = self.getMetricName()
        lab = self.getOrDefault("metricLabel")
        beta = self.getOrDefault("beta")
        if name == "f1":
            return m.weightedFMeasure(1.0)
        if name == "weightedFMeasure":
            return m.weightedFMeasure(beta)
        if name == "truePositiveRateByLabel":
            return m.truePositiveRate(lab)
        if name == "falsePositiveRateByLabel":
            return m.falsePositiveRate(lab)
        if name == "precisionByLabel":
            return m.precision(lab)
        if name == "recallByLabel":
            return m.recall(lab)
        if name == "fMeasureByLabel":
            return m.fMeasure(lab, beta)
        if name == "logLoss":
            return m.logLoss(self.getOrDefault("eps"))
        return getattr(m, name)

    def isLargerBetter(self):
        return self.getMetricName() not in ("weightedFalsePositiveRate", "falsePositiveRateByLabel", "logLoss",
                                            "hammingLoss")
