"""pyspark.ml-compatible estimators, models, evaluators and vectors."""
from .base import Estimator, Evaluator, Model, Pipeline, PipelineModel, Transformer  # noqa: F401
from .classification import MultilayerPerceptronClassificationModel, MultilayerPerceptronClassifier  # noqa: F401
from .evaluation import MulticlassClassificationEvaluator, MulticlassMetrics  # noqa: F401
from .linalg import DenseVector, SparseVector, Vectors  # noqa: F401
