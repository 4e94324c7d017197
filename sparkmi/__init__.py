"""sparkmi — a Spark-style deep-learning trainer built MI355X-first.

Capabilities of Makkan13/Machine_Learning---Apache-Spark (MLP / CNN / LSTM / Transformer
training, sequential and data-parallel, plus a Spark-MLlib-compatible
MultilayerPerceptronClassifier) on AMD Instinct MI355X: one executor process per GPU,
HBM-resident partitions, hand-written HIP/CDNA4 kernels (sparkmi._C), RCCL over xGMI for
gradient sync.  See README.md and SURVEY.md.
"""
__version__ = "0.1.0"
