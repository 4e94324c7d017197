"""Spark-style driver API: Session (SparkSession-lite), Frame (DataFrame-lite), Distributor
(TorchDistributor contract)."""
from .frame import Frame, Row  # noqa: F401
from .session import Conf, Session, SparkConf, SparkSession  # noqa: F401
from .distributor import Distributor, TorchDistributor  # noqa: F401
