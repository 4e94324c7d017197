"""Training engine: step runner (eager / HIP graph), trainer loop, recipe configs."""
from .config import TrainConfig, parse  # noqa: F401
from .runner import StepRunner  # noqa: F401
from .trainer import Trainer, setup_executor  # noqa: F401
