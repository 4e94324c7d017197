"""Data-parallel execution over RCCL (torch.distributed backend "nccl" on ROCm) or gloo (CPU)."""
from .ddp import DataParallel, broadcast_flat  # noqa: F401
from .dist import init_distributed, is_dist, rank, world_size, local_rank, barrier, destroy  # noqa: F401
