"""Distributor — the TorchDistributor contract on MI355X executors.

``Distributor(num_processes, local_mode=True, use_gpu=True).run(train_fn, *args, **kwargs)``
launches one executor process per MI355X (``use_gpu``) or per CPU worker, each with the
torchrun env contract, so code written for the reference (``dist.init_process_group(...)``
inside ``train_func``, distributed_cnn.py:149-193) runs unchanged; sparkmi code calls
``sparkmi.parallel.init_distributed()`` which picks RCCL ("nccl") on GPU executors.
Returns rank 0's return value.  ``train_object`` may also be a script path (its args follow).
``local_mode=False`` gives the cluster-mode contract: one barrier task per executor with its own
device and node rank, addresses exchanged before the run (sparkmi/runtime/launcher.py).
Extras over TorchDistributor: ``max_restarts`` (group restart on failure), a heartbeat +
progress hang detector (``progress_timeout``), and ``share_gpus`` (several executors per device,
e.g. multi-process tests on a one-GPU box).
"""
from ..runtime.launcher import launch


class Distributor:
    def __init__(self, num_processes=1, local_mode=True, use_gpu=True, max_restarts=0, heartbeat_timeout=None,
                 env=None, timeout=None, log_sink="default", progress_timeout=None, share_gpus=False):
        if num_processes < 1:
            raise ValueError("num_processes must be >= 1")
        self.num_processes = int(num_processes)
        self.local_mode = local_mode
        self.use_gpu = use_gpu
        self.max_restarts = max_restarts
        self.heartbeat_timeout = heartbeat_timeout
        self.env = env or {}
        self.timeout = timeout
        self.log_sink = log_sink
        self.progress_timeout = progress_timeout
        self.num_gpus = 0
        if use_gpu:
            from .session import visible_gpus
            n = visible_gpus()
            self.num_gpus = n
            if n and self.num_processes > n and not share_gpus:
                raise RuntimeError(f"requested {self.num_processes} GPU executors but only {n} GPUs are visible "
                                   "(share_gpus=True places several executors per device)")
            if n == 0:
                # no GPU on this host: run the executors on CPU (gloo), like use_gpu=False
                self.use_gpu = False

    def run(self, train_object, *args, **kwargs):
        from ..runtime.launcher import _default_sink
        sink = _default_sink if self.log_sink == "default" else self.log_sink
        return launch(train_object, args, kwargs, num_processes=self.num_processes, use_gpu=self.use_gpu,
                      max_restarts=self.max_restarts, heartbeat_timeout=self.heartbeat_timeout, env=self.env,
                      log_sink=sink, timeout=self.timeout, cluster=not self.local_mode, num_gpus=self.num_gpus,
                      progress_timeout=self.progress_timeout)


TorchDistributor = Distributor
