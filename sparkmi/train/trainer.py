"""Epoch/step training loop shared by every recipe.

One executor (= one MI355X, one process) runs ``Trainer.fit``: per step the StepRunner does
seed bump -> fused forward/loss -> fused backward (grads into the flat fp32 buffer; with
data parallelism bucketed RCCL all-reduces overlap the backward) -> fused optimizer, captured
in a HIP graph when running on a single executor.  Around it: ROCTx ranges, device-side
metrics accumulation (one host sync per ``log_every`` steps), fault-injection points,
periodic atomic checkpoints, and exact resume (model + optimizer + dropout seeds + RNG + epoch
+ batch cursor; the per-epoch shuffles are seeded by seed+epoch so the resumed order matches).

Reference loops this replaces: distributed_multilayer_perceptron.py:97-145,
distributed_cnn.py:149-193, distributed_lstm.py:156-205, pytorch_machine_translator.py:140-209.
"""
import time

import torch

from ..parallel import DataParallel, init_distributed
from ..runtime.fault import fault_point
from ..runtime.heartbeat import progress
from ..utils import trace
from ..utils.checkpoint import CheckpointManager
from ..utils.flat import FlatParams
from ..utils.metrics import MetricsLogger
from .runner import StepRunner


def setup_executor(cfg):
    """Process-group + device for this executor (RCCL on GPU executors, gloo on CPU)."""
    import os
    if cfg.device == "cpu":
        os.environ["SPARKMI_FORCE_CPU"] = "1"
    rank, world, device = init_distributed()
    torch.manual_seed(cfg.seed)
    from ..ops.rng import reset_salts
    reset_salts()  # same dropout salts as a fresh process: runs are reproducible in-process too
    return rank, world, device


class Trainer:
    def __init__(self, model, loss_fn, make_optimizer, cfg, device, rank=0, world=1, name="run", shadow=None,
                 fused_step=None, split_fn=None, flops_per_sample=None, fused_grad=None, sparse_cap=None,
                 fused_steps=None):
        self.model = model.to(device)
        self.cfg = cfg
        self.device = torch.device(device)
        self.rank, self.world = rank, world
        self.flat = FlatParams(self.model, device=self.device, shadow=shadow)
        self.opt = make_optimizer(self.flat)
        # sparse_cap: a bound on the ids per step (fixed list length: no host sync in the exchange)
        sparse = (self.model.sparse_rows(cap=sparse_cap) if getattr(cfg, "sparse_embedding", False)
                  and hasattr(self.model, "sparse_rows") else None)
        self.ddp = DataParallel(self.flat, bucket_mb=cfg.bucket_mb, zero=getattr(cfg, "zero", False),
                                sparse_rows=sparse) if world > 1 else None
        use_graph = bool(cfg.graph) and self.device.type == "cuda"
        # split_fn (data-parallel): the backward as several graphs, finished gradient buckets
        # reduced while the rest of the backward runs (StepRunner)
        # fused_step: a whole single-executor step in one kernel; fused_grad: forward + backward in
        # one kernel (the data-parallel step's local half, reduction and optimizer follow)
        self.runner = StepRunner(self.model, loss_fn, self.opt, ddp=self.ddp, graph=use_graph,
                                 fused_step=fused_step if world == 1 else None,
                                 fused_steps=fused_steps if world == 1 else None,
                                 fused_grad=fused_grad if world > 1 else None,
                                 split_fn=split_fn if (world > 1 and use_graph) else None)
        path = f"{cfg.metrics}.rank{rank}.jsonl" if cfg.metrics else None
        self.metrics = MetricsLogger(path, rank=rank, every=cfg.log_every, echo=cfg.verbose and rank == 0,
                                     extra={"run": name, "world": world}, flops_per_sample=flops_per_sample)
        self.ckpt = CheckpointManager(cfg.ckpt_dir, rank=rank) if cfg.ckpt_dir else None
        self.step = 0
        self.epoch = 0
        self.cursor = 0
        self.resumed_from = None

    def maybe_resume(self):
        if self.ckpt is None or not self.cfg.resume:
            return None
        meta = self.ckpt.restore(self.model, self.opt)
        if meta is None:
            return None
        self.step, self.epoch, self.cursor = meta["step"], meta["epoch"], meta["cursor"]
        self.resumed_from = self.ckpt.latest()
        return meta

    def _save(self, cursor):
        if self.ckpt is not None:
            self.runner.check()  # never checkpoint a model updated from a poisoned gradient
            with trace.range("checkpoint"):
                self.ckpt.save(self.step, self.model, self.opt, self.epoch, cursor)
            if self.world > 1:
                from ..parallel import barrier
                barrier()

    def _bind_loader(self, loader):
        """A fixed-buffer DeviceLoader: its gather runs inside the step (captured with it), the
        graphs read its static buffers in place, and ``cfg.unroll`` steps replay as one
        multi-step graph — the loop issues one launch per ``unroll`` shuffled steps."""
        if not (getattr(loader, "fixed", False) and self.device.type == "cuda" and self.runner.graph_requested):
            return 1
        loader.deferred = True
        gis = getattr(self.model, "gather_in_step", None)
        fused = self.runner.fused_step if self.world == 1 else self.runner.fused_grad
        if (gis is not None and fused is not None and self.runner.split_fn is None and len(loader.static) == 2
                and gis(self.opt, self.ddp if self.world > 1 else None, loader.static[0])):
            # the model's fused kernels read the shuffled batch from the dataset themselves (index
            # mode): no gather launch at all; the batch buffers carry the dataset + device cursor
            loader.static[0]._smi_gather = (loader.batch_size, loader.arrays[0], loader.arrays[1], loader._perm_buf,
                                            loader._cursor)
            self.runner.pre_step = None
        else:
            self.runner.pre_step = loader.pre_step
        self.runner.bind_inputs = True
        self.runner.unroll = max(1, int(getattr(self.cfg, "unroll", 1)))
        return self.runner.unroll

    def _group(self, it, U):
        """Up to U batches of ``it`` without crossing a log / checkpoint / max_steps boundary.
        The log boundary is the metrics logger's own (its step count restarts at 0 after a resume
        and it clamps log_every to >= 1): the group's summed loss goes to its last step, so a group
        spanning a record would credit one interval's losses to the next."""
        cfg = self.cfg
        n = min(U, self.metrics.until_flush())
        if self.ckpt is not None and cfg.ckpt_every:
            n = min(n, cfg.ckpt_every - self.step % cfg.ckpt_every)
        if cfg.max_steps:
            n = min(n, cfg.max_steps - self.step)
        group = []
        for _ in range(max(1, n)):
            b = next(it, None)
            if b is None:
                break
            group.append(b)
        return group

    def fit(self, loader, epochs, samples_per_batch=None):
        """Train over ``loader`` (an epoch-seeded DeviceLoader-like iterable) for ``epochs``."""
        cfg = self.cfg
        self.maybe_resume()
        U = self._bind_loader(loader)
        t0 = time.perf_counter()
        steps_run, last = 0, None
        done = False
        data_s, bytes0 = 0.0, 0
        self.runner.phase_timing = bool(getattr(cfg, "phase_timing", False))
        while self.epoch < epochs and not done:
            if hasattr(loader, "set_epoch"):
                loader.set_epoch(self.epoch)
            if hasattr(loader, "skip"):
                loader.skip = self.cursor
            i = self.cursor
            it = iter(loader)
            while True:
                td = time.perf_counter()
                with trace.range("data"):
                    group = self._group(it, U) if U > 1 else [b for b in (next(it, None),) if b is not None]
                if not group:
                    break
                data_s += time.perf_counter() - td
                n = samples_per_batch or int(group[0][0].shape[0])
                with trace.range("step"):
                    if len(group) > 1:
                        losses = []
                        self.runner.run_steps(group, losses)
                    else:
                        losses = [self.runner.step(*group[0])]
                # the group's losses summed once (one reduction, not one add per step): the metrics
                # mean over the interval is unchanged (groups never cross a log boundary)
                gsum = losses[0]
                if len(losses) > 1:
                    gsum = (self.runner.last_group_sum if (len(losses) == self.runner.unroll
                                                           and self.runner.last_group_sum is not None)
                            else torch.stack([l.reshape(()) for l in losses]).sum())
                last = losses[-1]
                for j in range(len(losses)):
                    lj = gsum if j == len(losses) - 1 else None
                    self.step += 1
                    steps_run += 1
                    i += 1
                    progress(self.step)  # heartbeat progress: a stuck collective stops this counter
                    if self.metrics.due():
                        self.runner.check()  # a lost data-parallel peer fails the group here
                        ph = self.runner.pop_phases()
                        ddp_bytes = self.ddp.bytes_reduced if self.ddp is not None else 0
                        extra = dict(ph, data_s=data_s / max(1, self.metrics.pending() + 1),
                                     bytes_reduced=ddp_bytes - bytes0)
                        bytes0, data_s = ddp_bytes, 0.0
                        self.metrics.step(lj, n * self.world, **extra)
                    else:
                        self.metrics.step(lj, n * self.world)
                    fault_point(self.step)
                if self.ckpt is not None and cfg.ckpt_every and self.step % cfg.ckpt_every == 0:
                    self.cursor = i
                    self._save(i)
                if cfg.max_steps and self.step >= cfg.max_steps:
                    done = True
                    break
            if not done:
                self.epoch += 1
                self.cursor = 0
                if self.ckpt is not None and not cfg.ckpt_every:
                    self._save(0)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - t0
        self.metrics.flush()
        return {"steps": steps_run, "global_step": self.step, "time_s": dt,
                "final_loss": float(last.item()) if last is not None else None,
                "resumed_from": self.resumed_from}

    def close(self):
        self.metrics.close()
        if self.ddp is not None:
            self.ddp.close()
