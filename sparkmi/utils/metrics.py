"""Per-rank structured metrics (fixes Q17: the reference only print()s).

``MetricsLogger.step(loss, n_samples)`` accumulates the loss ON DEVICE (no host sync per step,
so a HIP-graph step loop is not stalled) and every ``every`` steps synchronises once and appends
one JSON line: step, mean loss over the interval, samples/s and ms/step over the interval, plus
the phase breakdown the Trainer passes (data_s: host time waiting for the batch;
fwd_bwd_s / allreduce_s / optim_s: device time per phase from HIP events of eager steps;
bytes_reduced: gradient bytes handed to the collectives in the interval; with ``flops_per_sample``
also tflops: achieved model TFLOP/s of this rank).  ``aggregate()`` (driver side) combines
per-rank files into whole-job samples/s, the BASELINE metric.
"""
import json
import os
import time

import torch


class MetricsLogger:
    def __init__(self, path=None, rank=0, every=50, echo=False, extra=None, flops_per_sample=None):
        self.path = path
        self.flops_per_sample = flops_per_sample
        self.rank = rank
        self.every = max(1, int(every))
        self.echo = echo
        self.extra = dict(extra or {})
        self.records = []
        self._acc = None
        self._n = 0
        self._samples = 0
        self._step = 0
        self._t0 = None
        self._fh = None
        if path:
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            self._fh = open(path, "a", buffering=1)

    def _sync(self, t):
        if t is not None and t.is_cuda:
            torch.cuda.synchronize(t.device)

    def due(self):
        """True when the next step() call writes a record."""
        return (self._step + 1) % self.every == 0

    def pending(self):
        """Steps accumulated since the last record."""
        return self._n

    def until_flush(self):
        """step() calls left until (and including) the one that writes the next record: a group
        of steps whose summed loss is credited to its last step must not span a record."""
        return self.every - self._step % self.every

    def step(self, loss=None, n_samples=0, **scalars):
        if self._t0 is None:
            self._sync(loss)
            self._t0 = time.perf_counter()
        self._step += 1
        self._n += 1
        self._samples += int(n_samples)
        if loss is not None:
            v = loss.detach().float().reshape(())
            self._acc = v.clone() if self._acc is None else self._acc.add_(v)
        if self._step % self.every == 0:
            self.flush(**scalars)

    def flush(self, **scalars):
        if self._n == 0:
            return None
        self._sync(self._acc)
        now = time.perf_counter()
        dt = max(now - self._t0, 1e-12)
        rec = {"step": self._step, "rank": self.rank, "time": time.time(),
               "loss": float(self._acc.item()) / self._n if self._acc is not None else None,
               "samples_per_s": self._samples / dt, "ms_per_step": dt * 1e3 / self._n}
        if self.flops_per_sample:
            rec["tflops"] = self._samples * self.flops_per_sample / dt / 1e12
        rec.update(self.extra)
        rec.update({k: (float(v) if isinstance(v, (int, float)) or torch.is_tensor(v) else v) for k, v in scalars.items()})
        self.log_record(rec)
        self._acc, self._n, self._samples, self._t0 = None, 0, 0, now
        return rec

    def log(self, **fields):
        rec = {"step": self._step, "rank": self.rank, "time": time.time()}
        rec.update(fields)
        self.log_record(rec)
        return rec

    def log_record(self, rec):
        self.records.append(rec)
        if self._fh:
            self._fh.write(json.dumps(rec) + "\n")
        if self.echo:
            print(json.dumps(rec), flush=True)

    def close(self):
        self.flush()
        if self._fh:
            self._fh.close()
            self._fh = None


def read_jsonl(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


def aggregate(paths):
    """Whole-job throughput from per-rank JSONL files: sum over ranks of each rank's mean
    samples/s (ranks run concurrently), and the max per-rank ms/step."""
    total, worst = 0.0, 0.0
    for p in paths:
        recs = [r for r in read_jsonl(p) if "samples_per_s" in r]
        if not recs:
            continue
        total += sum(r["samples_per_s"] for r in recs) / len(recs)
        worst = max(worst, max(r["ms_per_step"] for r in recs))
    return {"samples_per_s": total, "ms_per_step_max": worst, "ranks": len(paths)}
