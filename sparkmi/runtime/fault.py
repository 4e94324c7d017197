"""Fault injection for failure-detection tests.

``SPARKMI_FAULT="rank:step:kind[:restart]"`` makes rank ``rank`` fail at training step ``step``
with kind ``exit`` (hard exit 17), ``raise`` (Python exception), ``hang`` (sleep forever, caught
by the heartbeat monitor), or ``segv`` (SIGSEGV to itself).  With ``:restart`` = N the fault
only fires on restart attempt N (TORCHELASTIC_RESTART_COUNT), so recovery can be tested.
Trainers call :func:`fault_point(step)` once per step.
"""
import os
import signal
import time


def _spec():
    s = os.environ.get("SPARKMI_FAULT")
    if not s:
        return None
    parts = s.split(":")
    rank, step, kind = int(parts[0]), int(parts[1]), parts[2]
    restart = int(parts[3]) if len(parts) > 3 else None
    return rank, step, kind, restart


def fault_point(step: int):
    spec = _spec()
    if spec is None:
        return
    rank, fstep, kind, restart = spec
    if int(os.environ.get("RANK", 0)) != rank or step != fstep:
        return
    if restart is not None and int(os.environ.get("TORCHELASTIC_RESTART_COUNT", 0)) != restart:
        return
    if kind == "exit":
        os._exit(17)
    if kind == "raise":
        raise RuntimeError(f"injected fault at step {step} on rank {rank}")
    if kind == "hang":
        while True:
            time.sleep(3600)
    if kind == "segv":
        os.kill(os.getpid(), signal.SIGSEGV)
    raise ValueError(f"unknown fault kind {kind}")
