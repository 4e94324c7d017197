"""Executor process entry point: ``python -m sparkmi.runtime.worker <job_dir>``.

Loads the cloudpickled (fn, args, kwargs) written by the launcher (a file this framework wrote
itself), starts a heartbeat thread, runs the function (or a script via runpy), and on rank 0
writes the cloudpickled return value back — the TorchDistributor contract
(rank 0's return value is the result of ``run``).

Heartbeat = liveness AND progress: the file ``hb.<rank>`` holds "<time> <progress>", where
progress is the counter the training loop advances through :func:`sparkmi.runtime.progress`
once per step.  The launcher treats a stale time (process wedged) and a progress counter that
stops moving while the thread still beats (main thread stuck, e.g. inside a collective whose
peer died or hangs) as failures of the whole group.

Cluster mode (``SPARKMI_CLUSTER=1``, TorchDistributor local_mode=False): every executor is a
barrier task with its own device; before running, the tasks exchange their addresses through
the job directory (the BarrierTaskContext.allGather of SURVEY C05) and task 0's address
becomes MASTER_ADDR."""
import os
import socket
import sys
import threading
import time
import traceback

from sparkmi.runtime import heartbeat as _hb


def _heartbeat(path, period):
    while True:
        try:
            tmp = path + ".tmp"
            with open(tmp, "w") as f:
                f.write(f"{time.time()} {_hb.current()}")
            os.replace(tmp, path)
        except OSError:
            pass
        time.sleep(period)


def _barrier_allgather(job, rank, world, timeout=120.0):
    """File-based allGather of the tasks' addresses; returns the list ordered by rank."""
    try:
        addr = socket.gethostbyname(socket.gethostname())
    except OSError:
        addr = "127.0.0.1"
    if os.environ.get("SPARKMI_CLUSTER_LOOPBACK", "1") == "1":
        addr = "127.0.0.1"  # single-host emulation of the cluster (the container's hostname may not resolve)
    tmp = os.path.join(job, f"addr.{rank}.tmp")
    with open(tmp, "w") as f:
        f.write(addr)
    os.replace(tmp, os.path.join(job, f"addr.{rank}"))
    t0 = time.time()
    while True:
        names = [os.path.join(job, f"addr.{r}") for r in range(world)]
        if all(os.path.exists(n) for n in names):
            return [open(n).read().strip() for n in names]
        if time.time() - t0 > timeout:
            raise RuntimeError("barrier allGather timed out")
        time.sleep(0.02)


def main():
    job = sys.argv[1]
    rank = int(os.environ.get("RANK", 0))
    period = float(os.environ.get("SPARKMI_HEARTBEAT_PERIOD", "1.0"))
    t = threading.Thread(target=_heartbeat, args=(os.path.join(job, f"hb.{rank}"), period), daemon=True)
    t.start()
    if os.environ.get("SPARKMI_CLUSTER") == "1":
        addrs = _barrier_allgather(job, rank, int(os.environ.get("WORLD_SIZE", 1)))
        os.environ["MASTER_ADDR"] = addrs[0]
        os.environ["SPARKMI_TASK_ADDRS"] = ",".join(addrs)
    import cloudpickle
    with open(os.path.join(job, "payload.pkl"), "rb") as f:
        kind, target, args, kwargs = cloudpickle.load(f)
    try:
        if kind == "script":
            import runpy
            sys.argv = [target] + [str(a) for a in args]
            runpy.run_path(target, run_name="__main__")
            result = None
        else:
            result = target(*args, **kwargs)
    except SystemExit as e:
        code = e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(code)
    except BaseException:
        traceback.print_exc()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(1)
    if rank == 0:
        tmp = os.path.join(job, "result.pkl.tmp")
        with open(tmp, "wb") as f:
            cloudpickle.dump(result, f)
        os.replace(tmp, os.path.join(job, "result.pkl"))
    sys.stdout.flush()
    sys.stderr.flush()
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            dist.destroy_process_group()
    except Exception:
        pass
    os._exit(0)


if __name__ == "__main__":
    main()
