"""Executor process entry point: ``python -m sparkmi.runtime.worker <job_dir>``.

Loads the cloudpickled (fn, args, kwargs) written by the launcher (a file this framework wrote
itself), starts a heartbeat thread, runs the function (or a script via runpy), and on rank 0
writes the cloudpickled return value back — the TorchDistributor contract
(rank 0's return value is the result of ``run``)."""
import os
import sys
import threading
import time
import traceback


def _heartbeat(path, period):
    while True:
        try:
            with open(path, "w") as f:
                f.write(str(time.time()))
        except OSError:
            pass
        time.sleep(period)


def main():
    job = sys.argv[1]
    rank = int(os.environ.get("RANK", 0))
    period = float(os.environ.get("SPARKMI_HEARTBEAT_PERIOD", "1.0"))
    t = threading.Thread(target=_heartbeat, args=(os.path.join(job, f"hb.{rank}"), period), daemon=True)
    t.start()
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
