"""Executor-group launcher (the TorchDistributor / torchrun role).

Spawns ``num_processes`` executor processes (one per MI355X when ``use_gpu``), each with the
torchrun env contract (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, GROUP_RANK, MASTER_ADDR,
MASTER_PORT, TORCHELASTIC_RESTART_COUNT), streams their stdout/stderr to the driver with rank
prefixes, and gives the group barrier semantics:
  * any rank exiting non-zero, a rank whose heartbeat goes stale (process wedged), or a rank
    whose PROGRESS counter stops moving while its heartbeat thread still beats (main thread
    stuck — e.g. blocked in a collective whose peer died; ``progress_timeout``) terminates the
    whole group (Spark barrier-stage semantics);
  * the group is relaunched up to ``max_restarts`` times (fresh rendezvous port; training code
    resumes from its last checkpoint, sparkmi.train.checkpoint);
  * rank 0's return value is returned.
Local mode (TorchDistributor local_mode=True, distributed_multilayer_perceptron.py:177-180): the
driver host runs ``torchrun --standalone --nproc_per_node=N``-style ranks (LOCAL_RANK = RANK, one
GPU each by LOCAL_RANK).  Cluster mode (local_mode=False, distributed_cnn.py:227-231,
distributed_lstm.py:211-215): every executor is a barrier TASK — LOCAL_RANK 0, LOCAL_WORLD_SIZE
1, NODE_RANK = GROUP_RANK = task id, its own device via HIP_VISIBLE_DEVICES, the tasks exchange
addresses before running (BarrierTaskContext.allGather) and task 0's address becomes
MASTER_ADDR; a failed task fails the stage, which is re-run from scratch (max_restarts).
Multi-node: with SPARKMI_NNODES / SPARKMI_NODE_RANK / MASTER_ADDR set on every node, each node's
driver launches its local ranks with global ranks node_rank * num_processes + local_rank.
"""
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time


class LaunchError(RuntimeError):
    def __init__(self, msg, rank=None, returncode=None, log_tail=""):
        # the failing rank's last log lines travel in the message (pytest / callers show them)
        super().__init__(msg + (f"\n--- rank {rank} log tail ---\n{log_tail}" if log_tail else ""))
        self.msg = msg
        self.rank, self.returncode, self.log_tail = rank, returncode, log_tail


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Streamer(threading.Thread):
    def __init__(self, pipe, rank, sink, tail):
        super().__init__(daemon=True)
        self.pipe, self.rank, self.sink, self.tail = pipe, rank, sink, tail

    def run(self):
        for raw in iter(self.pipe.readline, b""):
            line = raw.decode(errors="replace").rstrip("\n")
            self.tail.append(line)
            if len(self.tail) > 200:
                del self.tail[:100]
            if self.sink is not None:
                self.sink(f"[rank {self.rank}] {line}")
        self.pipe.close()


def _default_sink(line):
    print(line, flush=True)


def launch(target, args=(), kwargs=None, num_processes=1, use_gpu=True, max_restarts=0, heartbeat_timeout=None,
           env=None, log_sink=_default_sink, timeout=None, master_addr=None, cluster=False, num_gpus=None,
           progress_timeout=None):
    """Run ``target`` (callable or script path) on an executor group; returns rank 0's result."""
    import cloudpickle
    kwargs = kwargs or {}
    nnodes = int(os.environ.get("SPARKMI_NNODES", 1))
    node_rank = int(os.environ.get("SPARKMI_NODE_RANK", 0))
    world = nnodes * num_processes
    hb_timeout = heartbeat_timeout if heartbeat_timeout is not None else float(
        os.environ.get("SPARKMI_HEARTBEAT_TIMEOUT", "300"))
    pg_timeout = progress_timeout if progress_timeout is not None else float(
        os.environ.get("SPARKMI_PROGRESS_TIMEOUT", "0"))
    job = tempfile.mkdtemp(prefix="sparkmi_job_")
    kind = "script" if isinstance(target, str) else "callable"
    with open(os.path.join(job, "payload.pkl"), "wb") as f:
        cloudpickle.dump((kind, target, tuple(args), kwargs), f)
    attempt = 0
    try:
        while True:
            port = int(os.environ.get("MASTER_PORT")) if (nnodes > 1 and "MASTER_PORT" in os.environ) else free_port()
            addr = (master_addr or os.environ.get("MASTER_ADDR", "127.0.0.1")) if nnodes > 1 else (master_addr or "127.0.0.1")
            procs, tails, streamers = [], [], []
            for lr in range(num_processes):
                r = node_rank * num_processes + lr
                e = dict(os.environ)
                e.update(env or {})
                e.update({"RANK": str(r), "LOCAL_RANK": str(lr), "WORLD_SIZE": str(world),
                          "LOCAL_WORLD_SIZE": str(num_processes), "GROUP_RANK": str(node_rank),
                          "NODE_RANK": str(node_rank), "MASTER_ADDR": addr, "MASTER_PORT": str(port),
                          "TORCHELASTIC_RESTART_COUNT": str(attempt), "SPARKMI_JOB_DIR": job,
                          "PYTHONUNBUFFERED": "1"})
                if cluster:
                    # barrier task: its own node rank, one device, address agreed by allGather
                    e.update({"LOCAL_RANK": "0", "LOCAL_WORLD_SIZE": "1", "GROUP_RANK": str(r), "NODE_RANK": str(r),
                              "SPARKMI_CLUSTER": "1"})
                    if use_gpu and num_gpus:
                        e["HIP_VISIBLE_DEVICES"] = str(r % num_gpus)
                if world > 1:
                    e.setdefault("OMP_NUM_THREADS", "1")
                if not use_gpu:
                    e["SPARKMI_FORCE_CPU"] = "1"
                    e["HIP_VISIBLE_DEVICES"] = ""
                    e["CUDA_VISIBLE_DEVICES"] = ""
                root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
                e["PYTHONPATH"] = root + os.pathsep + e.get("PYTHONPATH", "")
                p = subprocess.Popen([sys.executable, "-m", "sparkmi.runtime.worker", job], env=e,
                                     stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
                tail = []
                s = _Streamer(p.stdout, r, log_sink, tail)
                s.start()
                procs.append(p)
                tails.append(tail)
                streamers.append(s)
            failure = _monitor(procs, job, node_rank * num_processes, hb_timeout, timeout, pg_timeout)
            for s in streamers:
                s.join(timeout=5)
            if failure is None:
                res = os.path.join(job, "result.pkl")
                if node_rank == 0 and os.path.exists(res):
                    with open(res, "rb") as f:
                        return cloudpickle.load(f)
                return None
            rank_fail, code, why = failure
            if attempt >= max_restarts:
                lr = rank_fail - node_rank * num_processes
                tail = "\n".join(tails[lr][-30:]) if 0 <= lr < len(tails) else ""
                raise LaunchError(f"executor rank {rank_fail} failed ({why}, exit code {code}); "
                                  f"group terminated after {attempt} restart(s)", rank_fail, code, tail)
            attempt += 1
            if log_sink:
                log_sink(f"[launcher] rank {rank_fail} failed ({why}); restarting group (attempt {attempt})")
            for f in os.listdir(job):
                if f.startswith(("hb.", "addr.")):
                    os.remove(os.path.join(job, f))
    finally:
        shutil.rmtree(job, ignore_errors=True)


def _kill_group(procs):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
    deadline = time.time() + 10
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()


def _read_hb(path):
    """(time, progress) of a heartbeat file, or None."""
    try:
        with open(path) as f:
            parts = f.read().split()
        return float(parts[0]), int(parts[1]) if len(parts) > 1 else 0
    except (OSError, ValueError, IndexError):
        return None


def _monitor(procs, job, rank0, hb_timeout, timeout, progress_timeout=0.0):
    """Wait for the group; returns None on success or (rank, code, reason) of the first failure."""
    start = time.time()
    seen = {}  # rank -> (progress value, wall time it last changed)
    while True:
        alive = 0
        for i, p in enumerate(procs):
            rc = p.poll()
            if rc is None:
                alive += 1
            elif rc != 0:
                _kill_group(procs)
                return rank0 + i, rc, "exited"
        if alive == 0:
            return None
        now = time.time()
        for i, p in enumerate(procs):
            if p.poll() is not None:
                continue
            hb = _read_hb(os.path.join(job, f"hb.{rank0 + i}"))
            if hb_timeout and now - start > hb_timeout:
                last = hb[0] if hb else start
                if now - last > hb_timeout:
                    _kill_group(procs)
                    return rank0 + i, None, f"heartbeat stale > {hb_timeout:.0f}s"
            if progress_timeout and hb is not None and hb[1] > 0:
                prev = seen.get(i)
                if prev is None or prev[0] != hb[1]:
                    seen[i] = (hb[1], now)
                elif now - prev[1] > progress_timeout:
                    _kill_group(procs)
                    return rank0 + i, None, f"progress stalled at step {hb[1]} for > {progress_timeout:.0f}s"
        if timeout and now - start > timeout:
            _kill_group(procs)
            return rank0, None, f"timeout {timeout}s"
        time.sleep(0.05)
