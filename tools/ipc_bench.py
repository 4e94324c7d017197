"""Staged vs zero-copy IPC two-shot all-reduce of one transformer-size gradient bucket (64 MiB),
N processes sharing the box's GPU (gloo for the handshakes).  On one device the "peer" reads are
local HBM reads, so this measures the HBM-traffic difference (the staging copy the zero-copy kernel
drops), not xGMI.  usage: python tools/ipc_bench.py [world ...]"""
import sys

sys.path.insert(0, ".")


def body(n, iters):
    import time
    import torch
    from sparkmi.parallel import init_distributed
    from sparkmi.parallel.comm import IpcAllReduce
    rank, world, dev = init_distributed()
    ar = IpcAllReduce(cap_floats=n)
    buf = torch.full((n,), float(rank + 1), device=dev)
    assert ar.register(buf)
    out = {}
    for algo in (2, 3, 2, 3):
        for _ in range(3):
            ar(buf, algo=algo)
        torch.cuda.synchronize()
        torch.distributed.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            ar(buf, algo=algo)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / iters * 1e3
        out[algo] = min(out.get(algo, 1e9), ms)
    ar.check()
    ar.close()
    allr = [None] * world
    torch.distributed.all_gather_object(allr, out)
    return {a: max(r[a] for r in allr) for a in out}


if __name__ == "__main__":
    from sparkmi.runtime.launcher import launch
    n = 16 << 20
    for w in [int(x) for x in sys.argv[1:]] or [2, 4]:
        r = launch(body, (n, 10), {}, num_processes=w, use_gpu=True, env={"SPARKMI_DIST_BACKEND": "gloo"},
                   log_sink=None, timeout=300)
        print(f"world {w}: 64 MiB bucket  staged two-shot {r[2]:.3f} ms  zero-copy two-shot {r[3]:.3f} ms  "
              f"({r[2] / r[3]:.2f}x)", flush=True)
