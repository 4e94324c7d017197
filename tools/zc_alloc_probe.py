"""Which gradient-buffer allocations the zero-copy IPC kernel can register reliably when the same
processes create and close several IpcAllReduce instances (the DP test grid's pattern): torch's
caching allocator vs sparkmi._comm.ipc_buffer (cached / uncached), freed after each instance.
4 ranks sharing the GPU.

Measured (profiles/r6_zero_copy_ipc.txt): a torch segment (never freed by the caching allocator,
so every registration exports the same allocation) registers and reduces exactly every time; an
allocation that is freed and replaced by a new one at the same address makes peers map stale
memory (wrong sums, sometimes in part of the buffer) — hence sparkmi/parallel/comm.py's lifetime
policy (pooled staging, one export per allocation, imports never closed) and the whole-buffer
self-test, which rejects such a registration (the 'own' rows fail it, as they must)."""
import sys

sys.path.insert(0, ".")


def body():
    import torch
    from torch.utils.dlpack import from_dlpack
    from sparkmi import _native
    from sparkmi.parallel import init_distributed
    from sparkmi.parallel.comm import IpcAllReduce
    rank, world, dev = init_distributed()
    C = _native.comm()
    n = 5 << 20
    out = []
    for rnd in range(3):
        for kind in ("torch", "own", "own_uc"):
            ar = IpcAllReduce(cap_floats=1 << 17)
            y = torch.ones(1024, device=dev)
            ar(y, algo=2)  # the staged path between registrations, as in the grid
            if kind == "torch":
                buf = torch.zeros(n, device=dev)
            else:
                buf = from_dlpack(C.ipc_buffer(n, dev.index or 0, kind == "own_uc"))
            ok = ar.register(buf)
            good = ok
            if ok:
                for it in range(3):
                    g = torch.Generator().manual_seed(it * 10 + rank)
                    buf[:65536].copy_(torch.randn(65536, generator=g).to(dev))
                    ar(buf[:65536], algo=3)
                    want = sum(torch.randn(65536, generator=torch.Generator().manual_seed(it * 10 + r))
                               for r in range(world))
                    good = good and torch.equal(buf[:65536].cpu(), want) if world <= 2 else good and bool(
                        (buf[:65536].cpu() - want).abs().max() < 1e-5)
            out.append((rnd, kind, ok, good, getattr(ar, "register_error", "")[:160]))
            ar.close()
            del buf
    allr = [None] * world
    torch.distributed.all_gather_object(allr, out)
    return allr


if __name__ == "__main__":
    from sparkmi.runtime.launcher import launch
    res = launch(body, (), {}, num_processes=4, use_gpu=True, env={"SPARKMI_DIST_BACKEND": "gloo"},
                 log_sink=None, timeout=300)
    for r, rows in enumerate(res):
        for row in rows:
            print(r, row, flush=True)
