"""The IPC region lifetime policy of sparkmi/parallel/comm.py on CPU, with a mock native module:
exported regions are pooled (never freed), a reused signal region is re-zeroed and a reused staging
region is not, an allocation is exported once, a peer handle is imported once.  Why: a freed and
re-exported allocation mapped stale memory on peers (tools/zc_alloc_probe.py,
profiles/r6_zero_copy_ipc.txt)."""
from sparkmi.parallel import comm


class _C:
    def __init__(self):
        self.allocs, self.zeroed, self.exports, self.opens = 0, [], [], []

    def ipc_alloc(self, nbytes):
        self.allocs += 1
        return 1000 * self.allocs, b"h%d" % self.allocs

    def ipc_memset0(self, p, nbytes):
        self.zeroed.append(p)

    def ipc_range(self, ptr):
        return ptr - ptr % 4096, 1 << 20

    def ipc_export(self, base):
        self.exports.append(base)
        return (b"e%d" % base, 0, 1 << 20)

    def ipc_open(self, h):
        self.opens.append(h)
        return 7_000_000 + len(self.opens)


def test_pool_export_import_once(monkeypatch):
    monkeypatch.setattr(comm, "_POOL", {})
    monkeypatch.setattr(comm, "_EXPORTS", {})
    monkeypatch.setattr(comm, "_IMPORTS", {})
    C = _C()
    p1, h1 = comm._alloc(C, 256, zero=True)
    assert C.allocs == 1
    comm._POOL.setdefault(256, []).append((p1, h1))  # what IpcAllReduce.close() does
    p2, h2 = comm._alloc(C, 256, zero=True)
    assert (p2, h2) == (p1, h1) and C.allocs == 1 and C.zeroed == [p1]  # reused and re-zeroed
    comm._POOL.setdefault(256, []).append((p2, h2))
    p3, _ = comm._alloc(C, 256, zero=False)
    assert p3 == p1 and C.zeroed == [p1]  # a staging region is not re-zeroed
    # one export per allocation (base, size), the byte offset of the pointer returned beside it
    ha, oa = comm._export(C, 4096 * 3 + 64)
    hb, ob = comm._export(C, 4096 * 3 + 128)
    assert ha == hb and (oa, ob) == (64, 128) and C.exports == [4096 * 3]
    # one import per peer handle, never closed
    assert comm._open(C, b"x") == comm._open(C, b"x") and C.opens == [b"x"]
