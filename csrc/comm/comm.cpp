// sparkmi._comm — native communication layer for executors (one process per MI355X):
//  * RCCL communicator (the C++ side of SURVEY §5.8 items 1/2/4): bootstrap from a unique id
//    exchanged through the c10d TCPStore, all-reduce / reduce-scatter / all-gather / broadcast
//    on raw device pointers on the caller's HIP stream (so they order with torch's kernels and
//    can sit inside HIP-graph captures), and ncclCommAbort for the failure path (a peer that died
//    or hangs must not leave the survivors blocked inside a collective).
//  * IPC one-shot all-reduce (item 3, csrc/comm/ipc_allreduce.hip): uncached staging + signal
//    regions, their hipIpcMemHandle export / import.
// librccl.so.1 and libamdhip64.so.7 resolve to the copies torch already loaded (same SONAMEs),
// so this module shares torch's HIP runtime and RCCL.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;
using u = uintptr_t;

#include "smi_ipc.h"
extern "C" int smi_ipc_allreduce(const IpcArgs* args, int blocks, hipStream_t st);

static void hchk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("sparkmi._comm.") + what + ": " + hipGetErrorString(e));
}
static void nchk(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("sparkmi._comm.") + what + ": " + ncclGetErrorString(r));
}

// ---------------------------------------------------------------- RCCL communicator
struct Comm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
};

static ncclDataType_t dtype_of(const std::string& d) {
  if (d == "float32") return ncclFloat32;
  if (d == "bfloat16") return ncclBfloat16;
  if (d == "float16") return ncclFloat16;
  if (d == "int32") return ncclInt32;
  if (d == "int64") return ncclInt64;
  if (d == "uint8") return ncclUint8;
  throw std::runtime_error("sparkmi._comm: unsupported dtype " + d);
}
static ncclRedOp_t op_of(const std::string& o) {
  if (o == "sum") return ncclSum;
  if (o == "max") return ncclMax;
  if (o == "min") return ncclMin;
  if (o == "avg") return ncclAvg;
  throw std::runtime_error("sparkmi._comm: unsupported op " + o);
}

PYBIND11_MODULE(_comm, m) {
  m.doc() = "sparkmi native communication layer: RCCL communicator + xGMI IPC one-shot all-reduce (gfx950)";

  m.def("rccl_version", []() {
    int v = 0;
    nchk(ncclGetVersion(&v), "ncclGetVersion");
    return v;
  });
  m.def("unique_id", []() {
    ncclUniqueId id;
    nchk(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
  });
  py::class_<Comm>(m, "Comm")
      .def(py::init([](py::bytes uid, int rank, int world, int device) {
             std::string s = uid;
             if (s.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("sparkmi._comm.Comm: bad unique id");
             ncclUniqueId id;
             std::memcpy(id.internal, s.data(), NCCL_UNIQUE_ID_BYTES);
             hchk(hipSetDevice(device), "hipSetDevice");
             auto* c = new Comm();
             c->rank = rank;
             c->world = world;
             ncclResult_t r;
             {
               py::gil_scoped_release nogil;  // blocks until every rank has joined
               r = ncclCommInitRank(&c->comm, world, id, rank);
             }
             if (r != ncclSuccess) {
               delete c;
               nchk(r, "ncclCommInitRank");
             }
             return c;
           }),
           py::arg("uid"), py::arg("rank"), py::arg("world"), py::arg("device"))
      .def_readonly("rank", &Comm::rank)
      .def_readonly("world", &Comm::world)
      .def("all_reduce", [](Comm& c, u send, u recv, long count, const std::string& dt, const std::string& op, u st) {
        nchk(ncclAllReduce((const void*)send, (void*)recv, (size_t)count, dtype_of(dt), op_of(op), c.comm,
                           (hipStream_t)st), "ncclAllReduce");
      })
      .def("reduce_scatter", [](Comm& c, u send, u recv, long recv_count, const std::string& dt, const std::string& op,
                                u st) {
        nchk(ncclReduceScatter((const void*)send, (void*)recv, (size_t)recv_count, dtype_of(dt), op_of(op), c.comm,
                               (hipStream_t)st), "ncclReduceScatter");
      })
      .def("all_gather", [](Comm& c, u send, u recv, long send_count, const std::string& dt, u st) {
        nchk(ncclAllGather((const void*)send, (void*)recv, (size_t)send_count, dtype_of(dt), c.comm, (hipStream_t)st),
             "ncclAllGather");
      })
      .def("broadcast", [](Comm& c, u send, u recv, long count, const std::string& dt, int root, u st) {
        nchk(ncclBroadcast((const void*)send, (void*)recv, (size_t)count, dtype_of(dt), root, c.comm, (hipStream_t)st),
             "ncclBroadcast");
      })
      .def("group_start", [](Comm&) { nchk(ncclGroupStart(), "ncclGroupStart"); })
      .def("group_end", [](Comm&) { nchk(ncclGroupEnd(), "ncclGroupEnd"); })
      .def("async_error", [](Comm& c) {
        ncclResult_t e = ncclSuccess;
        nchk(ncclCommGetAsyncError(c.comm, &e), "ncclCommGetAsyncError");
        return (int)e;
      })
      .def("abort", [](Comm& c) {  // failure path: tear down without waiting for peers
        if (c.comm) {
          ncclCommAbort(c.comm);
          c.comm = nullptr;
        }
      })
      .def("destroy", [](Comm& c) {
        if (c.comm) {
          ncclCommDestroy(c.comm);
          c.comm = nullptr;
        }
      });

  // ---------------------------------------------------------------- IPC regions
  // Allocate an uncached device region of `bytes` (zeroed) and its IPC handle.
  m.def("ipc_alloc", [](long bytes) {
    void* p = nullptr;
    hchk(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags");
    hchk(hipMemset(p, 0, (size_t)bytes), "hipMemset");
    hipIpcMemHandle_t h;
    hchk(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
    return py::make_tuple((u)p, py::bytes(reinterpret_cast<const char*>(&h), sizeof(h)));
  });
  m.def("ipc_open", [](py::bytes handle) {
    std::string s = handle;
    if (s.size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("sparkmi._comm.ipc_open: bad handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, s.data(), sizeof(h));
    void* p = nullptr;
    hchk(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    return (u)p;
  });
  m.def("ipc_close", [](u p) { hchk(hipIpcCloseMemHandle((void*)p), "hipIpcCloseMemHandle"); });
  m.def("ipc_free", [](u p) { hchk(hipFree((void*)p), "hipFree"); });
  // ctr: device uint32[2] = {epoch, ticket}, zero-initialised
  // spins: poll bound before a peer counts as lost (the bucket is then NaN-poisoned, *err set)
  m.def("ipc_allreduce", [](u buf, long n, std::vector<u> data, std::vector<u> sig, long cap, int rank, u ctr,
                            u err, int blocks, u st, long spins) {
    if (data.size() != sig.size() || data.empty() || data.size() > IPC_MAX_RANKS)
      throw std::runtime_error("sparkmi._comm.ipc_allreduce: bad peer lists");
    IpcArgs a{};
    a.buf = (float*)buf; a.n = n; a.cap = cap; a.rank = rank; a.world = (int)data.size();
    a.ep = (unsigned*)ctr; a.done = (unsigned*)ctr + 1;
    a.err = (int*)err;
    a.spins = spins > 0 ? spins : IPC_DEFAULT_SPINS;
    for (size_t i = 0; i < data.size(); ++i) { a.data[i] = (float*)data[i]; a.sig[i] = (unsigned*)sig[i]; }
    const int rc = smi_ipc_allreduce(&a, blocks, (hipStream_t)st);
    if (rc != 0) throw std::runtime_error("sparkmi._comm.ipc_allreduce failed: " +
                                          std::string(rc > 0 ? hipGetErrorString((hipError_t)rc) : "bad arguments"));
  });
  m.attr("IPC_MAX_RANKS") = IPC_MAX_RANKS;
  m.attr("IPC_MAX_BLOCKS") = IPC_MAX_BLOCKS;
  m.attr("IPC_DEFAULT_SPINS") = IPC_DEFAULT_SPINS;
}
