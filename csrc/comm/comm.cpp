// sparkmi._comm — native communication layer for executors (one process per MI355X): the xGMI
// IPC one-shot / two-shot all-reduce (csrc/comm/ipc_allreduce.hip) —
// uncached staging + signal regions, their hipIpcMemHandle export / import, the launch.  Bulk
// collectives stay on RCCL through torch's "nccl" process group (sparkmi/parallel/ddp.py);
// librccl.so.1 and libamdhip64.so.7 resolve to the copies torch already loaded (same SONAMEs).
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
extern "C" int smi_ipc_allreduce(const IpcArgs* args, int blocks, int algo, hipStream_t st);

static void hchk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("sparkmi._comm.") + what + ": " + hipGetErrorString(e));
}

PYBIND11_MODULE(_comm, m) {
  m.doc() = "sparkmi native communication layer: xGMI IPC one-shot / two-shot all-reduce (gfx950)";

  m.def("rccl_version", []() {  // the RCCL torch's "nccl" process group runs on (same SONAME)
    int v = 0;
    const ncclResult_t r = ncclGetVersion(&v);
    if (r != ncclSuccess) throw std::runtime_error(std::string("sparkmi._comm.ncclGetVersion: ") + ncclGetErrorString(r));
    return v;
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
  // ctr: device uint32[3] = {epoch, ticket, signal value}, zero-initialised
  // spins: poll bound before a peer counts as lost (the bucket is then NaN-poisoned, *err set)
  // algo: 1 one-shot, 2 two-shot (reduce-scatter + all-gather)
  // sgd_p / sgd_pbf / sgd_lr / sgd_step / sgd_seed / sgd_gscale: the optional plain-SGD epilogue of
  // the one-shot kernel (sgd_p = 0: a plain all-reduce)
  m.def("ipc_allreduce", [](u buf, long n, std::vector<u> data, std::vector<u> sig, long cap, int rank, u ctr,
                            u err, int blocks, u st, long spins, int algo, u sgd_p, u sgd_pbf, u sgd_lr, u sgd_step,
                            u sgd_seed, float sgd_gscale) {
    if (data.size() != sig.size() || data.empty() || data.size() > IPC_MAX_RANKS)
      throw std::runtime_error("sparkmi._comm.ipc_allreduce: bad peer lists");
    IpcArgs a{};
    a.buf = (float*)buf; a.n = n; a.cap = cap; a.rank = rank; a.world = (int)data.size();
    a.ep = (unsigned*)ctr; a.done = (unsigned*)ctr + 1; a.sv = (unsigned*)ctr + 2;
    a.err = (int*)err;
    a.spins = spins > 0 ? spins : IPC_DEFAULT_SPINS;
    for (size_t i = 0; i < data.size(); ++i) { a.data[i] = (float*)data[i]; a.sig[i] = (unsigned*)sig[i]; }
    a.p = (float*)sgd_p; a.pbf = (unsigned short*)sgd_pbf; a.lr = (const float*)sgd_lr; a.step = (float*)sgd_step;
    a.seed = (int*)sgd_seed; a.gscale = sgd_gscale;
    const int rc = smi_ipc_allreduce(&a, blocks, algo, (hipStream_t)st);
    if (rc != 0) throw std::runtime_error("sparkmi._comm.ipc_allreduce failed: " +
                                          std::string(rc > 0 ? hipGetErrorString((hipError_t)rc) : "bad arguments"));
  });
  m.attr("IPC_MAX_RANKS") = IPC_MAX_RANKS;
  m.attr("IPC_MAX_BLOCKS") = IPC_MAX_BLOCKS;
  m.attr("IPC_DEFAULT_SPINS") = IPC_DEFAULT_SPINS;
}
