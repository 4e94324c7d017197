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

// DLPack (the stable v0.x ABI torch.utils.dlpack.from_dlpack consumes): a device buffer this module
// allocated, handed to torch as a tensor that frees it when torch drops it
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor {
  void* data; DLDevice device; int32_t ndim; DLDataType dtype; int64_t* shape; int64_t* strides; uint64_t byte_offset;
};
struct DLManagedTensor { DLTensor dl_tensor; void* manager_ctx; void (*deleter)(DLManagedTensor*); };
struct OwnedBuf { DLManagedTensor mt; int64_t shape[1]; };
static void owned_deleter(DLManagedTensor* mt) {
  OwnedBuf* o = reinterpret_cast<OwnedBuf*>(mt);
  (void)hipFree(o->mt.dl_tensor.data);
  delete o;
}
static void capsule_dtor(PyObject* cap) {  // a capsule torch never consumed still frees its buffer
  if (PyCapsule_IsValid(cap, "dltensor")) {
    auto* mt = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
    if (mt && mt->deleter) mt->deleter(mt);
  }
}

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
  // A zeroed fp32 device buffer of n floats in an allocation of its own (hipExtMallocWithFlags, the
  // allocator of the IPC staging regions; cached unless `uncached`), as a DLPack capsule: the
  // gradient buffer the zero-copy kernel reads across processes lives in one (sparkmi/parallel/ddp.py)
  m.def("ipc_buffer", [](long n, int device, bool uncached) {
    int cur = 0;
    hchk(hipGetDevice(&cur), "hipGetDevice");
    hchk(hipSetDevice(device), "hipSetDevice");
    void* p = nullptr;
    hchk(hipExtMallocWithFlags(&p, (size_t)n * 4, uncached ? hipDeviceMallocUncached : hipDeviceMallocDefault),
         "hipExtMallocWithFlags");
    hchk(hipMemset(p, 0, (size_t)n * 4), "hipMemset");
    hchk(hipSetDevice(cur), "hipSetDevice");
    OwnedBuf* o = new OwnedBuf{};
    o->shape[0] = n;
    DLTensor& t = o->mt.dl_tensor;
    t.data = p;
    t.device = DLDevice{10 /* kDLROCM */, device};
    t.ndim = 1;
    t.dtype = DLDataType{2 /* kDLFloat */, 32, 1};
    t.shape = o->shape;
    t.strides = nullptr;
    t.byte_offset = 0;
    o->mt.manager_ctx = o;
    o->mt.deleter = owned_deleter;
    return py::reinterpret_steal<py::object>(PyCapsule_New(&o->mt, "dltensor", capsule_dtor));
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
  // Export an existing device allocation (e.g. a flat gradient buffer from torch's allocator) for
  // the zero-copy kernel: the IPC handle of the allocation holding `ptr` and ptr's byte offset in
  // it (a peer adds the offset to the base ipc_open returns)
  m.def("ipc_range", [](u ptr) {  // (base, bytes) of the allocation holding ptr
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hchk(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr), "hipMemGetAddressRange");
    return py::make_tuple((u)base, (long)size);
  });
  m.def("ipc_export", [](u ptr) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hchk(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr), "hipMemGetAddressRange");
    hipIpcMemHandle_t h;
    hchk(hipIpcGetMemHandle(&h, (void*)base), "hipIpcGetMemHandle");
    return py::make_tuple(py::bytes(reinterpret_cast<const char*>(&h), sizeof(h)), (long)(ptr - (u)base),
                          (long)size);
  });
  m.def("ipc_free", [](u p) { hchk(hipFree((void*)p), "hipFree"); });
  // re-zero a pooled region before it is handed out again (sparkmi/parallel/comm.py keeps exported
  // regions for the life of the process instead of freeing them)
  m.def("ipc_memset0", [](u p, long bytes) { hchk(hipMemset((void*)p, 0, (size_t)bytes), "hipMemset"); });
  // ctr: device uint32[3] = {epoch, ticket, signal value}, zero-initialised
  // spins: poll bound before a peer counts as lost (the bucket is then NaN-poisoned, *err set)
  // algo: 1 one-shot, 2 two-shot (reduce-scatter + all-gather), 3 zero-copy two-shot (data = every
  // rank's bucket itself, data[rank] == buf; no staging)
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
