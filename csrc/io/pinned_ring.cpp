// sparkmi._io — native host->HBM input pipeline (SURVEY §2.3 pinned_ring.cpp, §5.8 item 6): a ring
// of page-locked host slots that loader threads fill with gathered minibatch rows (row gather
// in C++ with the GIL released, several threads), each slot shipped to HBM with
// hipMemcpyAsync on a dedicated non-blocking copy stream and guarded by a HIP event, so the copy
// of batch i+1 runs under the compute of batch i and a slot is only refilled once its previous
// copy has landed.  The consumer makes its compute stream wait on the slot's event (no host
// sync on the hot path).  Reference: torch.utils.data.DataLoader(pin_memory=...) +
// .to(device) of the reference scripts (distributed_cnn.py:128-133, distributed_lstm.py:157-165).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;
using u = uintptr_t;

static void hchk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("sparkmi._io.") + what + ": " + hipGetErrorString(e));
}

struct PinnedRing {
  std::vector<void*> slots;
  std::vector<hipEvent_t> done;  // recorded on the copy stream after each slot's H2D copy
  std::vector<char> armed;       // slot has an outstanding copy event
  size_t slot_bytes = 0;
  int device = 0;
  hipStream_t copy = nullptr;
  int threads = 4;

  PinnedRing(size_t bytes, int nslots, int dev, int nthreads) : slot_bytes(bytes), device(dev), threads(nthreads) {
    if (nslots < 2 || bytes == 0) throw std::runtime_error("sparkmi._io.PinnedRing: need >= 2 slots of > 0 bytes");
    hchk(hipSetDevice(dev), "hipSetDevice");
    hchk(hipStreamCreateWithFlags(&copy, hipStreamNonBlocking), "hipStreamCreateWithFlags");
    slots.resize(nslots, nullptr);
    done.resize(nslots, nullptr);
    armed.resize(nslots, 0);
    for (int i = 0; i < nslots; ++i) {
      hchk(hipHostMalloc(&slots[i], bytes, hipHostMallocDefault), "hipHostMalloc");
      hchk(hipEventCreateWithFlags(&done[i], hipEventDisableTiming), "hipEventCreateWithFlags");
    }
  }
  ~PinnedRing() { release(); }

  void release() {
    if (copy) hipStreamSynchronize(copy);
    for (auto& e : done)
      if (e) { hipEventDestroy(e); e = nullptr; }
    for (auto& p : slots)
      if (p) { hipHostFree(p); p = nullptr; }
    if (copy) { hipStreamDestroy(copy); copy = nullptr; }
  }

  void check(int s) const {
    if (s < 0 || s >= (int)slots.size() || !slots[s]) throw std::runtime_error("sparkmi._io.PinnedRing: bad slot");
  }

  // block until slot s's previous copy has landed (the host may overwrite it afterwards)
  void acquire(int s) {
    check(s);
    if (armed[s]) {
      py::gil_scoped_release nogil;
      hchk(hipEventSynchronize(done[s]), "hipEventSynchronize");
    }
    armed[s] = 0;
  }

  // rows idx[0..n) of a host array (row_bytes each) -> slot s at byte offset off, in order
  void gather(int s, size_t off, u src, size_t row_bytes, u idx, long n) {
    check(s);
    if (off + row_bytes * (size_t)n > slot_bytes) throw std::runtime_error("sparkmi._io.PinnedRing.gather: slot overflow");
    const char* base = reinterpret_cast<const char*>(src);
    const int64_t* ix = reinterpret_cast<const int64_t*>(idx);
    char* dst = static_cast<char*>(slots[s]) + off;
    py::gil_scoped_release nogil;
    const int nt = (int)std::max<long>(1, std::min<long>(threads, n / 64));
    auto work = [&](int t) {
      const long lo = n * t / nt, hi = n * (t + 1) / nt;
      for (long i = lo; i < hi; ++i) std::memcpy(dst + (size_t)i * row_bytes, base + (size_t)ix[i] * row_bytes, row_bytes);
    };
    if (nt == 1) { work(0); return; }
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
  }

  // async H2D of slot s [off, off + nbytes) -> dst on the copy stream, after `after` (an event
  // recorded by the consumer when this device buffer was last released; 0 = none)
  void copy_async(int s, size_t off, size_t nbytes, u dst, u after) {
    check(s);
    if (off + nbytes > slot_bytes) throw std::runtime_error("sparkmi._io.PinnedRing.copy_async: slot overflow");
    if (after) hchk(hipStreamWaitEvent(copy, reinterpret_cast<hipEvent_t>(after), 0), "hipStreamWaitEvent");
    hchk(hipMemcpyAsync(reinterpret_cast<void*>(dst), static_cast<char*>(slots[s]) + off, nbytes,
                        hipMemcpyHostToDevice, copy), "hipMemcpyAsync");
  }

  // close slot s's copies: record its event (the consumer waits on it; acquire() blocks on it)
  void commit(int s) {
    check(s);
    hchk(hipEventRecord(done[s], copy), "hipEventRecord");
    armed[s] = 1;
  }

  // make `stream` (the consumer's compute stream) wait for slot s's copies — no host sync
  void wait(int s, u stream) {
    check(s);
    hchk(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), done[s], 0), "hipStreamWaitEvent");
  }

  py::memoryview view(int s) {
    check(s);
    return py::memoryview::from_memory(slots[s], (ssize_t)slot_bytes);
  }
};

PYBIND11_MODULE(_io, m) {
  m.doc() = "sparkmi native input pipeline: pinned host ring + threaded row gather + async H2D (MI355X)";
  py::class_<PinnedRing>(m, "PinnedRing")
      .def(py::init<size_t, int, int, int>(), py::arg("slot_bytes"), py::arg("nslots"), py::arg("device"),
           py::arg("threads") = 4)
      .def_readonly("slot_bytes", &PinnedRing::slot_bytes)
      .def_property_readonly("nslots", [](const PinnedRing& r) { return (int)r.slots.size(); })
      .def_property_readonly("copy_stream", [](const PinnedRing& r) { return (u)r.copy; })
      .def("acquire", &PinnedRing::acquire)
      .def("gather", &PinnedRing::gather)
      .def("copy_async", &PinnedRing::copy_async)
      .def("commit", &PinnedRing::commit)
      .def("wait", &PinnedRing::wait)
      .def("view", &PinnedRing::view)
      .def("release", &PinnedRing::release);
}
