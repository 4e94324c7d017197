// sparkmi._runtime: host-side C++ runtime (data IO and text processing).
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <cstdint>
#include <random>

namespace py = pybind11;
void register_libsvm(py::module_& m);
void register_text(py::module_& m);

// Deterministic Fisher-Yates permutation (mt19937_64) used for epoch shuffles on the host side.
static py::array_t<int64_t> permutation(int64_t n, uint64_t seed) {
  py::array_t<int64_t> out(n);
  auto o = out.mutable_unchecked<1>();
  for (int64_t i = 0; i < n; ++i) o(i) = i;
  std::mt19937_64 rng(seed);
  for (int64_t i = n - 1; i > 0; --i) {
    std::uniform_int_distribution<int64_t> d(0, i);
    std::swap(o(i), o(d(rng)));
  }
  return out;
}

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "sparkmi host runtime: libsvm IO, basic_english tokenizer, vocab encoder";
  register_libsvm(m);
  register_text(m);
  m.def("permutation", &permutation, py::arg("n"), py::arg("seed"));
}
