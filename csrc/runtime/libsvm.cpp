// libsvm text parser -> CSR (label f64, indptr i64, indices i32 (0-based), values f64).
//
// Replaces Spark's LibSVMRelation (spark.read.format("libsvm").load(path) at
// mllib_multilayer_perceptron_classifier.py:22-23, distributed_multilayer_perceptron.py:62-63):
// lines "label idx:val idx:val ..." with 1-based ascending indices; numFeatures = max index
// unless given.  Multi-threaded: the buffer is split on line boundaries, each thread parses its
// span into private vectors, spans are concatenated in order (deterministic output).
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {
struct Part {
  std::vector<double> labels;
  std::vector<int64_t> row_nnz;
  std::vector<int32_t> idx;
  std::vector<double> val;
  int64_t max_index = 0;
  std::string error;
};

void parse_span(const char* b, const char* e, Part& p) {
  const char* s = b;
  int64_t lineno = 0;
  while (s < e) {
    const char* eol = (const char*)memchr(s, '\n', e - s);
    if (!eol) eol = e;
    ++lineno;
    // skip leading whitespace; ignore blank lines and '#' comments
    const char* c = s;
    while (c < eol && (*c == ' ' || *c == '\t' || *c == '\r')) ++c;
    if (c < eol && *c != '#') {
      char* endp = nullptr;
      double lab = strtod(c, &endp);
      if (endp == c) { p.error = "bad label"; return; }
      c = endp;
      int64_t nnz = 0;
      int64_t prev = 0;
      while (c < eol) {
        while (c < eol && (*c == ' ' || *c == '\t' || *c == '\r')) ++c;
        if (c >= eol || *c == '#') break;
        long long ix = strtoll(c, &endp, 10);
        if (endp == c || *endp != ':') { p.error = "bad index"; return; }
        if (ix < 1 || ix <= prev) { p.error = "indices must be 1-based and ascending"; return; }
        prev = ix;
        c = endp + 1;
        double v = strtod(c, &endp);
        if (endp == c) { p.error = "bad value"; return; }
        c = endp;
        p.idx.push_back((int32_t)(ix - 1));
        p.val.push_back(v);
        if (ix > p.max_index) p.max_index = ix;
        ++nnz;
      }
      p.labels.push_back(lab);
      p.row_nnz.push_back(nnz);
    }
    s = eol + 1;
  }
}
}  // namespace

py::tuple parse_libsvm_buffer(const std::string& buf, int nthreads) {
  const char* data = buf.data();
  const size_t n = buf.size();
  if (nthreads < 1) nthreads = 1;
  if (n < (1u << 20)) nthreads = 1;
  std::vector<size_t> cuts{0};
  for (int t = 1; t < nthreads; ++t) {
    size_t pos = n * t / nthreads;
    while (pos < n && data[pos - 1] != '\n') ++pos;
    if (pos > cuts.back()) cuts.push_back(pos);
  }
  cuts.push_back(n);
  std::vector<Part> parts(cuts.size() - 1);
  {
    py::gil_scoped_release nogil;
    std::vector<std::thread> th;
    for (size_t i = 0; i + 1 < cuts.size(); ++i)
      th.emplace_back(parse_span, data + cuts[i], data + cuts[i + 1], std::ref(parts[i]));
    for (auto& t : th) t.join();
  }
  int64_t rows = 0, nnz = 0, maxi = 0;
  for (auto& p : parts) {
    if (!p.error.empty()) throw std::runtime_error("libsvm parse error: " + p.error);
    rows += (int64_t)p.labels.size();
    nnz += (int64_t)p.idx.size();
    maxi = std::max(maxi, p.max_index);
  }
  py::array_t<double> labels(rows);
  py::array_t<int64_t> indptr(rows + 1);
  py::array_t<int32_t> indices(nnz);
  py::array_t<double> values(nnz);
  auto L = labels.mutable_unchecked<1>();
  auto IP = indptr.mutable_unchecked<1>();
  auto IX = indices.mutable_unchecked<1>();
  auto VA = values.mutable_unchecked<1>();
  int64_t r = 0, k = 0;
  IP(0) = 0;
  for (auto& p : parts) {
    size_t off = 0;
    for (size_t i = 0; i < p.labels.size(); ++i) {
      L(r) = p.labels[i];
      for (int64_t j = 0; j < p.row_nnz[i]; ++j, ++off, ++k) { IX(k) = p.idx[off]; VA(k) = p.val[off]; }
      IP(r + 1) = k;
      ++r;
    }
  }
  return py::make_tuple(labels, indptr, indices, values, maxi);
}

py::tuple parse_libsvm_file(const std::string& path, int nthreads) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return parse_libsvm_buffer(ss.str(), nthreads);
}

void register_libsvm(py::module_& m) {
  m.def("parse_libsvm_buffer", &parse_libsvm_buffer, py::arg("buf"), py::arg("nthreads") = 4);
  m.def("parse_libsvm_file", &parse_libsvm_file, py::arg("path"), py::arg("nthreads") = 4);
}
