// Text pipeline: torchtext-compatible basic_english tokenizer, specials-first Vocab, and the
// Vocab -> AddToken(sos) -> Truncate -> AddToken(eos) -> ToTensor(pad) -> PadTransform chain
// fused into one batch encoder that writes an int64 [B, T] array.
//
// Reference: get_tokenizer('basic_english') (distributed_lstm.py:75),
// build_vocab_from_iterator(min_freq=1, specials=['<pad>','<sos>','<eos>','<unk>'],
// special_first=True) + set_default_index(<unk>) (distributed_lstm.py:87-94), and the
// T.Sequential transforms (distributed_lstm.py:96-107, pytorch_machine_translator.py:70-98).
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>
#include <algorithm>
#include <cctype>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

// basic_english: lowercase, then in order
//   '  -> " '  "   "  -> ""   . -> " . "   <br /> -> " "   , -> " , "   ( -> " ( "   ) -> " ) "
//   ! -> " ! "     ? -> " ? " ; -> " "     : -> " "       \s+ -> " "      then split on spaces.
// Sequential regex substitutions of single characters commute except for "<br />", which is
// matched on the text after the quote/period rules (it contains neither), so a single left-to-
// right scan is equivalent.
std::vector<std::string> tokenize_basic_english(const std::string& line) {
  std::string s;
  s.reserve(line.size() * 2);
  for (size_t i = 0; i < line.size(); ++i) {
    unsigned char c = (unsigned char)line[i];
    char lc = (char)std::tolower(c);
    if (lc == '<' && line.compare(i, 6, "<br />") == 0) { s += ' '; i += 5; continue; }
    switch (lc) {
      case '\'': s += " '  "; break;
      case '"': break;
      case '.': s += " . "; break;
      case ',': s += " , "; break;
      case '(': s += " ( "; break;
      case ')': s += " ) "; break;
      case '!': s += " ! "; break;
      case '?': s += " ? "; break;
      case ';': case ':': s += ' '; break;
      case ' ': case '\t': case '\n': case '\r': case '\f': case '\v': s += ' '; break;
      default: s += lc;
    }
  }
  std::vector<std::string> out;
  size_t i = 0;
  while (i < s.size()) {
    while (i < s.size() && s[i] == ' ') ++i;
    size_t j = i;
    while (j < s.size() && s[j] != ' ') ++j;
    if (j > i) out.emplace_back(s.substr(i, j - i));
    i = j;
  }
  return out;
}

std::vector<std::vector<std::string>> tokenize_batch(const std::vector<std::string>& lines) {
  std::vector<std::vector<std::string>> out(lines.size());
  for (size_t i = 0; i < lines.size(); ++i) out[i] = tokenize_basic_english(lines[i]);
  return out;
}

class Vocab {
 public:
  Vocab() = default;
  explicit Vocab(const std::vector<std::string>& itos) : itos_(itos) {
    for (size_t i = 0; i < itos_.size(); ++i) stoi_.emplace(itos_[i], (int64_t)i);
  }
  // counts: token -> frequency. Order: specials (if special_first), then freq desc, token asc.
  static Vocab build(const std::unordered_map<std::string, int64_t>& counts, int64_t min_freq,
                     const std::vector<std::string>& specials, bool special_first) {
    std::vector<std::pair<std::string, int64_t>> items;
    items.reserve(counts.size());
    for (auto& kv : counts) {
      if (std::find(specials.begin(), specials.end(), kv.first) != specials.end()) continue;
      if (kv.second >= min_freq) items.push_back(kv);
    }
    std::sort(items.begin(), items.end(), [](const auto& a, const auto& b) {
      if (a.second != b.second) return a.second > b.second;
      return a.first < b.first;
    });
    std::vector<std::string> itos;
    if (special_first) itos.insert(itos.end(), specials.begin(), specials.end());
    for (auto& kv : items) itos.push_back(kv.first);
    if (!special_first) itos.insert(itos.end(), specials.begin(), specials.end());
    return Vocab(itos);
  }
  int64_t size() const { return (int64_t)itos_.size(); }
  void set_default_index(int64_t i) { default_ = i; }
  int64_t default_index() const { return default_; }
  int64_t lookup(const std::string& t) const {
    auto it = stoi_.find(t);
    if (it != stoi_.end()) return it->second;
    if (default_ < 0) throw std::out_of_range("token '" + t + "' not in vocab and no default index");
    return default_;
  }
  bool contains(const std::string& t) const { return stoi_.count(t) > 0; }
  const std::vector<std::string>& itos() const { return itos_; }

  // Fused transform chain. max_len: Truncate length applied after sos (torchtext Truncate keeps
  // the first max_len items of [sos]+ids); pad_to: final length (0 = longest in batch).
  py::array_t<int64_t> encode_batch(const std::vector<std::vector<std::string>>& toks, int64_t sos, int64_t eos,
                                    int64_t max_len, int64_t pad, int64_t pad_to) const {
    std::vector<std::vector<int64_t>> ids(toks.size());
    size_t longest = 0;
    for (size_t i = 0; i < toks.size(); ++i) {
      auto& v = ids[i];
      if (sos >= 0) v.push_back(sos);
      for (auto& t : toks[i]) v.push_back(lookup(t));
      if (max_len > 0 && (int64_t)v.size() > max_len) v.resize(max_len);
      if (eos >= 0) v.push_back(eos);
      longest = std::max(longest, v.size());
    }
    const size_t T = pad_to > 0 ? std::max<size_t>((size_t)pad_to, 0) : longest;
    py::array_t<int64_t> out({(py::ssize_t)toks.size(), (py::ssize_t)T});
    auto O = out.mutable_unchecked<2>();
    for (size_t i = 0; i < toks.size(); ++i)
      for (size_t j = 0; j < T; ++j) O(i, j) = j < ids[i].size() ? ids[i][j] : pad;
    return out;
  }

 private:
  std::vector<std::string> itos_;
  std::unordered_map<std::string, int64_t> stoi_;
  int64_t default_ = -1;
};

std::unordered_map<std::string, int64_t> count_tokens(const std::vector<std::string>& lines) {
  std::unordered_map<std::string, int64_t> c;
  for (auto& l : lines)
    for (auto& t : tokenize_basic_english(l)) ++c[t];
  return c;
}

void register_text(py::module_& m) {
  m.def("tokenize_basic_english", &tokenize_basic_english);
  m.def("tokenize_batch", &tokenize_batch);
  m.def("count_tokens", &count_tokens);
  py::class_<Vocab>(m, "Vocab")
      .def(py::init<const std::vector<std::string>&>())
      .def_static("build", &Vocab::build, py::arg("counts"), py::arg("min_freq") = 1,
                  py::arg("specials") = std::vector<std::string>{}, py::arg("special_first") = true)
      .def("__len__", &Vocab::size)
      .def("__getitem__", &Vocab::lookup)
      .def("__contains__", &Vocab::contains)
      .def("set_default_index", &Vocab::set_default_index)
      .def("get_default_index", &Vocab::default_index)
      .def("get_itos", &Vocab::itos)
      .def("lookup_indices", [](const Vocab& v, const std::vector<std::string>& ts) {
        std::vector<int64_t> r;
        r.reserve(ts.size());
        for (auto& t : ts) r.push_back(v.lookup(t));
        return r;
      })
      .def("encode_batch", &Vocab::encode_batch, py::arg("tokens"), py::arg("sos") = -1, py::arg("eos") = -1,
           py::arg("max_len") = 0, py::arg("pad") = 0, py::arg("pad_to") = 0);
}
