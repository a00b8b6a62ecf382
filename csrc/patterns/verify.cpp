// Native verification of regex candidate lines and context-window extraction
// (SURVEY.md §2.4 N3 "line_index + context windows" and N4 "verify": "Confirms
// regex candidates flagged by N1 on the matched line only ... bit-exact with the
// Python regex oracle"). Replaces the log-parser's matching semantics behind
// J/service/LogParserRestClient.java:37-39.
//
// * RegexProg: a Pike VM (Thompson NFA simulation) over a bytecode the Python side
//   compiles from the sre_parse tree of each matcher (operator_amd/patterns/
//   nfa.py). Verification only asks "does the line contain a match" (re.search
//   is not None), which is independent of greedy / lazy order for the regular
//   subset compiled here (literals, classes, ., alternation, groups, bounded and
//   unbounded repeats, ^ $ \A \Z \b \B); a regex outside it (backreferences,
//   lookaround, ...) is marked for Python `re` by the compiler, so results are
//   exact by construction.
// * postprocess_hits: raw GPU factor hits (doc, factor, line, end offset) ->
//   matcher hits, verified on the candidate line, de-duplicated on (doc, matcher,
//   line) — the loop that used to run in Python per hit.
// * line_scan: matchers with no usable factor, run over every line natively.
// * contexts: the +-k line windows of each reported event, decoded to str.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <tuple>
#include <vector>

namespace py = pybind11;

namespace {

// Opcodes (keep in sync with operator_amd/patterns/nfa.py)
enum Op : int32_t { CHAR = 0, CLASS = 1, ANY = 2, SPLIT = 3, JMP = 4, ASSERT = 5, MATCH = 6 };
enum Assert : int32_t { BOL = 0, EOL = 1, WORDB = 2, NWORDB = 3 };

inline bool is_word(uint8_t c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
}

struct Prog {
  std::vector<std::array<int32_t, 3>> ins;
  std::vector<std::array<uint64_t, 4>> cls;
  bool valid = false;
};

class Matcher {
 public:
  explicit Matcher(const Prog& p) : p_(p), n_((int)p.ins.size()) {
    for (auto& l : lists_) {
      l.dense.resize(n_);
      l.sparse.assign(n_, -1);
    }
    stack_.reserve(n_ * 2);
  }

  // re.search(line) is not None
  bool search(const uint8_t* s, size_t len) {
    List* cur = &lists_[0];
    List* nxt = &lists_[1];
    cur->clear();
    for (size_t i = 0;; ++i) {
      add(*cur, 0, s, len, i);   // unanchored: a new thread at every position
      if (cur->matched) return true;
      if (i == len) return false;
      const uint8_t c = s[i];
      nxt->clear();
      for (int k = 0; k < cur->size; ++k) {
        const int pc = cur->dense[k];
        const auto& in = p_.ins[pc];
        bool ok = false;
        switch (in[0]) {
          case CHAR: ok = c == (uint8_t)in[1]; break;
          case CLASS: ok = (p_.cls[in[1]][c >> 6] >> (c & 63)) & 1; break;
          case ANY: ok = c != '\n'; break;
          default: break;
        }
        if (ok) add(*nxt, pc + 1, s, len, i + 1);
        if (nxt->matched) return true;
      }
      std::swap(cur, nxt);
      if (cur->size == 0 && i + 1 > len) return false;
    }
  }

 private:
  struct List {
    std::vector<int> dense, sparse;
    int size = 0;
    bool matched = false;
    void clear() {
      size = 0;
      matched = false;
    }
    bool has(int pc) const {
      const int d = sparse[pc];
      return d >= 0 && d < size && dense[d] == pc;
    }
    void put(int pc) {
      sparse[pc] = size;
      dense[size++] = pc;
    }
  };

  // epsilon closure of `pc` at position `pos` into `l` (consuming ops and MATCH kept)
  void add(List& l, int pc0, const uint8_t* s, size_t len, size_t pos) {
    stack_.clear();
    stack_.push_back(pc0);
    while (!stack_.empty()) {
      const int pc = stack_.back();
      stack_.pop_back();
      if (pc >= n_ || l.has(pc)) continue;
      l.put(pc);
      const auto& in = p_.ins[pc];
      switch (in[0]) {
        case JMP: stack_.push_back(in[1]); break;
        case SPLIT:
          stack_.push_back(in[2]);
          stack_.push_back(in[1]);
          break;
        case ASSERT: {
          bool ok = false;
          const bool wb = pos > 0 && is_word(s[pos - 1]);
          const bool wa = pos < len && is_word(s[pos]);
          switch (in[1]) {
            case BOL: ok = pos == 0; break;
            case EOL: ok = pos == len; break;
            case WORDB: ok = wb != wa; break;
            case NWORDB: ok = wb == wa; break;
          }
          if (ok) stack_.push_back(pc + 1);
          break;
        }
        case MATCH: l.matched = true; break;
        default: break;
      }
    }
  }

  const Prog& p_;
  int n_;
  List lists_[2];
  std::vector<int> stack_;
};

// A pattern set's compiled verifiers: entry m is matcher m's program, or invalid
// (the matcher needs no regex, or needs Python `re`).
class RegexSet {
 public:
  explicit RegexSet(const std::vector<py::object>& progs) {
    progs_.resize(progs.size());
    for (size_t m = 0; m < progs.size(); ++m) {
      if (progs[m].is_none()) continue;
      auto t = progs[m].cast<py::tuple>();
      const std::string ins = t[0].cast<std::string>(), cls = t[1].cast<std::string>();
      if (ins.size() % 12 != 0 || cls.size() % 32 != 0) throw std::invalid_argument("RegexSet: bad program");
      Prog& p = progs_[m];
      p.ins.resize(ins.size() / 12);
      std::memcpy(p.ins.data(), ins.data(), ins.size());
      p.cls.resize(cls.size() / 32);
      std::memcpy(p.cls.data(), cls.data(), cls.size());
      for (const auto& in : p.ins) {
        const int n = (int)p.ins.size();
        if (in[0] < CHAR || in[0] > MATCH) throw std::invalid_argument("RegexSet: bad opcode");
        if ((in[0] == SPLIT || in[0] == JMP) && (in[1] < 0 || in[1] >= n || (in[0] == SPLIT && (in[2] < 0 || in[2] >= n))))
          throw std::invalid_argument("RegexSet: jump out of range");
        if (in[0] == CLASS && (in[1] < 0 || in[1] >= (int)p.cls.size())) throw std::invalid_argument("RegexSet: class");
      }
      p.valid = !p.ins.empty();
    }
  }
  bool has(int m) const { return m >= 0 && m < (int)progs_.size() && progs_[m].valid; }
  const Prog& prog(int m) const { return progs_[m]; }
  size_t size() const { return progs_.size(); }

  bool search_one(int m, const py::bytes& line) const {
    if (!has(m)) throw std::invalid_argument("RegexSet: no native program for this matcher");
    const std::string_view v(PyBytes_AS_STRING(line.ptr()), (size_t)PyBytes_GET_SIZE(line.ptr()));
    Matcher mt(progs_[m]);
    return mt.search(reinterpret_cast<const uint8_t*>(v.data()), v.size());
  }

 private:
  std::vector<Prog> progs_;
};

std::vector<std::string_view> views(const std::vector<py::bytes>& docs) {
  std::vector<std::string_view> v;
  v.reserve(docs.size());
  for (const auto& d : docs) v.emplace_back(PyBytes_AS_STRING(d.ptr()), (size_t)PyBytes_GET_SIZE(d.ptr()));
  return v;
}

inline std::pair<size_t, size_t> line_bounds(std::string_view d, size_t off) {
  if (off > d.size()) off = d.size();
  size_t s = off;
  while (s > 0 && d[s - 1] != '\n') --s;
  const void* e = off < d.size() ? std::memchr(d.data() + off, '\n', d.size() - off) : nullptr;
  return {s, e ? (size_t)(static_cast<const char*>(e) - d.data()) : d.size()};
}

// raw [n, 4] (doc, factor, line, end_offset) -> (hits [k, 4] (doc, matcher, line, offset) sorted unique,
// pending [p, 4] candidates whose matcher needs Python re, one per (doc, matcher, line))
py::tuple postprocess_hits(py::array_t<int64_t, py::array::c_style | py::array::forcecast> raw,
                           py::array_t<int64_t, py::array::c_style | py::array::forcecast> fm_ptr,
                           py::array_t<int64_t, py::array::c_style | py::array::forcecast> fm_ids,
                           py::array_t<int8_t, py::array::c_style | py::array::forcecast> mode,
                           const std::vector<py::bytes>& docs, const RegexSet& rs) {
  if (raw.ndim() != 2 || (raw.shape(0) > 0 && raw.shape(1) != 4)) throw std::invalid_argument("raw must be [n, 4]");
  const int64_t n = raw.shape(0);
  const int64_t* r = raw.data();
  const int64_t* fp = fm_ptr.data();
  const int64_t* fi = fm_ids.data();
  const int8_t* md = mode.data();
  const int64_t nf = fm_ptr.size() - 1, nm = mode.size(), nfi = fm_ids.size();
  const auto dv = views(docs);
  using K = std::tuple<int64_t, int64_t, int64_t, int64_t>;   // doc, matcher, line, offset
  std::vector<K> cand;
  {
    py::gil_scoped_release nogil;
    for (int64_t i = 0; i < n; ++i) {
      const int64_t d = r[4 * i], f = r[4 * i + 1], l = r[4 * i + 2], o = r[4 * i + 3];
      if (f < 0 || f >= nf || d < 0 || d >= (int64_t)dv.size()) continue;
      for (int64_t j = fp[f]; j < fp[f + 1] && j < nfi; ++j) cand.emplace_back(d, fi[j], l, o);
    }
    std::sort(cand.begin(), cand.end());
  }
  std::vector<K> hits, pending;
  {
    py::gil_scoped_release nogil;
    std::vector<Matcher*> mts(nm, nullptr);
    std::vector<std::unique_ptr<Matcher>> own;
    for (size_t i = 0; i < cand.size(); ++i) {
      const auto& [d, m, l, o] = cand[i];
      if (i > 0 && std::get<0>(cand[i - 1]) == d && std::get<1>(cand[i - 1]) == m && std::get<2>(cand[i - 1]) == l)
        continue;   // one decision per (doc, matcher, line)
      if (m < 0 || m >= nm) continue;
      const int8_t mode_m = md[m];
      if (mode_m == 0) {
        hits.push_back(cand[i]);
      } else if (mode_m == 1 && rs.has((int)m)) {
        if (!mts[m]) {
          own.emplace_back(new Matcher(rs.prog((int)m)));
          mts[m] = own.back().get();
        }
        const auto [s, e] = line_bounds(dv[d], (size_t)o);
        if (mts[m]->search(reinterpret_cast<const uint8_t*>(dv[d].data()) + s, e - s)) hits.push_back(cand[i]);
      } else {
        pending.push_back(cand[i]);
      }
    }
  }
  auto to_arr = [](const std::vector<K>& v) {
    py::array_t<int64_t> a({(py::ssize_t)v.size(), (py::ssize_t)4});
    int64_t* p = a.mutable_data();
    for (size_t i = 0; i < v.size(); ++i) {
      p[4 * i] = std::get<0>(v[i]);
      p[4 * i + 1] = std::get<1>(v[i]);
      p[4 * i + 2] = std::get<2>(v[i]);
      p[4 * i + 3] = std::get<3>(v[i]);
    }
    return a;
  };
  return py::make_tuple(to_arr(hits), to_arr(pending));
}

// Every line of every doc against matcher m's program: [k, 4] (doc, m, line, offset)
// with offset = the last byte of the line (its start if empty), as the Python path.
py::array_t<int64_t> line_scan(const std::vector<py::bytes>& docs, const RegexSet& rs, int m) {
  if (!rs.has(m)) throw std::invalid_argument("line_scan: no native program");
  const auto dv = views(docs);
  std::vector<int64_t> out;
  {
    py::gil_scoped_release nogil;
    Matcher mt(rs.prog(m));
    for (size_t d = 0; d < dv.size(); ++d) {
      const auto v = dv[d];
      size_t s = 0;
      int64_t li = 0;
      while (true) {
        const void* e = s < v.size() ? std::memchr(v.data() + s, '\n', v.size() - s) : nullptr;
        const size_t le = e ? (size_t)(static_cast<const char*>(e) - v.data()) : v.size();
        if (mt.search(reinterpret_cast<const uint8_t*>(v.data()) + s, le - s)) {
          out.insert(out.end(), {(int64_t)d, (int64_t)m, li, (int64_t)(le > s ? le - 1 : s)});
        }
        if (!e) break;
        s = le + 1;
        ++li;
      }
    }
  }
  py::array_t<int64_t> a({(py::ssize_t)(out.size() / 4), (py::ssize_t)4});
  if (!out.empty()) std::memcpy(a.mutable_data(), out.data(), out.size() * 8);
  return a;
}

py::str decode(std::string_view v) {
  PyObject* o = PyUnicode_DecodeUTF8(v.data(), (Py_ssize_t)v.size(), "replace");
  if (!o) throw py::error_already_set();
  return py::reinterpret_steal<py::str>(o);
}

// For each (doc, offset, k): ([k lines before..., the line, k lines after...], the line),
// decoded UTF-8 with replacement — the +-k context window of a reported event.
py::list contexts(const std::vector<py::bytes>& docs, const std::vector<int64_t>& doc_idx,
                  const std::vector<int64_t>& offs, const std::vector<int64_t>& ks) {
  if (doc_idx.size() != offs.size() || offs.size() != ks.size()) throw std::invalid_argument("contexts: lengths");
  const auto dv = views(docs);
  py::list out(offs.size());
  std::vector<std::pair<size_t, size_t>> spans;
  for (size_t i = 0; i < offs.size(); ++i) {
    if (doc_idx[i] < 0 || doc_idx[i] >= (int64_t)dv.size()) throw std::out_of_range("contexts: doc index");
    const auto d = dv[doc_idx[i]];
    const auto [s, e] = line_bounds(d, (size_t)std::max<int64_t>(0, offs[i]));
    const int64_t k = std::max<int64_t>(0, ks[i]);
    spans.clear();
    size_t ps = s;
    for (int64_t j = 0; j < k && ps > 0; ++j) {   // lines before, nearest first
      const size_t pe = ps - 1;
      size_t b = pe;
      while (b > 0 && d[b - 1] != '\n') --b;
      spans.emplace_back(b, pe);
      ps = b;
    }
    std::reverse(spans.begin(), spans.end());
    spans.emplace_back(s, e);
    size_t ne = e;
    for (int64_t j = 0; j < k; ++j) {   // lines after
      if (ne >= d.size() || ne + 1 >= d.size()) break;
      const size_t ns = ne + 1;
      const void* f = std::memchr(d.data() + ns, '\n', d.size() - ns);
      ne = f ? (size_t)(static_cast<const char*>(f) - d.data()) : d.size();
      spans.emplace_back(ns, ne);
    }
    py::list ctx(spans.size());
    py::str line;
    for (size_t j = 0; j < spans.size(); ++j) {
      py::str t = decode(d.substr(spans[j].first, spans[j].second - spans[j].first));
      if (spans[j].first == s && spans[j].second == e) line = t;
      ctx[j] = t;
    }
    out[i] = py::make_tuple(ctx, line);
  }
  return out;
}

// The same (context lines, line) tuples from windows located on the GPU (line_index.hip
// context_spans): spans [n, 4] = (window start, window end, line start, line end) of doc
// doc_idx[i]; the window is split at every '\n' (the GPU already found the k lines).
py::list contexts_from_spans(const std::vector<py::bytes>& docs, const std::vector<int64_t>& doc_idx,
                             py::array_t<int64_t, py::array::c_style | py::array::forcecast> spans) {
  const auto dv = views(docs);
  if (spans.ndim() != 2 || spans.shape(1) != 4 || (size_t)spans.shape(0) < doc_idx.size())
    throw std::invalid_argument("contexts_from_spans: spans [n, 4]");
  const int64_t* sp = spans.data();
  py::list out(doc_idx.size());
  for (size_t i = 0; i < doc_idx.size(); ++i) {
    if (doc_idx[i] < 0 || doc_idx[i] >= (int64_t)dv.size()) throw std::out_of_range("contexts_from_spans: doc");
    const auto d = dv[doc_idx[i]];
    const int64_t* r = sp + 4 * i;
    if (r[0] < 0 || r[0] > r[2] || r[2] > r[3] || r[3] > r[1] || r[1] > (int64_t)d.size())
      throw std::out_of_range("contexts_from_spans: span outside its document");
    py::list ctx;
    size_t a = (size_t)r[0];
    const size_t we = (size_t)r[1];
    while (true) {
      const void* f = a < we ? std::memchr(d.data() + a, '\n', we - a) : nullptr;
      const size_t b = f ? (size_t)(static_cast<const char*>(f) - d.data()) : we;
      ctx.append(decode(d.substr(a, b - a)));
      if (!f) break;
      a = b + 1;
    }
    out[i] = py::make_tuple(ctx, decode(d.substr((size_t)r[2], (size_t)(r[3] - r[2]))));
  }
  return out;
}

}  // namespace

void register_verify(py::module_& m) {
  py::class_<RegexSet>(m, "RegexSet")
      .def(py::init<const std::vector<py::object>&>(), py::arg("programs"))
      .def("has", &RegexSet::has)
      .def("search", &RegexSet::search_one, py::arg("matcher"), py::arg("line"))
      .def("__len__", &RegexSet::size);
  m.def("postprocess_hits", &postprocess_hits, py::arg("raw"), py::arg("fm_ptr"), py::arg("fm_ids"), py::arg("mode"),
        py::arg("docs"), py::arg("regexes"));
  m.def("line_scan", &line_scan, py::arg("docs"), py::arg("regexes"), py::arg("matcher"));
  m.def("contexts", &contexts, py::arg("docs"), py::arg("doc_idx"), py::arg("offsets"), py::arg("k"));
  m.def("contexts_from_spans", &contexts_from_spans, py::arg("docs"), py::arg("doc_idx"), py::arg("spans"));
}
