// Host-side pattern data plane (operator_amd._patterns), CPU only.
//
//  * compile_dfa   (SURVEY.md §2.4 N1): literal factors -> Aho-Corasick trie ->
//    complete DFA over case-folded byte equivalence classes, states numbered
//    breadth-first (shallow = hot = first rows, staged in LDS by ac_scan),
//    uint16 table with an "has outputs" flag bit, CSR output lists.
//  * pack_docs: lays a batch of pod logs out for ac_scan (NUL-padded to a
//    multiple of the segment size) and memcpys them into a (pinned) staging
//    buffer with a thread pool, so H2D is one contiguous copy.
//  * score_events (SURVEY.md §2.4 N5 host path): turns verified factor hits
//    into scored events per doc (proximity search of secondary matchers), the
//    same algorithm as operator_amd/patterns/oracle.py.
//
// Replaces the reference's external log-parser (J/service/LogParserClient.java:36-55);
// the pattern schema and scoring are our design.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

constexpr int kMaxFactorLen = 64;
constexpr uint32_t kMaxStates = 32768;

inline uint8_t fold(uint8_t b) { return (b >= 'A' && b <= 'Z') ? uint8_t(b + 32) : b; }

py::dict compile_dfa(const std::vector<std::string>& factors) {
  // ---- byte classes: class 0 = every byte that occurs in no factor ----
  std::array<int, 256> cls{};
  cls.fill(0);
  int nclass = 1;
  for (const auto& f : factors) {
    if (f.empty()) throw std::invalid_argument("empty factor");
    if (f.size() > kMaxFactorLen) throw std::invalid_argument("factor longer than 64 bytes");
    for (unsigned char c : f) {
      if (c == 0 || c == '\n') throw std::invalid_argument("factor contains NUL or newline");
      const uint8_t b = fold(c);
      if (cls[b] == 0) cls[b] = nclass++;
    }
  }
  for (int b = 'A'; b <= 'Z'; ++b) cls[b] = cls[b + 32];
  int log2c = 3;
  while ((1 << log2c) < nclass) ++log2c;
  const int C = 1 << log2c;

  // ---- trie (goto function) ----
  std::vector<std::vector<int32_t>> go;  // [state][class] -> child or -1
  std::vector<std::vector<uint32_t>> own_out;
  std::vector<int> depth;
  go.emplace_back(C, -1);
  own_out.emplace_back();
  depth.push_back(0);
  size_t max_len = 0;
  for (size_t fi = 0; fi < factors.size(); ++fi) {
    int s = 0;
    for (unsigned char c : factors[fi]) {
      const int k = cls[fold(c)];
      if (go[s][k] < 0) {
        go[s][k] = static_cast<int32_t>(go.size());
        go.emplace_back(C, -1);
        own_out.emplace_back();
        depth.push_back(depth[s] + 1);
        if (go.size() > kMaxStates) throw std::length_error("pattern set exceeds 32768 DFA states");
      }
      s = go[s][k];
    }
    own_out[s].push_back(static_cast<uint32_t>(fi));
    max_len = std::max(max_len, factors[fi].size());
  }
  const size_t S = go.size();

  // ---- BFS: failure links, complete transitions, BFS renumbering ----
  std::vector<int32_t> fail(S, 0), order;
  order.reserve(S);
  std::vector<std::vector<int32_t>> delta(S, std::vector<int32_t>(C, 0));
  std::vector<std::vector<uint32_t>> out(S);
  std::deque<int32_t> q;
  order.push_back(0);
  for (int k = 0; k < C; ++k) {
    const int32_t c = go[0][k];
    if (c > 0) { fail[c] = 0; delta[0][k] = c; q.push_back(c); }
    else delta[0][k] = 0;
  }
  out[0] = own_out[0];
  while (!q.empty()) {
    const int32_t s = q.front();
    q.pop_front();
    order.push_back(s);
    out[s] = own_out[s];
    for (uint32_t o : out[fail[s]]) out[s].push_back(o);
    for (int k = 0; k < C; ++k) {
      const int32_t c = go[s][k];
      if (c > 0) {
        fail[c] = delta[fail[s]][k];
        delta[s][k] = c;
        q.push_back(c);
      } else {
        delta[s][k] = delta[fail[s]][k];
      }
    }
  }
  std::vector<uint32_t> rank(S);
  for (size_t i = 0; i < S; ++i) rank[order[i]] = static_cast<uint32_t>(i);

  std::string table(S * C * 2, '\0');
  auto* tab = reinterpret_cast<uint16_t*>(&table[0]);
  std::vector<uint32_t> out_off(S + 1, 0), out_ids;
  std::vector<int> depth_bfs(S);
  for (size_t i = 0; i < S; ++i) {
    const int32_t s = order[i];
    depth_bfs[i] = depth[s];
    for (int k = 0; k < C; ++k) {
      const int32_t n = delta[s][k];
      uint16_t e = static_cast<uint16_t>(rank[n]);
      if (!out[n].empty()) e |= 0x8000;
      tab[i * C + k] = e;
    }
    out_off[i] = static_cast<uint32_t>(out_ids.size());
    std::vector<uint32_t> o = out[s];
    std::sort(o.begin(), o.end());
    o.erase(std::unique(o.begin(), o.end()), o.end());
    out_ids.insert(out_ids.end(), o.begin(), o.end());
  }
  out_off[S] = static_cast<uint32_t>(out_ids.size());

  std::string cls_bytes(256, '\0');
  for (int b = 0; b < 256; ++b) cls_bytes[b] = static_cast<char>(cls[b]);
  py::dict d;
  d["cls_map"] = py::bytes(cls_bytes);
  d["log2_classes"] = log2c;
  d["num_classes_used"] = nclass;
  d["num_states"] = S;
  d["table"] = py::bytes(table);
  d["out_off"] = py::bytes(reinterpret_cast<const char*>(out_off.data()), out_off.size() * 4);
  d["out_ids"] = py::bytes(reinterpret_cast<const char*>(out_ids.data()), std::max<size_t>(out_ids.size(), 1) * 4);
  d["num_out"] = out_ids.size();
  d["max_len"] = max_len;
  d["depth"] = depth_bfs;
  return d;
}

// Profile-guided state numbering for ac_scan's LDS hot set. Breadth-first order
// is only a proxy for "often visited": on log text, 0.4 % of transitions leave
// the first 1024 BFS states, but with 128 chains per wave that puts 42 % of the
// wave's byte steps behind an L2 / Infinity-Cache round trip (measured on the
// 1000-pattern synthetic library). Here the DFA is walked over a sample of the
// text actually being scanned, states are ranked by visit count (root stays 0,
// unvisited states keep BFS order after the visited ones), and the table and
// output lists are permuted. Matches are invariant under renumbering; only the
// hot prefix the kernel stages in LDS changes. Returns the permuted arrays and
// the fraction of sampled transitions that land in the first `hot` states
// before and after.
py::dict reorder_dfa(const std::string& table_b, const std::string& out_off_b, const std::string& out_ids_b,
                     int log2c, int64_t num_states, const std::string& cls_b, const std::string& sample, int hot) {
  const int C = 1 << log2c;
  const int64_t S = num_states;
  if (static_cast<int64_t>(table_b.size()) != S * C * 2) throw std::invalid_argument("table size mismatch");
  if (static_cast<int64_t>(out_off_b.size()) != (S + 1) * 4) throw std::invalid_argument("out_off size mismatch");
  if (cls_b.size() != 256) throw std::invalid_argument("cls_map must have 256 entries");
  const auto* tab = reinterpret_cast<const uint16_t*>(table_b.data());
  const auto* off = reinterpret_cast<const uint32_t*>(out_off_b.data());
  const auto* ids = reinterpret_cast<const uint32_t*>(out_ids_b.data());
  const auto* cls = reinterpret_cast<const uint8_t*>(cls_b.data());
  std::vector<uint64_t> visits(S, 0);
  {
    py::gil_scoped_release nogil;
    uint32_t s = 0;
    for (unsigned char b : sample) {
      s = tab[(static_cast<size_t>(s) << log2c) | cls[b]] & 0x7fffu;
      ++visits[s];
    }
  }
  std::vector<uint32_t> order(S);
  for (int64_t i = 0; i < S; ++i) order[i] = static_cast<uint32_t>(i);
  // root first, then by visits (desc), ties in BFS order (stable)
  std::stable_sort(order.begin() + 1, order.end(), [&](uint32_t a, uint32_t b) { return visits[a] > visits[b]; });
  // The cold states (past the hot prefix) in CHAIN order: a cold excursion is a log
  // line matching a pattern literal, i.e. a walk down one trie path, one dependent
  // global-table read per byte in the kernel's exact re-walk. Numbered so that each
  // state's most-visited trie child (the goto edge: depth + 1) is the next state, the
  // walk follows `dfa_chain` bytes (16 states per 16-byte read) instead of the table.
  // Chains start at the shallowest unplaced state (depth = BFS distance from the root).
  const int64_t H = std::min<int64_t>(std::max(hot, 0), S);
  if (H < S) {
    std::vector<int32_t> depth(S, -1);
    std::vector<uint32_t> bfs;
    bfs.reserve(S);
    depth[0] = 0;
    bfs.push_back(0);
    for (size_t h = 0; h < bfs.size(); ++h) {
      const uint32_t s = bfs[h];
      for (int k = 0; k < C; ++k) {
        const uint32_t t = tab[static_cast<size_t>(s) * C + k] & 0x7fffu;
        if (depth[t] < 0) {
          depth[t] = depth[s] + 1;
          bfs.push_back(t);
        }
      }
    }
    std::vector<char> placed(S, 0);
    for (int64_t i = 0; i < H; ++i) placed[order[i]] = 1;
    std::vector<uint32_t> heads(order.begin() + H, order.end());
    std::stable_sort(heads.begin(), heads.end(), [&](uint32_t a, uint32_t b) { return depth[a] < depth[b]; });
    std::vector<uint32_t> chained(order.begin(), order.begin() + H);
    for (uint32_t h : heads) {
      for (uint32_t s = h; !placed[s];) {
        placed[s] = 1;
        chained.push_back(s);
        int64_t best = -1;
        for (int k = 0; k < C; ++k) {
          const uint32_t t = tab[static_cast<size_t>(s) * C + k] & 0x7fffu;
          if (!placed[t] && depth[t] == depth[s] + 1 && (best < 0 || visits[t] > visits[best])) best = t;
        }
        if (best < 0) break;
        s = static_cast<uint32_t>(best);
      }
    }
    order.swap(chained);
  }
  std::vector<uint32_t> rank(S);
  for (int64_t i = 0; i < S; ++i) rank[order[i]] = static_cast<uint32_t>(i);
  std::string nt(S * C * 2, '\0');
  auto* ntab = reinterpret_cast<uint16_t*>(&nt[0]);
  std::vector<uint32_t> noff(S + 1, 0), nids;
  nids.reserve(off[S]);
  for (int64_t i = 0; i < S; ++i) {
    const uint32_t o = order[i];
    for (int k = 0; k < C; ++k) {
      const uint16_t e = tab[static_cast<size_t>(o) * C + k];
      ntab[i * C + k] = static_cast<uint16_t>(rank[e & 0x7fffu] | (e & 0x8000u));
    }
    noff[i] = static_cast<uint32_t>(nids.size());
    for (uint32_t k = off[o]; k < off[o + 1]; ++k) nids.push_back(ids[k]);
  }
  noff[S] = static_cast<uint32_t>(nids.size());
  uint64_t total = 0, hot_before = 0, hot_after = 0;
  for (int64_t i = 0; i < S; ++i) {
    total += visits[i];
    if (i < hot) hot_before += visits[i];
    if (rank[i] < static_cast<uint32_t>(hot)) hot_after += visits[i];
  }
  py::dict d;
  d["table"] = py::bytes(nt);
  d["out_off"] = py::bytes(reinterpret_cast<const char*>(noff.data()), noff.size() * 4);
  d["out_ids"] = py::bytes(reinterpret_cast<const char*>(nids.data()), std::max<size_t>(nids.size(), 1) * 4);
  d["hot_before"] = total ? double(hot_before) / double(total) : 1.0;
  d["hot_after"] = total ? double(hot_after) / double(total) : 1.0;
  d["sampled"] = total;
  return d;
}

// Per-state chain byte for ac_scan's exact re-walk (csrc/kernels/scan.hip slow_sub):
// chain[s] = 0x40 | k | (0x80 if s + 1 has outputs) when class k takes s to s + 1, else 0.
// Only for <= 64 classes (all zero otherwise: the kernel then reads the table). Padded to
// a multiple of 16 bytes plus 16, so the kernel's aligned 16-byte window reads stay inside.
py::bytes dfa_chain(const std::string& table_b, int log2c, int64_t num_states) {
  const int C = 1 << log2c;
  const int64_t S = num_states;
  if (static_cast<int64_t>(table_b.size()) != S * C * 2) throw std::invalid_argument("table size mismatch");
  const auto* tab = reinterpret_cast<const uint16_t*>(table_b.data());
  std::string ch(static_cast<size_t>((S + 15) / 16 * 16 + 16), '\0');
  if (C <= 64) {
    for (int64_t s = 0; s + 1 < S; ++s)
      for (int k = 0; k < C; ++k) {
        const uint16_t e = tab[static_cast<size_t>(s) * C + k];
        if ((e & 0x7fffu) == static_cast<uint32_t>(s + 1)) {
          ch[s] = static_cast<char>(0x40 | k | ((e & 0x8000u) ? 0x80 : 0));
          break;
        }
      }
  }
  return py::bytes(ch);
}

// Layout: doc i occupies [first_seg[i]*seg, first_seg[i+1]*seg), content then NUL padding (>= 1 byte).
py::tuple plan_docs(const std::vector<size_t>& lens, int64_t seg) {
  if (seg < 64 || (seg & (seg - 1))) throw std::invalid_argument("seg_bytes must be a power of two >= 64");
  std::vector<int64_t> first(lens.size() + 1, 0);
  for (size_t i = 0; i < lens.size(); ++i) {
    const int64_t padded = (static_cast<int64_t>(lens[i]) + 1 + seg - 1) / seg;  // >= 1 NUL byte
    first[i + 1] = first[i] + padded;
  }
  return py::make_tuple(first.back() * seg, first);
}

// Copy docs into dst (uintptr, >= total bytes) per the plan, zero-filling padding. Multi-threaded.
void pack_docs(const std::vector<py::bytes>& docs, const std::vector<int64_t>& first, int64_t seg, uintptr_t dst,
               int threads) {
  if (first.size() != docs.size() + 1) throw std::invalid_argument("plan/doc count mismatch");
  std::vector<std::pair<const char*, size_t>> views(docs.size());
  for (size_t i = 0; i < docs.size(); ++i) {
    char* p = nullptr;
    Py_ssize_t n = 0;
    PyBytes_AsStringAndSize(docs[i].ptr(), &p, &n);
    views[i] = {p, static_cast<size_t>(n)};
    if (static_cast<int64_t>(n) + 1 > (first[i + 1] - first[i]) * seg) throw std::invalid_argument("plan too small");
  }
  char* out = reinterpret_cast<char*>(dst);
  auto work = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      char* d = out + first[i] * seg;
      const size_t cap = static_cast<size_t>((first[i + 1] - first[i]) * seg);
      std::memcpy(d, views[i].first, views[i].second);
      std::memset(d + views[i].second, 0, cap - views[i].second);
    }
  };
  py::gil_scoped_release nogil;
  threads = std::max(1, std::min<int>(threads, static_cast<int>(docs.size())));
  if (threads == 1) { work(0, docs.size()); return; }
  std::vector<std::thread> pool;
  const size_t per = (docs.size() + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const size_t lo = t * per, hi = std::min(docs.size(), lo + per);
    if (lo < hi) pool.emplace_back(work, lo, hi);
  }
  for (auto& th : pool) th.join();
}

// ---------------------------------------------------------------------------
// Event scoring. Inputs are per-hit arrays (doc, matcher, line) of VERIFIED,
// de-duplicated hits, plus per-pattern matcher tables. Algorithm (our design,
// mirrored exactly by operator_amd/patterns/oracle.py::score_doc):
//   for each primary hit (doc d, line L) of pattern p:
//     bonus = sum_j w_j * (1 - |dL_j| / (W_j + 1))  over secondaries j whose
//             nearest hit in doc d lies within |dL_j| <= W_j
//     score = confidence_p * (1 + bonus) / (1 + sum_j w_j)
// Events are sorted by (score desc, severity desc, doc line asc, pattern asc).
// ---------------------------------------------------------------------------
struct PatSpec {
  int primary;
  double confidence;
  int severity;
  std::vector<int> sec;
  std::vector<double> weight;
  std::vector<int> window;
};

py::list score_events(const std::vector<int64_t>& hit_doc, const std::vector<int64_t>& hit_matcher,
                      const std::vector<int64_t>& hit_line, int64_t num_docs, const std::vector<int64_t>& pat_primary,
                      const std::vector<double>& pat_conf, const std::vector<int64_t>& pat_sev,
                      const std::vector<std::vector<int64_t>>& pat_sec, const std::vector<std::vector<double>>& pat_w,
                      const std::vector<std::vector<int64_t>>& pat_win, int64_t num_matchers) {
  const size_t n = hit_doc.size();
  if (hit_matcher.size() != n || hit_line.size() != n) throw std::invalid_argument("hit arrays differ in length");
  const size_t P = pat_primary.size();
  // (doc, matcher) -> sorted lines
  std::vector<std::vector<std::pair<int64_t, int64_t>>> by_doc(num_docs);  // (matcher, line)
  for (size_t i = 0; i < n; ++i) {
    if (hit_doc[i] < 0 || hit_doc[i] >= num_docs) throw std::out_of_range("hit doc");
    by_doc[hit_doc[i]].emplace_back(hit_matcher[i], hit_line[i]);
  }
  std::vector<std::vector<int>> primary_of(num_matchers);
  for (size_t p = 0; p < P; ++p) {
    if (pat_primary[p] < 0 || pat_primary[p] >= num_matchers) throw std::out_of_range("pattern primary");
    primary_of[pat_primary[p]].push_back(static_cast<int>(p));
  }
  py::list result;
  for (int64_t d = 0; d < num_docs; ++d) {
    auto& v = by_doc[d];
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    struct Ev { double score; int sev; int64_t line; int pat; };
    std::vector<Ev> evs;
    auto nearest = [&](int64_t m, int64_t line) -> int64_t {
      auto lo = std::lower_bound(v.begin(), v.end(), std::make_pair(m, line));
      int64_t best = -1;
      if (lo != v.end() && lo->first == m) best = lo->second - line;
      if (lo != v.begin()) {
        auto pr = std::prev(lo);
        if (pr->first == m) {
          const int64_t dd = line - pr->second;
          if (best < 0 || dd < best) best = dd;
        }
      }
      return best;
    };
    for (const auto& h : v) {
      if (h.first >= num_matchers) continue;
      for (int p : primary_of[h.first]) {
        double bonus = 0.0, wsum = 0.0;
        for (size_t j = 0; j < pat_sec[p].size(); ++j) {
          const double w = pat_w[p][j];
          wsum += w;
          const int64_t dist = nearest(pat_sec[p][j], h.second);
          if (dist >= 0 && dist <= pat_win[p][j]) bonus += w * (1.0 - double(dist) / double(pat_win[p][j] + 1));
        }
        const double score = pat_conf[p] * (1.0 + bonus) / (1.0 + wsum);
        evs.push_back({score, static_cast<int>(pat_sev[p]), h.second, p});
      }
    }
    std::sort(evs.begin(), evs.end(), [](const Ev& a, const Ev& b) {
      if (a.score != b.score) return a.score > b.score;
      if (a.sev != b.sev) return a.sev > b.sev;
      if (a.line != b.line) return a.line < b.line;
      return a.pat < b.pat;
    });
    py::list dl;
    for (const auto& e : evs) dl.append(py::make_tuple(e.pat, e.line, e.score));
    result.append(dl);
  }
  return result;
}

}  // namespace

void register_verify(py::module_& m);   // verify.cpp (N3 / N4)

PYBIND11_MODULE(_patterns, m) {
  m.doc() = "operator_amd host pattern compiler / packer / scorer";
  m.def("compile_dfa", &compile_dfa, py::arg("factors"));
  m.def("dfa_chain", &dfa_chain, py::arg("table"), py::arg("log2_classes"), py::arg("num_states"));
  m.def("reorder_dfa", &reorder_dfa, py::arg("table"), py::arg("out_off"), py::arg("out_ids"), py::arg("log2_classes"),
        py::arg("num_states"), py::arg("cls_map"), py::arg("sample"), py::arg("hot"));
  m.def("plan_docs", &plan_docs, py::arg("lens"), py::arg("seg_bytes"));
  m.def("pack_docs", &pack_docs, py::arg("docs"), py::arg("first_seg"), py::arg("seg_bytes"), py::arg("dst"),
        py::arg("threads") = 8);
  m.def("score_events", &score_events);
  m.attr("MAX_FACTOR_LEN") = kMaxFactorLen;
  m.attr("MAX_STATES") = kMaxStates;
  register_verify(m);
}
