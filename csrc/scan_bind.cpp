// Bindings for the log-scan kernels (operator_amd._C.ac_scan / scan_fixup).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "kernels/scan.h"

namespace {

#define CHECK_T(t, dt) TORCH_CHECK((t).is_cuda() && (t).is_contiguous() && (t).scalar_type() == (dt), #t " must be a contiguous GPU tensor of ", dt)

void ac_scan(const at::Tensor& text, int64_t seg_bytes, const at::Tensor& cls_map, const at::Tensor& table,
             int64_t log2_classes, int64_t hot_states, const at::Tensor& out_off, const at::Tensor& out_ids,
             at::Tensor& matches, at::Tensor& match_count, at::Tensor& seg_nl, int64_t grid_blocks,
             const at::Tensor& hot_table, const at::Tensor& chain) {
  CHECK_T(text, at::kByte);
  CHECK_T(cls_map, at::kByte);
  CHECK_T(table, at::kShort);
  CHECK_T(out_off, at::kInt);
  CHECK_T(out_ids, at::kInt);
  CHECK_T(matches, at::kInt);
  CHECK_T(match_count, at::kInt);
  CHECK_T(seg_nl, at::kInt);
  CHECK_T(hot_table, at::kShort);
  CHECK_T(chain, at::kByte);
  TORCH_CHECK(hot_table.numel() == oamd::kScanHotStates * oamd::kScanHotStride,
              "hot_table must be [256 bytes x 258] (MatchEngine builds it)");
  TORCH_CHECK(seg_bytes >= 64 && (seg_bytes & (seg_bytes - 1)) == 0, "seg_bytes must be a power of two >= 64");
  TORCH_CHECK(text.numel() % seg_bytes == 0, "text must be padded to a multiple of seg_bytes");
  TORCH_CHECK(cls_map.numel() == 256, "class map must have 256 entries");
  const int64_t C = int64_t(1) << log2_classes;
  TORCH_CHECK(table.dim() == 2 && table.size(1) == C, "table must be [states, 2^log2_classes]");
  const int64_t S = table.size(0);
  TORCH_CHECK(S >= 1 && S <= 32768, "DFA must have 1..32768 states");
  TORCH_CHECK(chain.numel() >= (S + 15) / 16 * 16 + 16, "chain must have round_up(states, 16) + 16 bytes (dfa_chain)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(chain.data_ptr()) % 16 == 0, "chain must be 16-byte aligned");
  TORCH_CHECK(out_off.numel() == S + 1, "out_off must have states+1 entries");
  TORCH_CHECK(hot_states >= 1 && hot_states <= S && hot_states <= oamd::max_hot_states((int)log2_classes),
              "hot_states out of range");
  TORCH_CHECK(((hot_states * C) % 8) == 0, "hot table must be a multiple of 16 bytes");
  TORCH_CHECK(matches.dim() == 2 && matches.size(1) == 4, "matches must be [cap, 4] int32");
  TORCH_CHECK(match_count.numel() >= 1, "match_count needs one element");
  const int64_t n_segs = text.numel() / seg_bytes;
  TORCH_CHECK(seg_nl.numel() >= 2 * n_segs, "seg_nl needs 2 x segments entries (totals, split heads)");
  TORCH_CHECK(n_segs < (int64_t(1) << 32), "too many segments");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(text.device());
  const int rc = oamd::ac_scan(text.data_ptr<uint8_t>(), n_segs, (int)seg_bytes, cls_map.data_ptr<uint8_t>(),
                               reinterpret_cast<const uint16_t*>(table.data_ptr()), (int)S, (int)log2_classes,
                               (int)hot_states, reinterpret_cast<const uint32_t*>(out_off.data_ptr()),
                               reinterpret_cast<const uint32_t*>(out_ids.data_ptr()),
                               reinterpret_cast<oamd::MatchRec*>(matches.data_ptr()),
                               reinterpret_cast<uint32_t*>(match_count.data_ptr()), (uint32_t)matches.size(0),
                               reinterpret_cast<uint32_t*>(seg_nl.data_ptr()), (int)grid_blocks,
                               reinterpret_cast<const uint16_t*>(hot_table.data_ptr()), chain.data_ptr<uint8_t>(),
                               c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  TORCH_CHECK(rc == 0, "ac_scan launch failed rc=", rc);
}

void scan_fixup(at::Tensor& matches, const at::Tensor& match_count, const at::Tensor& seg_nl_excl,
                const at::Tensor& doc_first_seg, int64_t seg_bytes, const at::Tensor& seg_head) {
  CHECK_T(matches, at::kInt);
  CHECK_T(match_count, at::kInt);
  CHECK_T(seg_nl_excl, at::kLong);
  CHECK_T(doc_first_seg, at::kLong);
  TORCH_CHECK(matches.dim() == 2 && matches.size(1) == 4, "matches must be [cap, 4]");
  TORCH_CHECK(doc_first_seg.numel() >= 2, "doc_first_seg must have num_docs+1 >= 2 entries");
  CHECK_T(seg_head, at::kInt);
  TORCH_CHECK(seg_head.numel() >= seg_nl_excl.numel(), "seg_head needs one entry per segment");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(matches.device());
  const int rc = oamd::scan_fixup(reinterpret_cast<oamd::MatchRec*>(matches.data_ptr()),
                                  reinterpret_cast<const uint32_t*>(match_count.data_ptr()), (uint32_t)matches.size(0),
                                  seg_nl_excl.data_ptr<int64_t>(), doc_first_seg.data_ptr<int64_t>(),
                                  (int)doc_first_seg.numel() - 1, (int)seg_bytes,
                                  reinterpret_cast<const uint32_t*>(seg_head.data_ptr()), c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  TORCH_CHECK(rc == 0, "scan_fixup launch failed rc=", rc);
}

void line_prefix(const at::Tensor& cnt, at::Tensor& excl, at::Tensor& state) {
  CHECK_T(cnt, at::kInt);
  CHECK_T(excl, at::kLong);
  CHECK_T(state, at::kLong);
  const int64_t n = cnt.numel();
  TORCH_CHECK(n >= 1 && excl.numel() >= n + 1, "line_prefix: excl needs n + 1 entries");
  TORCH_CHECK(state.numel() >= ((oamd::line_prefix_state_words(n) + 1) & ~1ll), "line_prefix: state too small");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(cnt.device());
  const int rc = oamd::line_prefix(reinterpret_cast<const uint32_t*>(cnt.data_ptr()), n, excl.data_ptr<int64_t>(),
                                   reinterpret_cast<uint64_t*>(state.data_ptr()),
                                   c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  TORCH_CHECK(rc == 0, "line_prefix launch failed rc=", rc);
}

void doc_lines(const at::Tensor& excl, const at::Tensor& first, at::Tensor& doc_nl) {
  CHECK_T(excl, at::kLong);
  CHECK_T(first, at::kLong);
  CHECK_T(doc_nl, at::kLong);
  const int64_t nd = first.numel() - 1;
  TORCH_CHECK(nd >= 1 && doc_nl.numel() >= nd, "doc_lines: doc_nl needs one entry per doc");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(excl.device());
  const int rc = oamd::doc_lines(excl.data_ptr<int64_t>(), first.data_ptr<int64_t>(), (int)nd,
                                 doc_nl.data_ptr<int64_t>(), c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  TORCH_CHECK(rc == 0, "doc_lines launch failed rc=", rc);
}

void context_spans(const at::Tensor& text, const at::Tensor& doc_base, const at::Tensor& doc_len,
                   const at::Tensor& q, at::Tensor& out) {
  CHECK_T(text, at::kByte);
  CHECK_T(doc_base, at::kLong);
  CHECK_T(doc_len, at::kLong);
  CHECK_T(q, at::kLong);
  CHECK_T(out, at::kLong);
  TORCH_CHECK(q.dim() == 2 && q.size(1) == 3 && out.dim() == 2 && out.size(1) == 4 && out.size(0) >= q.size(0),
              "context_spans: q [n, 3], out [n, 4]");
  TORCH_CHECK(doc_base.numel() == doc_len.numel(), "context_spans: doc_base / doc_len");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(text.device());
  const int rc = oamd::context_spans(text.data_ptr<uint8_t>(), doc_base.data_ptr<int64_t>(),
                                     doc_len.data_ptr<int64_t>(), q.data_ptr<int64_t>(), (int)q.size(0),
                                     out.data_ptr<int64_t>(), c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  TORCH_CHECK(rc == 0, "context_spans launch failed rc=", rc);
}

}  // namespace

void register_scan_bindings(pybind11::module_& m) {
  m.def("line_prefix", &line_prefix);
  m.def("doc_lines", &doc_lines);
  m.def("context_spans", &context_spans);
  m.def("line_prefix_state_words", [](int64_t n) { return (oamd::line_prefix_state_words(n) + 1) & ~1ll; });
  m.def("ac_scan", &ac_scan);
  m.def("scan_fixup", &scan_fixup);
  m.def("max_hot_states", [](int64_t log2c) { return oamd::max_hot_states((int)log2c); });
  m.attr("SCAN_HOT_STRIDE") = oamd::kScanHotStride;
}
