// Launchers for the multi-pattern log scan.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace oamd {

// Match record written by ac_scan (16 B):
//   x = segment index, y = factor id, z = end byte offset inside the segment,
//   w = newlines seen in the segment before the match (v2: since the stream's start
//       when bit 31 is set, i.e. the stream began inside this segment).
// scan_fixup rewrites records in place as:
//   x = doc index, y = factor id, z = 0-based line in doc, w = end byte offset in doc.
struct MatchRec {
  uint32_t x, y, z, w;
};

int ac_scan(const uint8_t* text, int64_t n_segs, int seg_bytes, const uint8_t* cls_map,
            const uint16_t* table, int num_states, int log2_classes, int hot_states,
            const uint32_t* out_off, const uint32_t* out_ids, MatchRec* matches, uint32_t* match_count,
            uint32_t match_cap, uint32_t* seg_nl, int grid_blocks, const uint16_t* hot_table,
            const uint8_t* chain, hipStream_t stream);

// ac_scan v2's LDS image of the first min(num_states, 256) states: entry
// [byte * kScanHotStride + state] = table[state][cls_map[byte]] (built on the host).
constexpr int kScanHotStates = 256;
constexpr int kScanHotStride = kScanHotStates + 2;
// chain: per-state chain bytes of the exact re-walk (patterns.cpp dfa_chain), at least
// round_up(num_states, 16) + 16 bytes.

// seg_head: per-segment newline count of the part scanned by the stream that ends
// inside the segment (ac_scan v2; the second half of its seg_nl buffer).
int scan_fixup(MatchRec* matches, const uint32_t* match_count, uint32_t match_cap,
               const int64_t* seg_nl_excl, const int64_t* doc_first_seg, int num_docs, int seg_bytes,
               const uint32_t* seg_head, hipStream_t stream);

int max_hot_states(int log2_classes);

// line_index.hip (N3): exclusive prefix excl[0..n] (excl[n] = total) of the per-segment
// newline counts (decoupled look-back; `state` holds line_prefix_state_words(n) uint64,
// zeroed by the launcher), newlines per document, and the +-k context windows of reported
// events located in the resident text (q [nq, 3] = doc, offset, k; out [nq, 4] = window
// start, window end, line start, line end, document-relative).
int64_t line_prefix_state_words(int64_t n);
int line_prefix(const uint32_t* cnt, int64_t n, int64_t* excl, uint64_t* state, hipStream_t stream);
int doc_lines(const int64_t* excl, const int64_t* first, int ndocs, int64_t* doc_nl, hipStream_t stream);
int context_spans(const uint8_t* text, const int64_t* doc_base, const int64_t* doc_len, const int64_t* q, int nq,
                  int64_t* out, hipStream_t stream);

}  // namespace oamd
