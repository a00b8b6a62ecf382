// Launchers for the multi-pattern log scan.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace oamd {

// Match record written by ac_scan (16 B):
//   x = segment index, y = factor id, z = end byte offset inside the segment,
//   w = newlines seen in the segment before the match.
// scan_fixup rewrites records in place as:
//   x = doc index, y = factor id, z = 0-based line in doc, w = end byte offset in doc.
struct MatchRec {
  uint32_t x, y, z, w;
};

int ac_scan(const uint8_t* text, int64_t n_segs, int seg_bytes, const uint8_t* cls_map,
            const uint16_t* table, int num_states, int log2_classes, int hot_states,
            const uint32_t* out_off, const uint32_t* out_ids, MatchRec* matches, uint32_t* match_count,
            uint32_t match_cap, uint32_t* seg_nl, int grid_blocks, hipStream_t stream);

int scan_fixup(MatchRec* matches, const uint32_t* match_count, uint32_t match_cap,
               const int64_t* seg_nl_excl, const int64_t* doc_first_seg, int num_docs, int seg_bytes,
               hipStream_t stream);

int max_hot_states(int log2_classes);

}  // namespace oamd
