// Multi-pattern log scan: Aho-Corasick DFA walk over a batch of pod logs
// (SURVEY.md §2.4 N2 ac_scan + N3 line index), replacing the reference's
// external log-parser service (J/service/LogParserRestClient.java:37-39).
//
// Data layout (built by the host packer, csrc/patterns/patterns.cpp):
//   * docs are concatenated, each padded with >= 1 NUL byte up to a multiple
//     of `seg_bytes`. NUL is in no pattern, so it sends the DFA to the root:
//     no match can straddle two docs, and the kernel needs no doc table.
//   * the text is cut into segments of seg_bytes (power of two, >= 64); one
//     lane owns two segments ("streams") and walks them interleaved so two
//     independent dependent-load chains are in flight per lane.
//   * every stream first replays the 64 bytes before its segment (patterns
//     are <= 64 bytes) without emitting, so matches that straddle a segment
//     seam are found exactly once: by the segment in which they END.
// DFA layout (csrc/patterns/patterns.cpp): uint16 next-state table
// [states][classes], entry = next | 0x8000 if next has outputs; states are
// numbered breadth-first so the shallow states that a log stays in most of
// the time come first, and the first `hot_states` rows (<= 128 KiB) are
// staged in LDS. Bytes are mapped to (case-folded) classes via a 256-entry
// LDS map. Deep states fall back to the global table (L2 / Infinity Cache).
// One 1024-thread workgroup per CU (16 waves) keeps ~2k dependent chains in
// flight per CU; the walk is LDS-latency bound, text loads are 4 x 16 B per
// lane per 64-byte chunk, double-buffered one chunk ahead.
#include "common.h"
#include "scan.h"

namespace oamd {

constexpr int kScanThreads = 1024;
constexpr int kHotTableBytes = 128 * 1024;

int max_hot_states(int log2_classes) { return kHotTableBytes / (2 << log2_classes); }

struct ScanStream {
  uint32_t s;     // DFA state
  uint32_t nl;    // newlines seen in the own range so far
  int64_t base;   // byte offset of the segment start
  uint32_t seg;   // segment index
  bool active;
};

__device__ __forceinline__ void emit_matches(uint32_t state, uint32_t seg, uint32_t off, uint32_t nl,
                                             const uint32_t* __restrict__ out_off,
                                             const uint32_t* __restrict__ out_ids, MatchRec* __restrict__ matches,
                                             uint32_t* __restrict__ count, uint32_t cap) {
  const uint32_t b = out_off[state], e = out_off[state + 1];
  for (uint32_t k = b; k < e; ++k) {
    const uint32_t idx = atomicAdd(count, 1u);
    if (idx < cap) {
      MatchRec r;
      r.x = seg; r.y = out_ids[k]; r.z = off; r.w = nl;
      matches[idx] = r;
    }
  }
}

__global__ void __launch_bounds__(kScanThreads) ac_scan_kernel(
    const uint8_t* __restrict__ text, int64_t n_segs, int seg_bytes, const uint8_t* __restrict__ cls_map,
    const uint16_t* __restrict__ tg, int log2C, int hot_states, const uint32_t* __restrict__ out_off,
    const uint32_t* __restrict__ out_ids, MatchRec* __restrict__ matches, uint32_t* __restrict__ count,
    uint32_t cap, uint32_t* __restrict__ seg_nl) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* cls = smem;
  uint16_t* tl = reinterpret_cast<uint16_t*>(smem + 256);
  const int tid = threadIdx.x;
  if (tid < 16) reinterpret_cast<uint4*>(cls)[tid] = reinterpret_cast<const uint4*>(cls_map)[tid];
  const int hot_vec = (hot_states << log2C) >> 3;  // 16-B vectors
  for (int i = tid; i < hot_vec; i += kScanThreads)
    reinterpret_cast<uint4*>(tl)[i] = reinterpret_cast<const uint4*>(tg)[i];
  __syncthreads();

  const uint32_t H = static_cast<uint32_t>(hot_states);
  const int64_t n_pairs = (n_segs + 1) >> 1;
  const int chunks = seg_bytes >> 6;

  for (int64_t pi = (int64_t)blockIdx.x * kScanThreads + tid; pi < n_pairs;
       pi += (int64_t)gridDim.x * kScanThreads) {
    ScanStream st[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int64_t g = 2 * pi + k;
      st[k].active = g < n_segs;
      st[k].seg = static_cast<uint32_t>(g);
      st[k].base = g * (int64_t)seg_bytes;
      st[k].s = 0;
      st[k].nl = 0;
    }
    // chunk -1 is the 64-byte look-back (zeros for segment 0 / inactive streams)
    uint4 cur[2][4], nxt[2][4];
    auto load_chunk = [&](uint4 (&dst)[2][4], int c) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int64_t off = st[k].base + (int64_t)c * 64;
        if (st[k].active && off >= 0) {
          const uint4* p = reinterpret_cast<const uint4*>(text + off);
#pragma unroll
          for (int j = 0; j < 4; ++j) dst[k][j] = p[j];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) dst[k][j] = make_uint4(0, 0, 0, 0);
        }
      }
    };
    load_chunk(cur, -1);
    for (int c = -1; c < chunks; ++c) {
      if (c + 1 < chunks) load_chunk(nxt, c + 1);
      const bool own = c >= 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int wd = 0; wd < 4; ++wd) {
          const uint32_t wa = (wd == 0) ? cur[0][j].x : (wd == 1) ? cur[0][j].y : (wd == 2) ? cur[0][j].z : cur[0][j].w;
          const uint32_t wb = (wd == 0) ? cur[1][j].x : (wd == 1) ? cur[1][j].y : (wd == 2) ? cur[1][j].z : cur[1][j].w;
#pragma unroll
          for (int by = 0; by < 4; ++by) {
            const uint32_t ba = (wa >> (8 * by)) & 0xffu;
            const uint32_t bb = (wb >> (8 * by)) & 0xffu;
            const uint32_t ia = (st[0].s << log2C) | cls[ba];
            const uint32_t ib = (st[1].s << log2C) | cls[bb];
            const uint32_t ea = st[0].s < H ? tl[ia] : tg[ia];
            const uint32_t eb = st[1].s < H ? tl[ib] : tg[ib];
            st[0].s = ea & 0x7fffu;
            st[1].s = eb & 0x7fffu;
            if (own) {
              const uint32_t off = static_cast<uint32_t>(c * 64 + j * 16 + wd * 4 + by);
              if (ea & 0x8000u) emit_matches(st[0].s, st[0].seg, off, st[0].nl, out_off, out_ids, matches, count, cap);
              if (eb & 0x8000u) emit_matches(st[1].s, st[1].seg, off, st[1].nl, out_off, out_ids, matches, count, cap);
              st[0].nl += (ba == 10u);
              st[1].nl += (bb == 10u);
            }
          }
        }
      }
      if (c + 1 < chunks) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int j = 0; j < 4; ++j) cur[k][j] = nxt[k][j];
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (st[k].active) seg_nl[st[k].seg] = st[k].nl;
  }
}

int ac_scan(const uint8_t* text, int64_t n_segs, int seg_bytes, const uint8_t* cls_map, const uint16_t* table,
            int num_states, int log2_classes, int hot_states, const uint32_t* out_off, const uint32_t* out_ids,
            MatchRec* matches, uint32_t* match_count, uint32_t match_cap, uint32_t* seg_nl, int grid_blocks,
            hipStream_t stream) {
  if (n_segs == 0) return 0;
  if (seg_bytes < 64 || (seg_bytes & (seg_bytes - 1)) != 0) return -1;
  if (log2_classes < 3 || log2_classes > 8) return -2;
  if (num_states > 32768) return -3;
  if (hot_states > num_states) hot_states = num_states;
  if (hot_states > max_hot_states(log2_classes)) return -4;
  const size_t lds = 256 + (static_cast<size_t>(hot_states) << log2_classes) * 2;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(ac_scan_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        256 + kHotTableBytes);
    attr_set = true;
  }
  const int64_t pairs = (n_segs + 1) / 2;
  int64_t blocks = (pairs + kScanThreads - 1) / kScanThreads;
  if (grid_blocks > 0 && blocks > grid_blocks) blocks = grid_blocks;
  ac_scan_kernel<<<static_cast<int>(blocks), kScanThreads, lds, stream>>>(
      text, n_segs, seg_bytes, cls_map, table, log2_classes, hot_states, out_off, out_ids, matches, match_count,
      match_cap, seg_nl);
  OAMD_LAUNCH_CHECK();
  return 0;
}

// Rewrite segment-relative match records into (doc, factor, line, offset-in-doc).
// seg_nl_excl = exclusive prefix sum of per-segment newline counts (int64),
// doc_first_seg[num_docs + 1] = first segment of each doc (last = total).
__global__ void scan_fixup_kernel(MatchRec* __restrict__ m, const uint32_t* __restrict__ count, uint32_t cap,
                                  const int64_t* __restrict__ nl_excl, const int64_t* __restrict__ doc_first_seg,
                                  int num_docs, int seg_bytes) {
  const uint32_t n = min(*count, cap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    MatchRec r = m[i];
    const int64_t g = r.x;
    int lo = 0, hi = num_docs;  // find last doc with first_seg <= g
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (doc_first_seg[mid] <= g) lo = mid; else hi = mid;
    }
    const int64_t fs = doc_first_seg[lo];
    const int64_t line = nl_excl[g] - nl_excl[fs] + r.w;
    const int64_t off = (g - fs) * seg_bytes + r.z;
    r.x = static_cast<uint32_t>(lo);
    r.z = static_cast<uint32_t>(line);
    r.w = static_cast<uint32_t>(off);
    m[i] = r;
  }
}

int scan_fixup(MatchRec* matches, const uint32_t* match_count, uint32_t match_cap, const int64_t* seg_nl_excl,
               const int64_t* doc_first_seg, int num_docs, int seg_bytes, hipStream_t stream) {
  if (num_docs == 0 || match_cap == 0) return 0;
  scan_fixup_kernel<<<256, 256, 0, stream>>>(matches, match_count, match_cap, seg_nl_excl, doc_first_seg, num_docs,
                                            seg_bytes);
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
