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

static int scan_v1_requested();
constexpr int kHotWideStates = 256;  // ac_scan v2 hot set (full byte rows in LDS)

// hot-state capacity of the scan kernel in use (v2 by default; OAMD_SCAN=v1)
int max_hot_states(int log2_classes) {
  return scan_v1_requested() ? kHotTableBytes / (2 << log2_classes) : kHotWideStates;
}

struct ScanStream {
  uint32_t s;     // DFA state
  uint32_t nl;    // newlines seen in the own range so far
  int64_t base;   // byte offset of the segment start
  uint32_t seg;   // segment index
  bool active;
};

// Append the output patterns of `state` for every lane with `emit` set: one atomicAdd on
// the global counter per wave and round (ballot + popcount; the leader lane adds the
// round's total, each lane's slot is its rank among the wave's emitting lanes), not one
// per match -- a pattern that hits every line of a noisy log would otherwise serialise
// its whole wave on the counter. Rounds = the largest output set among the wave's lanes
// (usually 1). Correct under a partial EXEC mask: only active lanes take part.
__device__ __forceinline__ void emit_matches_wave(bool emit, uint32_t state, uint32_t seg, uint32_t off, uint32_t nl,
                                                  const uint32_t* __restrict__ out_off,
                                                  const uint32_t* __restrict__ out_ids,
                                                  MatchRec* __restrict__ matches, uint32_t* __restrict__ count,
                                                  uint32_t cap) {
  uint32_t k = 0, e = 0;
  if (emit) {
    k = out_off[state];
    e = out_off[state + 1];
  }
  const int lane = threadIdx.x & 63;
  for (;; ++k) {
    const bool has = k < e;
    const uint64_t m = __ballot(has);
    if (m == 0) break;
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, static_cast<uint32_t>(__popcll(m)));
    base = __shfl(base, leader, 64);
    if (has) {
      const uint32_t idx = base + static_cast<uint32_t>(__popcll(m & ((1ull << lane) - 1ull)));
      if (idx < cap) {
        MatchRec r;
        r.x = seg; r.y = out_ids[k]; r.z = off; r.w = nl;
        matches[idx] = r;
      }
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
              if (__ballot((ea & 0x8000u) != 0))
                emit_matches_wave((ea & 0x8000u) != 0, st[0].s, st[0].seg, off, st[0].nl, out_off, out_ids, matches,
                                  count, cap);
              if (__ballot((eb & 0x8000u) != 0))
                emit_matches_wave((eb & 0x8000u) != 0, st[1].s, st[1].seg, off, st[1].nl, out_off, out_ids, matches,
                                  count, cap);
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

// ---------------------------------------------------------------------------
// ac_scan v2 ("wide"): the default kernel (OAMD_SCAN=v1 selects the one above).
//
// v1 runs at 1.16 TB/s on 1.19 GB x 1000 patterns, and not because of the
// DFA: hipcc merges `s < H ? tl[i] : tg[i]` into ONE flat_load_ushort through a
// selected LDS-or-global address, so every byte step of every wave waits
// vmcnt(0) on a flat load. v2 (2.32 TB/s on the same input):
//   * hot states (the 256 most-visited after MatchEngine's profile-guided
//     renumbering: >= 99.9 % of visits on log text) are staged in LDS as FULL byte
//     rows, so a byte step is one ds_read_u16 and no class-map read. Layout
//     [byte][state], row stride 258 entries: the bank of (byte b, state s) is
//     (b + s/2) mod 32, so lanes sitting in the same state spread by byte value.
//     The image is built once on the host (MatchEngine.hot_table) and copied in
//     with 16-B loads;
//   * two passes per 64-byte chunk. The fast walk is branch-free: the state
//     register holds the raw table entry (next | 0x8000 "has outputs"), its low
//     byte indexes the hot row, and every entry is OR-ed into an accumulator. A
//     chunk that started in or entered a cold state (>= 256: from there on the
//     fast steps were wrong) or reached an output state is re-walked exactly from
//     its saved start state (class map + global table, match emission) behind one
//     wave-uniform branch per chunk: 3.7 % of wave-chunks on the synthetic corpus;
//   * newlines are counted per 4-byte word (SWAR zero-byte test + popcount);
//   * the text is cut into grid x 1024 equal streams (whole 64-byte chunks,
//     >= seg_bytes) instead of fixed segments, so every lane does the same work and
//     only a stream start replays the 64-byte look-back; a chunk is four
//     consecutive 16-B loads, so each 128-B line is requested in two bursts;
//   * per-segment newline counts are atomically accumulated (a segment is split
//     between at most two streams, since streams are >= seg_bytes long); the
//     stream that ends inside a segment also stores its part as seg_head[g], and
//     matches found after such a split carry bit 31 in .w so scan_fixup adds it.
// Measured alternatives (same input): 2 streams x 32-B chunks 2.02 TB/s; 2 x 64 B
// and 1 x 128 B need > 128 VGPRs with the exact path inlined and spill; a
// per-byte ballot branch for cold/output states instead of the two passes 1.95.
constexpr int kHotWide = kScanHotStates;
constexpr int kWideStride = kScanHotStride;
static_assert(kHotWideStates == kScanHotStates, "hot set sizes");
constexpr int kWideLds = 256 + kHotWide * kWideStride * 2;
constexpr int kScanLdsMax = 160 * 1024;
constexpr int kChainLdsMax = (kScanLdsMax - kWideLds) / 16 * 16;   // chain bytes staged in LDS

// 0x80 in each byte of w that is '\n' (exact: no carries between bytes)
__device__ __forceinline__ uint32_t newline_bits(uint32_t w) {
  const uint32_t x = w ^ 0x0a0a0a0au;
  return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
}

// PROBE (timing probes, OAMD_SCAN_PROBE; results are NOT valid): 1 = every lookup on a
// lane-private LDS bank (conflict-free, same dependent chain), 2 = real lookups without
// the exact re-walk, 3 = a VALU-only chain (no LDS); 4 = the real kernel with per-wave
// slow-path statistics, 5 = 4 + second-half-of-line text loads nontemporal, 6 = 4 +
// the slow path at raised wave priority (s_setprio), 7 = 4 + the re-walk block entered
// after every chunk (its non-walk code kept hot), 8 = two streams of 32-byte chunks per
// lane, 9 = the real kernel with the slow path at raised wave priority.
template <int NS, int CH, int NT = kScanThreads, int PROBE = 0>
__global__ void __launch_bounds__(NT) ac_scan_wide_kernel(
    const uint8_t* __restrict__ text, int64_t total, int64_t L, int64_t n_streams, int seg_shift,
    const uint8_t* __restrict__ cls_map, const uint16_t* __restrict__ tg, const uint16_t* __restrict__ hot_table,
    int log2C, int H, const uint32_t* __restrict__ out_off, const uint32_t* __restrict__ out_ids,
    MatchRec* __restrict__ matches, uint32_t* __restrict__ count, uint32_t cap, uint32_t* __restrict__ seg_nl,
    uint32_t* __restrict__ seg_head, const uint8_t* __restrict__ chain, uint32_t n_chain_lds) {
  constexpr int NV = CH / 16;  // 16-B loads per stream per chunk
  constexpr bool STATS = PROBE >= 4 && PROBE <= 7;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* cls = smem;
  uint16_t* tl = reinterpret_cast<uint16_t*>(smem + 256);
  const int tid = threadIdx.x;
  // class map + the host-built [byte][state] hot table + the first n_chain_lds chain
  // bytes: plain 16-B copies
  uint8_t* lchain = smem + 256 + kHotWide * kWideStride * 2;
  if (tid < 16) reinterpret_cast<uint4*>(cls)[tid] = reinterpret_cast<const uint4*>(cls_map)[tid];
  for (int i = tid; i < kHotWide * kWideStride * 2 / 16; i += NT)
    reinterpret_cast<uint4*>(tl)[i] = reinterpret_cast<const uint4*>(hot_table)[i];
  for (int i = tid; i < static_cast<int>(n_chain_lds / 16); i += NT)
    reinterpret_cast<uint4*>(lchain)[i] = reinterpret_cast<const uint4*>(chain)[i];
  __syncthreads();

  const int64_t k0 = NS * ((int64_t)blockIdx.x * NT + tid);
  if (k0 >= n_streams) return;  // no barrier follows
  const uint32_t seg_mask = (1u << seg_shift) - 1;
  const uint32_t cold_mask = (H >= kHotWide) ? 0x7f00u : 0xffffu;  // H < 256 only for tiny DFAs
  const uint32_t Hs = static_cast<uint32_t>(H);

  int64_t pos[NS], end[NS];
  uint32_t st[NS], nl[NS], mid = 0, act = 0;
  uint64_t t_begin = 0, t_slow = 0, t_sub = 0;   // STATS (PROBE 4-7): per-wave slow-path statistics
  uint32_t n_slow = 0, n_cold = 0, n_emit = 0, n_sub = 0, t_emit = 0, t_cold = 0;
  if constexpr (STATS) t_begin = clock64();
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int64_t b0 = (k0 + k) * L;
    pos[k] = b0;
    end[k] = b0 + L < total ? b0 + L : total;
    act |= ((k0 + k) < n_streams && b0 < total) ? (1u << k) : 0u;
    mid |= ((static_cast<uint64_t>(b0) & seg_mask) != 0) ? (1u << k) : 0u;
    st[k] = 0;
    nl[k] = 0;
  }

  typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
  // a chunk per stream as consecutive 16-B loads (plain, not nontemporal: the other
  // half of each 128-B line is read by the next chunk, from L2; nt loads measured
  // 1.6x slower)
  auto load = [&](u32x4_t (&dst)[NS][NV], int64_t delta, bool nt = false) {
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int64_t o = pos[k] + delta;
      if (o >= 0 && o < end[k] && (act >> k & 1u)) {
        const u32x4_t* p = reinterpret_cast<const u32x4_t*>(text + o);
        if (nt) {
#pragma unroll
          for (int v = 0; v < NV; ++v) dst[k][v] = __builtin_nontemporal_load(p + v);
        } else {
#pragma unroll
          for (int v = 0; v < NV; ++v) dst[k][v] = p[v];
        }
      } else {
#pragma unroll
        for (int v = 0; v < NV; ++v) dst[k][v] = u32x4_t{0u, 0u, 0u, 0u};
      }
    }
  };

  // Exact walk of one 16-byte sub-chunk `q` of stream k from state s (cold states
  // through the chain bytes / the global table) with match emission when `own`: the
  // rare path, and issue-bound (it shares its SIMD with three fast-walking waves), so
  // every byte costs few instructions: a byte step is its LDS read and one
  // wave-uniform cold test; output entries are collected per dword and emitted behind
  // one test per dword; newlines are counted per dword. Rolled over the 4 dwords
  // (picked by a 2-level select), unrolled over their bytes.
  auto slow_sub = [&](int k, const u32x4_t& q, int64_t at, uint32_t s, uint32_t nl_now, bool own) -> uint32_t {
#pragma unroll 1
    for (int d = 0; d < 4; ++d) {
      const uint32_t w01 = (d & 1) ? q[1] : q[0];
      const uint32_t w23 = (d & 1) ? q[3] : q[2];
      const uint32_t wv = (d & 2) ? w23 : w01;
      uint32_t es[4], omask = 0;
#pragma unroll
      for (int by = 0; by < 4; ++by) {
        const uint32_t b = (wv >> (8 * by)) & 0xffu;
        const uint32_t sk = s & 0x7fffu;
        uint32_t e = tl[b * kWideStride + (sk & 0xffu)];
        if (__ballot(sk >= Hs)) {
          uint64_t tc = 0;
          if constexpr (STATS) tc = clock64();
          // A cold state is usually one step down a pattern literal's trie path, numbered
          // so that the path's next state is sk + 1 (csrc/patterns/patterns.cpp
          // reorder_dfa): the chain byte (LDS, the rest of the CU's 160 KB) says which
          // class takes it there. Other transitions read the global table, as half of a
          // 32-bit read: a uint16 load here is merged with the LDS read above into one
          // flat_load through a selected address, and then EVERY byte of the re-walk
          // waits on a flat load (vmcnt + lgkmcnt).
          if (sk >= Hs) {
            const uint32_t c = cls[b];
            const uint32_t x = sk < n_chain_lds
                                   ? static_cast<uint32_t>(lchain[sk])
                                   : (reinterpret_cast<const uint32_t*>(chain)[sk >> 2] >> ((sk & 3u) * 8)) & 0xffu;
            if ((x & 0x40u) && (x & 0x3fu) == c) {
              e = (sk + 1) | ((x & 0x80u) << 8);
            } else {
              const uint32_t gi = (sk << log2C) | c;
              e = (reinterpret_cast<const uint32_t*>(tg)[gi >> 1] >> ((gi & 1u) << 4)) & 0xffffu;
            }
          }
          if constexpr (STATS) {   // per lane: cold steps and their cycles
            if (sk >= Hs) {
              ++n_cold;
              t_cold += static_cast<uint32_t>(clock64() - tc) + (e & 0u);
            }
          }
        }
        es[by] = e;
        omask |= ((e >> 15) & 1u) << by;
        s = e;
      }
      const uint32_t nlb = newline_bits(wv);
      if (__ballot(own && omask != 0)) {
        uint64_t te = 0;
        if constexpr (STATS) te = clock64();
#pragma unroll 1
        for (int by = 0; by < 4; ++by) {
          const bool hit = own && (omask >> by & 1u);
          if (__ballot(hit)) {
            const uint32_t e01 = (by & 1) ? es[1] : es[0];
            const uint32_t e23 = (by & 1) ? es[3] : es[2];
            const uint32_t e = (by & 2) ? e23 : e01;
            const uint64_t p = static_cast<uint64_t>(at + 4 * d + by);
            const uint32_t nl_at = nl_now + __builtin_popcount(nlb & ((1u << (8 * by)) - 1u));
            emit_matches_wave(hit, e & 0x7fffu, static_cast<uint32_t>(p >> seg_shift),
                              static_cast<uint32_t>(p) & seg_mask, nl_at | ((mid >> k & 1u) << 31), out_off,
                              out_ids, matches, count, cap);
          }
        }
        if constexpr (STATS) {   // per lane (the emitting lanes)
          if (own && omask != 0) {
            t_emit += static_cast<uint32_t>(clock64() - te);
            n_emit += __builtin_popcount(omask);
          }
        }
      }
      if (own) nl_now += __builtin_popcount(nlb);
    }
    return s;
  };

  // One chunk of every stream, the common case: one ds_read_u16 per byte and no
  // branch. The state register holds the raw entry (next | 0x8000 outputs), its low
  // byte indexes the hot row; `acc` ORs every entry of a 16-byte sub-chunk, so one test
  // per sub-chunk finds one that entered a cold state (>= 256: every later fast step
  // was wrong) or an output state (bit v of fl[k]). The chunk is then re-walked exactly
  // from its first flagged sub-chunk, one sub-chunk at a time, until the exact state
  // meets the fast walk's state at a sub-chunk boundary again (from there the fast walk
  // was exact; later flagged sub-chunks are re-walked from their saved start state).
  // Bit k of `own`: stream k's own range (count newlines, emit) rather than its look-back.
  auto walk = [&](const u32x4_t (&cur)[NS][NV], uint32_t own, int64_t delta) {
    uint32_t sv[NS][NV], nl0[NS], acc[NS], fl[NS], m[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      sv[k][0] = st[k];
      nl0[k] = nl[k];
      acc[k] = st[k] & 0x7fffu;   // a chunk that STARTS in a cold state is re-walked too
      fl[k] = 0;
      m[k] = (own >> k & 1u) ? (cold_mask | 0x8000u) : cold_mask;
    }
#pragma unroll
    for (int w = 0; w < CH / 4; ++w) {
      uint32_t wv[NS];
#pragma unroll
      for (int k = 0; k < NS; ++k) wv[k] = cur[k][w >> 2][w & 3];
#pragma unroll
      for (int by = 0; by < 4; ++by) {
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          const uint32_t b = (wv[k] >> (8 * by)) & 0xffu;
          if constexpr (PROBE == 1)
            st[k] = tl[((((b ^ st[k]) & 0x7fu) << 5) | (threadIdx.x & 31u)) << 1];
          else if constexpr (PROBE == 3)
            st[k] = ((st[k] * 0x9e37u) ^ b) & 0xffffu;
          else
            st[k] = tl[b * kWideStride + (st[k] & 0xffu)];
          acc[k] |= st[k];
        }
      }
#pragma unroll
      for (int k = 0; k < NS; ++k)
        if (own >> k & 1u) nl[k] += __builtin_popcount(newline_bits(wv[k]));
      if ((w & 3) == 3) {   // sub-chunk boundary
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          fl[k] |= (acc[k] & m[k]) ? (1u << (w >> 2)) : 0u;
          acc[k] = st[k] & 0x7fffu;   // the next sub-chunk is re-walked if it starts cold
          if ((w >> 2) + 1 < NV) sv[k][(w >> 2) + 1] = st[k];
        }
      }
      // keep the scheduler from hoisting the state-independent byte-offset math of
      // the whole chunk ahead of the chain (64 live VGPRs per stream, then spills)
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (PROBE >= 1 && PROBE <= 3) {
#pragma unroll
      for (int k = 0; k < NS; ++k)
        if (fl[k] == 0xfff0u + static_cast<uint32_t>(log2C) || sv[k][NV - 1] == 0xfff0u + static_cast<uint32_t>(log2C))
          seg_head[0] = st[k];   // keep the walk live
      return;
    }
    uint32_t any = PROBE == 7 ? 1u : 0u;
#pragma unroll
    for (int k = 0; k < NS; ++k) any |= fl[k];
    if (__ballot(any != 0)) {
      uint64_t t0 = 0;
      if constexpr (STATS) t0 = clock64();
      if constexpr (PROBE == 6 || PROBE == 9) __builtin_amdgcn_s_setprio(3);
#pragma unroll   // compile-time k and v: a runtime index would put st[]/sv[] in scratch
      for (int k = 0; k < NS; ++k) {
        if (PROBE != 7 && !__ballot(fl[k] != 0)) continue;
        const bool ownk = own >> k & 1u;
        bool sync = true;          // the fast walk's state at this sub-chunk's start is exact
        uint32_t s = 0, nlr = nl0[k];
#pragma unroll   // compile-time v: selecting cur[k][v] / sv[k][v] at run time puts them in scratch
        for (int v = 0; v < NV; ++v) {
          const u32x4_t& q = cur[k][v];
          const uint32_t sa = sv[k][v], sb = v + 1 < NV ? sv[k][v + 1 < NV ? v + 1 : v] : st[k];
          const bool need = fl[k] != 0 && (!sync || (fl[k] >> v & 1u));
          if (__ballot(need)) {
            uint64_t tw = 0;
            if constexpr (STATS) {
              ++n_sub;
              tw = clock64();
            }
            if (need) {
              s = slow_sub(k, q, pos[k] + delta + 16 * v, sync ? sa : s, nlr, ownk);
              sync = s == sb;
            }
            if constexpr (STATS) t_sub += __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(clock64() - tw));
          }
          if (ownk) {
#pragma unroll
            for (int d = 0; d < 4; ++d) nlr += __builtin_popcount(newline_bits(q[d]));
          }
        }
        if (!sync) st[k] = s;
      }
      if constexpr (PROBE == 6 || PROBE == 9) __builtin_amdgcn_s_setprio(0);
      if constexpr (STATS) {
        t_slow += clock64() - t0;
        ++n_slow;
      }
    }
  };

  u32x4_t cur[NS][NV], nxt[NS][NV];
  // look-back: the LB >= 64 bytes (the longest pattern) before each stream start,
  // walked from the root without emitting
  constexpr int LB = CH > 64 ? CH : 64;
#pragma unroll
  for (int lb = LB; lb > 0; lb -= CH) {
    load(cur, -lb);
    walk(cur, 0u, -lb);
  }
  load(cur, 0);
  const int64_t chunks = (L + CH - 1) / CH;
  for (int64_t c = 0; c < chunks; ++c) {
    // PROBE 5: the chunk that reads the second half of each 128-B line (L % 128 == 0)
    // loads it nontemporally: last use, so it is not kept in L2 over the DFA table
    if (c + 1 < chunks) load(nxt, CH, PROBE == 5 && (c & 1) == 0);
    uint32_t own = 0;
#pragma unroll
    for (int k = 0; k < NS; ++k) own |= ((act >> k & 1u) && pos[k] < end[k]) ? (1u << k) : 0u;
    walk(cur, own, 0);
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      // segment part complete: at a segment boundary or at the stream end (CH <= seg_bytes
      // and L % CH == 0, so a chunk ends at or before the next boundary)
      pos[k] += CH;
      if ((own >> k & 1u) && (((static_cast<uint64_t>(pos[k]) & seg_mask) == 0) || pos[k] >= end[k])) {
        const uint32_t g = static_cast<uint32_t>(static_cast<uint64_t>(pos[k] - 1) >> seg_shift);
        atomicAdd(seg_nl + g, nl[k]);
        if ((static_cast<uint64_t>(pos[k]) & seg_mask) != 0) seg_head[g] = nl[k];  // ends mid-segment
        nl[k] = 0;
        mid &= ~(1u << k);
      }
    }
    if (c + 1 < chunks) {
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int v = 0; v < NV; ++v) cur[k][v] = nxt[k][v];
    }
  }
  if constexpr (STATS) {
    // per-wave {cycles, slow-path cycles, slow-path entries, cold wave-steps, emission
    // cycles, emissions, re-walked sub-chunks, sub-chunk walk cycles, cold-step cycles, 0, 0, 0}
    // in the
    // upper half of the match buffer (timing probe only)
    // per-lane counters -> wave totals (counts) / the busiest lane (cycles)
    for (int o = 32; o > 0; o >>= 1) {
      n_cold += __shfl_xor(n_cold, o, 64);
      n_emit += __shfl_xor(n_emit, o, 64);
      t_cold = max(t_cold, (uint32_t)__shfl_xor(t_cold, o, 64));
      t_emit = max(t_emit, (uint32_t)__shfl_xor(t_emit, o, 64));
    }
    if ((tid & 63) == 0) {
      uint32_t* stats = reinterpret_cast<uint32_t*>(matches + cap / 2) +
                        12 * ((int64_t)blockIdx.x * (NT / 64) + (tid >> 6));
      stats[0] = static_cast<uint32_t>(clock64() - t_begin);
      stats[1] = static_cast<uint32_t>(t_slow);
      stats[2] = n_slow;
      stats[3] = n_cold;
      stats[4] = static_cast<uint32_t>(t_emit);
      stats[5] = n_emit;
      stats[6] = n_sub;
      stats[7] = static_cast<uint32_t>(t_sub);
      stats[8] = t_cold;
      stats[9] = 0;
      stats[10] = 0;
      stats[11] = 0;
    }
  }
}

static int scan_v1_requested() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("OAMD_SCAN");
    v = (e && e[0] == 'v' && e[1] == '1') ? 1 : 0;
  }
  return v;
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

int ac_scan(const uint8_t* text, int64_t n_segs, int seg_bytes, const uint8_t* cls_map, const uint16_t* table,
            int num_states, int log2_classes, int hot_states, const uint32_t* out_off, const uint32_t* out_ids,
            MatchRec* matches, uint32_t* match_count, uint32_t match_cap, uint32_t* seg_nl, int grid_blocks,
            const uint16_t* hot_table, const uint8_t* chain, hipStream_t stream) {
  if (n_segs == 0) return 0;
  if (!scan_v1_requested()) {
    if (hot_table == nullptr || chain == nullptr) return -8;
    if (seg_bytes < 64 || (seg_bytes & (seg_bytes - 1)) != 0) return -1;
    if (log2_classes < 3 || log2_classes > 8) return -2;
    if (num_states > 32768) return -3;
    int H = hot_states < num_states ? hot_states : num_states;
    if (H > kHotWide) H = kHotWide;
    if (H < 1) H = 1;
    // one stream of 64-byte chunks per lane (measured on MI355X, 1.19 GB x 1000 patterns:
    // 2.32 TB/s; 2 streams x 32 B 2.02, 1 x 128 B and 2 x 64 B spill registers)
    constexpr int NSv = 1, CHv = 64;
    const int threads = kScanThreads;
    static const int probe = [] {
      const char* e = getenv("OAMD_SCAN_PROBE");
      return e ? atoi(e) : 0;
    }();
    const void* fn = probe == 1   ? reinterpret_cast<const void*>(ac_scan_wide_kernel<NSv, CHv, kScanThreads, 1>)
                     : probe == 2 ? reinterpret_cast<const void*>(ac_scan_wide_kernel<NSv, CHv, kScanThreads, 2>)
                     : probe == 3 ? reinterpret_cast<const void*>(ac_scan_wide_kernel<NSv, CHv, kScanThreads, 3>)
                     : probe == 4 ? reinterpret_cast<const void*>(ac_scan_wide_kernel<NSv, CHv, kScanThreads, 4>)
                     : probe == 5 ? reinterpret_cast<const void*>(ac_scan_wide_kernel<NSv, CHv, kScanThreads, 5>)
                     : probe == 6 ? reinterpret_cast<const void*>(ac_scan_wide_kernel<NSv, CHv, kScanThreads, 6>)
                     : probe == 7 ? reinterpret_cast<const void*>(ac_scan_wide_kernel<NSv, CHv, kScanThreads, 7>)
                     : probe == 8 ? reinterpret_cast<const void*>(ac_scan_wide_kernel<2, 32>)
                     : probe == 9 ? reinterpret_cast<const void*>(ac_scan_wide_kernel<NSv, CHv, kScanThreads, 9>)
                                  : reinterpret_cast<const void*>(ac_scan_wide_kernel<NSv, CHv>);
    const int NSr = probe == 8 ? 2 : NSv, CHr = probe == 8 ? 32 : CHv;
    static bool attr_set = false;
    if (!attr_set) {
      if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kScanLdsMax) != hipSuccess) return -6;
      attr_set = true;
    }
    // the chain bytes of the first n_chain states in LDS (the rest from global memory)
    const int64_t n_chain_all = ((int64_t)num_states + 15) / 16 * 16;
    const uint32_t n_chain = static_cast<uint32_t>(n_chain_all < kChainLdsMax ? n_chain_all : kChainLdsMax);
    const int lds_bytes = kWideLds + static_cast<int>(n_chain);
    const int64_t total = n_segs * (int64_t)seg_bytes;
    const int64_t streams = (int64_t)(grid_blocks > 0 ? grid_blocks : num_cus()) * threads * NSr;
    int64_t L = (total + streams - 1) / streams;
    const int64_t Lq = probe == 5 ? 2 * CHr : CHr;
    L = ((L + Lq - 1) / Lq) * Lq;   // whole chunks (CH = 64 <= seg_bytes)
    if (L < seg_bytes) L = seg_bytes;
    const int64_t n_streams = (total + L - 1) / L;
    const int64_t per_block = (int64_t)threads * NSr;
    const int64_t blocks = (n_streams + per_block - 1) / per_block;
    int shift = 0;
    while ((1 << shift) < seg_bytes) ++shift;
    // seg_nl holds [n_segs] totals (atomically accumulated) then [n_segs] split-segment heads
    if (hipMemsetAsync(seg_nl, 0, sizeof(uint32_t) * 2 * n_segs, stream) != hipSuccess) return -5;
    uint32_t* seg_head = seg_nl + n_segs;
    const uint8_t* txt = text;
    const uint16_t* tgp = table;
    int l2c = log2_classes;
    void* args[] = {&txt, (void*)&total, &L, (void*)&n_streams, &shift, (void*)&cls_map, &tgp, (void*)&hot_table,
                    &l2c, &H,
                    (void*)&out_off, (void*)&out_ids, &matches, &match_count, &match_cap, &seg_nl, &seg_head,
                    (void*)&chain, (void*)&n_chain};
    if (hipLaunchKernel(fn, dim3(static_cast<unsigned>(blocks)), dim3(threads), args, lds_bytes, stream) !=
        hipSuccess)
      return -7;
    OAMD_LAUNCH_CHECK();
    return 0;
  }
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
                                  int num_docs, int seg_bytes, const uint32_t* __restrict__ seg_head) {
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
    // bit 31 of .w (ac_scan v2): the match's stream started inside segment g; the
    // newlines of the segment's head part (the previous stream's) come first
    const uint32_t head = (r.w & 0x80000000u) ? seg_head[g] : 0u;
    const int64_t line = nl_excl[g] - nl_excl[fs] + (r.w & 0x7fffffffu) + head;
    const int64_t off = (g - fs) * seg_bytes + r.z;
    r.x = static_cast<uint32_t>(lo);
    r.z = static_cast<uint32_t>(line);
    r.w = static_cast<uint32_t>(off);
    m[i] = r;
  }
}

int scan_fixup(MatchRec* matches, const uint32_t* match_count, uint32_t match_cap, const int64_t* seg_nl_excl,
               const int64_t* doc_first_seg, int num_docs, int seg_bytes, const uint32_t* seg_head,
               hipStream_t stream) {
  if (num_docs == 0 || match_cap == 0) return 0;
  scan_fixup_kernel<<<256, 256, 0, stream>>>(matches, match_count, match_cap, seg_nl_excl, doc_first_seg, num_docs,
                                            seg_bytes, seg_head);
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
