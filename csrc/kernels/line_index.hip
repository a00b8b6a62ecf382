// Line index and context windows of the pattern scan (replaces the
// log-parser's line splitting behind J/service/LogParserRestClient.java:37-39):
//
//  * line_prefix: exclusive prefix of the per-segment newline counts ac_scan produced
//    (single-pass decoupled look-back scan; tiles of 4096 counts, dynamic tile ids so a
//    tile only ever waits on tiles that are already running). Each tile publishes ONE
//    8-byte granule {status:2 | value:62} with an agent-scope relaxed atomic store and
//    looks back with agent-scope relaxed atomic loads (the data is the flag: no fences,
//    cdna_hip_programming.md §6 Guideline 16 R2); the granules and the tile counter are
//    zeroed by a memset in the launcher before every launch (replay-safe).
//  * doc_lines: newlines per document from that prefix (AnalysisResult totalLines).
//  * context_spans: the +-k line window of each reported event, located on the GPU in the
//    text the scan left resident: one wave per query walks 64 bytes per step with a
//    newline ballot, back to the k-th previous line start and on to the k-th following
//    line end; the host slices [window start, window end) and splits it into lines.
//    Same windows as verify.cpp `contexts` (lines before while the window start > 0,
//    lines after while the window end + 1 < the document's length).
#include "common.h"
#include "scan.h"

namespace oamd {

namespace {

constexpr int kLpThreads = 256;
constexpr int kLpItems = 16;                       // counts per thread
constexpr int kLpTile = kLpThreads * kLpItems;     // 4096 counts per tile
constexpr uint64_t kAgg = 1ull << 62, kPre = 2ull << 62, kValMask = (1ull << 62) - 1;
constexpr uint32_t kSpinMax = 1u << 24;

__device__ __forceinline__ uint64_t ld_granule(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st_granule(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

// state: [0] = tile counter (low 32 bits), [1] = error word (non-zero: a look-back gave up
// and this launch's prefix is wrong -- the host reruns the batch on the CPU path),
// [2 .. 2 + tiles) = tile granules
__global__ void __launch_bounds__(kLpThreads) line_prefix_kernel(const uint32_t* __restrict__ cnt, int64_t n,
                                                                 int64_t* __restrict__ excl,
                                                                 uint64_t* __restrict__ state) {
  __shared__ int64_t wsum[kLpThreads / 64];
  __shared__ int64_t tile_base;
  __shared__ uint32_t tile_id;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) tile_id = atomicAdd(reinterpret_cast<uint32_t*>(state), 1u);
  __syncthreads();
  const int64_t t = tile_id;
  uint64_t* gran = state + 2;
  const int64_t i0 = t * kLpTile + (int64_t)tid * kLpItems;
  uint32_t v[kLpItems];
#pragma unroll
  for (int j = 0; j < kLpItems; ++j) v[j] = (i0 + j < n) ? cnt[i0 + j] : 0u;
  int64_t mine = 0;
#pragma unroll
  for (int j = 0; j < kLpItems; ++j) mine += v[j];
  // block exclusive scan of the per-thread sums
  int64_t incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  int64_t before_wave = 0, agg = 0;
#pragma unroll
  for (int k = 0; k < kLpThreads / 64; ++k) {
    if (k < wid) before_wave += wsum[k];
    agg += wsum[k];
  }
  // publish the aggregate, then (wave 0) look back until a published inclusive prefix
  if (wid == 0) {
    int64_t base = 0;
    if (t == 0) {
      if (lane == 0) st_granule(gran, kPre | (uint64_t)agg);
    } else {
      if (lane == 0) st_granule(gran + t, kAgg | (uint64_t)agg);
      int64_t j = t - 1;
      uint32_t spins = 0;
      while (j >= 0) {
        const uint64_t g = ld_granule(gran + j);   // every lane reads the same word
        const uint64_t st = g & ~kValMask;
        if (st == 0) {
          if (++spins > kSpinMax) {   // bounded: a stalled predecessor cannot hang the GPU;
            if (lane == 0) st_granule(state + 1, 1ull);   // flag the launch, never a silent prefix
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        base += (int64_t)(g & kValMask);
        if (st == kPre) break;
        --j;
      }
      if (lane == 0) st_granule(gran + t, kPre | (uint64_t)(base + agg));
    }
    if (lane == 0) tile_base = base;
  }
  __syncthreads();
  int64_t run = tile_base + before_wave + incl - mine;
#pragma unroll
  for (int j = 0; j < kLpItems; ++j) {
    if (i0 + j < n) excl[i0 + j] = run;
    run += v[j];
  }
  if (i0 + kLpItems >= n && i0 < n) excl[n] = run;   // the thread holding the last count: total
}

__global__ void doc_lines_kernel(const int64_t* __restrict__ excl, const int64_t* __restrict__ first, int ndocs,
                                 int64_t* __restrict__ doc_nl) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d < ndocs) doc_nl[d] = excl[first[d + 1]] - excl[first[d]];
}

namespace {

// largest i in [lo, p) with t[i] == '\n', else lo - 1 (whole wave, uniform result)
__device__ __forceinline__ int64_t prev_nl(const uint8_t* __restrict__ t, int64_t lo, int64_t p, int lane) {
  while (p > lo) {
    const int64_t b = p - 64;
    const int64_t i = b + lane;
    const bool nl = i >= lo && t[i] == '\n';
    const uint64_t m = __ballot(nl);
    if (m) return b + 63 - __clzll(m);
    p = b;
  }
  return lo - 1;
}

// smallest i in [p, hi) with t[i] == '\n', else hi
__device__ __forceinline__ int64_t next_nl(const uint8_t* __restrict__ t, int64_t p, int64_t hi, int lane) {
  while (p < hi) {
    const int64_t i = p + lane;
    const bool nl = i < hi && t[i] == '\n';
    const uint64_t m = __ballot(nl);
    if (m) return p + __ffsll((long long)m) - 1;
    p += 64;
  }
  return hi;
}

}  // namespace

// q: [nq, 3] (doc, byte offset, k); out: [nq, 4] doc-relative (window start, window end,
// line start, line end)
__global__ void __launch_bounds__(256) context_spans_kernel(const uint8_t* __restrict__ text,
                                                            const int64_t* __restrict__ doc_base,
                                                            const int64_t* __restrict__ doc_len,
                                                            const int64_t* __restrict__ q, int nq,
                                                            int64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int qi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qi >= nq) return;
  const int64_t d = q[3 * qi], k = max((int64_t)0, q[3 * qi + 2]);
  const int64_t base = doc_base[d], len = doc_len[d];
  const uint8_t* td = text + base;
  const int64_t off = min(max((int64_t)0, q[3 * qi + 1]), len);
  const int64_t s = prev_nl(td, 0, off, lane) + 1;
  const int64_t e = off < len ? next_nl(td, off, len, lane) : len;
  int64_t ws = s;
  for (int64_t j = 0; j < k && ws > 0; ++j) ws = prev_nl(td, 0, ws - 1, lane) + 1;
  int64_t we = e;
  for (int64_t j = 0; j < k; ++j) {
    if (we >= len || we + 1 >= len) break;
    we = next_nl(td, we + 1, len, lane);
  }
  if (lane == 0) {
    out[4 * qi] = ws;
    out[4 * qi + 1] = we;
    out[4 * qi + 2] = s;
    out[4 * qi + 3] = e;
  }
}

int64_t line_prefix_state_words(int64_t n) { return 2 + (n + kLpTile - 1) / kLpTile; }

int line_prefix(const uint32_t* cnt, int64_t n, int64_t* excl, uint64_t* state, hipStream_t stream) {
  if (n < 1) return -1;
  const int64_t tiles = (n + kLpTile - 1) / kLpTile;
  if (tiles >= (1ll << 31)) return -2;
  // zero the counter + granules (a multiple of 16 B from the allocation's start)
  const int64_t words = (line_prefix_state_words(n) + 1) & ~1ll;
  const hipError_t e = hipMemsetAsync(state, 0, words * 8, stream);
  if (e != hipSuccess) return (int)e;
  line_prefix_kernel<<<(unsigned)tiles, kLpThreads, 0, stream>>>(cnt, n, excl, state);
  OAMD_LAUNCH_CHECK();
  return 0;
}

int doc_lines(const int64_t* excl, const int64_t* first, int ndocs, int64_t* doc_nl, hipStream_t stream) {
  if (ndocs < 1) return 0;
  doc_lines_kernel<<<(ndocs + 255) / 256, 256, 0, stream>>>(excl, first, ndocs, doc_nl);
  OAMD_LAUNCH_CHECK();
  return 0;
}

int context_spans(const uint8_t* text, const int64_t* doc_base, const int64_t* doc_len, const int64_t* q, int nq,
                  int64_t* out, hipStream_t stream) {
  if (nq < 1) return 0;
  context_spans_kernel<<<(nq + 3) / 4, 256, 0, stream>>>(text, doc_base, doc_len, q, nq, out);
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
