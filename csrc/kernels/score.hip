// Pattern-event scoring on the GPU (SURVEY.md §2.4 N5 "score_reduce").
//
// Input: verified matcher hits sorted by (doc, matcher, line), unique, with a
// CSR doc index; the pattern table as CSR arrays. Two kernels:
//   * score_events_kernel — one thread per (primary hit, pattern using that
//     matcher as primary): the proximity bonus of every secondary matcher is the
//     nearest hit of that matcher in the same doc (binary search over the doc's
//     sorted (matcher, line) keys), weighted by 1 - dist / (window + 1):
//       score = conf * (1 + sum_j w_j * prox_j) / (1 + sum_j w_j)
//     (the same formula, in fp64, as patterns/oracle.py and the host scorer);
//   * rank_events_kernel — one workgroup per doc: bitonic sort of the doc's
//     events in LDS by (score desc, severity desc, line asc, pattern asc), plus
//     the summary reductions (highest severity, significant count).
// The reference delegates all of this to its external log-parser
// (J/service/LogParserClient.java:36-55); the algorithm is our design.
#include "common.h"
#include "kernels.h"

namespace oamd {

__device__ __forceinline__ int64_t hit_key(int64_t matcher, int64_t line) { return (matcher << 32) | line; }

// keys[] = (matcher << 32 | line) of one doc, ascending. Nearest |line - l| of matcher m, or -1.
__device__ int64_t nearest_line(const int64_t* keys, int n, int64_t m, int64_t line) {
  int lo = 0, hi = n;  // first key >= (m, line)
  const int64_t k = hit_key(m, line);
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (keys[mid] < k) lo = mid + 1; else hi = mid;
  }
  int64_t best = -1;
  if (lo < n && (keys[lo] >> 32) == m) best = (keys[lo] & 0xffffffffLL) - line;
  if (lo > 0 && (keys[lo - 1] >> 32) == m) {
    const int64_t d = line - (keys[lo - 1] & 0xffffffffLL);
    if (best < 0 || d < best) best = d;
  }
  return best;
}

__global__ void score_events_kernel(const int64_t* __restrict__ keys, const int* __restrict__ hit_doc,
                                    const int* __restrict__ doc_ptr, int n_hits,
                                    const int* __restrict__ prim_ptr, const int* __restrict__ prim_pat,
                                    const int* __restrict__ ev_ptr,  // exclusive scan of patterns per hit
                                    const int* __restrict__ sec_ptr, const int* __restrict__ sec_matcher,
                                    const double* __restrict__ sec_w, const int* __restrict__ sec_win,
                                    const double* __restrict__ conf, int num_matchers,
                                    double* __restrict__ ev_score, int* __restrict__ ev_pat, int* __restrict__ ev_line) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= n_hits) return;
  const int64_t m = keys[h] >> 32, line = keys[h] & 0xffffffffLL;
  if (m >= num_matchers) return;
  const int d = hit_doc[h];
  const int64_t* dk = keys + doc_ptr[d];
  const int dn = doc_ptr[d + 1] - doc_ptr[d];
  int out = ev_ptr[h];
  for (int i = prim_ptr[m]; i < prim_ptr[m + 1]; ++i, ++out) {
    const int p = prim_pat[i];
    double bonus = 0.0, wsum = 0.0;
    for (int j = sec_ptr[p]; j < sec_ptr[p + 1]; ++j) {
      const double w = sec_w[j];
      wsum += w;
      const int64_t dist = nearest_line(dk, dn, sec_matcher[j], line);
      if (dist >= 0 && dist <= sec_win[j]) bonus += w * (1.0 - double(dist) / double(sec_win[j] + 1));
    }
    ev_score[out] = conf[p] * (1.0 + bonus) / (1.0 + wsum);
    ev_pat[out] = p;
    ev_line[out] = static_cast<int>(line);
  }
}

// One workgroup (256 threads) per doc; events of doc d are [ev_doc_ptr[d], ev_doc_ptr[d+1]).
// Writes the permutation `order` (global event indices, ranked) and summary[d] =
// (highest severity rank or -1, significant events, total events).
constexpr int kRankCap = 2048;  // events per doc sorted in LDS (the host ranks larger docs)

__global__ void __launch_bounds__(256) rank_events_kernel(const int* __restrict__ ev_doc_ptr,
                                                          const double* __restrict__ ev_score,
                                                          const int* __restrict__ ev_pat,
                                                          const int* __restrict__ ev_line,
                                                          const int* __restrict__ severity, double significance,
                                                          int* __restrict__ order, int* __restrict__ summary) {
  __shared__ double s_score[kRankCap];
  __shared__ int s_idx[kRankCap];
  __shared__ int red_sev[4], red_sig[4];
  const int d = blockIdx.x, tid = threadIdx.x;
  const int base = ev_doc_ptr[d], n = ev_doc_ptr[d + 1] - base;
  int sev = -1, sig = 0;
  for (int i = tid; i < n; i += 256) {
    sev = max(sev, severity[ev_pat[base + i]]);
    sig += ev_score[base + i] >= significance ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) {
    sev = max(sev, __shfl_xor(sev, o, kWave));
    sig += __shfl_xor(sig, o, kWave);
  }
  if ((tid & 63) == 0) { red_sev[tid >> 6] = sev; red_sig[tid >> 6] = sig; }
  __syncthreads();
  if (tid == 0) {
    summary[3 * d] = max(max(red_sev[0], red_sev[1]), max(red_sev[2], red_sev[3]));
    summary[3 * d + 1] = red_sig[0] + red_sig[1] + red_sig[2] + red_sig[3];
    summary[3 * d + 2] = n;
  }
  if (n > kRankCap) return;  // ranked on the host
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (int i = tid; i < np2; i += 256) {
    s_idx[i] = i < n ? base + i : -1;
    s_score[i] = i < n ? ev_score[base + i] : 0.0;
  }
  __syncthreads();
  // "a before b" = higher score, then higher severity, lower line, lower pattern; padding last
  auto before = [&](int ia, double sa, int ib, double sb) -> bool {
    if (ia < 0) return false;
    if (ib < 0) return true;
    if (sa != sb) return sa > sb;
    const int va = severity[ev_pat[ia]], vb = severity[ev_pat[ib]];
    if (va != vb) return va > vb;
    if (ev_line[ia] != ev_line[ib]) return ev_line[ia] < ev_line[ib];
    return ev_pat[ia] < ev_pat[ib];
  };
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < np2; i += 256) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;  // ascending-in-"before" order for this run
          const bool swap = up ? before(s_idx[l], s_score[l], s_idx[i], s_score[i])
                               : before(s_idx[i], s_score[i], s_idx[l], s_score[l]);
          if (swap) {
            const int ti = s_idx[i]; s_idx[i] = s_idx[l]; s_idx[l] = ti;
            const double ts = s_score[i]; s_score[i] = s_score[l]; s_score[l] = ts;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < n; i += 256) order[base + i] = s_idx[i];
}

int score_events(const int64_t* keys, const int* hit_doc, const int* doc_ptr, int n_hits, int n_docs,
                 const int* prim_ptr, const int* prim_pat, const int* ev_ptr, const int* ev_doc_ptr,
                 const int* sec_ptr, const int* sec_matcher, const double* sec_w, const int* sec_win,
                 const double* conf, const int* severity, int num_matchers, double significance, double* ev_score,
                 int* ev_pat, int* ev_line, int* order, int* summary, hipStream_t stream) {
  if (n_docs == 0) return 0;
  if (n_hits > 0) {
    score_events_kernel<<<(n_hits + 255) / 256, 256, 0, stream>>>(keys, hit_doc, doc_ptr, n_hits, prim_ptr, prim_pat,
                                                                 ev_ptr, sec_ptr, sec_matcher, sec_w, sec_win, conf,
                                                                 num_matchers, ev_score, ev_pat, ev_line);
    OAMD_LAUNCH_CHECK();
  }
  rank_events_kernel<<<n_docs, 256, 0, stream>>>(ev_doc_ptr, ev_score, ev_pat, ev_line, severity, significance,
                                                 order, summary);
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
