// Paged decode attention, split-KV ("flash-decoding"), GQA.
//
// One query token per sequence. Workgroup = (split of 256 cached tokens,
// kv-head, sequence); the G = Hq/Hkv query heads sharing the kv-head are
// processed together so every K/V row is read from HBM exactly once.
// This op is HBM-bound (B x ctx x Hkv x 512 B per layer), so the structure is
// built around bytes in flight, not arithmetic:
//   * every lane issues ALL of its K loads (16 x 16 B) and V loads (16 x 16 B)
//     at kernel entry — 64 KiB of K+V per workgroup in flight — and the
//     QK^T, softmax and PV work then runs under that traffic;
//   * S = K Q^T runs on MFMA (v_mfma_f32_16x16x32_bf16, K tile = A operand,
//     the G query heads zero-padded to 16 columns = B operand), so no
//     cross-lane reduction is needed for the dot products;
//   * softmax is two-pass over the split (max, then exp2/sum) in LDS — no
//     online rescaling; PV runs on the VALU (16 B V rows per lane, P read as
//     one ds_read_b128 per token for G = 4) and reduces over the 4 token
//     sub-slots with 2 xor-shuffles.
// Fragment maps (cdna_hip_programming.md §3): A lane l -> A[l&15][8(l>>4)+j];
// B lane l -> B[8(l>>4)+j][l&15]; C col = l&15, row = 4(l>>4)+r. The dims of a
// k-step are permuted so lane group g covers dims 32g..32g+31 over the 4
// k-steps (Q uses the same permutation, so the contraction is unchanged).
// KV cache layout: [pages, Hkv, page_size, D] bf16.
#include "common.h"
#include "kernels.h"

namespace oamd {

constexpr int kSplit = 256;  // tokens per split == threads per block

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ u16x8 ld16(const bf16_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(p));
}

// Work list: one item per (sequence, 256-token split) that actually holds tokens,
// built on the device from seq_lens so a captured graph needs no host data.
// Empty workgroups are expensive (measured ~22 ns each: at B = 256 a grid sized
// for the model's max context spent more time dispatching empty splits than
// attending), so live items are packed first and the grid is sized by the
// caller's per-call bound.
// work[0] = total items, work[1 + i] = (b << 8) | split, i < total.
__global__ void attn_decode_plan_kernel(const int* __restrict__ seq_lens, int B, int max_tokens, int num_splits,
                                        int* __restrict__ work) {
  __shared__ int pre[1025];
  const int tid = threadIdx.x;
  int total = 0;
  for (int base = 0; base < B; base += 1024) {
    const int b = base + tid;
    int ns = 0;
    if (b < B) {
      const int len = min(seq_lens[b], max_tokens);
      ns = min((len + kSplit - 1) / kSplit, num_splits);
    }
    pre[tid + 1] = ns;
    if (tid == 0) pre[0] = 0;
    __syncthreads();
    if (tid == 0)
      for (int i = 1; i <= 1024; ++i) pre[i] += pre[i - 1];
    __syncthreads();
    if (b < B)
      for (int s = 0; s < ns; ++s) work[1 + total + pre[tid] + s] = (b << 8) | s;
    total += pre[1024];
    __syncthreads();
  }
  if (tid == 0) work[0] = total;
}

template <int G>
__device__ __forceinline__ void attn_decode_item(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int* __restrict__ block_tables, const int* __restrict__ seq_lens,
    bf16_t* __restrict__ out, float* __restrict__ o_part, float* __restrict__ ml_part, int Hkv,
    int page_size, int log2_page, int max_pages, int num_splits, float scale_log2, int b, int s, int kvh) {
  constexpr int D = 128;
  constexpr int GP = (G < 4) ? 4 : G;  // score row stride (float4-aligned)
  __shared__ __attribute__((aligned(16))) float sc[kSplit * GP];   // [token][head]
  __shared__ __attribute__((aligned(16))) float red[4 * G * D];
  __shared__ float wred[4][G];

  __shared__ int pg_lds[kSplit / 16 + 2];

  const int Hq = Hkv * G;
  const int len = min(seq_lens[b], max_pages * page_size);  // never index past the block table
  const int start = s * kSplit;
  const int n = min(len - start, kSplit);  // >= 1: the plan only lists non-empty splits
  const int ns_b = (len + kSplit - 1) / kSplit;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l15 = lane & 15, lg = lane >> 4;
  // Stage this split's page ids in LDS. The data loads below then depend only on
  // LDS (lgkmcnt), so hipcc can issue all of them back to back; a per-token
  // global block-table load would share vmcnt with the data loads and force a
  // vmcnt(0) before every one of them.
  const int page0 = start >> log2_page;
  const int npg = min(((start + n - 1) >> log2_page) - page0 + 1, kSplit / 16 + 2);
  if (tid < npg) pg_lds[tid] = block_tables[(int64_t)b * max_pages + page0 + tid];
  __syncthreads();
  auto row_off = [&](int t) -> int64_t {  // t already clamped to [0, n)
    const int tok = start + t;
    const int64_t page = pg_lds[(tok >> log2_page) - page0];
    return ((page * Hkv + kvh) * page_size + (tok & (page_size - 1))) * (int64_t)D;
  };

  // ---- q first (the first MFMA needs it), as the B operand: column = head ----
  u16x8 qb[4];
  {
    const int hq = kvh * G + (l15 < G ? l15 : 0);
    const bf16_t* qp = q + ((int64_t)b * Hq + hq) * D + 32 * lg;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qb[ks] = *reinterpret_cast<const u16x8*>(qp + 8 * ks);
  }
  // ---- then every K and V load of this lane, branch-free (rows past n are clamped
  // duplicates; their scores are masked to -inf and their P to 0) ----
  u16x8 kf[4][4];  // [tile][kstep]: token w*64 + 16*i + l15, dims 32*lg + 8*ks
  u16x8 vf[16];    // token w*64 + 4*it + lg, dims 8*l15
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bf16_t* p = kc + row_off(min(w * 64 + 16 * i + l15, n - 1)) + 32 * lg;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) kf[i][ks] = ld16(p + 8 * ks);
  }
#pragma unroll
  for (int it = 0; it < 16; ++it) vf[it] = ld16(vc + row_off(min(w * 64 + 4 * it + lg, n - 1)) + 8 * l15);
  if (l15 >= G) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qb[ks] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }

  // ---- S = K Q^T on MFMA, scaled scores -> LDS [token][head] ----
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, kf[i][ks]),
                                                    __builtin_bit_cast(bf16x8_t, qb[ks]), acc, 0, 0, 0);
    if (l15 < G) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = w * 64 + 16 * i + 4 * lg + r;
        sc[t * GP + l15] = (t < n) ? acc[r] * scale_log2 : -INFINITY;
      }
    }
  }
  __syncthreads();

  // ---- two-pass softmax over the split: thread tid <-> token tid ----
  float mh[G], lh[G];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const float m = wave_max(sc[tid * GP + h]);
    if (lane == 0) wred[w][h] = m;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < G; ++h) mh[h] = fmaxf(fmaxf(wred[0][h], wred[1][h]), fmaxf(wred[2][h], wred[3][h]));
  __syncthreads();
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const float sv = sc[tid * GP + h];
    const float p = (tid < n) ? exp2f(sv - mh[h]) : 0.f;
    sc[tid * GP + h] = p;
    const float ls = wave_sum(p);
    if (lane == 0) wred[w][h] = ls;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < G; ++h) lh[h] = wred[0][h] + wred[1][h] + wred[2][h] + wred[3][h];

  // ---- O = P V on the VALU (V already in registers) ----
  float acc[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[h][j] = 0.f;
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int t = w * 64 + 4 * it + lg;
    float p[G];
    if constexpr (G % 4 == 0) {
#pragma unroll
      for (int h4 = 0; h4 < G; h4 += 4) {
        const f32x4 pv = *reinterpret_cast<const f32x4*>(&sc[t * GP + h4]);
        p[h4] = pv[0]; p[h4 + 1] = pv[1]; p[h4 + 2] = pv[2]; p[h4 + 3] = pv[3];
      }
    } else {
#pragma unroll
      for (int h = 0; h < G; ++h) p[h] = sc[t * GP + h];
    }
    float vv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) vv[j] = bf2f(vf[it][j]);
#pragma unroll
    for (int h = 0; h < G; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[h][j] += p[h] * vv[j];
  }
  // reduce over the 4 token sub-slots of the wave (lanes l, l^16, l^32, l^48)
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = acc[h][j];
      a += __shfl_xor(a, 16, kWave);
      a += __shfl_xor(a, 32, kWave);
      acc[h][j] = a;
    }
  if (lg == 0) {
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float* r = red + (w * G + h) * D + 8 * l15;
      *reinterpret_cast<f32x4*>(r) = f32x4{acc[h][0], acc[h][1], acc[h][2], acc[h][3]};
      *reinterpret_cast<f32x4*>(r + 4) = f32x4{acc[h][4], acc[h][5], acc[h][6], acc[h][7]};
    }
  }
  __syncthreads();
  for (int e = tid; e < G * D; e += 256) {
    const int h = e / D, d = e % D;
    const float o = red[(0 * G + h) * D + d] + red[(1 * G + h) * D + d] + red[(2 * G + h) * D + d] +
                    red[(3 * G + h) * D + d];
    const int hq = kvh * G + h;
    if (ns_b == 1) {  // whole context in this split: final output, combine skips it
      const float l = lh[h];
      out[((int64_t)b * Hq + hq) * D + d] = f2bf(l > 0.f ? o / l : 0.f);
    } else {
      o_part[(((int64_t)b * Hq + hq) * num_splits + s) * D + d] = o;
      if (d == 0) {
        float* ml = ml_part + (((int64_t)b * Hq + hq) * num_splits + s) * 2;
        ml[0] = mh[h];
        ml[1] = lh[h];
      }
    }
  }
}

template <int G>
__global__ void __launch_bounds__(256, (G <= 4 ? 3 : 2)) attn_decode_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int* __restrict__ block_tables, const int* __restrict__ seq_lens,
    bf16_t* __restrict__ out, float* __restrict__ o_part, float* __restrict__ ml_part, int Hkv,
    int page_size, int log2_page, int max_pages, int num_splits, float scale_log2,
    const int* __restrict__ work) {
  const int wi = blockIdx.x;
  if (wi >= work[0]) return;  // grid is sized for the host's bound; the plan may hold fewer items
  const int item = work[1 + wi];
  attn_decode_item<G>(q, kc, vc, block_tables, seq_lens, out, o_part, ml_part, Hkv, page_size, log2_page,
                      max_pages, num_splits, scale_log2, item >> 8, item & 255, blockIdx.y);
}

// Combine the per-split partials: grid (B*Hq), block D threads.
__global__ void attn_decode_combine_kernel(const float* __restrict__ o_part, const float* __restrict__ ml_part,
                                           const int* __restrict__ seq_lens, bf16_t* __restrict__ out, int Hq,
                                           int num_splits, int max_tokens) {
  constexpr int D = 128;
  const int bh = blockIdx.x, b = bh / Hq, d = threadIdx.x;
  const int len = min(seq_lens[b], max_tokens);
  const int ns = min(num_splits, (len + kSplit - 1) / kSplit);
  if (ns == 1) return;  // written directly by the attention kernel
  if (ns == 0) {
    out[(int64_t)bh * D + d] = 0;
    return;
  }
  const float* ml = ml_part + (int64_t)bh * num_splits * 2;
  float M = -INFINITY;
  for (int s = 0; s < ns; ++s) M = fmaxf(M, ml[2 * s]);
  float L = 0.f, o = 0.f;
  for (int s = 0; s < ns; ++s) {
    const float wgt = exp2f(ml[2 * s] - M);
    L += wgt * ml[2 * s + 1];
    o += wgt * o_part[((int64_t)bh * num_splits + s) * D + d];
  }
  out[(int64_t)bh * D + d] = f2bf(L > 0.f ? o / L : 0.f);
}

int attn_decode(const bf16_t* q, const bf16_t* k_cache, const bf16_t* v_cache, const int* block_tables,
                const int* seq_lens, bf16_t* out, float* o_part, float* ml_part, int* work, int B, int Hq,
                int Hkv, int head_dim, int page_size, int max_pages, int num_splits, float scale,
                hipStream_t stream) {
  if (B == 0) return 0;
  if (head_dim != 128) return -1;
  if (page_size < 16 || (page_size & (page_size - 1)) != 0) return -2;  // pg_lds holds <= 18 pages
  int log2p = 0;
  while ((1 << log2p) < page_size) ++log2p;
  const int G = Hq / Hkv;
  if (num_splits > 255) return -4;  // split index is packed in 8 bits
  const float scale_log2 = scale * 1.4426950408889634f;
  attn_decode_plan_kernel<<<1, 1024, 0, stream>>>(seq_lens, B, max_pages * page_size, num_splits, work);
  OAMD_LAUNCH_CHECK();
  // One workgroup per (work item, kv head). num_splits is the caller's bound on the
  // splits of the longest sequence in THIS call (not the model's max context): the
  // engine captures one graph per bound, so the grid has no empty splits when the
  // batch is length-uniform, and the packed work list keeps the live items first.
  dim3 grid(B * num_splits, Hkv, 1);
#define OAMD_DEC(GG)                                                                                 \
  attn_decode_kernel<GG><<<grid, 256, 0, stream>>>(q, k_cache, v_cache, block_tables, seq_lens, out, \
                                                   o_part, ml_part, Hkv, page_size, log2p, max_pages,  \
                                                   num_splits, scale_log2, work)
  switch (G) {
    case 1: OAMD_DEC(1); break;
    case 2: OAMD_DEC(2); break;
    case 4: OAMD_DEC(4); break;
    case 8: OAMD_DEC(8); break;
    default: return -3;
  }
#undef OAMD_DEC
  OAMD_LAUNCH_CHECK();
  attn_decode_combine_kernel<<<B * Hq, 128, 0, stream>>>(o_part, ml_part, seq_lens, out, Hq, num_splits,
                                                         max_pages * page_size);
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
