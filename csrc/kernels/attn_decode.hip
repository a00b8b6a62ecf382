// Paged decode attention, split-KV ("flash-decoding"), GQA.
//
// One query token per sequence. Workgroup = (split of 256 cached tokens,
// kv-head, sequence); the G = Hq/Hkv query heads that share the kv-head are
// processed together so each K/V row is read from HBM once for all of them.
// With G <= 8 query rows per kv head this is a streaming, memory-bound op, so
// K/V go straight to VGPRs with 16-B loads (cdna_hip_programming.md App. B
// "Attention decode": GEMV-like, no LDS round trip for the stream) and the
// dot products run on the VALU; the VALU budget per token (~40 SIMD cycles
// for G = 4) is well under the ~200 SIMD cycles per 512 B of K+V that the
// HBM rate allows per CU.
//
// Two phases per split, so there is no online-softmax rescaling at all:
//   1. s[h][t] = q_h . k_t for all tokens of the split -> LDS (4 KB at G = 4)
//   2. block max/sum per head, p = exp2(s - m), o_h = sum_t p[h][t] v_t
// Lane mapping (both phases): token sub-slot = lane >> 4 (4 tokens per wave
// step), dims 8*(lane & 15) .. +8 (one 16-B load per lane per token).
// KV cache layout: [pages, Hkv, page_size, D] bf16 (a kv-head's tokens of one
// page are contiguous: 4 consecutive tokens = 1 KiB per wave load).
#include "common.h"
#include "kernels.h"

namespace oamd {

constexpr int kSplit = 256;  // tokens per split == threads per block

template <int G>
__global__ void __launch_bounds__(256) attn_decode_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int* __restrict__ block_tables, const int* __restrict__ seq_lens,
    bf16_t* __restrict__ out, float* __restrict__ o_part, float* __restrict__ ml_part, int Hkv,
    int page_size, int log2_page, int max_pages, int num_splits, float scale_log2) {
  constexpr int D = 128;
  __shared__ __attribute__((aligned(16))) float sc[G * kSplit];
  __shared__ __attribute__((aligned(16))) float red[4 * G * D];
  __shared__ float wred[4][G];

  const int s = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int Hq = Hkv * G;
  const int len = min(seq_lens[b], max_pages * page_size);  // never index past the block table
  const int start = s * kSplit;
  if (start >= len && !(num_splits == 1 && len == 0)) return;  // empty split: combine skips it
  const int n = min(len - start, kSplit);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, sub = lane >> 4;
  const int dl = (lane & 15) * 8;
  const int* bt = block_tables + (int64_t)b * max_pages;

  // q for the G heads of this kv head, this lane's 8 dims, pre-scaled into log2 domain
  float qf[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const u16x8 qv = *reinterpret_cast<const u16x8*>(q + ((int64_t)b * Hq + kvh * G + h) * D + dl);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[h][j] = bf2f(qv[j]) * scale_log2;
  }

  auto row_off = [&](int t) -> int64_t {
    const int tok = start + t;
    const int64_t page = bt[tok >> log2_page];
    return ((page * Hkv + kvh) * page_size + (tok & (page_size - 1))) * (int64_t)D + dl;
  };

  // ---- phase 1: scores ----
#pragma unroll 4
  for (int it = 0; it < kSplit / 16; ++it) {
    const int t = it * 16 + w * 4 + sub;
    if (t < n) {
      const u16x8 kv = *reinterpret_cast<const u16x8*>(kc + row_off(t));
      float kf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[j] = bf2f(kv[j]);
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) d += qf[h][j] * kf[j];
        d = group_sum<16>(d);
        if ((lane & 15) == 0) sc[h * kSplit + t] = d;
      }
    }
  }
  __syncthreads();

  // ---- block softmax per head (thread tid <-> token tid) ----
  float mh[G], lh[G];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const float v = tid < n ? sc[h * kSplit + tid] : -INFINITY;
    const float m = wave_max(v);
    if (lane == 0) wred[w][h] = m;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < G; ++h) mh[h] = fmaxf(fmaxf(wred[0][h], wred[1][h]), fmaxf(wred[2][h], wred[3][h]));
  __syncthreads();
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const float p = tid < n ? exp2f(sc[h * kSplit + tid] - mh[h]) : 0.f;
    if (tid < n) sc[h * kSplit + tid] = p;
    const float ls = wave_sum(p);
    if (lane == 0) wred[w][h] = ls;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < G; ++h) lh[h] = wred[0][h] + wred[1][h] + wred[2][h] + wred[3][h];

  // ---- phase 2: o = P V ----
  float acc[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[h][j] = 0.f;
#pragma unroll 4
  for (int it = 0; it < kSplit / 16; ++it) {
    const int t = it * 16 + w * 4 + sub;
    if (t < n) {
      const u16x8 vv = *reinterpret_cast<const u16x8*>(vc + row_off(t));
#pragma unroll
      for (int h = 0; h < G; ++h) {
        const float p = sc[h * kSplit + t];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[h][j] += p * bf2f(vv[j]);
      }
    }
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
  if (sub == 0) {
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float* r = red + (w * G + h) * D + dl;
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
    if (num_splits == 1) {
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

// Combine the per-split partials: grid (B*Hq), block D threads.
__global__ void attn_decode_combine_kernel(const float* __restrict__ o_part, const float* __restrict__ ml_part,
                                           const int* __restrict__ seq_lens, bf16_t* __restrict__ out, int Hq,
                                           int num_splits) {
  constexpr int D = 128;
  const int bh = blockIdx.x, b = bh / Hq, d = threadIdx.x;
  const int len = seq_lens[b];
  const int ns = min(num_splits, (len + kSplit - 1) / kSplit);
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
                const int* seq_lens, bf16_t* out, float* o_part, float* ml_part, int B, int Hq, int Hkv,
                int head_dim, int page_size, int max_pages, int num_splits, float scale,
                hipStream_t stream) {
  if (B == 0) return 0;
  if (head_dim != 128) return -1;
  if (page_size <= 0 || (page_size & (page_size - 1)) != 0) return -2;
  int log2p = 0;
  while ((1 << log2p) < page_size) ++log2p;
  const int G = Hq / Hkv;
  const float scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(num_splits, Hkv, B);
#define OAMD_DEC(GG)                                                                                 \
  attn_decode_kernel<GG><<<grid, 256, 0, stream>>>(q, k_cache, v_cache, block_tables, seq_lens, out, \
                                                   o_part, ml_part, Hkv, page_size, log2p, max_pages,  \
                                                   num_splits, scale_log2)
  switch (G) {
    case 1: OAMD_DEC(1); break;
    case 2: OAMD_DEC(2); break;
    case 4: OAMD_DEC(4); break;
    case 8: OAMD_DEC(8); break;
    default: return -3;
  }
#undef OAMD_DEC
  OAMD_LAUNCH_CHECK();
  if (num_splits > 1) {
    attn_decode_combine_kernel<<<B * Hq, 128, 0, stream>>>(o_part, ml_part, seq_lens, out, Hq, num_splits);
    OAMD_LAUNCH_CHECK();
  }
  return 0;
}

}  // namespace oamd
