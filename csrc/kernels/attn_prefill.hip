// Causal flash attention for prefill, variable-length packed sequences, GQA,
// on MFMA.
//
// Work item = (64-row query block of one sequence, query head). 4 waves; each
// wave owns 16 query rows. Per 64-key tile:
//   S = Q K^T      16 x v_mfma_f32_16x16x32_bf16 per wave (Q in registers)
//   online softmax in the C-fragment layout (row max/sum over 16 lanes)
//   O += P V       16 x MFMA per wave, P bounced through a per-wave LDS image
// K is staged row-major and V transposed ([d][key]) in LDS, both XOR-swizzled
// on 16-B chunks so every ds_read_b128 of a 16-lane group hits 16 distinct
// bank slots (cdna_hip_programming.md §5.5 T2).
// Fragment maps for 16x16x32 bf16 (cdna_hip_programming.md §3):
//   A: lane l -> A[l&15][8(l>>4)+j]   B: lane l -> B[8(l>>4)+j][l&15]
//   C: col = l&15, row = 4(l>>4)+i
#include "common.h"
#include "kernels.h"

namespace oamd {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8_t as_bf8(u16x8 v) { return __builtin_bit_cast(bf16x8_t, v); }

__global__ void __launch_bounds__(256) attn_prefill_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    bf16_t* __restrict__ o, const int* __restrict__ cu_seqlens, const int* __restrict__ work_seq,
    const int* __restrict__ work_q0, int Hq, int Hkv, float scale_log2) {
  constexpr int D = 128, BQ = 64, BK = 64;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[BK * D];       // [key][d], 256-B rows
  __shared__ __attribute__((aligned(16))) bf16_t Vt[D * BK];       // [d][key], 128-B rows
  __shared__ __attribute__((aligned(16))) bf16_t Ps[4][16 * BK];   // per wave [row][key]

  const int wi = blockIdx.x, hq = blockIdx.y;
  const int kvh = hq / (Hq / Hkv);
  const int seq = work_seq[wi];
  const int s0 = cu_seqlens[seq];
  const int slen = cu_seqlens[seq + 1] - s0;
  const int q0 = work_q0[wi];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l15 = lane & 15, lhi = lane >> 4;

  // Q fragments (A operand) for this wave's 16 rows, 4 k-steps over D = 128
  u16x8 qa[4];
  {
    const int row = q0 + w * 16 + l15;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (row < slen)
        qa[s] = *reinterpret_cast<const u16x8*>(q + ((int64_t)(s0 + row) * Hq + hq) * D + 32 * s + 8 * lhi);
      else
        qa[s] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }

  f32x4 oacc[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) oacc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[4], lrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { mrow[i] = -INFINITY; lrow[i] = 0.f; }

  const int kend = min(slen, q0 + BQ);  // causal: keys < last row of the block + 1
  const int ntiles = (kend + BK - 1) / BK;
  char* ks_b = reinterpret_cast<char*>(Ks);
  char* vt_b = reinterpret_cast<char*>(Vt);
  char* ps_b = reinterpret_cast<char*>(Ps[w]);

  for (int kt = 0; kt < ntiles; ++kt) {
    const int kb = kt * BK;
    __syncthreads();
    // ---- stage K (row-major, swizzled) and V (transposed, swizzled) ----
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = tid + r * 256;
      const int key = c >> 4, ch = c & 15;
      u16x8 kv = u16x8{0, 0, 0, 0, 0, 0, 0, 0}, vv = kv;
      if (kb + key < slen) {
        const int64_t off = ((int64_t)(s0 + kb + key) * Hkv + kvh) * D + ch * 8;
        kv = *reinterpret_cast<const u16x8*>(k + off);
        vv = *reinterpret_cast<const u16x8*>(v + off);
      }
      *reinterpret_cast<u16x8*>(ks_b + key * 256 + ((ch ^ (key & 15)) << 4)) = kv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = ch * 8 + j;
        const int pc = (key >> 3) ^ ((d >> 1) & 7);
        *reinterpret_cast<bf16_t*>(vt_b + d * 128 + (pc << 4) + ((key & 7) << 1)) = vv[j];
      }
    }
    __syncthreads();

    // ---- S = Q K^T ----
    f32x4 sacc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      sacc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int key = 16 * n + l15;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int ch = 4 * s + lhi;
        const u16x8 kb8 = *reinterpret_cast<const u16x8*>(ks_b + key * 256 + ((ch ^ (key & 15)) << 4));
        sacc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(qa[s]), as_bf8(kb8), sacc[n], 0, 0, 0);
      }
    }

    // ---- online softmax (rows 4*lhi+i, key col l15 + 16n) ----
    const bool diag = (kb + BK > q0 + w * 16);  // some key may exceed some row of this wave
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qrow = q0 + w * 16 + 4 * lhi + i;
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int key = kb + 16 * n + l15;
        float sv = sacc[n][i] * scale_log2;
        if (key >= slen || (diag && key > qrow)) sv = -INFINITY;
        sacc[n][i] = sv;
        mx = fmaxf(mx, sv);
      }
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, kWave));
      const float mnew = fmaxf(mrow[i], mx);
      const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
      alpha[i] = exp2f(mrow[i] - msafe);
      float rs = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const float p = exp2f(sacc[n][i] - msafe);
        sacc[n][i] = p;
        rs += p;
      }
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) rs += __shfl_xor(rs, o2, kWave);
      lrow[i] = lrow[i] * alpha[i] + rs;
      mrow[i] = mnew;
    }
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) oacc[m][i] *= alpha[i];

    // ---- P -> LDS (bf16), re-read as A fragments ----
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * lhi + i, key = 16 * n + l15;
        const int pc = (key >> 3) ^ ((r >> 1) & 7);
        *reinterpret_cast<bf16_t*>(ps_b + r * 128 + (pc << 4) + ((key & 7) << 1)) = f2bf(sacc[n][i]);
      }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    u16x8 pa[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = 4 * s + lhi;
      pa[s] = *reinterpret_cast<const u16x8*>(ps_b + l15 * 128 + ((ch ^ ((l15 >> 1) & 7)) << 4));
    }
    // ---- O += P V ----
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int d = 16 * m + l15;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = 4 * s + lhi;
        const u16x8 vb = *reinterpret_cast<const u16x8*>(vt_b + d * 128 + ((ch ^ ((d >> 1) & 7)) << 4));
        oacc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(pa[s]), as_bf8(vb), oacc[m], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  // ---- epilogue ----
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = q0 + w * 16 + 4 * lhi + i;
    if (row < slen) {
      const float inv = lrow[i] > 0.f ? 1.f / lrow[i] : 0.f;
      bf16_t* dst = o + ((int64_t)(s0 + row) * Hq + hq) * D;
#pragma unroll
      for (int m = 0; m < 8; ++m) dst[16 * m + l15] = f2bf(oacc[m][i] * inv);
    }
  }
}

// ---------------------------------------------------------------------------
// v2: GQA-grouped, software-pipelined. A block is (16 x RG query rows, one KV
// head) with 8 waves: wave w computes query head kvh * G + (w % G) for rows
// 16 (w / G) .. +16 (G = Hq / Hkv in {1, 2, 4, 8}, RG = 8 / G), so every staged
// K/V tile feeds all G query heads that share it (v1 staged it once per query
// head). The next tile's K/V is loaded into registers while the current tile's
// MFMAs run and is written to LDS after the barrier, so global-load latency
// hides behind compute instead of being paid once per tile.
template <int G>
__global__ void __launch_bounds__(512) attn_prefill_gqa_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    bf16_t* __restrict__ o, const int* __restrict__ cu_seqlens, const int* __restrict__ work_seq,
    const int* __restrict__ work_q0, int Hq, int Hkv, float scale_log2) {
  constexpr int D = 128, BK = 64, RG = 8 / G, BQ = 16 * RG;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[BK * D];       // [key][d], 256-B rows
  __shared__ __attribute__((aligned(16))) bf16_t Vt[D * BK];       // [d][key], 128-B rows
  __shared__ __attribute__((aligned(16))) bf16_t Ps[8][16 * BK];   // per wave [row][key]

  const int wi = blockIdx.x, kvh = blockIdx.y;
  const int seq = work_seq[wi];
  const int s0 = cu_seqlens[seq];
  const int slen = cu_seqlens[seq + 1] - s0;
  const int q0 = work_q0[wi];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l15 = lane & 15, lhi = lane >> 4;
  const int hq = kvh * G + (w % G);
  const int rbase = q0 + 16 * (w / G);  // this wave's first query row

  u16x8 qa[4];
  {
    const int row = rbase + l15;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (row < slen)
        qa[s] = *reinterpret_cast<const u16x8*>(q + ((int64_t)(s0 + row) * Hq + hq) * D + 32 * s + 8 * lhi);
      else
        qa[s] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  f32x4 oacc[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) oacc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[4], lrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { mrow[i] = -INFINITY; lrow[i] = 0.f; }

  const int kend = min(slen, q0 + BQ);
  const int ntiles = (kend + BK - 1) / BK;
  // rows of this wave that exist at all: a wave past the sequence end only stages
  const bool active = rbase < slen;
  const int wend = min(slen, rbase + 16);  // keys this wave can see: < wend
  char* ks_b = reinterpret_cast<char*>(Ks);
  char* vt_b = reinterpret_cast<char*>(Vt);
  char* ps_b = reinterpret_cast<char*>(Ps[w]);

  // K/V chunk c = tid + 512 r (r < 2): key c >> 4, 16-B chunk c & 15 of the 256-B row
  u16x8 kr[2], vr[2];
  auto load_tile = [&](int kb) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + r * 512;
      const int key = c >> 4, ch = c & 15;
      kr[r] = vr[r] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (kb + key < slen) {
        const int64_t off = ((int64_t)(s0 + kb + key) * Hkv + kvh) * D + ch * 8;
        kr[r] = *reinterpret_cast<const u16x8*>(k + off);
        vr[r] = *reinterpret_cast<const u16x8*>(v + off);
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + r * 512;
      const int key = c >> 4, ch = c & 15;
      *reinterpret_cast<u16x8*>(ks_b + key * 256 + ((ch ^ (key & 15)) << 4)) = kr[r];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = ch * 8 + j;
        const int pc = (key >> 3) ^ ((d >> 1) & 7);
        *reinterpret_cast<bf16_t*>(vt_b + d * 128 + (pc << 4) + ((key & 7) << 1)) = vr[r][j];
      }
    }
  };

  load_tile(0);
  for (int kt = 0; kt < ntiles; ++kt) {
    const int kb = kt * BK;
    __syncthreads();  // previous tile fully consumed
    store_tile();
    __syncthreads();
    if (kt + 1 < ntiles) load_tile(kb + BK);  // in flight during this tile's MFMAs
    if (!active || kb >= wend) continue;      // no visible key in this tile for this wave

    f32x4 sacc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      sacc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int key = 16 * n + l15;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int ch = 4 * s + lhi;
        const u16x8 kb8 = *reinterpret_cast<const u16x8*>(ks_b + key * 256 + ((ch ^ (key & 15)) << 4));
        sacc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(qa[s]), as_bf8(kb8), sacc[n], 0, 0, 0);
      }
    }
    const bool diag = (kb + BK > rbase);
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qrow = rbase + 4 * lhi + i;
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int key = kb + 16 * n + l15;
        float sv = sacc[n][i] * scale_log2;
        if (key >= slen || (diag && key > qrow)) sv = -INFINITY;
        sacc[n][i] = sv;
        mx = fmaxf(mx, sv);
      }
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, kWave));
      const float mnew = fmaxf(mrow[i], mx);
      const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
      alpha[i] = exp2f(mrow[i] - msafe);
      float rs = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const float p = exp2f(sacc[n][i] - msafe);
        sacc[n][i] = p;
        rs += p;
      }
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) rs += __shfl_xor(rs, o2, kWave);
      lrow[i] = lrow[i] * alpha[i] + rs;
      mrow[i] = mnew;
    }
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) oacc[m][i] *= alpha[i];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * lhi + i, key = 16 * n + l15;
        const int pc = (key >> 3) ^ ((r >> 1) & 7);
        *reinterpret_cast<bf16_t*>(ps_b + r * 128 + (pc << 4) + ((key & 7) << 1)) = f2bf(sacc[n][i]);
      }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    u16x8 pa[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = 4 * s + lhi;
      pa[s] = *reinterpret_cast<const u16x8*>(ps_b + l15 * 128 + ((ch ^ ((l15 >> 1) & 7)) << 4));
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int d = 16 * m + l15;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = 4 * s + lhi;
        const u16x8 vb = *reinterpret_cast<const u16x8*>(vt_b + d * 128 + ((ch ^ ((d >> 1) & 7)) << 4));
        oacc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(pa[s]), as_bf8(vb), oacc[m], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (!active) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = rbase + 4 * lhi + i;
    if (row < slen) {
      const float inv = lrow[i] > 0.f ? 1.f / lrow[i] : 0.f;
      bf16_t* dst = o + ((int64_t)(s0 + row) * Hq + hq) * D;
#pragma unroll
      for (int m = 0; m < 8; ++m) dst[16 * m + l15] = f2bf(oacc[m][i] * inv);
    }
  }
}

int attn_prefill_block_q(int Hq, int Hkv) {
  if (Hkv <= 0 || Hq % Hkv != 0) return 64;
  const int G = Hq / Hkv;
  return (G == 1 || G == 2 || G == 4 || G == 8) ? 16 * (8 / G) : 64;
}

int attn_prefill(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, const int* cu_seqlens,
                 const int* work_seq, const int* work_q0, int num_work, int Hq, int Hkv, int head_dim,
                 float scale, int block_q, hipStream_t stream) {
  if (num_work == 0) return 0;
  if (head_dim != 128) return -1;
  if (Hq % Hkv != 0) return -3;
  const float sl2 = scale * 1.4426950408889634f;
  const int G = Hq / Hkv;
  const bool gqa = (G == 1 || G == 2 || G == 4 || G == 8) && block_q == 16 * (8 / G);
  if (gqa) {
    dim3 grid(num_work, Hkv);
#define OAMD_PF2(GG) \
  attn_prefill_gqa_kernel<GG><<<grid, 512, 0, stream>>>(q, k, v, o, cu_seqlens, work_seq, work_q0, Hq, Hkv, sl2)
    switch (G) {
      case 1: OAMD_PF2(1); break;
      case 2: OAMD_PF2(2); break;
      case 4: OAMD_PF2(4); break;
      default: OAMD_PF2(8); break;
    }
#undef OAMD_PF2
  } else if (block_q == 64) {
    dim3 grid(num_work, Hq);
    attn_prefill_kernel<<<grid, 256, 0, stream>>>(q, k, v, o, cu_seqlens, work_seq, work_q0, Hq, Hkv, sl2);
  } else {
    return -4;
  }
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
