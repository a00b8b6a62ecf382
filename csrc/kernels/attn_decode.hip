// Paged decode attention, GQA, streaming split-KV.
//
// One query token per sequence. Workgroup = (sequence, split, kv-head); the
// G = Hq/Hkv query heads sharing the kv-head are processed together so every
// K/V row is read from HBM exactly once. The op is HBM-bound
// (B x ctx x Hkv x 512 B per layer), so the structure is built around keeping
// bytes in flight for the WHOLE life of a workgroup:
//   * a workgroup walks its token range in chunks of 4 x TW tokens (TW per
//     wave), with the K/V registers double-buffered: the loads of chunk c+1
//     are issued before chunk c is consumed (counted vmcnt, no drain), and the
//     consume of chunk c requests chunk c+2 into the registers it frees (K right
//     after the S MFMAs, V after P.V). tools/probe/kv_stream.hip measured why that
//     matters: the same paged K/V stream with no compute reads at 6.3-6.6 TB/s,
//     and a dependent per-chunk compute chain of the consume's length costs ~10 %;
//   * the first two chunks are requested before the LDS page table / q are set
//     up (page ids from scalar loads), and a sequence's kv-heads are dispatched
//     back to back;
//   * the per-call split count is chosen by the host so that only small
//     batches are split (B x Hkv workgroups already fill 256 CUs at B >= 128):
//     at serving batch sizes there is no partial output, no combine kernel and
//     no per-call planning kernel at all;
//   * each wave runs its own online softmax (running max / sum per head kept
//     per lane, rescale factors broadcast with v_readlane) — no block barrier
//     inside the loop; the 4 waves are merged once at the end through LDS;
//   * S = K Q^T on MFMA (v_mfma_f32_16x16x32_bf16, K tile = A operand, the G
//     heads zero-padded to 16 columns = B operand); P V on the VALU from the V
//     rows already in registers (16 B per lane, P read back as float4).
// Fragment maps (cdna_hip_programming.md §3): A lane l -> A[l&15][8(l>>4)+j];
// B lane l -> B[8(l>>4)+j][l&15]; C col = l&15, row = 4(l>>4)+r. The dims of a
// k-step are permuted so lane group g covers dims 32g..32g+31 over the 4
// k-steps (Q uses the same permutation, so the contraction is unchanged).
// KV cache layout: [pages, Hkv, page_size, D] bf16. V rows are token-major; K is
// stored in 16-token tiles laid out [ks 4][lg 4][token 16][8 dims] (d = 32*lg +
// 8*ks + j), so each K fragment load (fixed ks) is ONE contiguous 1 KB wave
// access instead of 16 token rows x 64 B (written that way by rope_kv).
// FP8 cache (OCP e4m3fn, per-tensor scales): the same layout with 1-byte elements,
// so every load moves half the bytes. K fragments are widened to bf16 in registers
// (exact) for the bf16 MFMA against the bf16 query; V
// to fp32 (v_cvt_pk_f32_fp8) for the VALU P.V. k_scale rides in the softmax scale,
// v_scale multiplies the output.
#include "common.h"
#include "kernels.h"

namespace oamd {

constexpr int kMaxPagesLds = 1024;  // page ids of one split staged in LDS

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ u16x8 ld16(const bf16_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(p));
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// Per-element-type access to the cache: a fragment is 8 consecutive elements
// (16 B of bf16, 8 B of fp8).
template <typename KV>
struct KVT;
template <>
struct KVT<bf16_t> {
  using frag = u16x8;
  static __device__ __forceinline__ frag load(const bf16_t* p) { return ld16(p); }
  static __device__ __forceinline__ u16x8 to_bf16(const frag& f) { return f; }
  static __device__ __forceinline__ void to_f32(const frag& f, float (&o)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf2f(f[j]);
  }
};
template <>
struct KVT<uint8_t> {
  using frag = u32x2;
  static __device__ __forceinline__ frag load(const uint8_t* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
  }
  // fp8 -> fp32 (v_cvt_pk_f32_fp8) then the upper halves of two floats into one dword
  // (v_perm_b32): exact, as every e4m3 value is a bf16 value. (The one-instruction
  // v_cvt_scalef32_pk_bf16_fp8 form was mis-packed by hipcc: it duplicated the low
  // half into both halves of the register.)
  static __device__ __forceinline__ u16x8 to_bf16(const frag& f) {
    u32x4 d;
    const unsigned w[2] = {f[0], f[1]};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2_t lo = __builtin_amdgcn_cvt_pk_f32_fp8(w[h], false);
      const f32x2_t hi = __builtin_amdgcn_cvt_pk_f32_fp8(w[h], true);
      d[2 * h] = __builtin_amdgcn_perm(__float_as_uint(lo[1]), __float_as_uint(lo[0]), 0x07060302u);
      d[2 * h + 1] = __builtin_amdgcn_perm(__float_as_uint(hi[1]), __float_as_uint(hi[0]), 0x07060302u);
    }
    return __builtin_bit_cast(u16x8, d);
  }
  static __device__ __forceinline__ void to_f32(const frag& f, float (&o)[8]) {
    const unsigned w[2] = {f[0], f[1]};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2_t lo = __builtin_amdgcn_cvt_pk_f32_fp8(w[h], false);
      const f32x2_t hi = __builtin_amdgcn_cvt_pk_f32_fp8(w[h], true);
      o[4 * h + 0] = lo[0];
      o[4 * h + 1] = lo[1];
      o[4 * h + 2] = hi[0];
      o[4 * h + 3] = hi[1];
    }
  }
};

// 8 bf16 values -> the cache element type (bf16 as is; fp8: e4m3(x * inv), saturated),
// exactly as rope.hip stores them
template <typename KV>
__device__ __forceinline__ void cache_put8(KV* dst, const u16x8& v, float inv) {
  if constexpr (sizeof(KV) == 2) {
    *reinterpret_cast<u16x8*>(dst) = v;
  } else {
    auto f = [&](int j) { return fminf(fmaxf(bf2f(v[j]) * inv, -448.f), 448.f); };
    int lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(f(0), f(1), lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(f(2), f(3), lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(f(4), f(5), hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(f(6), f(7), hi, true);
    *reinterpret_cast<uint2*>(dst) = uint2{(unsigned)lo, (unsigned)hi};
  }
}

// One bf16 value as the attention kernel sees it once it is in the cache: bf16 as is;
// fp8: the e4m3 code of x * inv as a float (the scale is applied by the caller, as for
// streamed K / V)
template <typename KV>
__device__ __forceinline__ float kv_value(bf16_t x, float inv) {
  if constexpr (sizeof(KV) == 2) {
    return bf2f(x);
  } else {
    const float v = fminf(fmaxf(bf2f(x) * inv, -448.f), 448.f);
    const int pk = __builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false);
    return __builtin_amdgcn_cvt_pk_f32_fp8(pk, false)[0];
  }
}

// Token range of split s of a sequence of `len` tokens cut into at most
// `num_splits` pieces of a multiple of `chunk` tokens. Shared with the combine
// kernel so both agree on how many splits a sequence really has.
__device__ __forceinline__ int split_len(int len, int num_splits, int chunk) {
  const int per = (len + num_splits - 1) / num_splits;
  return (per + chunk - 1) / chunk * chunk;
}

template <typename KV, int NT>
struct KVRegs {
  typename KVT<KV>::frag k[NT][4];   // K tile i: token 16i + l15, dims 32*lg + 8*ks
  typename KVT<KV>::frag v[4 * NT];  // token 4*it + lg, dims 8*l15
};

template <int G, int NT, typename KV = bf16_t>
__global__ void __launch_bounds__(256, (NT == 1 && G <= 4) ? 3 : 2)
    // kc / vc not __restrict__: the fused RoPE stores the new token's K/V through them
    attn_decode_kernel(const bf16_t* __restrict__ q, const KV* kc, const KV* vc,
                       const int* __restrict__ block_tables, const int* __restrict__ seq_lens,
                       bf16_t* __restrict__ out, float* __restrict__ o_part, float* __restrict__ ml_part, int Hkv,
                       int page_size, int log2_page, int max_pages, int num_splits, float scale_log2,
                       float v_scale, int head_minor, DecodeRope rp, float k_inv, float v_inv) {
  using T = KVT<KV>;
  constexpr int D = 128;
  constexpr int TW = 16 * NT;  // tokens per wave per chunk
  constexpr int CH = 4 * TW;   // tokens per workgroup per chunk
  constexpr int GP = (G < 4) ? 4 : G;
  __shared__ int pg_lds[kMaxPagesLds];
  // per-wave P tile [token][head], then the per-(token group, head) rescale factors [lg][head]
  __shared__ __attribute__((aligned(16))) float pw[4][TW * GP + 4 * GP];
  __shared__ __attribute__((aligned(16))) float red[4][G][D];
  __shared__ float mls[4][G][2];
  __shared__ u16x8 q_lds[4][64];
  // fused RoPE (rp.cos_t set): items = G query-head + 1 key-head rotations (8 per head,
  // 8 + 8 dims each) and 16 value copies (8 dims); per (item, split-K slab) fp32 partials
  constexpr int NI = (G + 1) * 8 + 16;
  __shared__ __attribute__((aligned(16))) float rp_part[NI * kRopeMaxS * 16];
  __shared__ u16x8 kv_new[2][16];   // the new token's k, v (bf16, dims 8i..8i+7)
  __shared__ float s_new[G];        // its scores (log2 domain) per head

  // work item of this workgroup: (sequence, split, kv-head); head_minor dispatches the
  // kv-heads of one sequence back to back (they read different head slices of the
  // same pages), else one kv-head across all sequences first
  int b, s, kvh;
  if (head_minor) {
    const int lin = blockIdx.x + gridDim.x * blockIdx.y;
    kvh = lin % Hkv;
    const int rest = lin / Hkv;
    b = rest / num_splits;
    s = rest - b * num_splits;
  } else {
    b = blockIdx.x / num_splits;
    s = blockIdx.x - b * num_splits;
    kvh = blockIdx.y;
  }
  const int Hq = Hkv * G;
  const int len = min(seq_lens[b], max_pages * page_size);  // never index past the block table
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lg = lane >> 4;
  if (len <= 0) {  // padding row: zero output (written once, by split 0)
    if (s == 0)
      for (int e = tid; e < G * D; e += 256) out[((int64_t)b * Hq + kvh * G) * D + e] = 0;
    return;
  }
  const int per = split_len(len, num_splits, CH);
  const int start = s * per;
  if (start >= len) return;  // this sequence has fewer splits than the grid
  const int end = min(len, start + per);
  const int ns_b = (len + per - 1) / per;
  const int nch = (end - start + CH - 1) / CH;
  const bool fused = rp.cos_t != nullptr;
  const bool writer = fused && end == len;   // this split holds the new token (position len - 1)
  const int end_s = writer ? len - 1 : end;  // the streamed cache tokens (the new one is not there yet)

  // Page ids of the split -> LDS: the steady-state data loads depend only on LDS
  // (lgkmcnt), never on a global load that would share vmcnt with them. The first
  // two chunks do not wait for that: their page ids come straight from the block
  // table (wave-uniform scalar loads), so their K/V requests leave before the LDS
  // page table and q are even written (one dependent latency less per workgroup).
  const int page0 = start >> log2_page;
  const int npg = ((end - 1) >> log2_page) - page0 + 1;
  const int* btb = block_tables + (int64_t)b * max_pages + page0;
  // Fused RoPE, phase 1: every (item, slab) pair loads its 16 fp32 partials (x1: dims
  // g..g+7 of the head, x2: dims 64+g..; a value copy only x1), at most 2 pairs per
  // thread, all issued before any K/V load so their LDS writes never wait for K/V
  const int ncol = (Hq + 2 * Hkv) * D;
  const int nS = rp.xp ? rp.S : 1;
  f32x4 rv[2][4];
  f32x4 csv[4];   // cos (g..g+7) | sin (g..g+7) of a rotation item's position, prefetched
  auto rp_col = [&](int item) -> int {   // first column of an item's x1
    if (item < (G + 1) * 8) {
      const int h = item >> 3, g = (item & 7) * 8;
      return (h < G ? (kvh * G + h) : (Hq + kvh)) * D + g;
    }
    return (Hq + Hkv + kvh) * D + (item - (G + 1) * 8) * 8;
  };
  if (fused) {
    if (tid < (G + 1) * 8) {
      const int pp = min(len - 1, rp.max_pos - 1), g = (tid & 7) * 8;
      const float* cr = rp.cos_t + (int64_t)pp * (D / 2) + g;
      const float* sr = rp.sin_t + (int64_t)pp * (D / 2) + g;
      csv[0] = *reinterpret_cast<const f32x4*>(cr);
      csv[1] = *reinterpret_cast<const f32x4*>(cr + 4);
      csv[2] = *reinterpret_cast<const f32x4*>(sr);
      csv[3] = *reinterpret_cast<const f32x4*>(sr + 4);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pr = tid + 256 * k;
      if (pr < NI * nS) {
        const int item = pr % NI, sl = pr / NI, col = rp_col(item);
        const bool rot = item < (G + 1) * 8;
        if (rp.xp) {
          const float* src = rp.xp + (int64_t)sl * rp.slab + (int64_t)b * ncol + col;
          rv[k][0] = *reinterpret_cast<const f32x4*>(src);
          rv[k][1] = *reinterpret_cast<const f32x4*>(src + 4);
          rv[k][2] = rot ? *reinterpret_cast<const f32x4*>(src + 64) : f32x4{0.f, 0.f, 0.f, 0.f};
          rv[k][3] = rot ? *reinterpret_cast<const f32x4*>(src + 68) : f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
          const bf16_t* src = rp.qkv + (int64_t)b * ncol + col;
          const u16x8 x1 = *reinterpret_cast<const u16x8*>(src);
          const u16x8 x2 = rot ? *reinterpret_cast<const u16x8*>(src + 64) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            rv[k][0][j] = bf2f(x1[j]);
            rv[k][1][j] = bf2f(x1[4 + j]);
            rv[k][2][j] = bf2f(x2[j]);
            rv[k][3][j] = bf2f(x2[4 + j]);
          }
        }
      }
    }
  }
  const int pid0 = tid < npg ? btb[tid] : 0;   // issued before any K/V load (vmcnt is in order)
  u16x8 qv[4];
  if (w == 0 && !fused) {
    const int hq = kvh * G + (l15 < G ? l15 : 0);
    const bf16_t* qp = q + ((int64_t)b * Hq + hq) * D + 32 * lg;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qv[ks] = *reinterpret_cast<const u16x8*>(qp + 8 * ks);
  }

  const int64_t head_off = (int64_t)kvh * page_size * D;
  const int64_t page_stride = (int64_t)Hkv * page_size * D;
  // Every token a wave reads for one 16-token tile lies in ONE page (page_size >= 16,
  // tiles 16-aligned; a tile wholly past `end` reads token end - 1 only), so each
  // tile needs one page lookup and 32-bit in-page offsets.
  auto tile_lds = [&](int base) -> int64_t {
    const int t0 = min(base, end - 1);
    return (int64_t)pg_lds[(t0 >> log2_page) - page0] * page_stride + head_off;
  };
  auto tile_bt = [&](int base) -> int64_t {
    const int t0 = min(base, end - 1);
    return (int64_t)btb[(t0 >> log2_page) - page0] * page_stride + head_off;
  };
  // Branch-free chunk load: rows past `end` are clamped duplicates (masked later).
  // K and V halves separately: a buffer's K registers are free as soon as the chunk's
  // S = K Q^T MFMAs have read them, so the next-but-one chunk's K is requested there,
  // a whole softmax + P.V earlier than its V.
  auto load_k = [&](KVRegs<KV, NT>& r, int c, auto tile_base) {
    const int base = start + c * CH + w * TW;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      const int tok = min(base + 16 * i + l15, end - 1);
      const int t16 = tok & 15;
      // tile of `tok`: its 16-token-aligned row, then (lg*16 + t16)*8 inside each ks block
      const KV* p = kc + tile_base(base + 16 * i) + ((tok & (page_size - 1)) - t16) * D + (lg * 16 + t16) * 8;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) r.k[i][ks] = T::load(p + ks * 512);
    }
  };
  auto load_v = [&](KVRegs<KV, NT>& r, int c, auto tile_base) {
    const int base = start + c * CH + w * TW;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      const KV* pv = vc + tile_base(base + 16 * i) + 8 * l15;
#pragma unroll
      for (int it = 4 * i; it < 4 * i + 4; ++it)   // token 16i + 4lg + (it - 4i): the S group lg
        r.v[it] = T::load(pv + (min(base + 16 * i + 4 * lg + (it - 4 * i), end - 1) & (page_size - 1)) * D);
    }
  };
  // Double-buffered stream over the chunks: the next chunk's loads are always in
  // flight while the current one is consumed, and the consume of chunk c requests
  // chunk c + 2 into the registers it frees. Loads past the last chunk re-read the
  // last chunk (branch-free, L2 hits) so hipcc's wait counts stay exact.
  KVRegs<KV, NT> ra, rb;
  load_k(ra, 0, tile_bt);
  load_v(ra, 0, tile_bt);
  load_k(rb, min(1, nch - 1), tile_bt);
  load_v(rb, min(1, nch - 1), tile_bt);
  if (tid < npg) pg_lds[tid] = pid0;
  for (int i = tid + 256; i < npg; i += 256) pg_lds[i] = btb[i];   // > 256 pages: rare
  // q as the MFMA B operand (column = head, zero past G), staged once in LDS and read per
  // k-step (16 VGPRs fewer per lane than q in registers)
  if (fused) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pr = tid + 256 * k;
      if (pr < NI * nS) {
        float* dst = rp_part + ((pr % NI) * kRopeMaxS + pr / NI) * 16;
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4*>(dst + 4 * j) = rv[k][j];
      }
    }
    if (l15 >= G && w == 0) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) q_lds[ks][lane] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  } else if (w == 0) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) q_lds[ks][lane] = l15 < G ? qv[ks] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  __syncthreads();
  if (fused) {
    // Fused RoPE, phase 2: one thread per item sums its slabs in order (+ bias), rounds
    // to bf16 and rotates (neox form) exactly as rope_kv does; q goes to the MFMA operand,
    // the new token's k / v to LDS (its attention term is merged after the stream, its
    // cache store issued at the very end: no store -> load hazard inside the kernel)
    if (tid < NI) {
      const int item = tid, col = rp_col(item);
      const bool rot = item < (G + 1) * 8;
      float x1[8], x2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x1[j] = x2[j] = 0.f;
      for (int sl = 0; sl < nS; ++sl) {
        const f32x4* src = reinterpret_cast<const f32x4*>(rp_part + (item * kRopeMaxS + sl) * 16);
        const f32x4 p0 = src[0], p1 = src[1], p2 = src[2], p3 = src[3];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x1[j] += p0[j];
          x1[4 + j] += p1[j];
          x2[j] += p2[j];
          x2[4 + j] += p3[j];
        }
      }
      if (rp.bias) {
        const u16x8 b1 = *reinterpret_cast<const u16x8*>(rp.bias + col);
        const u16x8 b2 = rot ? *reinterpret_cast<const u16x8*>(rp.bias + col + 64) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          x1[j] += bf2f(b1[j]);
          x2[j] += bf2f(b2[j]);
        }
      }
      if (rot) {
        const int h = item >> 3, g = (item & 7) * 8;
        u16x8 o1, o2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float c = csv[j >> 2][j & 3], sn = csv[2 + (j >> 2)][j & 3];
          const float a = bf2f(f2bf(x1[j])), bb = bf2f(f2bf(x2[j]));
          o1[j] = f2bf(a * c - bb * sn);
          o2[j] = f2bf(bb * c + a * sn);
        }
        if (h < G) {
          q_lds[(g & 31) >> 3][h + 16 * (g >> 5)] = o1;
          q_lds[(g & 31) >> 3][h + 16 * (2 + (g >> 5))] = o2;
        } else {
          kv_new[0][g >> 3] = o1;
          kv_new[0][8 + (g >> 3)] = o2;
        }
      } else {
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(x1[j]);
        kv_new[1][item - (G + 1) * 8] = o;
      }
    }
    __syncthreads();
    if (writer && tid >= 64 && tid < 96) {   // the new token into the cache, for the next steps:
      // issued here (wave 1; nothing in this kernel reads it) instead of delaying the end
      const int ti = tid - 64, pos_new = len - 1;
      const int64_t page = block_tables[(int64_t)b * max_pages + (pos_new >> log2_page)];
      const int off = pos_new & (page_size - 1), t16 = off & 15;
      const int64_t row = page * page_stride + head_off + (int64_t)off * D;
      if (ti < 16) {   // tiled K: [16-token tile][ks][lg][token][8 dims], dim d = 32 lg + 8 ks + j
        const int d = 8 * ti;
        cache_put8(const_cast<KV*>(kc) + row - (int64_t)t16 * D + ((((d & 31) >> 3) * 4 + (d >> 5)) * 16 + t16) * 8,
                   kv_new[0][ti], k_inv);
      } else {
        cache_put8(const_cast<KV*>(vc) + row + 8 * (ti - 16), kv_new[1][ti - 16], v_inv);
      }
    }
  }

  // Online softmax per (head, token group): lane (l15, lg) of the S = K Q^T tile holds head
  // l15 of tokens 4lg..4lg+3 of every 16-token tile, and the P.V lanes (dims 8 l15.., lg)
  // accumulate exactly those tokens, so each token group keeps its own running max / sum
  // and a chunk needs no cross-lane reduction at all (the rescale factors ride the P tile
  // through LDS); the 4 groups are merged once, after the stream.
  float m_run = -1e30f, l_run = 0.f;  // finite start: no inf - inf
  float acc[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[h][j] = 0.f;
  float* pwv = pw[w];

  // consume chunk c from r, refilling r with chunk `nc` (K after the MFMAs, V at the end)
  auto consume = [&](KVRegs<KV, NT>& r, int c, int nc) {
    const int base = start + c * CH + w * TW;
    float sc[NT][4];
    float m_new = m_run;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, T::to_bf16(r.k[i][ks])),
                                                  __builtin_bit_cast(bf16x8_t, q_lds[ks][lane]), a, 0, 0, 0);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int tok = base + 16 * i + 4 * lg + rr;
        sc[i][rr] = (tok < end_s) ? a[rr] * scale_log2 : -INFINITY;
        m_new = fmaxf(m_new, sc[i][rr]);
      }
    }
    load_k(r, nc, tile_lds);
    const float alpha = exp2f(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float p = exp2f(sc[i][rr] - m_new);
        psum += p;
        if (l15 < G) pwv[(16 * i + 4 * lg + rr) * GP + l15] = p;
      }
    l_run = l_run * alpha + psum;
    m_run = m_new;
    if (l15 < G) pwv[TW * GP + lg * GP + l15] = alpha;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    auto row4 = [&](const float* src, float (&dst)[G]) {   // G floats of one LDS row
      if constexpr (G % 4 == 0) {
#pragma unroll
        for (int h4 = 0; h4 < G; h4 += 4) {
          const f32x4 v4 = *reinterpret_cast<const f32x4*>(src + h4);
          dst[h4] = v4[0]; dst[h4 + 1] = v4[1]; dst[h4 + 2] = v4[2]; dst[h4 + 3] = v4[3];
        }
      } else {
#pragma unroll
        for (int h = 0; h < G; ++h) dst[h] = src[h];
      }
    };
    float al[G];
    row4(pwv + TW * GP + lg * GP, al);
#pragma unroll
    for (int h = 0; h < G; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[h][j] *= al[h];
#pragma unroll
    for (int it = 0; it < 4 * NT; ++it) {
      const int t = 16 * (it >> 2) + 4 * lg + (it & 3);
      float p[G];
      row4(pwv + t * GP, p);
      float vv[8];
      T::to_f32(r.v[it], vv);
#pragma unroll
      for (int h = 0; h < G; ++h)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[h][j] += p[h] * vv[j];
    }
    load_v(r, nc, tile_lds);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  for (int c = 0; c < nch; c += 2) {
    consume(ra, c, min(c + 2, nch - 1));
    if (c + 1 < nch) consume(rb, c + 1, min(c + 3, nch - 1));
  }

  // ---- merge the 4 token groups of each wave, then the 4 waves ----
  {
    float M = m_run;   // lane (head l15, group lg)
    M = fmaxf(M, __shfl_xor(M, 16, kWave));
    M = fmaxf(M, __shfl_xor(M, 32, kWave));
    const float f = exp2f(m_run - M);
    float L = l_run * f;
    L += __shfl_xor(L, 16, kWave);
    L += __shfl_xor(L, 32, kWave);
    m_run = M;
    l_run = L;
    if (l15 < G) pwv[TW * GP + lg * GP + l15] = f;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const float fg = pwv[TW * GP + lg * GP + h];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[h][j] *= fg;
    }
  }
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
      float* rr = &red[w][h][8 * l15];
      *reinterpret_cast<f32x4*>(rr) = f32x4{acc[h][0], acc[h][1], acc[h][2], acc[h][3]};
      *reinterpret_cast<f32x4*>(rr + 4) = f32x4{acc[h][4], acc[h][5], acc[h][6], acc[h][7]};
    }
    if (l15 < G) {
      mls[w][l15][0] = m_run;
      mls[w][l15][1] = l_run;
    }
  }
  if (writer && w == 0) {   // the new token's scores: q . k over 128 dims, 16 lanes per head
#pragma unroll
    for (int h0 = 0; h0 < G; h0 += 4) {
      const int h = h0 + lg;
      float sdot = 0.f;
      if (h < G) {
        const u16x8 qv8 = q_lds[l15 & 3][h + 16 * (l15 >> 2)];
        const u16x8 kv8 = kv_new[0][l15];
#pragma unroll
        for (int t = 0; t < 8; ++t) sdot += bf2f(qv8[t]) * kv_value<KV>(kv8[t], k_inv);
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) sdot += __shfl_xor(sdot, o, 16);
      if (h < G && l15 == 0) s_new[h] = sdot * scale_log2;
    }
  }
  __syncthreads();
  for (int e = tid; e < G * D; e += 256) {
    const int h = e / D, d = e % D;
    float M = mls[0][h][0];
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) M = fmaxf(M, mls[ww][h][0]);
    if (writer) M = fmaxf(M, s_new[h]);
    float o = 0.f, L = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float f = exp2f(mls[ww][h][0] - M);
      o += f * red[ww][h][d];
      L += f * mls[ww][h][1];
    }
    if (writer) {   // + the new token (p = exp2(s - M), its v as the cache holds it)
      const float f = exp2f(s_new[h] - M);
      o += f * kv_value<KV>(kv_new[1][d >> 3][d & 7], v_inv);
      L += f;
    }
    o *= v_scale;
    const int hq = kvh * G + h;
    if (ns_b == 1) {  // whole context in this workgroup: final output, no combine
      out[((int64_t)b * Hq + hq) * D + d] = f2bf(L > 0.f ? o / L : 0.f);
    } else {
      o_part[(((int64_t)b * Hq + hq) * num_splits + s) * D + d] = o;
      if (d == 0) {
        float* ml = ml_part + (((int64_t)b * Hq + hq) * num_splits + s) * 2;
        ml[0] = M;
        ml[1] = L;
      }
    }
  }
}

// Combine the per-split partials of split sequences: grid (B*Hq), D threads.
__global__ void attn_decode_combine_kernel(const float* __restrict__ o_part, const float* __restrict__ ml_part,
                                           const int* __restrict__ seq_lens, bf16_t* __restrict__ out, int Hq,
                                           int num_splits, int max_tokens, int chunk) {
  constexpr int D = 128;
  const int bh = blockIdx.x, b = bh / Hq, d = threadIdx.x;
  const int len = min(seq_lens[b], max_tokens);
  if (len <= 0) return;  // zeroed by the attention kernel
  const int per = split_len(len, num_splits, chunk);
  const int ns = (len + per - 1) / per;
  if (ns == 1) return;  // written directly by the attention kernel
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

// Split combine fused with the o-projection's input quantization (fp8 W8A8 models): one
// 1024-thread block per token row of Hq x 128 outputs. Each element is the bf16 of the
// split-KV combine (or the attention kernel's own bf16 output for a row of one split),
// exactly as attn_decode_combine_kernel writes it; the row is then quantized per token
// to e4m3fn exactly as quantize_fp8_rows does (amax of the bf16 values / 448), so the
// separate quantization pass over `out` disappears.
template <int MAXV>
__global__ void __launch_bounds__(1024) attn_decode_combine_q8_kernel(
    const float* __restrict__ o_part, const float* __restrict__ ml_part, const int* __restrict__ seq_lens,
    const bf16_t* __restrict__ out, uint8_t* __restrict__ q8, float* __restrict__ sx, int Hq, int num_splits,
    int max_tokens, int chunk) {
  constexpr int D = 128;
  constexpr int NT = 1024;
  __shared__ float red[NT / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int len = min(seq_lens[b], max_tokens);
  const int per = len > 0 ? split_len(len, num_splits, chunk) : 1;
  const int ns = len > 0 ? (len + per - 1) / per : 1;
  const int n = Hq * D;
  float v[MAXV];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int e = tid + i * NT;
    v[i] = 0.f;
    if (e < n) {
      const int h = e / D, d = e % D;
      const int64_t bh = (int64_t)b * Hq + h;
      if (len <= 0 || ns == 1 || num_splits == 1) {
        v[i] = bf2f(out[bh * D + d]);
      } else {
        const float* ml = ml_part + bh * num_splits * 2;
        float M = -INFINITY;
        for (int s = 0; s < ns; ++s) M = fmaxf(M, ml[2 * s]);
        float L = 0.f, o = 0.f;
        for (int s = 0; s < ns; ++s) {
          const float wgt = exp2f(ml[2 * s] - M);
          L += wgt * ml[2 * s + 1];
          o += wgt * o_part[(bh * num_splits + s) * D + d];
        }
        v[i] = bf2f(f2bf(L > 0.f ? o / L : 0.f));
      }
      amax = fmaxf(amax, fabsf(v[i]));
    }
  }
  amax = wave_max(amax);
  if ((tid & 63) == 0) red[tid >> 6] = amax;
  __syncthreads();
  amax = 0.f;
#pragma unroll
  for (int k = 0; k < NT / 64; ++k) amax = fmaxf(amax, red[k]);
  const float sc = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / sc;
  if (tid == 0) sx[b] = sc;
  uint8_t* qr = q8 + (int64_t)b * n;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int e = tid + i * NT;
    if (e < n) {
      const int pk = __builtin_amdgcn_cvt_pk_fp8_f32(v[i] * inv, 0.f, 0, false);
      qr[e] = static_cast<uint8_t>(pk & 0xff);
    }
  }
}

int attn_decode(const bf16_t* q, const void* k_cache, const void* v_cache, bool fp8, float k_scale, float v_scale,
                const int* block_tables, const int* seq_lens, bf16_t* out, float* o_part, float* ml_part, int B,
                int Hq, int Hkv, int head_dim, int page_size, int max_pages, int num_splits, float scale, int variant,
                hipStream_t stream, uint8_t* q8, float* sx, const DecodeRope* rope) {
  if (B == 0) return 0;
  DecodeRope rp{};
  if (rope != nullptr) {
    if (rope->cos_t == nullptr || rope->sin_t == nullptr || (rope->qkv == nullptr && rope->xp == nullptr)) return -7;
    if (rope->xp != nullptr && (rope->S < 1 || rope->S > kRopeMaxS)) return -8;
    if ((Hq / Hkv + 1) * 8 + 16 > 256 || ((Hq / Hkv + 1) * 8 + 16) * (rope->xp ? rope->S : 1) > 512) return -9;
    rp = *rope;
  }
  if (head_dim != 128) return -1;
  if (page_size < 16 || (page_size & (page_size - 1)) != 0) return -2;
  if (max_pages > kMaxPagesLds) return -4;
  if (num_splits < 1) return -5;
  int log2p = 0;
  while ((1 << log2p) < page_size) ++log2p;
  const int G = Hq / Hkv;
  const float scale_log2 = scale * k_scale * 1.4426950408889634f;
  // variant bits 0-1: 0 = default (NT = 1: 16 tokens per wave per chunk, 162 VGPRs at
  // G = 4 -> 3 workgroups/CU); 2 = NT = 2 (32 tokens per wave, 2 workgroups/CU;
  // bf16: 244 VGPRs, measured 3-5 % slower at B = 256). G > 4 stays NT = 1.
  // Bit 2: the old dispatch order (below).
  int chunk = 0;
  dim3 grid(B * num_splits, Hkv, 1);
#define OAMD_DEC(GG, NTT, KVT_)                                                                           \
  do {                                                                                                    \
    attn_decode_kernel<GG, NTT, KVT_><<<grid, 256, 0, stream>>>(                                         \
        q, static_cast<const KVT_*>(k_cache), static_cast<const KVT_*>(v_cache), block_tables, seq_lens, \
        out, o_part, ml_part, Hkv, page_size, log2p, max_pages, num_splits, scale_log2, v_scale, hm, rp,  \
        1.f / k_scale, 1.f / v_scale);                                                                   \
    chunk = 64 * NTT;                                                                                     \
  } while (0)
  const bool nt2 = (variant & 3) == 2;
  // kv-heads of one sequence dispatched back to back (default; tools/bench_attn.py at B = 256:
  // -0.5..-1 % vs one kv-head across all sequences first, which variant bit 2 selects)
  const int hm = (variant & 4) ? 0 : 1;
  if (fp8) {
    switch (G) {
      case 1: if (nt2) OAMD_DEC(1, 2, uint8_t); else OAMD_DEC(1, 1, uint8_t); break;
      case 2: if (nt2) OAMD_DEC(2, 2, uint8_t); else OAMD_DEC(2, 1, uint8_t); break;
      case 4: if (nt2) OAMD_DEC(4, 2, uint8_t); else OAMD_DEC(4, 1, uint8_t); break;
      case 3: OAMD_DEC(3, 1, uint8_t); break;
      case 5: OAMD_DEC(5, 1, uint8_t); break;
      case 6: OAMD_DEC(6, 1, uint8_t); break;
      case 7: OAMD_DEC(7, 1, uint8_t); break;
      case 8: OAMD_DEC(8, 1, uint8_t); break;
      default: return -3;
    }
  } else {
    switch (G) {
      case 1: if (nt2) OAMD_DEC(1, 2, bf16_t); else OAMD_DEC(1, 1, bf16_t); break;
      case 2: if (nt2) OAMD_DEC(2, 2, bf16_t); else OAMD_DEC(2, 1, bf16_t); break;
      case 4: if (nt2) OAMD_DEC(4, 2, bf16_t); else OAMD_DEC(4, 1, bf16_t); break;
      // groups of Llama-3.2-3B (24/8), Qwen2.5-32B (40/8), Qwen2.5-7B (28/4)
      case 3: OAMD_DEC(3, 1, bf16_t); break;
      case 5: OAMD_DEC(5, 1, bf16_t); break;
      case 6: OAMD_DEC(6, 1, bf16_t); break;
      case 7: OAMD_DEC(7, 1, bf16_t); break;
      case 8: OAMD_DEC(8, 1, bf16_t); break;
      default: return -3;
    }
  }
#undef OAMD_DEC
  OAMD_LAUNCH_CHECK();
  if (q8 != nullptr) {   // combine (if split) + per-token e4m3fn rows for the fp8 o-projection
    const int n = Hq * 128;
    if (n <= 1024)
      attn_decode_combine_q8_kernel<1><<<B, 1024, 0, stream>>>(o_part, ml_part, seq_lens, out, q8, sx, Hq, num_splits,
                                                               max_pages * page_size, chunk);
    else if (n <= 4096)
      attn_decode_combine_q8_kernel<4><<<B, 1024, 0, stream>>>(o_part, ml_part, seq_lens, out, q8, sx, Hq,
                                                               num_splits, max_pages * page_size, chunk);
    else if (n <= 8192)
      attn_decode_combine_q8_kernel<8><<<B, 1024, 0, stream>>>(o_part, ml_part, seq_lens, out, q8, sx, Hq,
                                                               num_splits, max_pages * page_size, chunk);
    else
      return -6;
    OAMD_LAUNCH_CHECK();
    return 0;
  }
  if (num_splits > 1) {
    attn_decode_combine_kernel<<<B * Hq, 128, 0, stream>>>(o_part, ml_part, seq_lens, out, Hq, num_splits,
                                                           max_pages * page_size, chunk);
    OAMD_LAUNCH_CHECK();
  }
  return 0;
}

}  // namespace oamd
