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

// Token range of split s of a sequence of `len` tokens cut into at most
// `num_splits` pieces of a multiple of `chunk` tokens. Shared with the combine
// kernel so both agree on how many splits a sequence really has.
__device__ __forceinline__ int split_len(int len, int num_splits, int chunk) {
  const int per = (len + num_splits - 1) / num_splits;
  return (per + chunk - 1) / chunk * chunk;
}

// 4 bf16 values (packed) -> 4 cache elements (bf16: as is; fp8: e4m3(x * inv), saturated)
template <typename KV>
struct Put4;
template <>
struct Put4<bf16_t> {
  static __device__ __forceinline__ void put(bf16_t* dst, uint2 v, float) { *reinterpret_cast<uint2*>(dst) = v; }
};
template <>
struct Put4<uint8_t> {
  static __device__ __forceinline__ void put(uint8_t* dst, uint2 v, float inv) {
    auto f = [&](uint32_t w, bool hi) {
      return fminf(fmaxf(__uint_as_float(hi ? (w & 0xffff0000u) : (w << 16)) * inv, -448.f), 448.f);
    };
    int o = 0;
    o = __builtin_amdgcn_cvt_pk_fp8_f32(f(v.x, false), f(v.x, true), o, false);
    o = __builtin_amdgcn_cvt_pk_fp8_f32(f(v.y, false), f(v.y, true), o, true);
    *reinterpret_cast<int*>(dst) = o;
  }
};

// Row b, columns col..col+3 of the QKV projection as rope_kv sees them: bf16(sum of the S
// fp32 slabs in slab order (+ bias)), or the bf16 row (+ bias, then rounded). SC: slab
// count known at compile time (1, 4, 8: every slab load issued before the first add) or
// 9 (runtime S).
template <int SC>
__device__ __forceinline__ f32x4 qkv4(const DecRope& r, int b, int ncol, int col) {
  f32x4 a;
  if (r.xp != nullptr) {
    const float* p = r.xp + (int64_t)b * ncol + col;
    a = *reinterpret_cast<const f32x4*>(p);
    if constexpr (SC > 1 && SC <= 8) {
      f32x4 t[SC - 1];
#pragma unroll
      for (int k = 1; k < SC; ++k) t[k - 1] = *reinterpret_cast<const f32x4*>(p + k * r.slab);
#pragma unroll
      for (int k = 1; k < SC; ++k) a += t[k - 1];
    } else if constexpr (SC == 9) {
      for (int k = 1; k < r.S; ++k) a += *reinterpret_cast<const f32x4*>(p + k * r.slab);
    }
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(r.row + (int64_t)b * r.row_stride + col);
    a = f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
              __uint_as_float(u.y & 0xffff0000u)};
  }
  if (r.bias != nullptr) {
    const uint2 u = *reinterpret_cast<const uint2*>(r.bias + col);
    a += f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = bf2f(f2bf(a[j]));
  return a;
}

// rotate-half RoPE of 4 (x1, x2 = x1's dims + 64) pairs -> packed bf16 (rope_pair: rope_kv's numerics)
__device__ __forceinline__ void rope4(const f32x4& x1, const f32x4& x2, const float* cr, const float* sr, uint2& o1,
                                      uint2& o2) {
  const f32x4 c = *reinterpret_cast<const f32x4*>(cr), sn = *reinterpret_cast<const f32x4*>(sr);
  float r1[4], r2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) rope_pair(x1[j], x2[j], c[j], sn[j], r1[j], r2[j]);
  o1 = make_uint2(pack_bf2(r1[0], r1[1]), pack_bf2(r1[2], r1[3]));
  o2 = make_uint2(pack_bf2(r2[0], r2[1]), pack_bf2(r2[2], r2[3]));
}

template <typename KV, int NT>
struct KVRegs {
  typename KVT<KV>::frag k[NT][4];   // K tile i: token 16i + l15, dims 32*lg + 8*ks
  typename KVT<KV>::frag v[4 * NT];  // token 4*it + lg, dims 8*l15
};

// FR (fused RoPE, DecRope): 0 = q comes rotated from rope_kv; else q is rotated here from
// the QKV projection (FR = its slab class for qkv4: 1, 4, 8, 9) and the workgroup whose
// split ends the sequence writes the decode token's K / V into the cache first.
template <int G, int NT, typename KV = bf16_t, int FR = 0>
__global__ void __launch_bounds__(256, (NT == 1 && G <= 4) ? 3 : 2)
    attn_decode_kernel(const bf16_t* __restrict__ q, const KV* __restrict__ kc, const KV* __restrict__ vc,
                       const int* __restrict__ block_tables, const int* __restrict__ seq_lens,
                       bf16_t* __restrict__ out, float* __restrict__ o_part, float* __restrict__ ml_part, int Hkv,
                       int page_size, int log2_page, int max_pages, int num_splits, float scale_log2,
                       float v_scale, int head_minor, DecRope rp) {
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

  // Page ids of the split -> LDS: the steady-state data loads depend only on LDS
  // (lgkmcnt), never on a global load that would share vmcnt with them. The first
  // two chunks do not wait for that: their page ids come straight from the block
  // table (wave-uniform scalar loads), so their K/V requests leave before the LDS
  // page table and q are even written (one dependent latency less per workgroup).
  const int page0 = start >> log2_page;
  const int npg = ((end - 1) >> log2_page) - page0 + 1;
  const int* btb = block_tables + (int64_t)b * max_pages + page0;
  const int pid0 = tid < npg ? btb[tid] : 0;   // issued before any K/V load (vmcnt is in order)
  u16x8 qv[4];
  if (FR == 0 && w == 0) {
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
  bool kv_new = false;
  if constexpr (FR == 0) {
    if (w == 0) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) q_lds[ks][lane] = l15 < G ? qv[ks] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  } else {
    // rope_kv's decode work, while the first two chunks are in flight. q: thread (head h,
    // quad) rotates dims 4 quad.. and 4 quad + 64.. of head kvh*G + h into its q_lds slots
    // (dim d of head h: q_lds[(d % 32) / 8][16 (d / 32) + h], element d % 8)
    const int ncol = (Hq + 2 * Hkv) * D;
    int64_t p = rp.pos[b];
    p = p < 0 ? 0 : (p >= rp.max_pos ? rp.max_pos - 1 : p);
    const float* cr = rp.cos_t + p * (D / 2);
    const float* sr = rp.sin_t + p * (D / 2);
    uint16_t* ql = reinterpret_cast<uint16_t*>(&q_lds[0][0]);
    auto qidx = [&](int d, int h) { return ((((d & 31) >> 3) * 64 + (d >> 5) * 16 + h) << 3) + (d & 7); };
    if ((lane & 15) >= G) q_lds[w][lane] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};   // 4 waves x 64 = every slot
    if (tid < G * 16) {
      const int h = tid >> 4, d0 = (tid & 15) * 4;
      const int col = (kvh * G + h) * D + d0;
      const f32x4 x1 = qkv4<FR>(rp, b, ncol, col), x2 = qkv4<FR>(rp, b, ncol, col + D / 2);
      uint2 o1, o2;
      rope4(x1, x2, cr + d0, sr + d0, o1, o2);
      *reinterpret_cast<uint2*>(ql + qidx(d0, h)) = o1;
      *reinterpret_cast<uint2*>(ql + qidx(d0 + D / 2, h)) = o2;
    }
    // the decode token (position len - 1) belongs to the split that ends the sequence: its
    // workgroup writes the token's rotated K and its V for head kvh (wave 2: lanes 0-15 K
    // pairs, 16-47 V quads) and drains the stores before the barrier below
    const int64_t slot = rp.slots[b];
    kv_new = end == len && slot >= 0;
    if (kv_new && w == 2 && lane < 48) {
      const int64_t page = slot >> log2_page, off = slot & (page_size - 1);
      KV* kdst = const_cast<KV*>(kc) + (page * Hkv * page_size + (off & ~15)) * D + (int64_t)kvh * page_size * D;
      KV* vdst = const_cast<KV*>(vc) + (page * Hkv * page_size + off) * D + (int64_t)kvh * page_size * D;
      const int t16 = static_cast<int>(off & 15);
      // tiled K (rope_kv): [ks][lg][token][8 dims], d = 32 lg + 8 ks + j
      auto kofs = [&](int d) { return ((((d & 31) >> 3) * 4 + (d >> 5)) * 16 + t16) * 8 + (d & 7); };
      if (lane < 16) {
        const int d0 = lane * 4, col = (Hq + kvh) * D + d0;
        const f32x4 x1 = qkv4<FR>(rp, b, ncol, col), x2 = qkv4<FR>(rp, b, ncol, col + D / 2);
        uint2 o1, o2;
        rope4(x1, x2, cr + d0, sr + d0, o1, o2);
        Put4<KV>::put(kdst + kofs(d0), o1, rp.k_inv);
        Put4<KV>::put(kdst + kofs(d0 + D / 2), o2, rp.k_inv);
      } else {
        const int d0 = (lane - 16) * 4, col = (Hq + Hkv + kvh) * D + d0;
        const f32x4 v = qkv4<FR>(rp, b, ncol, col);
        Put4<KV>::put(vdst + d0, make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])), rp.v_inv);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if constexpr (FR != 0) {
    // the token's chunk (or a chunk of clamped copies of it) already requested above read the
    // slot before it was written: request it again, now that the stores have landed
    if (kv_new && nch <= 2) {
      if (nch == 1) {
        load_k(ra, 0, tile_lds);
        load_v(ra, 0, tile_lds);
      } else {
        load_k(rb, 1, tile_lds);
        load_v(rb, 1, tile_lds);
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
        sc[i][rr] = (tok < end) ? a[rr] * scale_log2 : -INFINITY;
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
  __syncthreads();
  for (int e = tid; e < G * D; e += 256) {
    const int h = e / D, d = e % D;
    float M = mls[0][h][0];
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) M = fmaxf(M, mls[ww][h][0]);
    float o = 0.f, L = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float f = exp2f(mls[ww][h][0] - M);
      o += f * red[ww][h][d];
      L += f * mls[ww][h][1];
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
  constexpr int kMaxStats = 2048;   // Hq x splits per row staged in LDS (host-checked)
  __shared__ float red[NT / 64];
  // per (head, split): the split's running max, then its combine weight; per head: the row sum.
  // Loaded by all threads at once (one round trip) instead of a dependent load per split in
  // every element's loop (two chains of `splits` L2 round trips per element).
  __shared__ float wst[kMaxStats];
  __shared__ float lst[kMaxStats];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int len = min(seq_lens[b], max_tokens);
  const int per = len > 0 ? split_len(len, num_splits, chunk) : 1;
  const int ns = len > 0 ? (len + per - 1) / per : 1;
  const bool split = !(len <= 0 || ns == 1 || num_splits == 1);
  const int n = Hq * D;
  if (split) {
    for (int i = tid; i < Hq * ns; i += NT) {
      const int h = i / ns, sp = i - h * ns;
      const float* ml = ml_part + (((int64_t)b * Hq + h) * num_splits + sp) * 2;
      wst[i] = ml[0];
      lst[i] = ml[1];
    }
    __syncthreads();
    if (tid < Hq) {   // the same order and arithmetic as attn_decode_combine_kernel
      float M = -INFINITY;
      for (int sp = 0; sp < ns; ++sp) M = fmaxf(M, wst[tid * ns + sp]);
      float L = 0.f;
      for (int sp = 0; sp < ns; ++sp) {
        const float wgt = exp2f(wst[tid * ns + sp] - M);
        L += wgt * lst[tid * ns + sp];
        wst[tid * ns + sp] = wgt;
      }
      lst[tid * ns] = L;
    }
    __syncthreads();
  }
  float v[MAXV];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int e = tid + i * NT;
    v[i] = 0.f;
    if (e < n) {
      const int h = e / D, d = e % D;
      const int64_t bh = (int64_t)b * Hq + h;
      if (!split) {
        v[i] = bf2f(out[bh * D + d]);
      } else {
        const float* op = o_part + bh * num_splits * D + d;
        const float* wg = wst + h * ns;
        float o = 0.f;
        int sp = 0;
        for (; sp + 4 <= ns; sp += 4) {   // four independent loads in flight
          const float x0 = op[(int64_t)sp * D], x1 = op[(int64_t)(sp + 1) * D];
          const float x2 = op[(int64_t)(sp + 2) * D], x3 = op[(int64_t)(sp + 3) * D];
          o += wg[sp] * x0;
          o += wg[sp + 1] * x1;
          o += wg[sp + 2] * x2;
          o += wg[sp + 3] * x3;
        }
        for (; sp < ns; ++sp) o += wg[sp] * op[(int64_t)sp * D];
        const float L = lst[h * ns];
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
                hipStream_t stream, uint8_t* q8, float* sx, const DecRope* rope) {
  if (B == 0) return 0;
  if (head_dim != 128) return -1;
  if (page_size < 16 || (page_size & (page_size - 1)) != 0) return -2;
  if (max_pages > kMaxPagesLds) return -4;
  if (num_splits < 1) return -5;
  if (rope != nullptr && (rope->pos == nullptr || rope->slots == nullptr || rope->cos_t == nullptr ||
                          rope->sin_t == nullptr || rope->max_pos < 1 ||
                          (rope->xp == nullptr ? rope->row == nullptr : rope->S < 1)))
    return -8;
  // validate every launch of this call before the first one: nothing is enqueued on a bad shape
  if (q8 != nullptr && Hq * 128 > 8192) return -6;
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
  DecRope rp{};
  int fr = 0;
  if (rope != nullptr) {
    rp = *rope;
    fr = rp.xp == nullptr ? 1 : (rp.S == 1 || rp.S == 4 || rp.S == 8) ? rp.S : 9;
  }
#define OAMD_DEC_K(GG, NTT, KVT_, FRR)                                                                    \
  attn_decode_kernel<GG, NTT, KVT_, FRR><<<grid, 256, 0, stream>>>(                                       \
      q, static_cast<const KVT_*>(k_cache), static_cast<const KVT_*>(v_cache), block_tables, seq_lens,   \
      out, o_part, ml_part, Hkv, page_size, log2p, max_pages, num_splits, scale_log2, v_scale, hm, rp)
#define OAMD_DEC(GG, NTT, KVT_)                                                                           \
  do {                                                                                                    \
    if (fr == 0) {                                                                                        \
      OAMD_DEC_K(GG, NTT, KVT_, 0);                                                                       \
      chunk = 64 * NTT;                                                                                   \
    } else {   /* fused RoPE: the NT = 1 schedule */                                                     \
      switch (fr) {                                                                                       \
        case 1: OAMD_DEC_K(GG, 1, KVT_, 1); break;                                                        \
        case 4: OAMD_DEC_K(GG, 1, KVT_, 4); break;                                                        \
        case 8: OAMD_DEC_K(GG, 1, KVT_, 8); break;                                                        \
        default: OAMD_DEC_K(GG, 1, KVT_, 9); break;                                                       \
      }                                                                                                   \
      chunk = 64;                                                                                         \
    }                                                                                                     \
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
#undef OAMD_DEC_K
  OAMD_LAUNCH_CHECK();
  if (q8 != nullptr) {   // combine (if split) + per-token e4m3fn rows for the fp8 o-projection
    const int n = Hq * 128;
    int q8_splits = num_splits;
    if (num_splits > 1 && Hq * num_splits > 2048) {
      // more (head, split) statistics than attn_decode_combine_q8_kernel stages in LDS (e.g. a
      // 64-head model at 64 splits): combine into `out` with the plain kernel first, then
      // quantize those bf16 rows (num_splits = 1 makes the q8 kernel read `out`) -- the same
      // bf16 values, one extra pass over the row
      attn_decode_combine_kernel<<<B * Hq, 128, 0, stream>>>(o_part, ml_part, seq_lens, out, Hq, num_splits,
                                                             max_pages * page_size, chunk);
      OAMD_LAUNCH_CHECK();
      q8_splits = 1;
    }
    if (n <= 1024)
      attn_decode_combine_q8_kernel<1><<<B, 1024, 0, stream>>>(o_part, ml_part, seq_lens, out, q8, sx, Hq, q8_splits,
                                                               max_pages * page_size, chunk);
    else if (n <= 4096)
      attn_decode_combine_q8_kernel<4><<<B, 1024, 0, stream>>>(o_part, ml_part, seq_lens, out, q8, sx, Hq,
                                                               q8_splits, max_pages * page_size, chunk);
    else
      attn_decode_combine_q8_kernel<8><<<B, 1024, 0, stream>>>(o_part, ml_part, seq_lens, out, q8, sx, Hq,
                                                               q8_splits, max_pages * page_size, chunk);
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
