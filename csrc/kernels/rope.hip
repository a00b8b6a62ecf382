// Fused RoPE + paged KV-cache write.
//
// Input is the packed output of the fused QKV projection, one row per token:
//   qkv[t] = [ q(Hq*D) | k(Hkv*D) | v(Hkv*D) ]  (bf16)
// Rotary embedding (neox / rotate-half form, as HF Llama) is applied to q and
// k using a host-precomputed fp32 cos/sin table [max_pos, D/2] (no on-device
// trig: cdna_hip_programming.md App. B "Element-wise"). Outputs:
//   q_out  [T, Hq, D]            rotated q (always)
//   k_out/v_out [T, Hkv, D]      rotated k / copied v (optional, prefill path)
//   k_cache/v_cache [pages, Hkv, P, D] at slot_mapping[t] (optional; slot<0 skips);
//   K is stored in 16-token MFMA tiles (see attn_decode.hip), V row-major
// With an fp8 cache (OCP e4m3fn) K and V are stored as e4m3(bf16(x) / scale),
// saturated to +-448, 8 bytes per 8-element group (same layouts as bf16).
// An optional bf16 bias [(Hq + 2Hkv) D] (Qwen2's q/k/v projection bias) is added
// in fp32 before the one bf16 rounding of the split-K slab sum (HF numerics:
// bf16(x W^T + b)); on a bf16 qkv row it is added after that row's rounding.
#include "common.h"
#include "kernels.h"

namespace oamd {

// One 64-lane workgroup per (token, 64 work items): a token's (Hq + Hkv) x D/16
// rotation items and Hkv x D/8 copy items are spread over ceil(items / 64)
// workgroups, so a decode batch of 256 tokens is ~1.8k workgroups instead of 256
// (the split-K form, which sums S fp32 slabs per element, was latency-bound at
// one 256-thread workgroup per token: 7.8 us + a separate 5.5 us reduce kernel).
constexpr int kRopeItems = 64;

// 8 bf16 values -> the cache element type (bf16: as is; fp8: e4m3(x * inv_scale))
template <typename KV>
struct CacheStore;
template <>
struct CacheStore<bf16_t> {
  static __device__ __forceinline__ void put(bf16_t* dst, const u16x8& v, float) {
    *reinterpret_cast<u16x8*>(dst) = v;
  }
};
template <>
struct CacheStore<uint8_t> {
  static __device__ __forceinline__ void put(uint8_t* dst, const u16x8& v, float inv) {
    auto f = [&](int j) { return fminf(fmaxf(bf2f(v[j]) * inv, -448.f), 448.f); };
    int lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(f(0), f(1), lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(f(2), f(3), lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(f(4), f(5), hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(f(6), f(7), hi, true);
    *reinterpret_cast<uint2*>(dst) = uint2{(unsigned)lo, (unsigned)hi};
  }
};

// SC: compile-time split-K slab count (0: runtime S), so all S slab loads of a group
// are issued before the first add (a runtime-trip-count loop waited for each in turn).
template <int D, typename KV, int SC, int NI = kRopeItems>
__global__ void __launch_bounds__(NI) rope_kv_kernel(
    const bf16_t* __restrict__ qkv, int64_t qkv_stride, const int64_t* __restrict__ pos,
    const float* __restrict__ cos_t, const float* __restrict__ sin_t, int Hq, int Hkv,
    bf16_t* __restrict__ q_out, bf16_t* __restrict__ k_out, bf16_t* __restrict__ v_out,
    KV* __restrict__ k_cache, KV* __restrict__ v_cache,
    const int64_t* __restrict__ slots, int page_size, int64_t max_pos,
    const float* __restrict__ xp, int S, int64_t slab, const bf16_t* __restrict__ bias, float k_inv,
    float v_inv) {
  constexpr int HALF = D / 2;
  constexpr int GPH = HALF / 8;  // 8-element groups per half-head
  const int t = blockIdx.x;
  const bf16_t* row = qkv + t * qkv_stride;
  const int ncol = (Hq + 2 * Hkv) * D;
  // 8 consecutive qkv values of this row: from the bf16 row, or (xp set) the bf16
  // rounding of the sum of S fp32 split-K slabs of the QKV projection
  auto ld8 = [&](int col) -> u16x8 {
    if (!xp && !bias) return *reinterpret_cast<const u16x8*>(row + col);
    f32x4 lo, hi;
    if (xp) {
      const float* pr = xp + (int64_t)t * ncol + col;
      lo = *reinterpret_cast<const f32x4*>(pr);
      hi = *reinterpret_cast<const f32x4*>(pr + 4);
      if constexpr (SC > 1) {
        f32x4 pl[SC - 1], ph[SC - 1];
#pragma unroll
        for (int sp = 1; sp < SC; ++sp) {
          pl[sp - 1] = *reinterpret_cast<const f32x4*>(pr + sp * slab);
          ph[sp - 1] = *reinterpret_cast<const f32x4*>(pr + sp * slab + 4);
        }
#pragma unroll
        for (int sp = 1; sp < SC; ++sp) {
          lo += pl[sp - 1];
          hi += ph[sp - 1];
        }
      } else if constexpr (SC == 0) {
        for (int sp = 1; sp < S; ++sp) {
          lo += *reinterpret_cast<const f32x4*>(pr + sp * slab);
          hi += *reinterpret_cast<const f32x4*>(pr + sp * slab + 4);
        }
      }
    } else {
      const u16x8 r = *reinterpret_cast<const u16x8*>(row + col);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lo[j] = bf2f(r[j]);
        hi[j] = bf2f(r[4 + j]);
      }
    }
    if (bias) {
      const u16x8 bb = *reinterpret_cast<const u16x8*>(bias + col);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lo[j] += bf2f(bb[j]);
        hi[j] += bf2f(bb[4 + j]);
      }
    }
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = f2bf(lo[j]);
      o[4 + j] = f2bf(hi[j]);
    }
    return o;
  };
  int64_t p = pos[t];
  if (p < 0) p = 0;
  if (p >= max_pos) p = max_pos - 1;
  const float* cr = cos_t + p * HALF;
  const float* sr = sin_t + p * HALF;
  int64_t slot = slots ? slots[t] : -1;
  int64_t cache_base_k = -1, tile_base_k = -1;  // V row / K tile of this token (+ h*page_size*D)
  int t16 = 0;
  if (slot >= 0) {
    const int64_t page = slot / page_size, off = slot % page_size;
    cache_base_k = (page * Hkv * page_size + off) * D;
    tile_base_k = (page * Hkv * page_size + (off & ~15)) * D;
    t16 = static_cast<int>(off & 15);
  }
  const int rot_items = (Hq + Hkv) * GPH;
  const int copy_items = Hkv * (D / 8);
  {
    const int it = blockIdx.y * NI + threadIdx.x;
    if (it >= rot_items + copy_items) return;
    if (it < rot_items) {
      const int h = it / GPH, g = (it % GPH) * 8;
      const u16x8 x1 = ld8(h * D + g);
      const u16x8 x2 = ld8(h * D + HALF + g);
      const f32x4 c0 = *reinterpret_cast<const f32x4*>(cr + g);
      const f32x4 c1 = *reinterpret_cast<const f32x4*>(cr + g + 4);
      const f32x4 s0 = *reinterpret_cast<const f32x4*>(sr + g);
      const f32x4 s1 = *reinterpret_cast<const f32x4*>(sr + g + 4);
      u16x8 o1, o2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = j < 4 ? c0[j & 3] : c1[j & 3];
        const float s = j < 4 ? s0[j & 3] : s1[j & 3];
        float r1, r2;
        rope_pair(bf2f(x1[j]), bf2f(x2[j]), c, s, r1, r2);
        o1[j] = f2bf(r1);
        o2[j] = f2bf(r2);
      }
      if (h < Hq) {
        bf16_t* dst = q_out + ((int64_t)t * Hq + h) * D;
        *reinterpret_cast<u16x8*>(dst + g) = o1;
        *reinterpret_cast<u16x8*>(dst + HALF + g) = o2;
      } else {
        const int kh = h - Hq;
        if (k_out) {
          bf16_t* dst = k_out + ((int64_t)t * Hkv + kh) * D;
          *reinterpret_cast<u16x8*>(dst + g) = o1;
          *reinterpret_cast<u16x8*>(dst + HALF + g) = o2;
        }
        if (cache_base_k >= 0) {
          // tiled K layout (attn_decode.hip): [16-token tile][ks][lg][token][8 dims],
          // dim d = 32*lg + 8*ks + j
          KV* tile = k_cache + tile_base_k + (int64_t)kh * page_size * D;
          const int d1 = g, d2 = HALF + g;
          CacheStore<KV>::put(tile + ((((d1 & 31) >> 3) * 4 + (d1 >> 5)) * 16 + t16) * 8, o1, k_inv);
          CacheStore<KV>::put(tile + ((((d2 & 31) >> 3) * 4 + (d2 >> 5)) * 16 + t16) * 8, o2, k_inv);
        }
      }
    } else {
      const int ci = it - rot_items;
      const int kh = ci / (D / 8), g = (ci % (D / 8)) * 8;
      const u16x8 v = ld8((Hq + Hkv + kh) * D + g);
      if (v_out) *reinterpret_cast<u16x8*>(v_out + ((int64_t)t * Hkv + kh) * D + g) = v;
      if (cache_base_k >= 0) CacheStore<KV>::put(v_cache + cache_base_k + (int64_t)kh * page_size * D + g, v, v_inv);
    }
  }
}

int rope_kv(const bf16_t* qkv, int64_t qkv_stride, const int64_t* pos, const float* cos_t,
            const float* sin_t, int tokens, int Hq, int Hkv, int head_dim, bf16_t* q_out,
            bf16_t* k_out, bf16_t* v_out, void* k_cache, void* v_cache,
            const int64_t* slots, int page_size, int64_t max_pos, const float* xp, int S,
            const bf16_t* bias, bool fp8_cache, float k_scale, float v_scale, hipStream_t stream) {
  if (tokens == 0) return 0;
  if (head_dim != 128) return -1;
  const int64_t slab = (int64_t)tokens * (Hq + 2 * Hkv) * head_dim;
  const int items = (Hq + Hkv) * (head_dim / 16) + Hkv * (head_dim / 8);
  static const int ni = [] { const char* e = getenv("OAMD_ROPE_ITEMS"); return e && e[0] == '6' ? 64 : 256; }();   // OAMD_ROPE_ITEMS=64: one-wave workgroups
  const dim3 grid(tokens, (items + ni - 1) / ni);
  const int sc = xp == nullptr ? 1 : S;
#define OAMD_ROPE(KVT, SCC, KI, VI)                                                                              \
  if (ni == 256)                                                                                                 \
    rope_kv_kernel<128, KVT, SCC, 256><<<grid, 256, 0, stream>>>(                                                \
        qkv, qkv_stride, pos, cos_t, sin_t, Hq, Hkv, q_out, k_out, v_out, static_cast<KVT*>(k_cache),          \
        static_cast<KVT*>(v_cache), slots, page_size, max_pos, xp, S, slab, bias, KI, VI);                      \
  else                                                                                                           \
    rope_kv_kernel<128, KVT, SCC><<<grid, kRopeItems, 0, stream>>>(                                             \
        qkv, qkv_stride, pos, cos_t, sin_t, Hq, Hkv, q_out, k_out, v_out, static_cast<KVT*>(k_cache),          \
        static_cast<KVT*>(v_cache), slots, page_size, max_pos, xp, S, slab, bias, KI, VI)
#define OAMD_ROPE_S(KVT, KI, VI)                   \
  switch (sc) {                                    \
    case 1: OAMD_ROPE(KVT, 1, KI, VI); break;      \
    case 2: OAMD_ROPE(KVT, 2, KI, VI); break;      \
    case 4: OAMD_ROPE(KVT, 4, KI, VI); break;      \
    case 5: OAMD_ROPE(KVT, 5, KI, VI); break;      \
    case 8: OAMD_ROPE(KVT, 8, KI, VI); break;      \
    default: OAMD_ROPE(KVT, 0, KI, VI); break;     \
  }
  if (fp8_cache) {
    OAMD_ROPE_S(uint8_t, 1.f / k_scale, 1.f / v_scale)
  } else {
    OAMD_ROPE_S(bf16_t, 1.f, 1.f)
  }
#undef OAMD_ROPE_S
#undef OAMD_ROPE
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
