// Shared device helpers for the gfx950 (CDNA4) kernels of operator_amd.
//
// Conventions used by every kernel in csrc/kernels:
//   * bf16 tensors are carried as raw uint16_t; conversions go through the
//     hardware cvt (plain cast of __hip_bfloat16) so NaN stays NaN
//     (MI355X_MICROARCH.md "Correctness boundaries").
//   * every global bf16 access is vectorised to 16 B per lane (8 x bf16),
//     cdna_hip_programming.md Guideline 13.
//   * wave size is hard-coded to 64 (never warpSize-derived constants).
//   * launchers take raw device pointers + hipStream_t so they can be captured
//     into a hipGraph by the caller (no allocation / sync inside a launcher).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace oamd {

constexpr int kWave = 64;

typedef uint16_t bf16_t;
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return __builtin_bit_cast(bf16_t, b);
}

// Pack two floats into two bf16 (lo in the low half).
// rotate-half RoPE of one (x[d], x[d + D/2]) pair with explicit FMAs: one numerics for
// rope_kv and the RoPE folded into decode attention (no compiler-chosen contraction)
__device__ __forceinline__ void rope_pair(float a, float b, float c, float s, float& o1, float& o2) {
  o1 = __builtin_fmaf(a, c, -(b * s));
  o2 = __builtin_fmaf(b, c, a * s);
}

__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Sum within aligned groups of `width` lanes (width power of two <= 64).
template <int WIDTH>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = WIDTH / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Block-wide sum for blockDim.x = NT (multiple of 64). `scratch` >= NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += scratch[i];
  __syncthreads();
  return t;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must
// be bijective"): consecutive logical tiles land on the same XCD (same L2).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nx = 8;
  if (nwg <= nx) return orig;
  const int q = nwg / nx, r = nwg % nx, xcd = orig % nx;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / nx;
}

// Element offset of (row r, column c) in the fragment-major "tiled" activation layout that
// gemm_xr reads: [K/64 step][rows/16 token block][2 k-half][64 lanes][8], lane = r % 16 +
// 16 ((c % 32) / 8) -- one K-step of all rows is contiguous, each 1 KiB is one MFMA
// B-fragment (rows % 16 == 0, K % 64 == 0).
__device__ __forceinline__ int64_t xr_tiled_off(int r, int c, int rows) {
  return ((((int64_t)(c >> 6) * (rows >> 4) + (r >> 4)) * 2 + ((c >> 5) & 1)) * 64 + (r & 15) + 16 * ((c & 31) >> 3)) * 8 +
         (c & 7);
}

// Counter-based RNG for Gumbel sampling, so a captured graph replays deterministic
// per (seed, step, row, col). The 64-bit finalizer runs once per row and yields two
// 32-bit keys; the per-column hash is a 32-bit two-round mix with the second key
// injected between the rounds (8 VALU ops per column instead of the ~20 of a 64-bit
// mix: the sampler's vocab loop is ALU-bound). Host mirror: ops/reference.py.
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ uint32_t hash_col(uint32_t c, uint32_t k1, uint32_t k2) {
  uint32_t h = c ^ k1;
  h ^= h >> 16; h *= 0x7feb352du;
  h ^= h >> 15; h ^= k2; h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}

// Open (0,1) with 23 bits: both ends are exact floats (max 1 - 2^-24), so -log(-log(u))
// stays finite. (24 bits + 0.5 rounded the top value to exactly 1.0f, whose Gumbel
// noise is +inf: a column that won regardless of its logit.)
__device__ __forceinline__ float uniform01(uint32_t h) {
  return (static_cast<float>(h >> 9) + 0.5f) * (1.0f / 8388608.0f);
}

}  // namespace oamd

#define OAMD_LAUNCH_CHECK()                                                     \
  do {                                                                          \
    hipError_t e__ = hipGetLastError();                                         \
    if (e__ != hipSuccess) return static_cast<int>(e__);                        \
  } while (0)
