// Token sampler: temperature + Gumbel-max over the
// vocabulary (or one tensor-parallel vocab shard: col_offset + out_val let the
// caller take the max over shards, Gumbel-max being decomposable), greedy when temperature <= 0. One 1024-thread block per row;
// each thread keeps a (value, index) pair over a grid-stride of the vocab with
// 16-B loads, then a wave + LDS argmax. The noise is a counter-based hash of
// (seed[row], position[row], column), so a captured hipGraph replays to the
// same tokens and the kernel needs no RNG state on the device.
#include "common.h"
#include "kernels.h"

namespace oamd {

template <typename T>
__device__ __forceinline__ float load_logit(const T* p, int64_t i);
template <>
__device__ __forceinline__ float load_logit<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float load_logit<bf16_t>(const bf16_t* p, int64_t i) { return bf2f(p[i]); }

__device__ __forceinline__ void argmax_merge(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
}

template <typename T>
__global__ void __launch_bounds__(1024) sample_kernel(const T* __restrict__ logits, int64_t stride, int vocab,
                                                      const float* __restrict__ temperature,
                                                      const int64_t* __restrict__ seeds,
                                                      const int64_t* __restrict__ positions,
                                                      int64_t* __restrict__ out_tokens, int64_t col_offset,
                                                      float* __restrict__ out_val) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const int row = blockIdx.x;
  const T* lr = logits + row * stride;
  const float temp = temperature[row];
  const bool greedy = !(temp > 0.f);
  // Perturbed values are compared in base 2: x/T - ln(-ln u) = ln2 * (x log2e / T -
  // log2(-log2 u)) - ln(ln2), a monotone map, so the loop pays one FMA and two v_log_f32
  // per column and the winner is mapped back once (out_val stays in natural units).
  constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f, kNegLnLn2 = 0.36651292058166435f;
  const float inv_t = greedy ? 1.f : kLog2e / temp;
  const uint64_t key = mix64((static_cast<uint64_t>(seeds[row]) * 0x9E3779B97F4A7C15ULL) ^
                             (static_cast<uint64_t>(positions[row]) << 32));
  const uint32_t k1 = static_cast<uint32_t>(key), k2 = static_cast<uint32_t>(key >> 32);
  const uint32_t c0 = static_cast<uint32_t>(col_offset);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  auto visit = [&](float x, int i) {
    if (!greedy) {
      const float u = uniform01(hash_col(c0 + static_cast<uint32_t>(i), k1, k2));
      // -log2(u) >= 8.6e-8 exactly; the clamp only guards a hardware log rounding to 0
      x = x * inv_t - __builtin_amdgcn_logf(fmaxf(-__builtin_amdgcn_logf(u), 5.9604645e-8f));
    }
    argmax_merge(bv, bi, x, i);
  };
  // 16-B loads over the aligned body of the row (8 bf16 / 4 fp32 per lane), scalar tail.
  // argmax_merge is a total order (value, then smaller index), so the visiting order
  // does not change the result.
  constexpr int VEC = 16 / static_cast<int>(sizeof(T));
  const int nv = (reinterpret_cast<uintptr_t>(lr) & 15) == 0 ? vocab / VEC : 0;
  auto visit16 = [&](const uint4& raw, int v) {
    const uint32_t wv[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (sizeof(T) == 2) {
        visit(__uint_as_float(wv[k] << 16), VEC * v + 2 * k);
        visit(__uint_as_float(wv[k] & 0xffff0000u), VEC * v + 2 * k + 1);
      } else {
        visit(__uint_as_float(wv[k]), VEC * v + k);
      }
    }
  };
  // UNR row vectors per thread requested before any is consumed: one dependent HBM round
  // trip per UNR vectors instead of per vector (the loop was latency-bound: ~16 trips
  // of 16 B per thread for a 128k vocab row)
  constexpr int UNR = 4;
  const uint4* lv = reinterpret_cast<const uint4*>(lr);
  const int step = blockDim.x;
  int v0 = threadIdx.x;
  for (; v0 + (UNR - 1) * step < nv; v0 += UNR * step) {
    uint4 raw[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) raw[u] = lv[v0 + u * step];
#pragma unroll
    for (int u = 0; u < UNR; ++u) visit16(raw[u], v0 + u * step);
  }
  for (int v = v0; v < nv; v += step) visit16(lv[v], v);
  for (int i = nv * VEC + threadIdx.x; i < vocab; i += blockDim.x) visit(load_logit<T>(lr, i), i);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, kWave);
    const int oi = __shfl_xor(bi, o, kWave);
    argmax_merge(bv, bi, ov, oi);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { sv[w] = bv; si[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = sv[0];
    int id = si[0];
    for (int j = 1; j < (int)(blockDim.x >> 6); ++j) argmax_merge(v, id, sv[j], si[j]);
    out_tokens[row] = ((id == 0x7fffffff) ? 0 : id) + col_offset;
    if (out_val) out_val[row] = greedy ? v : v * kLn2 + kNegLnLn2;
  }
}

int sample_tokens(const void* logits, bool logits_bf16, int64_t stride, int rows, int vocab,
                  const float* temperature, const int64_t* seeds, const int64_t* positions,
                  int64_t* out_tokens, int64_t col_offset, float* out_val, hipStream_t stream) {
  if (rows == 0) return 0;
  if (logits_bf16)
    sample_kernel<bf16_t><<<rows, 1024, 0, stream>>>(static_cast<const bf16_t*>(logits), stride, vocab,
                                                     temperature, seeds, positions, out_tokens, col_offset, out_val);
  else
    sample_kernel<float><<<rows, 1024, 0, stream>>>(static_cast<const float*>(logits), stride, vocab,
                                                    temperature, seeds, positions, out_tokens, col_offset, out_val);
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
