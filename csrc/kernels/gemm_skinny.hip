// Skinny-M GEMM for small decode buckets: Y[M, N] = X[M, K] . W[N, K]^T with
// M <= 32 ("decode uses skinny-M ... with weight streaming").
//
// At M = 1..32 the step is a pure weight stream (16 GB of bf16 weights per 8B
// decode step): the kernel's only job is to keep enough W bytes in flight to
// run HBM at full rate. Structure (cdna_hip_programming.md §5, row "GEMV /
// M <= 16 decode weights": straight to VGPRs, deep unroll, no LDS round trip):
//   * a block owns a 16-row tile of W (two for the fused SwiGLU: the gate rows
//     and the matching up rows 64 rows later) and its 4 waves split K;
//   * each wave streams its K range in 32-deep steps: lane l loads 16 B of W
//     row (l & 15) at k = 8 (l >> 4) -- exactly the A-fragment of
//     v_mfma_f32_16x16x32_bf16 -- and the matching 16 B of X rows (l & 15) as
//     the B-fragment (X is tiny and L2-resident); U steps are issued before
//     the first MFMA, so every wave keeps U x 1 KB of W in flight;
//   * the MFMA does the M-way reuse for free (16 output columns = 16 rows of
//     X per instruction; 2 instructions for M in 17..32) -- no cross-lane
//     shuffle reductions as in a VALU GEMV;
//   * the 4 per-wave partial tiles are summed through LDS, then stored as bf16,
//     as fp32 split-K slabs (consumed by rmsnorm / rope_kv), or through the
//     SwiGLU epilogue (HF rounding points, as gemm.hip).
// Split-K across blocks (gridDim.y = S) only adds parallelism for short-N shapes.
#include "common.h"
#include "kernels.h"

namespace oamd {

typedef __bf16 bf16x8s_t __attribute__((ext_vector_type(8)));

namespace sk {
constexpr int kWaves = 4;
constexpr int kThreads = kWaves * 64;
constexpr int kU = 8;  // k-steps (32 deep) in flight per wave
enum { kStore = 0, kPartial = 1, kSilu = 2 };
}  // namespace sk

// NT = W tiles per block (2 for SwiGLU: gate + up), MT = 16-column X tiles (M <= 16 * MT).
template <int NT, int MT, int EPI>
__global__ void __launch_bounds__(sk::kThreads) gemm_skinny_kernel(const bf16_t* __restrict__ X,
                                                                 const bf16_t* __restrict__ W,
                                                                 bf16_t* __restrict__ Y, float* __restrict__ P,
                                                                 int M, int N, int K, int S) {
  __shared__ float red[sk::kWaves][NT * MT][64 * 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 15, kq = lane >> 4;
  // W rows of this block's tile(s)
  int rows[NT];
  if constexpr (EPI == sk::kSilu) {
    const int g = blockIdx.x >> 2, sub = blockIdx.x & 3;  // 128-row gate|up group, 16-row slice
    rows[0] = g * 128 + sub * 16;
    rows[NT - 1] = g * 128 + 64 + sub * 16;
  } else {
    rows[0] = blockIdx.x * 16;
  }
  const int kz = blockIdx.y;
  const int Kb = K / S;             // this block's K range
  const int Kw = Kb / sk::kWaves;   // this wave's
  const int k0 = kz * Kb + w * Kw;
  const int steps = Kw / 32;

  const u16x8* wp[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wp[t] = reinterpret_cast<const u16x8*>(W + (int64_t)(rows[t] + r) * K + k0 + kq * 8);
  const u16x8* xp[MT];
  bool xv[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int m = j * 16 + r;
    xv[j] = m < M;
    xp[j] = reinterpret_cast<const u16x8*>(X + (int64_t)(xv[j] ? m : 0) * K + k0 + kq * 8);
  }
  f32x4 acc[NT][MT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const u16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  int s = 0;
  for (; s + sk::kU <= steps; s += sk::kU) {
    u16x8 a[sk::kU][NT], b[sk::kU][MT];
#pragma unroll
    for (int u = 0; u < sk::kU; ++u) {
#pragma unroll
      for (int t = 0; t < NT; ++t) a[u][t] = __builtin_nontemporal_load(wp[t] + (s + u) * 4);
#pragma unroll
      for (int j = 0; j < MT; ++j) b[u][j] = xv[j] ? xp[j][(s + u) * 4] : zero;
    }
#pragma unroll
    for (int u = 0; u < sk::kU; ++u)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < MT; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8s_t, a[u][t]),
                                                              __builtin_bit_cast(bf16x8s_t, b[u][j]), acc[t][j], 0, 0,
                                                              0);
  }
  for (; s < steps; ++s) {  // remainder (< kU steps)
    u16x8 a[NT], b[MT];
#pragma unroll
    for (int t = 0; t < NT; ++t) a[t] = __builtin_nontemporal_load(wp[t] + s * 4);
#pragma unroll
    for (int j = 0; j < MT; ++j) b[j] = xv[j] ? xp[j][s * 4] : zero;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < MT; ++j)
        acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8s_t, a[t]),
                                                            __builtin_bit_cast(bf16x8s_t, b[j]), acc[t][j], 0, 0, 0);
  }

  // ---- sum the 4 waves' partial tiles: C lane l -> W row 4 (l >> 4) + i, X row (column) l & 15
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[w][t * MT + j][i * 64 + lane] = acc[t][j][i];
  __syncthreads();
  // thread -> (tile pair j, element e): 64 lanes x 4 regs per tile
  for (int e = tid; e < MT * 256; e += sk::kThreads) {
    const int j = e >> 8, i = (e >> 6) & 3, l = e & 63;
    const int m = j * 16 + (l & 15);
    const int rr = 4 * (l >> 4) + i;  // row within the 16-row tile
    float v[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      v[t] = 0.f;
#pragma unroll
      for (int ww = 0; ww < sk::kWaves; ++ww) v[t] += red[ww][t * MT + j][i * 64 + l];
    }
    if (m >= M) continue;
    if constexpr (EPI == sk::kSilu) {
      const float g = bf2f(f2bf(v[0]));
      const float u = bf2f(f2bf(v[NT - 1]));
      const float sg = bf2f(f2bf(g / (1.f + __expf(-g))));
      const int f = (blockIdx.x >> 2) * 64 + (blockIdx.x & 3) * 16 + rr;
      Y[(int64_t)m * (N / 2) + f] = f2bf(sg * u);
    } else if constexpr (EPI == sk::kPartial) {
      P[((int64_t)kz * M + m) * N + rows[0] + rr] = v[0];
    } else {
      Y[(int64_t)m * N + rows[0] + rr] = f2bf(v[0]);
    }
  }
}

int gemm_skinny(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int S, bool silu_gu,
                hipStream_t stream) {
  if (M < 1 || M > 32) return -1;
  if (S < 1 || S > 8 || K % (S * sk::kWaves * 32) != 0) return -2;
  if (silu_gu && (S != 1 || N % 128 != 0)) return -3;
  if (N % 16 != 0) return -4;
  if (S > 1 && P == nullptr) return -5;
  const int MT = M <= 16 ? 1 : 2;
  if (silu_gu) {
    const dim3 grid(N / 32, 1);  // one block per (16 gate rows, 16 up rows)
    if (MT == 1) gemm_skinny_kernel<2, 1, sk::kSilu><<<grid, sk::kThreads, 0, stream>>>(X, W, Y, P, M, N, K, 1);
    else gemm_skinny_kernel<2, 2, sk::kSilu><<<grid, sk::kThreads, 0, stream>>>(X, W, Y, P, M, N, K, 1);
  } else {
    const dim3 grid(N / 16, S);
    if (S > 1) {
      if (MT == 1) gemm_skinny_kernel<1, 1, sk::kPartial><<<grid, sk::kThreads, 0, stream>>>(X, W, Y, P, M, N, K, S);
      else gemm_skinny_kernel<1, 2, sk::kPartial><<<grid, sk::kThreads, 0, stream>>>(X, W, Y, P, M, N, K, S);
    } else {
      if (MT == 1) gemm_skinny_kernel<1, 1, sk::kStore><<<grid, sk::kThreads, 0, stream>>>(X, W, Y, P, M, N, K, 1);
      else gemm_skinny_kernel<1, 2, sk::kStore><<<grid, sk::kThreads, 0, stream>>>(X, W, Y, P, M, N, K, 1);
    }
  }
  OAMD_LAUNCH_CHECK();
  if (S > 1 && Y != nullptr) {  // Y == nullptr: the consumer sums the slabs
    const int64_t MN = (int64_t)M * N;
    if (MN % 4 != 0) return -6;
    return splitk_reduce(P, Y, MN, S, stream);
  }
  return 0;
}

}  // namespace oamd
