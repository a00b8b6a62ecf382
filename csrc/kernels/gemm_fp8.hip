// FP8 (OCP e4m3fn) W8A8 GEMM for the large explanation models (SURVEY.md §2.4
// N8; BASELINE config 5, Llama-3-70B): Y[M, N] = (X8[M, K] . W8[N, K]^T) *
// sx[m] * sw[n], bf16 out, fp32 accumulate.
//
// * Weights are quantized once per output channel (sw[n] = amax / 448) and
//   activations per token at run time (quantize_fp8_rows: sx[m] = amax / 448),
//   so the MFMA runs on raw e4m3 operands with unit block scales and the two
//   scale vectors are applied once in the epilogue.
// * v_mfma_scale_f32_16x16x128_f8f6f4 (E8M0 scale 127 = 1.0): 4x the K of the
//   bf16 16x16x32 form at 2x its cycles — twice the bf16 MFMA rate — and half
//   the bytes per weight, which is what decode (weight-streaming) needs.
// * Same pipeline as gemm.hip: LDS-DMA (global_load_lds_dwordx4) of full
//   128-B lines (= 128 K-elements per row) into a 3-deep ring, counted vmcnt,
//   raw s_barrier, split-K slabs for narrow N, M tiles of BM rows. Rows past M
//   are clamped duplicates on load and skipped on store, so any M works.
// * Fragment read = 32 K-bytes per lane (two ds_read_b128 of chunks 2g, 2g+1).
//   The LDS XOR swizzle differs from the bf16 kernel's: slot = chunk ^
//   (bit1(row) | bit2(row) << 2) makes those reads conflict-free (exhaustive
//   check over the four ds_read_b128 lane groups).
#include "common.h"
#include "kernels.h"

namespace oamd {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));

namespace f8 {

constexpr int kBK = 128;  // K elements (bytes) per stage: one 128-B line per row
constexpr int kStages = 3;
constexpr int kWaves = 8;

template <int BM, int BN>
struct Cfg {
  static constexpr int WM = 4, WN = kWaves / WM;
  static constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  static constexpr int ROWS = BM + BN;
  static constexpr int STAGE_BYTES = ROWS * kBK;
  static constexpr int GL = ROWS / 8 / kWaves;
  static constexpr int LDS_BYTES = kStages * STAGE_BYTES;
  static_assert(ROWS % (8 * kWaves) == 0, "stage rows must split evenly over the waves");
};

__device__ __forceinline__ int swz(int row, int chunk) {
  return chunk ^ (((row >> 1) & 1) | (((row >> 2) & 1) << 2));
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

}  // namespace f8

template <int BM, int BN, bool PARTIAL>
__global__ void __launch_bounds__(f8::kWaves * 64, 1)
    gemm_fp8_kernel(const uint8_t* __restrict__ X, const uint8_t* __restrict__ W, const float* __restrict__ sx,
                    const float* __restrict__ sw, bf16_t* __restrict__ Y, float* __restrict__ P, int M, int N, int K,
                    int S, int wnt) {
  using C = f8::Cfg<BM, BN>;
  __shared__ __attribute__((aligned(1024))) char lds[C::LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kz = blockIdx.x % S, nt = blockIdx.x / S;
  const int n0 = nt * BN, m0 = blockIdx.y * BM;
  // K-slice kz = K-steps [kz * TK / S, (kz + 1) * TK / S) (uneven when S does not divide TK)
  const int TK = K / f8::kBK, t0 = kz * TK / S, kbase = t0 * f8::kBK, T = (kz + 1) * TK / S - t0;

  const int lrow = lane >> 3, lslot = lane & 7;
  auto issue = [&](int t, int buf) {
    const int k0 = kbase + t * f8::kBK;
    char* sbase = lds + buf * C::STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < C::GL; ++i) {
      const int q = w + f8::kWaves * i;
      const int row = 8 * q + lrow;
      const int chunk = f8::swz(row, lslot);
      const uint8_t* src = (row < BM) ? X + (int64_t)min(m0 + row, M - 1) * K + k0 + chunk * 16
                                      : W + (int64_t)(n0 + row - BM) * K + k0 + chunk * 16;
      if (wnt && row >= BM)   // wave-uniform (8-row pieces): weights stream non-temporal
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sbase + q * 1024), 16, 0, 2);
      else
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sbase + q * 1024), 16, 0, 0);
    }
  };

  const int wm = w / C::WN, wn = w % C::WN;
  const int l15 = lane & 15, lg = lane >> 4;
  f32x4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto frag = [&](const char* sbase, int row) -> v8i {
    const v4i lo = *reinterpret_cast<const v4i*>(sbase + row * 128 + (f8::swz(row, 2 * lg) << 4));
    const v4i hi = *reinterpret_cast<const v4i*>(sbase + row * 128 + (f8::swz(row, 2 * lg + 1) << 4));
    return v8i{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto compute = [&](int buf) {
    const char* sbase = lds + buf * C::STAGE_BYTES;
    v8i a[C::FM], b[C::FN];
#pragma unroll
    for (int i = 0; i < C::FM; ++i) a[i] = frag(sbase, wm * (BM / C::WM) + 16 * i + l15);
#pragma unroll
    for (int j = 0; j < C::FN; ++j) b[j] = frag(sbase, BM + wn * (BN / C::WN) + 16 * j + l15);
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i][j], 0, 0, 0, 127, 0, 127);
  };

  issue(0, 0);
  if (T > 1) issue(1, 1);
  for (int t = 0; t < T; ++t) {
    if (t + 1 < T) f8::wait_vmcnt<C::GL>();
    else f8::wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < T) issue(t + 2, (t + 2) % f8::kStages);
    compute(t % f8::kStages);
  }

#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
      const int col = n0 + wn * (BN / C::WN) + 16 * j + l15;
      const float scol = sw[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * (BM / C::WM) + 16 * i + 4 * lg + r;
        if (row >= M) continue;
        const float v = acc[i][j][r] * sx[row] * scol;
        if constexpr (PARTIAL) P[((int64_t)kz * M + row) * N + col] = v;
        else Y[(int64_t)row * N + col] = f2bf(v);
      }
    }
}

// Per-row dynamic quantization: sx[m] = max|x[m, :]| / 448, q = e4m3fn(x / sx).
// One 256-thread block per row. Rows of up to 256 x 8 x MAXV elements are loaded ONCE
// into registers (all loads in flight together), reduced, then quantized from the
// registers: a decode row is latency-bound, and the former two streaming passes with
// a dependent load per step cost 12.6 us for a 64 x 8192 block (profiles/tp8_sim_*).
// SILU: the input is the 64-feature-interleaved gate|up projection [M, 2K] and the
// row quantized is bf16(bf16(silu(bf16 g)) * bf16 u) — the SwiGLU and the down
// projection's input quantization in one kernel.
// P (SILU only): the gate|up rows are S fp32 split-K slabs [S, M, 2K] instead of bf16 `x`;
// they are summed in slab order and bf16-rounded first (== splitk_reduce_fp32 then SILU).
// SC (SILU with slabs): compile-time slab count, so every slab load of an element is issued
// before the first add (0: runtime S, one slab per loop trip).
template <int MAXV, bool SILU, int SC = 0>
__global__ void __launch_bounds__(256) quantize_rows_reg_kernel(const bf16_t* __restrict__ x, uint8_t* __restrict__ q,
                                                                float* __restrict__ sx, int K, int64_t ld,
                                                                const float* __restrict__ P, int S) {
  __shared__ float red[4];
  const int64_t m = blockIdx.x;
  const bf16_t* xr = x + m * ld;
  const int nv = K >> 3;
  float v[MAXV][8];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * 256;
    if (vi < nv) {
      if constexpr (SILU) {
        const int c = (vi >> 3) * 128 + (vi & 7) * 8;   // 64-feature blocks: gate then up
        u16x8 gv, uv;
        if (P != nullptr) {
          const int64_t MN = (int64_t)gridDim.x * 2 * K;
          const float* pr = P + m * 2 * K + c;
          f32x4 g0 = *reinterpret_cast<const f32x4*>(pr), g1 = *reinterpret_cast<const f32x4*>(pr + 4);
          f32x4 u0 = *reinterpret_cast<const f32x4*>(pr + 64), u1 = *reinterpret_cast<const f32x4*>(pr + 68);
          if constexpr (SC > 1) {
            f32x4 sl[SC - 1][4];
#pragma unroll
            for (int s = 1; s < SC; ++s) {
              const float* ps = pr + s * MN;
              sl[s - 1][0] = *reinterpret_cast<const f32x4*>(ps);
              sl[s - 1][1] = *reinterpret_cast<const f32x4*>(ps + 4);
              sl[s - 1][2] = *reinterpret_cast<const f32x4*>(ps + 64);
              sl[s - 1][3] = *reinterpret_cast<const f32x4*>(ps + 68);
            }
#pragma unroll
            for (int s = 1; s < SC; ++s) {   // slab order, as splitk_reduce_fp32
              g0 += sl[s - 1][0];
              g1 += sl[s - 1][1];
              u0 += sl[s - 1][2];
              u1 += sl[s - 1][3];
            }
          } else if constexpr (SC == 0) {
            for (int s = 1; s < S; ++s) {
              const float* ps = pr + s * MN;
              g0 += *reinterpret_cast<const f32x4*>(ps);
              g1 += *reinterpret_cast<const f32x4*>(ps + 4);
              u0 += *reinterpret_cast<const f32x4*>(ps + 64);
              u1 += *reinterpret_cast<const f32x4*>(ps + 68);
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            gv[j] = f2bf(g0[j]);
            gv[j + 4] = f2bf(g1[j]);
            uv[j] = f2bf(u0[j]);
            uv[j + 4] = f2bf(u1[j]);
          }
        } else {
          gv = *reinterpret_cast<const u16x8*>(xr + c);
          uv = *reinterpret_cast<const u16x8*>(xr + c + 64);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float g = bf2f(gv[j]);
          v[i][j] = bf2f(f2bf(bf2f(f2bf(g / (1.f + __expf(-g)))) * bf2f(uv[j])));
        }
      } else {
        const u16x8 xv = *reinterpret_cast<const u16x8*>(xr + vi * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(xv[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[i][j]));
    }
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) sx[m] = s;
  uint8_t* qr = q + m * (int64_t)K;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * 256;
    if (vi < nv) {
      int lo = 0, hi = 0;
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][0] * inv, v[i][1] * inv, lo, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][2] * inv, v[i][3] * inv, lo, true);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][4] * inv, v[i][5] * inv, hi, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][6] * inv, v[i][7] * inv, hi, true);
      *reinterpret_cast<uint2*>(qr + vi * 8) = make_uint2(static_cast<uint32_t>(lo), static_cast<uint32_t>(hi));
    }
  }
}

// Rows longer than the register path: two streaming passes.
__global__ void quantize_fp8_rows_kernel(const bf16_t* __restrict__ x, uint8_t* __restrict__ q,
                                         float* __restrict__ sx, int K, int64_t ld) {
  __shared__ float red[4];
  const int64_t m = blockIdx.x;
  const bf16_t* xr = x + m * ld;
  float amax = 0.f;
  for (int c = threadIdx.x * 8; c < K; c += 256 * 8) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(xr + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(bf2f(v[j])));
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) sx[m] = s;
  uint8_t* qr = q + m * (int64_t)K;
  for (int c = threadIdx.x * 8; c < K; c += 256 * 8) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(xr + c);
    uint2 o;
    int lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[0]) * inv, bf2f(v[1]) * inv, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[2]) * inv, bf2f(v[3]) * inv, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[4]) * inv, bf2f(v[5]) * inv, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[6]) * inv, bf2f(v[7]) * inv, hi, true);
    o.x = static_cast<uint32_t>(lo);
    o.y = static_cast<uint32_t>(hi);
    *reinterpret_cast<uint2*>(qr + c) = o;
  }
}

int quantize_fp8_rows(const bf16_t* x, uint8_t* q, float* sx, int M, int K, int64_t ld, hipStream_t stream) {
  if (M == 0) return 0;
  if (K % 8 != 0) return -1;
  const int nv = K / 8;
  if (nv <= 256 * 2) quantize_rows_reg_kernel<2, false><<<M, 256, 0, stream>>>(x, q, sx, K, ld, nullptr, 1);
  else if (nv <= 256 * 4) quantize_rows_reg_kernel<4, false><<<M, 256, 0, stream>>>(x, q, sx, K, ld, nullptr, 1);
  else if (nv <= 256 * 8) quantize_rows_reg_kernel<8, false><<<M, 256, 0, stream>>>(x, q, sx, K, ld, nullptr, 1);
  else quantize_fp8_rows_kernel<<<M, 256, 0, stream>>>(x, q, sx, K, ld);
  OAMD_LAUNCH_CHECK();
  return 0;
}

int silu_quantize_fp8(const bf16_t* gu, const float* P, int S, uint8_t* q, float* sx, int M, int inter, int64_t ld,
                      hipStream_t stream) {
  if (M == 0) return 0;
  if (inter % 64 != 0 || (gu == nullptr) == (P == nullptr) || S < 1) return -1;
  const int nv = inter / 8;
  const int sc = P == nullptr ? 1 : S;
#define OAMD_SQ(MV)                                                                                       \
  switch (sc) {                                                                                           \
    case 1: quantize_rows_reg_kernel<MV, true, 1><<<M, 256, 0, stream>>>(gu, q, sx, inter, ld, P, S); break; \
    case 2: quantize_rows_reg_kernel<MV, true, 2><<<M, 256, 0, stream>>>(gu, q, sx, inter, ld, P, S); break; \
    case 4: quantize_rows_reg_kernel<MV, true, 4><<<M, 256, 0, stream>>>(gu, q, sx, inter, ld, P, S); break; \
    case 8: quantize_rows_reg_kernel<MV, true, 8><<<M, 256, 0, stream>>>(gu, q, sx, inter, ld, P, S); break; \
    default: quantize_rows_reg_kernel<MV, true, 0><<<M, 256, 0, stream>>>(gu, q, sx, inter, ld, P, S); break; \
  }
  if (nv <= 256 * 2) { OAMD_SQ(2) }
  else if (nv <= 256 * 4) { OAMD_SQ(4) }
  else if (nv <= 256 * 8) { OAMD_SQ(8) }
  else return -2;
#undef OAMD_SQ
  OAMD_LAUNCH_CHECK();
  return 0;
}

__global__ void splitk_reduce_fp32_kernel(const float* __restrict__ P, bf16_t* __restrict__ Y, int64_t MN, int S) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= MN) return;
  f32x4 a = *reinterpret_cast<const f32x4*>(P + i);
  for (int s = 1; s < S; ++s) a += *reinterpret_cast<const f32x4*>(P + s * MN + i);
  uint2 o;
  o.x = pack_bf2(a[0], a[1]);
  o.y = pack_bf2(a[2], a[3]);
  *reinterpret_cast<uint2*>(Y + i) = o;
}

int gemm_fp8(const uint8_t* X, const uint8_t* W, const float* sx, const float* sw, bf16_t* Y, float* P, int M,
             int N, int K, int S, int BN, int BM, hipStream_t stream) {
  if (M <= 0) return 0;
  if (BM != 64 && BM != 128 && BM != 256) return -1;
  if ((BN != 64 && BN != 128) || N % BN != 0) return -2;
  if (S < 1 || S > 16 || K % f8::kBK != 0 || K / f8::kBK < S) return -3;
  if (S > 1 && P == nullptr) return -4;
  const dim3 grid((N / BN) * S, (M + BM - 1) / BM);
  static const int wnt = [] { const char* e = getenv("OAMD_FP8_WNT"); return e && e[0] == '0' ? 0 : 1; }();
#define OAMD_G8(BMM, BNN)                                                                                     \
  if (S > 1)                                                                                                  \
    gemm_fp8_kernel<BMM, BNN, true><<<grid, f8::kWaves * 64, 0, stream>>>(X, W, sx, sw, Y, P, M, N, K, S, wnt); \
  else gemm_fp8_kernel<BMM, BNN, false><<<grid, f8::kWaves * 64, 0, stream>>>(X, W, sx, sw, Y, P, M, N, K, S, wnt)
#define OAMD_G8M(BMM) \
  if (BN == 64) { OAMD_G8(BMM, 64); } else { OAMD_G8(BMM, 128); }
  switch (BM) {
    case 64: OAMD_G8M(64); break;
    case 128: OAMD_G8M(128); break;
    default: OAMD_G8M(256); break;
  }
#undef OAMD_G8M
#undef OAMD_G8
  OAMD_LAUNCH_CHECK();
  if (S > 1 && Y != nullptr) {   // Y == nullptr: the consumer sums the slabs
    const int64_t MN = (int64_t)M * N;
    splitk_reduce_fp32_kernel<<<(MN / 4 + 255) / 256, 256, 0, stream>>>(P, Y, MN, S);
    OAMD_LAUNCH_CHECK();
  }
  return 0;
}

}  // namespace oamd
